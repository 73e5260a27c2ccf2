#!/bin/bash
# Round-5 opening run: the GPU suite under -x with the 30 slowest tests
# reported, the default bench line (with the new L2 counter pass), and the
# FETCH_SIZE / TCC_EA0_RDREQ calibration for dword gathers.
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "1100 python -u -m pytest tests -x -m gpu -q --durations=30 --timeout 300 --timeout-method thread" \
 "700 python3 bench.py > gpurun_out/bench.log 2>&1; grep ^{ gpurun_out/bench.log | tail -n 1 > gpurun_out/bench.json" \
 "400 bash tools/microbench/run_fetch_cal.sh"
