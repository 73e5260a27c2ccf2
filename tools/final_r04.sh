#!/bin/bash
# Round-4 closing evidence on one GPU box: the pipeline/fusion parity file,
# smoke, the default bench line (counter passes + CPU baseline) and the
# rocprofv3 kernel-trace stats of a bench run.
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_stream_order.py -v --timeout 300 --timeout-method thread" \
 "150 python -c 'import __graft_entry__ as g; g.smoke()'" \
 "600 python3 bench.py > gpurun_out/bench.log 2>&1; grep ^{ gpurun_out/bench.log | tail -n 1 > gpurun_out/bench.json" \
 "400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof -o run -- python3 bench.py --steps 2 --warmup 1 --pmc off --no-cpu-baseline"
