#!/bin/bash
# Round 5: the device-block cache (dev_alloc / dev_free): the whole GPU suite,
# then the 49-view cfg4 sequential CLI (one view at a time vs the default,
# maps compared byte for byte) with the host phase timings.
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "1000 python -u -m pytest tests -x -m gpu -q --durations=10 --timeout 300 --timeout-method thread" \
 "600 env ACMMP_HOST_TIMING=1 python3 -u tools/pipeline_times.py 49 1600 1200 20 cli_serial,cli > gpurun_out/cli_devpool.jsonl 2> gpurun_out/cli_devpool.err"
