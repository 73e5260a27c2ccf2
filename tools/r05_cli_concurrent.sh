#!/bin/bash
# Round 5: the sequential CLI with the non-geometric passes' views in flight
# (--concurrent_views 2, the default) against one view at a time: the CLI
# parity tests, then the 49-view cfg4 timing of both with a byte comparison.
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pipeline.py" \
 "900 python3 -u tools/pipeline_times.py 49 1600 1200 20 cli_serial,cli > gpurun_out/cli_concurrent.jsonl"
