#!/bin/bash
# Round 5: the CLI's JBU views run concurrently too: the pipeline parity file,
# then the cfg4 CLI (default first, one view at a time last, maps compared).
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pipeline.py tests/test_gpu_vp_cli.py" \
 "600 python3 -u tools/pipeline_times.py 49 1600 1200 20 cli,cli_serial,cli_serial_last > gpurun_out/cli_jbu.jsonl"
