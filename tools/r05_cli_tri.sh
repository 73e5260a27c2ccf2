#!/bin/bash
# Round 5: ProcessProblem's planar block with one triangulation for the
# picture and the prior, the PNG encoded beside the second PatchMatch: the
# pipeline and planar parity files, then the cfg4 sequential CLI timing
# (one view at a time vs the default, maps compared byte for byte).
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pipeline.py tests/test_gpu_planar.py" \
 "600 env ACMMP_HOST_TIMING=1 python3 -u tools/pipeline_times.py 49 1600 1200 20 cli_serial,cli > gpurun_out/cli_tri.jsonl 2> gpurun_out/cli_tri.err"
