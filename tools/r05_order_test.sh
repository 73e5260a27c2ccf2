#!/bin/bash
# Round 5: the CLI's --order jacobi on one GPU against the oracle pipeline.
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "300 python -u -m pytest tests/test_gpu_vp_cli.py -k 'order or world1' -m gpu -x -v --timeout 200 --timeout-method thread"
