#!/bin/bash
# Round 5, GPU session 2a: parity of the product (Phase A pipelined from
# iteration 1 of a photometric pass, every geometric iteration) and of the
# stream forced fully on / off; per-pass A/B of the pipeline switch.
export TMPDIR=/tmp
V=acmmp_amd/lib/variants
B=acmmp_amd/lib/libacmmp_amd.so
P="tests/test_gpu_parity.py tests/test_gpu_sweep_views.py"
bash tools/gpu_steps.sh \
 "600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_sweep_views.py tests/test_gpu_planar.py -m gpu -x -q --timeout 300 --timeout-method thread" \
 "300 ACMMP_PIPE_FROM=0,0 python -u -m pytest $P -m gpu -x -q --timeout 200 --timeout-method thread" \
 "300 ACMMP_PIPE_FROM=99,99 python -u -m pytest $P -m gpu -x -q --timeout 200 --timeout-method thread" \
 "500 bash tools/ab.sh pass base=$V/libacmmp_amd_base.so p10=$B p99=$B@ACMMP_PIPE_FROM=99,99 p11=$B@ACMMP_PIPE_FROM=1,1 p00=$B@ACMMP_PIPE_FROM=0,0"
