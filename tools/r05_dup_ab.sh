#!/bin/bash
# Round 5: Phase A copies the cost of a candidate identical to an earlier one
# (product) vs running its call (nodup = make variant NAME=nodup
# EXTRA=-DACMMP_DUP_SKIP=0): hot-path parity, per-pass times, PMC passes.
export TMPDIR=/tmp
V=acmmp_amd/lib/variants
B=acmmp_amd/lib/libacmmp_amd.so
bash tools/gpu_steps.sh \
 "600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_sweep_views.py -m gpu -x -q --timeout 300 --timeout-method thread" \
 "400 bash tools/ab.sh pass nodup=$V/libacmmp_amd_nodup.so dup=$B" \
 "500 bash tools/ab.sh pmc nodup=$V/libacmmp_amd_nodup.so dup=$B"
rm -rf gpurun_out/ab_nodup gpurun_out/ab_dup
