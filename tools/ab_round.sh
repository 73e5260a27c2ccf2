#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
V=acmmp_amd/lib/variants/libacmmp_amd_pl.so
echo "== product u8"; timeout -k 10 120 python3 tools/quick_time.py 1600 1200 8 > gpurun_out/ab_u8.log 2>&1 || exit $?
grep -o '"launch_ms": [0-9.]*' gpurun_out/ab_u8.log
echo "== product h16"; ACMMP_TEXEL=h16 timeout -k 10 120 python3 tools/quick_time.py 1600 1200 8 > gpurun_out/ab_h16.log 2>&1 || exit $?
grep -o '"launch_ms": [0-9.]*' gpurun_out/ab_h16.log
echo "== packed lerp u8"; ACMMP_LIB=$V timeout -k 10 120 python3 tools/quick_time.py 1600 1200 8 > gpurun_out/ab_pl.log 2>&1 || exit $?
grep -o '"launch_ms": [0-9.]*' gpurun_out/ab_pl.log
echo "== product u8 again"; timeout -k 10 120 python3 tools/quick_time.py 1600 1200 8 > gpurun_out/ab_u8b.log 2>&1 || exit $?
grep -o '"launch_ms": [0-9.]*' gpurun_out/ab_u8b.log
echo "== parity of packed lerp"
ACMMP_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep_views.py tests/test_gpu_headline.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pl_tests.log 2>&1; rc=$?
tail -3 gpurun_out/pl_tests.log
exit $rc
