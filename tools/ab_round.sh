#!/bin/bash
# A/B of k_sweep launch time (tools/quick_time.py, photometric cfg2 view, 3
# runs each) for the product library, the product with ACMMP_TEXEL=h16, and
# each variant library given, then the core parity tests on every variant.
# Usage (on the GPU box): bash tools/ab_round.sh [variant.so ...]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
qt() {  # qt <log> [env...]
  local log=$1; shift
  env "$@" timeout -k 10 120 python3 tools/quick_time.py 1600 1200 8 > "gpurun_out/$log" 2>&1 || exit $?
  grep -o '"launch_ms": [0-9.]*' "gpurun_out/$log"
}
echo "== product u8"; qt ab_u8.log
echo "== product h16"; qt ab_h16.log ACMMP_TEXEL=h16
for v in "$@"; do echo "== $v"; qt "ab_$(basename "$v" .so).log" ACMMP_LIB="$v"; done
echo "== product u8 again"; qt ab_u8b.log
for v in "$@"; do
  echo "== parity of $v"
  ACMMP_LIB=$v timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep_views.py \
    tests/test_gpu_headline.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/ab_tests.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
