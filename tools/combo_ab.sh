#!/bin/bash
# k_sweep launch time for texel form x row skew combinations (env only)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in "u8 0" "h16 16" "u8 16" "h16 0" "h16 1" "u8 1" "h16 4" "u8 0"; do
  set -- $c
  echo "== $1 skew $2"
  ACMMP_TEXEL=$1 ACMMP_PAD_SKEW=$2 timeout -k 10 120 python3 tools/quick_time.py 1600 1200 8 > gpurun_out/combo.log 2>&1 || exit $?
  grep -o '"launch_ms": [0-9.]*' gpurun_out/combo.log | tail -n 2 | tr '\n' ' '; echo
done
exit 0
