#!/bin/bash
# Timing-only diagnostic builds (results are NOT valid): k_sweep launch time
# with the source gathers replaced by index arithmetic (ACMMP_DIAG_NOGATHER)
# or the sample loop's LDS reads removed (ACMMP_DIAG_NOLDS), beside the product.
# Usage (on the GPU box): bash tools/diag_time.sh variant.so ...
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "" "$@" ""; do
  echo "== ${v:-product}"
  if [ -n "$v" ]; then export ACMMP_LIB=$v; else unset ACMMP_LIB; fi
  timeout -k 10 120 python3 tools/quick_time.py 1600 1200 8 > gpurun_out/diag.log 2>&1 || exit $?
  grep -o '"launch_ms": [0-9.]*' gpurun_out/diag.log | tail -n 2 | tr '\n' ' '; echo
done
exit 0
