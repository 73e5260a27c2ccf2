#!/bin/bash
# Row-skew A/B of the padded source records (ACMMP_PAD_SKEW records): the TD
# microbenchmark's pitch patterns, then k_sweep launch time per skew.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/microbench/run_td.sh | tail -n 9 || exit $?
for k in 0 1 4 8 16 24 0; do
  echo "== skew $k"
  ACMMP_PAD_SKEW=$k timeout -k 10 120 python3 tools/quick_time.py 1600 1200 8 > gpurun_out/skew_$k.log 2>&1 || exit $?
  grep -o '"launch_ms": [0-9.]*' gpurun_out/skew_$k.log | tail -n 2
done
exit 0
