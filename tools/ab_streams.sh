#!/bin/bash
# bench.py (2 timed steps, photometric + geometric cfg2, no PMC, no CPU leg)
# at 1..4 engines (views in flight, one HIP stream each) per GPU.
set -o pipefail
mkdir -p gpurun_out
for n in "$@"; do
  echo "== streams $n"
  timeout -k 10 240 python3 bench.py --steps 2 --warmup 1 --pmc off --no-cpu-baseline --streams "$n" \
    > "gpurun_out/ab_streams_$n.log" 2>&1 || exit $?
  grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' "gpurun_out/ab_streams_$n.log"
done
