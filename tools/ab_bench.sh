#!/bin/bash
# bench.py (2 timed steps, photometric + geometric cfg2) per library
for lib in "$@"; do
  echo "== $lib"
  ACMMP_LIB=$lib timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --pmc off --no-cpu-baseline > gpurun_out/abb.log 2>&1 || exit $?
  grep -o '"value": [0-9.]*\|"launch_ms": [0-9.]*\|a launch spans [0-9.]* ms' gpurun_out/abb.log
done
