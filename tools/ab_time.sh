#!/bin/bash
# quick_time.py (3 RunPatchMatch at 1600x1200, 8 iterations, photometric) per
# library variant: usage tools/ab_time.sh lib1.so lib2.so ...
for lib in "$@"; do
  echo "== $lib"
  ACMMP_LIB=$lib timeout -k 10 120 python3 tools/quick_time.py 1600 1200 8 2>&1 | grep -o '"launch_ms": [0-9.]*' | tail -2
  rc=${PIPESTATUS[0]}
  if [ $rc -ne 0 ]; then exit $rc; fi
done
