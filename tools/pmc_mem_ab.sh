#!/bin/bash
# A/B memory-side traffic of library variants: FETCH_SIZE and WRITE_SIZE of
# every kernel in separate rocprofv3 --pmc passes of tools/quick_time.py
# (3 RunPatchMatch at 1600x1200, 8 iterations). Summarise with
# tools/pmc_ab.py gpurun_out/mem_*.
# usage: tools/pmc_mem_ab.sh name=path/to/lib.so [name=path ...]
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%=*}; lib=${spec#*=}
  for ctr in FETCH_SIZE WRITE_SIZE; do
    ACMMP_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --kernel-include-regex k_sweep --pmc $ctr -f csv -d gpurun_out/mem_$name/$ctr -o run -- \
      python3 tools/quick_time.py 1600 1200 8 > gpurun_out/mem_${name}_$ctr.log 2>&1
    rc=$?
    echo "$name $ctr rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
