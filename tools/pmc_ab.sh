#!/bin/bash
# A/B hardware counters of k_sweep for library variants: three rocprofv3 --pmc
# passes of tools/quick_time.py (3 RunPatchMatch at 1600x1200, 8 iterations)
# per library; summarise with tools/pmc_ab.py gpurun_out/ab_*.
# usage: tools/pmc_ab.sh name=path/to/lib.so[@VAR=value] [name=path ...]
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU GRBM_GUI_ACTIVE TD_TD_BUSY_sum TA_TA_BUSY_sum"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_ADDR_CONFLICT SQ_INSTS_VMEM_WR TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE"
# L1 (TCP) side: cache accesses (tag lookups) and misses to L2 per gather
P3="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_READ_sum TCP_PENDING_STALL_CYCLES_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE"
for spec in "$@"; do
  # name=lib[@VAR=value] (tools/ab.sh's syntax)
  name=${spec%%=*}; rest=${spec#*=}; lib=${rest%%@*}; envv=""; [ "$rest" != "$lib" ] && envv=${rest#*@}
  i=0
  for set in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    env ACMMP_LIB=$lib $envv timeout -k 10 120 rocprofv3 --kernel-trace --kernel-include-regex k_sweep --pmc $set -f csv -d gpurun_out/ab_$name/p$i -o run -- \
      python3 tools/quick_time.py 1600 1200 8 > gpurun_out/ab_${name}_p$i.log 2>&1
    rc=$?
    echo "$name pass $i rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
