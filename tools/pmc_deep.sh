#!/bin/bash
# Per-dispatch PMC passes of quick_time.py (one RunPatchMatch x3 at 1600x1200,
# 8 iterations); summarise with tools/pmc_phase.py gpurun_out/pmcd*.
# Usage: tools/pmc_deep.sh [iters]
export TMPDIR=/tmp
it=${1:-8}
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCP_LATENCY_sum" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
           "TA_BUSY_avr TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum" \
           "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU TCP_TCR_TCP_STALL_CYCLES_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-include-regex k_sweep --pmc $set -f csv -d gpurun_out/pmcd$i -o run -- python3 tools/quick_time.py 1600 1200 $it > gpurun_out/pmcd$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
