#!/bin/bash
# Where does the geometric pass's extra time go? Three rocprofv3 --pmc passes
# (tools/pmc_ab.sh's counter sets) of tools/pass_times.py 1 (cfg2: 10 views,
# photometric then geometric pass, twice); tools/geom_pmc.py splits the last
# repetition's k_sweep dispatches into the 160 photometric and the 160
# geometric launches and prints both side by side.
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU GRBM_GUI_ACTIVE TD_TD_BUSY_sum TA_TA_BUSY_sum"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_ADDR_CONFLICT SQ_INSTS_VMEM_WR TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE"
P3="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_READ_sum TCP_PENDING_STALL_CYCLES_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE"
i=0
for set in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --kernel-include-regex k_sweep --pmc $set -f csv -d gpurun_out/geom_pmc/p$i -o run -- \
    python3 tools/pass_times.py 1 > gpurun_out/geom_pmc_p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 120 python3 tools/geom_pmc.py gpurun_out/geom_pmc > gpurun_out/geom_pmc.txt
rc=$?; cat gpurun_out/geom_pmc.txt; rm -rf gpurun_out/geom_pmc; exit $rc
