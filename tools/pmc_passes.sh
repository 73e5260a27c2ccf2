export TMPDIR=/tmp
i=0
for set in "VALUBusy VALUUtilization" "TA_BUSY_avr TD_TD_BUSY_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum" "MemUnitStalled OccupancyPercent"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set -f csv -d gpurun_out/pmc$i -o run -- python3 tools/quick_time.py 1600 1200 2 > gpurun_out/pmc$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
