#!/bin/bash
# fetch_cal.hip: L2 memory-side read counters against known line counts
# (three PMC passes, each within gfx950's 4 TCC slots), then the summary.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/fetch_cal
B=./tools/microbench/fetch_cal
timeout -k 10 60 $B > gpurun_out/fetch_cal/time.log 2>&1 || exit $?
cat gpurun_out/fetch_cal/time.log
P1="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
P2="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum TCC_REQ_sum TCP_TCC_READ_REQ_sum"
P3="FETCH_SIZE TCC_BUBBLE_sum"
i=0
for set in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set -f csv -d gpurun_out/fetch_cal/p$i -o run -- $B \
    > gpurun_out/fetch_cal/p$i.log 2>&1 || exit $?
done
python3 tools/microbench/fetch_cal_summary.py gpurun_out/fetch_cal
