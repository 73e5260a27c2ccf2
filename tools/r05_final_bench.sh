#!/bin/bash
# Round 5 closing evidence (2/2): smoke, the default bench line (three
# counter passes + CPU baseline), and the rocprofv3 kernel-trace stats of a
# bench run (two views sharing the GPU, as timed).
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "150 python -c 'import __graft_entry__ as g; g.smoke()'" \
 "700 python3 bench.py > gpurun_out/bench.log 2>&1; grep ^{ gpurun_out/bench.log | tail -n 1 > gpurun_out/bench.json" \
 "400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof -o run -- python3 bench.py --steps 2 --warmup 1 --pmc off --no-cpu-baseline"
rm -rf gpurun_out/bench_pmc
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats.csv \;
rm -rf gpurun_out/prof
