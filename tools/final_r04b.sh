#!/bin/bash
# Round-4 closing evidence after the latency fixes (geometric fetches ahead,
# batched searches): smoke, the default bench line (counter passes + CPU
# baseline), the rocprofv3 kernel-trace stats of a bench run, and the
# per-pass kernel split on one stream.
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "150 python -c 'import __graft_entry__ as g; g.smoke()'" \
 "600 python3 bench.py > gpurun_out/bench.log 2>&1; grep ^{ gpurun_out/bench.log | tail -n 1 > gpurun_out/bench.json" \
 "400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof -o run -- python3 bench.py --steps 2 --warmup 1 --pmc off --no-cpu-baseline" \
 "200 python3 tools/pass_times.py 3 > gpurun_out/pass_times.json"
