#!/bin/bash
# Round-end evidence in one GPU call: parity tests, smoke, the PMC traffic
# passes of bench.py's k_sweep (FETCH_SIZE / WRITE_SIZE, one run each),
# their summary into profiles/pmc_sweep.json (read by bench.py as
# roofline.traffic), the bench line, and the rocprofv3 kernel-trace stats of
# the same bench command. Outputs land in gpurun_out/; copy the ones to keep
# into profiles/<round>_*. Stops at the first failing step.
# Usage (on the GPU box): bash tools/refresh_profiles.sh
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <timeout> <log> <cmd...>
  local to=$1 log=$2; shift 2
  echo "=== $* (timeout $to)"
  timeout -k 10 "$to" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "=== rc=$rc"
  tail -n 4 "gpurun_out/$log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step 600 tests.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step 120 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
step 240 pmc_fetch.log rocprofv3 --pmc FETCH_SIZE -f csv -d gpurun_out/pmc_fetch -o run -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
step 240 pmc_write.log rocprofv3 --pmc WRITE_SIZE -f csv -d gpurun_out/pmc_write -o run -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
step 60 pmc_summary.log python3 tools/pmc_summary.py gpurun_out/pmc_fetch/run_counter_collection.csv \
  gpurun_out/pmc_write/run_counter_collection.csv 1600 1200 10 profiles/pmc_sweep.json
cp profiles/pmc_sweep.json gpurun_out/pmc_sweep.json
step 300 bench.log python3 bench.py --steps 3 --warmup 1
grep '^{' gpurun_out/bench.log | tail -n 1 > gpurun_out/bench.json
step 300 prof.log rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof -o run -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline
exit 0
