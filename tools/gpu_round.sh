#!/bin/bash
# One GPU call: parity suite, smoke, the default bench line (with its in-run
# counter passes and CPU baseline) and the rocprofv3 kernel-trace stats of a
# bench run. Every step has its own time limit; a test FAILURE (pytest rc 1)
# does not stop the later steps, anything else (fault, abort, time limit)
# ends the call there.
# Usage (on the GPU box): bash tools/gpu_round.sh [pytest selection...]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <timeout> <log> <ok-codes> <cmd...>
  local to=$1 log=$2 ok=$3; shift 3
  echo "=== $* (timeout $to)"
  timeout -k 10 "$to" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "=== rc=$rc"
  tail -n 6 "gpurun_out/$log"
  case " $ok " in *" $rc "*) ;; *) exit $rc ;; esac
}
sel=${*:-tests}
step 1500 tests.log "0 1" python -u -m pytest $sel -m gpu -v --timeout 120 --timeout-method thread
step 120 smoke.log "0" python -c "import __graft_entry__ as g; g.smoke()"
step 600 bench.log "0" python3 bench.py
grep '^{' gpurun_out/bench.log | tail -n 1 > gpurun_out/bench.json
step 400 prof.log "0" rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof -o run -- \
  python3 bench.py --steps 2 --warmup 1 --pmc off --no-cpu-baseline
exit 0
