#!/bin/bash
# A/B of library variants on one GPU box (replaces round 4's ab_r4*.sh one-offs).
#
#   bash tools/ab.sh <mode> name=lib.so[@VAR=value] [name=lib.so[@VAR=value] ...]
#
# (@VAR=value sets one environment variable for that side, e.g.
# pipe=acmmp_amd/lib/libacmmp_amd.so@ACMMP_PIPE_FROM=99,99)
# Libraries are the product (acmmp_amd/lib/libacmmp_amd.so) or variants built
# in this container before the call by
#   make -C acmmp_amd/csrc variant NAME=<name> [REV=<commit>] [EXTRA="-D..."]
# (-> acmmp_amd/lib/variants/libacmmp_amd_<name>.so; DESIGN.md §5 names the
# command for each measured row). Modes, each run over the list twice,
# interleaved (A B A B), so drift on the shared box hits both sides:
#   pass    per-pass launch times (tools/pass_times.py) -> gpurun_out/ab_pass.jsonl
#   bench   bench.py, 2 timed steps, no counters, no CPU leg -> value / launch_ms
#   pmc     three rocprofv3 --pmc passes per library (tools/pmc_ab.sh), then
#           the side-by-side summary (tools/pmc_ab.py)
#   parity  the hot-path parity files with each library (ACMMP_LIB)
# Every GPU step has its own time limit; a fault, abort or time limit ends
# the call there.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
mode=$1; shift
# name=lib[@VAR=value] -> name, lib, envassign
split_spec() { name=${1%%=*}; rest=${1#*=}; lib=${rest%%@*}; envv=""; [ "$rest" != "$lib" ] && envv=${rest#*@}; }
[ $# -ge 1 ] || { echo "usage: tools/ab.sh pass|bench|pmc|parity name=lib.so ..."; exit 2; }
case "$mode" in
  pass)
    for round in 1 2; do
      for spec in "$@"; do
        split_spec "$spec"
        t=$(env ACMMP_LIB=$lib $envv timeout -k 10 150 python3 tools/pass_times.py 2)
        rc=$?; echo "{\"name\": \"$name\", \"round\": $round, \"t\": ${t:-null}}" >> gpurun_out/ab_pass.jsonl
        echo "pass $name round $round rc=$rc"; [ $rc -eq 0 ] || exit $rc
      done
    done
    cat gpurun_out/ab_pass.jsonl ;;
  bench)
    for round in 1 2; do
      for spec in "$@"; do
        split_spec "$spec"
        env ACMMP_LIB=$lib $envv timeout -k 10 240 python3 bench.py --steps 2 --warmup 1 --pmc off --no-cpu-baseline \
          > "gpurun_out/ab_bench_${name}_$round.log" 2>&1
        rc=$?; echo "bench $name round $round rc=$rc"; [ $rc -eq 0 ] || exit $rc
        grep -o '"value": [0-9.]*\|"launch_ms": [0-9.]*' "gpurun_out/ab_bench_${name}_$round.log" | tr '\n' ' '; echo
      done
    done ;;
  pmc)
    timeout -k 10 $((200 * $#)) bash tools/pmc_ab.sh "$@" || exit $?
    dirs=""; for spec in "$@"; do dirs="$dirs gpurun_out/ab_${spec%%=*}"; done
    timeout -k 10 120 python3 tools/pmc_ab.py $dirs ;;
  parity)
    for spec in "$@"; do
      split_spec "$spec"
      env ACMMP_LIB=$lib $envv timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py \
        tests/test_gpu_sweep_views.py tests/test_gpu_texel_modes.py tests/test_gpu_planar.py -m gpu -x -q \
        --timeout 200 --timeout-method thread > "gpurun_out/ab_parity_$name.log" 2>&1
      rc=$?; echo "parity $name rc=$rc"; tail -n 3 "gpurun_out/ab_parity_$name.log"
      [ $rc -eq 0 ] || exit $rc
    done ;;
  *) echo "unknown mode $mode"; exit 2 ;;
esac
