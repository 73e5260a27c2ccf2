#!/bin/bash
# Runs GPU steps in order; stops at the first step that faults, aborts, times
# out or segfaults (exit >= 124 or a signal), continuing past plain test
# failures (exit 1). Usage: tools/gpu_steps.sh "<timeout> <cmd>" ...
mkdir -p gpurun_out
i=0
for spec in "$@"; do
  i=$((i+1))
  to="${spec%% *}"; cmd="${spec#* }"
  echo "=== step $i (timeout $to): $cmd" | tee -a gpurun_out/steps.log
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/step$i.log" 2>&1
  rc=$?
  echo "=== step $i rc=$rc" | tee -a gpurun_out/steps.log
  tail -n 30 "gpurun_out/step$i.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -eq 137 ]; then
    echo "stopping after step $i (rc=$rc)"; exit $rc
  fi
done
exit 0
