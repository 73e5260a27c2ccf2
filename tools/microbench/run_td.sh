#!/bin/bash
# TD cycles per gather wave-instruction for every td_gather pattern (one PMC pass)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 ./tools/microbench/td_gather > gpurun_out/td_time.log 2>&1 || exit $?
cat gpurun_out/td_time.log
timeout -s KILL 90 rocprofv3 --pmc TD_TD_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE -f csv -d gpurun_out/td -o run -- ./tools/microbench/td_gather > gpurun_out/td_pmc.log 2>&1 || exit $?
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/td/run_counter_collection.csv")))
d = collections.defaultdict(dict)
for r in rows:
    d[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
ids = sorted(d)
for k, i in enumerate(ids):
    if k % 3 == 2:
        c = d[i]
        print("pattern", k // 3, "TD cyc/inst %.1f" % (c["TD_TD_BUSY_sum"] / c["TA_BUFFER_READ_WAVEFRONTS_sum"]))
PY
