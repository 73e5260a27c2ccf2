#!/bin/bash
# td_rule.hip: TCP accesses and TD cycles per gather wave-instruction by lane
# -> line sharing pattern (one PMC pass each, 3 dispatches per pattern).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rule
B=./tools/microbench/td_rule
timeout -k 10 60 $B > gpurun_out/rule/time.log 2>&1 || exit $?
cat gpurun_out/rule/time.log
timeout -s KILL 90 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TOTAL_READ_sum TA_BUFFER_READ_WAVEFRONTS_sum -f csv -d gpurun_out/rule/tcp -o run -- $B > gpurun_out/rule/tcp.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TD_TD_BUSY_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE -f csv -d gpurun_out/rule/td -o run -- $B > gpurun_out/rule/td.log 2>&1 || exit $?
python3 - <<'PY'
import csv, collections, glob, json
c = collections.defaultdict(dict)
for f in glob.glob("gpurun_out/rule/*/run_counter_collection.csv"):
    rows = list(csv.DictReader(open(f)))
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})
    pos = {d: k for k, d in enumerate(ids)}
    for r in rows:
        c[pos[int(r["Dispatch_Id"])]][r["Counter_Name"]] = float(r["Counter_Value"])
insts = 4096 * 4 * 64 * 8
out = []
for k in sorted(c):
    if k % 3 == 2:
        d = {n: round(v / insts, 3) for n, v in c[k].items() if n != "GRBM_GUI_ACTIVE"}
        d["pattern"] = k // 3
        out.append(d)
        print(json.dumps(d))
json.dump(out, open("gpurun_out/rule/table.json", "w"), indent=1)
PY
