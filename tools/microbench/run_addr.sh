#!/bin/bash
# Address form vs TA/TD/TCP cost (td_addr.hip): timing, then one PMC pass per
# counter group (rocprofv3 does not split counters over passes), then a table
# of counts per load wave-instruction for (shape, form).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/addr
B=./tools/microbench/td_addr
timeout -k 10 60 $B > gpurun_out/addr/time.log 2>&1 || exit $?
cat gpurun_out/addr/time.log
pass() {  # pass <name> <counters...>
  local n=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -f csv -d gpurun_out/addr/$n -o run -- $B > gpurun_out/addr/$n.log 2>&1 || exit $?
}
pass td TD_TD_BUSY_sum TD_LOAD_WAVEFRONT_sum GRBM_GUI_ACTIVE
pass ta TA_TA_BUSY_sum TA_TOTAL_WAVEFRONTS_sum
pass tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TOTAL_READ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TAGRAM0_REQ_sum
pass stall TA_ADDR_STALLED_BY_TD_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum
python3 - <<'PY'
import csv, collections, glob, json
c = collections.defaultdict(dict)
for f in glob.glob("gpurun_out/addr/*/run_counter_collection.csv"):
    rows = list(csv.DictReader(open(f)))
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})
    pos = {d: k for k, d in enumerate(ids)}
    for r in rows:
        c[pos[int(r["Dispatch_Id"])]][r["Counter_Name"]] = float(r["Counter_Value"])
forms = ["idxen", "offen", "flat", "global-saddr", "global-vaddr"]
insts = 4096 * 4 * 64 * 8
out = []
for k in sorted(c):
    if k % 3 != 2:
        continue
    shape, form = k // 15, (k // 3) % 5
    d = {n: v / insts for n, v in c[k].items() if n != "GRBM_GUI_ACTIVE"}
    d.update(shape=shape, form=forms[form])
    out.append(d)
    print(json.dumps(d))
json.dump(out, open("gpurun_out/addr/table.json", "w"), indent=1)
PY
