#!/bin/bash
# td_pair.hip: TD cycles and TCP accesses per gather wave-instruction of
# dword quad gathers vs 64-bit pair-record gathers (+ masked fallbacks) on
# k_sweep's lane geometry; one PMC pass, 3 dispatches per (map, mode).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pair
B=./tools/microbench/td_pair
timeout -k 10 60 $B > gpurun_out/pair/time.log 2>&1 || exit $?
cat gpurun_out/pair/time.log
timeout -s KILL 90 rocprofv3 --pmc TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE -f csv -d gpurun_out/pair/pmc -o run -- $B > gpurun_out/pair/pmc.log 2>&1 || exit $?
python3 - <<'PY'
import csv, collections, glob, json
c = collections.defaultdict(dict)
for f in glob.glob("gpurun_out/pair/pmc/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_pair" in r["Kernel_Name"]:  # not the hipMemset fills
            c[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
out = []
for k, d in enumerate(sorted(c)):
    if k % 3 == 2:  # the third of each (map, mode)'s dispatches
        v = c[d]
        w = v["TA_BUFFER_READ_WAVEFRONTS_sum"]
        rec = {"map": k // 12, "mode": (k // 3) % 4, "gather_insts_M": round(w / 1e6, 3),
               "td_per_inst": round(v["TD_TD_BUSY_sum"] / w, 2),
               "tcp_per_inst": round(v["TCP_TOTAL_CACHE_ACCESSES_sum"] / w, 2),
               "td_total_M": round(v["TD_TD_BUSY_sum"] / 1e6, 2)}
        out.append(rec)
        print(json.dumps(rec))
json.dump(out, open("gpurun_out/pair/table.json", "w"), indent=1)
PY
