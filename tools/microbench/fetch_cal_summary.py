"""Summary of tools/microbench/run_fetch_cal.sh: per pattern, the memory-side
read counters per 128-B line the pattern touches (mean of dispatches 2 and 3
of each pattern)."""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
timing = [json.loads(l) for l in open(os.path.join(d, "time.log")) if l.startswith("{")]
c = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
    rows = [r for r in csv.DictReader(open(f)) if "k_cal" in r["Kernel_Name"]]
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})
    pos = {x: k for k, x in enumerate(ids)}
    for r in rows:
        k = pos[int(r["Dispatch_Id"])]
        if k % 3:
            c[k // 3][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = []
for p in sorted(c):
    t = timing[p]
    lines = t["lines_touched"]
    row = {"pattern": p, "lines_touched": lines, "ms": t["ms"]}
    for n, v in sorted(c[p].items()):
        m = sum(v) / len(v)
        row[n + "_per_line"] = round(m / lines, 4) if n != "FETCH_SIZE" else None
        if n == "FETCH_SIZE":
            row["FETCH_SIZE_bytes_per_line"] = round(m * 1024 / lines, 2)
    out.append(row)
    print(json.dumps(row))
json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1)
