"""Per-launch k_sweep durations by launch index of a RunPatchMatch (colour
0/1 of iterations 0..7), from rocprofv3 --kernel-trace CSVs of
tools/quick_time.py (3 RunPatchMatch, 16 launches each; the mean over the
last two): shows whether a kernel change helps early (random planes) or late
(converged planes) iterations.

usage: python tools/launch_profile.py <trace dir> [<trace dir> ...]"""
import csv
import glob
import json
import os
import sys

for d in sys.argv[1:]:
    rows = []
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if "k_sweep" in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
    rows.sort()
    ms = [t for _, t in rows]
    runs = [ms[i:i + 16] for i in range(0, len(ms) - len(ms) % 16, 16)][1:]
    per = [round(sum(r[k] for r in runs) / len(runs), 3) for k in range(16)] if runs else []
    print(json.dumps({"dir": d, "launches": len(ms), "per_launch_ms": per,
                      "mean_ms": round(sum(per) / len(per), 3) if per else None}))
