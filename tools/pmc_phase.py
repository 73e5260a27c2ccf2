"""Summarise tools/pmc_deep.sh output: per-counter means of the k_sweep
dispatches of the LAST RunPatchMatch, split into the first iteration
(2 launches) and the last two iterations (4 launches).

usage: python tools/pmc_phase.py gpurun_out/pmcd1 gpurun_out/pmcd2 ...
"""
import csv
import glob
import sys
from collections import defaultdict


def main():
    early, late = defaultdict(list), defaultdict(list)
    for d in sys.argv[1:]:
        for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            per = defaultdict(dict)
            for r in csv.DictReader(open(path)):
                if "k_sweep" not in r["Kernel_Name"]:
                    continue
                per[r["Counter_Name"]][int(r["Dispatch_Id"])] = float(r["Counter_Value"])
            for name, byd in per.items():
                ids = sorted(byd)
                n = len(ids) // 3  # launches per RunPatchMatch
                last = ids[-n:]
                early[name] += [byd[i] for i in last[:2]]
                late[name] += [byd[i] for i in last[-4:]]
    for name in sorted(early):
        e = sum(early[name]) / len(early[name])
        l = sum(late[name]) / len(late[name])
        print(f"{name:40s} early {e:16.4g}   late {l:16.4g}")


if __name__ == "__main__":
    main()
