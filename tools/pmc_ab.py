"""Summary of tools/pmc_ab.sh: per library variant, means over the k_sweep
dispatches of the last RunPatchMatch (16 launches) of each counter, plus
derived per-launch figures.
usage: python tools/pmc_ab.py gpurun_out/ab_<name> [...]"""
import csv, glob, sys
from collections import defaultdict


def load(d):
    per = defaultdict(dict)
    dur = {}
    for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            if "k_sweep" in r["Kernel_Name"]:
                per[r["Counter_Name"]][(path, int(r["Dispatch_Id"]))] = float(r["Counter_Value"])
    for path in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            if "k_sweep" in r["Kernel_Name"]:
                dur[(path, int(r["Dispatch_Id"]))] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    out = {}
    for name, byd in per.items():
        keys = sorted(byd)
        out[name] = sum(byd[k] for k in keys[-16:]) / 16
    ks = sorted(dur)
    out["ms"] = sum(dur[k] for k in ks[-16:]) / 16
    return out


for d in sys.argv[1:]:
    c = load(d)
    gui = c.get("GRBM_GUI_ACTIVE", 1) / 8
    print(f"== {d}: {c['ms']:.3f} ms/launch (profiled)")
    for k in sorted(c):
        print(f"   {k:32s} {c[k]:16.4g}")
    wc = c.get("SQ_WAVE_CYCLES", 0)
    if wc:
        print(f"   VALU busy / wave-cycles {c['SQ_ACTIVE_INST_VALU'] / wc:.3f}  LDS {c['SQ_ACTIVE_INST_LDS'] / wc:.3f}"
              f"  VMEM {c['SQ_ACTIVE_INST_VMEM'] / wc:.3f}  wait_any {c['SQ_WAIT_ANY'] / wc:.3f}  wait_inst {c['SQ_WAIT_INST_ANY'] / wc:.3f}")
    print(f"   TD busy {c.get('TD_TD_BUSY_sum', 0) / (gui * 256):.3f}  TA busy {c.get('TA_TA_BUSY_sum', 0) / (gui * 256):.3f}"
          f"  LDS conflict/idx {c.get('SQ_LDS_BANK_CONFLICT', 0) / max(c.get('SQ_LDS_IDX_ACTIVE', 1), 1):.3f}")
    tw = c.get("TA_BUFFER_READ_WAVEFRONTS_sum", 0)
    if tw and "TCP_TOTAL_CACHE_ACCESSES_sum" in c:
        print(f"   per buffer-read wave-instruction: TD cycles {c.get('TD_TD_BUSY_sum', 0) / tw:.2f}"
              f"  TCP accesses {c['TCP_TOTAL_CACHE_ACCESSES_sum'] / tw:.2f}"
              f"  L1 misses to L2 {c.get('TCP_TCC_READ_REQ_sum', 0) / tw:.2f}")
