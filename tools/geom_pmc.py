"""Summary of tools/geom_pmc.sh: the k_sweep dispatches of pass_times.py's
last repetition split into its photometric and geometric launches (160 each
at cfg2), per-launch means of every counter and the derived figures of
tools/pmc_ab.py, side by side.
usage: python tools/geom_pmc.py gpurun_out/geom_pmc"""
import csv
import glob
import sys
from collections import defaultdict

N = 160  # k_sweep launches per pass: 10 views x 8 iterations x 2 colours


def load(d):
    """{counter: [per-dispatch values in dispatch order]} per pass directory,
    with the kernel-trace durations as 'ms'."""
    out = defaultdict(list)
    for p in sorted(glob.glob(f"{d}/p*")):
        per = defaultdict(dict)
        for path in glob.glob(f"{p}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(path)):
                if "k_sweep" in r["Kernel_Name"]:
                    per[r["Counter_Name"]][int(r["Dispatch_Id"])] = float(r["Counter_Value"])
        for name, byd in per.items():
            if name not in out:
                out[name] = [byd[k] for k in sorted(byd)]
        if "ms" not in out:
            dur = {}
            for path in glob.glob(f"{p}/**/*kernel_trace.csv", recursive=True):
                for r in csv.DictReader(open(path)):
                    if "k_sweep" in r["Kernel_Name"]:
                        dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            out["ms"] = [dur[k] for k in sorted(dur)]
    return out


def derived(c):
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    gui = c.get("GRBM_GUI_ACTIVE", 1) / 8
    tw = c.get("TA_BUFFER_READ_WAVEFRONTS_sum", 0) or 1
    return {"VALU busy / wave-cycles": c.get("SQ_ACTIVE_INST_VALU", 0) / wc,
            "wait_any / wave-cycles": c.get("SQ_WAIT_ANY", 0) / wc,
            "wait_inst / wave-cycles": c.get("SQ_WAIT_INST_ANY", 0) / wc,
            "TD busy": c.get("TD_TD_BUSY_sum", 0) / (gui * 256),
            "TD cycles / gather": c.get("TD_TD_BUSY_sum", 0) / tw,
            "TCP accesses / gather": c.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0) / tw,
            "L1 misses / gather": c.get("TCP_TCC_READ_REQ_sum", 0) / tw}


def main():
    c = load(sys.argv[1])
    sides = {}
    for name, vals in c.items():
        if len(vals) < 2 * N:
            continue
        last = vals[-2 * N:]
        sides.setdefault("photometric", {})[name] = sum(last[:N]) / N
        sides.setdefault("geometric", {})[name] = sum(last[N:]) / N
    ph, ge = sides["photometric"], sides["geometric"]
    print(f"{'per k_sweep launch (cfg2, mean of 160)':40s} {'photometric':>14s} {'geometric':>14s} {'geo/photo':>10s}")
    for k in sorted(ph):
        r = ge[k] / ph[k] if ph[k] else float("nan")
        print(f"{k:40s} {ph[k]:14.5g} {ge[k]:14.5g} {r:10.3f}")
    dp, dg = derived(ph), derived(ge)
    for k in dp:
        print(f"{k:40s} {dp[k]:14.4f} {dg[k]:14.4f}")


if __name__ == "__main__":
    main()
