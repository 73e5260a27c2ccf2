"""Summary of tools/sweep_pmc.sh: the k_sweep dispatches of pass_times.py's
last repetition split into its photometric and geometric launches
((nsrc + 1) views x 8 iterations x 2 colours each), per-launch means of every
counter, and the derived figures side by side; the last line is the same as
JSON (profiles/r06_*_pmc.json).

usage: python tools/sweep_pmc.py <dir with p1..p5> <nsrc> [W H]

Derived (per launch; GRBM_GUI_ACTIVE is summed over the 8 XCDs, one TD per CU,
256 CUs; SQ_ACTIVE_INST_VALU in quad-cycles summed over waves):
  TD busy                = TD_TD_BUSY_sum / (GUI / 8 * 256)
  VALU busy (SIMD)       = 4 * SQ_ACTIVE_INST_VALU / (GUI / 8 * 256 * 4)
  gathers                = TA_BUFFER_READ_WAVEFRONTS_sum (the source-image
                           buffer_load wave-instructions; nothing else in
                           k_sweep is a buffer load)
  flat reads / writes    = TA_FLAT_{READ,WRITE}_WAVEFRONTS_sum: scratch
                           (cost_array and spills), state and depth-map global
                           loads, state stores
  NCC calls / pixel-iter = gathers / SQ_WAVES / 36 (wave-level calls: a call
                           with some lanes masked counts once)
  non-gather share of L1 = (TCP accesses - gathers * accesses per gather) is
                           not separable from the counters alone; the bound
                           used: a coalesced dword per lane is
                           8 L1 accesses (one 64-B line per 8-lane group), so
                           8 x (flat reads + flat writes) of the TCP accesses
                           (an upper bound: float4 state loads are 2x that,
                           but they are < 3 % of the flat instructions)
  write amplification    = WRITE_SIZE / compulsory state writes (plane 16 +
                           cost 4 + selected views 4 B per pixel of the colour)
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def load(d):
    out = defaultdict(list)
    for p in sorted(glob.glob(f"{d}/p[0-9]")):
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


def derived(c, pixels_colour):
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    cyc = c.get("GRBM_GUI_ACTIVE", 1) / 8
    g = c.get("TA_BUFFER_READ_WAVEFRONTS_sum", 0) or 1
    fr = c.get("TA_FLAT_READ_WAVEFRONTS_sum", 0)
    fw = c.get("TA_FLAT_WRITE_WAVEFRONTS_sum", 0)
    tcp = c.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0) or 1
    compulsory = 24.0 * pixels_colour
    return {
        "ms_profiled": c.get("ms", 0),
        "VALU busy / wave-cycles": c.get("SQ_ACTIVE_INST_VALU", 0) / wc,
        "VALU busy (SIMD share)": 4 * c.get("SQ_ACTIVE_INST_VALU", 0) / (cyc * 256 * 4),
        "wait_any / wave-cycles": c.get("SQ_WAIT_ANY", 0) / wc,
        "wait_inst / wave-cycles": c.get("SQ_WAIT_INST_ANY", 0) / wc,
        "TD busy": c.get("TD_TD_BUSY_sum", 0) / (cyc * 256),
        "TD cycles / gather": c.get("TD_TD_BUSY_sum", 0) / g,
        "TCP accesses / gather": tcp / g,
        "L1 misses / gather": c.get("TCP_TCC_READ_REQ_sum", 0) / g,
        "gathers": g,
        "flat reads": fr,
        "flat writes": fw,
        "NCC calls / pixel-iter (wave-level)": g / (c.get("SQ_WAVES", 0) or 1) / 36,
        "non-gather L1 accesses bound": 8 * (fr + fw),
        "non-gather share of L1 accesses (bound)": 8 * (fr + fw) / tcp,
        "L1 write accesses": c.get("TCP_TOTAL_WRITE_sum", 0),
        "L1 write share of accesses": c.get("TCP_TOTAL_WRITE_sum", 0) / tcp,
        "write bytes": c.get("WRITE_SIZE", 0) * 1024,
        "compulsory write bytes": compulsory,
        "write amplification": c.get("WRITE_SIZE", 0) * 1024 / compulsory,
        "read bytes (2 x FETCH_SIZE)": 2 * c.get("FETCH_SIZE", 0) * 1024,
        "L2 hit rate": c.get("TCC_HIT_sum", 0) / ((c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0)) or 1),
    }


def main():
    d, ns = sys.argv[1], int(sys.argv[2])
    W = int(sys.argv[3]) if len(sys.argv) > 3 else 1600
    H = int(sys.argv[4]) if len(sys.argv) > 4 else 1200
    n = (ns + 1) * 8 * 2  # launches per pass
    c = load(d)
    sides = {"photometric": {}, "geometric": {}}
    for name, vals in c.items():
        if len(vals) < 2 * n:
            continue
        last = vals[-2 * n:]
        sides["photometric"][name] = sum(last[:n]) / n
        sides["geometric"][name] = sum(last[n:]) / n
    ph, ge = sides["photometric"], sides["geometric"]
    print(f"k_sweep_f<NS, u8> with nsrc {ns}, {W}x{H}: per launch, mean of {n}")
    print(f"{'counter':40s} {'photometric':>14s} {'geometric':>14s} {'geo/photo':>10s}")
    for k in sorted(ph):
        r = ge.get(k, 0) / ph[k] if ph[k] else float("nan")
        print(f"{k:40s} {ph[k]:14.5g} {ge.get(k, 0):14.5g} {r:10.3f}")
    pc = (W * H) // 2
    dp, dg = derived(ph, pc), derived(ge, pc)
    for k in dp:
        print(f"{k:40s} {dp[k]:14.5g} {dg[k]:14.5g}")
    print(json.dumps({"nsrc": ns, "W": W, "H": H, "launches_per_side": n, "counters": sides,
                      "derived": {"photometric": dp, "geometric": dg}}))


if __name__ == "__main__":
    main()
