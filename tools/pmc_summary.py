"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of k_sweep into
profiles/pmc_sweep.json (HBM-side bytes per launch, the roofline `traffic`).

Per MI355X_MICROARCH.md §HBM and cdna_hip_programming.md §7: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced stream, so the read side is doubled; both counters count at the L2's
memory side, so Infinity-Cache hits are included (an upper bound on HBM bytes).
Steady state = launches after the first 4 (cold caches excluded).

usage: python tools/pmc_summary.py <fetch_counter_collection.csv> <write_counter_collection.csv>
       <width> <height> <num_images> [out.json]
"""
import csv
import json
import statistics
import sys


def load(path, name):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == name and "k_sweep" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return [float(r["Counter_Value"]) for r in rows]


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    W, H, N = int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    out = sys.argv[6] if len(sys.argv) > 6 else "profiles/pmc_sweep.json"
    f_ss = statistics.mean(fetch[4:]) if len(fetch) > 4 else statistics.mean(fetch)
    w_ss = statistics.mean(write[4:]) if len(write) > 4 else statistics.mean(write)
    res = {
        "kernel": "k_sweep",
        "width": W,
        "height": H,
        "num_images": N,
        "launches": len(fetch),
        "fetch_size_kib_mean": f_ss,
        "write_size_kib_mean": w_ss,
        "fetch_bytes_raw": f_ss * 1024,
        "write_bytes": w_ss * 1024,
        "hbm_bytes_per_launch": (2 * f_ss + w_ss) * 1024,
        "note": "FETCH doubled per the gfx950 calibration for wide streams (upper bound for the dword "
                "gathers of this kernel); memory-side L2 counters include Infinity-Cache hits",
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
