"""In-run hardware-counter passes of bench.py (rank 0, N=1).

bench.py calls `collect()` BEFORE it touches the GPU: each pass is a child
process `rocprofv3 --kernel-trace --pmc <counters> -- python3 bench.py
--pmc-child ...` that runs one bench step of the same workload on one engine
(one HIP stream), so every k_sweep dispatch is measured alone. Counters per
pass respect the gfx950 slot limits (TCC 4: FETCH_SIZE takes 3, WRITE_SIZE 2;
TA 2, TD 2, GRBM 2, SQ 8), so no pass asks for more than the hardware holds.

Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE / WRITE_SIZE are KiB at the
L2's memory side (Infinity-Cache hits included, so an upper bound on HBM
bytes); FETCH_SIZE reports half the bytes of wide coalesced streams on gfx950
and is doubled here (an upper bound again for this kernel's dword gathers).

Derived per k_sweep launch (mean over the step's launches):
  hbm_bytes      = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
  td_busy_frac   = TD_TD_BUSY_sum / (GRBM_GUI_ACTIVE / XCDS * CUS)
                   (GRBM_GUI_ACTIVE is summed over the 8 XCDs; one TD per CU)
  gather_insts   = TA_BUFFER_READ_WAVEFRONTS_sum (buffer_load wave-instructions)
  td_cyc_per_inst = TD_TD_BUSY_sum / gather_insts
  valu_busy_frac = 4 * SQ_ACTIVE_INST_VALU / (GRBM_GUI_ACTIVE / XCDS * CUS * 4)
                   (the counter is in quad-cycles summed over waves; 4 SIMDs per
                   CU, one VALU issue per SIMD: the share of SIMD cycles that
                   execute VALU, the second roofline of this kernel)
  valu_insts     = SQ_INSTS_VALU (wave-instructions)
  duration_ms    = kernel-trace end - start of the same dispatches (profiled;
                   bench.py reports its own un-profiled HIP-event duration too)
"""
from __future__ import annotations

import csv
import glob
import os
import signal
import statistics
import subprocess
import sys
import time

CUS = 256
XCDS = 8

PASSES = [
    ("fetch", ["FETCH_SIZE", "GRBM_GUI_ACTIVE", "TD_TD_BUSY_sum", "TA_BUFFER_READ_WAVEFRONTS_sum",
               "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS", "SQ_WAVES"]),
    ("write", ["WRITE_SIZE", "GRBM_GUI_ACTIVE", "TA_TA_BUSY_sum", "SQ_INSTS_VMEM_WR", "SQ_ACTIVE_INST_VALU",
               "SQ_INSTS_VALU", "TCP_TOTAL_CACHE_ACCESSES_sum", "TA_BUFFER_READ_WAVEFRONTS_sum"]),
    # L2 side: hit/miss, L1->L2 read requests, memory-side
    # read requests (all, and the 128-B ones), within the 4 TCC slots
    ("l2", ["TCC_HIT_sum", "TCC_MISS_sum", "TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_128B_sum", "TCP_TCC_READ_REQ_sum",
            "TA_BUFFER_READ_WAVEFRONTS_sum", "GRBM_GUI_ACTIVE"]),
]

# Memory-side read bytes, calibrated for dword gathers by
# tools/microbench/fetch_cal.hip (profiles/r05_fetch_cal.json): a 2 GiB
# buffer read with dwordx4 streams, dword streams and one dword per 128-B
# line, 64-B half line, 32-B sector or random line gives exactly one
# TCC_EA0_RDREQ_128B per touched 128-B line in every pattern, and FETCH_SIZE
# = 64 B per line: FETCH_SIZE tallies a 128-B request as 64 B whatever the
# access width. So read bytes = 128 x RDREQ_128B + 64 x the other requests
# (32-B requests are counted as 64 here: an upper bound; the fetch pass's
# FETCH_SIZE x 2 is the same figure when every request is 128 B).


def _run(cmd, log, timeout):
    """Child in its own process group; killed as a group on timeout."""
    with open(log, "w") as f:
        p = subprocess.Popen(cmd, stdout=f, stderr=subprocess.STDOUT, start_new_session=True)
        try:
            return p.wait(timeout=timeout)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
            return -9


def _counters(folder):
    per = {}
    for path in glob.glob(os.path.join(folder, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if "k_sweep" not in r["Kernel_Name"]:
                continue
            per.setdefault(r["Counter_Name"], {})[int(r["Dispatch_Id"])] = float(r["Counter_Value"])
    return per


def _durations(folder):
    out = []
    for path in glob.glob(os.path.join(folder, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if "k_sweep" in r["Kernel_Name"]:
                out.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    return out


def collect(bench_py: str, child_args: list, out_dir: str, timeout: float = 150.0) -> dict | None:
    """Runs the counter passes; returns the per-launch figures or None when
    rocprofv3 is absent or a pass fails (the bench line then says why)."""
    import shutil
    if shutil.which("rocprofv3") is None:
        return {"error": "rocprofv3 not found"}
    os.makedirs(out_dir, exist_ok=True)
    env_py = sys.executable or "python3"
    res = {"passes": {}}
    for name, counters in PASSES:
        d = os.path.join(out_dir, name)
        cmd = ["rocprofv3", "--kernel-trace", "--pmc", *counters, "-f", "csv", "-d", d, "-o", "run", "--",
               env_py, bench_py, "--pmc-child", *child_args]
        t0 = time.time()
        print(f"[bench] counter pass '{name}': {' '.join(counters)}", file=sys.stderr, flush=True)
        rc = _run(cmd, os.path.join(out_dir, f"{name}.log"), timeout)
        if rc != 0:
            return {"error": f"counter pass {name} exited {rc} (log {out_dir}/{name}.log)"}
        res["passes"][name] = {"counters": _counters(d), "durations_ms": _durations(d),
                               "wall_s": round(time.time() - t0, 1)}
        # the per-dispatch CSVs are read: drop them (tens of MB per pass; the
        # summary and the pass logs stay), so gpurun_out stays small enough
        # to come back from the box
        shutil.rmtree(d, ignore_errors=True)
    return summarize(res)


def summarize(res: dict) -> dict:
    f = res["passes"]["fetch"]["counters"]
    w = res["passes"]["write"]["counters"]
    l2 = res["passes"].get("l2", {}).get("counters", {})

    def mean(m, name):
        vals = list(m.get(name, {}).values())
        return statistics.mean(vals) if vals else float("nan")

    fetch_kib = mean(f, "FETCH_SIZE")
    write_kib = mean(w, "WRITE_SIZE")
    td_busy = mean(f, "TD_TD_BUSY_sum")
    gui = mean(f, "GRBM_GUI_ACTIVE")
    insts = mean(f, "TA_BUFFER_READ_WAVEFRONTS_sum")
    durs = res["passes"]["fetch"]["durations_ms"]
    launches = len(f.get("FETCH_SIZE", {}))
    cyc_per_cu = gui / XCDS
    return {
        "launches": launches,
        "fetch_bytes_raw": fetch_kib * 1024,
        "write_bytes": write_kib * 1024,
        "hbm_bytes": (2 * fetch_kib + write_kib) * 1024,
        "td_busy_frac": td_busy / (cyc_per_cu * CUS) if cyc_per_cu > 0 else float("nan"),
        "ta_busy_frac": mean(w, "TA_TA_BUSY_sum") / ((mean(w, "GRBM_GUI_ACTIVE") / XCDS) * CUS),
        "gather_insts": insts,
        "td_cyc_per_inst": td_busy / insts if insts > 0 else float("nan"),
        "vmem_rd_insts": mean(f, "SQ_INSTS_VMEM_RD"),
        "vmem_wr_insts": mean(w, "SQ_INSTS_VMEM_WR"),
        "lds_insts": mean(f, "SQ_INSTS_LDS"),
        "waves": mean(f, "SQ_WAVES"),
        "valu_insts": mean(w, "SQ_INSTS_VALU"),
        # one TD cycle per L1 access (profiles/r04_td_addressing.md)
        "tcp_accesses_per_gather": (mean(w, "TCP_TOTAL_CACHE_ACCESSES_sum") / mean(w, "TA_BUFFER_READ_WAVEFRONTS_sum")
                                    if mean(w, "TA_BUFFER_READ_WAVEFRONTS_sum") > 0 else float("nan")),
        "valu_busy_frac": 4 * mean(w, "SQ_ACTIVE_INST_VALU") / ((mean(w, "GRBM_GUI_ACTIVE") / XCDS) * CUS * 4),
        "gpu_cycles_per_xcd": cyc_per_cu,
        "profiled_ms": statistics.mean(durs) if durs else float("nan"),
        "clock_ghz": cyc_per_cu / (statistics.mean(durs) * 1e6) if durs else float("nan"),
        **l2_figures(l2, mean),
    }


def l2_figures(l2: dict, mean) -> dict:
    """Per-launch L2 figures of the 'l2' pass (empty when the pass is absent)."""
    if not l2:
        return {}
    hit, miss = mean(l2, "TCC_HIT_sum"), mean(l2, "TCC_MISS_sum")
    rdreq, r128 = mean(l2, "TCC_EA0_RDREQ_sum"), mean(l2, "TCC_EA0_RDREQ_128B_sum")
    gathers = mean(l2, "TA_BUFFER_READ_WAVEFRONTS_sum")
    out = {
        "l2_hit_rate": hit / (hit + miss) if hit + miss > 0 else float("nan"),
        "l2_hits": hit,
        "l2_misses": miss,
        "l1_to_l2_read_reqs": mean(l2, "TCP_TCC_READ_REQ_sum"),
        "l1_to_l2_reqs_per_gather": mean(l2, "TCP_TCC_READ_REQ_sum") / gathers if gathers > 0 else float("nan"),
        "ea_read_reqs": rdreq,
        "ea_read_reqs_128b": r128,
        "read_bytes_calibrated": 128.0 * r128 + 64.0 * (rdreq - r128),
    }
    return out
