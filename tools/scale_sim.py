"""Simulated N-rank cfg4 wall time from per-pass times measured on ONE GPU
("a simulated 8-rank cfg4 timing from the measured
per-view times (LPT plus the stream tail)").

Measured here (one MI355X, the synthetic cfg4 folder of pipeline_times.py):
  * every pass of acmmp_amd.distributed at world 1 with 2 views in flight
    (t_eff = pass compute / V: a view's share of the 2-stream throughput) and
    with 1 view in flight (t_alone = pass compute / V: a view alone on the
    GPU, what the odd view of a rank costs);
  * the row-band split (acmmp_amd.band) of one fine-scale view into N bands:
    each band's acmmp_run_patchmatch_band with its halo callback reduced to
    the stream synchronisation (the rows it would receive are stale; the
    time is that of a participant), the planar-prior rebuild on the full
    image included (every participant builds the prior), as a fraction of
    the unsplit run of the same view;
  * the host phases (decode, JBU, .dmb writes) and RunFusion in-process.

Modelled (stated in the output, not measured: one GPU cannot):
  * xGMI: halo exchange HALO_LATENCY_S per half-sweep (RCCL P2P of
    23 rows x Wh x 24 B, 0.44 MB at 1600 px), and all-gathers received at
    XGMI_GBPS per GPU;
  * host phases split evenly over the ranks except RunFusion (rank 0).

usage: python tools/scale_sim.py [views] [width] [height] [nsrc] [world] > gpurun_out/scale_sim.jsonl
The simulation itself (`simulate`) is a pure function, tested on CPU in
tests/test_scale_sim.py.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from acmmp_amd.distributed import lpt_assign, plan_views  # noqa: E402

HALO_LATENCY_S = 60e-6   # one RCCL P2P halo exchange (send + receive both neighbours)
XGMI_GBPS = 100.0        # all-gather bytes received per GPU per second (GB/s)


def _rank_time(n_whole: int, t_eff: float, t_alone: float) -> float:
    """A rank's whole views with 2 in flight: pairs at the 2-stream
    throughput, an odd last view alone."""
    return (n_whole // 2) * 2 * t_eff + (n_whole % 2) * t_alone


def simulate(passes: list, band: dict, host: dict, V: int, world: int, split_tail: bool,
             halo_latency_s: float = HALO_LATENCY_S, xgmi_gbps: float = XGMI_GBPS) -> dict:
    """passes: per pass {"kind": "planar"|"geom", "t_eff": s, "t_alone": s,
    "map_bytes": one view's depth map, "exchanges": halo exchanges of one
    view's run}; band: {kind: fraction of t_alone one band participant
    spends}; host: {"load": s, "jbu": s, "flush": s, "fusion": s,
    "image_bytes": all images of one scale summed}. Equal-cost views
    (cfg4). Returns the simulated wall time and its parts."""
    costs = [1.0] * V
    if split_tail:
        assignment, split = plan_views(costs, world, True)
    else:
        assignment, split = lpt_assign(costs, world), []
    whole = [[v for v in a if v not in split] for a in assignment]
    slots = max(len(a) for a in assignment)
    compute = ideal = exchange = 0.0
    for p in passes:
        t_rank = max(_rank_time(len(w), p["t_eff"], p["t_alone"]) for w in whole)
        t_split = len(split) * (band[p["kind"]] * p["t_alone"] + p["exchanges"] * halo_latency_s
                                + p["map_bytes"] * 5 / (xgmi_gbps * 1e9))  # band gather: planes + costs
        compute += t_rank + t_split
        ideal += V * p["t_eff"] / world
        # the depth all-gather: every rank receives the other ranks' padded slots
        exchange += slots * (world - 1) * p["map_bytes"] / (xgmi_gbps * 1e9)
    images = host["image_bytes"] * (world - 1) / world / (xgmi_gbps * 1e9)
    host_s = (host["load"] + host["jbu"] + host["flush"]) / world + images
    wall = compute + exchange + host_s + host["fusion"]
    return {"world": world, "split_tail": split_tail, "split_views": len(split),
            "views_per_rank": [len(a) for a in assignment],
            "compute_s": compute, "ideal_compute_s": ideal, "compute_efficiency": ideal / compute,
            "depth_allgather_s": exchange, "host_s": host_s, "fusion_s": host["fusion"], "wall_s": wall,
            "non_compute_share": (wall - compute) / wall,
            "non_compute_share_without_fusion": (exchange + host_s) / (compute + exchange + host_s)}


def _passes_of(log2: list, log1: list, V: int, band_exchanges: dict) -> list:
    out = []
    for a, b in zip(log2, log1):
        kind = "geom" if a["geom"] else "planar"
        h, w = a["shape"]
        out.append({"pass": a["pass"], "kind": kind, "shape": [h, w], "t_eff": a["compute_s"] / V,
                    "t_alone": b["compute_s"] / V, "map_bytes": h * w * 4,
                    "exchanges": band_exchanges[kind]})
    return out


def measure_bands(pipe, world: int, v: int = 0) -> dict:
    """One fine-scale view split into `world` bands (see the module doc)."""
    import torch
    from acmmp_amd.band import bands
    from acmmp_amd.distributed import engine_compute, engine_setup
    pipe._map([])
    eng = pipe.pool.engines[0]
    out = {}
    for kind, args in (("planar", (False, True, False, False)), ("geom", (True, False, False, True))):
        t = pipe._task(v, *args)
        H, W = t.images[0].shape
        whole = []
        for _ in range(2):
            pipe._sync()
            t0 = time.perf_counter()
            engine_compute(t, eng)
            whole.append(time.perf_counter() - t0)
        planes = torch.empty((H, W, 4), dtype=torch.float32, device=pipe.tdev)
        costs = torch.empty((H, W), dtype=torch.float32, device=pipe.tdev)
        n_ex = [0]

        def ex(halo):
            torch.cuda.ExternalStream(int(halo.stream), device=pipe.tdev).synchronize()
            n_ex[0] += 1

        per_band = []
        for lo, hi in bands(H, world):
            engine_setup(t, eng)
            eng.synchronize()
            t0 = time.perf_counter()
            for run in range(2 if t.planar else 1):
                if run:
                    eng.prepare_planar_prior()
                eng.run_band(lo, hi, ex)
                eng.export_results(planes.data_ptr(), costs.data_ptr(), 0)
                eng.synchronize()
            per_band.append(time.perf_counter() - t0)
        out[kind] = {"shape": [H, W], "whole_s": min(whole), "band_s": per_band,
                     "fraction": max(per_band) / min(whole), "exchanges": n_ex[0] // len(per_band)}
    pipe._shutdown()
    return out


def main():
    import torch
    from acmmp_amd import pipeline
    from acmmp_amd.distributed import ViewParallelPipeline
    from pipeline_times import write_cfg4_dense
    a = sys.argv
    V = int(a[1]) if len(a) > 1 else 49
    W = int(a[2]) if len(a) > 2 else 1600
    H = int(a[3]) if len(a) > 3 else 1200
    NSRC = int(a[4]) if len(a) > 4 else 20
    world = int(a[5]) if len(a) > 5 else 8

    def emit(**kw):
        print(json.dumps(kw), flush=True)

    tmp, dense = write_cfg4_dense(V, W, H, NSRC)
    runs = {}
    for c in (2, 1):
        t0 = time.perf_counter()
        pipe = ViewParallelPipeline(dense, f"/ACMMP_c{c}", device=0, concurrent_views=c)
        pipe.run()
        torch.cuda.synchronize()
        runs[c] = pipe
        emit(step=f"world1_concurrent{c}", s=round(time.perf_counter() - t0, 2),
             phases_s={k: round(v, 3) for k, v in sorted(pipe.phase_s.items())},
             passes=[{k: (round(x, 4) if isinstance(x, float) else x) for k, x in p.items()} for p in pipe.pass_log])
    band = measure_bands(runs[1], world)
    emit(step="band_split_one_view", world=world, **band)
    t0 = time.perf_counter()
    points = pipeline.run_fusion(dense, dense + "/ACMMP_c2")
    fusion_s = time.perf_counter() - t0
    emit(step="fusion_in_process", points=points, s=round(fusion_s, 2))
    ph = runs[2].phase_s
    image_bytes = sum(int(h) * int(w) * 4 for h, w in runs[2]._shapes().values())
    host = {"load": ph["load"], "jbu": ph.get("jbu", 0.0), "flush": ph.get("flush_writes", 0.0),
            "fusion": fusion_s, "image_bytes": image_bytes}
    passes = _passes_of(runs[2].pass_log, runs[1].pass_log, V, {k: b["exchanges"] for k, b in band.items()})
    fractions = {k: b["fraction"] for k, b in band.items()}
    for split_tail in (False, True):
        r = simulate(passes, fractions, host, V, world, split_tail)
        emit(step="simulated", model={"halo_latency_s": HALO_LATENCY_S, "xgmi_gbps": XGMI_GBPS},
             **{k: (round(x, 4) if isinstance(x, float) else x) for k, x in r.items()})
    import shutil
    shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
