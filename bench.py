#!/usr/bin/env python3
"""PatchMatch throughput benchmark (BASELINE.json metric) on 1..N MI355X.

Workload (BASELINE.json configs[1], "cfg2"): per GPU, 10 reference views at
1600x1200, each with its 9 nearest source views (N = 10 images per problem),
8 PatchMatch iterations, a photometric pass over the GPU's views, an RCCL
all-gather of the depth maps, then a geometric-consistency pass over the same
views (it reads the neighbours' depth maps: the real exchange step).

One "step" = photometric pass + all-gather + geometric pass, run by
`acmmp_amd.resident` (the same code the parity test
tests/test_gpu_headline.py drives): images, plane/cost state and depth maps
stay in HBM, every RunPatchMatch's results are exported device-to-device.
Weak scaling: every rank owns one copy of the 10-view cfg2 scene (global
view ids rank*10 + k), so per-GPU work is identical for every N. Sources span
ranks as the reference's pair lists span views (src/ACMMP.cpp:619-634): source
j of view (r, k) is scene view pairs[k][j] as held by rank (r + 1 + j) mod N,
and every view has its own Philox key (1234 + global id, as the pass drivers
key seed + ref_image_id), so the copies' depth maps differ and each geometric
pass reads other ranks' gathered maps (at N = 1 every source is the rank's
own view, as before).

value = RunPatchMatch pixels processed by all ranks (2 passes x views x W x H)
/ max-over-ranks wall time of the K timed steps, in Mpix/s (per pass; a
reference view's photometric + geometric result is value / 2).

Rank 0 at N=1 also runs, BEFORE touching the GPU, two rocprofv3 counter
passes of one step (tools/bench_pmc.py) for the roofline block, and after the
timed region the CPU oracle on a bounded sample (cpu_baseline).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

BASELINE_METRIC = "Mpixels/sec PatchMatch (1600×1200, 8 iters) at 1/2/4/8 GPUs; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def logical_bytes_per_pixel_iter(num_images: int, geom: bool) -> int:
    """SURVEY §8d / BASELINE.md §3 gather-byte model per pixel-iteration:
    14*(N-1) NCC calls x 724 B + 572 B of state, + 14*(N-1)*4 B in geometric
    passes. Logical bytes (counted as if nothing were cached)."""
    b = 14 * (num_images - 1) * 724 + 572
    if geom:
        b += 14 * (num_images - 1) * 4
    return b


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--views", type=int, default=10, help="reference views per GPU")
    ap.add_argument("--nsrc", type=int, default=9)
    ap.add_argument("--width", type=int, default=1600)
    ap.add_argument("--height", type=int, default=1200)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", default="800x600", help="ref-view crop timed on the CPU oracle")
    ap.add_argument("--streams", type=int, default=2,
                    help="engines (HIP streams) per GPU running different views concurrently")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend (nccl = RCCL over xGMI; gloo only to test on one GPU)")
    ap.add_argument("--pmc", default="auto", choices=["auto", "off"],
                    help="in-run rocprofv3 counter passes for the roofline (rank 0, N=1)")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    # tests only (tests/test_gpu_bench_exchange.py): one process holding the
    # views of every rank of a world of this size, no collective; and the
    # final state of every owned view saved as .npy files
    ap.add_argument("--emulate-ranks", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--dump", default="", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


VIEW_SEED = 1234  # Philox key of global view g: VIEW_SEED + g (acmmp_params.seed_lo)


def view_sources(k: int, rank: int, world: int, views: int, pairs, nsrc: int) -> list:
    """Global source ids of reference view k of `rank`: source j is scene
    view pairs[k][j] as held by rank (rank + 1 + j) mod world, so a rank's
    geometric pass reads the gathered depth maps of the other ranks (the
    reference's source lists span views, src/ACMMP.cpp:619-634; at world 1
    every source is the rank's own copy)."""
    return [((rank + 1 + j) % world) * views + pairs[k][j] for j in range(nsrc)]


def host_cpu():
    model = platform.processor() or ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    return model, os.cpu_count() or 1, avail


def main():
    args = parse()
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    rank_env = int(os.environ.get("RANK", "0"))
    pmc = None
    if args.pmc == "auto" and not args.pmc_child and "WORLD_SIZE" not in os.environ:
        # counter passes first: child processes, before this process touches the GPU
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import bench_pmc
        child = ["--views", str(args.views), "--nsrc", str(args.nsrc), "--width", str(args.width),
                 "--height", str(args.height), "--iters", str(args.iters), "--steps", "1", "--warmup", "0"]
        pmc = bench_pmc.collect(os.path.abspath(__file__), child, os.path.join(ROOT, "gpurun_out", "bench_pmc"))

    import torch
    import torch.distributed as dist

    world, rank = world_env, rank_env
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    dev_index = local_rank % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    backend = args.backend
    # launched by torch.distributed.run (WORLD_SIZE in the env): a process
    # group even at world size 1, so the RCCL all-gather runs in every case
    distributed = "WORLD_SIZE" in os.environ and not args.pmc_child
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)

    from acmmp_amd import default_params, scene
    from acmmp_amd.resident import EnginePool, ResidentViews, geometric_view, photometric_view

    if args.views < args.nsrc + 1:
        raise SystemExit(f"--views {args.views} cannot supply {args.nsrc} source views per problem")
    streams = 1 if args.pmc_child else args.streams
    emulate = args.emulate_ranks if (args.emulate_ranks > 1 and not distributed) else 0
    views_world = emulate or world  # ranks whose views the global view set holds
    V = args.views * views_world
    W, H = args.width, args.height
    setup = scene.scene_setup(num_views=args.views, width=W, height=H)
    here = range(emulate) if emulate else [rank]  # the ranks whose views this process owns
    mine = [r * args.views + k for r in here for k in range(args.views)]
    srcs = {r * args.views + k: view_sources(k, r, views_world, args.views, setup.pairs, args.nsrc)
            for r in here for k in range(args.views)}
    # a rank's copy of scene view m and every other rank's copy are the same
    # image and camera (one rendered tensor per scene view, shared by ids)
    rendered = {k: scene.render_torch(setup, k, device) for k in range(args.views)}
    needed = sorted(set(mine) | {i for v in mine for i in srcs[v]})
    images = {g: rendered[g % args.views] for g in needed}
    cams = {g: setup.camera(g % args.views) for g in needed}
    torch.cuda.synchronize()

    n_img = 1 + args.nsrc
    pool = EnginePool(dev_index, streams, timing=True)
    rv = ResidentViews(pool, cams, images, srcs, mine, H, W, total_views=V if distributed else None,
                       view_seed=VIEW_SEED)
    all_depth = rv.all_depth
    photo_params = default_params()
    photo_params.max_iterations = args.iters
    geom_params = default_params()
    geom_params.max_iterations = args.iters  # BASELINE cfg2: 8 iterations in both passes
    geom_params.geom_consistency = 1
    work = list(enumerate(mine))

    phase_s = {"photometric": 0.0, "exchange": 0.0, "geometric": 0.0}

    def step():
        # every pass ends with its views' streams synchronised (EnginePool.finish),
        # so the host clock between the phases times them without extra waits
        t0 = time.perf_counter()
        rv.photometric_pass(photo_params)
        t1 = time.perf_counter()
        if distributed:
            if backend == "nccl":  # RCCL over xGMI, device buffers
                dist.all_gather_into_tensor(rv.all_depth, rv.my_depth)
            else:  # gloo (tests on one GPU): staged through host memory
                host = torch.empty((V, H, W), dtype=torch.float32)
                dist.all_gather_into_tensor(host, rv.my_depth.cpu())
                rv.all_depth.copy_(host)
            # the engines' streams do not wait on torch's/RCCL's: finish the
            # gather before a geometric view borrows all_depth
            torch.cuda.synchronize()
        t2 = time.perf_counter()
        rv.geometric_pass(geom_params)
        t3 = time.perf_counter()
        phase_s["photometric"] += t1 - t0
        phase_s["exchange"] += t2 - t1
        phase_s["geometric"] += t3 - t2

    for _ in range(args.warmup):
        step()
    pool.reset_timing()
    for k in phase_s:
        phase_s[k] = 0.0
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    mine_row = [elapsed, phase_s["photometric"], phase_s["exchange"], phase_s["geometric"], float(len(mine))]
    rows = [mine_row]
    if distributed and world > 1:
        # every rank's own times (the headline takes the max of the walls)
        tt = torch.tensor(mine_row, dtype=torch.float64, device=device if backend == "nccl" else "cpu")
        gathered = [torch.empty_like(tt) for _ in range(world)]
        dist.all_gather(gathered, tt)
        rows = [[float(x) for x in g.cpu().tolist()] for g in gathered]
        elapsed = max(r[0] for r in rows)
    timed_ms, timed_launches = pool.sweep_ms, pool.sweep_launches
    if args.dump:
        # final state of every owned view: the geometric pass's planes and
        # costs, and the photometric depth maps the exchange carried
        os.makedirs(args.dump, exist_ok=True)
        for k, v in enumerate(mine):
            np.save(os.path.join(args.dump, f"geom_planes_{v:03d}.npy"), rv.planes[k].cpu().numpy())
            np.save(os.path.join(args.dump, f"geom_costs_{v:03d}.npy"), rv.costs[k].cpu().numpy())
            np.save(os.path.join(args.dump, f"photo_depth_{v:03d}.npy"), rv.my_depth[k].cpu().numpy())
    if args.pmc_child or emulate:
        pool.close()
        return

    # one photometric + one geometric view alone on one stream: the
    # un-overlapped duration of a k_sweep launch (HIP events on the engine's
    # stream), the denominator of the roofline fractions
    iso_pool = EnginePool(dev_index, 1, timing=True)
    eng = iso_pool.engines[0]
    k0, v0 = work[0]
    ids0 = [v0] + srcs[v0]
    photometric_view(iso_pool, eng, photo_params, [cams[i] for i in ids0], [images[i].data_ptr() for i in ids0],
                     rv.planes[k0].data_ptr(), rv.costs[k0].data_ptr(), rv.my_depth[k0].data_ptr())
    geometric_view(iso_pool, eng, geom_params, [cams[i] for i in ids0], [images[i].data_ptr() for i in ids0],
                   [all_depth[i].data_ptr() for i in ids0], rv.planes[k0].data_ptr(), rv.costs[k0].data_ptr())
    iso_ms = iso_pool.sweep_ms / max(iso_pool.sweep_launches, 1)
    iso_pool.close()

    pix_total = 2 * args.views * world * W * H * args.steps
    value = pix_total / elapsed / 1e6
    P = W * H
    logical = (P / 2) * (logical_bytes_per_pixel_iter(n_img, False) + logical_bytes_per_pixel_iter(n_img, True)) / 2
    result = {
        "metric": BASELINE_METRIC,
        "value": round(value, 4),
        "unit": "Mpix/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded analytic scene rendered into HBM; no DTU data offline)",
        "config": {
            "workload": f"cfg2: {args.views} ref views/GPU at {W}x{H}, {n_img} images/problem, "
                        f"{args.iters} iters, photometric + "
                        + (f"{'RCCL' if backend == 'nccl' else 'gloo'} depth all-gather + " if distributed else "")
                        + "geometric pass",
            "geom_iters_note": f"the geometric pass runs {args.iters} iterations as BASELINE cfg2 states; the "
                               "reference's SetGeomConsistencyParams forces 2 (src/ACMMP.cpp:447-454)",
            "views_per_gpu": args.views,
            "sources": "source j of view (rank r, k) = scene view pairs[k][j] held by rank (r + 1 + j) mod N "
                       "(cross-rank reads in every geometric pass at N > 1); Philox key 1234 + global view id",
            "width": W,
            "height": H,
            "num_images": n_img,
            "iters": args.iters,
            "parallelism": f"view-parallel x{world} (one process per GPU, "
                           f"{('RCCL' if backend == 'nccl' else 'gloo') if distributed else 'no'} "
                           f"all-gather of depth maps between the passes; {streams} views in flight per GPU on "
                           f"{streams} HIP streams)",
            "value_counts": "RunPatchMatch pixels (2 passes per view); per reference view (photometric + "
                            f"geometric) = {value / 2:.2f} Mpix/s",
            "residency": "images, state and depth maps stay in HBM; results exported device-to-device "
                         "(no per-run D2H copy as in the reference's RunPatchMatch, src/ACMMP.cu:1453-1454)",
            "ranks": rank_fields(rows, args.steps,
                                 ("RCCL" if backend == "nccl" else "gloo") if distributed else None),
        },
        "roofline": roofline(pmc, iso_ms, logical, timed_ms, timed_launches, streams, num_images=n_img,
                             pixels_per_launch=P / 2),
    }

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args, setup, images, cams, srcs, mine, all_depth, value)
    if rank == 0:
        print(json.dumps(result), flush=True)
    pool.close()
    if distributed:
        dist.destroy_process_group()


def rank_fields(rows, steps, exchange):
    """Per-rank attribution of the timed region: each row is
    one rank's [wall s, photometric s, depth all-gather s, geometric s,
    views], summed over the timed steps. Reports the spread of the pass
    times over ranks, the all-gather's ms per step and each rank's view
    count; the headline `value` is unchanged (max-over-ranks wall)."""
    walls = [r[0] for r in rows]
    passes = [r[1] + r[3] for r in rows]
    gather_ms = [r[2] / steps * 1e3 for r in rows]
    return {
        "world": len(rows),
        "views_per_rank": [int(r[4]) for r in rows],
        "wall_s": {"min": round(min(walls), 4), "max": round(max(walls), 4)},
        "pass_s_per_step": {"min": round(min(passes) / steps, 4), "max": round(max(passes) / steps, 4)},
        "photometric_s_per_step": [round(r[1] / steps, 4) for r in rows],
        "geometric_s_per_step": [round(r[3] / steps, 4) for r in rows],
        "depth_allgather_ms_per_step": ({"min": round(min(gather_ms), 3), "max": round(max(gather_ms), 3),
                                         "backend": exchange} if exchange else None),
        "note": "host clock around each phase of every timed step on every rank (the passes end synchronised); "
                "pass = photometric + geometric; the all-gather time includes waiting for the slowest rank",
    }


def performed_bytes_per_pixel_iter(ncc_calls: float, geom: bool) -> float:
    """The §8d byte model with the NCC calls the kernel actually performs per
    pixel-iteration in place of the model's 14 (N-1)."""
    return ncc_calls * (724 + (4 if geom else 0)) + 572


def roofline(pmc, iso_ms, logical_bytes, timed_ms, timed_launches, streams, num_images=10,
             pixels_per_launch=800 * 1200):
    """The dominant kernel's roofline (k_sweep, >90 % of the step's GPU time),
    in the contract's form: bound "hbm", achieved = ALGORITHMIC bytes per
    launch (SURVEY §8d's gather-byte model: every NCC sample's texels counted
    as if uncached) / launch time, peak = 8 TB/s, traffic = the HBM bytes the
    PMC counters see per launch. The model counts L1-served gathers, so frac
    exceeds 1 and `traffic` is far below the algorithmic bytes: the kernel is
    not HBM-bound. What binds it is reported beside it: the texture-data (TD)
    path that serves the gathers (`binding_unit`: TD busy fraction, one TD
    cycle per L1 cache access, profiles/r04_td_addressing.md), the VALU
    (`valu`) and the physical HBM fraction (`hbm_physical`). Durations: the
    un-overlapped HIP-event time of one launch (iso_ms, one stream);
    rocprofv3's profiled duration is in `pmc`."""
    achieved = logical_bytes / (iso_ms / 1e3) / 1e9
    out = {
        "bound": "hbm",
        "kernel": "k_sweep (CheckerboardPropagation)",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "frac_is_algorithmic": True,
        "frac_note": "algorithmic (L1-served) bytes over the HBM peak, not an HBM utilisation: see "
                     "hbm_physical_frac (PMC bytes) and binding_unit / valu for what binds the kernel",
        "hbm_physical_frac": None,
        "traffic": None,
        "algorithmic_bytes_per_launch": round(logical_bytes),
        "model": "SURVEY §8d / BASELINE.md §3: per pixel-iteration 14 (N-1) NCC x 724 B + 572 B state "
                 "(+ 14 (N-1) x 4 B geometric), P/2 pixels per launch, photometric/geometric mean; "
                 "frac > 1 = served from L1, not HBM",
        "launch_ms": round(iso_ms, 3),
        "launch_ms_note": "HIP events on the engine stream, one launch alone (one photometric + one geometric "
                          "view on one stream after the timed region); in the timed region "
                          f"{streams} views share the GPU and a launch spans "
                          f"{timed_ms / max(timed_launches, 1):.3f} ms",
    }
    if not pmc or "error" in pmc:
        out["pmc"] = (pmc or {}).get("error", "counter passes skipped")
        return out
    clock_hz = pmc["clock_ghz"] * 1e9
    insts = pmc["gather_insts"]
    hbm_gbs = pmc["hbm_bytes"] / (iso_ms / 1e3) / 1e9
    out.update({
        "hbm_physical_frac": round(hbm_gbs / HBM_PEAK_GBS, 4),
        "traffic": round(pmc["hbm_bytes"]),
        "traffic_note": "(2 x FETCH_SIZE + WRITE_SIZE) KiB x 1024 per launch, memory side of L2 (Infinity-Cache "
                        "hits included), FETCH doubled per the gfx950 calibration",
        "hbm_physical": {
            "achieved": round(hbm_gbs, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(hbm_gbs / HBM_PEAK_GBS, 4),
        },
        "binding_unit": {
            "bound": "td-gather",
            "achieved": round(insts / (iso_ms / 1e3) / 1e9, 2),
            "peak": round(256 * clock_hz / pmc["td_cyc_per_inst"] / 1e9, 2),
            "unit": "Ginst/s",
            "frac": round(pmc["td_busy_frac"], 4),
            "td_cycles_per_gather": round(pmc["td_cyc_per_inst"], 2),
            "l1_accesses_per_gather": (round(pmc["tcp_accesses_per_gather"], 2)
                                       if pmc.get("tcp_accesses_per_gather") == pmc.get("tcp_accesses_per_gather")
                                       else None),
            "model": "achieved = TA_BUFFER_READ_WAVEFRONTS_sum per launch / launch_ms; peak = 256 CUs x clock "
                     "(GRBM_GUI_ACTIVE/8 / profiled duration) / (TD_TD_BUSY_sum / TA_BUFFER_READ_WAVEFRONTS_sum); "
                     "frac = TD_TD_BUSY_sum / (256 x GRBM_GUI_ACTIVE/8)",
        },
        "valu": {
            "bound": "valu",
            "frac": round(pmc["valu_busy_frac"], 4),
            "insts": round(pmc["valu_insts"]),
            "note": "share of SIMD cycles issuing VALU (4 x SQ_ACTIVE_INST_VALU quad-cycles / (1024 SIMDs x "
                    "GRBM_GUI_ACTIVE/8))",
        },
        "pmc": {k: (round(v, 4) if isinstance(v, float) else v) for k, v in pmc.items()},
    })
    # The model counts 14 (N-1) NCC calls per pixel-iteration, as the
    # reference computes them; the product skips the calls of views with a
    # zero sampled weight (the reference multiplies their cost by 0 and adds
    # it, src/ACMMP.cu:747-751, :1083-1089), so it performs fewer: measured as
    # gather wave-instructions / waves / 36 samples (wave-level calls: a call
    # with some lanes masked counts once, so this is an upper bound on the
    # per-pixel calls performed).
    waves = pmc.get("waves") or 0
    if waves > 0 and insts > 0:
        calls = insts / waves / 36
        model_calls = 14 * (num_images - 1)
        perf_bytes = pixels_per_launch * (performed_bytes_per_pixel_iter(calls, False) +
                                          performed_bytes_per_pixel_iter(calls, True)) / 2
        perf_gbs = perf_bytes / (iso_ms / 1e3) / 1e9
        out.update({
            "ncc_calls_per_pixel_iter": round(calls, 2),
            "ncc_calls_per_pixel_iter_model": model_calls,
            "performed_bytes_per_launch": round(perf_bytes),
            "achieved_performed": round(perf_gbs, 1),
            "frac_performed": round(perf_gbs / HBM_PEAK_GBS, 4),
            "performed_note": "ncc_calls_per_pixel_iter = TA_BUFFER_READ_WAVEFRONTS_sum / SQ_WAVES / 36 (wave-level "
                              "NCC calls the kernel issues); the model's 14 (N-1) includes the zero-weight calls "
                              "the reference computes and discards (src/ACMMP.cu:747-751), which the product skips "
                              "bit-exactly; frac_performed = the §8d bytes with the performed calls / launch_ms "
                              "/ 8 TB/s",
        })
    if "l2_hit_rate" in pmc:
        out["l2"] = {
            "hit_rate": round(pmc["l2_hit_rate"], 4),
            "l1_to_l2_reqs_per_gather": round(pmc["l1_to_l2_reqs_per_gather"], 3),
            "memory_side_read_reqs": round(pmc["ea_read_reqs"]),
            "memory_side_read_reqs_128b": round(pmc["ea_read_reqs_128b"]),
            "read_bytes_calibrated": round(pmc["read_bytes_calibrated"]),
            "note": "TCC_HIT/(HIT+MISS), TCP_TCC_READ_REQ per gather wave-instruction, TCC_EA0_RDREQ(_128B) per "
                    "launch; read bytes = 128 x RDREQ_128B + 64 x the other requests, calibrated for dword gathers "
                    "(tools/microbench/fetch_cal.hip, profiles/r05_fetch_cal.json)",
        }
    return out


def cpu_baseline(args, setup, images, cams, srcs, mine, all_depth, gpu_value):
    """CPU oracle (oracle/acmmp_oracle.c, OpenMP) on bounded samples of the
    same work: (1) cfg1 in full (5 views 400x300, 3 iters, photometric);
    (2) the cfg2 step on a crop of reference view 0 (principal point shifted)
    against its full-size source views: photometric, then geometric with the
    GPU's photometric depth maps of the sources, 8 iterations each — the
    per-pixel work of the GPU step."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: baseline leg only
    from acmmp_amd import ACMMP, default_params, scene
    from acmmp_amd._abi import Camera

    from acmmp_amd import load_library
    # every host thread this process may use: the smallest of the affinity
    # mask, the cgroup CPU quota and OMP_NUM_THREADS, the launcher's declared
    # budget (the library's own pools use the same count)
    threads = int(load_library().acmmp_host_threads())
    model, ncpu, avail = host_cpu()
    oracle.build()

    # (1) cfg1 in full, CPU and GPU, same N and iterations
    sc1 = scene.make_scene(num_views=5, width=400, height=300)
    c1, i1 = sc1.problem(0, 4)
    p1 = default_params()
    p1.max_iterations = 3
    with ACMMP(0) as eng:
        eng.set_params(p1)
        eng.set_images(c1, i1)
        prm1 = eng.params
        eng.RunPatchMatch()  # warm
        g0 = time.perf_counter()
        reps = 20
        for _ in range(reps):
            eng.RunPatchMatch()
        g1 = (time.perf_counter() - g0) / reps
    t0 = time.perf_counter()
    oracle.run_patchmatch(prm1, c1, i1, nthreads=threads)
    t1 = time.perf_counter() - t0

    # (2) cfg2 crop, photometric + geometric
    cw, ch = (int(v) for v in args.cpu_sample.split("x"))
    v = mine[0]
    ids = [v] + srcs[v]
    imgs = [images[i].cpu().numpy() for i in ids]
    cs = [cams[i] for i in ids]
    x0 = (args.width - cw) // 2
    y0 = (args.height - ch) // 2
    ref = Camera.from_buffer_copy(bytes(cs[0]))
    ref.K[2] = cs[0].K[2] - x0
    ref.K[5] = cs[0].K[5] - y0
    ref.width, ref.height = cw, ch
    imgs[0] = np.ascontiguousarray(imgs[0][y0:y0 + ch, x0:x0 + cw])
    cs = [ref] + cs[1:]
    p = default_params()
    p.max_iterations = args.iters
    p.depth_min = cs[0].depth_min * 0.6
    p.depth_max = cs[0].depth_max * 1.2
    depths = [all_depth[i].cpu().numpy() for i in ids]
    t0 = time.perf_counter()
    ph = oracle.run_patchmatch(p, cs, imgs, nthreads=threads)
    t_photo = time.perf_counter() - t0
    depths[0] = np.ascontiguousarray(ph["planes"][..., 3])
    pg = default_params()
    pg.max_iterations = args.iters
    pg.geom_consistency = 1
    pg.depth_min, pg.depth_max = p.depth_min, p.depth_max
    t0 = time.perf_counter()
    oracle.run_patchmatch(pg, cs, imgs, depths=depths, planes=ph["planes"], costs=ph["costs"], nthreads=threads)
    t_geom = time.perf_counter() - t0
    cpu_value = 2 * cw * ch / (t_photo + t_geom) / 1e6
    return {
        "value": round(cpu_value, 5),
        "unit": "Mpix/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{cw}x{ch} crop of ref view {v} (K shifted) vs {len(ids) - 1} full {args.width}x{args.height} "
                  f"source views, {args.iters} iters, photometric {t_photo:.2f} s + geometric {t_geom:.2f} s "
                  f"(the GPU step's per-pixel work)",
        "cpu_model": model,
        "nproc": ncpu,
        "cpus_available": avail,
        "cores_note": (f"cores = the {threads} host threads this process is granted (affinity mask, cgroup "
                       f"quota and OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', 'unset')}: a shared GPU "
                       f"box gives one GPU's process a {threads}-CPU share of its {avail} threads); on an "
                       "unshared host the oracle uses every core" if threads < avail else
                       "cores = every host thread available to the process"),
        "value_per_core": round(cpu_value / threads, 6),
        "all_core_estimate": round(cpu_value / threads * avail, 4),
        "all_core_estimate_note": f"value_per_core x {avail} available threads: linear OpenMP scaling, an upper "
                                  "bound for the CPU (the pixel loop is embarrassingly parallel per colour; "
                                  "measured efficiency 0.93-1.02 at 2-8 threads, profiles/r06_cpu_scaling.jsonl); "
                                  "an extrapolation, not a measurement, beyond the threads granted",
        "speedup_gpu_vs_cpu": round(gpu_value / cpu_value, 1),
        "speedup_gpu_vs_all_core_estimate": round(gpu_value / (cpu_value / threads * avail), 1),
        "cfg1": {
            "workload": "5 views 400x300, 3 iters, photometric (BASELINE configs[0]), in full",
            "cpu_s": round(t1, 3),
            "gpu_s": round(g1, 5),
            "cpu_mpix_s": round(400 * 300 / t1 / 1e6, 4),
            "gpu_mpix_s": round(400 * 300 / g1 / 1e6, 2),
            "speedup": round(t1 / g1, 1),
        },
    }


if __name__ == "__main__":
    main()
