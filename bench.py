#!/usr/bin/env python3
"""PatchMatch throughput benchmark (BASELINE.json metric) on 1..N MI355X.

Workload (BASELINE.json configs[1], "cfg2"): per GPU, 10 reference views at
1600x1200, each with its 9 nearest source views (N = 10 images per problem),
8 PatchMatch iterations, a photometric pass over the GPU's views, an RCCL
all-gather of the depth maps, then a geometric-consistency pass over the same
views (it reads the neighbours' depth maps: the real exchange step).

One "step" = photometric pass + all-gather + geometric pass. Weak scaling:
every rank owns one copy of the 10-view cfg2 problem (global view ids
rank*10 + k), so per-GPU work is identical for every N; the depth maps of all
ranks are all-gathered (RCCL over xGMI) and the geometric pass reads its
sources from the gathered buffer. Inputs are rendered straight into HBM before
timing (synthetic, seeded).

value = total pixels processed by all ranks (2 passes x views x W x H) /
max-over-ranks wall time of the K timed steps, in Mpix/s. Each GPU keeps two
views in flight (two engines, each on its own HIP stream, --streams 2): the
tail of one view's sweep launch fills with the other's blocks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

BASELINE_METRIC = "Mpixels/sec PatchMatch (1600×1200, 8 iters) at 1/2/4/8 GPUs; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def algorithmic_bytes_per_pixel_iter(num_images: int, geom: bool) -> int:
    """SURVEY §8d / BASELINE.md §3 gather-byte model per pixel-iteration:
    14*(N-1) NCC calls x 724 B + 572 B of state, + 14*(N-1)*4 B in geometric
    passes."""
    b = 14 * (num_images - 1) * 724 + 572
    if geom:
        b += 14 * (num_images - 1) * 4
    return b


def parse():
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
    ap.add_argument("--profile-dir", default=None, help="write per-run timing JSON here")
    ap.add_argument("--streams", type=int, default=2,
                    help="engines (HIP streams) per GPU running different views concurrently")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend for N>1 (nccl = RCCL over xGMI; gloo only to test on one GPU)")
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    dev_index = local_rank % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    backend = args.backend
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)

    from acmmp_amd import ACMMP, default_params, scene

    # Weak scaling: every rank owns one copy of the cfg2 problem (the same
    # 10-view arc, so per-GPU work is identical for every N); global view id
    # = rank * views + k. The depth maps of ALL ranks are all-gathered between
    # the passes and the geometric pass reads its sources from the gathered
    # buffer, as a view-parallel pipeline does.
    if args.views < args.nsrc + 1:
        raise SystemExit(f"--views {args.views} cannot supply {args.nsrc} source views per problem")
    V = args.views * world
    W, H = args.width, args.height
    setup = scene.scene_setup(num_views=args.views, width=W, height=H)
    base_id = rank * args.views
    mine = list(range(base_id, base_id + args.views))
    srcs = {base_id + k: [base_id + j for j in setup.pairs[k][:args.nsrc]] for k in range(args.views)}
    images = {base_id + k: scene.render_torch(setup, k, device) for k in range(args.views)}
    cams = {base_id + k: setup.camera(k) for k in range(args.views)}
    torch.cuda.synchronize()

    n_img = 1 + args.nsrc
    planes = torch.empty((args.views, H, W, 4), dtype=torch.float32, device=device)
    costs = torch.empty((args.views, H, W), dtype=torch.float32, device=device)
    my_depth = torch.empty((args.views, H, W), dtype=torch.float32, device=device)
    all_depth = torch.empty((V, H, W), dtype=torch.float32, device=device) if world > 1 else my_depth

    # one engine (own HIP stream) per concurrent view: with --streams > 1 the
    # views of a pass run in rounds of `streams`, their kernels overlapping on
    # the GPU (the tail of one view's launch fills with the other's blocks)
    engines = [ACMMP(dev_index) for _ in range(max(args.streams, 1))]
    for e in engines:
        e.set_timing(True)
    base = default_params()
    base.max_iterations = args.iters

    sweep_stats = {"photo": [0.0, 0], "geom": [0.0, 0]}

    def launch_view(eng, k: int, v: int, geom: bool):
        ids = [v] + srcs[v]
        eng.set_params(base)
        eng.set_images_device([cams[i] for i in ids], [images[i].data_ptr() for i in ids])
        if geom:
            p = eng.params
            p.geom_consistency = 1
            p.max_iterations = args.iters  # BASELINE cfg2: 8 iterations in both passes
            eng.set_params(p)
            # global view ids index the gathered maps (world == 1: my_depth)
            eng.set_depth_maps_device([all_depth[i].data_ptr() for i in ids])
            eng.set_plane_hypotheses_device(planes[k].data_ptr(), costs[k].data_ptr())
        eng.run_async()
        if not geom:
            eng.export_results(planes[k].data_ptr(), costs[k].data_ptr(), my_depth[k].data_ptr())

    stats_lock = threading.Lock()

    def finish_view(eng, geom: bool):
        eng.synchronize()
        t = eng.timing()
        with stats_lock:
            st = sweep_stats["geom" if geom else "photo"]
            st[0] += t["sweep_ms"]
            st[1] += t["sweep_launches"]

    def run_pass(geom: bool):
        # one host thread per engine takes the next view off a shared queue as
        # soon as its own previous view finished (no lockstep rounds, so a view
        # that ends early does not leave the GPU to its partner's tail); the
        # library calls release the GIL (ctypes)
        work = list(enumerate(mine))
        if len(engines) == 1:
            for k, v in work:
                launch_view(engines[0], k, v, geom)
                finish_view(engines[0], geom)
            return
        errors = []

        def worker(eng):
            try:
                while True:
                    with stats_lock:
                        if not work or errors:
                            return
                        k, v = work.pop(0)
                    launch_view(eng, k, v, geom)
                    finish_view(eng, geom)
            except BaseException as e:  # re-raised on the main thread
                with stats_lock:
                    errors.append(e)

        threads = [threading.Thread(target=worker, args=(e,)) for e in engines]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        if errors:
            raise errors[0]


    def step():
        run_pass(geom=False)
        if world > 1:
            if backend == "nccl":  # RCCL over xGMI, device buffers
                dist.all_gather_into_tensor(all_depth, my_depth)
            else:  # gloo (tests on one GPU): staged through host memory
                host = torch.empty((V, H, W), dtype=torch.float32)
                dist.all_gather_into_tensor(host, my_depth.cpu())
                all_depth.copy_(host)
            torch.cuda.synchronize()
        run_pass(geom=True)

    for _ in range(args.warmup):
        step()
    for st in sweep_stats.values():
        st[0], st[1] = 0.0, 0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=device if backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    pix_total = 2 * args.views * world * W * H * args.steps
    value = pix_total / elapsed / 1e6
    # roofline of the dominant kernel (k_sweep), timed with hipEvents on the
    # engine stream: algorithmic bytes per launch / mean launch time
    P = W * H
    bytes_photo = (P / 2) * algorithmic_bytes_per_pixel_iter(n_img, False) * sweep_stats["photo"][1]
    bytes_geom = (P / 2) * algorithmic_bytes_per_pixel_iter(n_img, True) * sweep_stats["geom"][1]
    sweep_ms = sweep_stats["photo"][0] + sweep_stats["geom"][0]
    launches = sweep_stats["photo"][1] + sweep_stats["geom"][1]
    # with S engines running S views at a time, S sweep launches overlap on the
    # GPU: each one's HIP-event duration (what rocprofv3 also reports) spans
    # the shared time, so the kernel's own rate uses duration / S
    S = len(engines)
    achieved = (bytes_photo + bytes_geom) / (sweep_ms / S / 1e3) / 1e9 if sweep_ms > 0 else 0.0
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_sweep.json")
    if os.path.exists(pmc_path):
        try:
            pmc = json.load(open(pmc_path))
            if pmc.get("width") == W and pmc.get("height") == H and pmc.get("num_images") == n_img:
                traffic = pmc.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

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
                        f"{args.iters} iters, photometric + RCCL depth all-gather + geometric pass",
            "views_per_gpu": args.views,
            "width": W,
            "height": H,
            "num_images": n_img,
            "iters": args.iters,
            "parallelism": f"view-parallel x{world} (one process per GPU, {'RCCL' if backend == 'nccl' else 'gloo'} "
                           f"all-gather of depth maps between the passes; {S} views in flight per GPU on "
                           f"{S} HIP streams)",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "k_sweep (CheckerboardPropagation)",
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "model": "gather-byte model, SURVEY §8d: B_iter = 14*(N-1)*724 + 572 (+14*(N-1)*4 geom) "
                     "bytes per pixel-iteration, P/2 pixels per launch",
            "note": "gather bytes are logical (counted as if uncached, BASELINE.md §3); frac > 1 means "
                    "they are served from LDS/L1/L2 — traffic is the PMC-measured memory-side fetch+write",
            "sweep_launches": launches,
            "mean_launch_ms": round(sweep_ms / max(launches, 1), 3),
            "concurrent_launches": S,
            "effective_launch_ms": round(sweep_ms / S / max(launches, 1), 3),
            "timing": "achieved = algorithmic bytes per launch / effective_launch_ms; mean_launch_ms is the "
                      "HIP-event duration of one launch while S views' launches share the GPU (S engine "
                      "streams), the figure rocprofv3's kernel stats report for the same command",
        },
    }

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args, setup, images, cams, srcs, mine)
    if rank == 0:
        print(json.dumps(result), flush=True)
    for e in engines:
        e.close()
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(args, setup, images, cams, srcs, mine):
    """CPU oracle (oracle/acmmp_oracle.c, OpenMP) timed on a bounded sample of
    the same workload: a crop of the first reference view (principal point
    shifted) against its full-size source views, photometric, same iterations.
    Per-pixel work equals the full run's."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: baseline leg only
    from acmmp_amd import default_params
    from acmmp_amd._abi import Camera

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
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    oracle.build()
    t0 = time.perf_counter()
    oracle.run_patchmatch(p, cs, imgs, nthreads=threads)
    dt = time.perf_counter() - t0
    return {
        "value": round(cw * ch / dt / 1e6, 5),
        "unit": "Mpix/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{cw}x{ch} crop of ref view {v} (K shifted) vs {len(ids) - 1} full {args.width}x{args.height} "
                  f"source views, {args.iters} iters, photometric, {dt:.2f} s",
    }


if __name__ == "__main__":
    main()
