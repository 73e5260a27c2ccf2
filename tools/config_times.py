"""Per-configuration GPU timings of BASELINE.json's other configs (one GPU,
synthetic scene rendered into HBM, inputs resident before timing):

  cfg1  5 views at 400x300, 3 iterations, photometric (one RunPatchMatch)
  cfg3  10 views at 1600x1200: photometric pass (8 iterations), planar-prior
        construction (support points -> Delaunay -> prior planes), then the
        planar-prior pass (SetPlanarPriorParams, 8 iterations)
  cfg5  10 views at 6048x4032 (ETH3D native size), 8 iterations, photometric

Each line: ms per phase (median of `reps` after one warm-up) and Mpix/s of
the RunPatchMatch passes. cfg2 is bench.py's workload; cfg4 (49 views, 8
GPUs) is the distributed driver's and runs on the driver's 8-GPU node.
usage: python tools/config_times.py [reps] > gpurun_out/configs.jsonl
"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from acmmp_amd import ACMMP, default_params, scene  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 3
dev = torch.device("cuda", 0)


def _problem(W, H, n):
    setup = scene.scene_setup(num_views=n, width=W, height=H)
    ids = [0] + list(setup.pairs[0][: n - 1])
    imgs = [scene.render_torch(setup, i, dev) for i in ids]
    torch.cuda.synchronize()
    return [setup.camera(i) for i in ids], imgs


def _timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3


def photometric(name, W, H, n, iters):
    cams, imgs = _problem(W, H, n)
    ms = []
    with ACMMP(0) as eng:
        p = default_params()
        p.max_iterations = iters
        eng.set_params(p)
        eng.set_images_device(cams, [im.data_ptr() for im in imgs])
        for r in range(REPS + 1):
            t = _timed(eng.RunPatchMatch)
            if r:
                ms.append(t)
        bits = eng.texel_bits()
    m = statistics.median(ms)
    print(json.dumps({"config": name, "W": W, "H": H, "num_images": n, "iters": iters, "texel_bits": bits,
                      "run_ms": round(m, 3), "mpix_per_s": round(W * H / m / 1e3, 3)}), flush=True)


def planar(name, W, H, n, iters):
    cams, imgs = _problem(W, H, n)
    rows = []
    with ACMMP(0) as eng:
        for r in range(REPS + 1):
            p = default_params()
            p.max_iterations = iters
            eng.set_params(p)
            eng.set_images_device(cams, [im.data_ptr() for im in imgs])
            t_photo = _timed(eng.RunPatchMatch)
            box = {}
            t_prior = _timed(lambda: box.update(n=eng.prepare_planar_prior()))
            t_planar = _timed(eng.RunPatchMatch)
            if r:
                rows.append((t_photo, t_prior, t_planar, box["n"]))
    med = [statistics.median(x[i] for x in rows) for i in range(3)]
    total = sum(med)
    print(json.dumps({"config": name, "W": W, "H": H, "num_images": n, "iters": iters,
                      "photometric_ms": round(med[0], 3), "prior_build_ms": round(med[1], 3),
                      "planar_pass_ms": round(med[2], 3), "support_points": rows[-1][3][0],
                      "triangles": rows[-1][3][1], "total_ms": round(total, 3),
                      "mpix_per_s": round(2 * W * H / total / 1e3, 3)}), flush=True)


if __name__ == "__main__":
    photometric("cfg1", 400, 300, 5, 3)
    planar("cfg3", 1600, 1200, 10, 8)
    photometric("cfg5", 6048, 4032, 10, 8)
