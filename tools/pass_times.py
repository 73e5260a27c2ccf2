"""k_sweep time per launch of the photometric and the geometric pass of the
cfg2 step separately (one engine, one stream, HIP events), and of the
geometric pass with the geometric cost's depth fetch counted: the bench's
launch_ms is their mean.

usage: python tools/pass_times.py [reps] > gpurun_out/pass_times.json
(PASS_NSRC=<n> in the environment: n source views instead of cfg2's 9, so the
NS 16 / 20 / 32 kernel buckets can be timed.)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from acmmp_amd import default_params, scene  # noqa: E402
from acmmp_amd.resident import EnginePool, geometric_view, photometric_view  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 3
W, H, ITERS = 1600, 1200, 8
NSRC = int(os.environ.get("PASS_NSRC", "9"))
dev = torch.device("cuda", 0)


def main():
    setup = scene.scene_setup(num_views=NSRC + 1, width=W, height=H)
    V = NSRC + 1
    imgs = [scene.render_torch(setup, i, dev) for i in range(V)]
    cams = [setup.camera(i) for i in range(V)]
    torch.cuda.synchronize()
    pool = EnginePool(0, 1, timing=True)
    eng = pool.engines[0]
    photo = default_params()
    photo.max_iterations = ITERS
    geom = default_params()
    geom.max_iterations = ITERS
    geom.geom_consistency = 1
    planes = [torch.empty((H, W, 4), dtype=torch.float32, device=dev) for _ in range(V)]
    costs = [torch.empty((H, W), dtype=torch.float32, device=dev) for _ in range(V)]
    depth = [torch.empty((H, W), dtype=torch.float32, device=dev) for _ in range(V)]
    ids = {v: [v] + list(setup.pairs[v][:NSRC]) for v in range(V)}
    out = {"W": W, "H": H, "nsrc": NSRC, "iters": ITERS, "photometric_ms": [], "geometric_ms": []}
    for rep in range(REPS + 1):
        pool.reset_timing()
        for v in range(V):  # the photometric pass of the cfg2 step: every view's depth
            photometric_view(pool, eng, photo, [cams[i] for i in ids[v]], [imgs[i].data_ptr() for i in ids[v]],
                             planes[v].data_ptr(), costs[v].data_ptr(), depth[v].data_ptr())
        torch.cuda.synchronize()
        p_ms = pool.sweep_ms / max(pool.sweep_launches, 1)
        pool.reset_timing()
        for v in range(V):
            geometric_view(pool, eng, geom, [cams[i] for i in ids[v]], [imgs[i].data_ptr() for i in ids[v]],
                           [depth[i].data_ptr() for i in ids[v]], planes[v].data_ptr(), costs[v].data_ptr())
        torch.cuda.synchronize()
        g_ms = pool.sweep_ms / max(pool.sweep_launches, 1)
        if rep:
            out["photometric_ms"].append(round(p_ms, 3))
            out["geometric_ms"].append(round(g_ms, 3))
    pool.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
