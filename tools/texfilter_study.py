"""Pin A4's effect on the result: cfg2-shaped views (1600x1200, N=10,
8 iterations, photometric then geometric, synthetic scene with analytic
ground truth) run with pin A4's fp32 bilinear fractions and with the CUDA
texture unit's 8-bit fractions (acmmp_params.texture_filter8, the reference's
cudaFilterModeLinear, src/ACMMP.cpp:659). Reports, per mode, the share of
pixels within 1 % / 0.5 % of the true depth and the median relative error,
and between the modes the share of pixels whose depths differ by more than
1 %. usage: python tools/texfilter_study.py [views] > gpurun_out/texfilter.json"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from acmmp_amd import ACMMP, default_params, scene  # noqa: E402

V = int(sys.argv[1]) if len(sys.argv) > 1 else 4
W, H, N = 1600, 1200, 10
dev = torch.device("cuda", 0)
setup = scene.scene_setup(num_views=V + N, width=W, height=H)
imgs = {i: scene.render_torch(setup, i, dev) for i in range(V + N)}
torch.cuda.synchronize()


def run(v, q8, depths=None, state=None):
    ids = [v] + setup.pairs[v][:N - 1]
    with ACMMP(0) as eng:
        p = default_params()
        p.max_iterations = 8
        p.texture_filter8 = q8
        if depths is not None:
            p.geom_consistency = 1
        eng.set_params(p)
        eng.set_images_device([setup.camera(i) for i in ids], [imgs[i].data_ptr() for i in ids])
        if depths is not None:
            eng.set_depth_maps([depths[i] for i in ids])
            eng.set_plane_hypotheses(*state)
        eng.RunPatchMatch()
        return eng.plane_hypotheses(), eng.costs()


out = {"views": V, "width": W, "height": H, "num_images": N, "iters": 8}
res = {}
for q8 in (0, 1):
    photo = {}
    for v in range(V + N):  # every view the geometric pass reads needs a depth map
        photo[v] = run(v, q8)
    depths = {v: photo[v][0][..., 3] for v in photo}
    geom = {v: run(v, q8, depths, photo[v]) for v in range(V)}
    res[q8] = geom
    within1, within05, med = [], [], []
    for v in range(V):
        gt = scene.render_torch(setup, v, dev, with_depth=True)[1].cpu().numpy()
        d = geom[v][0][..., 3]
        ok = gt > 0
        rel = np.abs(d - gt)[ok] / gt[ok]
        within1.append(float((rel < 0.01).mean()))
        within05.append(float((rel < 0.005).mean()))
        med.append(float(np.median(rel)))
    out["fp32_fractions" if q8 == 0 else "texture_8bit_fractions"] = {
        "within_1pct": round(float(np.mean(within1)), 5), "within_0.5pct": round(float(np.mean(within05)), 5),
        "median_rel_err": float(np.mean(med))}
diff = []
for v in range(V):
    a, b = res[0][v][0][..., 3], res[1][v][0][..., 3]
    diff.append(float((np.abs(a - b) > 0.01 * np.abs(a)).mean()))
out["modes_differ_over_1pct"] = round(float(np.mean(diff)), 5)
print(json.dumps(out))
