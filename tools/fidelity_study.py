"""How much the pinned arithmetic matters to the result.

The oracle and the GPU agree bit-exactly, but both use pinned semantics where
the reference's CUDA build differs: fp32 bilinear fractions (pin A4) where
the texture unit uses 1.8 fixed point, and IEEE division / sqrt / Cephes-style
exp, sin, cos with no FMA contraction where the reference is built with
--use_fast_math and nvcc's default fmad (src/CMakeLists.txt:19). This study
runs cfg2-shaped views (1600x1200, N=10, 8 iterations, photometric then
geometric, synthetic scene with analytic ground truth) in

  pinned          the product (bit-exact with the oracle)
  tex8            + acmmp_params.texture_filter8 (8-bit bilinear fractions)
  cuda_numerics   tex8 in a build with the reference's CUDA numerics
                  (make cuda-numerics: fast intrinsics, approximate div/sqrt,
                  FTZ, contraction; acmmp_amd/lib/variants/)

and reports per mode the share of pixels within 1 % / 0.5 % of the true depth
and the median relative error, and between modes the share of pixels whose
depths differ by more than 1 %.

usage (each library in its own process):
  python tools/fidelity_study.py run pinned,tex8 gpurun_out/fid_a.npz
  ACMMP_LIB=acmmp_amd/lib/variants/libacmmp_amd_cuda_numerics.so \\
      python tools/fidelity_study.py run cuda_numerics gpurun_out/fid_b.npz
  python tools/fidelity_study.py compare gpurun_out/fid_a.npz gpurun_out/fid_b.npz > profiles/...json
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

V, W, H, N = 4, 1600, 1200, 10


def run(modes, out_path):
    import torch
    from acmmp_amd import ACMMP, default_params, scene
    dev = torch.device("cuda", 0)
    setup = scene.scene_setup(num_views=V + N, width=W, height=H)
    imgs = {i: scene.render_torch(setup, i, dev) for i in range(V + N)}
    gts = {v: scene.render_torch(setup, v, dev, with_depth=True)[1].cpu().numpy() for v in range(V)}
    torch.cuda.synchronize()

    def one(v, tex8, depths=None, state=None):
        ids = [v] + setup.pairs[v][:N - 1]
        with ACMMP(0) as eng:
            p = default_params()
            p.max_iterations = 8
            p.texture_filter8 = tex8
            if depths is not None:
                p.geom_consistency = 1
            eng.set_params(p)
            eng.set_images_device([setup.camera(i) for i in ids], [imgs[i].data_ptr() for i in ids])
            if depths is not None:
                eng.set_depth_maps([depths[i] for i in ids])
                eng.set_plane_hypotheses(*state)
            eng.RunPatchMatch()
            return eng.plane_hypotheses(), eng.costs()

    saved = {f"gt{v}": gts[v] for v in range(V)}
    # flat pixels: the 11 x 11 patch around them holds one grey value (the
    # scene's textureless patches), where var_ref sits at the 1e-5 test
    pool = torch.nn.functional.max_pool2d
    for v in range(V):
        im = imgs[v][None, None]
        rng = pool(im, 11, 1, 5) + pool(-im, 11, 1, 5)
        saved[f"flat{v}"] = (rng[0, 0] == 0).cpu().numpy()
    for mode in modes:
        tex8 = 0 if mode == "pinned" else 1
        photo = {v: one(v, tex8) for v in range(V + N)}  # every depth map a geometric pass reads
        depths = {v: photo[v][0][..., 3] for v in photo}
        for v in range(V):
            saved[f"{mode}_{v}"] = one(v, tex8, depths, photo[v])[0][..., 3]
    np.savez_compressed(out_path, **saved)


def compare(paths):
    d = {}
    for p in paths:
        with np.load(p) as z:
            d.update({k: z[k] for k in z.files})
    modes = sorted({k.rsplit("_", 1)[0] for k in d if not k.startswith(("gt", "flat"))},
                   key=lambda m: ["pinned", "tex8", "cuda_numerics"].index(m) if m in
                   ["pinned", "tex8", "cuda_numerics"] else 9)
    out = {"views": V, "width": W, "height": H, "num_images": N, "iters": 8, "accuracy": {}, "modes_differ_over_1pct": {}}
    out["flat_share"] = round(float(np.mean([d[f"flat{v}"][d[f"gt{v}"] > 0].mean() for v in range(V)])), 5)
    for m in modes:
        acc = {}
        for part in ("all", "textured", "flat"):
            w1, w05, med = [], [], []
            for v in range(V):
                gt, dep, flat = d[f"gt{v}"], d[f"{m}_{v}"], d[f"flat{v}"]
                ok = gt > 0
                if part == "textured":
                    ok = ok & ~flat
                elif part == "flat":
                    ok = ok & flat
                rel = np.abs(dep - gt)[ok] / gt[ok]
                w1.append(float((rel < 0.01).mean()))
                w05.append(float((rel < 0.005).mean()))
                med.append(float(np.median(rel)))
            acc[part] = {"within_1pct": round(float(np.mean(w1)), 5), "within_0.5pct": round(float(np.mean(w05)), 5),
                         "median_rel_err": float(np.mean(med))}
        out["accuracy"][m] = acc
    for i, a in enumerate(modes):
        for b in modes[i + 1:]:
            res = {}
            for part in ("all", "textured", "flat"):
                diff = []
                for v in range(V):
                    x, y, flat = d[f"{a}_{v}"], d[f"{b}_{v}"], d[f"flat{v}"]
                    sel = np.ones_like(flat) if part == "all" else (~flat if part == "textured" else flat)
                    diff.append(float((np.abs(x - y) > 0.01 * np.abs(x))[sel].mean()))
                res[part] = round(float(np.mean(diff)), 5)
            out["modes_differ_over_1pct"][f"{a}_vs_{b}"] = res
    print(json.dumps(out))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2].split(","), sys.argv[3])
    else:
        compare(sys.argv[2:])
