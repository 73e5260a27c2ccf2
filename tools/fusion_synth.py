"""A RunFusion input without a GPU: the synthetic scene rendered on the CPU
(render_numpy, analytic depth and world normals) written as a dense folder
plus the .dmb maps a geometric pass would leave (depths_geom.dmb,
normals.dmb, costs.dmb), perturbed like PatchMatch output — relative depth
noise, normal noise, a share of outlier depths and holes — so the approval
walk sees consistent, inconsistent and masked hits.

usage: python tools/fusion_synth.py <out_dir> [views] [width] [height] [nsrc] [seed]
Writes <out_dir>/dense (images, cams, pair.txt) and <out_dir>/dense/ACMMP/2333_*.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from acmmp_amd import io as aio  # noqa: E402
from acmmp_amd import scene  # noqa: E402


def write(out, V=20, W=800, H=600, nsrc=10, seed=7, arc_deg=1.8):
    rng = np.random.default_rng(seed)
    setup = scene.scene_setup(num_views=V, width=W, height=H, arc_deg=arc_deg)
    views = [scene.render_numpy(setup, i) for i in range(V)]
    dense = os.path.join(out, "dense")
    sc = scene.Scene(views=views, pairs=setup.pairs)
    scene.write_dense_folder(sc, dense, num_src=nsrc)
    for i, v in enumerate(views):
        d = v.depth * (1 + rng.normal(0, 0.002, v.depth.shape)).astype(np.float32)
        out_mask = rng.random(d.shape) < 0.05
        d = np.where(out_mask, rng.uniform(300, 800, d.shape), d).astype(np.float32)
        d = np.where(rng.random(d.shape) < 0.02, 0, d).astype(np.float32)
        n = v.normal + rng.normal(0, 0.02, v.normal.shape)
        n = (n / np.maximum(np.linalg.norm(n, axis=-1, keepdims=True), 1e-6)).astype(np.float32)
        folder = aio.result_folder(os.path.join(dense, "ACMMP"), i)
        os.makedirs(folder, exist_ok=True)
        aio.write_dmb(os.path.join(folder, "depths_geom.dmb"), d)
        aio.write_dmb(os.path.join(folder, "normals.dmb"), n)
        aio.write_dmb(os.path.join(folder, "costs.dmb"), np.zeros_like(d))
    return dense


if __name__ == "__main__":
    a = sys.argv
    args = [int(x) for x in a[2:7]]
    print(write(a[1], *args))
