"""The reference's pass driver restated over the CPU oracle (TEST
INFRASTRUCTURE): ProcessProblem (src/acmmp_definitions.cpp:245-403) and
main_ACMMP's single-scale pass order (src/main_ACMMP.cpp:114-139), in
Gauss-Seidel order (views in sequence, each reading the latest maps) or
Jacobi order (every view of a pass reads the previous pass's maps).

Inputs are read independently of the library: images through Pillow's
libjpeg in grayscale-draft mode (cv::imread(IMREAD_GRAYSCALE)), cameras and
pair.txt through acmmp_amd.io's numpy readers. The Delaunay triangulation is
the library's host routine (validated on its own in test_planar_host.py)."""
import os

import numpy as np

import oracle
from acmmp_amd import default_params, delaunay_triangulation
from acmmp_amd import io as aio


def load_gray(path):
    from PIL import Image
    im = Image.open(path)
    im.draft("L", im.size)
    return np.asarray(im, dtype=np.float32)


def _params(cam0, n, geom, multi, seed_lo, seed_hi):
    p = default_params()
    f32 = np.float32
    p.num_images = n
    p.depth_min = float(f32(cam0.depth_min) * f32(0.6))
    p.depth_max = float(f32(cam0.depth_max) * f32(1.2))
    p.disparity_min = float(f32(cam0.K[0]) * f32(p.baseline) / f32(p.depth_max))
    p.disparity_max = float(f32(cam0.K[0]) * f32(p.baseline) / f32(p.depth_min))
    if geom:
        p.geom_consistency = 1
        p.max_iterations = 2
        p.multi_geometry = int(multi)
    p.seed_lo = seed_lo
    p.seed_hi = seed_hi
    return p


class OraclePipeline:
    """Keeps the 'files' of the output folder in a dict: maps[(view, name)]."""

    def __init__(self, dense, seed=1234):
        self.dense = dense
        self.seed = seed
        self.problems = aio.read_pair(os.path.join(dense, "pair.txt"))
        self.images, self.cams = {}, {}
        for p in self.problems:
            i = p.ref_image_id
            self.images[i] = load_gray(os.path.join(dense, "images", "%08d.jpg" % i))
            cam = aio.read_camera(os.path.join(dense, "cams", "%08d_cam.txt" % i))
            cam.height, cam.width = self.images[i].shape
            self.cams[i] = cam
        self.maps = {}

    def process_problem(self, idx, geom, planar, multi, seed_hi, maps_in):
        pr = self.problems[idx]
        ids = [pr.ref_image_id] + list(pr.src_image_ids)
        cams = [self.cams[i] for i in ids]
        imgs = [self.images[i] for i in ids]
        p = _params(cams[0], len(ids), geom, multi, self.seed + pr.ref_image_id, seed_hi)
        kw = {}
        if geom:
            suffix = "depths_geom" if multi else "depths"
            kw["depths"] = [maps_in[(i, suffix)] for i in ids]
            ref = pr.ref_image_id
            kw["planes"] = np.concatenate([maps_in[(ref, "normals")], maps_in[(ref, suffix)][..., None]], -1)
            kw["costs"] = maps_in[(ref, "costs")]
        out = oracle.run_patchmatch(p, cams, imgs, **kw)
        if planar:
            H, W = imgs[0].shape
            pts = oracle.support_points(out["costs"])
            tris = delaunay_triangulation(W, H, pts)
            _, mask, prior = oracle.planar_prior(cams[0], out["planes"][..., 3], p.depth_min, p.depth_max, tris)
            p.planar_prior = 1
            p.rng_stream = 1
            out = oracle.run_patchmatch(p, cams, imgs, planes=out["planes"], costs=out["costs"],
                                        prior_planes=prior, masks=mask)
        res = {"normals": out["planes"][..., :3].copy(), "costs": out["costs"]}
        res["depths_geom" if geom else "depths"] = out["planes"][..., 3].copy()
        return res

    def run_pass(self, geom, planar, multi, seed_hi, order="sequential"):
        snapshot = dict(self.maps)
        for idx, pr in enumerate(self.problems):
            src = self.maps if order == "sequential" else snapshot
            res = self.process_problem(idx, geom, planar, multi, seed_hi, src)
            for k, v in res.items():
                self.maps[(pr.ref_image_id, k)] = v

    def run_single_scale(self, order="sequential", geom_iterations=2):
        self.run_pass(False, True, False, 0, order)
        for g in range(geom_iterations):
            self.run_pass(True, False, g > 0, 1 + g, order)
        return self.maps
