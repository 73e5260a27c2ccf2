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


def resize_linear(src, dw, dh):
    """cv::resize INTER_LINEAR of a float image, restated (see test_image_io)."""
    sh, sw = src.shape
    sx, sy = sw / dw, sh / dh
    if sx == 2 and sy == 2:
        r = src.reshape(dh, 2, dw, 2)
        return ((r[:, 0, :, 0] + r[:, 0, :, 1]) + (r[:, 1, :, 0] + r[:, 1, :, 1])) * np.float32(0.25)

    def coeffs(n, s, size):
        f = np.array([np.float32((i + 0.5) * s - 0.5) for i in range(n)], dtype=np.float32)
        i0 = np.floor(f).astype(np.int64)
        a = (f - i0.astype(np.float32)).astype(np.float32)
        a[i0 < 0] = 0
        i0[i0 < 0] = 0
        hi = i0 >= size - 1
        a[hi] = 0
        i0[hi] = size - 1
        return i0, np.minimum(i0 + 1, size - 1), a

    x0, x1, ax = coeffs(dw, sx, sw)
    y0, y1, ay = coeffs(dh, sy, sh)
    one = np.float32(1)
    rows = src[:, x0] * (one - ax) + src[:, x1] * ax
    return rows[y0] * (one - ay)[:, None] + rows[y1] * ay[:, None]


def rescale(img, cam, max_image_size):
    """InputInitialization's per-view rescale (src/ACMMP.cpp:564-598)."""
    import copy
    H, W = img.shape
    cam = copy.copy(cam)
    if W <= max_image_size and H <= max_image_size:
        return img, cam
    f32 = np.float32
    factor = min(f32(max_image_size) / f32(W), f32(max_image_size) / f32(H))
    nw, nh = int(np.round(f32(W) * factor)), int(np.round(f32(H) * factor))
    sx, sy = f32(nw) / f32(W), f32(nh) / f32(H)
    K = list(cam.K)
    K[0], K[2], K[4], K[5] = f32(K[0]) * sx, f32(K[2]) * sx, f32(K[4]) * sy, f32(K[5]) * sy
    for k in (0, 2, 4, 5):
        cam.K[k] = float(K[k])
    cam.width, cam.height = nw, nh
    return resize_linear(img, nw, nh), cam


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
        self.full_images, self.full_cams = dict(self.images), dict(self.cams)

    def set_scale(self, cur_sizes):
        """Images and cameras of every view at its problem's cur_image_size
        (sources use the size of the problem with their id, as the reference)."""
        for i in self.full_images:
            self.images[i], self.cams[i] = rescale(self.full_images[i], self.full_cams[i], cur_sizes[i])

    def process_problem(self, idx, geom, planar, multi, seed_hi, maps_in, hier=False, seeded=False):
        pr = self.problems[idx]
        ids = [pr.ref_image_id] + list(pr.src_image_ids)
        cams = [self.cams[i] for i in ids]
        imgs = [self.images[i] for i in ids]
        p = _params(cams[0], len(ids), geom, multi, self.seed + pr.ref_image_id, seed_hi)
        kw = {}
        if seeded:  # pSampler + SetPlanarPrior (src/acmmp_definitions.cpp:275-281)
            depth_u16, normals_bgr = self.priors[idx]
            cam = cams[idx] if idx < len(cams) else cams[0]  # GetCamera(idx), as the reference
            H, W = imgs[0].shape
            kw["seed_planes"] = oracle.prior_plane_estimate(depth_u16, normals_bgr, cam, H, W)
            p.seeded = 1
        if hier:  # CudaSpaceInitialization hierarchy branch (src/ACMMP.cpp:745-808)
            ref = pr.ref_image_id
            H, W = imgs[0].shape
            up = maps_in[(ref, "depths")]
            nrm, cst = maps_in[(ref, "normals")], maps_in[(ref, "costs")]
            sh, sw = cst.shape
            p.hierarchy = 1
            upsample = (sw != H or sh != W)
            p.upsample = int(upsample)
            if upsample:
                p.scaled_cols, p.scaled_rows = float(sw), float(sh)
            w = cst if upsample else up.reshape(-1)[: sh * sw].reshape(sh, sw)
            kw["scaled_planes"] = np.concatenate([nrm, w[..., None]], -1).astype(np.float32)
            planes = np.zeros((H, W, 4), np.float32)
            planes[..., 3] = up
            kw["planes"] = planes
            kw["pre_costs"] = np.zeros((H, W), np.float32)
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
            extra = {"seed_planes": kw["seed_planes"]} if seeded else {}
            if hier:
                extra = {"pre_costs": out["pre_costs"], "scaled_planes": kw["scaled_planes"]}
            out = oracle.run_patchmatch(p, cams, imgs, planes=out["planes"], costs=out["costs"],
                                        prior_planes=prior, masks=mask, **extra)
        res = {"normals": out["planes"][..., :3].copy(), "costs": out["costs"]}
        res["depths_geom" if geom else "depths"] = out["planes"][..., 3].copy()
        return res

    def run_pass(self, geom, planar, multi, seed_hi, order="sequential", hier=False, seeded=False):
        snapshot = dict(self.maps)
        for idx, pr in enumerate(self.problems):
            src = self.maps if order == "sequential" else snapshot
            res = self.process_problem(idx, geom, planar, multi, seed_hi, src, hier, seeded)
            for k, v in res.items():
                self.maps[(pr.ref_image_id, k)] = v

    def run_single_scale(self, order="sequential", geom_iterations=2, priors=None):
        """priors: {problem index: (depth uint16, normals uint16 BGR)} seeds the
        first pass (main_ACMMP -p)."""
        self.priors = priors
        self.run_pass(False, True, False, 0, order, seeded=priors is not None)
        for g in range(geom_iterations):
            self.run_pass(True, False, g > 0, 1 + g, order)
        return self.maps

    def run_multi_scale(self, order="sequential", geom_iterations=2):
        """main_ACMMP's scale loop (src/main_ACMMP.cpp:96-176) with
        ComputeMultiScaleSettings (src/acmmp_definitions.cpp:207-243)."""
        maxsz, ndown = {}, {}
        for pr in self.problems:
            H, W = self.full_images[pr.ref_image_id].shape
            m = min(max(H, W), 3200)
            maxsz[pr.ref_image_id] = m
            k = 0
            while m > 1000:
                m //= 2
                k += 1
            ndown[pr.ref_image_id] = k
        max_down = max(ndown.values())
        cur = {}
        seed_hi = 0
        first = True
        while max_down >= 0:
            for i in ndown:
                if ndown[i] >= 0:
                    cur[i] = int(maxsz[i] / 2.0 ** ndown[i])
                    ndown[i] -= 1
            self.set_scale(cur)
            if first:
                first = False
                self.run_pass(False, True, False, seed_hi, order)
            else:
                for pr in self.problems:  # JointBilateralUpsampling (src/acmmp_definitions.cpp:405-438)
                    i = pr.ref_image_id
                    up, isc = oracle.jbu(self.images[i], self.maps[(i, "depths_geom")])
                    if up is not None:
                        self.maps[(i, "depths")] = up
                self.run_pass(False, True, False, seed_hi, order, hier=True)
            seed_hi += 1
            for g in range(geom_iterations):
                self.run_pass(True, False, g > 0, seed_hi, order)
                seed_hi += 1
            max_down -= 1
        return self.maps
