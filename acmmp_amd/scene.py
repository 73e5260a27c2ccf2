"""Seeded synthetic multi-view scenes with analytic ground truth.

No DTU/ETH3D data exists offline, so benchmarks and parity tests
use analytically rendered views of a DTU-like setup:

* cameras on an arc around the object, 1600x1200 pinhole with DTU-like
  intrinsics (fx ~ 2892 px), depth range line `300 2.6041666666666665 192 800`
  (python_scripts/refactor_dir.py:10);
* a slanted background plane, a sphere and a box, textured with band-limited
  3-D sinusoid noise whose wavelength is 4-16 px at the render resolution, with
  ~10 % textureless patches (exercises the var < 1e-5 path of
  ComputeBilateralNCC, src/ACMMP.cu:423-425);
* images are quantised to uint8 (emulating the reference's 8-bit grayscale JPEG
  input, src/ACMMP.cpp:539) and returned as float32.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _abi
from .engine import make_camera

DEPTH_LINE = (300.0, 2.6041666666666665, 192.0, 800.0)


@dataclass
class View:
    K: np.ndarray       # 3x3
    R: np.ndarray       # 3x3 world->cam
    t: np.ndarray       # 3
    image: np.ndarray   # (H, W) float32, uint8-valued
    depth: np.ndarray   # (H, W) float32 ground-truth z-depth (0 = no hit)
    normal: np.ndarray  # (H, W, 3) float32 ground-truth world normal

    @property
    def camera(self) -> _abi.Camera:
        h, w = self.image.shape
        return make_camera(self.K, self.R, self.t, w, h, DEPTH_LINE[0], DEPTH_LINE[3])


@dataclass
class Scene:
    views: list
    pairs: list  # pairs[i] = list of source view ids for ref i (best first)

    def problem(self, ref: int, nsrc: int):
        """(cameras, images) for ref + its first nsrc sources."""
        ids = [ref] + list(self.pairs[ref][:nsrc])
        return [self.views[i].camera for i in ids], [self.views[i].image for i in ids]


def _look_at(C: np.ndarray, target: np.ndarray, up=np.array([0.0, -1.0, 0.0])):
    z = target - C
    z /= np.linalg.norm(z)
    x = np.cross(up, z)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    R = np.stack([x, y, z])  # rows: camera axes in world
    t = -R @ C
    return R, t


class _Texture:
    def __init__(self, rng: np.random.Generator, wavelength_mm: tuple, n: int = 40):
        d = rng.normal(size=(n, 3))
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        lam = rng.uniform(wavelength_mm[0], wavelength_mm[1], size=n)
        self.f = (d / lam[:, None]) * 2.0 * np.pi
        self.phase = rng.uniform(0, 2 * np.pi, size=n)
        self.amp = rng.uniform(0.5, 1.0, size=n)
        # low-frequency field selecting textureless patches
        d2 = rng.normal(size=(6, 3))
        d2 /= np.linalg.norm(d2, axis=1, keepdims=True)
        self.f2 = d2 / rng.uniform(40.0, 80.0, size=6)[:, None] * 2.0 * np.pi
        self.p2 = rng.uniform(0, 2 * np.pi, size=6)

    def __call__(self, X: np.ndarray) -> np.ndarray:
        s = np.sin(X @ self.f.T + self.phase) @ self.amp
        s = s / np.sqrt(0.5 * np.sum(self.amp ** 2))
        val = 127.5 + 60.0 * np.tanh(0.9 * s)
        low = np.sin(X @ self.f2.T + self.p2).sum(axis=1) / np.sqrt(3.0)
        flat = low > 1.28  # ~10 % of the surface
        val = np.where(flat, 128.0, val)
        return val


def _intersect(Cw: np.ndarray, D: np.ndarray):
    """Nearest hit of rays C + s D with the scene. Returns s (inf = miss) and
    world normals."""
    n_rays = D.shape[0]
    best = np.full(n_rays, np.inf)
    nrm = np.zeros((n_rays, 3))
    # background plane n.X = d
    pn = np.array([0.25, -0.15, 1.0])
    pn /= np.linalg.norm(pn)
    pd = -160.0
    den = D @ pn
    with np.errstate(divide="ignore", invalid="ignore"):
        s = (pd - Cw @ pn) / den
    ok = (s > 1e-3) & np.isfinite(s) & (s < best)
    best = np.where(ok, s, best)
    nrm[ok] = -pn if (Cw @ pn) < pd else pn
    # sphere
    cs, r = np.array([-20.0, 10.0, 0.0]), 85.0
    oc = Cw - cs
    b = D @ oc
    c = oc @ oc - r * r
    disc = b * b - c
    sq = np.sqrt(np.maximum(disc, 0.0))
    s = -b - sq
    ok = (disc > 0) & (s > 1e-3) & (s < best)
    best = np.where(ok, s, best)
    X = Cw + s[:, None] * D
    nrm[ok] = ((X - cs) / r)[ok]
    # axis-aligned box
    bmin, bmax = np.array([60.0, -40.0, -60.0]), np.array([150.0, 50.0, 20.0])
    with np.errstate(divide="ignore", invalid="ignore"):
        t1 = (bmin - Cw) / D
        t2 = (bmax - Cw) / D
    tmin = np.minimum(t1, t2)
    tmax = np.maximum(t1, t2)
    tn = tmin.max(axis=1)
    tf = tmax.min(axis=1)
    ok = (tn <= tf) & (tn > 1e-3) & (tn < best)
    best = np.where(ok, tn, best)
    axis = np.argmax(tmin, axis=1)
    bn = np.zeros((n_rays, 3))
    bn[np.arange(n_rays), axis] = -np.sign(D[np.arange(n_rays), axis])
    nrm[ok] = bn[ok]
    return best, nrm


@dataclass
class SceneSetup:
    """Everything but the pixels: cameras, texture, view pairs."""

    width: int
    height: int
    K: np.ndarray
    poses: list      # (R, t, C, azimuth) per view
    texture: "_Texture"
    pairs: list

    def camera(self, i: int) -> _abi.Camera:
        R, t, _, _ = self.poses[i]
        return make_camera(self.K, R, t, self.width, self.height, DEPTH_LINE[0], DEPTH_LINE[3])


def scene_setup(num_views: int = 10, width: int = 1600, height: int = 1200, seed: int = 0x5EED,
                arc_deg: float = 6.0, radius: float = 600.0) -> SceneSetup:
    rng = np.random.default_rng(seed)
    fx = fy = 2892.33 * width / 1600.0
    cx, cy = 823.2 * width / 1600.0, 619.1 * height / 1200.0
    K = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1.0]])
    px_mm = radius / fx
    tex = _Texture(rng, (4.0 * px_mm, 16.0 * px_mm))
    poses = []
    for i in range(num_views):
        az = np.deg2rad(arc_deg * (i - (num_views - 1) / 2.0))
        el = np.deg2rad(15.0 + 3.0 * ((i % 3) - 1))
        C = radius * np.array([np.sin(az) * np.cos(el), -np.sin(el), -np.cos(az) * np.cos(el)])
        R, t = _look_at(C, np.array([0.0, 0.0, 0.0]))
        poses.append((R, t, C, az))
    angles = np.array([p[3] for p in poses])
    pairs = []
    for i in range(num_views):
        order = np.argsort(np.abs(angles - angles[i]), kind="stable")
        pairs.append([int(j) for j in order if j != i])
    return SceneSetup(width=width, height=height, K=K, poses=poses, texture=tex, pairs=pairs)


def render_numpy(setup: SceneSetup, i: int) -> View:
    R, t, C, _ = setup.poses[i]
    K, width, height = setup.K, setup.width, setup.height
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    ys, xs = np.mgrid[0:height, 0:width].astype(np.float64)
    dc = np.stack([(xs - cx) / fx, (ys - cy) / fy, np.ones_like(xs)], axis=-1).reshape(-1, 3)
    Dw = dc @ R  # R^T d for row vectors
    norm = np.linalg.norm(Dw, axis=1, keepdims=True)
    D = Dw / norm
    s, nrm = _intersect(C, D)
    hit = np.isfinite(s)
    X = C + np.where(hit, s, 0.0)[:, None] * D
    val = np.where(hit, setup.texture(X), 40.0)
    img = np.clip(np.rint(val), 0, 255).astype(np.float32).reshape(height, width)
    z = np.where(hit, s / norm[:, 0], 0.0).astype(np.float32).reshape(height, width)
    return View(K=K.astype(np.float32), R=R.astype(np.float32), t=t.astype(np.float32),
                image=img, depth=z, normal=nrm.astype(np.float32).reshape(height, width, 3))


def render_torch(setup: SceneSetup, i: int, device, with_depth: bool = False, rows_per_chunk: int = 256):
    """Same scene rendered with torch on `device` (fp64 geometry); returns the
    (H, W) float32 image tensor on the device (and, with_depth, the camera-z
    depth map, 0 where no surface is hit). Used by bench.py and the GPU tests
    to build inputs directly in HBM; pixel values may differ from
    render_numpy in rare rounding cases (not used for parity).

    Elementwise products only (no BLAS calls, whose algorithm choice at
    24-Mpix shapes changed results between calls) and bounded chunks of rows,
    so the output is deterministic and the temporaries stay small at ETH3D
    sizes."""
    import torch

    R, t, C, _ = setup.poses[i]
    K, width, height = setup.K, setup.width, setup.height
    dt = torch.float64
    tex = setup.texture
    pn = np.array([0.25, -0.15, 1.0])
    pn = pn / np.linalg.norm(pn)
    cs = np.array([-20.0, 10.0, 0.0])
    bmin, bmax = np.array([60.0, -40.0, -60.0]), np.array([150.0, 50.0, 20.0])
    Cpn = float(C @ pn)
    oc = C - cs
    occ = float(oc @ oc)

    def lin(cols, coef):  # sum_k cols[k] * coef[k] (coef: host fp64 scalars or rows)
        out = cols[0] * coef[0]
        for k in range(1, len(cols)):
            out = out + cols[k] * coef[k]
        return out

    img = torch.empty((height, width), dtype=torch.float32, device=device)
    dep = torch.empty((height, width), dtype=torch.float32, device=device) if with_depth else None
    xs1 = torch.arange(width, dtype=dt, device=device)
    f = [torch.tensor(tex.f[:, k], dtype=dt, device=device) for k in range(3)]
    f2 = [torch.tensor(tex.f2[:, k], dtype=dt, device=device) for k in range(3)]
    phase = torch.tensor(tex.phase, dtype=dt, device=device)
    p2 = torch.tensor(tex.p2, dtype=dt, device=device)
    amp = torch.tensor(tex.amp, dtype=dt, device=device)
    amp_norm = float(np.sqrt(0.5 * np.sum(tex.amp ** 2)))
    for r0 in range(0, height, rows_per_chunk):
        r1 = min(height, r0 + rows_per_chunk)
        ys, xs = torch.meshgrid(torch.arange(r0, r1, dtype=dt, device=device), xs1, indexing="ij")
        dc = [((xs - K[0, 2]) / K[0, 0]).reshape(-1), ((ys - K[1, 2]) / K[1, 1]).reshape(-1)]
        dc.append(torch.ones_like(dc[0]))
        Dw = [lin(dc, R[:, j]) for j in range(3)]  # R^T d
        nrm = torch.sqrt(Dw[0] * Dw[0] + Dw[1] * Dw[1] + Dw[2] * Dw[2])
        D = [d / nrm for d in Dw]
        best = torch.full_like(nrm, float("inf"))
        # background plane
        s = (-160.0 - Cpn) / lin(D, pn)
        ok = (s > 1e-3) & torch.isfinite(s) & (s < best)
        best = torch.where(ok, s, best)
        # sphere
        b = lin(D, oc)
        disc = b * b - (occ - 85.0 * 85.0)
        s = -b - torch.sqrt(torch.clamp(disc, min=0.0))
        ok = (disc > 0) & (s > 1e-3) & (s < best)
        best = torch.where(ok, s, best)
        # axis-aligned box
        t1 = [(bmin[k] - C[k]) / D[k] for k in range(3)]
        t2 = [(bmax[k] - C[k]) / D[k] for k in range(3)]
        tn = torch.maximum(torch.maximum(torch.minimum(t1[0], t2[0]), torch.minimum(t1[1], t2[1])),
                           torch.minimum(t1[2], t2[2]))
        tf = torch.minimum(torch.minimum(torch.maximum(t1[0], t2[0]), torch.maximum(t1[1], t2[1])),
                           torch.maximum(t1[2], t2[2]))
        ok = (tn <= tf) & (tn > 1e-3) & (tn < best)
        best = torch.where(ok, tn, best)
        hit = torch.isfinite(best)
        sh = torch.where(hit, best, torch.zeros_like(best))
        X = [C[k] + sh * D[k] for k in range(3)]
        arg = lin([x[:, None] for x in X], f) + phase
        sv = (torch.sin(arg) * amp).sum(dim=1) / amp_norm
        val = 127.5 + 60.0 * torch.tanh(0.9 * sv)
        low = torch.sin(lin([x[:, None] for x in X], f2) + p2).sum(dim=1) / float(np.sqrt(3.0))
        val = torch.where(low > 1.28, torch.full_like(val, 128.0), val)
        val = torch.where(hit, val, torch.full_like(val, 40.0))
        img[r0:r1] = torch.clamp(torch.round(val), 0, 255).to(torch.float32).reshape(r1 - r0, width)
        if with_depth:
            dep[r0:r1] = torch.where(hit, best / torch.sqrt(dc[0] * dc[0] + dc[1] * dc[1] + 1.0),
                                     torch.zeros_like(best)).to(torch.float32).reshape(r1 - r0, width)
    return (img, dep) if with_depth else img


def make_scene(num_views: int = 10, width: int = 1600, height: int = 1200, seed: int = 0x5EED,
               arc_deg: float = 6.0, radius: float = 600.0) -> Scene:
    """Render `num_views` views on an arc (arc_deg apart) at width x height."""
    setup = scene_setup(num_views, width, height, seed, arc_deg, radius)
    return Scene(views=[render_numpy(setup, i) for i in range(num_views)], pairs=setup.pairs)


def write_dense_folder(scene: Scene, folder: str, fmt: str = "jpg", quality: int = 95,
                       num_src: int | None = None) -> None:
    """A COLMAP-converted dense folder (images/%08d.jpg, cams/%08d_cam.txt,
    pair.txt) as colmap2mvsnet_acm.py writes it (:426-445), for the scene's
    views. The depth line is DEPTH_LINE."""
    import os
    from . import io as _io
    os.makedirs(os.path.join(folder, "images"), exist_ok=True)
    os.makedirs(os.path.join(folder, "cams"), exist_ok=True)
    for i, v in enumerate(scene.views):
        img = np.clip(np.rint(v.image), 0, 255).astype(np.uint8)
        path = os.path.join(folder, "images", "%08d.%s" % (i, fmt))
        if fmt == "jpg":
            from PIL import Image
            Image.fromarray(img, "L").save(path, "JPEG", quality=quality)
        elif fmt == "pgm":
            with open(path, "wb") as f:
                f.write(b"P5\n%d %d\n255\n" % (img.shape[1], img.shape[0]) + img.tobytes())
        else:
            raise ValueError(fmt)
        _io.write_camera(os.path.join(folder, "cams", "%08d_cam.txt" % i), v.K, v.R, v.t, DEPTH_LINE[0],
                         DEPTH_LINE[1], DEPTH_LINE[2], DEPTH_LINE[3])
    sel = []
    for i in range(len(scene.views)):
        srcs = list(scene.pairs[i])[: num_src or len(scene.pairs[i])]
        sel.append([(s, len(srcs) - k) for k, s in enumerate(srcs)])
    _io.write_pair(os.path.join(folder, "pair.txt"), sel)
