"""ctypes front-end of the CPU oracle (oracle/acmmp_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg — never by the product package acmmp_amd/.
The oracle restates src/ACMMP.cu (rlav440/ACMMP) on the CPU with the pinned
semantics of SURVEY.md Appendix A; see the header of acmmp_oracle.c.
Parity unpinned against reference outputs (unbuildable here, clock64()-seeded):
pinned by known-answer tests, Philox vectors and the colmap fixtures only.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")

_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB):
        subprocess.run(["make", "-C", HERE, "-s"], check=True)
    return LIB


def _load():
    global _lib
    if _lib is not None:
        return _lib
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    from acmmp_amd import _abi  # struct layouts only
    build()
    lib = C.CDLL(LIB)
    FP = C.POINTER(C.c_float)
    U32P = C.POINTER(C.c_uint32)
    IP = C.POINTER(C.c_int)
    P = C.POINTER(_abi.Params)
    CAM = C.POINTER(_abi.Camera)
    lib.acmmp_oracle_run_patchmatch.restype = C.c_int
    lib.acmmp_oracle_run_patchmatch.argtypes = [P, C.c_int, CAM, C.POINTER(FP), C.POINTER(FP), IP, IP,
                                                FP, FP, U32P, FP, FP, U32P, FP, FP, C.c_int]
    lib.acmmp_oracle_eval_costs.restype = C.c_int
    lib.acmmp_oracle_eval_costs.argtypes = [P, C.c_int, CAM, C.POINTER(FP), FP, FP, FP, U32P, C.c_int]
    lib.acmmp_oracle_eval_geom_costs.restype = C.c_int
    lib.acmmp_oracle_eval_geom_costs.argtypes = [P, C.c_int, CAM, C.POINTER(FP), C.POINTER(FP), FP, FP, C.c_int]
    lib.acmmp_oracle_ncc.restype = C.c_float
    lib.acmmp_oracle_ncc.argtypes = [P, CAM, CAM, FP, FP, C.c_int, C.c_int, FP]
    lib.acmmp_oracle_homography.restype = None
    lib.acmmp_oracle_homography.argtypes = [CAM, CAM, FP, FP]
    lib.acmmp_oracle_philox.restype = C.c_uint32
    lib.acmmp_oracle_philox.argtypes = [C.c_uint32] * 6
    lib.acmmp_oracle_philox4.restype = None
    lib.acmmp_oracle_philox4.argtypes = [C.c_uint32] * 6 + [U32P]
    lib.acmmp_oracle_uniform.restype = C.c_float
    lib.acmmp_oracle_uniform.argtypes = [C.c_uint32] * 6
    for name in ("expf", "sinf", "cosf", "acosf"):
        fn = getattr(lib, "acmmp_oracle_" + name)
        fn.restype = C.c_float
        fn.argtypes = [C.c_float]
    lib.acmmp_oracle_checkerboard_rows.restype = C.c_int
    lib.acmmp_oracle_checkerboard_rows.argtypes = [C.c_int]
    I32P = C.POINTER(C.c_int32)
    lib.acmmp_oracle_support_points.restype = C.c_int
    lib.acmmp_oracle_support_points.argtypes = [FP, C.c_int, C.c_int, I32P]
    lib.acmmp_oracle_prior_plane.restype = None
    lib.acmmp_oracle_prior_plane.argtypes = [CAM, FP, C.c_int, I32P, FP]
    lib.acmmp_oracle_planar_prior.restype = None
    lib.acmmp_oracle_planar_prior.argtypes = [CAM, FP, C.c_int, C.c_int, C.c_float, C.c_float, I32P, C.c_int,
                                              FP, U32P, FP]
    lib.acmmp_oracle_prior_plane_estimate.restype = None
    lib.acmmp_oracle_prior_plane_estimate.argtypes = [C.POINTER(C.c_uint16), C.c_int, C.c_int, C.c_int,
                                                      C.POINTER(C.c_uint16), C.c_int, CAM, C.c_int, C.c_int, FP]
    lib.acmmp_oracle_set_p3_fused.restype = None
    lib.acmmp_oracle_set_p3_fused.argtypes = [C.c_int]
    lib.acmmp_oracle_p3_fused.restype = C.c_int
    lib.acmmp_oracle_jbu.restype = C.c_int
    lib.acmmp_oracle_jbu.argtypes = [FP, C.c_int, C.c_int, FP, C.c_int, C.c_int, FP]
    _lib = lib
    return lib


class p3_unfused:
    """Context manager: the oracle's NCC with r01's unfused P3 form (every
    product and moment rounded separately) instead of the inferred nvcc
    contraction the product pins; for comparisons only."""

    def __enter__(self):
        _load().acmmp_oracle_set_p3_fused(0)
        return self

    def __exit__(self, *exc):
        _load().acmmp_oracle_set_p3_fused(1)


def _f(a):
    return a.ctypes.data_as(C.POINTER(C.c_float)) if a is not None else None


def _u(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint32)) if a is not None else None


def _arrays(arrs):
    arrs = [np.ascontiguousarray(a, dtype=np.float32) for a in arrs]
    return arrs, (C.POINTER(C.c_float) * len(arrs))(*[_f(a) for a in arrs])


def run_patchmatch(params, cams, images, depths=None, planes=None, costs=None, pre_costs=None,
                   prior_planes=None, masks=None, scaled_planes=None, seed_planes=None, nthreads=0):
    """CPU RunPatchMatch. Returns dict(planes (H,W,4), costs, selected_views, pre_costs)."""
    from acmmp_amd import _abi
    lib = _load()
    n = len(cams)
    W, H = cams[0].width, cams[0].height
    cam_arr = (_abi.Camera * n)(*cams)
    imgs, img_ptrs = _arrays(images)
    dep_keep, dep_ptrs = (None, None)
    dw = dh = None
    if depths is not None:
        dep_keep, dep_ptrs = _arrays(depths)
        dw = (C.c_int * n)(*[d.shape[1] for d in dep_keep])
        dh = (C.c_int * n)(*[d.shape[0] for d in dep_keep])
    pl = np.zeros((H, W, 4), np.float32) if planes is None else np.array(planes, np.float32, copy=True)
    co = np.zeros((H, W), np.float32) if costs is None else np.array(costs, np.float32, copy=True)
    sv = np.zeros((H, W), np.uint32)
    pc = np.zeros((H, W), np.float32) if pre_costs is None else np.array(pre_costs, np.float32, copy=True)
    pp = None if prior_planes is None else np.ascontiguousarray(prior_planes, np.float32)
    mk = None if masks is None else np.ascontiguousarray(masks, np.uint32)
    sp = None if scaled_planes is None else np.ascontiguousarray(scaled_planes, np.float32)
    sd = None if seed_planes is None else np.ascontiguousarray(seed_planes, np.float32)
    prm = _abi.Params()
    C.memmove(C.byref(prm), C.byref(params), C.sizeof(prm))
    prm.num_images = n
    rc = lib.acmmp_oracle_run_patchmatch(C.byref(prm), n, cam_arr, img_ptrs, dep_ptrs, dw, dh, _f(pl), _f(co),
                                         _u(sv), _f(pc), _f(pp), _u(mk), _f(sp), _f(sd), int(nthreads))
    if rc != 0:
        raise RuntimeError(f"oracle run_patchmatch failed: {rc}")
    return {"planes": pl, "costs": co, "selected_views": sv, "pre_costs": pc}


def eval_costs(params, cams, images, planes, nthreads=0):
    from acmmp_amd import _abi
    lib = _load()
    n = len(cams)
    W, H = cams[0].width, cams[0].height
    cam_arr = (_abi.Camera * n)(*cams)
    imgs, img_ptrs = _arrays(images)
    pl = np.ascontiguousarray(planes, np.float32)
    out = np.zeros((H, W, n - 1), np.float32)
    init = np.zeros((H, W), np.float32)
    views = np.zeros((H, W), np.uint32)
    prm = _abi.Params()
    C.memmove(C.byref(prm), C.byref(params), C.sizeof(prm))
    prm.num_images = n
    rc = lib.acmmp_oracle_eval_costs(C.byref(prm), n, cam_arr, img_ptrs, _f(pl), _f(out), _f(init), _u(views),
                                     int(nthreads))
    if rc != 0:
        raise RuntimeError("oracle eval_costs failed")
    return out, init, views


def eval_geom_costs(params, cams, images, depths, planes, nthreads=0):
    from acmmp_amd import _abi
    lib = _load()
    n = len(cams)
    W, H = cams[0].width, cams[0].height
    cam_arr = (_abi.Camera * n)(*cams)
    imgs, img_ptrs = _arrays(images)
    deps, dep_ptrs = _arrays(depths)
    pl = np.ascontiguousarray(planes, np.float32)
    out = np.zeros((H, W, n - 1), np.float32)
    prm = _abi.Params()
    C.memmove(C.byref(prm), C.byref(params), C.sizeof(prm))
    prm.num_images = n
    rc = lib.acmmp_oracle_eval_geom_costs(C.byref(prm), n, cam_arr, img_ptrs, dep_ptrs, _f(pl), _f(out),
                                          int(nthreads))
    if rc != 0:
        raise RuntimeError("oracle eval_geom_costs failed")
    return out


def ncc(params, ref_cam, src_cam, ref_img, src_img, px, py, plane):
    lib = _load()
    r = np.ascontiguousarray(ref_img, np.float32)
    s = np.ascontiguousarray(src_img, np.float32)
    pl = np.ascontiguousarray(plane, np.float32)
    return float(lib.acmmp_oracle_ncc(C.byref(params), C.byref(ref_cam), C.byref(src_cam), _f(r), _f(s),
                                      int(px), int(py), _f(pl)))


def homography(ref_cam, src_cam, plane):
    lib = _load()
    pl = np.ascontiguousarray(plane, np.float32)
    H = np.zeros(9, np.float32)
    lib.acmmp_oracle_homography(C.byref(ref_cam), C.byref(src_cam), _f(pl), _f(H))
    return H.reshape(3, 3)


def uniform(seed_lo, seed_hi, pix, draw, phase, stream):
    return float(_load().acmmp_oracle_uniform(seed_lo, seed_hi, pix, draw, phase, stream))


def philox_x(k0, k1, c0, c1, c2, c3):
    return int(_load().acmmp_oracle_philox(k0, k1, c0, c1, c2, c3))


def philox4(k0, k1, c0, c1, c2, c3):
    out = np.zeros(4, np.uint32)
    _load().acmmp_oracle_philox4(k0, k1, c0, c1, c2, c3, out.ctypes.data_as(C.POINTER(C.c_uint32)))
    return [int(v) for v in out]


def math_fn(name, x):
    return float(getattr(_load(), "acmmp_oracle_" + name)(float(x)))


def checkerboard_rows(H):
    return int(_load().acmmp_oracle_checkerboard_rows(int(H)))


def _i(a):
    return a.ctypes.data_as(C.POINTER(C.c_int32))


def support_points(costs):
    """GetSupportPoints (src/ACMMP.cpp:868-894) on a (H, W) cost map."""
    lib = _load()
    c = np.ascontiguousarray(costs, dtype=np.float32)
    h, w = c.shape
    out = np.empty(((w // 5 + 1) * (h // 5 + 1), 2), dtype=np.int32)
    n = lib.acmmp_oracle_support_points(_f(c), w, h, _i(out))
    return out[:n].copy()


def planar_prior(cam, depths, depth_min, depth_max, triangles):
    """Raster + GetPriorPlaneParams + range check + label expansion
    (src/acmmp_definitions.cpp:332-370, src/ACMMP.cpp:811-831, 920-958) for a
    triangle list already restricted to the image. Returns (planes, mask, prior)."""
    lib = _load()
    d = np.ascontiguousarray(depths, dtype=np.float32)
    h, w = d.shape
    tr = np.ascontiguousarray(triangles, dtype=np.int32).reshape(-1, 6)
    planes = np.zeros((max(tr.shape[0], 1), 4), dtype=np.float32)
    mask = np.zeros((h, w), dtype=np.uint32)
    prior = np.zeros((h, w, 4), dtype=np.float32)
    lib.acmmp_oracle_planar_prior(C.byref(cam), _f(d), w, h, float(depth_min), float(depth_max), _i(tr),
                                  int(tr.shape[0]), _f(planes), _u(mask), _f(prior))
    return planes[: tr.shape[0]], mask, prior


def jbu(image, depth):
    """JBU_cu / RunJBU (src/ACMMP.cu:1458-1516, src/ACMMP.cpp:1008-1087).
    Returns (upsampled depth or None when Imagescale == 1, Imagescale)."""
    lib = _load()
    im = np.ascontiguousarray(image, dtype=np.float32)
    d = np.ascontiguousarray(depth, dtype=np.float32)
    out = np.zeros_like(im)
    isc = lib.acmmp_oracle_jbu(_f(im), im.shape[1], im.shape[0], _f(d), d.shape[1], d.shape[0], _f(out))
    return (None if isc == 1 else out), isc


def prior_plane_estimate(depth_u16, normals_bgr_u16, cam, rows, cols):
    """pSampler::GetPriorPlaneEstimate (src/acmmp_definitions.cpp:99-177) on
    decoded maps: depth (H, W[, C]) uint16, normals (H, W, 3) uint16 in BGR."""
    lib = _load()
    d = np.ascontiguousarray(depth_u16, dtype=np.uint16)
    n = np.ascontiguousarray(normals_bgr_u16, dtype=np.uint16)
    dh, dw = d.shape[:2]
    dc = 1 if d.ndim == 2 else d.shape[2]
    out = np.zeros((rows, cols, 4), np.float32)
    u16 = C.POINTER(C.c_uint16)
    lib.acmmp_oracle_prior_plane_estimate(d.ctypes.data_as(u16), dw, dh, dc, n.ctypes.data_as(u16), n.shape[1],
                                          C.byref(cam), rows, cols, _f(out))
    return out
