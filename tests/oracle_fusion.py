"""RunFusion (src/acmmp_definitions.cpp:828-1043) restated in Python with
float32 scalar arithmetic — TEST INFRASTRUCTURE, the checker of
acmmp_amd/csrc/acmmp_fusion.cpp. Same order dependence as the reference
(masks updated as points are approved; used_list never reset per pixel).
expf / acosf come from the C math library (ctypes), as in the C++ build;
colours are decoded by Pillow (libjpeg), depth/normal maps read as .dmb."""
import ctypes
import math
import os

import numpy as np

from acmmp_amd import io as aio

_libm = ctypes.CDLL("libm.so.6")
_libm.expf.restype = ctypes.c_float
_libm.expf.argtypes = [ctypes.c_float]
_libm.acosf.restype = ctypes.c_float
_libm.acosf.argtypes = [ctypes.c_float]
f32 = np.float32


def _world(x, y, depth, cam):
    K, R, t = [f32(v) for v in cam.K], [f32(v) for v in cam.R], [f32(v) for v in cam.t]
    px = depth * (f32(x) - K[2]) / K[0]
    py = depth * (f32(y) - K[5]) / K[4]
    pz = depth
    tx = R[0] * px + R[3] * py + R[6] * pz
    ty = R[1] * px + R[4] * py + R[7] * pz
    tz = R[2] * px + R[5] * py + R[8] * pz
    cx = -(R[0] * t[0] + R[3] * t[1] + R[6] * t[2])
    cy = -(R[1] * t[0] + R[4] * t[1] + R[7] * t[2])
    cz = -(R[2] * t[0] + R[5] * t[1] + R[8] * t[2])
    return (tx + cx, ty + cy, tz + cz)


def _project(X, cam):
    K, R, t = [f32(v) for v in cam.K], [f32(v) for v in cam.R], [f32(v) for v in cam.t]
    tx = R[0] * X[0] + R[1] * X[1] + R[2] * X[2] + t[0]
    ty = R[3] * X[0] + R[4] * X[1] + R[5] * X[2] + t[1]
    tz = R[6] * X[0] + R[7] * X[1] + R[8] * X[2] + t[2]
    depth = K[6] * tx + K[7] * ty + K[8] * tz
    px = (K[0] * tx + K[1] * ty + K[2] * tz) / depth
    py = (K[3] * tx + K[4] * ty + K[5] * tz) / depth
    return px, py, depth


def _angle(a, b):
    dot = a[0] * b[0] + a[1] * b[1] + a[2] * b[2]
    ang = f32(_libm.acosf(float(dot)))
    return f32(0.0) if ang != ang else ang


def _initial_mask(dense, mask_folder, ref_id, shape):
    """:881-905: cv::imread(mask, -1) (the file's depth and channels, colour as
    B, G, R[, A]), mask = (mask < 128) / 255, then read and written with
    at<uchar>(r, c), i.e. byte c of row r of the (possibly multi-channel)
    mask. Masks of the depth map's size only (cv::resize is then the identity)."""
    from PIL import Image
    a = np.asarray(Image.open(os.path.join(dense, mask_folder, "%08d.png" % ref_id)))
    if a.ndim == 3:
        a = np.concatenate([a[..., 2::-1], a[..., 3:]], -1)  # RGB[A] -> BGR[A]
    H, W = shape
    assert a.shape[:2] == (H, W)
    rows = a.reshape(H, -1)
    return (rows[:, :W] < 128).astype(np.uint8)


def run_fusion(dense, out, geom=True, consistency_scalar=0.3, con_num_thresh=1, mask_folder=None):
    from PIL import Image
    problems = aio.read_pair(os.path.join(dense, "pair.txt"))
    index = {p.ref_image_id: i for i, p in enumerate(problems)}
    imgs, cams, depths, normals, masks = [], [], [], [], []
    for p in problems:
        rgb = np.asarray(Image.open(os.path.join(dense, "images", "%08d.jpg" % p.ref_image_id)).convert("RGB"))
        imgs.append(rgb[..., ::-1])
        cams.append(aio.read_camera(os.path.join(dense, "cams", "%08d_cam.txt" % p.ref_image_id)))
        rf = aio.result_folder(out, p.ref_image_id)
        depths.append(aio.read_dmb(os.path.join(rf, "depths_geom.dmb" if geom else "depths.dmb")))
        normals.append(aio.read_dmb(os.path.join(rf, "normals.dmb")))
        masks.append(np.zeros(depths[-1].shape, np.uint8) if mask_folder is None else
                     _initial_mask(dense, mask_folder, p.ref_image_id, depths[-1].shape))
    cloud = []
    for i, p in enumerate(problems):
        H, W = depths[i].shape
        srcs = [index[s] for s in p.src_image_ids]
        used = [(-1, -1)] * len(srcs)
        depth_max = f32(cams[i].depth_max)
        for r in range(H):
            for c in range(W):
                if masks[i][r, c] == 1:
                    continue
                ref_depth = f32(depths[i][r, c])
                ref_normal = [f32(v) for v in normals[i][r, c]]
                if ref_depth <= 0.0 or ref_depth >= depth_max:
                    continue
                X = _world(c, r, ref_depth, cams[i])
                num_consistent = 0
                dyn = f32(0.0)
                for j, s in enumerate(srcs):
                    sh, sw = depths[s].shape
                    px, py, _ = _project(X, cams[s])
                    src_r = int(py + f32(0.5))
                    src_c = int(px + f32(0.5))
                    if 0 <= src_c < sw and 0 <= src_r < sh:
                        if masks[s][src_r, src_c] == 1:
                            continue
                        src_depth = f32(depths[s][src_r, src_c])
                        src_normal = [f32(v) for v in normals[s][src_r, src_c]]
                        if src_depth <= 0.0:
                            continue
                        tX = _world(src_c, src_r, src_depth, cams[s])
                        tx, ty, proj_depth = _project(tX, cams[i])
                        reproj = f32(math.sqrt(float(f32(c) - tx) ** 2 + float(f32(r) - ty) ** 2))
                        rel = abs(proj_depth - ref_depth) / ref_depth
                        ang = _angle(ref_normal, src_normal)
                        if reproj < 2.0 and rel < f32(0.01) and ang < f32(0.174533):
                            used[j] = (src_c, src_r)
                            tmp_index = reproj + f32(200) * rel + ang * f32(10)
                            dyn = dyn + f32(_libm.expf(float(-tmp_index)))
                            num_consistent += 1
                if num_consistent >= con_num_thresh and dyn > f32(consistency_scalar) * f32(num_consistent):
                    b, g, rr = (int(v) for v in imgs[i][r, c])
                    cloud.append((X, ref_normal, (rr, g, b)))
                    for j, s in enumerate(srcs):
                        if used[j][0] == -1:
                            continue
                        masks[s][used[j][1], used[j][0]] = 1
    return cloud


def read_ply(path):
    with open(path, "rb") as f:
        data = f.read()
    head, body = data.split(b"end_header\n", 1)
    n = int([l for l in head.split(b"\n") if l.startswith(b"element vertex")][0].split()[-1])
    rec = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("nx", "<f4"), ("ny", "<f4"), ("nz", "<f4"),
                    ("r", "u1"), ("g", "u1"), ("b", "u1")])
    return np.frombuffer(body, dtype=rec, count=n)


def _metric(i, r, c, ref_depth, ref_normal, cams, s, src_r, src_c, src_depth, src_normal):
    if not src_depth > 0:
        return (f32(1e6), f32(1e6), f32(1e6))
    tX = _world(src_c, src_r, src_depth, cams[s])
    tx, ty, proj_depth = _project(tX, cams[i])
    reproj = f32(math.sqrt(float(f32(c) - tx) ** 2 + float(f32(r) - ty) ** 2))
    rel = abs(proj_depth - ref_depth) / ref_depth
    return (reproj, rel, _angle(ref_normal, src_normal))


def _cmetrics(i, r, c, ref_depth, ref_normal, cams, s, src_r, src_c, maps):
    depths, normals, pdepths, pnormals = maps
    res = [_metric(i, r, c, ref_depth, ref_normal, cams, s, src_r, src_c, f32(d[s][src_r, src_c]),
                   [f32(v) for v in nn[s][src_r, src_c]]) for d, nn in ((depths, normals), (pdepths, pnormals))]
    th = [m[0] < 2.0 and m[1] < f32(0.01) and m[2] < f32(0.174533) for m in res]
    dc = [f32(_libm.expf(float(-(m[0] + f32(200) * m[1] + m[2] * f32(10))))) for m in res]
    if th[0] and th[1]:
        return (max(dc[0], dc[1]), src_c, src_r, True, s)
    if th[0]:
        return (dc[0], src_c, src_r, True, s)
    if th[1]:
        return (dc[1], src_c, src_r, True, s)
    return (f32(0), src_c, src_r, False, -1)


def run_prior_aware_fusion(dense, out, fusion_folder, geom=True, consistency_scalar=0.3, con_num_thresh=1,
                           penalty=0):
    """RunPriorAwareFusion (src/acmmp_definitions.cpp:573-826) restated."""
    from PIL import Image
    problems = aio.read_pair(os.path.join(dense, "pair.txt"))
    index = {p.ref_image_id: i for i, p in enumerate(problems)}
    suffix = "depths_geom.dmb" if geom else "depths.dmb"
    imgs, cams, depths, normals, pdepths, pnormals, masks = [], [], [], [], [], [], []
    for p in problems:
        rgb = np.asarray(Image.open(os.path.join(dense, "images", "%08d.jpg" % p.ref_image_id)).convert("RGB"))
        imgs.append(rgb[..., ::-1])
        cams.append(aio.read_camera(os.path.join(dense, "cams", "%08d_cam.txt" % p.ref_image_id)))
        rf, pf = aio.result_folder(fusion_folder, p.ref_image_id), aio.result_folder(out, p.ref_image_id)
        depths.append(aio.read_dmb(os.path.join(rf, suffix)))
        normals.append(aio.read_dmb(os.path.join(rf, "normals.dmb")))
        pdepths.append(aio.read_dmb(os.path.join(pf, suffix)))
        pnormals.append(aio.read_dmb(os.path.join(pf, "normals.dmb")))
        masks.append(np.zeros(depths[-1].shape, np.uint8))
    maps = (depths, normals, pdepths, pnormals)
    cloud = []
    for i, p in enumerate(problems):
        H, W = depths[i].shape
        srcs = [index[s] for s in p.src_image_ids]

        def cands(r, c, ref_depth, ref_normal):
            out_c = []
            for s in srcs:
                sh, sw = depths[s].shape
                X = _world(c, r, ref_depth, cams[i])
                px, py, _ = _project(X, cams[s])
                src_r, src_c = int(py + f32(0.5)), int(px + f32(0.5))
                if 0 <= src_c < sw and 0 <= src_r < sh:
                    if masks[s][src_r, src_c] == 1:
                        continue
                    out_c.append(_cmetrics(i, r, c, ref_depth, ref_normal, cams, s, src_r, src_c, maps))
            return out_c

        for r in range(H):
            for c in range(W):
                if masks[i][r, c] == 1:
                    continue
                rd, rpd = f32(depths[i][r, c]), f32(pdepths[i][r, c])
                rn = [f32(v) for v in normals[i][r, c]]
                rpn = [f32(v) for v in pnormals[i][r, c]]
                if rd <= 0.0 and rpd <= 0.0:
                    continue
                c0, c1, n0, n1, d0, d1, t0, t1 = [], [], 0, 0, f32(0), f32(0), False, False
                if rd > 0.0:
                    c0 = cands(r, c, rd, rn)
                    for k in c0:
                        if k[3]:
                            n0 += 1
                            d0 = d0 + k[0]
                    t0 = n0 >= con_num_thresh and d0 > f32(consistency_scalar) * f32(n0)
                if rpd > 0.0:
                    c1 = cands(r, c, rpd, rpn)
                    for k in c1:
                        if k[3]:
                            n1 += 1
                            d1 = d1 + k[0]
                    t1 = n1 >= con_num_thresh and d1 > f32(consistency_scalar) * f32(n1)
                if t0 and t1:
                    passing = True
                    it, gd, gn = (c1, rpd, rpn) if n1 >= n0 else (c0, rd, rn)
                elif t1:
                    passing = n1 >= con_num_thresh + penalty
                    it, gd, gn = c1, rpd, rpn
                else:
                    passing = t0 and n0 >= con_num_thresh + penalty
                    it, gd, gn = c0, rd, rn
                if passing:
                    b, g, rr = (int(v) for v in imgs[i][r, c])
                    cloud.append((_world(c, r, gd, cams[i]), gn, (rr, g, b)))
                    for k in it:
                        if k[3]:
                            masks[k[4]][k[2], k[1]] = 1
    return cloud
