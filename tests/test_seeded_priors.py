"""Seeded priors (pSampler, src/acmmp_definitions.cpp:8-177) without a GPU:
the library's PNG reader (cv::imread IMREAD_UNCHANGED: BGR order, 16-bit)
against arrays written by an independent encoder (all five row filters) and
by Pillow, and GetPriorPlaneEstimate against the oracle restatement."""
import os
import struct
import zlib

import numpy as np
import pytest

import oracle
from acmmp_amd import _abi, make_camera, pipeline
import ctypes as C


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    return a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)


def write_png(path, arr, bit_depth=16, filters=(0, 1, 2, 3, 4)):
    """Minimal PNG encoder: arr (H, W) or (H, W, C) in RGB(A) order."""
    a = np.asarray(arr)
    if a.ndim == 2:
        a = a[..., None]
    H, W, Cn = a.shape
    ctype = {1: 0, 2: 4, 3: 2, 4: 6}[Cn]
    dt = ">u2" if bit_depth == 16 else "u1"
    raw = a.astype(dt).reshape(H, -1).view(np.uint8).reshape(H, -1)
    bpp = Cn * bit_depth // 8
    out = bytearray()
    prev = np.zeros(raw.shape[1], np.int64)
    for y in range(H):
        f = filters[y % len(filters)]
        cur = raw[y].astype(np.int64)
        res = np.zeros_like(cur)
        for i in range(len(cur)):
            left = cur[i - bpp] if i >= bpp else 0
            ul = prev[i - bpp] if i >= bpp else 0
            pred = [0, left, prev[i], (left + prev[i]) >> 1, _paeth(left, prev[i], ul)][f]
            res[i] = (cur[i] - pred) & 0xFF
        out.append(f)
        out += bytes(res.astype(np.uint8))
        prev = cur

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", W, H, bit_depth, ctype, 0, 0, 0))
    png += chunk(b"IDAT", zlib.compress(bytes(out))) + chunk(b"IEND", b"")
    with open(path, "wb") as fh:
        fh.write(png)


def read_png(path):
    lib = _abi.load_library()
    w, h, c, bd = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    rc = lib.acmmp_read_png(path.encode(), None, 0, C.byref(w), C.byref(h), C.byref(c), C.byref(bd))
    assert rc == _abi.ERR_ARG
    out = np.empty((h.value, w.value, c.value), np.uint16)
    rc = lib.acmmp_read_png(path.encode(), out.ctypes.data_as(C.POINTER(C.c_uint16)), out.size, C.byref(w),
                            C.byref(h), C.byref(c), C.byref(bd))
    assert rc == 0
    return out, bd.value


@pytest.mark.parametrize("channels", [1, 3, 4])
def test_png16_all_filters(tmp_path, channels):
    rng = np.random.default_rng(channels)
    arr = rng.integers(0, 65536, size=(13, 17, channels), dtype=np.uint16)
    p = str(tmp_path / "a.png")
    write_png(p, arr)
    got, bd = read_png(p)
    exp = arr if channels == 1 else np.concatenate([arr[..., 2::-1], arr[..., 3:]], -1)  # RGB(A) -> BGR(A)
    assert bd == 16
    np.testing.assert_array_equal(got, exp)


def test_png8_pillow(tmp_path):
    from PIL import Image
    rng = np.random.default_rng(3)
    rgb = rng.integers(0, 256, size=(21, 11, 3), dtype=np.uint8)
    p = str(tmp_path / "b.png")
    Image.fromarray(rgb, "RGB").save(p)
    got, bd = read_png(p)
    np.testing.assert_array_equal(got, rgb[..., ::-1])
    g16 = rng.integers(0, 65536, size=(9, 14), dtype=np.uint16)
    p2 = str(tmp_path / "c.png")
    Image.fromarray(g16).save(p2)  # mode I;16
    got2, bd2 = read_png(p2)
    assert bd2 == 16
    np.testing.assert_array_equal(got2[..., 0], g16)


def _write_priors(dense, cam_id, depth_u16, normals_rgb_u16):
    os.makedirs(dense + "priors/depths", exist_ok=True)
    os.makedirs(dense + "priors/normals", exist_ok=True)
    write_png(dense + "priors/depths/%08d.png" % cam_id, depth_u16)
    write_png(dense + "priors/normals/%08d.png" % cam_id, normals_rgb_u16)


@pytest.mark.parametrize("scale", [1, 2])
def test_prior_plane_estimate_matches_oracle(tmp_path, scale):
    rows, cols = 12, 16
    dense = str(tmp_path / "dense") + "/"
    rng = np.random.default_rng(scale)
    depth = rng.integers(0, 65536, size=(rows * scale, cols * scale), dtype=np.uint16)
    n = rng.normal(size=(rows * scale, cols * scale, 3))
    n /= np.linalg.norm(n, axis=-1, keepdims=True)
    normals = np.clip((n + 1.0) * 32768.0, 0, 65535).astype(np.uint16)
    _write_priors(dense, 2, depth, normals)
    cam = make_camera([[100.0, 0, 7.5], [0, 100.0, 5.5], [0, 0, 1]], np.eye(3), np.zeros(3), cols, rows, 300.0, 800.0)
    assert pipeline.priors_available(dense, 3) and not pipeline.priors_available(dense, 4)
    got = pipeline.prior_plane_estimate(dense, 2, cam, rows, cols)
    ref = oracle.prior_plane_estimate(depth, normals[..., ::-1], cam, rows, cols)
    np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))
