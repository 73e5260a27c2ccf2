"""Host decoded-image cache (acmmp_pipeline.cpp load_image): a cached decode is
served only while the file is unchanged; a rewritten image is decoded again.
CPU only: acmmp_load_view is host code (InputInitialization's per-view load,
src/ACMMP.cpp:536-598)."""
import ctypes as C
import os

import numpy as np

from acmmp_amd import _abi
from acmmp_amd import io as aio


def _write_pgm(path, img):
    with open(path, "wb") as f:
        f.write(b"P5\n%d %d\n255\n" % (img.shape[1], img.shape[0]) + img.astype(np.uint8).tobytes())


def _load(lib, dense, h, w):
    cam = _abi.Camera()
    out = np.empty((h, w), dtype=np.float32)
    rc = lib.acmmp_load_view(dense.encode(), 0, 4096, out.ctypes.data_as(C.POINTER(C.c_float)), out.size,
                             C.byref(cam))
    assert rc == 0, lib.acmmp_pipeline_last_error().decode()
    return out


def test_rewritten_image_is_decoded_again(tmp_path):
    lib = _abi.load_library()
    dense = str(tmp_path)
    os.makedirs(os.path.join(dense, "images"))
    os.makedirs(os.path.join(dense, "cams"))
    K = np.array([[100.0, 0, 16], [0, 100.0, 12], [0, 0, 1]])
    aio.write_camera(os.path.join(dense, "cams", "00000000_cam.txt"), K, np.eye(3), np.zeros(3), 1.0, 1.0, 192, 10.0)
    rng = np.random.default_rng(7)
    path = os.path.join(dense, "images", "00000000.pgm")
    a = rng.integers(0, 256, (24, 32))
    _write_pgm(path, a)
    np.testing.assert_array_equal(_load(lib, dense, 24, 32), a)
    np.testing.assert_array_equal(_load(lib, dense, 24, 32), a)  # served from the cache
    b = 255 - a
    _write_pgm(path, b)
    st = os.stat(path)
    os.utime(path, ns=(st.st_atime_ns, st.st_mtime_ns + 1_000_000_000))  # a later mtime, whatever the clock
    np.testing.assert_array_equal(_load(lib, dense, 24, 32), b)
