"""The reference's on-disk formats in numpy (no OpenCV).

  cams/%08d_cam.txt  ReadCamera         src/ACMMP.cpp:154-179
                     (producer: python_scripts/colmap2mvsnet_acm.py:426-439)
  pair.txt           GenerateSampleList src/acmmp_definitions.cpp:179-205
                     (producer: python_scripts/colmap2mvsnet_acm.py:440-445)
  *.dmb              read/write{Depth,Normal}Dmb src/ACMMP.cpp:264-380:
                     int32 type=1, h, w, nb, then h*w*nb float32, HWC.
  2333_%08d/         per-view output folder (src/acmmp_definitions.cpp:254-258)
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np

from . import _abi


@dataclass
class Problem:
    """struct Problem (src/acmmp_definitions.h:57-63)."""

    ref_image_id: int
    src_image_ids: list = field(default_factory=list)
    max_image_size: int = 6400
    num_downscale: int = 0
    cur_image_size: int = 6400


def read_dmb(path: str) -> np.ndarray:
    """Returns (h, w) for nb == 1, else (h, w, nb). Raises on a bad header
    (the reference returns -1 and callers ignore it, src/ACMMP.cpp:282-285)."""
    with open(path, "rb") as f:
        hdr = np.frombuffer(f.read(16), dtype="<i4")
        if hdr.size != 4 or hdr[0] != 1:
            raise ValueError(f"{path}: not a type-1 .dmb file")
        h, w, nb = (int(v) for v in hdr[1:])
        data = np.frombuffer(f.read(h * w * nb * 4), dtype="<f4")
    if data.size != h * w * nb:
        raise ValueError(f"{path}: truncated")
    data = data.reshape(h, w, nb).copy()
    return data[:, :, 0] if nb == 1 else data


def write_dmb(path: str, arr: np.ndarray) -> None:
    a = np.ascontiguousarray(arr, dtype="<f4")
    if a.ndim == 2:
        a = a[:, :, None]
    h, w, nb = a.shape
    with open(path, "wb") as f:
        f.write(np.array([1, h, w, nb], dtype="<i4").tobytes())
        f.write(a.tobytes())


def read_camera(path: str) -> _abi.Camera:
    """ReadCamera: whitespace-token parser of the MVSNet cam.txt layout."""
    toks = open(path).read().split()
    i = 1  # skip "extrinsic"
    cam = _abi.Camera()
    vals = [float(v) for v in toks[i:i + 16]]
    i += 16
    for r in range(3):
        cam.R[3 * r + 0], cam.R[3 * r + 1], cam.R[3 * r + 2] = vals[4 * r:4 * r + 3]
        cam.t[r] = vals[4 * r + 3]
    i += 1  # "intrinsic"
    kv = [float(v) for v in toks[i:i + 9]]
    i += 9
    for k in range(9):
        cam.K[k] = kv[k]
    cam.depth_min = float(toks[i])
    cam.depth_max = float(toks[i + 3])
    return cam


def write_camera(path: str, K, R, t, depth_min: float, interval: float, depth_num: float,
                 depth_max: float) -> None:
    """Same layout as colmap2mvsnet_acm.py:430-439."""
    E = np.eye(4)
    E[:3, :3] = np.asarray(R, dtype=np.float64)
    E[:3, 3] = np.asarray(t, dtype=np.float64).reshape(3)
    K = np.asarray(K, dtype=np.float64)
    with open(path, "w") as f:
        f.write("extrinsic\n")
        for j in range(4):
            f.write(" ".join(repr(float(v)) for v in E[j]) + " \n")
        f.write("\nintrinsic\n")
        for j in range(3):
            f.write(" ".join(repr(float(v)) for v in K[j]) + " \n")
        f.write("\n%f %f %f %f\n" % (depth_min, interval, depth_num, depth_max))


def read_pair(path: str) -> list[Problem]:
    """GenerateSampleList: sources with score <= 0 are dropped (:198)."""
    toks = open(path).read().split()
    n = int(toks[0])
    i = 1
    problems = []
    for _ in range(n):
        ref = int(toks[i])
        m = int(toks[i + 1])
        i += 2
        srcs = []
        for _ in range(m):
            sid, score = int(toks[i]), float(toks[i + 1])
            i += 2
            if score <= 0.0:
                continue
            srcs.append(sid)
        problems.append(Problem(ref_image_id=ref, src_image_ids=srcs))
    return problems


def write_pair(path: str, view_sel: list[list[tuple[int, float]]]) -> None:
    with open(path, "w") as f:
        f.write("%d\n" % len(view_sel))
        for i, sel in enumerate(view_sel):
            f.write("%d\n%d " % (i, len(sel)))
            for image_id, s in sel:
                f.write("%d %d " % (image_id, s))
            f.write("\n")


def result_folder(output_folder: str, ref_image_id: int) -> str:
    return os.path.join(output_folder, "2333_%08d" % ref_image_id)


def read_image_gray(path: str) -> np.ndarray:
    """cv::imread(path, IMREAD_GRAYSCALE) -> float32 (src/ACMMP.cpp:538-541)
    through the library's decoder (baseline JPEG luminance / PGM / PFM)."""
    import ctypes as C
    lib = _abi.load_library()
    w, h = C.c_int(0), C.c_int(0)
    rc = lib.acmmp_image_size(path.encode(), C.byref(w), C.byref(h))
    if rc != 0:
        raise IOError(f"{path}: cannot read image header (status {rc})")
    out = np.empty((h.value, w.value), dtype=np.float32)
    rc = lib.acmmp_read_image_gray(path.encode(), out.ctypes.data_as(C.POINTER(C.c_float)), out.size,
                                   C.byref(w), C.byref(h))
    if rc != 0:
        raise IOError(f"{path}: cannot decode image (status {rc})")
    return out


def image_size(path: str) -> tuple[int, int]:
    """(width, height) from the file header."""
    import ctypes as C
    lib = _abi.load_library()
    w, h = C.c_int(0), C.c_int(0)
    rc = lib.acmmp_image_size(path.encode(), C.byref(w), C.byref(h))
    if rc != 0:
        raise IOError(f"{path}: cannot read image header (status {rc})")
    return w.value, h.value


def resize_linear(img: np.ndarray, width: int, height: int) -> np.ndarray:
    """cv::resize(..., INTER_LINEAR) of a float image (src/ACMMP.cpp:589)."""
    import ctypes as C
    lib = _abi.load_library()
    src = np.ascontiguousarray(img, dtype=np.float32)
    out = np.empty((height, width), dtype=np.float32)
    fp = C.POINTER(C.c_float)
    rc = lib.acmmp_resize_linear(src.ctypes.data_as(fp), src.shape[1], src.shape[0], out.ctypes.data_as(fp),
                                 width, height)
    if rc != 0:
        raise ValueError(f"acmmp_resize_linear failed (status {rc})")
    return out


def read_image_bgr(path: str) -> np.ndarray:
    """cv::imread(path, IMREAD_COLOR) -> (H, W, 3) uint8 BGR (baseline JPEG or 8-bit PNG)."""
    import ctypes as C
    lib = _abi.load_library()
    w, h = C.c_int(0), C.c_int(0)
    rc = lib.acmmp_read_image_bgr(path.encode(), None, 0, C.byref(w), C.byref(h))
    if rc != _abi.ERR_ARG:
        raise IOError(f"{path}: cannot decode image (status {rc})")
    out = np.empty((h.value, w.value, 3), dtype=np.uint8)
    rc = lib.acmmp_read_image_bgr(path.encode(), out.ctypes.data_as(C.POINTER(C.c_uint8)), out.size, C.byref(w),
                                  C.byref(h))
    if rc != 0:
        raise IOError(f"{path}: cannot decode image (status {rc})")
    return out
