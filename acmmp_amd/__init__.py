"""acmmp_amd — MI355X-native ACMMP PatchMatch MVS engine.

The product is libacmmp_amd.so (acmmp_amd/csrc: hand-written gfx950 HIP
kernels behind the C-ABI in include/acmmp.h). This package is its Python host
mirror: the reference's `ACMMP` class surface (engine.ACMMP), the reference's
on-disk formats (io), seeded synthetic scenes (scene) and the multi-view pass
driver (driver).
"""
from ._abi import Camera, Params, default_params, load_library  # noqa: F401
from .engine import ACMMP, AcmmpError, make_camera, device_count, delaunay_triangulation, joint_bilateral_upsample  # noqa: F401

__all__ = ["ACMMP", "AcmmpError", "Camera", "Params", "default_params", "load_library",
           "make_camera", "device_count"]
