"""ctypes mirror of include/acmmp.h (the C-ABI of libacmmp_amd.so).

Struct layouts must match the header byte for byte; tests/test_abi.py checks
the sizes and that every declared symbol is exported.
"""
from __future__ import annotations

import ctypes as C
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "acmmp.h")
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libacmmp_amd.so")

MAX_IMAGES = 33

OK = 0
ERR_ARG = -1
ERR_STATE = -2
ERR_HIP = -3
ERR_IO = -4
ERR_UNSUPPORTED = -5


class Camera(C.Structure):
    """== struct Camera (src/acmmp_definitions.h:47-55), 100 bytes."""

    _fields_ = [
        ("K", C.c_float * 9),
        ("R", C.c_float * 9),
        ("t", C.c_float * 3),
        ("height", C.c_int32),
        ("width", C.c_int32),
        ("depth_min", C.c_float),
        ("depth_max", C.c_float),
    ]


class Params(C.Structure):
    """== struct PatchMatchParams (src/ACMMP.h:32-56) + RNG key."""

    _fields_ = [
        ("max_iterations", C.c_int32),
        ("patch_size", C.c_int32),
        ("num_images", C.c_int32),
        ("max_image_size", C.c_int32),
        ("radius_increment", C.c_int32),
        ("sigma_spatial", C.c_float),
        ("sigma_color", C.c_float),
        ("top_k", C.c_int32),
        ("baseline", C.c_float),
        ("depth_min", C.c_float),
        ("depth_max", C.c_float),
        ("disparity_min", C.c_float),
        ("disparity_max", C.c_float),
        ("scaled_cols", C.c_float),
        ("scaled_rows", C.c_float),
        ("geom_consistency", C.c_int32),
        ("planar_prior", C.c_int32),
        ("multi_geometry", C.c_int32),
        ("hierarchy", C.c_int32),
        ("upsample", C.c_int32),
        ("seeded", C.c_int32),
        ("seed_lo", C.c_uint32),
        ("seed_hi", C.c_uint32),
        ("rng_stream", C.c_uint32),
        ("texture_filter8", C.c_int32),
        ("reserved", C.c_int32 * 4),
    ]


class Timing(C.Structure):
    _fields_ = [
        ("init_ms", C.c_float),
        ("sweep_ms", C.c_float),
        ("sweep_launches", C.c_int32),
        ("finalize_ms", C.c_float),
        ("total_ms", C.c_float),
    ]


def default_params() -> Params:
    """Reference defaults of PatchMatchParams (src/ACMMP.h:32-56), pure Python
    (no library needed) — must equal acmmp_default_params()."""
    p = Params()
    p.max_iterations = 2
    p.patch_size = 11
    p.num_images = 5
    p.max_image_size = 3200
    p.radius_increment = 2
    p.sigma_spatial = 5.0
    p.sigma_color = 3.0
    p.top_k = 4
    p.baseline = 0.54
    p.depth_min = 0.0
    p.depth_max = 1.0
    p.disparity_min = 0.0
    p.disparity_max = 1.0
    p.seed_lo = 0x5EED
    p.seed_hi = 0
    p.rng_stream = 0
    return p


class Problem(C.Structure):
    """acmmp_problem == struct Problem (src/acmmp_definitions.h:57-63)."""
    _fields_ = [
        ("ref_image_id", C.c_int32),
        ("num_src_images", C.c_int32),
        ("src_image_ids", C.c_int32 * (MAX_IMAGES - 1)),
        ("max_image_size", C.c_int32),
        ("num_downscale", C.c_int32),
        ("cur_image_size", C.c_int32),
    ]

    @property
    def sources(self) -> list:
        return list(self.src_image_ids[: self.num_src_images])


class PassOptions(C.Structure):
    """acmmp_pass_options: ProcessProblem's flags (src/acmmp_definitions.cpp:245-250)."""
    _fields_ = [
        ("device", C.c_int32),
        ("geom_consistency", C.c_int32),
        ("planar_prior", C.c_int32),
        ("hierarchy", C.c_int32),
        ("multi_geometry", C.c_int32),
        ("seeded", C.c_int32),
        ("max_iterations", C.c_int32),
        ("seed_lo", C.c_uint32),
        ("seed_hi", C.c_uint32),
        ("write_triangulation", C.c_int32),
        ("verbose", C.c_int32),
        ("reserved", C.c_int32 * 5),
    ]


_FP = C.POINTER(C.c_float)
_U32P = C.POINTER(C.c_uint32)
class BandHalo(C.Structure):
    """acmmp_band_halo (include/acmmp.h): the rows one half-sweep of a
    row-band split run exchanges with the neighbouring bands."""
    _fields_ = [("colour", C.c_int32), ("Wh", C.c_int32), ("plane", C.c_void_p), ("cost", C.c_void_p),
                ("sv", C.c_void_p), ("stream", C.c_void_p),
                ("send_up_lo", C.c_int32), ("send_up_hi", C.c_int32),
                ("send_down_lo", C.c_int32), ("send_down_hi", C.c_int32),
                ("recv_up_lo", C.c_int32), ("recv_up_hi", C.c_int32),
                ("recv_down_lo", C.c_int32), ("recv_down_hi", C.c_int32)]


BAND_HALO = 23  # ACMMP_BAND_HALO
BandExchangeFn = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(BandHalo))

_CTX = C.c_void_p

# name -> (restype, argtypes)
_I32P = C.POINTER(C.c_int32)

SIGNATURES = {
    "acmmp_default_params": (None, [C.POINTER(Params)]),
    "acmmp_create": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "acmmp_destroy": (None, [_CTX]),
    "acmmp_release_device_cache": (C.c_int, [C.c_int]),
    "acmmp_device_cache_bytes": (C.c_int64, [C.c_int]),
    "acmmp_last_error": (C.c_char_p, [_CTX]),
    "acmmp_set_params": (C.c_int, [_CTX, C.POINTER(Params)]),
    "acmmp_get_params": (C.c_int, [_CTX, C.POINTER(Params)]),
    "acmmp_set_geom_consistency_params": (C.c_int, [_CTX, C.c_int]),
    "acmmp_set_planar_prior_params": (C.c_int, [_CTX]),
    "acmmp_set_hierarchy_params": (C.c_int, [_CTX]),
    "acmmp_set_images": (C.c_int, [_CTX, C.c_int, C.POINTER(Camera), C.POINTER(_FP), C.c_int]),
    "acmmp_set_depth_maps": (C.c_int, [_CTX, C.POINTER(_FP)]),
    "acmmp_set_depth_maps_device": (C.c_int, [_CTX, C.POINTER(C.c_void_p), C.POINTER(C.c_int32)]),
    "acmmp_set_images_device": (C.c_int, [_CTX, C.c_int, C.POINTER(Camera), C.POINTER(C.c_void_p),
                                          C.POINTER(C.c_int32), C.c_int]),
    "acmmp_set_plane_hypotheses_device": (C.c_int, [_CTX, C.c_void_p, C.c_void_p]),
    "acmmp_wait_stream": (C.c_int, [_CTX, C.c_void_p]),
    "acmmp_texture_create": (C.c_int, [C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)]),
    "acmmp_texture_destroy": (None, [C.c_void_p]),
    "acmmp_texture_bits": (C.c_int, [C.c_void_p]),
    "acmmp_set_images_textures": (C.c_int, [_CTX, C.c_int, C.POINTER(Camera), C.POINTER(C.c_void_p), C.c_int]),
    "acmmp_export_results": (C.c_int, [_CTX, C.c_void_p, C.c_void_p, C.c_void_p]),
    "acmmp_set_plane_hypotheses": (C.c_int, [_CTX, _FP, _FP]),
    "acmmp_set_hierarchy_inputs": (C.c_int, [_CTX, _FP, C.c_int, C.c_int, _FP]),
    "acmmp_set_hierarchy_inputs_device": (C.c_int, [_CTX, C.c_void_p, C.c_int, C.c_int, C.c_void_p]),
    "acmmp_set_seed_prior": (C.c_int, [_CTX, _FP]),
    "acmmp_set_planar_prior": (C.c_int, [_CTX, _FP, C.c_int, _U32P]),
    "acmmp_get_support_points": (C.c_int, [_CTX, _I32P, C.c_int, C.POINTER(C.c_int)]),
    "acmmp_delaunay_triangulation": (C.c_int, [C.c_int, C.c_int, _I32P, C.c_int, _I32P, C.c_int,
                                               C.POINTER(C.c_int)]),
    "acmmp_build_planar_prior": (C.c_int, [_CTX, _I32P, C.c_int, _FP, _U32P]),
    "acmmp_prepare_planar_prior": (C.c_int, [_CTX, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "acmmp_joint_bilateral_upsample": (C.c_int, [C.c_int, _FP, C.c_int, C.c_int, _FP, C.c_int, C.c_int, _FP,
                                                 C.POINTER(C.c_int)]),
    "acmmp_joint_bilateral_upsample_device": (C.c_int, [C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                                        C.c_int, C.c_void_p, C.POINTER(C.c_int)]),
    "acmmp_run_patchmatch": (C.c_int, [_CTX]),
    "acmmp_run_patchmatch_async": (C.c_int, [_CTX]),
    "acmmp_synchronize": (C.c_int, [_CTX]),
    "acmmp_run_patchmatch_band": (C.c_int, [_CTX, C.c_int, C.c_int, BandExchangeFn, C.c_void_p]),
    "acmmp_get_plane_hypotheses": (C.c_int, [_CTX, _FP, C.c_size_t]),
    "acmmp_get_costs": (C.c_int, [_CTX, _FP, C.c_size_t]),
    "acmmp_get_selected_views": (C.c_int, [_CTX, _U32P, C.c_size_t]),
    "acmmp_get_device_results": (C.c_int, [_CTX, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]),
    "acmmp_get_reference_size": (C.c_int, [_CTX, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "acmmp_get_camera": (C.c_int, [_CTX, C.c_int, C.POINTER(Camera)]),
    "acmmp_eval_costs": (C.c_int, [_CTX, _FP, _FP, _FP, _U32P]),
    "acmmp_eval_geom_costs": (C.c_int, [_CTX, _FP, _FP]),
    "acmmp_set_timing": (C.c_int, [_CTX, C.c_int]),
    "acmmp_get_timing": (C.c_int, [_CTX, C.POINTER(Timing)]),
    "acmmp_selftest_reciprocal": (C.c_int, [C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "acmmp_get_texel_bits": (C.c_int, [_CTX]),
    "acmmp_device_count": (C.c_int, []),
    "acmmp_version": (C.c_char_p, []),
    "acmmp_host_threads": (C.c_int, []),
    "acmmp_generate_sample_list": (C.c_int, [C.c_char_p, C.POINTER(Problem), C.c_int, C.POINTER(C.c_int)]),
    "acmmp_compute_multiscale_settings": (C.c_int, [C.c_char_p, C.POINTER(Problem), C.c_int, C.POINTER(C.c_int)]),
    "acmmp_input_initialization": (C.c_int, [_CTX, C.c_char_p, C.c_char_p, C.POINTER(Problem), C.c_int, C.c_int]),
    "acmmp_load_view": (C.c_int, [C.c_char_p, C.c_int, C.c_int, _FP, C.c_size_t, C.POINTER(Camera)]),
    "acmmp_space_initialization": (C.c_int, [_CTX, C.c_char_p, C.POINTER(Problem)]),
    "acmmp_process_problem": (C.c_int, [C.c_char_p, C.c_char_p, C.POINTER(Problem), C.c_int, C.c_int,
                                        C.POINTER(PassOptions)]),
    "acmmp_joint_bilateral_upsampling": (C.c_int, [C.c_char_p, C.c_char_p, C.POINTER(Problem), C.c_int, C.c_int]),
    "acmmp_pipeline_last_error": (C.c_char_p, []),
    "acmmp_run_fusion": (C.c_int, [C.c_char_p, C.c_char_p, C.POINTER(Problem), C.c_int, C.c_int, C.c_float, C.c_int,
                                   C.c_char_p, C.c_char_p, C.c_int, C.POINTER(C.c_int)]),
    "acmmp_fusion_last_error": (C.c_char_p, []),
    "acmmp_run_prior_aware_fusion": (C.c_int, [C.c_char_p, C.c_char_p, C.c_char_p, C.POINTER(Problem), C.c_int,
                                               C.c_int, C.c_float, C.c_int, C.c_int, C.POINTER(C.c_int)]),
    "acmmp_priors_available": (C.c_int, [C.c_char_p, C.c_int]),
    "acmmp_prior_plane_estimate": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(Camera), C.c_int, C.c_int, _FP]),
    "acmmp_read_png": (C.c_int, [C.c_char_p, C.POINTER(C.c_uint16), C.c_size_t, C.POINTER(C.c_int),
                                 C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "acmmp_get_reference_image": (C.c_int, [_CTX, _FP, C.c_size_t]),
    "acmmp_prior_plane_params": (C.c_int, [C.POINTER(Camera), _I32P, _FP, _FP]),
    "acmmp_depth_from_plane_param": (C.c_float, [C.POINTER(Camera), _FP, C.c_int, C.c_int]),
    "acmmp_read_image_bgr": (C.c_int, [C.c_char_p, C.POINTER(C.c_uint8), C.c_size_t, C.POINTER(C.c_int),
                                       C.POINTER(C.c_int)]),
    "acmmp_read_image_gray": (C.c_int, [C.c_char_p, _FP, C.c_size_t, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "acmmp_image_size": (C.c_int, [C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "acmmp_resize_linear": (C.c_int, [_FP, C.c_int, C.c_int, _FP, C.c_int, C.c_int]),
    "acmmp_read_camera": (C.c_int, [C.c_char_p, C.POINTER(Camera)]),
    "acmmp_read_dmb": (C.c_int, [C.c_char_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                 C.POINTER(C.c_int32), _FP, C.c_size_t]),
    "acmmp_write_dmb": (C.c_int, [C.c_char_p, C.c_int32, C.c_int32, C.c_int32, _FP]),
}


def header_symbols(path: str = HEADER) -> list[str]:
    """Function names declared in include/acmmp.h."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(acmmp_[a-z0-9_]+)\s*\(", text)))


_lib = None


def load_library(path: str | None = None) -> C.CDLL:
    """Load libacmmp_amd.so (built in-tree by __graft_entry__.build()).

    Raises a clear error when the native library is missing: there is no
    Python or CPU fallback for the product path.
    """
    global _lib
    if _lib is not None:
        return _lib
    # ACMMP_LIB selects an alternative in-tree build (A/B variants)
    path = path or os.environ.get("ACMMP_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise RuntimeError(
            f"libacmmp_amd.so not found at {path}: build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
    # One HIP runtime per process: torch ships its own libamdhip64 (same
    # soname as /opt/rocm's). Loaded first, it also serves this library; the
    # other order leaves two runtimes and torch then finds no device.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:  # an older A/B build without this entry point: calling it raises AttributeError
            continue
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib
