"""The reference's pass driver (src/main_ACMMP.cpp:96-176,
src/acmmp_definitions.cpp:179-438) over the library's C-ABI.

`run_sequential` is the single-process schedule of main_ACMMP: views in order
inside a pass, so a second geometric pass reads maps already rewritten in the
same pass (Gauss-Seidel). The same loop ships as the C++ command-line tool
`acmmp_amd/lib/acmmp_main`; this module drives it in-process and is the base of
the view-parallel driver (acmmp_amd/distributed.py).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Sequence

from . import _abi
from .engine import AcmmpError

MAX_PROBLEMS = 1 << 14


def _err(what: str, rc: int):
    lib = _abi.load_library()
    msg = lib.acmmp_pipeline_last_error().decode(errors="replace")
    raise AcmmpError(f"{what} failed (status {rc}): {msg}")


def generate_sample_list(dense_folder: str) -> list:
    """GenerateSampleList (src/acmmp_definitions.cpp:179-205)."""
    lib = _abi.load_library()
    buf = (_abi.Problem * MAX_PROBLEMS)()
    n = C.c_int(0)
    rc = lib.acmmp_generate_sample_list(dense_folder.encode(), buf, MAX_PROBLEMS, C.byref(n))
    if rc != 0:
        _err("GenerateSampleList", rc)
    return [buf[i] for i in range(n.value)]


def _array(problems: Sequence):
    arr = (_abi.Problem * len(problems))()
    for i, p in enumerate(problems):
        arr[i] = p
    return arr


def compute_multiscale_settings(dense_folder: str, problems: list) -> int:
    """ComputeMultiScaleSettings (src/acmmp_definitions.cpp:207-243); updates
    `problems` in place, returns max_num_downscale."""
    lib = _abi.load_library()
    arr = _array(problems)
    k = C.c_int(-1)
    rc = lib.acmmp_compute_multiscale_settings(dense_folder.encode(), arr, len(problems), C.byref(k))
    if rc != 0:
        _err("ComputeMultiScaleSettings", rc)
    problems[:] = [arr[i] for i in range(len(problems))]
    return k.value


def priors_available(dense_folder: str, num_cams: int) -> bool:
    """pSampler::confirm_using_prior (src/acmmp_definitions.cpp:8-29, 91-93)."""
    return bool(_abi.load_library().acmmp_priors_available(dense_folder.encode(), num_cams))


def prior_plane_estimate(dense_folder: str, cam_num: int, cam, rows: int, cols: int):
    """pSampler::GetPriorPlaneEstimate (src/acmmp_definitions.cpp:99-177)."""
    import numpy as np
    out = np.empty((rows, cols, 4), dtype=np.float32)
    rc = _abi.load_library().acmmp_prior_plane_estimate(dense_folder.encode(), cam_num, C.byref(cam), rows, cols,
                                                        out.ctypes.data_as(C.POINTER(C.c_float)))
    if rc != 0:
        _err("GetPriorPlaneEstimate", rc)
    return out


def pass_options(geom_consistency=False, planar_prior=False, hierarchy=False, multi_geometry=False,
                 device=0, max_iterations=0, seed_lo=1234, seed_hi=0, write_triangulation=True,
                 verbose=False, seeded=False) -> _abi.PassOptions:
    o = _abi.PassOptions()
    o.seeded = int(seeded)
    o.device = device
    o.geom_consistency = int(geom_consistency)
    o.planar_prior = int(planar_prior)
    o.hierarchy = int(hierarchy)
    o.multi_geometry = int(multi_geometry)
    o.max_iterations = max_iterations
    o.seed_lo = seed_lo & 0xFFFFFFFF
    o.seed_hi = seed_hi & 0xFFFFFFFF
    o.write_triangulation = int(write_triangulation)
    o.verbose = int(verbose)
    return o


def process_problem(dense_folder: str, output_folder: str, problems: Sequence, idx: int,
                    options: _abi.PassOptions) -> None:
    """ProcessProblem (src/acmmp_definitions.cpp:245-403)."""
    lib = _abi.load_library()
    rc = lib.acmmp_process_problem(dense_folder.encode(), output_folder.encode(), _array(problems), len(problems),
                                   idx, C.byref(options))
    if rc != 0:
        _err("ProcessProblem", rc)


def joint_bilateral_upsampling(dense_folder: str, output_folder: str, problem, acmmp_size: int,
                               device: int = 0) -> None:
    """JointBilateralUpsampling (src/acmmp_definitions.cpp:405-438)."""
    lib = _abi.load_library()
    rc = lib.acmmp_joint_bilateral_upsampling(dense_folder.encode(), output_folder.encode(), C.byref(problem),
                                              acmmp_size, device)
    if rc != 0:
        _err("JointBilateralUpsampling", rc)


def scale_step(problems: list) -> None:
    """cur_image_size for the next scale (src/main_ACMMP.cpp:99-106)."""
    for p in problems:
        if p.num_downscale >= 0:
            p.cur_image_size = int(p.max_image_size / (2.0 ** p.num_downscale))
            p.num_downscale -= 1


def run_sequential(dense_folder: str, output_dir: str | None = None, device: int = 0, max_iterations: int = 0,
                   seed: int = 1234, write_triangulation: bool = True, geom_iterations: int = 2,
                   verbose: bool = False, prior: bool = False, concurrent_views: int = 2) -> str:
    """main_ACMMP's multi-scale loop without fusion; returns the output folder.
    prior=True is the -p flag: seeded first pass, default folder /ACMMP_PRIOR.

    The views of a pass that reads no file written in the same pass (every
    pass but the multi-geometry ones: a first geometric pass reads its
    sources' depths.dmb, which it does not write) run `concurrent_views` at a
    time, each call with its own engine and stream (the C-ABI call releases
    the GIL); the outputs are those of one view at a time, as in acmmp_main."""
    problems = generate_sample_list(dense_folder)
    max_num_downscale = compute_multiscale_settings(dense_folder, problems)
    if prior and not priors_available(dense_folder, len(problems)):
        raise AcmmpError("Initialisation from a prior was requested, but no suitable priors were found.")
    if output_dir is None:
        output_dir = "/ACMMP_PRIOR" if prior else "/ACMMP"
    output_folder = dense_folder + output_dir
    os.makedirs(output_folder, exist_ok=True)
    state = {"pass": 0}

    def for_views(lanes, fn):
        """fn(0..n-1), `lanes` at a time; the first failing view in order
        raises, as the one-at-a-time loop would."""
        lanes = max(1, min(lanes, len(problems)))
        if lanes == 1:
            for i in range(len(problems)):
                fn(i)
            return
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(lanes) as ex:
            for f in [ex.submit(fn, i) for i in range(len(problems))]:
                f.result()

    def run_pass(geom, planar, hier, multi, seeded=False):
        opts = [pass_options(geom, planar, hier, multi, device, max_iterations, seed + p.ref_image_id,
                             state["pass"], write_triangulation, verbose, seeded) for p in problems]
        for_views(1 if (geom and multi) else concurrent_views,
                  lambda i: process_problem(dense_folder, output_folder, problems, i, opts[i]))
        state["pass"] += 1

    first = True
    while max_num_downscale >= 0:
        scale_step(problems)
        if first:
            first = False
            run_pass(False, True, False, False, prior)
        else:
            # each view upsamples its own coarse map into its own folder
            for_views(concurrent_views, lambda i: joint_bilateral_upsampling(
                dense_folder, output_folder, problems[i], problems[i].cur_image_size, device))
            run_pass(False, True, True, False)
        for g in range(geom_iterations):
            run_pass(True, False, False, g > 0)
        max_num_downscale -= 1
    return output_folder


def run_fusion(dense_folder: str, output_folder: str, problems=None, geom_consistency: bool = True,
               consistency_scalar: float = 0.3, num_consistent_thresh: int = 1, image_dir: str = "/images",
               mask_folder: str = " ", write_debug_images: bool = False) -> int:
    """RunFusion (src/acmmp_definitions.cpp:828-1043): writes
    <output_folder>/ACMMP_model.ply; returns the number of fused points."""
    if problems is None:
        problems = generate_sample_list(dense_folder)
    lib = _abi.load_library()
    n = C.c_int(0)
    rc = lib.acmmp_run_fusion(dense_folder.encode(), output_folder.encode(), _array(problems), len(problems),
                              int(geom_consistency), float(consistency_scalar), int(num_consistent_thresh),
                              image_dir.encode(), mask_folder.encode(), int(write_debug_images), C.byref(n))
    if rc != 0:
        raise AcmmpError(f"RunFusion failed (status {rc}): {lib.acmmp_fusion_last_error().decode()}")
    return n.value


def run_prior_aware_fusion(dense_folder: str, output_folder: str, fusion_folder: str, problems=None,
                           geom_consistency: bool = True, consistency_scalar: float = 0.3,
                           num_consistent_thresh: int = 1, single_match_penalty: int = 0) -> int:
    """RunPriorAwareFusion (src/acmmp_definitions.cpp:573-826): writes
    <output_folder>/ACMMP_prior_model.ply; returns the number of points."""
    if problems is None:
        problems = generate_sample_list(dense_folder)
    lib = _abi.load_library()
    n = C.c_int(0)
    rc = lib.acmmp_run_prior_aware_fusion(dense_folder.encode(), output_folder.encode(), fusion_folder.encode(),
                                          _array(problems), len(problems), int(geom_consistency),
                                          float(consistency_scalar), int(num_consistent_thresh),
                                          int(single_match_penalty), C.byref(n))
    if rc != 0:
        raise AcmmpError(f"RunPriorAwareFusion failed (status {rc}): {lib.acmmp_fusion_last_error().decode()}")
    return n.value
