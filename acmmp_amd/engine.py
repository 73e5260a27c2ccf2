"""Python host mirror of the reference's `ACMMP` class (src/ACMMP.h:58-124)
over the C-ABI of libacmmp_amd.so.

Method names follow the reference so a caller of the C++ class finds the same
surface; bulk numpy accessors replace the per-pixel getter loops of
`ProcessProblem` (src/acmmp_definitions.cpp:287-295). Every call goes to the
native HIP engine — there is no CPU fallback: a missing library or GPU raises.
"""
from __future__ import annotations

import ctypes as C
import sys
from typing import Sequence

import numpy as np

from . import _abi


class AcmmpError(RuntimeError):
    pass


def make_camera(K, R, t, width: int, height: int, depth_min: float, depth_max: float) -> _abi.Camera:
    cam = _abi.Camera()
    for i, v in enumerate(np.asarray(K, dtype=np.float32).reshape(9)):
        cam.K[i] = float(v)
    for i, v in enumerate(np.asarray(R, dtype=np.float32).reshape(9)):
        cam.R[i] = float(v)
    for i, v in enumerate(np.asarray(t, dtype=np.float32).reshape(3)):
        cam.t[i] = float(v)
    cam.width = int(width)
    cam.height = int(height)
    cam.depth_min = float(depth_min)
    cam.depth_max = float(depth_max)
    return cam


def _fptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _uptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_uint32))


def _iptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_int32))


def delaunay_triangulation(width: int, height: int, points: np.ndarray) -> np.ndarray:
    """DelaunayTriangulation (src/ACMMP.cpp:896-918): exact Delaunay of integer
    points in [0,width) x [0,height); (m, 6) int32 triangles x1 y1 x2 y2 x3 y3,
    only those with all corners in the image. Host code, no GPU needed."""
    lib = _abi.load_library()
    pts = np.ascontiguousarray(points, dtype=np.int32).reshape(-1, 2)
    cap = 2 * pts.shape[0] + 16
    tris = np.empty((cap, 6), dtype=np.int32)
    n = C.c_int(0)
    rc = lib.acmmp_delaunay_triangulation(int(width), int(height), _iptr(pts), int(pts.shape[0]), _iptr(tris),
                                          cap, C.byref(n))
    if rc != 0:
        raise AcmmpError(f"acmmp_delaunay_triangulation failed (status {rc})")
    return tris[: n.value].copy()


def joint_bilateral_upsample(image: np.ndarray, depth: np.ndarray, device: int = 0):
    """RunJBU + JBU_cu (src/ACMMP.cpp:1008-1087, src/ACMMP.cu:1458-1549) on the
    GPU. Returns (upsampled depth at the image's size, Imagescale); the depth
    is None when Imagescale == 1 (the reference writes nothing then)."""
    lib = _abi.load_library()
    im = np.ascontiguousarray(image, dtype=np.float32)
    d = np.ascontiguousarray(depth, dtype=np.float32)
    out = np.empty_like(im)
    isc = C.c_int(0)
    rc = lib.acmmp_joint_bilateral_upsample(int(device), _fptr(im), im.shape[1], im.shape[0], _fptr(d), d.shape[1],
                                            d.shape[0], _fptr(out), C.byref(isc))
    if rc != 0:
        raise AcmmpError(f"acmmp_joint_bilateral_upsample failed (status {rc})")
    return (None if isc.value <= 1 else out), isc.value


def joint_bilateral_upsample_device(d_image: int, width: int, height: int, d_depth: int, depth_width: int,
                                    depth_height: int, d_out: int, device: int = 0) -> int:
    """joint_bilateral_upsample on device buffers (row-major, unpadded
    float32: image and out width x height, depth depth_width x
    depth_height). Returns Imagescale; d_out is written only when it is > 1."""
    lib = _abi.load_library()
    isc = C.c_int(0)
    rc = lib.acmmp_joint_bilateral_upsample_device(int(device), C.c_void_p(int(d_image)), int(width), int(height),
                                                   C.c_void_p(int(d_depth)), int(depth_width), int(depth_height),
                                                   C.c_void_p(int(d_out)), C.byref(isc))
    if rc != 0:
        raise AcmmpError(f"acmmp_joint_bilateral_upsample_device failed (status {rc})")
    return isc.value


class Texture:
    """~ a CUDA texture object (src/ACMMP.cpp:640-662): the padded footprint
    records of one device-resident image, built once and borrowed by every
    engine/run that uses the image (acmmp_texture_create). Keep the image
    tensor alive while the texture is used."""

    def __init__(self, d_image: int, width: int, height: int, pitch: int | None = None, device: int = 0):
        self._lib = _abi.load_library()
        h = C.c_void_p()
        rc = self._lib.acmmp_texture_create(int(device), C.c_void_p(int(d_image)), int(pitch or width), int(width),
                                            int(height), C.byref(h))
        if rc != 0:
            raise AcmmpError(f"acmmp_texture_create failed (status {rc})")
        self._h = h
        self.width, self.height = int(width), int(height)

    @classmethod
    def of(cls, image, device: int = 0) -> "Texture":
        """From an (H, W) float32 device tensor."""
        return cls(image.data_ptr(), image.shape[1], image.shape[0], image.stride(0), device)

    @property
    def handle(self):
        return self._h

    @property
    def bits(self) -> int:
        return int(self._lib.acmmp_texture_bits(self._h))

    def close(self):
        if getattr(self, "_h", None):
            self._lib.acmmp_texture_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


def device_count() -> int:
    return int(_abi.load_library().acmmp_device_count())


def release_device_cache(device: int = -1) -> None:
    """Gives the library's cached device blocks (and idle streams/events) of
    `device` (-1: every device) back to the HIP runtime
    (acmmp_release_device_cache)."""
    rc = _abi.load_library().acmmp_release_device_cache(int(device))
    if rc != _abi.OK:
        raise AcmmpError(f"acmmp_release_device_cache({device}) failed with status {rc}")


def device_cache_bytes(device: int = -1) -> int:
    """Bytes of device blocks the library's cache holds (acmmp_device_cache_bytes)."""
    return int(_abi.load_library().acmmp_device_cache_bytes(int(device)))


class ACMMP:
    """One PatchMatch engine bound to one GPU (`ACMMP acmmp;` +
    `cudaSetDevice`, src/acmmp_definitions.cpp:253-260)."""

    def __init__(self, device: int = 0, params: _abi.Params | None = None):
        self._lib = _abi.load_library()
        ctx = C.c_void_p()
        rc = self._lib.acmmp_create(int(device), C.byref(ctx))
        if rc != _abi.OK:
            raise AcmmpError(f"acmmp_create(device={device}) failed with status {rc} "
                             "(no HIP device visible?)")
        self._ctx = ctx
        self.device = int(device)
        self._keep = []  # host buffers referenced by the last upload
        if params is not None:
            self.set_params(params)

    # ------------------------------------------------------------ lifetime
    def close(self):
        if getattr(self, "_ctx", None):
            self._lib.acmmp_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc: int, what: str):
        if rc != _abi.OK:
            msg = self._lib.acmmp_last_error(self._ctx)
            raise AcmmpError(f"{what}: status {rc}: {msg.decode() if msg else ''}")

    # -------------------------------------------------------------- params
    @property
    def params(self) -> _abi.Params:
        p = _abi.Params()
        self._check(self._lib.acmmp_get_params(self._ctx, C.byref(p)), "acmmp_get_params")
        return p

    def set_params(self, p: _abi.Params):
        self._check(self._lib.acmmp_set_params(self._ctx, C.byref(p)), "acmmp_set_params")

    def update_params(self, **kw):
        p = self.params
        for k, v in kw.items():
            setattr(p, k, v)
        self.set_params(p)

    def SetGeomConsistencyParams(self, multi_geometry: bool = False):
        """src/ACMMP.cpp:447-454 (also forces max_iterations = 2)."""
        self._check(self._lib.acmmp_set_geom_consistency_params(self._ctx, int(bool(multi_geometry))),
                    "SetGeomConsistencyParams")

    def SetPlanarPriorParams(self):
        self._check(self._lib.acmmp_set_planar_prior_params(self._ctx), "SetPlanarPriorParams")

    def SetHierarchyParams(self):
        self._check(self._lib.acmmp_set_hierarchy_params(self._ctx), "SetHierarchyParams")

    # -------------------------------------------------------------- inputs
    def set_images(self, cams: Sequence[_abi.Camera], images: Sequence[np.ndarray],
                   keep_depth_range: bool = False):
        """In-memory InputInitialization + CudaSpaceInitialization
        (src/ACMMP.cpp:525-681): images[0] is the reference view."""
        n = len(cams)
        if n != len(images):
            raise ValueError("cams/images length mismatch")
        imgs = [np.ascontiguousarray(im, dtype=np.float32) for im in images]
        for cam, im in zip(cams, imgs):
            if im.shape != (cam.height, cam.width):
                raise ValueError(f"image shape {im.shape} != camera {(cam.height, cam.width)}")
        cam_arr = (_abi.Camera * n)(*cams)
        ptrs = (C.POINTER(C.c_float) * n)(*[_fptr(im) for im in imgs])
        self._check(self._lib.acmmp_set_images(self._ctx, n, cam_arr, ptrs, int(keep_depth_range)),
                    "acmmp_set_images")

    def texel_bits(self) -> int:
        """16 when the gathers read f16 difference quads, 8 for u8 quads, 32
        for fp32 row pairs (acmmp_get_texel_bits)."""
        return int(self._lib.acmmp_get_texel_bits(self._ctx))

    def set_depth_maps(self, depths: Sequence[np.ndarray]):
        ds = [np.ascontiguousarray(d, dtype=np.float32) for d in depths]
        ptrs = (C.POINTER(C.c_float) * len(ds))(*[_fptr(d) for d in ds])
        self._check(self._lib.acmmp_set_depth_maps(self._ctx, ptrs), "acmmp_set_depth_maps")

    def wait_stream(self, stream_handle: int | None):
        """acmmp_wait_stream: the engine stream waits (on the device, no host
        wait) for everything enqueued so far on `stream_handle` (a
        hipStream_t; 0/None = the legacy default stream)."""
        self._check(self._lib.acmmp_wait_stream(self._ctx, C.c_void_p(int(stream_handle or 0) or None)),
                    "acmmp_wait_stream")

    def _after_producer(self):
        """Orders the engine stream (non-blocking) after torch's current stream
        on this device before a *_device setter borrows or copies a caller
        buffer: buffers the caller built with torch ops (a gathered band, a
        collective's output, a torch.cat) may still be being written there.
        A no-op when torch is not loaded or has not touched the GPU."""
        torch = sys.modules.get("torch")
        if torch is None or not torch.cuda.is_initialized():
            return
        self.wait_stream(torch.cuda.current_stream(self.device).cuda_stream)

    def set_depth_maps_device(self, device_ptrs: Sequence[int], pitches: Sequence[int] | None = None):
        """Borrow device-resident depth maps (e.g. slices of an RCCL
        all-gather); the caller keeps them alive until the run completes."""
        self._after_producer()
        arr = (C.c_void_p * len(device_ptrs))(*[C.c_void_p(int(p)) for p in device_ptrs])
        pit = None if pitches is None else (C.c_int32 * len(pitches))(*pitches)
        self._check(self._lib.acmmp_set_depth_maps_device(self._ctx, arr, pit), "acmmp_set_depth_maps_device")

    def set_images_device(self, cams: Sequence[_abi.Camera], device_ptrs: Sequence[int],
                          pitches: Sequence[int] | None = None, keep_depth_range: bool = False):
        """Zero-copy set_images: borrow device-resident images."""
        self._after_producer()
        n = len(cams)
        cam_arr = (_abi.Camera * n)(*cams)
        arr = (C.c_void_p * n)(*[C.c_void_p(int(p)) for p in device_ptrs])
        pit = None if pitches is None else (C.c_int32 * n)(*pitches)
        self._check(self._lib.acmmp_set_images_device(self._ctx, n, cam_arr, arr, pit, int(keep_depth_range)),
                    "acmmp_set_images_device")

    def set_images_textures(self, cams: Sequence[_abi.Camera], textures: Sequence["Texture"],
                            keep_depth_range: bool = False):
        """set_images_device from prebuilt textures (no per-run padding)."""
        self._after_producer()
        n = len(cams)
        cam_arr = (_abi.Camera * n)(*cams)
        arr = (C.c_void_p * n)(*[t.handle for t in textures])
        self._check(self._lib.acmmp_set_images_textures(self._ctx, n, cam_arr, arr, int(keep_depth_range)),
                    "acmmp_set_images_textures")

    def set_plane_hypotheses_device(self, d_planes: int, d_costs: int):
        """Previous state from device buffers, copied on the engine stream
        after the producer's writes (acmmp_wait_stream)."""
        self._after_producer()
        self._check(self._lib.acmmp_set_plane_hypotheses_device(self._ctx, C.c_void_p(int(d_planes)),
                                                                C.c_void_p(int(d_costs))),
                    "acmmp_set_plane_hypotheses_device")

    def export_results(self, d_planes: int = 0, d_costs: int = 0, d_depth: int = 0):
        """Device-to-device copy of the last results (enqueued on the engine
        stream; call synchronize() before another stream reads them). The
        copy is ordered after torch's current stream: the destination may be
        memory torch's allocator just recycled from a tensor still in use
        there."""
        self._after_producer()
        self._check(self._lib.acmmp_export_results(self._ctx, C.c_void_p(int(d_planes) or None),
                                                   C.c_void_p(int(d_costs) or None),
                                                   C.c_void_p(int(d_depth) or None)),
                    "acmmp_export_results")

    def set_plane_hypotheses(self, planes: np.ndarray, costs: np.ndarray):
        """Previous-pass (world normal, depth) + costs (src/ACMMP.cpp:718-742)."""
        pl = np.ascontiguousarray(planes, dtype=np.float32)
        co = np.ascontiguousarray(costs, dtype=np.float32)
        self._check(self._lib.acmmp_set_plane_hypotheses(self._ctx, _fptr(pl), _fptr(co)),
                    "acmmp_set_plane_hypotheses")

    def set_hierarchy_inputs(self, scaled_planes: np.ndarray, upsampled_depth: np.ndarray):
        sp = np.ascontiguousarray(scaled_planes, dtype=np.float32)
        ud = np.ascontiguousarray(upsampled_depth, dtype=np.float32)
        sh, sw = sp.shape[:2]
        self._check(self._lib.acmmp_set_hierarchy_inputs(self._ctx, _fptr(sp), sw, sh, _fptr(ud)),
                    "acmmp_set_hierarchy_inputs")

    def set_hierarchy_inputs_device(self, d_scaled_planes: int, scaled_w: int, scaled_h: int,
                                    d_upsampled_depth: int):
        """Hierarchy inputs from device buffers (scaled planes scaled_h x
        scaled_w float4, upsampled depth at the reference size); they must
        stay valid until the next run has completed."""
        self._after_producer()
        self._check(self._lib.acmmp_set_hierarchy_inputs_device(self._ctx, C.c_void_p(int(d_scaled_planes)),
                                                                int(scaled_w), int(scaled_h),
                                                                C.c_void_p(int(d_upsampled_depth))),
                    "acmmp_set_hierarchy_inputs_device")

    def SetPlanarPrior(self, prior: np.ndarray):
        """Seeded plane priors (src/ACMMP.cpp:476-523); sets params.seeded."""
        pr = np.ascontiguousarray(prior, dtype=np.float32)
        self._check(self._lib.acmmp_set_seed_prior(self._ctx, _fptr(pr)), "SetPlanarPrior")

    def CudaPlanarPriorInitialization(self, plane_params: np.ndarray, mask: np.ndarray):
        """src/ACMMP.cpp:811-831: triangle planes + per-pixel label mask."""
        pp = np.ascontiguousarray(plane_params, dtype=np.float32).reshape(-1, 4)
        mk = np.ascontiguousarray(mask, dtype=np.uint32)
        self._check(self._lib.acmmp_set_planar_prior(self._ctx, _fptr(pp), int(pp.shape[0]), _uptr(mk)),
                    "CudaPlanarPriorInitialization")

    # ------------------------------------------------- planar prior (a17)
    def GetSupportPoints(self) -> np.ndarray:
        """src/ACMMP.cpp:868-894 on the resident results: (n, 2) int32 (x, y)."""
        w, h = self.size
        cap = (w // 5 + 1) * (h // 5 + 1)
        xy = np.empty((cap, 2), dtype=np.int32)
        n = C.c_int(0)
        self._check(self._lib.acmmp_get_support_points(self._ctx, _iptr(xy), cap, C.byref(n)), "GetSupportPoints")
        return xy[: n.value].copy()

    def DelaunayTriangulation(self, points: np.ndarray) -> np.ndarray:
        """src/ACMMP.cpp:896-918 over this view's image rectangle."""
        w, h = self.size
        return delaunay_triangulation(w, h, points)

    def build_planar_prior(self, triangles: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
        """Raster + GetPriorPlaneParams + range check + CudaPlanarPriorInitialization
        (src/acmmp_definitions.cpp:332-376) on the device; returns the fitted
        planes (one float4 per in-image triangle) and the final label mask."""
        w, h = self.size
        tr = np.ascontiguousarray(triangles, dtype=np.int32).reshape(-1, 6)
        planes = np.empty((max(tr.shape[0], 1), 4), dtype=np.float32)
        mask = np.empty((h, w), dtype=np.uint32)
        self._check(self._lib.acmmp_build_planar_prior(self._ctx, _iptr(tr), int(tr.shape[0]), _fptr(planes),
                                                       _uptr(mask)), "acmmp_build_planar_prior")
        inside = ((tr[:, 0::2] >= 0) & (tr[:, 0::2] < w) & (tr[:, 1::2] >= 0) & (tr[:, 1::2] < h)).all(axis=1)
        return planes[: int(inside.sum())], mask

    def prepare_planar_prior(self) -> tuple[int, int]:
        """Support points -> Delaunay -> prior build -> SetPlanarPriorParams.
        Returns (support points, triangles)."""
        npts, ntri = C.c_int(0), C.c_int(0)
        self._check(self._lib.acmmp_prepare_planar_prior(self._ctx, C.byref(npts), C.byref(ntri)),
                    "acmmp_prepare_planar_prior")
        return npts.value, ntri.value

    # ----------------------------------------------------------------- run
    def RunPatchMatch(self):
        """src/ACMMP.cu:1378-1456."""
        self._check(self._lib.acmmp_run_patchmatch(self._ctx), "RunPatchMatch")

    def run_async(self):
        self._check(self._lib.acmmp_run_patchmatch_async(self._ctx), "acmmp_run_patchmatch_async")

    def synchronize(self):
        self._check(self._lib.acmmp_synchronize(self._ctx), "acmmp_synchronize")

    def run_band(self, row_lo: int, row_hi: int, exchange):
        """acmmp_run_patchmatch_band: this participant's rows [row_lo, row_hi)
        of a row-band split RunPatchMatch; `exchange(halo: _abi.BandHalo)`
        trades the halo rows after every half-sweep (acmmp_amd.band). A
        Python exception in it fails the run and is re-raised here."""
        err = []

        def cb(_user, halo):
            try:
                exchange(halo.contents)
                return 0
            except BaseException as e:  # noqa: BLE001 — re-raised below
                err.append(e)
                return 1

        fn = _abi.BandExchangeFn(cb)
        rc = self._lib.acmmp_run_patchmatch_band(self._ctx, int(row_lo), int(row_hi), fn, None)
        if err:
            raise err[0]
        self._check(rc, "acmmp_run_patchmatch_band")

    def set_timing(self, enable: bool = True):
        self._check(self._lib.acmmp_set_timing(self._ctx, int(enable)), "acmmp_set_timing")

    def timing(self) -> dict:
        t = _abi.Timing()
        self._check(self._lib.acmmp_get_timing(self._ctx, C.byref(t)), "acmmp_get_timing")
        return {k: getattr(t, k) for k, _ in _abi.Timing._fields_}

    # ------------------------------------------------------------- outputs
    @property
    def size(self) -> tuple[int, int]:
        w, h = C.c_int(), C.c_int()
        self._check(self._lib.acmmp_get_reference_size(self._ctx, C.byref(w), C.byref(h)),
                    "acmmp_get_reference_size")
        return w.value, h.value

    def GetReferenceImageWidth(self) -> int:
        return self.size[0]

    def GetReferenceImageHeight(self) -> int:
        return self.size[1]

    def GetCamera(self, index: int) -> _abi.Camera:
        cam = _abi.Camera()
        self._check(self._lib.acmmp_get_camera(self._ctx, int(index), C.byref(cam)), "GetCamera")
        return cam

    def GetMinDepth(self) -> float:
        return self.params.depth_min

    def GetMaxDepth(self) -> float:
        return self.params.depth_max

    def plane_hypotheses(self) -> np.ndarray:
        w, h = self.size
        out = np.empty((h, w, 4), dtype=np.float32)
        self._check(self._lib.acmmp_get_plane_hypotheses(self._ctx, _fptr(out), w * h),
                    "acmmp_get_plane_hypotheses")
        return out

    def costs(self) -> np.ndarray:
        w, h = self.size
        out = np.empty((h, w), dtype=np.float32)
        self._check(self._lib.acmmp_get_costs(self._ctx, _fptr(out), w * h), "acmmp_get_costs")
        return out

    def selected_views(self) -> np.ndarray:
        w, h = self.size
        out = np.empty((h, w), dtype=np.uint32)
        self._check(self._lib.acmmp_get_selected_views(self._ctx, _uptr(out), w * h),
                    "acmmp_get_selected_views")
        return out

    def device_results(self) -> tuple[int, int]:
        p, c = C.c_void_p(), C.c_void_p()
        self._check(self._lib.acmmp_get_device_results(self._ctx, C.byref(p), C.byref(c)),
                    "acmmp_get_device_results")
        return int(p.value or 0), int(c.value or 0)

    def GetPlaneHypothesis(self, index: int) -> tuple[float, float, float, float]:
        """Per-pixel getter of the reference (src/ACMMP.cpp:848-851); prefer
        plane_hypotheses() for bulk reads."""
        pl = self.plane_hypotheses().reshape(-1, 4)[index]
        return tuple(float(v) for v in pl)

    def GetCost(self, index: int) -> float:
        return float(self.costs().reshape(-1)[index])

    # ------------------------------------------------------ kernel-level T1
    def eval_costs(self, planes: np.ndarray):
        w, h = self.size
        n = self.params.num_images
        pl = np.ascontiguousarray(planes, dtype=np.float32)
        out = np.empty((h, w, n - 1), dtype=np.float32)
        init = np.empty((h, w), dtype=np.float32)
        views = np.empty((h, w), dtype=np.uint32)
        self._check(self._lib.acmmp_eval_costs(self._ctx, _fptr(pl), _fptr(out), _fptr(init), _uptr(views)),
                    "acmmp_eval_costs")
        return out, init, views

    def eval_geom_costs(self, planes: np.ndarray) -> np.ndarray:
        w, h = self.size
        n = self.params.num_images
        pl = np.ascontiguousarray(planes, dtype=np.float32)
        out = np.empty((h, w, n - 1), dtype=np.float32)
        self._check(self._lib.acmmp_eval_geom_costs(self._ctx, _fptr(pl), _fptr(out)), "acmmp_eval_geom_costs")
        return out
