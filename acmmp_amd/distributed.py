"""View-parallel pass driver: one process per GPU.

Within a pass every view's RunPatchMatch is independent, so views are sharded
across ranks (LPT on W*H*(N-1)) and each rank runs its views on its own GPU
with no communication. Between passes the only data another view needs is
source depth maps (src/ACMMP.cpp:608-635; used as depth_images[j+1] in
src/ACMMP.cu:753, 1064, 1085), so each pass ends with ONE all-gather of the
f32 depth maps (`all_gather_into_tensor` = RCCL over xGMI with the nccl
backend; padded to the largest map since RCCL has no all-gatherv). Normals,
costs and the planar/hierarchy inputs stay on the rank that owns the view.

Schedule: Jacobi — every view of a pass reads the previous pass's maps. The
reference's second geometric pass is Gauss-Seidel (src/main_ACMMP.cpp:
159-172); the single-process drivers (`pipeline.run_sequential`, the
acmmp_main CLI) keep that order, and tests/oracle_pipeline.py restates both.

The pass / exchange logic is independent of the engine: `compute` and `jbu`
are injectable, which is how the world-size-2 gloo tests exercise it on CPU.
Outputs are the reference's .dmb files, written by the owning rank.
"""
from __future__ import annotations

import os
import time
from collections import defaultdict
from contextlib import contextmanager
from dataclasses import dataclass, field
from typing import Callable, Optional

import numpy as np
import torch
import torch.distributed as dist

from . import _abi
from . import io as aio
from . import pipeline
from .engine import ACMMP, AcmmpError, joint_bilateral_upsample_device


def lpt_assign(costs: list, world: int) -> list:
    """Longest-processing-time-first: views sorted by cost (desc, then index)
    go to the least-loaded rank (ties: lowest rank). Per-rank lists ascending."""
    load = [0.0] * world
    out = [[] for _ in range(world)]
    for v in sorted(range(len(costs)), key=lambda i: (-costs[i], i)):
        r = min(range(world), key=lambda k: (load[k], k))
        out[r].append(v)
        load[r] += costs[v]
    return [sorted(o) for o in out]


def plan_views(costs: list, world: int, split_tail: bool) -> tuple:
    """The pass's view placement: (assignment, split). Without split_tail,
    assignment = lpt_assign and split = []. With it, the V mod world
    cheapest views — the tail that leaves some ranks one view longer than
    the others — are split into row bands over ALL ranks (acmmp_amd.band,
    bit-exact to the unsplit run) and the rest are LPT-assigned; each split
    view still has one owner rank (least loaded first), which decodes its
    image into the all-gathers and writes its .dmb files."""
    n = len(costs)
    r = n % world if split_tail and world > 1 else 0
    order = sorted(range(n), key=lambda i: (-costs[i], i))
    split = sorted(order[n - r:]) if r else []
    whole = [v for v in range(n) if v not in set(split)]
    sub = lpt_assign([costs[v] for v in whole], world)
    assignment = [[whole[k] for k in a] for a in sub]
    load = [sum(costs[v] for v in a) for a in assignment]
    for v in split:
        k = min(range(world), key=lambda q: (load[q], q))
        assignment[k].append(v)
        load[k] += costs[v]
    return [sorted(a) for a in assignment], split


class DepthExchange:
    """All-gather of per-view depth maps of different sizes over a padded
    [world * slots, Hmax, Wmax] buffer with all_gather_into_tensor (RCCL has
    no all-gatherv). The gathered maps are returned as views into one buffer
    on `out_device` (row pitch Wmax), so a geometric pass borrows them without
    a copy (acmmp_set_depth_maps_device takes the pitch)."""

    def __init__(self, assignment: list, shapes: dict, device: torch.device, group=None,
                 out_device: Optional[torch.device] = None):
        self.assignment = assignment
        self.shapes = shapes
        self.device = device
        self.out_device = out_device or device
        self.group = group
        self.slots = max(1, max(len(a) for a in assignment))
        self.hmax = max(h for h, _ in shapes.values())
        self.wmax = max(w for _, w in shapes.values())

    def gather(self, rank: int, local: dict) -> dict:
        world = len(self.assignment)
        send = torch.zeros((self.slots, self.hmax, self.wmax), dtype=torch.float32, device=self.device)
        for k, v in enumerate(self.assignment[rank]):
            h, w = self.shapes[v]
            send[k, :h, :w] = local[v].to(self.device)
        if dist.is_initialized():  # RCCL (nccl backend) or gloo; world size 1 included
            recv = torch.empty((world * self.slots, self.hmax, self.wmax), dtype=torch.float32, device=self.device)
            dist.all_gather_into_tensor(recv, send, group=self.group)
        else:
            recv = send
        recv = recv.to(self.out_device)
        if recv.is_cuda:
            # the engines' HIP streams do not wait on torch's / RCCL's: the
            # gathered maps are complete before any view borrows them
            torch.cuda.current_stream(recv.device).synchronize()
        out = {}
        for r in range(world):  # concatenated along dim 0: rank r's slots at [r * slots, (r + 1) * slots)
            for k, v in enumerate(self.assignment[r]):
                h, w = self.shapes[v]
                out[v] = recv[r * self.slots + k, :h, :w]
        return out


@dataclass
class ViewTask:
    """Everything one ProcessProblem call needs, resident on the tensor
    device."""
    index: int                 # problem index
    ref_id: int
    ids: list                  # image ids, ref first
    cams: list                 # acmmp_camera per image (rescaled)
    images: list               # float32 tensors (H, W) per image
    geom: bool
    planar: bool
    hierarchy: bool
    multi: bool
    seed_lo: int
    seed_hi: int
    max_iterations: int
    depths: Optional[list] = None          # source depth maps (tensor views, any row pitch), geom passes
    state: Optional[tuple] = None          # (planes (H,W,4), costs (H,W)) tensors, geom passes
    hier_inputs: Optional[tuple] = None    # (scaled planes (sh,sw,4), upsampled depth (H,W)) tensors
    textures: Optional[list] = None        # engine.Texture per image (prebuilt footprint records)


@dataclass
class ViewResult:
    planes: torch.Tensor   # (H, W, 4): world normal xyz + depth
    costs: torch.Tensor    # (H, W)
    extra: dict = field(default_factory=dict)


def _view_params(t: ViewTask) -> _abi.Params:
    """ProcessProblem's parameter set-up (src/acmmp_definitions.cpp:253-268):
    defaults, SetGeomConsistencyParams (geom: 2 iterations, src/ACMMP.cpp:
    447-454), SetHierarchyParams, the per-view RNG key, -iterations."""
    p = _abi.default_params()
    if t.geom:
        p.geom_consistency = 1
        p.max_iterations = 2
        if t.multi:
            p.multi_geometry = 1
    if t.hierarchy:
        p.hierarchy = 1
    p.seed_lo = t.seed_lo & 0xFFFFFFFF
    p.seed_hi = t.seed_hi & 0xFFFFFFFF
    if t.max_iterations > 0:
        p.max_iterations = t.max_iterations
    return p


def engine_compute(t: ViewTask, eng: ACMMP) -> ViewResult:
    """ProcessProblem's per-view work (src/acmmp_definitions.cpp:260-379) on
    a pooled engine: images, previous state and source depth maps borrowed
    from HBM, results exported device-to-device into fresh tensors (the
    previous pass's tensors may still be read by the .dmb writers)."""
    ref = t.images[0]
    H, W = ref.shape
    planes = torch.empty((H, W, 4), dtype=torch.float32, device=ref.device)
    costs = torch.empty((H, W), dtype=torch.float32, device=ref.device)
    engine_setup(t, eng)
    gpu_ms = 0.0
    eng.run_async()
    if t.planar:
        eng.synchronize()
        gpu_ms += _run_ms(eng)
        eng.prepare_planar_prior()
        eng.run_async()
    eng.export_results(planes.data_ptr(), costs.data_ptr(), 0)
    eng.synchronize()
    gpu_ms += _run_ms(eng)
    return ViewResult(planes, costs, {"gpu_ms": gpu_ms})


def engine_setup(t: ViewTask, eng: ACMMP):
    """ProcessProblem's inputs for one view on an engine (parameters, images,
    and per pass kind the previous state, source depth maps and hierarchy
    inputs), borrowed from HBM."""
    eng.set_params(_view_params(t))
    if t.textures is not None:
        eng.set_images_textures(t.cams, t.textures)
    else:
        eng.set_images_device(t.cams, [im.data_ptr() for im in t.images], [im.stride(0) for im in t.images])
    if t.geom:
        eng.set_depth_maps_device([d.data_ptr() for d in t.depths], [d.stride(0) for d in t.depths])
        eng.set_plane_hypotheses_device(t.state[0].data_ptr(), t.state[1].data_ptr())
    if t.hierarchy:
        scaled, up = t.hier_inputs
        eng.set_hierarchy_inputs_device(scaled.data_ptr(), scaled.shape[1], scaled.shape[0], up.data_ptr())


def _run_ms(eng: ACMMP) -> float:
    """Device time (HIP events) of the engine's last RunPatchMatch, 0 when
    its timing is off."""
    return eng.timing()["total_ms"] if getattr(eng, "timing_on", False) else 0.0


def gpu_jbu(device: int):
    """JointBilateralUpsampling on resident tensors: (upsampled depth tensor at
    the image's size or None, Imagescale)."""
    def run(image: torch.Tensor, depth: torch.Tensor):
        image = image.contiguous()
        depth = depth.contiguous()
        out = torch.empty_like(image)
        torch.cuda.current_stream(image.device).synchronize()  # the JBU stream does not wait on torch's
        isc = joint_bilateral_upsample_device(image.data_ptr(), image.shape[1], image.shape[0], depth.data_ptr(),
                                              depth.shape[1], depth.shape[0], out.data_ptr(), device)
        return (out if isc > 1 else None), isc
    return run


class ViewParallelPipeline:
    """main_ACMMP's multi-scale pass loop (src/main_ACMMP.cpp:96-176), views
    sharded over the ranks of `group` (default: the world).

    Device-resident (multi-GPU keeps maps resident and writes
    .dmb at pass end): images stay in HBM per scale, every view's planes /
    costs stay on the device between passes, the gathered depth maps are
    borrowed in place, one pool of engines (one HIP stream each) is reused
    for every view and pass, and the .dmb files are written by a writer pool
    from device-to-host copies while the next pass computes."""

    def __init__(self, dense_folder: str, output_dir: str = "/ACMMP", device: int = 0, seed: int = 1234,
                 max_iterations: int = 0, geom_iterations: int = 2, group=None,
                 compute: Optional[Callable] = None, jbu: Optional[Callable] = None, write_outputs: bool = True,
                 comm_device: Optional[torch.device] = None, tensor_device: Optional[torch.device] = None,
                 concurrent_views: int = 2, timing: bool = False, split_tail: bool = True):
        self.dense = dense_folder
        self.output_folder = dense_folder + output_dir
        self.device = device
        self.seed = seed
        self.max_iterations = max_iterations
        self.geom_iterations = geom_iterations
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.compute = compute or engine_compute
        self.jbu = jbu or gpu_jbu(device)
        self.write_outputs = write_outputs
        # views of a pass computed at once (each on its own pooled engine /
        # HIP stream, from a thread: ctypes drops the GIL in every library
        # call), so one view's launches fill the tail of another's
        self.concurrent_views = max(int(concurrent_views), 1)
        self.pool = None
        # per-phase wall seconds (and summed RunPatchMatch device ms with
        # timing=True: HIP events around each run, engines' timing on)
        self.timing = timing
        self.phase_s = defaultdict(float)
        self.gpu_ms = 0.0
        self._writer = None  # .dmb writer pool (created on the first write)
        self._pending = []
        if tensor_device is None:
            tensor_device = torch.device("cuda", device) if torch.cuda.is_available() else torch.device("cpu")
        self.tdev = tensor_device
        if comm_device is None:
            # RCCL exchanges device tensors; gloo stages them through the host;
            # without a process group there is no exchange and the maps stay put
            backend = dist.get_backend(group) if dist.is_initialized() else None
            comm_device = torch.device("cpu") if backend == "gloo" else self.tdev
        self.cdev = comm_device
        self.problems = pipeline.generate_sample_list(dense_folder)
        self.index_of = {p.ref_image_id: i for i, p in enumerate(self.problems)}
        self.max_num_downscale = pipeline.compute_multiscale_settings(dense_folder, self.problems)
        costs = []
        for p in self.problems:
            w, h = aio.image_size(self._image_path(p.ref_image_id))
            costs.append(float(w * h * max(p.num_src_images, 1)))
        # the tail views are split in row bands over all ranks (engine runs
        # only: the injected CPU stand-ins compute whole views)
        self.split_tail = bool(split_tail) and self.world > 1 and self.compute is engine_compute
        self.assignment, self.split = plan_views(costs, self.world, self.split_tail)
        self._split_checked = False
        self.owned = self.assignment[self.rank]                  # decoded, gathered and written here
        self.mine = [v for v in self.owned if v not in self.split]  # computed whole here
        self.state = {}     # own views: problem index -> ViewResult (latest pass)
        self.depths = {}    # every view: problem index -> depth tensor view (previous pass, gathered)
        self.pass_index = 0
        self.pass_log = []  # per pass: kind and wall seconds of its phases (tools/scale_sim.py)

    # ------------------------------------------------------------- inputs
    def _image_path(self, image_id: int) -> str:
        base = os.path.join(self.dense, "images", "%08d" % image_id)
        for ext in (".jpg", ".pgm", ".pfm"):
            if os.path.exists(base + ext):
                return base + ext
        return base + ".jpg"

    def _load_views(self):
        """Images + cameras of every image my views need, at their problem's
        cur_image_size (InputInitialization, src/ACMMP.cpp:536-598), decoded
        once per node: each rank decodes the reference images of ITS views
        and one padded all-gather (RCCL over xGMI, like the depth maps)
        hands every rank all of them; the cameras come from the headers."""
        import ctypes as C
        lib = _abi.load_library()
        if not self._split_checked:
            self._check_split()
        need = set()
        for v in self.mine + self.split:
            p = self.problems[v]
            need.add(p.ref_image_id)
            need.update(p.sources)
        for i in sorted(need):
            if i not in self.index_of:
                raise AcmmpError(f"source id {i} is not a problem index (pair.txt ids must be 0..n-1)")

        def load(item):  # on a pool thread: the library call drops the GIL; its error slot is per thread
            i, pixels = item
            size = self.problems[self.index_of[i]].cur_image_size
            cam = _abi.Camera()
            rc = lib.acmmp_load_view(self.dense.encode(), i, size, None, 0, C.byref(cam))
            if rc not in (0, _abi.ERR_ARG):
                raise AcmmpError(f"acmmp_load_view({i}) failed: {lib.acmmp_pipeline_last_error().decode()}")
            if not pixels:
                return None, cam
            img = np.empty((cam.height, cam.width), dtype=np.float32)
            rc = lib.acmmp_load_view(self.dense.encode(), i, size, img.ctypes.data_as(C.POINTER(C.c_float)),
                                     img.size, C.byref(cam))
            if rc != 0:
                raise AcmmpError(f"acmmp_load_view({i}) failed: {lib.acmmp_pipeline_last_error().decode()}")
            return img, cam

        from concurrent.futures import ThreadPoolExecutor
        order = sorted(need)
        own = [self.problems[v].ref_image_id for v in self.owned]
        work = [(i, False) for i in order] + [(i, True) for i in own]
        with ThreadPoolExecutor(max_workers=max(1, min(lib.acmmp_host_threads(), len(work)))) as ex:
            loaded = list(ex.map(load, work))  # re-raises the first failure in id order
        self.cams = {i: cam for i, (_, cam) in zip(order, loaded[:len(order)])}
        mine_imgs = {v: torch.from_numpy(img) for v, (img, _) in zip(self.owned, loaded[len(order):])}
        shapes = self._shapes()
        for v, img in mine_imgs.items():
            if tuple(img.shape) != shapes[v]:
                raise AcmmpError(f"view {self.problems[v].ref_image_id}: image size disagrees with its header")
        gathered = DepthExchange(self.assignment, shapes, self.cdev, self.group,
                                 out_device=self.tdev).gather(self.rank, mine_imgs)
        # pitched views into the gathered buffer (row pitch Wmax)
        self.images = {i: gathered[self.index_of[i]] for i in order}
        self._sync()
        # one texture (padded footprint records) per image and scale, shared by
        # every view and pass of the scale (engine runs only)
        self.textures = {}
        if self.compute is engine_compute and self.tdev.type == "cuda":
            from .engine import Texture
            self.textures = {i: Texture.of(im, self.device) for i, im in self.images.items()}

    def _check_split(self):
        """A view is split only if every band holds the 23-row halo at the
        coarsest scale (this first load's shapes; later scales are larger);
        otherwise its owner computes it whole."""
        self._split_checked = True
        shapes = self._shapes()
        keep = [v for v in self.split if shapes[v][0] >= self.world * _abi.BAND_HALO]
        self.split = keep
        self.mine = [v for v in self.owned if v not in keep]

    @contextmanager
    def _timed(self, name: str):
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self.phase_s[name] += time.perf_counter() - t0

    def _sync(self):
        """Torch's queued work on the tensor device is complete (the engines'
        streams do not wait on torch's stream)."""
        if self.tdev.type == "cuda":
            torch.cuda.current_stream(self.tdev).synchronize()

    def _shapes(self):
        shapes = {}
        for i, p in enumerate(self.problems):
            w, h = aio.image_size(self._image_path(p.ref_image_id))
            m = p.cur_image_size
            if w > m or h > m:
                f = min(np.float32(m) / np.float32(w), np.float32(m) / np.float32(h))
                w, h = int(np.round(np.float32(w) * f)), int(np.round(np.float32(h) * f))
            shapes[i] = (h, w)
        return shapes

    # --------------------------------------------------------------- pass
    def _map(self, tasks):
        if self.compute is not engine_compute:  # injected stand-in (CPU tests): no engines
            return [self.compute(t, None) for t in tasks]
        if self.pool is None:
            from .resident import EnginePool
            self.pool = EnginePool(self.device, self.concurrent_views, timing=self.timing)
            for e in self.pool.engines:
                e.timing_on = self.timing
        return self.pool.map(lambda eng, t: self.compute(t, eng), tasks)

    def _task(self, v: int, geom: bool, planar: bool, hierarchy: bool, multi: bool) -> ViewTask:
        p = self.problems[v]
        ids = [p.ref_image_id] + p.sources
        t = ViewTask(index=v, ref_id=p.ref_image_id, ids=ids, cams=[self.cams[i] for i in ids],
                     images=[self.images[i] for i in ids],
                     textures=[self.textures[i] for i in ids] if self.textures else None,
                     geom=geom, planar=planar, hierarchy=hierarchy,
                     multi=multi, seed_lo=self.seed + p.ref_image_id, seed_hi=self.pass_index,
                     max_iterations=self.max_iterations)
        if geom:
            t.depths = [self.depths[self.index_of[i]] for i in ids]
            prev = self.state[v]
            t.state = (prev.planes, prev.costs)
        if hierarchy:
            t_h = time.perf_counter()
            prev = self.state[v]
            H, W = t.images[0].shape
            up = prev.extra["jbu_depth"]
            sh, sw = prev.costs.shape
            upsample = sw != H or sh != W  # src/ACMMP.cpp:766, rows/cols swap included
            w = prev.costs if upsample else up.reshape(-1)[: sh * sw].reshape(sh, sw)
            scaled = torch.cat([prev.planes[..., :3], w[..., None]], -1).contiguous()
            t.hier_inputs = (scaled, up.contiguous())
            self.phase_s["hier_inputs"] += time.perf_counter() - t_h
        return t

    def _run_split(self, t: ViewTask) -> ViewResult:
        """One view's pass split in row bands over every rank of the group
        (acmmp_amd.band): the halos travel after every half-sweep (RCCL P2P,
        or gloo), the bands are all-gathered, so every rank holds the view's
        full state afterwards — bit-identical to the unsplit run."""
        from .band import bands, run_split
        if self.pool is None:
            self._map([])
        eng = self.pool.engines[0]
        engine_setup(t, eng)
        members = [dist.get_global_rank(self.group, k) if self.group is not None else k for k in range(self.world)]
        H = t.images[0].shape[0]
        planes, costs = run_split(eng, bands(H, self.world), members, self.rank, self.tdev, self.cdev, self.group,
                                  planar_prior=t.planar)
        return ViewResult(planes, costs, {})

    def run_pass(self, geom: bool, planar: bool, hierarchy: bool, multi: bool, exchange: DepthExchange):
        tasks = [self._task(v, geom, planar, hierarchy, multi) for v in self.mine]
        t0 = time.perf_counter()
        with self._timed("compute"):
            self._sync()
            results = self._map(tasks)
        t1 = time.perf_counter()
        local = {}
        for t, res in zip(tasks, results):  # in view order, as the sequential loop
            v = t.index
            self.state[v] = res
            self.gpu_ms += res.extra.get("gpu_ms", 0.0)
            local[v] = res.planes[..., 3]
            if self.write_outputs:
                self._write(t.ref_id, res, geom)
        # the tail views, every rank on a band of each
        for v in self.split:
            with self._timed("split_compute"):
                t = self._task(v, geom, planar, hierarchy, multi)
                self._sync()
                res = self._run_split(t)
            self.state[v] = res
            if v in self.owned:
                local[v] = res.planes[..., 3]
                if self.write_outputs:
                    self._write(t.ref_id, res, geom)
        t2 = time.perf_counter()
        with self._timed("exchange"):
            self.depths = exchange.gather(self.rank, local)
        self.pass_log.append({"pass": self.pass_index, "geom": geom, "planar": planar, "hierarchy": hierarchy,
                              "multi": multi, "views": len(self.mine), "split_views": len(self.split),
                              "shape": list(tasks[0].images[0].shape) if tasks else None,
                              "compute_s": t1 - t0, "split_s": t2 - t1, "exchange_s": time.perf_counter() - t2})
        self.pass_index += 1

    def _write(self, ref_id: int, res: ViewResult, geom: bool):
        """Queues the view's three .dmb files on the writer pool: they are
        outputs only (nothing in this driver reads them back), so the device-
        to-host copies and the writes run while the next pass computes. Each
        pass's results are fresh tensors, so no later pass overwrites what a
        writer still reads; the files of one view are written in pass order
        (a view's writes go to one writer thread)."""
        folder = aio.result_folder(self.output_folder, ref_id)
        os.makedirs(folder, exist_ok=True)
        planes, costs = res.planes, res.costs

        def write():
            pl = planes.cpu().numpy()
            aio.write_dmb(os.path.join(folder, "depths_geom.dmb" if geom else "depths.dmb"), pl[..., 3])
            aio.write_dmb(os.path.join(folder, "normals.dmb"), pl[..., :3])
            aio.write_dmb(os.path.join(folder, "costs.dmb"), costs.cpu().numpy())

        if self._writer is None:
            from concurrent.futures import ThreadPoolExecutor
            self._writer = [ThreadPoolExecutor(max_workers=1) for _ in range(4)]
        self._pending.append(self._writer[ref_id % len(self._writer)].submit(write))

    def _flush_writes(self):
        pending, self._pending = self._pending, []
        first = None
        for f in pending:
            try:
                f.result()
            except BaseException as e:  # every write is awaited; the first error is raised
                first = first or e
        if first is not None:
            raise first

    def _shutdown(self):
        if self._writer is not None:
            for w in self._writer:
                w.shutdown()
            self._writer = None
        if self.pool is not None:
            self.pool.close()
            self.pool = None

    def run(self) -> str:
        os.makedirs(self.output_folder, exist_ok=True)
        max_down = self.max_num_downscale
        first = True
        try:
            while max_down >= 0:
                pipeline.scale_step(self.problems)
                with self._timed("load"):
                    self._load_views()
                exchange = DepthExchange(self.assignment, self._shapes(), self.cdev, self.group,
                                         out_device=self.tdev)
                if first:
                    first = False
                    self.run_pass(False, True, False, False, exchange)
                else:
                    with self._timed("jbu"):
                        for v in self.mine + self.split:  # JointBilateralUpsampling, resident (split: on every rank)
                            p = self.problems[v]
                            img = self.images[p.ref_image_id]
                            up, isc = self.jbu(img, self.state[v].planes[..., 3])
                            if up is None:
                                raise AcmmpError(f"view {p.ref_image_id}: JBU image scale 1 (nothing to upsample)")
                            self.state[v].extra["jbu_depth"] = up
                    self.run_pass(False, True, True, False, exchange)
                for g in range(self.geom_iterations):
                    self.run_pass(True, False, False, g > 0, exchange)
                max_down -= 1
            with self._timed("flush_writes"):
                self._flush_writes()
        except BaseException:
            try:
                self._flush_writes()  # no write is left running; the pass's error wins
            except BaseException:
                pass
            raise
        finally:
            self._shutdown()
        if dist.is_initialized() and self.world > 1:
            dist.barrier(group=self.group)
        return self.output_folder


def main():
    """python -m torch.distributed.run --nproc-per-node N -m acmmp_amd.distributed <dense_folder> [...]"""
    import argparse
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("dense_folder")
    ap.add_argument("--output_dir", default="/ACMMP")
    ap.add_argument("--iterations", type=int, default=0)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--backend", default=None, help="nccl (RCCL, default with GPUs) or gloo")
    ap.add_argument("--concurrent_views", type=int, default=2,
                    help="views computed at once per GPU (one engine / HIP stream each)")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        backend = args.backend or ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
        dist.init_process_group(backend)
    pipe = ViewParallelPipeline(args.dense_folder, args.output_dir, device=local_rank, seed=args.seed,
                                max_iterations=args.iterations, concurrent_views=args.concurrent_views)
    out = pipe.run()
    if pipe.rank == 0:
        print(f"Depth/normal/cost maps written under {out}")
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
