"""Device-resident pass execution: a pool of engines (one HIP stream each) on
one GPU that runs the views of a pass with their inputs and outputs kept in
HBM.

This is the schedule `bench.py` times and the view-parallel driver
(`distributed.py`) uses:

* `EnginePool` owns S engines. One host thread per engine takes the next view
  of the pass off a shared queue as soon as its previous view finished (the
  library's ctypes calls release the GIL), so S views are in flight and the
  tail of one view's sweep launch fills with another's blocks.
* `photometric_view` / `geometric_view` are one view's RunPatchMatch
  (src/ACMMP.cu:1378-1456) with images borrowed from HBM
  (`acmmp_set_images_device`), the previous pass's state and the gathered
  depth maps borrowed from HBM (`acmmp_set_plane_hypotheses_device`,
  `acmmp_set_depth_maps_device`), and the results exported device-to-device
  (`acmmp_export_results`) into caller-owned buffers — the pass order of
  src/main_ACMMP.cpp:123-137 without the host round trips of ProcessProblem
  (src/acmmp_definitions.cpp:287-295).

Engines are reused across views and passes: every view starts from
`set_params(params)`, which resets all flags, so no state of an earlier view
leaks into a later one (the state buffers an engine keeps are either
overwritten by set_plane_hypotheses_device or not read, see k_init).
"""
from __future__ import annotations

import threading
from typing import Callable, Optional, Sequence

from . import _abi
from .engine import ACMMP


class EnginePool:
    """S engines on one device. `map(fn, jobs)` calls fn(engine, job) for
    every job, S at a time, and returns the results in job order."""

    def __init__(self, device: int, streams: int = 2, timing: bool = False):
        self.device = device
        self.engines = [ACMMP(device) for _ in range(max(int(streams), 1))]
        for e in self.engines:
            e.set_timing(timing)
        self.timing = timing
        self._lock = threading.Lock()
        self.sweep_ms = 0.0
        self.sweep_launches = 0

    def __len__(self):
        return len(self.engines)

    def close(self):
        for e in self.engines:
            e.close()
        self.engines = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def reset_timing(self):
        with self._lock:
            self.sweep_ms, self.sweep_launches = 0.0, 0

    def finish(self, eng: ACMMP):
        """Waits for the engine's stream; accumulates its sweep timing."""
        eng.synchronize()
        if self.timing:
            t = eng.timing()
            with self._lock:
                self.sweep_ms += t["sweep_ms"]
                self.sweep_launches += t["sweep_launches"]

    def map(self, fn: Callable, jobs: Sequence):
        jobs = list(jobs)
        results = [None] * len(jobs)
        if len(self.engines) == 1 or len(jobs) <= 1:
            for k, job in enumerate(jobs):
                results[k] = fn(self.engines[0], job)
            return results
        queue = list(range(len(jobs)))
        errors = []

        def worker(eng):
            try:
                while True:
                    with self._lock:
                        if not queue or errors:
                            return
                        k = queue.pop(0)
                    results[k] = fn(eng, jobs[k])
            except BaseException as e:  # re-raised on the calling thread
                with self._lock:
                    errors.append(e)

        threads = [threading.Thread(target=worker, args=(e,)) for e in self.engines]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        if errors:
            raise errors[0]
        return results


def _set_images(eng: ACMMP, cams, image_ptrs, pitches, textures):
    if textures is not None:  # prebuilt footprint records: no per-run padding
        eng.set_images_textures(cams, textures)
    else:
        eng.set_images_device(cams, image_ptrs, pitches)


def photometric_view(pool: EnginePool, eng: ACMMP, params: _abi.Params, cams: Sequence[_abi.Camera],
                     image_ptrs: Sequence[int], planes_out: int, costs_out: int, depth_out: int = 0,
                     pitches: Optional[Sequence[int]] = None, textures: Optional[Sequence] = None) -> _abi.Params:
    """Photometric RunPatchMatch of one view; results exported to device
    buffers (planes (H,W,4), costs (H,W), depth (H,W) = planes[..., 3]).
    Images come from `textures` (engine.Texture, one per view) when given,
    else borrowed from `image_ptrs`. Returns the parameters the run used."""
    eng.set_params(params)
    _set_images(eng, cams, image_ptrs, pitches, textures)
    used = eng.params
    eng.run_async()
    eng.export_results(planes_out, costs_out, depth_out)
    pool.finish(eng)
    return used


def geometric_view(pool: EnginePool, eng: ACMMP, params: _abi.Params, cams: Sequence[_abi.Camera],
                   image_ptrs: Sequence[int], depth_ptrs: Sequence[int], planes: int, costs: int,
                   planes_out: int = 0, costs_out: int = 0, depth_out: int = 0,
                   pitches: Optional[Sequence[int]] = None,
                   depth_pitches: Optional[Sequence[int]] = None, textures: Optional[Sequence] = None) -> _abi.Params:
    """Geometric-consistency RunPatchMatch of one view from the previous
    pass's state (planes/costs, device) and the source depth maps (device,
    e.g. slices of an all-gather). `params` must carry geom_consistency and
    the pass's max_iterations. Outputs default to overwriting the inputs."""
    eng.set_params(params)
    _set_images(eng, cams, image_ptrs, pitches, textures)
    eng.set_depth_maps_device(depth_ptrs, depth_pitches)
    eng.set_plane_hypotheses_device(planes, costs)
    used = eng.params
    eng.run_async()
    eng.export_results(planes_out or planes, costs_out or costs, depth_out)
    pool.finish(eng)
    return used


class ResidentViews:
    """The views one rank owns, resident in HBM: images (borrowed tensors),
    per-view planes (H,W,4) / costs / depth of the last pass, and the depth
    maps of every view the geometric pass reads (`all_depth`, indexed by
    global view id: a slice of an all-gather, or this rank's own maps).

    A pass is `pool.map` over the owned views; the exchange between passes is
    the caller's (`gather(my_depth, all_depth)`). This is bench.py's step and
    the cfg2 parity test's (tests/test_gpu_headline.py)."""

    def __init__(self, pool: EnginePool, cams: dict, images: dict, sources: dict, mine: Sequence[int],
                 height: int, width: int, total_views: Optional[int] = None, base_id: int = 0,
                 view_seed: Optional[int] = None):
        import torch
        from .engine import Texture
        self.pool = pool
        self.cams, self.images, self.sources = cams, images, sources
        # one texture per image tensor, shared by every view id that maps to
        # it (bench.py's rank copies of one scene), engine and pass
        by_tensor = {}
        self.textures = {}
        for i, im in images.items():
            key = (im.data_ptr(), tuple(im.shape))
            if key not in by_tensor:
                by_tensor[key] = Texture.of(im, pool.device)
            self.textures[i] = by_tensor[key]
        self.mine = list(mine)
        self.base_id = base_id
        # view_seed: every view's Philox key is view_seed + its global id (as
        # the pass drivers key seed + ref_image_id), else the params' own key
        self.view_seed = view_seed
        dev = next(iter(images.values())).device
        n = len(self.mine)
        self.planes = torch.empty((n, height, width, 4), dtype=torch.float32, device=dev)
        self.costs = torch.empty((n, height, width), dtype=torch.float32, device=dev)
        self.my_depth = torch.empty((n, height, width), dtype=torch.float32, device=dev)
        # without an exchange the geometric pass reads this rank's own maps
        self.all_depth = (self.my_depth if total_views is None else
                          torch.empty((total_views, height, width), dtype=torch.float32, device=dev))
        self.used_params = {}

    def _ids(self, v):
        return [v] + list(self.sources[v])

    def _depth_index(self, i):
        return i if self.all_depth is not self.my_depth else self.mine.index(i)

    def _params_of(self, params: _abi.Params, v: int) -> _abi.Params:
        if self.view_seed is None:
            return params
        p = type(params).from_buffer_copy(params)
        p.seed_lo = (self.view_seed + v) & 0xFFFFFFFF
        return p

    def photometric_pass(self, params: _abi.Params):
        def one(eng, kv):
            k, v = kv
            ids = self._ids(v)
            self.used_params[("photo", v)] = photometric_view(
                self.pool, eng, self._params_of(params, v), [self.cams[i] for i in ids],
                [self.images[i].data_ptr() for i in ids],
                self.planes[k].data_ptr(), self.costs[k].data_ptr(), self.my_depth[k].data_ptr(),
                textures=[self.textures[i] for i in ids])
        self.pool.map(one, list(enumerate(self.mine)))

    def geometric_pass(self, params: _abi.Params):
        """`params` carries geom_consistency and the pass's iterations; the
        state (planes/costs) of each view is read and rewritten in place, the
        source depths come from all_depth (not rewritten: Jacobi order)."""
        def one(eng, kv):
            k, v = kv
            ids = self._ids(v)
            self.used_params[("geom", v)] = geometric_view(
                self.pool, eng, self._params_of(params, v), [self.cams[i] for i in ids],
                [self.images[i].data_ptr() for i in ids],
                [self.all_depth[self._depth_index(i)].data_ptr() for i in ids],
                self.planes[k].data_ptr(), self.costs[k].data_ptr(), textures=[self.textures[i] for i in ids])
        self.pool.map(one, list(enumerate(self.mine)))
