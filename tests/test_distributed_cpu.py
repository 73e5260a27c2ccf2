"""View-parallel driver (acmmp_amd/distributed.py) on CPU with
the gloo backend: LPT sharding, the padded depth all-gather, and the Jacobi
pass schedule at world size 2 against world size 1, single- and multi-scale.
The per-view engine and JBU are replaced by deterministic stand-ins here (no
GPU in this container); tests/test_gpu_distributed.py runs the real engine."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from acmmp_amd import io as aio
from acmmp_amd import scene
from acmmp_amd.distributed import DepthExchange, ViewParallelPipeline, ViewResult, lpt_assign, plan_views


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_lpt_assign():
    assert lpt_assign([1, 1, 1, 1], 2) == [[0, 2], [1, 3]]
    assert lpt_assign([5, 1, 1, 1, 1, 1], 2) == [[0], [1, 2, 3, 4, 5]]
    a = lpt_assign([3.0, 2.0, 2.0, 1.0, 1.0, 1.0, 4.0], 3)
    assert sorted(v for r in a for v in r) == list(range(7))
    assert lpt_assign([1, 2], 4)[2:] == [[], []]


def test_plan_views_split_tail():
    """cfg4 at 8 ranks: 49 equal views -> 48 whole views, 6 per rank, and
    the 49th split over all ranks, owned by rank 0."""
    a, split = plan_views([1.0] * 49, 8, True)
    assert split == [48]
    assert [len(r) for r in a] == [7] + [6] * 7 and 48 in a[0]
    assert sorted(v for r in a for v in r) == list(range(49))
    # no tail: nothing split; split_tail off: plain LPT
    assert plan_views([1.0] * 16, 8, True) == (lpt_assign([1.0] * 16, 8), [])
    assert plan_views([1.0] * 49, 8, False) == (lpt_assign([1.0] * 49, 8), [])
    # unequal views: the cheapest ones are split
    a, split = plan_views([4.0, 1.0, 3.0, 2.0, 5.0], 2, True)
    assert split == [1] and sorted(v for r in a for v in r) == list(range(5))


def fake_compute(t, eng=None):
    """Deterministic stand-in for ProcessProblem's engine work: depends on the
    view's images, on every source depth map (geom) and on its own state.
    Tensors in, tensors out, like the real engine_compute."""
    img = t.images[0].cpu().numpy().astype(np.float64)
    H, W = img.shape
    depth = 500.0 + img / 10.0 + 3.0 * t.seed_hi
    if t.geom:
        depth = depth + sum(float(d.cpu().double().mean()) for d in t.depths) / 100.0
        depth = depth + t.state[0][..., 3].cpu().numpy() / 1000.0 + (7.0 if t.multi else 0.0)
    if t.hierarchy:
        depth = depth + t.hier_inputs[1].cpu().numpy() / 100.0 + float(t.hier_inputs[0].double().mean())
    planes = np.zeros((H, W, 4), np.float32)
    planes[..., 2] = -1.0
    planes[..., 3] = depth
    costs = (img / 255.0).astype(np.float32)
    if t.planar:
        costs = costs * 0.5
    return ViewResult(torch.from_numpy(planes), torch.from_numpy(costs))


def fake_jbu(image, depth):
    """Tensors in, tensor out, like the driver's gpu_jbu."""
    H, W = image.shape
    ys = (np.arange(H) * depth.shape[0] // H)[:, None]
    xs = (np.arange(W) * depth.shape[1] // W)[None, :]
    return torch.from_numpy(depth.cpu().numpy()[ys, xs].astype(np.float32)), 2


def _worker(rank, world, port, dense, out_dir, q):
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        pipe = ViewParallelPipeline(dense, out_dir, compute=fake_compute, jbu=fake_jbu,
                                    tensor_device=torch.device("cpu"))
        pipe.run()
        q.put((rank, pipe.mine))
    finally:
        dist.destroy_process_group()


def _run_world(dense, out_dir, world):
    if world == 1:
        pipe = ViewParallelPipeline(dense, out_dir, compute=fake_compute, jbu=fake_jbu,
                                    tensor_device=torch.device("cpu"))
        pipe.run()
        return {0: pipe.mine}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, dense, out_dir, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    return dict(q.get(timeout=5) for _ in range(world))


def _exchange_worker(rank, world, port, q):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        assignment = [[0, 2, 3], [1]]
        shapes = {0: (5, 7), 1: (3, 4), 2: (6, 2), 3: (1, 1)}
        ex = DepthExchange(assignment, shapes, torch.device("cpu"))
        local = {v: torch.full(shapes[v], float(10 * v + rank)) for v in assignment[rank]}
        got = ex.gather(rank, local)
        q.put((rank, {v: (tuple(t.shape), float(t.sum())) for v, t in got.items()}))
    finally:
        dist.destroy_process_group()


def test_depth_exchange_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    res = dict(q.get(timeout=5) for _ in range(2))
    shapes = {0: (5, 7), 1: (3, 4), 2: (6, 2), 3: (1, 1)}
    owner = {0: 0, 2: 0, 3: 0, 1: 1}
    for r in range(2):
        for v, (shape, s) in res[r].items():
            assert shape == shapes[v]
            assert s == (10 * v + owner[v]) * shapes[v][0] * shapes[v][1]


def _dense(tmp_path, W, H, views=4):
    d = str(tmp_path / f"dense_{W}")
    sc = scene.make_scene(num_views=views, width=W, height=H)
    scene.write_dense_folder(sc, d, fmt="pgm", num_src=2)
    return d


@pytest.mark.parametrize("W,H", [(96, 72), (1010, 760)])
def test_world2_equals_world1(tmp_path, W, H):
    dense = _dense(tmp_path, W, H)
    mine1 = _run_world(dense, "/W1", 1)
    mine2 = _run_world(dense, "/W2", 2)
    assert mine1[0] == [0, 1, 2, 3]
    assert sorted(mine2[0] + mine2[1]) == [0, 1, 2, 3] and mine2[0] and mine2[1]
    for v in range(4):
        for name in ("depths", "depths_geom", "normals", "costs"):
            a = aio.read_dmb(os.path.join(aio.result_folder(dense + "/W1", v), name + ".dmb"))
            b = aio.read_dmb(os.path.join(aio.result_folder(dense + "/W2", v), name + ".dmb"))
            np.testing.assert_array_equal(a, b)
    if W > 1000:  # two scales: the final maps are at full size
        assert aio.read_dmb(os.path.join(aio.result_folder(dense + "/W2", 0), "depths_geom.dmb")).shape == (H, W)
