"""View-parallel driver with the real engine: two ranks sharing
the box's one GPU (gloo carries the depth all-gather between them; on an
8-GPU node the same code uses RCCL) against the oracle pipeline in Jacobi
order, every output .dmb bit-exact. Also world size 1 in-process."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from acmmp_amd import scene
from acmmp_amd.distributed import ViewParallelPipeline
from oracle_pipeline import OraclePipeline
from test_gpu_pipeline import _compare

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, dense, q):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        pipe = ViewParallelPipeline(dense, "/VP2", device=0, tensor_device=torch.device("cuda", 0),
                                    comm_device=torch.device("cpu"))
        pipe.run()
        q.put((rank, pipe.mine))
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def dense(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("vp"))
    sc = scene.make_scene(num_views=5, width=160, height=120)
    scene.write_dense_folder(sc, d, num_src=4)
    return d


@pytest.fixture(scope="module")
def jacobi_maps(dense):
    return OraclePipeline(dense).run_single_scale("jacobi")


@pytest.mark.parametrize("concurrent", [1, 2])
def test_world1_matches_oracle_jacobi(dense, jacobi_maps, concurrent):
    """World size 1; concurrent=2 computes two views at once on two engines
    (HIP streams) from two threads — the outputs must not change."""
    out = ViewParallelPipeline(dense, f"/VP1c{concurrent}", device=0, concurrent_views=concurrent).run()
    assert _compare(out, jacobi_maps) == 5 * 4


def test_world2_matches_oracle_jacobi(dense, jacobi_maps):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, dense, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    mine = dict(q.get(timeout=5) for _ in range(2))
    assert sorted(mine[0] + mine[1]) == list(range(5)) and mine[0] and mine[1]
    assert _compare(dense + "/VP2", jacobi_maps) == 5 * 4
