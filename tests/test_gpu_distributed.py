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
from parity_util import assert_dmb_trees_equal
from test_gpu_pipeline import _compare

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, dense, q, backend="gloo", out="/VP2", split_tail=True):
    if backend == "nccl":
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                                device_id=torch.device("cuda", 0))
        comm = torch.device("cuda", 0)  # RCCL: the all-gather runs on device buffers
    else:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        comm = torch.device("cpu")
    try:
        pipe = ViewParallelPipeline(dense, out, device=0, tensor_device=torch.device("cuda", 0),
                                    comm_device=comm, split_tail=split_tail)
        pipe.run()
        q.put((rank, (pipe.owned, pipe.split)))
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


def _spawn(world, dense, backend, out, split_tail=True):
    """Runs the driver on `world` ranks; returns {rank: (owned views, split views)}."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, dense, q, backend, out, split_tail))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    return dict(q.get(timeout=5) for _ in range(world))


@pytest.mark.parametrize("split_tail", [False, True])
def test_world2_matches_oracle_jacobi(dense, jacobi_maps, split_tail):
    """5 views on 2 ranks: with split_tail the odd view is computed in two
    row bands, one per rank, with the halos exchanged every half-sweep."""
    out = "/VP2s" if split_tail else "/VP2"
    got = _spawn(2, dense, "gloo", out, split_tail)
    assert sorted(got[0][0] + got[1][0]) == list(range(5)) and got[0][0] and got[1][0]
    assert got[0][1] == got[1][1] == ([4] if split_tail else [])
    assert _compare(dense + out, jacobi_maps) == 5 * 4


def test_world1_nccl_process_group_matches_oracle_jacobi(dense, jacobi_maps):
    """A real RCCL process group (world size 1): DepthExchange.gather runs
    all_gather_into_tensor on device buffers through RCCL after every pass,
    and the engines borrow the gathered maps (torch/RCCL stream
    ordering before the borrow)."""
    got = _spawn(1, dense, "nccl", "/VPN")
    assert got[0] == (list(range(5)), [])
    assert _compare(dense + "/VPN", jacobi_maps) == 5 * 4


@pytest.mark.timeout(600)
def test_world2_multi_scale_matches_oracle_jacobi(ms4_dense, ms4_oracle_maps):
    """cfg4's schedule (src/main_ACMMP.cpp:96-176) view-parallel: two scales
    (1010x760 -> 505x380 first), photometric + planar, two geometric passes,
    JBU, hierarchy + planar, two geometric passes — two ranks on the one GPU
    against the oracle pipeline in Jacobi order, every .dmb bit-exact."""
    d = ms4_dense
    got = _spawn(2, d, "gloo", "/VPMS")
    assert sorted(got[0][0] + got[1][0]) == list(range(4)) and got[0][0] and got[1][0]
    assert _compare(d + "/VPMS", ms4_oracle_maps) == 4 * 4


@pytest.mark.timeout(600)
def test_world2_multi_scale_split_tail_matches_oracle_jacobi(ms3_dense, ms3_oracle_maps):
    """The same schedule with 3 views on 2 ranks: the third view is split in
    row bands over both ranks in every pass — photometric + planar prior
    (prior built on both ranks from the gathered first run), geometric,
    JBU + hierarchy — and every .dmb stays bit-exact to the oracle."""
    d = ms3_dense
    got = _spawn(2, d, "gloo", "/VPMS3")
    assert got[0][1] == got[1][1] == [2]
    assert sorted(got[0][0] + got[1][0]) == [0, 1, 2]
    assert _compare(d + "/VPMS3", ms3_oracle_maps) == 3 * 4


def test_bench_under_torchrun_nccl_world1():
    """bench.py through torch.distributed.run at world size 1: a process
    group, the RCCL all-gather between the passes, one JSON line."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", "1", "--steps", "1", "--warmup", "0", "--width", "400", "--height", "300",
           "--pmc", "off", "--no-cpu-baseline", "--backend", "nccl"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == 1 and res["value"] > 0
    assert "RCCL all-gather" in res["config"]["parallelism"]


@pytest.mark.timeout(900)
def test_world8_split_tail_multi_scale_matches_world1(tmp_path):
    """The 8-rank path a node runs, rehearsed on the one GPU (8 gloo ranks
    sharing it): 17 views -> 2 whole views per rank and the 17th split in
    8 row bands (47 rows each at the coarse scale, 95 at the fine one) in
    every pass of the multi-scale schedule; every .dmb bit-identical to the
    world-1 run (which the tests above pin to the oracle)."""
    d = str(tmp_path / "dense17")
    sc = scene.make_scene(num_views=17, width=1010, height=760)
    scene.write_dense_folder(sc, d, num_src=4)
    got = _spawn(8, d, "gloo", "/VP8")
    assert all(got[r][1] == [16] for r in range(8))
    assert sorted(v for r in range(8) for v in got[r][0]) == list(range(17))
    ViewParallelPipeline(d, "/VP1", device=0).run()
    assert_dmb_trees_equal(d + "/VP8", d + "/VP1", range(17), "world 8 vs world 1")
