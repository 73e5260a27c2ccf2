"""C++ view-parallel driver (`acmmp_main --view_parallel`, acmmp_amd/csrc/
acmmp_vp.cpp): one process per GPU, views sharded
per pass, depth maps all-gathered between passes — RCCL at world size 1 (the
same ncclAllGather an 8-GPU node runs), and two ranks sharing the box's one
GPU through the TCP exchange (RCCL refuses two ranks on one device). Every
.dmb must be bit-identical to the oracle pipeline in Jacobi order, which the
Python driver (tests/test_gpu_distributed.py) also matches."""
import os
import socket
import subprocess

import pytest

from acmmp_amd import scene
from oracle_pipeline import OraclePipeline
from test_gpu_pipeline import _compare

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "acmmp_amd", "lib", "acmmp_main")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(dense, out, world, exchange, extra=(), timeout=400):
    """`world` ranks of acmmp_main --view_parallel on device 0; returns their outputs."""
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port - 1), ACMMP_RDZV_PORT=str(port))
        cmd = [EXE, dense, "--view_parallel", "--exchange", exchange, "--device", "0", "--output_dir", out,
               "--quiet"] + list(extra)
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        so, se = p.communicate(timeout=timeout)
        outs.append((p.returncode, so, se))
    for rc, so, se in outs:
        assert rc == 0, se[-3000:]
    return outs


@pytest.fixture(scope="module")
def dense(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("cvp"))
    sc = scene.make_scene(num_views=5, width=160, height=120)
    scene.write_dense_folder(sc, d, num_src=4)
    return d


@pytest.fixture(scope="module")
def jacobi_maps(dense):
    return OraclePipeline(dense).run_single_scale("jacobi")


def test_world1_rccl_matches_oracle_jacobi(dense, jacobi_maps):
    _launch(dense, "/CVP1", 1, "rccl", ["--no_fusion"])
    assert _compare(dense + "/CVP1", jacobi_maps) == 5 * 4


def test_order_jacobi_on_one_gpu_matches_oracle(dense, jacobi_maps):
    """a one-GPU run offers both pass orders; `--order jacobi`
    (no launcher, no rank environment) gives the Jacobi pipeline's maps."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([EXE, dense, "--order", "jacobi", "--output_dir", "/CVPO", "--no_fusion", "--quiet"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert _compare(dense + "/CVPO", jacobi_maps) == 5 * 4


@pytest.mark.parametrize("split", [True, False])
def test_world2_tcp_matches_oracle_jacobi_and_fuses(dense, jacobi_maps, split):
    """5 views on 2 ranks: by default the 5th is computed by both ranks as
    two row bands (halos all-gathered after every half-sweep)."""
    out = "/CVP2" if split else "/CVP2w"
    _launch(dense, out, 2, "tcp", [] if split else ["--no_split_tail"])
    assert _compare(dense + out, jacobi_maps) == 5 * 4
    # rank 0 fused the maps after the last pass (main_ACMMP's RunFusion)
    assert os.path.getsize(os.path.join(dense + out, "ACMMP_model.ply")) > 1000


@pytest.mark.timeout(900)
def test_world2_tcp_multi_scale_matches_oracle_jacobi(ms4_dense, ms4_oracle_maps):
    """Two scales (1010x760 -> 505x380 first): planar pass, two geometric
    passes, JBU + hierarchy + planar, two geometric passes."""
    d = ms4_dense
    _launch(d, "/CVPMS", 2, "tcp", ["--no_fusion"], timeout=600)
    assert _compare(d + "/CVPMS", ms4_oracle_maps) == 4 * 4


@pytest.mark.timeout(900)
def test_world2_tcp_multi_scale_split_tail_matches_oracle_jacobi(ms3_dense, ms3_oracle_maps):
    """3 views on 2 ranks through the multi-scale schedule: the third view in
    two row bands in every pass (planar prior rebuilt on both ranks, JBU and
    hierarchy inputs on both), every .dmb bit-exact."""
    d = ms3_dense
    _launch(d, "/CVPMS3", 2, "tcp", ["--no_fusion"], timeout=600)
    assert _compare(d + "/CVPMS3", ms3_oracle_maps) == 3 * 4


@pytest.mark.timeout(900)
def test_world2_tcp_cfg4_source_count(tmp_path):
    """cfg4's problem shape (each view with its 20 best sources, N = 21:
    colmap2mvsnet_acm.py:415) through the whole schedule at world 2 — the
    NS=32 kernel bucket inside the driver, planar prior and both geometric
    passes — bit-exact against the oracle pipeline in Jacobi order."""
    d = str(tmp_path / "dense_n21")
    sc = scene.make_scene(num_views=22, width=160, height=120)
    scene.write_dense_folder(sc, d, num_src=20)
    _launch(d, "/CVPN21", 2, "tcp", ["--no_fusion"], timeout=600)
    maps = OraclePipeline(d).run_single_scale("jacobi")
    assert _compare(d + "/CVPN21", maps) == 22 * 4
