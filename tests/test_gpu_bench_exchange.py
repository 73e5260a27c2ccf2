"""bench.py's N > 1 exchange is load-bearing: sources span
ranks (bench.view_sources), so every rank's geometric pass reads depth maps
that only the all-gather delivers. A world-2 run over gloo with both ranks on
the one GPU must leave every view's geometric planes and costs bit-identical
to one process that holds both ranks' views and reads the maps directly
(`--emulate-ranks 2`, no collective); and the two rank copies of a scene view
must have different depth maps (their own Philox keys), so a missing, partial
or mis-ordered all-gather would change the outputs."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from parity_util import assert_bit_exact

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMMON = ["--steps", "1", "--warmup", "0", "--views", "10", "--nsrc", "9", "--width", "320", "--height", "240",
          "--iters", "3", "--no-cpu-baseline", "--pmc", "off", "--streams", "2"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(600)
def test_world2_gloo_geometric_outputs_equal_one_process(tmp_path):
    d2, d1 = str(tmp_path / "world2"), str(tmp_path / "one")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--backend", "gloo", "--dump", d2, *COMMON]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--emulate-ranks", "2", "--dump", d1,
                        *COMMON], capture_output=True, text=True, timeout=400, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    names = sorted(os.listdir(d1))
    assert sorted(os.listdir(d2)) == names and len(names) == 3 * 20
    for n in names:
        assert_bit_exact(np.load(os.path.join(d2, n)), np.load(os.path.join(d1, n)), f"world 2 vs one process: {n}")
    # the copies differ, so reading the wrong rank's slot would show
    for m in range(10):
        a = np.load(os.path.join(d1, f"photo_depth_{m:03d}.npy"))
        b = np.load(os.path.join(d1, f"photo_depth_{10 + m:03d}.npy"))
        assert (a.view(np.uint32) != b.view(np.uint32)).mean() > 0.1, m
