"""Sanitizer tier: the host C/C++ of the product
library (JPEG / PNG / PNM decoders, .dmb and camera readers, Delaunay,
resize, RunFusion / RunPriorAwareFusion) and the CPU oracle, built with
AddressSanitizer + UndefinedBehaviorSanitizer (tests/asan/Makefile) and run
on valid inputs and on deterministic mutations of them (byte flips,
truncations, extreme header fields, duplicated / inserted ranges). Any
sanitizer report fails the test. CPU only; the GPU kernels are covered by the
-m gpu parity suite (GPU sanitizers are not available on the pool)."""
import fcntl
import os
import shutil
import subprocess

import numpy as np
import pytest

from acmmp_amd import io as aio

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN_DIR = os.path.join(ROOT, "tests", "asan")
DRIVER = os.path.join(ASAN_DIR, "build", "asan_driver")
ENV = dict(os.environ,
           ASAN_OPTIONS="detect_leaks=1:allocator_may_return_null=1:halt_on_error=1:abort_on_error=0",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", OMP_NUM_THREADS="2")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="g++ with libasan needed")


@pytest.fixture(scope="module")
def driver():
    # one make at a time (pytest-xdist workers would otherwise relink the
    # driver while another worker executes it: ETXTBSY)
    os.makedirs(os.path.join(ASAN_DIR, "build"), exist_ok=True)
    with open(os.path.join(ASAN_DIR, "build", ".make.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        r = subprocess.run(["make", "-s", "-C", ASAN_DIR], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return DRIVER


def run(args, cwd, timeout=300):
    r = subprocess.run(args, cwd=cwd, env=ENV, capture_output=True, text=True, timeout=timeout)
    out = r.stdout + r.stderr
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    return out


@pytest.fixture(scope="module")
def fixtures(tmp_path_factory):
    from PIL import Image
    d = tmp_path_factory.mktemp("asan_fx")
    rng = np.random.default_rng(1)
    g = (rng.random((37, 53)) * 255).astype(np.uint8)
    c = (rng.random((33, 47, 3)) * 255).astype(np.uint8)
    Image.fromarray(g, "L").save(d / "g.jpg", quality=90)
    Image.fromarray(g, "L").save(d / "g_rst.jpg", quality=75, restart_marker_blocks=2)
    Image.fromarray(c, "RGB").save(d / "c420.jpg", quality=85)
    Image.fromarray(c, "RGB").save(d / "c444.jpg", quality=85, subsampling=0)
    Image.fromarray(c, "RGB").save(d / "c422.jpg", quality=60, subsampling=1)
    # 16-bit quantisation tables (DQT Pq = 1, SOF1): coefficients x 2000 reach
    # the IDCT's pass-2 sums, the case its 64-bit widening is for
    Image.fromarray(g, "L").save(d / "g_q16.jpg", qtables=[[min(2000, 1 + 40 * i) for i in range(64)]])
    # progressive (SOF2): band scans, EOB runs, refinement bits
    Image.fromarray(g, "L").save(d / "g_prog.jpg", quality=90, progressive=True)
    Image.fromarray(c, "RGB").save(d / "c_prog.jpg", quality=85, progressive=True, restart_marker_blocks=2)
    Image.fromarray(g, "L").save(d / "g.png")
    Image.fromarray(c, "RGB").save(d / "c.png")
    Image.fromarray(np.dstack([c, c[..., :1]]), "RGBA").save(d / "c4.png")
    Image.fromarray((rng.random((20, 30)) * 65535).astype(np.uint16)).save(d / "g16.png")
    (d / "g.pgm").write_bytes(b"P5\n53 37\n255\n" + g.tobytes())
    aio.write_dmb(str(d / "d.dmb"), rng.random((17, 23)).astype(np.float32))
    aio.write_dmb(str(d / "n.dmb"), rng.random((17, 23, 3)).astype(np.float32))
    aio.write_camera(str(d / "cam.txt"), np.eye(3, dtype=np.float32) * 500, np.eye(3, dtype=np.float32),
                     np.zeros(3, np.float32), 1.0, 0.01, 192, 5.0)
    return d


IMAGES = ["g.jpg", "g_rst.jpg", "g_q16.jpg", "g_prog.jpg", "c_prog.jpg", "c420.jpg", "c444.jpg", "c422.jpg", "g.png", "c.png", "c4.png", "g16.png", "g.pgm"]


@pytest.mark.parametrize("name", IMAGES)
def test_image_decoders_fuzzed(driver, fixtures, name):
    run([driver, "image", name, "3000", str(IMAGES.index(name) + 1)], cwd=fixtures)


@pytest.mark.parametrize("name,kind", [("d.dmb", "dmb"), ("n.dmb", "dmb"), ("cam.txt", "cam")])
def test_dmb_and_camera_readers_fuzzed(driver, fixtures, name, kind):
    run([driver, kind, name, "2000", "7"], cwd=fixtures)


def test_delaunay_and_resize(driver, tmp_path):
    run([driver, "delaunay", "300", "3"], cwd=tmp_path)
    run([driver, "resize", "200", "4"], cwd=tmp_path)


def test_oracle_branches(driver, tmp_path):
    """RunPatchMatch restatement: photometric, geometric, planar prior,
    hierarchy (upsample), the T1 cost vectors and JBU, at an odd size."""
    run([driver, "oracle", "9"], cwd=tmp_path, timeout=600)


def test_fusion_and_prior_aware_fusion(driver, tmp_path):
    from test_fusion import _dense_with_maps
    d, out = _dense_with_maps(tmp_path)
    probs = [f"{i}:{(i + 1) % 4},{(i + 2) % 4}" for i in range(4)]
    assert "points=" in run([driver, "fusion", d, out, "-"] + probs, cwd=tmp_path)
    prior = d + "/ACMMP_PRIOR"
    for i in range(4):
        src, dst = aio.result_folder(out, i), aio.result_folder(prior, i)
        os.makedirs(dst, exist_ok=True)
        for name in ("depths_geom.dmb", "normals.dmb"):
            shutil.copy(os.path.join(src, name), os.path.join(dst, name))
    assert "points=" in run([driver, "fusion", d, prior, out] + probs, cwd=tmp_path)
