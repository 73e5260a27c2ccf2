"""End-to-end pass driver on the GPU (ProcessProblem + main_ACMMP's pass
order, src/acmmp_definitions.cpp:245-403, src/main_ACMMP.cpp:96-176) on a
synthetic COLMAP-style dense folder (JPEG images, cam.txt, pair.txt), against
the oracle restatement of the same passes. Every output .dmb is compared
bit-exactly (NaN == NaN)."""
import os
import subprocess

import numpy as np
import pytest

from acmmp_amd import io as aio
from acmmp_amd import pipeline, scene
from oracle_pipeline import OraclePipeline
from parity_util import assert_bit_exact

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dense(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("dense"))
    sc = scene.make_scene(num_views=5, width=160, height=120)
    scene.write_dense_folder(sc, d, num_src=4)
    return d


def _compare(out_folder, maps):
    n = 0
    for (view, name), arr in maps.items():
        got = aio.read_dmb(os.path.join(aio.result_folder(out_folder, view), name + ".dmb"))
        assert_bit_exact(got, arr, f"view {view} {name}")
        n += 1
    return n


def test_pipeline_sequential_matches_oracle(dense):
    out = pipeline.run_sequential(dense, "/ACMMP")
    maps = OraclePipeline(dense).run_single_scale("sequential")
    assert _compare(out, maps) == 5 * 4
    for v in range(5):
        assert os.path.getsize(os.path.join(aio.result_folder(out, v), "triangulation.png")) > 1000


def test_cli_matches_in_process_driver(dense):
    exe = os.path.join(ROOT, "acmmp_amd", "lib", "acmmp_main")
    r = subprocess.run([exe, dense, "--output_dir", "/CLI", "--quiet"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert os.path.getsize(os.path.join(dense + "/CLI", "ACMMP_model.ply")) > 1000  # RunFusion ran
    a, b = dense + "/ACMMP", dense + "/CLI"
    if not os.path.isdir(a):
        pipeline.run_sequential(dense, "/ACMMP")
    for v in range(5):
        for name in ("depths", "depths_geom", "normals", "costs"):
            x = aio.read_dmb(os.path.join(aio.result_folder(a, v), name + ".dmb"))
            y = aio.read_dmb(os.path.join(aio.result_folder(b, v), name + ".dmb"))
            assert_bit_exact(y, x, f"CLI view {v} {name}")


def test_multi_scale_jbu_hierarchy_matches_oracle(tmp_path):
    """Two scales (1010x760 -> 505x380 first): photometric + planar and two
    geometric passes at the coarse scale, then JBU, the hierarchy + planar
    pass and two geometric passes at full size."""
    d = str(tmp_path / "dense")
    sc = scene.make_scene(num_views=3, width=1010, height=760)
    scene.write_dense_folder(sc, d, num_src=1)
    out = pipeline.run_sequential(d, "/ACMMP", write_triangulation=False)
    maps = OraclePipeline(d).run_multi_scale("sequential")
    assert _compare(out, maps) == 3 * 4
    assert aio.read_dmb(os.path.join(aio.result_folder(out, 0), "depths_geom.dmb")).shape == (760, 1010)


def test_seeded_pipeline_matches_oracle(tmp_path):
    """main_ACMMP -p: the first pass is seeded from 16-bit prior PNGs
    (pSampler, src/acmmp_definitions.cpp:99-177, SetPlanarPrior)."""
    from test_seeded_priors import _write_priors
    d = str(tmp_path / "dense") + "/"
    sc = scene.make_scene(num_views=4, width=128, height=96)
    scene.write_dense_folder(sc, d, num_src=3)
    rng = np.random.default_rng(5)
    priors = {}
    for i, v in enumerate(sc.views):
        dep = np.clip((v.depth - 300.0) / 500.0 * 65535.0 + rng.normal(0, 300, v.depth.shape), 0, 65535)
        dep = np.where(v.depth > 0, dep, 30000).astype(np.uint16)
        nrm = np.clip((v.normal + 1.0) * 32768.0, 0, 65535).astype(np.uint16)
        _write_priors(d, i, dep, nrm)
        priors[i] = (dep, nrm[..., ::-1])
    out = pipeline.run_sequential(d, prior=True, write_triangulation=False)
    assert out.endswith("/ACMMP_PRIOR")
    maps = OraclePipeline(d).run_single_scale("sequential", priors=priors)
    assert _compare(out, maps) == 4 * 4


def test_cli_fusion_of_gpu_maps_matches_restatement(dense):
    """RunFusion (src/acmmp_definitions.cpp:828-1043) over the maps the GPU
    passes wrote: the C++ CLI's PLY against the Python restatement
    (tests/oracle_fusion.py) over the same maps, record for record,
    bit-exact. Record order: the reference writes its PLY records from an
    `omp parallel for` with an `omp critical` fwrite (src/ACMMP.cpp:405-432),
    i.e. in a nondeterministic order; ours keep the fusion's own point order
    (pixel order of each view, views in pair.txt order), so a reference PLY of
    the same maps equals ours as a multiset of records."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oracle_fusion import read_ply, run_fusion
    from test_fusion import _compare_cloud
    exe = os.path.join(ROOT, "acmmp_amd", "lib", "acmmp_main")
    r = subprocess.run([exe, dense, "--output_dir", "/CLIF", "--quiet"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    ply = read_ply(os.path.join(dense + "/CLIF", "ACMMP_model.ply"))
    ref = run_fusion(dense, dense + "/CLIF")
    assert len(ref) > 1000
    _compare_cloud(ply, ref)
