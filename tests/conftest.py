import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) — run with -m gpu")


@pytest.fixture(scope="session")
def has_gpu():
    from acmmp_amd import _abi
    try:
        return _abi.load_library().acmmp_device_count() > 0
    except Exception:
        return False


# GPU files in the order the round-end run (`pytest -x -m gpu`) should reach
# them: kernel- and oracle-level parity of the hot path first, so one failing
# multi-process driver test can never hide it; the
# multi-process drivers (several ranks sharing the box's GPU) last.
_FIRST = ["test_gpu_parity", "test_gpu_headline", "test_gpu_sweep_views", "test_gpu_texel_modes",
          "test_gpu_planar", "test_gpu_pipeline", "test_gpu_wide", "test_gpu_jbu"]
_LAST = ["test_gpu_band", "test_gpu_distributed", "test_gpu_vp_cli", "test_gpu_cfg4"]


# Multi-scale driver inputs shared by test_gpu_distributed.py and
# test_gpu_vp_cli.py (same scenes, so the oracle pipeline — the slow part —
# runs once per session; each driver writes its own output subfolder).
def _ms_dense(tmp_path_factory, views):
    from acmmp_amd import scene
    d = str(tmp_path_factory.mktemp(f"dense_ms{views}"))
    sc = scene.make_scene(num_views=views, width=1010, height=760)
    scene.write_dense_folder(sc, d, num_src=2)
    return d


@pytest.fixture(scope="session")
def ms4_dense(tmp_path_factory):
    """4 views at 1010x760, 2 sources each: two scales of cfg4's schedule."""
    return _ms_dense(tmp_path_factory, 4)


@pytest.fixture(scope="session")
def ms3_dense(tmp_path_factory):
    """3 views at 1010x760: at world 2 the third is split in row bands."""
    return _ms_dense(tmp_path_factory, 3)


@pytest.fixture(scope="session")
def ms4_oracle_maps(ms4_dense):
    from oracle_pipeline import OraclePipeline
    return OraclePipeline(ms4_dense).run_multi_scale("jacobi")


@pytest.fixture(scope="session")
def ms3_oracle_maps(ms3_dense):
    from oracle_pipeline import OraclePipeline
    return OraclePipeline(ms3_dense).run_multi_scale("jacobi")


def _file_rank(item):
    name = os.path.splitext(os.path.basename(str(item.fspath)))[0]
    if name in _FIRST:
        return _FIRST.index(name)
    if name in _LAST:
        return 100 + _LAST.index(name)
    return 50


def pytest_collection_modifyitems(session, config, items):
    items.sort(key=_file_rank)  # stable: the order inside a file is kept
