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


def _file_rank(item):
    name = os.path.splitext(os.path.basename(str(item.fspath)))[0]
    if name in _FIRST:
        return _FIRST.index(name)
    if name in _LAST:
        return 100 + _LAST.index(name)
    return 50


def pytest_collection_modifyitems(session, config, items):
    items.sort(key=_file_rank)  # stable: the order inside a file is kept
