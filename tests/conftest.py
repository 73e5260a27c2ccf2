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
