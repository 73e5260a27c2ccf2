"""JBU (src/ACMMP.cu:1458-1549, src/ACMMP.cpp:1008-1087) on the GPU vs the CPU
oracle, bit-exact, for Imagescale 2 and 4 and a non-integer size ratio."""
import numpy as np
import pytest

import oracle
from acmmp_amd import joint_bilateral_upsample

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("W,H,sw,sh", [(160, 120, 80, 60), (96, 64, 24, 16), (101, 77, 50, 38)])
def test_jbu_matches_oracle(W, H, sw, sh):
    rng = np.random.default_rng(W)
    img = np.clip(rng.normal(128, 50, (H, W)), 0, 255).astype(np.float32).round()
    dep = rng.uniform(400, 800, (sh, sw)).astype(np.float32)
    dep[rng.random((sh, sw)) < 0.05] = 0.0
    ours, isc = joint_bilateral_upsample(img, dep)
    ref, risc = oracle.jbu(img, dep)
    assert isc == risc >= 2
    np.testing.assert_array_equal(ours.view(np.uint32), ref.view(np.uint32))


def test_jbu_same_size_writes_nothing():
    img = np.zeros((40, 50), np.float32)
    out, isc = joint_bilateral_upsample(img, np.ones((40, 50), np.float32))
    assert out is None and isc == 1


@pytest.mark.parametrize("W,H,sw,sh", [(160, 120, 80, 60), (101, 77, 50, 38)])
def test_jbu_device_buffers_match_oracle(W, H, sw, sh):
    """The view-parallel driver's resident JBU (acmmp_joint_bilateral_upsample_device)."""
    import torch
    from acmmp_amd.engine import joint_bilateral_upsample_device
    rng = np.random.default_rng(W + 1)
    img = np.clip(rng.normal(128, 50, (H, W)), 0, 255).astype(np.float32).round()
    dep = rng.uniform(400, 800, (sh, sw)).astype(np.float32)
    dev = torch.device("cuda", 0)
    ti, td = torch.from_numpy(img).to(dev), torch.from_numpy(dep).to(dev)
    to = torch.full_like(ti, -1.0)
    torch.cuda.synchronize()
    isc = joint_bilateral_upsample_device(ti.data_ptr(), W, H, td.data_ptr(), sw, sh, to.data_ptr())
    ref, risc = oracle.jbu(img, dep)
    assert isc == risc >= 2
    np.testing.assert_array_equal(to.cpu().numpy().view(np.uint32), ref.view(np.uint32))
