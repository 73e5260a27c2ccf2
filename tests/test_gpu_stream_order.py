"""acmmp_wait_stream (include/acmmp.h): an engine's `*_device` setters and
export run on its own non-blocking stream, ordered after torch's current
stream by ACMMP._after_producer. Here torch's stream is held ~0.2 s behind
(torch.cuda._sleep) before it writes the buffers an engine then copies:
without the ordering the engine would copy the old contents."""
import numpy as np
import pytest
import torch

from acmmp_amd import ACMMP, default_params, scene

pytestmark = pytest.mark.gpu

SLEEP = 400_000_000  # GPU clock cycles (~0.2 s)


@pytest.fixture(scope="module")
def eng():
    sc = scene.make_scene(num_views=3, width=64, height=48)
    cams, imgs = sc.problem(0, 2)
    e = ACMMP(0)
    p = default_params()
    p.max_iterations = 1
    e.set_params(p)
    e.set_images(cams, imgs)
    yield e
    e.close()


def test_setter_waits_for_torch_stream(eng):
    W, H = eng.size
    dev = torch.device("cuda", 0)
    planes = torch.zeros((H, W, 4), dtype=torch.float32, device=dev)
    costs = torch.zeros((H, W), dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    torch.cuda._sleep(SLEEP)           # torch's stream is busy for a while ...
    planes.fill_(1.5)                  # ... before these writes land
    costs.fill_(0.25)
    eng.set_plane_hypotheses_device(planes.data_ptr(), costs.data_ptr())
    out_p = torch.empty_like(planes)
    out_c = torch.empty_like(costs)
    eng.export_results(out_p.data_ptr(), out_c.data_ptr(), 0)
    eng.synchronize()
    torch.cuda.synchronize()
    assert (out_p == 1.5).all().item() and (out_c == 0.25).all().item()


def test_export_waits_for_torch_stream(eng):
    """The export's destination may still be in use on torch's stream (the
    caching allocator recycles memory in stream order): the export lands
    after torch's pending writes to it, never under them."""
    W, H = eng.size
    dev = torch.device("cuda", 0)
    planes = torch.full((H, W, 4), 2.0, dtype=torch.float32, device=dev)
    costs = torch.full((H, W), 0.5, dtype=torch.float32, device=dev)
    eng.set_plane_hypotheses_device(planes.data_ptr(), costs.data_ptr())
    eng.synchronize()
    dst_p = torch.empty_like(planes)
    dst_c = torch.empty_like(costs)
    torch.cuda._sleep(SLEEP)
    dst_p.fill_(-1.0)                  # a pending torch write the export must follow
    dst_c.fill_(-1.0)
    eng.export_results(dst_p.data_ptr(), dst_c.data_ptr(), 0)
    eng.synchronize()
    torch.cuda.synchronize()
    assert np.array_equal(dst_p.cpu().numpy(), planes.cpu().numpy())
    assert np.array_equal(dst_c.cpu().numpy(), costs.cpu().numpy())
