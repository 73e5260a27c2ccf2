"""Views of 2^24 padded records or more (ETH3D high-res at native size,
BASELINE cfg5: 6048x4032): the gather kernels then form the record index with
an integer 24x24-bit multiply-add instead of the exact-fp32 form
(acmmp_kernels.hip, ncc_sums_rows<FAST, WIDE>).

  * ACMMP_WIDE_INDEX=1 forces that path at oracle-sized inputs, so it is held
    to the same bit-exact parity as the default path (T1 cost vectors, T3
    RunPatchMatch);
  * at 6048x4032 the path is selected by size; the NCC costs of random
    hypotheses are checked bit-exactly against the oracle's ComputeBilateralNCC
    on a sample of pixels spread over the whole image (the oracle cannot run
    24 Mpix in test time), and RunPatchMatch runs end to end against the
    analytic depth.
"""
import numpy as np
import pytest

import oracle
from acmmp_amd import ACMMP, default_params, scene
from parity_util import assert_bit_exact

pytestmark = pytest.mark.gpu


def _params(iters=2):
    p = default_params()
    p.max_iterations = iters
    return p


def _random_planes(K, H, W, seed):
    """Camera-frame planes (n, d), n facing the camera, depth in [400, 800]."""
    rng = np.random.default_rng(seed)
    n = rng.normal(size=(H, W, 3)).astype(np.float32)
    n[..., 2] = -np.abs(n[..., 2]) - 0.5
    n /= np.linalg.norm(n, axis=-1, keepdims=True)
    depth = rng.uniform(400, 800, size=(H, W)).astype(np.float32)
    ys, xs = np.mgrid[0:H, 0:W].astype(np.float32)
    X = np.stack([depth * (xs - K[0, 2]) / K[0, 0], depth * (ys - K[1, 2]) / K[1, 1], depth], -1)
    d = -(n * X).sum(-1)
    return np.concatenate([n, d[..., None]], -1).astype(np.float32)


@pytest.fixture(params=["h16", "u8", "f32"])
def wide_index(monkeypatch, request):
    """Forced integer record index, with every texel form (f16 difference
    quads / u8 quads / fp32 row pairs, tests/test_gpu_texel_modes.py)."""
    monkeypatch.setenv("ACMMP_WIDE_INDEX", "1")
    monkeypatch.setenv("ACMMP_TEXEL", request.param)


def test_forced_wide_index_cost_vectors(wide_index):
    sc = scene.make_scene(num_views=10, width=80, height=60, arc_deg=4.0)
    cams, imgs = sc.problem(0, 9)
    H, W = imgs[0].shape
    planes = _random_planes(np.array(cams[0].K).reshape(3, 3), H, W, seed=9)
    with ACMMP(0) as eng:
        eng.set_params(_params())
        eng.set_images(cams, imgs)
        prm = eng.params
        g_cost, g_init, g_views = eng.eval_costs(planes)
    r_cost, r_init, r_views = oracle.eval_costs(prm, cams, imgs, planes)
    assert_bit_exact(g_cost, r_cost, "ncc cost vectors (wide index)")
    assert_bit_exact(g_init, r_init, "initial cost (wide index)")
    assert_bit_exact(g_views, r_views, "initial selected views (wide index)")
    assert (r_cost < 2).mean() > 0.05


def test_forced_wide_index_run_patchmatch(wide_index):
    sc = scene.make_scene(num_views=6, width=128, height=96)
    cams, imgs = sc.problem(0, 5)
    with ACMMP(0) as eng:
        eng.set_params(_params(2))
        eng.set_images(cams, imgs)
        prm = eng.params
        eng.RunPatchMatch()
        pl, co, sv = eng.plane_hypotheses(), eng.costs(), eng.selected_views()
    ref = oracle.run_patchmatch(prm, cams, imgs)
    assert_bit_exact(pl, ref["planes"], "planes (wide index)")
    assert_bit_exact(co, ref["costs"], "costs (wide index)")
    assert_bit_exact(sv, ref["selected_views"], "selected views (wide index)")


@pytest.fixture(scope="module")
def eth3d_views():
    """cfg5: 10 views at 6048x4032 rendered straight into HBM."""
    import torch

    setup = scene.scene_setup(num_views=10, width=6048, height=4032)
    ids = [0] + list(setup.pairs[0][:9])
    dev = torch.device("cuda", 0)
    imgs = [scene.render_torch(setup, i, dev) for i in ids]
    torch.cuda.synchronize()
    return setup, ids, imgs


def test_eth3d_native_size_ncc_sample(eth3d_views):
    setup, ids, imgs = eth3d_views
    ids, imgs = ids[:3], imgs[:3]
    cams = [setup.camera(i) for i in ids]
    H, W = imgs[0].shape
    assert (W + 3 + 15) // 16 * 16 * (H + 2) >= 1 << 24  # takes the wide path by size
    K = np.array(cams[0].K).reshape(3, 3)
    planes = _random_planes(K, H, W, seed=5)
    with ACMMP(0) as eng:
        eng.set_params(_params())
        eng.set_images_device(cams, [im.data_ptr() for im in imgs])
        prm = eng.params
        g_cost, _, _ = eng.eval_costs(planes)
    host = [im.cpu().numpy() for im in imgs]
    rng = np.random.default_rng(1)
    # pixels everywhere, plus the last rows and columns (largest record indices)
    ys = np.concatenate([rng.integers(0, H, 600), [H - 1] * 20, rng.integers(H - 8, H, 20)])
    xs = np.concatenate([rng.integers(0, W, 600), rng.integers(0, W, 20), [W - 1] * 20])
    ref = np.array([[oracle.ncc(prm, cams[0], cams[v], host[0], host[v], x, y, planes[y, x])
                     for v in range(1, len(ids))] for y, x in zip(ys, xs)], np.float32)
    assert_bit_exact(g_cost[ys, xs], ref, "ncc costs at 6048x4032")
    assert (ref < 2).mean() > 0.05


def test_eth3d_native_size_run_patchmatch(eth3d_views):
    setup, ids, imgs = eth3d_views
    cams = [setup.camera(i) for i in ids]
    H, W = imgs[0].shape
    import time

    with ACMMP(0) as eng:
        eng.set_params(_params(8))
        eng.set_images_device(cams, [im.data_ptr() for im in imgs])
        t0 = time.perf_counter()
        eng.RunPatchMatch()
        dt = time.perf_counter() - t0
        pl, co = eng.plane_hypotheses(), eng.costs()
    assert pl.shape == (H, W, 4) and co.shape == (H, W)
    assert np.isfinite(pl[..., 3]).all()
    fin = co[np.isfinite(co)]  # NaN: no view selected (the reference's 0/0)
    print(f"cfg5 6048x4032, 9 sources, 8 iterations: {dt:.2f} s incl. D2H "
          f"({W * H / dt / 1e6:.1f} Mpix/s), finite {fin.size / co.size:.3f}, "
          f"cost<0.5 {(fin < 0.5).mean():.3f}")
    assert fin.min() >= 0 and fin.max() <= 2.0
    assert (co < 0.5).mean() > 0.7
    # depth against the analytic scene where the match is confident
    gt = scene.render_torch(setup, ids[0], imgs[0].device, with_depth=True)[1].cpu().numpy()
    ok = np.isfinite(co) & (co < 0.3) & (gt > 0)
    rel = np.abs(pl[..., 3] - gt)[ok] / gt[ok]
    assert ok.mean() > 0.1 and np.median(rel) < 0.01
