"""GPU (libacmmp_amd.so, gfx950) vs CPU oracle parity — the parity tiers of
SURVEY §8c, all held to BIT-EXACTNESS (NaN == NaN):

  T1  kernel level: NCC cost vectors, init cost + selected views, geometric
      consistency cost, for fixed random hypothesis sets;
  T2  one checkerboard iteration from the same init;
  T3  end-to-end RunPatchMatch (init, N iterations, depth/normal, filter).

Sizes are small so the oracle finishes in seconds; edge cases follow the
reference's boundary logic (borders, odd sizes, the skipped last row of the
checkerboard grid, textureless input -> NaN costs, 1 and 20 source views).
"""
import numpy as np
import pytest

import oracle
from acmmp_amd import ACMMP, default_params, make_camera, scene
from parity_util import assert_bit_exact, rel_depth_agreement

pytestmark = pytest.mark.gpu


def _params(iters=2, **kw):
    p = default_params()
    p.max_iterations = iters
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def _random_planes(cams, H, W, seed):
    """Camera-frame planes (n, d) with n facing the camera, depth in range."""
    rng = np.random.default_rng(seed)
    K = np.array(cams[0].K).reshape(3, 3)
    n = rng.normal(size=(H, W, 3))
    n[..., 2] = -np.abs(n[..., 2]) - 0.5
    n /= np.linalg.norm(n, axis=-1, keepdims=True)
    depth = rng.uniform(400, 800, size=(H, W))
    ys, xs = np.mgrid[0:H, 0:W]
    X = np.stack([depth * (xs - K[0, 2]) / K[0, 0], depth * (ys - K[1, 2]) / K[1, 1], depth], -1)
    d = -(n * X).sum(-1)
    return np.concatenate([n, d[..., None]], -1).astype(np.float32)


@pytest.fixture(scope="module")
def small_scene():
    return scene.make_scene(num_views=10, width=128, height=96)


def _gpu_run(p, cams, imgs, depths=None, state=None):
    with ACMMP(0) as eng:
        eng.set_params(p)
        eng.set_images(cams, imgs)
        if depths is not None:
            eng.set_depth_maps(depths)
        if state is not None:
            eng.set_plane_hypotheses(*state)
        prm = eng.params
        eng.RunPatchMatch()
        return prm, eng.plane_hypotheses(), eng.costs(), eng.selected_views()


@pytest.mark.parametrize("nsrc", [1, 4, 9, 20])
def test_t1_cost_vectors(nsrc):
    sc = scene.make_scene(num_views=nsrc + 1, width=80, height=60, arc_deg=4.0)
    cams, imgs = sc.problem(0, nsrc)
    H, W = imgs[0].shape
    planes = _random_planes(cams, H, W, seed=nsrc)
    p = _params()
    with ACMMP(0) as eng:
        eng.set_params(p)
        eng.set_images(cams, imgs)
        prm = eng.params
        g_cost, g_init, g_views = eng.eval_costs(planes)
    r_cost, r_init, r_views = oracle.eval_costs(prm, cams, imgs, planes)
    assert_bit_exact(g_cost, r_cost, "ncc cost vectors")
    assert_bit_exact(g_init, r_init, "initial cost")
    assert_bit_exact(g_views, r_views, "initial selected views")
    assert (r_cost < 2).mean() > 0.05  # the hypotheses do exercise the full NCC


def test_t1_geom_cost(small_scene):
    cams, imgs = small_scene.problem(0, 4)
    ids = [0] + small_scene.pairs[0][:4]
    depths = [small_scene.views[i].depth for i in ids]
    H, W = imgs[0].shape
    planes = _random_planes(cams, H, W, seed=3)
    p = _params(geom_consistency=1)
    with ACMMP(0) as eng:
        eng.set_params(p)
        eng.set_images(cams, imgs)
        eng.set_depth_maps(depths)
        prm = eng.params
        g = eng.eval_geom_costs(planes)
    r = oracle.eval_geom_costs(prm, cams, imgs, depths, planes)
    assert_bit_exact(g, r, "geometric consistency cost")


def test_t1_geom_cost_extreme_values(small_scene):
    """The geometric cost at the edges of float arithmetic: source depths 0,
    +-inf, NaN, negative, subnormal, tiny and huge, and hypotheses whose depth
    is 0, NaN, tiny or huge, against the oracle's IEEE divisions (the
    quotient windows of DESIGN §5's Markstein variant lie at 2^-60 / 2^60)."""
    cams, imgs = small_scene.problem(0, 4)
    ids = [0] + small_scene.pairs[0][:4]
    H, W = imgs[0].shape
    rng = np.random.default_rng(11)
    special = np.array([0.0, np.inf, -np.inf, np.nan, -500.0, 1e-40, 1e-30, 2.0 ** -61, 2.0 ** -59,
                        2.0 ** 59, 2.0 ** 61, 1e30, 3e38], np.float32)
    depths = []
    for i in ids:
        d = small_scene.views[i].depth.astype(np.float32).copy()
        m = rng.random(d.shape) < 0.3
        d[m] = rng.choice(special, size=int(m.sum()))
        depths.append(d)
    planes = _random_planes(cams, H, W, seed=5)
    scale = np.array([1.0, 0.0, np.nan, 1e-30, 2.0 ** -62, 2.0 ** 62, 1e30, -1.0], np.float32)
    m = rng.random((H, W)) < 0.3
    planes[..., 3][m] *= rng.choice(scale, size=int(m.sum()))
    p = _params(geom_consistency=1)
    with ACMMP(0) as eng:
        eng.set_params(p)
        eng.set_images(cams, imgs)
        eng.set_depth_maps(depths)
        prm = eng.params
        g = eng.eval_geom_costs(planes)
    r = oracle.eval_geom_costs(prm, cams, imgs, depths, planes)
    assert_bit_exact(g, r, "geometric consistency cost, extreme values")
    assert np.isfinite(r).mean() > 0.5 and (r < 3.0).mean() > 0.05


@pytest.mark.parametrize("iters", [0, 1])
def test_t2_init_and_one_sweep(small_scene, iters):
    cams, imgs = small_scene.problem(0, 9)
    prm, pl, co, sv = _gpu_run(_params(iters), cams, imgs)
    ref = oracle.run_patchmatch(prm, cams, imgs)
    assert_bit_exact(pl, ref["planes"], f"planes after {iters} iterations")
    assert_bit_exact(co, ref["costs"], "costs")
    assert_bit_exact(sv, ref["selected_views"], "selected views")


@pytest.mark.parametrize("sigma_spatial,sigma_color,top_k", [(3.5, 7.0, 2), (6.0, 1.5, 6)])
def test_t3_nondefault_patch_parameters(small_scene, sigma_spatial, sigma_color, top_k):
    """PatchMatchParams' bilateral sigmas (the patch weights, src/ACMMP.cu:
    360-380) and top_k (the initial cost's best-k mean and selected views,
    :434-471) at values other than the defaults: GPU and oracle bit-exact."""
    cams, imgs = small_scene.problem(0, 9)
    p = _params(2, sigma_spatial=sigma_spatial, sigma_color=sigma_color, top_k=top_k)
    prm, pl, co, sv = _gpu_run(p, cams, imgs)
    assert (prm.sigma_spatial, prm.sigma_color, prm.top_k) == (sigma_spatial, sigma_color, top_k)
    ref = oracle.run_patchmatch(prm, cams, imgs)
    assert_bit_exact(pl, ref["planes"], "planes")
    assert_bit_exact(co, ref["costs"], "costs")
    assert_bit_exact(sv, ref["selected_views"], "selected views")
    _, pl_default, _, _ = _gpu_run(_params(2), cams, imgs)
    assert not np.array_equal(pl, pl_default)  # the parameters reach the kernels


def test_t3_photometric_cfg1_shape():
    """cfg1: 5 views at 400x300, 3 iterations, photometric (the reference's
    CPU-sized configuration)."""
    sc = scene.make_scene(num_views=5, width=400, height=300)
    cams, imgs = sc.problem(2, 4)
    prm, pl, co, sv = _gpu_run(_params(3), cams, imgs)
    ref = oracle.run_patchmatch(prm, cams, imgs)
    assert_bit_exact(pl, ref["planes"], "planes")
    assert_bit_exact(co, ref["costs"], "costs")
    assert_bit_exact(sv, ref["selected_views"], "selected views")
    assert rel_depth_agreement(pl, ref["planes"], ref["costs"]) == 1.0
    # and the reconstruction is meaningful against the analytic ground truth
    gt = sc.views[2].depth
    ok = (gt > 0) & (co < 0.3)
    rel = np.abs(pl[..., 3] - gt) / np.maximum(gt, 1)
    assert np.median(rel[ok]) < 0.005


def test_t3_texture_filter8_emulation():
    """texture_filter8: the CUDA texture unit's 8-bit bilinear fractions
    (cudaFilterModeLinear, src/ACMMP.cpp:659 / src/ACMMP.cu:394) instead of
    pin A4's fp32 ones — GPU and oracle bit-exact in this mode too, and the
    result still reconstructs the analytic depth (the mode exists to measure
    pin A4's effect: tools/fidelity_study.py)."""
    sc = scene.make_scene(num_views=5, width=400, height=300)
    cams, imgs = sc.problem(2, 4)
    prm, pl, co, sv = _gpu_run(_params(3, texture_filter8=1), cams, imgs)
    assert prm.texture_filter8 == 1
    ref = oracle.run_patchmatch(prm, cams, imgs)
    assert_bit_exact(pl, ref["planes"], "planes")
    assert_bit_exact(co, ref["costs"], "costs")
    assert_bit_exact(sv, ref["selected_views"], "selected views")
    gt = sc.views[2].depth
    ok = (gt > 0) & (co < 0.3)
    rel = np.abs(pl[..., 3] - gt) / np.maximum(gt, 1)
    assert np.median(rel[ok]) < 0.005
    # the mode changes results (it is not a no-op)
    _, pl32, _, _ = _gpu_run(_params(3), cams, imgs)
    assert not np.array_equal(pl32, pl)


def test_t3_geometric_pass(small_scene):
    """Photometric pass over 4 views, then a geometric pass (Jacobi order)
    that reads their depth maps, as ProcessProblem does between passes."""
    V, nsrc = 4, 3
    outs = {}
    for ref in range(V):
        ids = [ref] + [j for j in small_scene.pairs[ref] if j < V][:nsrc]
        cams = [small_scene.views[i].camera for i in ids]
        imgs = [small_scene.views[i].image for i in ids]
        prm, pl, co, sv = _gpu_run(_params(2), cams, imgs)
        outs[ref] = (pl, co)
    for ref in range(V):
        ids = [ref] + [j for j in small_scene.pairs[ref] if j < V][:nsrc]
        cams = [small_scene.views[i].camera for i in ids]
        imgs = [small_scene.views[i].image for i in ids]
        depths = [outs[i][0][..., 3] for i in ids]
        state = (outs[ref][0], outs[ref][1])
        p = _params(2)
        p.geom_consistency = 1
        prm, pl, co, sv = _gpu_run(p, cams, imgs, depths=depths, state=state)
        ref_out = oracle.run_patchmatch(prm, cams, imgs, depths=depths, planes=state[0], costs=state[1])
        assert_bit_exact(pl, ref_out["planes"], f"geom planes view {ref}")
        assert_bit_exact(co, ref_out["costs"], f"geom costs view {ref}")


@pytest.mark.parametrize("W,H", [(37, 33), (40, 65), (9, 7), (64, 31)])
def test_t3_odd_sizes_and_skipped_row(W, H):
    """Odd sizes; H=33/65 hit the reference grid's skipped last row."""
    sc = scene.make_scene(num_views=4, width=W, height=H)
    cams, imgs = sc.problem(1, 3)
    prm, pl, co, sv = _gpu_run(_params(2), cams, imgs)
    ref = oracle.run_patchmatch(prm, cams, imgs)
    assert_bit_exact(pl, ref["planes"], "planes")
    assert_bit_exact(co, ref["costs"], "costs")
    if H in (33, 65):
        assert oracle.checkerboard_rows(H) == H - 1


@pytest.mark.parametrize("level,nan_share", [(100.0, 1.0), (77.0, None)])
def test_t3_textureless(level, nan_share):
    """Constant images. Every patch has the same weighted moments, so whether
    an NCC is cost_max depends only on the sign and size of the contracted
    variance residual fma(sum_rr, inv, -m*m) (pin P3) against kMinVar:
    - level 100: residual < 1e-5 -> every NCC 2, all sampling probabilities 0,
      weight norm 0 -> NaN costs (src/ACMMP.cu:1034, :1075, :1091);
    - level 77: residual > 1e-5 and var_ref == var_src == covar -> cost 0
      wherever the centre maps into the source image, 2 (cost_max) for a view
      where it does not (a border pixel's weighted mean can then be above 0),
      NaN where no view was sampled.
    Both sides must agree bit-exactly either way."""
    W, H = 48, 40
    cams = []
    K = np.array([[100.0, 0, 24], [0, 100.0, 20], [0, 0, 1]])
    for i in range(3):
        R = np.eye(3)
        t = np.array([-5.0 * i, 0, 0])
        cams.append(make_camera(K, R, t, W, H, 300, 800))
    imgs = [np.full((H, W), level, np.float32) for _ in range(3)]
    prm, pl, co, sv = _gpu_run(_params(2), cams, imgs)
    ref = oracle.run_patchmatch(prm, cams, imgs)
    nan = np.isnan(ref["costs"])
    if nan_share is not None:
        assert nan.mean() == nan_share
    else:
        fin = ref["costs"][~nan]
        assert 0 < nan.mean() < 0.1 and np.all((fin >= 0.0) & (fin <= 2.0)) and (fin == 0.0).mean() > 0.95
    assert_bit_exact(pl, ref["planes"], "planes")
    assert_bit_exact(co, ref["costs"], "costs")


def test_rng_stream_reseeds_second_run(small_scene):
    """A second RunPatchMatch on the same engine draws a new stream (the
    reference re-seeds with clock64()); parity holds for both runs."""
    cams, imgs = small_scene.problem(3, 4)
    with ACMMP(0) as eng:
        eng.set_params(_params(1))
        eng.set_images(cams, imgs)
        prm0 = eng.params
        eng.RunPatchMatch()
        a = eng.plane_hypotheses()
        prm1 = eng.params
        eng.RunPatchMatch()
        b = eng.plane_hypotheses()
    assert prm1.rng_stream == prm0.rng_stream + 1
    assert not np.array_equal(a, b)
    assert_bit_exact(b, oracle.run_patchmatch(prm1, cams, imgs)["planes"], "second run")


def test_fast_reciprocal_is_exact_on_this_device():
    """The sweep's fast 1/z (v_rcp_f32 + one fma Newton step) must equal the
    IEEE division for EVERY float32 in its exponent window — the exhaustive
    proof that makes the fast path bit-identical to the pinned semantics."""
    import ctypes as C
    from acmmp_amd import _abi
    m, n = C.c_uint64(), C.c_uint64()
    assert _abi.load_library().acmmp_selftest_reciprocal(0, C.byref(m), C.byref(n)) == 0
    assert n.value == 2 * 250 * (1 << 23)  # both signs, exponents -125..124, all mantissas
    assert m.value == 0


def _cam_planes_from_truth(view, cam):
    """Camera-frame plane hypotheses (n, d) from the analytic ground truth."""
    H, W = view.depth.shape
    K = np.array(cam.K).reshape(3, 3)
    R = np.array(cam.R).reshape(3, 3)
    n = view.normal @ R.T  # world -> camera
    flip = n[..., 2] > 0
    n[flip] *= -1
    ys, xs = np.mgrid[0:H, 0:W]
    z = np.where(view.depth > 0, view.depth, 600.0)
    X = np.stack([z * (xs - K[0, 2]) / K[0, 0], z * (ys - K[1, 2]) / K[1, 1], z], -1)
    d = -(n * X).sum(-1)
    return np.concatenate([n, d[..., None]], -1).astype(np.float32)


def test_planar_prior_second_run(small_scene):
    """ProcessProblem's planar-prior flow (src/acmmp_definitions.cpp:306-379):
    run, install triangle planes + label mask, SetPlanarPriorParams, run again
    (random re-init + restricted propagation/refinement, src/ACMMP.cu:1095-1147,
    :722-775)."""
    cams, imgs = small_scene.problem(1, 4)
    H, W = imgs[0].shape
    planes_gt = _cam_planes_from_truth(small_scene.views[1], cams[0])
    # 12 x 12 px "triangles": one plane per cell, taken from the cell centre;
    # a band of unlabelled pixels keeps the mask > 0 / == 0 paths mixed
    lab = (np.arange(H)[:, None] // 12) * ((W + 11) // 12) + (np.arange(W)[None, :] // 12)
    mask = (lab + 1).astype(np.uint32)
    mask[:, W // 2 - 3:W // 2 + 3] = 0
    nlab = int(lab.max()) + 1
    plane_params = np.zeros((nlab, 4), np.float32)
    for l in range(nlab):
        yy, xx = np.argwhere(lab == l)[len(np.argwhere(lab == l)) // 2]
        plane_params[l] = planes_gt[yy, xx]
    with ACMMP(0) as eng:
        eng.set_params(_params(2))
        eng.set_images(cams, imgs)
        prm0 = eng.params
        eng.RunPatchMatch()
        first = (eng.plane_hypotheses(), eng.costs())
        eng.SetPlanarPriorParams()
        eng.CudaPlanarPriorInitialization(plane_params, mask)
        prm1 = eng.params
        eng.RunPatchMatch()
        second = (eng.plane_hypotheses(), eng.costs(), eng.selected_views())
    ref0 = oracle.run_patchmatch(prm0, cams, imgs)
    assert_bit_exact(first[0], ref0["planes"], "first run planes")
    per_pixel = np.where(mask[..., None] > 0, plane_params[np.maximum(mask.astype(np.int64) - 1, 0)], 0)
    ref1 = oracle.run_patchmatch(prm1, cams, imgs, planes=ref0["planes"], costs=ref0["costs"],
                                 prior_planes=per_pixel, masks=mask)
    assert prm1.planar_prior == 1 and prm1.rng_stream == 1
    assert_bit_exact(second[0], ref1["planes"], "planar-prior planes")
    assert_bit_exact(second[1], ref1["costs"], "planar-prior costs")
    assert_bit_exact(second[2], ref1["selected_views"], "planar-prior selected views")


def test_planar_prior_init_branch_with_geom(small_scene):
    """The planar-prior INIT branch (src/ACMMP.cu:640-661) is reachable only
    with geom_consistency or hierarchy set; exercise it with geom."""
    cams, imgs = small_scene.problem(2, 3)
    ids = [2] + small_scene.pairs[2][:3]
    depths = [small_scene.views[i].depth for i in ids]
    H, W = imgs[0].shape
    rng = np.random.default_rng(5)
    state_planes = np.concatenate([small_scene.views[2].normal, small_scene.views[2].depth[..., None]], -1)
    state_costs = rng.uniform(0, 0.3, size=(H, W)).astype(np.float32)
    prior = _cam_planes_from_truth(small_scene.views[2], cams[0])
    prior[..., 3] = small_scene.views[2].depth  # the init branch reads .w as a depth (:645)
    mask = (rng.uniform(size=(H, W)) < 0.7).astype(np.uint32)
    pp = prior.reshape(-1, 4)
    labels = (np.arange(H * W) + 1).astype(np.uint32).reshape(H, W) * mask
    p = _params(1)
    p.geom_consistency = 1
    p.planar_prior = 1
    with ACMMP(0) as eng:
        eng.set_params(p)
        eng.set_images(cams, imgs)
        eng.set_depth_maps(depths)
        eng.set_plane_hypotheses(state_planes, state_costs)
        eng.CudaPlanarPriorInitialization(pp, labels)
        prm = eng.params
        eng.RunPatchMatch()
        got = (eng.plane_hypotheses(), eng.costs())
    per_pixel = np.where(mask[..., None] > 0, prior, 0).astype(np.float32)
    ref = oracle.run_patchmatch(prm, cams, imgs, depths=depths, planes=state_planes, costs=state_costs,
                                prior_planes=per_pixel, masks=labels)
    assert_bit_exact(got[0], ref["planes"], "planes")
    assert_bit_exact(got[1], ref["costs"], "costs")


@pytest.mark.parametrize("device_inputs", [False, True])
@pytest.mark.parametrize("same_size", [False, True])
def test_hierarchy_init(small_scene, same_size, device_inputs):
    """Hierarchical init (src/ACMMP.cpp:745-808, src/ACMMP.cu:663-703):
    upsample branch (upscale_normal) from a half-resolution map, and the
    non-upsample branch reached through the reference's rows/cols swap
    (src/ACMMP.cpp:766), plus the hierarchy gate (:1163-1167)."""
    cams, imgs = small_scene.problem(4, 4)
    H, W = imgs[0].shape
    rng = np.random.default_rng(9)
    v = small_scene.views[4]
    if same_size:
        # scaled map "W x H" transposed-equal: the swap test says no upsample
        sh, sw = W, H
        scaled = np.zeros((sh, sw, 4), np.float32)
        flat = np.concatenate([v.normal, v.depth[..., None]], -1).reshape(-1, 4)
        scaled.reshape(-1, 4)[:] = flat
    else:
        sh, sw = H // 2, W // 2
        scaled = np.concatenate([v.normal[::2, ::2], rng.uniform(0, 1, (sh, sw, 1))], -1).astype(np.float32)
    up_depth = np.where(v.depth > 0, v.depth, 700.0).astype(np.float32)
    p = _params(2)
    p.hierarchy = 1
    with ACMMP(0) as eng:
        eng.set_params(p)
        eng.set_images(cams, imgs)
        if device_inputs:  # acmmp_set_hierarchy_inputs_device (the view-parallel driver's path)
            import torch
            ts = torch.from_numpy(scaled).cuda()
            tu = torch.from_numpy(up_depth).cuda()
            torch.cuda.synchronize()
            eng.set_hierarchy_inputs_device(ts.data_ptr(), sw, sh, tu.data_ptr())
        else:
            eng.set_hierarchy_inputs(scaled, up_depth)
        prm = eng.params
        eng.RunPatchMatch()
        got = (eng.plane_hypotheses(), eng.costs())
    assert prm.upsample == (0 if same_size else 1)
    planes_in = np.zeros((H, W, 4), np.float32)
    planes_in[..., 3] = up_depth
    ref = oracle.run_patchmatch(prm, cams, imgs, planes=planes_in, pre_costs=np.zeros((H, W), np.float32),
                                scaled_planes=scaled)
    assert_bit_exact(got[0], ref["planes"], "planes")
    assert_bit_exact(got[1], ref["costs"], "costs")


def test_seeded_init(small_scene):
    """Seeded priors (pSampler -> SetPlanarPrior, src/ACMMP.cu:634-639)."""
    cams, imgs = small_scene.problem(5, 4)
    seed = _cam_planes_from_truth(small_scene.views[5], cams[0])
    with ACMMP(0) as eng:
        eng.set_params(_params(2))
        eng.set_images(cams, imgs)
        eng.SetPlanarPrior(seed)
        prm = eng.params
        eng.RunPatchMatch()
        got = (eng.plane_hypotheses(), eng.costs())
    assert prm.seeded == 1
    ref = oracle.run_patchmatch(prm, cams, imgs, seed_planes=seed)
    assert_bit_exact(got[0], ref["planes"], "planes")
    assert_bit_exact(got[1], ref["costs"], "costs")
