"""Planar-prior construction on the GPU vs the CPU oracle:
support points, plane fit + raster + range check, and the full
ProcessProblem planar block followed by the second RunPatchMatch
(src/acmmp_definitions.cpp:301-379), all bit-exact (NaN == NaN)."""
import numpy as np
import pytest

import oracle
from acmmp_amd import ACMMP, default_params, scene
from parity_util import assert_bit_exact

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def first_pass():
    sc = scene.make_scene(num_views=6, width=160, height=120)
    cams, imgs = sc.problem(0, 5)
    p = default_params()
    p.max_iterations = 3
    eng = ACMMP(0)
    eng.set_params(p)
    eng.set_images(cams, imgs)
    eng.RunPatchMatch()
    yield eng, cams, imgs, eng.params
    eng.close()


def test_support_points_match_oracle(first_pass):
    eng, *_ = first_pass
    costs = eng.costs()
    pts = eng.GetSupportPoints()
    ref = oracle.support_points(costs)
    assert pts.shape[0] > 50
    np.testing.assert_array_equal(pts, ref)


def test_prior_planes_raster_and_range_match_oracle(first_pass):
    eng, cams, imgs, prm = first_pass
    planes_now = eng.plane_hypotheses()
    pts = eng.GetSupportPoints()
    tris = eng.DelaunayTriangulation(pts)
    assert tris.shape[0] > 1.5 * pts.shape[0]
    planes, mask = eng.build_planar_prior(tris)
    ref_planes, ref_mask, _ = oracle.planar_prior(cams[0], planes_now[..., 3], prm.depth_min, prm.depth_max, tris)
    assert_bit_exact(planes, ref_planes, "prior plane params")
    np.testing.assert_array_equal(mask, ref_mask)
    assert (mask > 0).mean() > 0.5


def test_raster_overlaps_later_triangle_wins(first_pass):
    """Overlapping triangles (not Delaunay output): the sequential overwrite of
    the reference equals the GPU's atomicMax of labels."""
    eng, cams, imgs, prm = first_pass
    planes_now = eng.plane_hypotheses()
    W, H = eng.size
    rng = np.random.default_rng(7)
    tris = rng.integers(0, [W, H, W, H, W, H], size=(60, 6)).astype(np.int32)
    tris[5] = [0, 0, W - 1, 0, 0, H - 1]           # large triangle, long edges
    tris[6] = [3, 3, 3, 3, 9, 9]                   # degenerate (repeated corner)
    tris[7] = [-1, 0, 5, 5, 6, 0]                  # outside the image: dropped
    planes, mask = eng.build_planar_prior(tris)
    inside = ((tris[:, 0::2] >= 0) & (tris[:, 0::2] < W) & (tris[:, 1::2] >= 0) & (tris[:, 1::2] < H)).all(1)
    ref_planes, ref_mask, _ = oracle.planar_prior(cams[0], planes_now[..., 3], prm.depth_min, prm.depth_max,
                                                  tris[inside])
    assert_bit_exact(planes, ref_planes, "prior plane params")
    np.testing.assert_array_equal(mask, ref_mask)


def test_planar_pass_end_to_end(first_pass):
    """Second RunPatchMatch with the prior built on the device vs the oracle
    fed the oracle-built prior of the same triangles."""
    sc = scene.make_scene(num_views=6, width=160, height=120)
    cams, imgs = sc.problem(2, 5)
    p = default_params()
    p.max_iterations = 2
    with ACMMP(0) as eng:
        eng.set_params(p)
        eng.set_images(cams, imgs)
        prm0 = eng.params
        eng.RunPatchMatch()
        first_planes, first_costs = eng.plane_hypotheses(), eng.costs()
        pts = eng.GetSupportPoints()
        tris = eng.DelaunayTriangulation(pts)
        npts, ntri = eng.prepare_planar_prior()
        assert (npts, ntri) == (pts.shape[0], tris.shape[0])
        prm1 = eng.params
        eng.RunPatchMatch()
        second = (eng.plane_hypotheses(), eng.costs(), eng.selected_views())
    assert prm1.planar_prior == 1
    ref0 = oracle.run_patchmatch(prm0, cams, imgs)
    assert_bit_exact(first_planes, ref0["planes"], "first run planes")
    _, mask, prior = oracle.planar_prior(cams[0], ref0["planes"][..., 3], prm1.depth_min, prm1.depth_max, tris)
    ref1 = oracle.run_patchmatch(prm1, cams, imgs, planes=ref0["planes"], costs=ref0["costs"],
                                 prior_planes=prior, masks=mask)
    assert_bit_exact(second[0], ref1["planes"], "planar pass planes")
    assert_bit_exact(second[1], ref1["costs"], "planar pass costs")
    assert_bit_exact(second[2], ref1["selected_views"], "planar pass selected views")


@pytest.mark.timeout(900)
def test_cfg3_full_size_planar_pass():
    """cfg3 (BASELINE configs[2]) at its full size: one 1600x1200 reference
    view with 9 sources, 8 iterations — photometric run, planar prior built
    on the device (support points, Delaunay, raster, plane fit, range check),
    planar-prior run — bit-exact against the oracle at every stage."""
    import torch
    dev = torch.device("cuda", 0)
    setup = scene.scene_setup(num_views=10, width=1600, height=1200)
    ids = [0] + setup.pairs[0][:9]
    timgs = [scene.render_torch(setup, i, dev) for i in ids]
    imgs = [t.cpu().numpy() for t in timgs]
    cams = [setup.camera(i) for i in ids]
    p = default_params()
    p.max_iterations = 8
    with ACMMP(0) as eng:
        eng.set_params(p)
        eng.set_images(cams, imgs)
        prm0 = eng.params
        eng.RunPatchMatch()
        first_planes, first_costs = eng.plane_hypotheses(), eng.costs()
        pts = eng.GetSupportPoints()
        tris = eng.DelaunayTriangulation(pts)
        npts, ntri = eng.prepare_planar_prior()
        assert (npts, ntri) == (pts.shape[0], tris.shape[0]) and ntri > 10000
        prm1 = eng.params
        eng.RunPatchMatch()
        second = (eng.plane_hypotheses(), eng.costs(), eng.selected_views())
    ref0 = oracle.run_patchmatch(prm0, cams, imgs)
    assert_bit_exact(first_planes, ref0["planes"], "cfg3 photometric planes")
    assert_bit_exact(first_costs, ref0["costs"], "cfg3 photometric costs")
    np.testing.assert_array_equal(pts, oracle.support_points(ref0["costs"]))
    _, mask, prior = oracle.planar_prior(cams[0], ref0["planes"][..., 3], prm1.depth_min, prm1.depth_max, tris)
    ref1 = oracle.run_patchmatch(prm1, cams, imgs, planes=ref0["planes"], costs=ref0["costs"],
                                 prior_planes=prior, masks=mask)
    assert_bit_exact(second[0], ref1["planes"], "cfg3 planar pass planes")
    assert_bit_exact(second[1], ref1["costs"], "cfg3 planar pass costs")
    assert_bit_exact(second[2], ref1["selected_views"], "cfg3 planar pass selected views")
