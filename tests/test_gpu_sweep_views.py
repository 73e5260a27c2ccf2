"""End-to-end RunPatchMatch parity across source-view counts: every array
bucket of the templated kernels (NS = 4, 9, 16, 20, 32) through the sweep's
packed refinement (refine_costs_compact: items of several lanes per pass,
ceil(5 c_j / active lanes) passes per view), at sizes whose last waves are
partial (odd widths/heights), photometric and geometric. Bit-exact against
the oracle (src/ACMMP.cu:707-784 for the refinement, :1080-1173 for the
accept logic it feeds).
"""
import numpy as np
import pytest

import oracle
from acmmp_amd import ACMMP, default_params, scene
from parity_util import assert_bit_exact

pytestmark = pytest.mark.gpu


def _params(iters, **kw):
    p = default_params()
    p.max_iterations = iters
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def _run(p, cams, imgs, depths=None):
    with ACMMP(0) as eng:
        eng.set_params(p)
        eng.set_images(cams, imgs)
        if depths is not None:
            eng.set_depth_maps(depths)
        prm = eng.params
        eng.RunPatchMatch()
        return prm, eng.plane_hypotheses(), eng.costs(), eng.selected_views()


def _check(prm, cams, imgs, got, what, depths=None):
    if depths is None:
        ref = oracle.run_patchmatch(prm, cams, imgs)
    else:
        ref = oracle.run_patchmatch(prm, cams, imgs, depths=depths)
    pl, co, sv = got
    assert_bit_exact(pl, ref["planes"], f"planes ({what})")
    assert_bit_exact(co, ref["costs"], f"costs ({what})")
    assert_bit_exact(sv, ref["selected_views"], f"selected views ({what})")


@pytest.mark.parametrize("nsrc,W,H", [(1, 61, 45), (2, 64, 48), (5, 53, 41), (12, 48, 37), (20, 45, 33),
                                      (31, 40, 29)])
def test_sweep_parity_across_view_counts(nsrc, W, H):
    sc = scene.make_scene(num_views=nsrc + 1, width=W, height=H, arc_deg=4.0)
    cams, imgs = sc.problem(0, nsrc)
    prm, pl, co, sv = _run(_params(2), cams, imgs)
    _check(prm, cams, imgs, (pl, co, sv), f"nsrc={nsrc}")
    # the refinement really runs with several sampled views per pixel
    if nsrc >= 5:
        counts = np.vectorize(lambda m: bin(int(m)).count("1"))(sv)
        assert counts.max() >= 2


@pytest.mark.parametrize("nsrc", [12, 20, 25])
def test_geometric_sweep_many_views(nsrc):
    """A photometric pass, then a geometric pass from its state that reads
    the source views' ground-truth depth maps (geom_cost on every sampled
    view of every packed refinement item)."""
    sc = scene.make_scene(num_views=nsrc + 1, width=56, height=42, arc_deg=4.0)
    cams, imgs = sc.problem(0, nsrc)
    ids = [0] + sc.pairs[0][:nsrc]
    depths = [sc.views[i].depth for i in ids]
    _, pl0, co0, _ = _run(_params(2), cams, imgs)
    p = _params(2, geom_consistency=1)
    with ACMMP(0) as eng:
        eng.set_params(p)
        eng.set_images(cams, imgs)
        eng.set_depth_maps(depths)
        eng.set_plane_hypotheses(pl0, co0)
        prm = eng.params
        eng.RunPatchMatch()
        pl, co, sv = eng.plane_hypotheses(), eng.costs(), eng.selected_views()
    ref = oracle.run_patchmatch(prm, cams, imgs, depths=depths, planes=pl0, costs=co0)
    assert_bit_exact(pl, ref["planes"], f"geom planes nsrc={nsrc}")
    assert_bit_exact(co, ref["costs"], f"geom costs nsrc={nsrc}")
    assert_bit_exact(sv, ref["selected_views"], f"geom selected views nsrc={nsrc}")
