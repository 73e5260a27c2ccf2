"""Texel storage of the gather kernels (acmmp_kernels.hip, TX template bits):
u8 quads (4 B per bilinear footprint) when every view is integer-valued in
[0, 255], fp32 row pairs otherwise. The choice changes the memory format
only: both must be bit-identical to the oracle, and the automatic choice must
fall back to fp32 for any view that u8 cannot hold exactly (fractional
values, out-of-range values, -0.0, NaN).
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


def _run(cams, imgs, iters=2):
    with ACMMP(0) as eng:
        eng.set_params(_params(iters))
        eng.set_images(cams, imgs)
        bits = eng.texel_bits()
        prm = eng.params
        eng.RunPatchMatch()
        return bits, prm, eng.plane_hypotheses(), eng.costs(), eng.selected_views()


def _check(prm, cams, imgs, pl, co, sv, what):
    ref = oracle.run_patchmatch(prm, cams, imgs)
    assert_bit_exact(pl, ref["planes"], f"planes ({what})")
    assert_bit_exact(co, ref["costs"], f"costs ({what})")
    assert_bit_exact(sv, ref["selected_views"], f"selected views ({what})")


@pytest.fixture(scope="module")
def prob():
    sc = scene.make_scene(num_views=6, width=112, height=84)
    return sc.problem(0, 5)


@pytest.mark.parametrize("force_f32", [False, True])
def test_both_texel_forms_match_oracle(prob, monkeypatch, force_f32):
    cams, imgs = prob
    if force_f32:
        monkeypatch.setenv("ACMMP_TEXEL_F32", "1")
    bits, prm, pl, co, sv = _run(cams, imgs)
    assert bits == (32 if force_f32 else 8)
    _check(prm, cams, imgs, pl, co, sv, f"{bits}-bit texels")


@pytest.mark.parametrize("kind", ["fraction", "above_255", "negative_zero", "nan"])
def test_non_u8_views_fall_back_to_f32(prob, kind):
    cams, imgs = prob
    imgs = [im.copy() for im in imgs]
    tgt = imgs[3]  # one source view decides for the whole problem
    if kind == "fraction":
        tgt[10:20, 10:20] += 0.25
    elif kind == "above_255":
        tgt[5, 7] = 256.0
    elif kind == "negative_zero":
        tgt[tgt == 0] = 0.0
        tgt[0, 0] = -0.0
    else:
        tgt[40, 50] = np.nan
    bits, prm, pl, co, sv = _run(cams, imgs)
    assert bits == 32
    _check(prm, cams, imgs, pl, co, sv, kind)


def test_u8_quads_at_image_borders():
    """Clamp-to-edge through the quad records: tiny odd-sized views whose
    patches mostly project outside the source image."""
    sc = scene.make_scene(num_views=4, width=21, height=17)
    cams, imgs = sc.problem(0, 3)
    bits, prm, pl, co, sv = _run(cams, imgs, iters=3)
    assert bits == 8
    _check(prm, cams, imgs, pl, co, sv, "u8 borders")
