"""Texel storage of the gather kernels (acmmp_kernels.hip, TX template bits),
the most compact form every view fits: u8 quads (4 B per bilinear footprint)
when every view is integer-valued in [0, 255], else f16 difference quads
(8 B) when every stored value (texels and the fp32 row differences) is exact
in f16, else fp32 row pairs (16 B). ACMMP_TEXEL=u8|h16|f32 restricts the
attempt to one form. The choice changes the memory format only: every form must
be bit-identical to the oracle, and the automatic choice must fall back to
fp32 for any view the compact form cannot hold exactly.
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


@pytest.mark.parametrize("form,bits", [(None, 8), ("h16", 16), ("u8", 8), ("f32", 32)])
def test_every_texel_form_matches_oracle(prob, monkeypatch, form, bits):
    cams, imgs = prob
    if form is not None:
        monkeypatch.setenv("ACMMP_TEXEL", form)
    got, prm, pl, co, sv = _run(cams, imgs)
    assert got == bits
    _check(prm, cams, imgs, pl, co, sv, f"{bits}-bit texels")


def test_texel_f32_switch(prob, monkeypatch):
    cams, imgs = prob
    monkeypatch.setenv("ACMMP_TEXEL_F32", "1")
    assert _run(cams, imgs)[0] == 32


def _perturb(imgs, kind):
    imgs = [im.copy() for im in imgs]
    tgt = imgs[3]  # one source view decides for the whole problem
    if kind == "quarter":          # exact in f16, not u8
        tgt[10:20, 10:20] += 0.25
    elif kind == "third":          # exact in neither
        tgt[10:20, 10:20] += np.float32(1.0 / 3.0)
    elif kind == "above_255":      # exact in f16, not u8
        tgt[5, 7] = 256.0
    elif kind == "beyond_f16":     # above the f16 range
        tgt[5, 7] = 70000.0
    elif kind == "odd_4097":       # an integer f16 cannot hold (13 bits)
        tgt[5, 7] = 4097.0
    elif kind == "negative_zero":  # f16 holds -0.0, u8 does not
        tgt[tgt == 0] = 0.0
        tgt[0, 0] = -0.0
    elif kind == "inf":
        tgt[30, 31] = np.inf
    else:
        tgt[40, 50] = np.nan
    return imgs


# (perturbation, bits when h16 is tried, bits when u8 is tried)
CASES = [("quarter", 16, 32), ("third", 32, 32), ("above_255", 16, 32), ("beyond_f16", 32, 32),
         ("odd_4097", 32, 32), ("negative_zero", 16, 32), ("inf", 32, 32), ("nan", 32, 32)]


@pytest.mark.parametrize("kind,bits_h16,bits_u8", CASES)
@pytest.mark.parametrize("form", [None, "h16", "u8"])
def test_views_the_compact_form_cannot_hold(prob, monkeypatch, kind, bits_h16, bits_u8, form):
    cams, imgs = prob
    imgs = _perturb(imgs, kind)
    if form is not None:
        monkeypatch.setenv("ACMMP_TEXEL", form)
    bits, prm, pl, co, sv = _run(cams, imgs)
    # the default chain tries u8, then h16
    want = {"h16": bits_h16, "u8": bits_u8, None: bits_u8 if bits_u8 != 32 else bits_h16}[form]
    assert bits == want
    _check(prm, cams, imgs, pl, co, sv, f"{kind} ({bits}-bit)")


@pytest.mark.parametrize("form,bits", [("h16", 16), ("u8", 8)])
def test_quads_at_image_borders(monkeypatch, form, bits):
    """Clamp-to-edge through the quad records: tiny odd-sized views whose
    patches mostly project outside the source image."""
    monkeypatch.setenv("ACMMP_TEXEL", form)
    sc = scene.make_scene(num_views=4, width=21, height=17)
    cams, imgs = sc.problem(0, 3)
    got, prm, pl, co, sv = _run(cams, imgs, iters=3)
    assert got == bits
    _check(prm, cams, imgs, pl, co, sv, f"{form} borders")


@pytest.mark.parametrize("mixed", [None, "h16", "f32"])
def test_textures_match_oracle(prob, mixed):
    """acmmp_texture_create + acmmp_set_images_textures (records built once,
    borrowed by the engine: the drivers' and bench's path). mixed: one view
    holds fractional texels, so its texture falls back from u8 quads to f16
    difference quads (quarter steps, exact in f16: the texture's records are
    re-sized for the second form it tries) or to fp32 (thirds), while the
    others are u8 quads; the engine then re-pads the problem in the common
    form (the least compact)."""
    import torch
    from acmmp_amd.engine import Texture
    cams, imgs = prob
    imgs = [np.asarray(im, np.float32).copy() for im in imgs]
    if mixed == "h16":
        imgs[3] = imgs[3] + 0.25
    elif mixed == "f32":
        imgs[3] = imgs[3] + np.float32(1.0 / 3.0)
    odd = {None: 8, "h16": 16, "f32": 32}[mixed]
    dev = torch.device("cuda", 0)
    timgs = [torch.from_numpy(im).to(dev) for im in imgs]
    torch.cuda.synchronize()
    tex = [Texture.of(t, 0) for t in timgs]
    assert [t.bits for t in tex] == [odd if i == 3 else 8 for i in range(len(tex))]
    with ACMMP(0) as eng:
        eng.set_params(_params(2))
        eng.set_images_textures(cams, tex)
        assert eng.texel_bits() == (32 if mixed == "f32" else 16 if mixed else 8)
        prm = eng.params
        eng.RunPatchMatch()
        pl, co, sv = eng.plane_hypotheses(), eng.costs(), eng.selected_views()
    _check(prm, cams, imgs, pl, co, sv, f"textures, {mixed or 'u8'}")
