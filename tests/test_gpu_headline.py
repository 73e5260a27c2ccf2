"""Parity of the headline benchmark's exact path (BASELINE configs[1], cfg2):
the `acmmp_amd.resident` schedule bench.py times — two views per launch
(acmmp_run_patchmatch_batch on one stream), images borrowed from HBM
(set_images_device), results exported device-to-device (export_results) and
fed back through set_depth_maps_device / set_plane_hypotheses_device —
N = 10 images per problem, 8 iterations,
photometric then geometric, the pass order of src/main_ACMMP.cpp:123-137 and
one RunPatchMatch per view (src/ACMMP.cu:1378-1456).

Every view's planes (world normal + depth) and costs after each pass are
compared BIT-EXACTLY with the CPU oracle run on the same inputs and the
parameters the engine used:
  * 10 views at 400x300 (every view, both passes);
  * one full 1600x1200 reference view (photometric, then geometric from its
    own photometric state and the GPU's photometric depth maps of the 9
    sources, the inputs both sides share).
"""
import numpy as np
import pytest
import torch

import oracle
from acmmp_amd import default_params, scene
from acmmp_amd.resident import EnginePool, ResidentViews
from parity_util import assert_bit_exact

pytestmark = pytest.mark.gpu


def _cfg2(width, height, views=10, nsrc=9, iters=8, streams=2, mode="batch"):
    dev = torch.device("cuda", 0)
    setup = scene.scene_setup(num_views=views, width=width, height=height)
    images = {k: scene.render_torch(setup, k, dev) for k in range(views)}
    cams = {k: setup.camera(k) for k in range(views)}
    srcs = {k: setup.pairs[k][:nsrc] for k in range(views)}
    torch.cuda.synchronize()
    pool = EnginePool(0, streams, mode=mode)
    rv = ResidentViews(pool, cams, images, srcs, range(views), height, width)
    photo = default_params()
    photo.max_iterations = iters
    geom = default_params()
    geom.max_iterations = iters
    geom.geom_consistency = 1
    rv.photometric_pass(photo)
    torch.cuda.synchronize()
    out = {"photo": (rv.planes.cpu().numpy(), rv.costs.cpu().numpy(), rv.my_depth.cpu().numpy())}
    rv.geometric_pass(geom)
    torch.cuda.synchronize()
    out["geom"] = (rv.planes.cpu().numpy(), rv.costs.cpu().numpy())
    imgs = {k: images[k].cpu().numpy() for k in range(views)}
    pool.close()
    return rv, cams, imgs, srcs, out


def _problem(cams, imgs, srcs, v):
    ids = [v] + list(srcs[v])
    return ids, [cams[i] for i in ids], [imgs[i] for i in ids]


@pytest.mark.timeout(600)
def test_cfg2_bench_path_10_views_400x300():
    rv, cams, imgs, srcs, out = _cfg2(400, 300)
    g_pl, g_co, g_dep = out["photo"]
    ref_photo = {}
    for v in range(10):
        ids, cs, ims = _problem(cams, imgs, srcs, v)
        ref = oracle.run_patchmatch(rv.used_params[("photo", v)], cs, ims)
        assert_bit_exact(g_pl[v], ref["planes"], f"photometric planes view {v}")
        assert_bit_exact(g_co[v], ref["costs"], f"photometric costs view {v}")
        assert_bit_exact(g_dep[v], ref["planes"][..., 3], f"exported depth view {v}")
        ref_photo[v] = ref
    geo_pl, geo_co = out["geom"]
    for v in range(10):
        ids, cs, ims = _problem(cams, imgs, srcs, v)
        prm = rv.used_params[("geom", v)]
        assert prm.geom_consistency == 1 and prm.max_iterations == 8
        ref = oracle.run_patchmatch(prm, cs, ims, depths=[ref_photo[i]["planes"][..., 3] for i in ids],
                                    planes=ref_photo[v]["planes"], costs=ref_photo[v]["costs"])
        assert_bit_exact(geo_pl[v], ref["planes"], f"geometric planes view {v}")
        assert_bit_exact(geo_co[v], ref["costs"], f"geometric costs view {v}")
    # the pass did reconstruct something: most pixels confident after geom
    assert (np.isfinite(geo_co) & (geo_co < 0.5)).mean() > 0.5


@pytest.mark.timeout(900)
def test_cfg2_bench_path_full_1600x1200_view():
    rv, cams, imgs, srcs, out = _cfg2(1600, 1200)
    v = 0
    ids, cs, ims = _problem(cams, imgs, srcs, v)
    g_pl, g_co, g_dep = out["photo"]
    ref = oracle.run_patchmatch(rv.used_params[("photo", v)], cs, ims)
    assert_bit_exact(g_pl[v], ref["planes"], "photometric planes (1600x1200)")
    assert_bit_exact(g_co[v], ref["costs"], "photometric costs (1600x1200)")
    depths = [ref["planes"][..., 3]] + [g_dep[i] for i in ids[1:]]
    geo = oracle.run_patchmatch(rv.used_params[("geom", v)], cs, ims, depths=depths, planes=ref["planes"],
                                costs=ref["costs"])
    geo_pl, geo_co = out["geom"]
    assert_bit_exact(geo_pl[v], geo["planes"], "geometric planes (1600x1200)")
    assert_bit_exact(geo_co[v], geo["costs"], "geometric costs (1600x1200)")


def test_cfg2_batched_launch_equals_streams_and_single_view_runs():
    """The pool's schedules give the same maps: S = 2 and S = 4 views per
    launch (4 + 4 + 2: batches of different sizes), two engines on two
    streams, and one view per launch."""
    outs = {}
    for name, (streams, mode) in {"b2": (2, "batch"), "b4": (4, "batch"), "s2": (2, "streams"),
                                  "one": (1, "batch")}.items():
        _, _, _, _, out = _cfg2(200, 150, iters=3, streams=streams, mode=mode)
        outs[name] = out
    for name in ("b4", "s2", "one"):
        for ph in ("photo", "geom"):
            for a, b in zip(outs["b2"][ph], outs[name][ph]):
                assert_bit_exact(b, a, f"{name} vs b2 {ph}")


def test_run_batch_mixed_problems_match_single_runs():
    """acmmp_run_patchmatch_batch with engines of different source-view
    buckets and image sizes: compatible engines share launches (4 sources,
    two sizes in one launch), the others run in their own groups; every
    engine's result equals its own acmmp_run_patchmatch."""
    from acmmp_amd import ACMMP
    probs = []
    for (w, h, nsrc, ref) in [(96, 72, 4, 0), (128, 96, 4, 1), (96, 72, 9, 2), (80, 60, 4, 3), (64, 48, 2, 4)]:
        sc = scene.make_scene(num_views=10, width=w, height=h)
        probs.append(sc.problem(ref, nsrc))
    p = default_params()
    p.max_iterations = 2
    single = []
    for cams, imgs in probs:
        with ACMMP(0) as eng:
            eng.set_params(p)
            eng.set_images(cams, imgs)
            eng.RunPatchMatch()
            single.append((eng.plane_hypotheses(), eng.costs(), eng.selected_views()))
    engines = [ACMMP(0) for _ in probs]
    try:
        for eng, (cams, imgs) in zip(engines, probs):
            eng.set_params(p)
            eng.set_images(cams, imgs)
        ACMMP.run_batch(engines)
        for k, eng in enumerate(engines):
            eng.synchronize()
            assert_bit_exact(eng.plane_hypotheses(), single[k][0], f"planes of problem {k}")
            assert_bit_exact(eng.costs(), single[k][1], f"costs of problem {k}")
            assert_bit_exact(eng.selected_views(), single[k][2], f"selected views of problem {k}")
    finally:
        for eng in engines:
            eng.close()
