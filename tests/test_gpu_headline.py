"""Parity of the headline benchmark's exact path (BASELINE configs[1], cfg2):
the `acmmp_amd.resident` schedule bench.py times — two engines on two HIP
streams fed from a shared queue, images borrowed from HBM
(set_images_device), run_async, results exported device-to-device
(export_results) and fed back through set_depth_maps_device /
set_plane_hypotheses_device — N = 10 images per problem, 8 iterations,
photometric then geometric, the pass order of src/main_ACMMP.cpp:123-137 and
one RunPatchMatch per view (src/ACMMP.cu:1378-1456), each view with the
bench's own Philox key (bench.VIEW_SEED + view id).

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

import bench  # the bench's per-view Philox keys (conftest puts the repo root on sys.path)
from parity_util import assert_bit_exact

pytestmark = pytest.mark.gpu


def _cfg2(width, height, views=10, nsrc=9, iters=8, streams=2):
    dev = torch.device("cuda", 0)
    setup = scene.scene_setup(num_views=views, width=width, height=height)
    images = {k: scene.render_torch(setup, k, dev) for k in range(views)}
    cams = {k: setup.camera(k) for k in range(views)}
    srcs = {k: setup.pairs[k][:nsrc] for k in range(views)}
    torch.cuda.synchronize()
    pool = EnginePool(0, streams)
    rv = ResidentViews(pool, cams, images, srcs, range(views), height, width, view_seed=bench.VIEW_SEED)
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
