"""RunFusion port (acmmp_amd/csrc/acmmp_fusion.cpp) on CPU:
a synthetic dense folder with ground-truth-derived depth/normal maps is fused
by the library and by the Python restatement (tests/oracle_fusion.py); the
binary PLY must match point for point, bit-exactly."""
import os

import numpy as np
import pytest

from acmmp_amd import io as aio
from acmmp_amd import pipeline, scene
from oracle_fusion import read_ply, run_fusion


def _dense_with_maps(tmp_path, W=72, H=54, views=4):
    d = str(tmp_path / "dense")
    sc = scene.make_scene(num_views=views, width=W, height=H)
    scene.write_dense_folder(sc, d, num_src=2)
    # colour images (the fusion reads IMREAD_COLOR)
    from PIL import Image
    for i, v in enumerate(sc.views):
        g = np.clip(np.rint(v.image), 0, 255).astype(np.uint8)
        rgb = np.stack([g, 255 - g, np.roll(g, 3, 1)], -1)
        Image.fromarray(rgb, "RGB").save(os.path.join(d, "images", "%08d.jpg" % i), "JPEG", quality=92)
    out = d + "/ACMMP"
    rng = np.random.default_rng(1)
    for i, v in enumerate(sc.views):
        rf = aio.result_folder(out, i)
        os.makedirs(rf, exist_ok=True)
        depth = np.where(v.depth > 0, v.depth * (1 + rng.normal(0, 0.002, v.depth.shape)), 0).astype(np.float32)
        depth[rng.random(depth.shape) < 0.05] = 0.0
        nrm = v.normal + rng.normal(0, 0.02, v.normal.shape)
        nrm /= np.linalg.norm(nrm, axis=-1, keepdims=True)
        aio.write_dmb(os.path.join(rf, "depths_geom.dmb"), depth)
        aio.write_dmb(os.path.join(rf, "normals.dmb"), nrm.astype(np.float32))
    return d, out


def test_fusion_matches_python_restatement(tmp_path):
    d, out = _dense_with_maps(tmp_path)
    n = pipeline.run_fusion(d, out, write_debug_images=True)
    ply = read_ply(os.path.join(out, "ACMMP_model.ply"))
    ref = run_fusion(d, out)
    assert n == len(ply) == len(ref) and n > 1000
    xyz = np.array([p[0] for p in ref], np.float32)
    nrm = np.array([p[1] for p in ref], np.float32)
    col = np.array([p[2] for p in ref], np.uint8)
    got_xyz = np.stack([ply["x"], ply["y"], ply["z"]], -1)
    got_nrm = np.stack([ply["nx"], ply["ny"], ply["nz"]], -1)
    np.testing.assert_array_equal(got_xyz.view(np.uint32), xyz.view(np.uint32))
    np.testing.assert_array_equal(got_nrm.view(np.uint32), nrm.view(np.uint32))
    np.testing.assert_array_equal(np.stack([ply["r"], ply["g"], ply["b"]], -1), col)
    assert os.path.exists(os.path.join(d, "approved_pixels_cam_0.png"))


def test_fusion_ply_chunks_write_the_same_bytes(tmp_path, monkeypatch):
    """The PLY is formed and written in chunks on the fusion pool: with chunks
    of 97 points (dozens of chunks, most records straddling nothing, every
    boundary at an odd byte offset) the file is byte-identical to the
    default single-chunk write, for RunFusion (pooled) and the prior-aware
    fusion (sequential chunks)."""
    d, out = _dense_with_maps(tmp_path)
    path = os.path.join(out, "ACMMP_model.ply")
    n = pipeline.run_fusion(d, out)
    whole = open(path, "rb").read()
    monkeypatch.setenv("ACMMP_PLY_CHUNK_POINTS", "97")
    assert pipeline.run_fusion(d, out) == n and n > 20 * 97
    assert open(path, "rb").read() == whole
    prior = os.path.join(out, "ACMMP_prior_model.ply")
    monkeypatch.delenv("ACMMP_PLY_CHUNK_POINTS")
    pipeline.run_prior_aware_fusion(d, out, out)
    whole = open(prior, "rb").read()
    monkeypatch.setenv("ACMMP_PLY_CHUNK_POINTS", "97")
    pipeline.run_prior_aware_fusion(d, out, out)
    assert open(prior, "rb").read() == whole


@pytest.mark.parametrize("kind", ["gray8", "bgr8", "gray16"])
def test_fusion_with_masks_matches_restatement(tmp_path, kind):
    """RunFusion's mask folder (src/acmmp_definitions.cpp:881-905): masked
    pixels are skipped as references and as sources from the start. The mask
    is read as cv::imread(-1) reads it and indexed as the reference indexes
    it (at<uchar>(r, c): byte c of row r, which for a colour mask is channel
    c % 3 of pixel c / 3); 8-bit gray, 8-bit colour and 16-bit gray PNGs."""
    from PIL import Image
    d, out = _dense_with_maps(tmp_path)
    os.makedirs(os.path.join(d, "masks"))
    rng = np.random.default_rng(5)
    for i in range(4):
        H, W = 54, 72
        if kind == "bgr8":
            m = rng.integers(60, 256, (H, W, 3)).astype(np.uint8)
            img = Image.fromarray(m, "RGB")
        elif kind == "gray16":
            img = Image.fromarray(rng.integers(40, 400, (H, W)).astype(np.uint16))
        else:
            img = Image.fromarray(rng.integers(70, 256, (H, W)).astype(np.uint8), "L")
        img.save(os.path.join(d, "masks", "%08d.png" % i))
    n = pipeline.run_fusion(d, out, mask_folder="masks")
    ply = read_ply(os.path.join(out, "ACMMP_model.ply"))
    ref = run_fusion(d, out, mask_folder="masks")
    free = run_fusion(d, out)
    assert 100 < n < len(free)
    _compare_cloud(ply, ref)


def test_fusion_photometric_maps_and_thresholds_match_restatement(tmp_path):
    """geom_consistency = false reads depths.dmb (:867-870), and the two
    thresholds (:1007) change which pixels are approved; both against the
    restatement, PLY point for point."""
    d, out = _dense_with_maps(tmp_path)
    rng = np.random.default_rng(3)
    for i in range(4):
        rf = aio.result_folder(out, i)
        dep = aio.read_dmb(os.path.join(rf, "depths_geom.dmb"))
        dep = np.where(rng.random(dep.shape) < 0.2, dep * np.float32(1.004), dep).astype(np.float32)
        aio.write_dmb(os.path.join(rf, "depths.dmb"), dep)
    for geom, scalar, thresh in ((False, 0.3, 1), (True, 0.4, 2), (False, 0.35, 2)):
        n = pipeline.run_fusion(d, out, geom_consistency=geom, consistency_scalar=scalar, num_consistent_thresh=thresh)
        ref = run_fusion(d, out, geom=geom, consistency_scalar=scalar, con_num_thresh=thresh)
        assert n > 1000, (geom, scalar, thresh, n)
        _compare_cloud(read_ply(os.path.join(out, "ACMMP_model.ply")), ref)


def test_fusion_thresholds_reduce_points(tmp_path):
    d, out = _dense_with_maps(tmp_path)
    n1 = pipeline.run_fusion(d, out, num_consistent_thresh=1)
    n2 = pipeline.run_fusion(d, out, num_consistent_thresh=2)
    n3 = pipeline.run_fusion(d, out, consistency_scalar=0.9)
    assert n1 > n2 > 0 and n1 > n3


def _compare_cloud(ply, ref):
    assert len(ply) == len(ref)
    xyz = np.array([p[0] for p in ref], np.float32).reshape(-1, 3)
    nrm = np.array([p[1] for p in ref], np.float32).reshape(-1, 3)
    col = np.array([p[2] for p in ref], np.uint8).reshape(-1, 3)
    np.testing.assert_array_equal(np.stack([ply["x"], ply["y"], ply["z"]], -1).view(np.uint32), xyz.view(np.uint32))
    np.testing.assert_array_equal(np.stack([ply["nx"], ply["ny"], ply["nz"]], -1).view(np.uint32),
                                  nrm.view(np.uint32))
    np.testing.assert_array_equal(np.stack([ply["r"], ply["g"], ply["b"]], -1), col)


def test_prior_aware_fusion_matches_python_restatement(tmp_path):
    from oracle_fusion import run_prior_aware_fusion
    d, out = _dense_with_maps(tmp_path)
    # a second reconstruction (the "prior" run's output folder) with perturbed maps
    prior = d + "/ACMMP_PRIOR"
    rng = np.random.default_rng(2)
    for i in range(4):
        src, dst = aio.result_folder(out, i), aio.result_folder(prior, i)
        os.makedirs(dst, exist_ok=True)
        dep = aio.read_dmb(os.path.join(src, "depths_geom.dmb"))
        dep = np.where(rng.random(dep.shape) < 0.3, dep * 1.05, dep).astype(np.float32)
        dep[rng.random(dep.shape) < 0.1] = 0.0
        aio.write_dmb(os.path.join(dst, "depths_geom.dmb"), dep)
        aio.write_dmb(os.path.join(dst, "normals.dmb"), aio.read_dmb(os.path.join(src, "normals.dmb")))
    for penalty in (0, 1):
        n = pipeline.run_prior_aware_fusion(d, prior, out, single_match_penalty=penalty)
        ply = read_ply(os.path.join(prior, "ACMMP_prior_model.ply"))
        ref = run_prior_aware_fusion(d, prior, out, penalty=penalty)
        assert n > 500
        _compare_cloud(ply, ref)
