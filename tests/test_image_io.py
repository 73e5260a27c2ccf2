"""Image input of InputInitialization without OpenCV (src/ACMMP.cpp:525-601):
the library's baseline-JPEG luminance decoder is checked pixel-exact against
libjpeg(-turbo) through Pillow in grayscale-draft mode (libjpeg's
JCS_GRAYSCALE output, which is what cv::imread(IMREAD_GRAYSCALE) returns),
over subsampling modes, qualities, restart intervals and odd sizes; PGM/PFM
round trips; cv::resize INTER_LINEAR restated in numpy."""
import io as _io
import os

import numpy as np
import pytest

from acmmp_amd import io

PIL = pytest.importorskip("PIL.Image")


def _pil_gray(path):
    im = PIL.open(path)
    im.draft("L", im.size)
    assert im.mode == "L"
    return np.asarray(im, dtype=np.float32)


def _texture(w, h, seed):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    base = 128 + 60 * np.sin(x / 7.0) * np.cos(y / 11.0) + rng.normal(0, 25, (h, w))
    return np.clip(base, 0, 255).astype(np.uint8)


@pytest.mark.parametrize("w,h,sub,q,rst", [
    (64, 48, 0, 95, 0),      # 4:4:4
    (123, 77, 2, 90, 0),     # 4:2:0, odd sizes (partial MCUs)
    (200, 150, 1, 75, 0),    # 4:2:2
    (97, 131, 2, 100, 3),    # restart interval
    (40, 33, 2, 30, 1),      # low quality, restart every MCU
])
def test_jpeg_colour_matches_libjpeg(tmp_path, w, h, sub, q, rst):
    g = _texture(w, h, w * h)
    rgb = np.stack([g, np.roll(g, 3, 1), 255 - g], -1)
    path = str(tmp_path / "00000000.jpg")
    kw = dict(quality=q, subsampling=sub)
    if rst:
        kw["restart_marker_blocks"] = rst
    PIL.fromarray(rgb, "RGB").save(path, "JPEG", **kw)
    ours = io.read_image_gray(path)
    np.testing.assert_array_equal(ours, _pil_gray(path))
    assert io.image_size(path) == (w, h)


@pytest.mark.parametrize("w,h,q", [(64, 48, 95), (111, 67, 50)])
def test_jpeg_grayscale_matches_libjpeg(tmp_path, w, h, q):
    path = str(tmp_path / "g.jpg")
    PIL.fromarray(_texture(w, h, 5), "L").save(path, "JPEG", quality=q)
    np.testing.assert_array_equal(io.read_image_gray(path), _pil_gray(path))


@pytest.mark.parametrize("w,h,mode,kw", [
    (64, 48, "L", {}),                                      # gray, DC + AC band scans
    (40, 33, "L", dict(quality=30)),                        # partial blocks, low quality
    (123, 77, "RGB", dict(subsampling=2)),                  # 4:2:0, interleaved DC scans
    (200, 150, "RGB", dict(subsampling=1, quality=90)),     # 4:2:2
    (97, 131, "RGB", dict(subsampling=0, quality=100)),     # 4:4:4, many refinement bits
    (97, 131, "RGB", dict(subsampling=2, restart_marker_blocks=3)),  # restarts reset the EOB runs
    (301, 211, "RGB", dict(quality=75, optimize=True)),     # long EOB runs
])
def test_jpeg_progressive_matches_libjpeg(tmp_path, w, h, mode, kw):
    """Progressive JPEG (SOF2): the spectral-selection and successive-
    approximation scans of libjpeg's simple progression script — DC first,
    AC first bands, DC and AC refinement — pixel-exact against libjpeg's
    grayscale output and, for colour files, its RGB output (cv::imread of a
    camera JPEG the converter copied verbatim, colmap2mvsnet_acm.py:453-454)."""
    g = _texture(w, h, w * h + 7)
    img = PIL.fromarray(g, "L") if mode == "L" else PIL.fromarray(np.stack([g, np.roll(g, 5, 0), 255 - g], -1), "RGB")
    path = str(tmp_path / "p.jpg")
    img.save(path, "JPEG", progressive=True, **kw)
    assert PIL.open(path).info.get("progressive") or PIL.open(path).info.get("progression")
    np.testing.assert_array_equal(io.read_image_gray(path), _pil_gray(path))
    assert io.image_size(path) == (w, h)
    if mode == "RGB":
        ref = np.asarray(PIL.open(path).convert("RGB"))
        np.testing.assert_array_equal(io.read_image_bgr(path), ref[..., ::-1])


def test_jpeg_arithmetic_and_lossless_are_rejected(tmp_path):
    """SOF9..SOF11 (arithmetic) and SOF3 (lossless) stay unsupported: a
    baseline file with its SOF marker rewritten must be refused, not misread."""
    path = str(tmp_path / "b.jpg")
    PIL.fromarray(_texture(32, 32, 1), "L").save(path, "JPEG")
    data = bytearray(open(path, "rb").read())
    i = data.find(b"\xff\xc0")
    for marker in (0xC3, 0xC9, 0xCA):
        data[i + 1] = marker
        bad = str(tmp_path / ("m%x.jpg" % marker))
        open(bad, "wb").write(bytes(data))
        with pytest.raises(IOError):
            io.read_image_gray(bad)


def test_pgm_and_pfm(tmp_path):
    g = _texture(31, 17, 2)
    p = str(tmp_path / "a.pgm")
    with open(p, "wb") as f:
        f.write(b"P5\n# comment\n31 17\n255\n" + g.tobytes())
    np.testing.assert_array_equal(io.read_image_gray(p), g.astype(np.float32))
    fl = np.random.default_rng(0).normal(size=(9, 13)).astype(np.float32)
    p2 = str(tmp_path / "b.pfm")
    with open(p2, "wb") as f:
        f.write(b"Pf\n13 9\n-1.0\n" + np.ascontiguousarray(fl[::-1]).astype("<f4").tobytes())
    np.testing.assert_array_equal(io.read_image_gray(p2), fl)
    with pytest.raises(IOError):
        io.read_image_gray(str(tmp_path / "missing.jpg"))


def _resize_ref(src, dw, dh):
    """OpenCV INTER_LINEAR for CV_32F restated (coefficients in float)."""
    sh, sw = src.shape
    sx, sy = sw / dw, sh / dh
    if sx == 2 and sy == 2:
        r = src.reshape(dh, 2, dw, 2)
        return ((r[:, 0, :, 0] + r[:, 0, :, 1]) + (r[:, 1, :, 0] + r[:, 1, :, 1])) * np.float32(0.25)

    def coeffs(n, s, size):
        f = np.array([np.float32((i + 0.5) * s - 0.5) for i in range(n)], dtype=np.float32)
        i0 = np.floor(f).astype(np.int64)
        a = (f - i0.astype(np.float32)).astype(np.float32)
        a[i0 < 0] = 0
        i0[i0 < 0] = 0
        hi = i0 >= size - 1
        a[hi] = 0
        i0[hi] = size - 1
        return i0, np.minimum(i0 + 1, size - 1), a

    x0, x1, ax = coeffs(dw, sx, sw)
    y0, y1, ay = coeffs(dh, sy, sh)
    one = np.float32(1)
    rows = src[:, x0] * (one - ax) + src[:, x1] * ax
    return rows[y0] * (one - ay)[:, None] + rows[y1] * ay[:, None]


@pytest.mark.parametrize("sw,sh,dw,dh", [(64, 48, 32, 24), (6048 // 16, 4032 // 16, 200, 133), (50, 40, 37, 29)])
def test_resize_linear(sw, sh, dw, dh):
    src = _texture(sw, sh, 9).astype(np.float32)
    np.testing.assert_array_equal(io.resize_linear(src, dw, dh), _resize_ref(src, dw, dh))


@pytest.mark.parametrize("w,h,sub,q,rst", [
    (64, 48, 0, 95, 0), (123, 77, 2, 90, 0), (200, 150, 1, 75, 0), (97, 131, 2, 100, 3), (41, 33, 2, 30, 1),
    (2, 2, 2, 90, 0),
])
def test_jpeg_colour_bgr_matches_libjpeg(tmp_path, w, h, sub, q, rst):
    """cv::imread(IMREAD_COLOR): libjpeg fancy upsampling + YCbCr tables."""
    g = _texture(w, h, 3 * w + h)
    rgb = np.stack([g, np.roll(g, 5, 0), 255 - np.roll(g, 2, 1)], -1)
    path = str(tmp_path / "c.jpg")
    kw = dict(quality=q, subsampling=sub)
    if rst:
        kw["restart_marker_blocks"] = rst
    PIL.fromarray(rgb, "RGB").save(path, "JPEG", **kw)
    ref = np.asarray(PIL.open(path).convert("RGB"))
    np.testing.assert_array_equal(io.read_image_bgr(path), ref[..., ::-1])


def test_gray_jpeg_as_bgr(tmp_path):
    path = str(tmp_path / "g.jpg")
    PIL.fromarray(_texture(30, 20, 1), "L").save(path, "JPEG", quality=80)
    got = io.read_image_bgr(path)
    ref = np.asarray(PIL.open(path))
    for k in range(3):
        np.testing.assert_array_equal(got[..., k], ref)
