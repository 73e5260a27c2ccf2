"""CPU tier: the C-ABI library loads without a GPU and exports every symbol
include/acmmp.h declares; struct layouts match; the reference's on-disk
formats round-trip through both the C and the Python readers, pinned by
fixtures written by the reference's own converter (tests/golden/colmap_fixture,
made by tools/gen_colmap_fixture.py from python_scripts/colmap2mvsnet_acm.py)."""
import ctypes as C
import json
import os

import numpy as np
import pytest

from acmmp_amd import _abi, io

GOLD = os.path.join(os.path.dirname(__file__), "golden", "colmap_fixture")


@pytest.fixture(scope="module")
def lib():
    return _abi.load_library()


def test_every_header_symbol_is_exported(lib):
    syms = _abi.header_symbols()
    assert len(syms) >= 35
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(syms) == set(_abi.SIGNATURES), "ctypes mirror out of sync with include/acmmp.h"


def test_struct_layouts():
    assert C.sizeof(_abi.Camera) == 100  # == struct Camera of the reference
    assert C.sizeof(_abi.Params) == 4 * 29
    assert C.sizeof(_abi.Timing) == 20


def test_default_params_match_reference(lib):
    p = _abi.Params()
    lib.acmmp_default_params(C.byref(p))
    q = _abi.default_params()
    assert bytes(p) == bytes(q)
    # src/ACMMP.h:32-56
    assert (p.max_iterations, p.patch_size, p.radius_increment, p.top_k) == (2, 11, 2, 4)
    assert (p.sigma_spatial, p.sigma_color) == (5.0, 3.0)


def test_no_gpu_fails_loudly(lib, has_gpu):
    if has_gpu:
        pytest.skip("GPU present")
    ctx = C.c_void_p()
    assert lib.acmmp_create(0, C.byref(ctx)) != _abi.OK
    assert not ctx.value
    from acmmp_amd import ACMMP, AcmmpError
    with pytest.raises(AcmmpError):
        ACMMP(0)


def test_null_context_is_safe(lib):
    assert lib.acmmp_last_error(None) == b"null context"
    lib.acmmp_destroy(None)
    assert lib.acmmp_set_timing(None, 1) == _abi.ERR_ARG


def test_dmb_roundtrip_c_and_python(tmp_path, lib):
    rng = np.random.default_rng(1)
    depth = rng.uniform(300, 800, size=(7, 9)).astype(np.float32)
    normal = rng.normal(size=(7, 9, 3)).astype(np.float32)
    # python writer -> C reader
    p = str(tmp_path / "depths.dmb")
    io.write_dmb(p, depth)
    h, w, nb = C.c_int32(), C.c_int32(), C.c_int32()
    buf = np.zeros(63, np.float32)
    assert lib.acmmp_read_dmb(p.encode(), C.byref(h), C.byref(w), C.byref(nb),
                              buf.ctypes.data_as(C.POINTER(C.c_float)), buf.size) == 0
    assert (h.value, w.value, nb.value) == (7, 9, 1)
    np.testing.assert_array_equal(buf.reshape(7, 9), depth)
    # C writer -> python reader (3 channels, HWC)
    q = str(tmp_path / "normals.dmb")
    assert lib.acmmp_write_dmb(q.encode(), 7, 9, 3, normal.ctypes.data_as(C.POINTER(C.c_float))) == 0
    np.testing.assert_array_equal(io.read_dmb(q), normal)
    raw = open(q, "rb").read()
    assert np.frombuffer(raw[:16], "<i4").tolist() == [1, 7, 9, 3]  # src/ACMMP.cpp:363-371
    assert len(raw) == 16 + 7 * 9 * 3 * 4


def test_dmb_bad_header_rejected(tmp_path, lib):
    p = tmp_path / "bad.dmb"
    p.write_bytes(np.array([2, 1, 1, 1], "<i4").tobytes() + b"\0\0\0\0")
    h, w, nb = C.c_int32(), C.c_int32(), C.c_int32()
    assert lib.acmmp_read_dmb(str(p).encode(), C.byref(h), C.byref(w), C.byref(nb), None, 0) == _abi.ERR_IO
    with pytest.raises(ValueError):
        io.read_dmb(str(p))
    assert lib.acmmp_read_dmb(b"/nonexistent/x.dmb", C.byref(h), C.byref(w), C.byref(nb), None, 0) == _abi.ERR_IO


def test_read_camera_reference_fixture(lib):
    truth = json.load(open(os.path.join(GOLD, "model_truth.json")))
    for i, v in enumerate(truth["views"]):
        path = os.path.join(GOLD, "cams", "%08d_cam.txt" % i)
        c_cam = _abi.Camera()
        assert lib.acmmp_read_camera(path.encode(), C.byref(c_cam)) == 0
        py_cam = io.read_camera(path)
        assert bytes(c_cam) == bytes(py_cam)
        np.testing.assert_allclose(np.array(c_cam.K).reshape(3, 3), truth["K"], rtol=1e-6)
        np.testing.assert_allclose(np.array(c_cam.R).reshape(3, 3), v["R"], atol=1e-6)
        np.testing.assert_allclose(np.array(c_cam.t), v["t"], atol=1e-3)
        assert 0 < c_cam.depth_min < c_cam.depth_max


def test_read_pair_reference_fixture(tmp_path):
    problems = io.read_pair(os.path.join(GOLD, "pair.txt"))
    assert [p.ref_image_id for p in problems] == [0, 1, 2]
    assert all(len(p.src_image_ids) == 2 and p.ref_image_id not in p.src_image_ids for p in problems)
    # GenerateSampleList drops sources with score <= 0 (src/acmmp_definitions.cpp:198)
    io.write_pair(str(tmp_path / "pair.txt"), [[(1, 3), (2, 0)], [(0, 5)], [(0, 0), (1, 0)]])
    got = io.read_pair(str(tmp_path / "pair.txt"))
    assert [p.src_image_ids for p in got] == [[1], [0], []]


def test_camera_writer_roundtrip(tmp_path, lib):
    K = np.array([[2892.33, 0, 823.2], [0, 2883.17, 619.07], [0, 0, 1]])
    R = np.eye(3)
    t = np.array([1.5, -2.25, 600.125])
    path = str(tmp_path / "00000007_cam.txt")
    io.write_camera(path, K, R, t, 300, 2.6041666666666665, 192, 800)
    cam = _abi.Camera()
    assert lib.acmmp_read_camera(path.encode(), C.byref(cam)) == 0
    assert (cam.depth_min, cam.depth_max) == (300.0, 800.0)
    np.testing.assert_allclose(np.array(cam.t), t, rtol=1e-7)


def test_cpp_class_shim_compiles_and_links(tmp_path):
    """include/acmmp.hpp (the C++ `class ACMMP` surface) builds against the
    library; host-only calls work without a GPU, engine creation fails loudly."""
    import shutil
    import subprocess
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = tmp_path / "shim.cpp"
    src.write_text(r'''
#include <acmmp.hpp>
#include <cstdio>
int main() {
    acmmp::Problem p = acmmp::make_problem(3, {1, 2, 4});
    int32_t xy[10] = {0, 0, 10, 0, 0, 10, 10, 10, 5, 4};
    int32_t t[6 * 32];
    int n = 0;
    int rc = acmmp_delaunay_triangulation(20, 20, xy, 5, t, 32, &n);
    bool threw = false;
    if (acmmp_device_count() == 0) {
        try { acmmp::ACMMP a(0); } catch (const acmmp::Error &e) { threw = true; }
    } else {
        threw = true;
    }
    std::printf("%d %d %d %d\n", p.num_src_images, rc, n, threw ? 1 : 0);
    return 0;
}
''')
    exe = tmp_path / "shim"
    lib = os.path.join(root, "acmmp_amd", "lib")
    subprocess.run([gxx, "-std=c++17", "-I" + os.path.join(root, "include"), str(src), "-L" + lib, "-lacmmp_amd",
                    "-Wl,-rpath," + lib, "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    assert out == ["3", "0", "4", "1"]


def test_cli_order_flag_validated():
    """`acmmp_main --order sequential|jacobi`: a bad value is
    a usage error (exit 2) before any device is touched."""
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "acmmp_amd", "lib", "acmmp_main")
    if not os.path.exists(exe):
        pytest.skip("acmmp_main not built")
    r = subprocess.run([exe, "--order", "sideways", "/nonexistent"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "--order sequential|jacobi" in r.stderr
    r = subprocess.run([exe, "--help"], capture_output=True, text=True, timeout=60)
    assert "--order sequential|jacobi" in r.stdout + r.stderr
