"""Host-side planar-prior pieces without a GPU: the library's exact Delaunay
triangulation (DelaunayTriangulation, src/ACMMP.cpp:896-918) checked by the
empty-circumcircle property in exact integer arithmetic and against Qhull,
and the oracle's plane fit / raster against analytic known answers."""
import numpy as np
import pytest

import oracle
from acmmp_amd import delaunay_triangulation, make_camera


def _incircle(a, b, c, d):
    adx, ady = a[0] - d[0], a[1] - d[1]
    bdx, bdy = b[0] - d[0], b[1] - d[1]
    cdx, cdy = c[0] - d[0], c[1] - d[1]
    return ((adx * adx + ady * ady) * (bdx * cdy - cdx * bdy) + (bdx * bdx + bdy * bdy) * (cdx * ady - adx * cdy)
            + (cdx * cdx + cdy * cdy) * (adx * bdy - bdx * ady))


def _orient(a, b, c):
    return (b[0] - a[0]) * (c[1] - a[1]) - (b[1] - a[1]) * (c[0] - a[0])


def _check_triangulation(tris, pts):
    P = [tuple(int(v) for v in p) for p in pts]
    directed = set()
    for t in tris.tolist():
        a, b, c = (t[0], t[1]), (t[2], t[3]), (t[4], t[5])
        assert _orient(a, b, c) > 0, "triangles are counter-clockwise and non-degenerate"
        for e in ((a, b), (b, c), (c, a)):
            assert e not in directed, "a directed edge belongs to one triangle (no overlap)"
            directed.add(e)
        for d in P:
            assert _incircle(a, b, c, d) <= 0, "empty circumcircle"
    used = {p for t in tris.tolist() for p in ((t[0], t[1]), (t[2], t[3]), (t[4], t[5]))}
    assert used <= set(P)


@pytest.mark.parametrize("seed", [0, 1])
def test_delaunay_random_points_exact(seed):
    rng = np.random.default_rng(seed)
    pts = np.unique(rng.integers(0, [120, 90], size=(150, 2)), axis=0)
    tris = delaunay_triangulation(120, 90, pts)
    _check_triangulation(tris, pts)
    assert tris.shape[0] >= 2 * len(pts) - 40


def test_delaunay_cocircular_grid():
    """Support points sit on a 5-px lattice: many co-circular quadruples."""
    g = np.stack(np.meshgrid(np.arange(0, 60, 5), np.arange(0, 45, 5)), -1).reshape(-1, 2)
    g = g[np.random.default_rng(3).random(len(g)) < 0.85]
    tris = delaunay_triangulation(60, 45, g)
    _check_triangulation(tris, g)


def test_delaunay_subset_of_qhull():
    """In general position the Delaunay triangulation is unique: every
    triangle produced must be one of Qhull's."""
    spatial = pytest.importorskip("scipy.spatial")
    rng = np.random.default_rng(11)
    pts = np.unique(rng.integers(0, [400, 300], size=(400, 2)), axis=0)
    ours = {frozenset(map(tuple, t.reshape(3, 2).tolist())) for t in delaunay_triangulation(400, 300, pts)}
    q = spatial.Delaunay(pts.astype(np.float64))
    theirs = {frozenset(map(tuple, pts[s].tolist())) for s in q.simplices}
    P = [tuple(p) for p in pts.tolist()]
    for t in ours - theirs:  # only co-circular ties may differ from Qhull
        a, b, c = sorted(t)
        if _orient(a, b, c) < 0:
            b, c = c, b
        assert any(_incircle(a, b, c, d) == 0 for d in P if d not in t)
    assert len(ours) >= 0.9 * len(theirs)


def test_delaunay_edge_cases():
    assert delaunay_triangulation(10, 10, np.zeros((0, 2), np.int32)).shape == (0, 6)
    assert delaunay_triangulation(10, 10, np.array([[1, 1], [5, 5]])).shape == (0, 6)
    assert delaunay_triangulation(10, 10, np.array([[1, 1], [2, 2], [3, 3]])).shape == (0, 6)  # collinear
    t = delaunay_triangulation(10, 10, np.array([[1, 1], [8, 1], [1, 8], [1, 1]]))  # duplicate point
    assert t.shape == (1, 6)


def _cam(W=64, H=48):
    K = [[100.0, 0, 31.5], [0, 100.0, 23.5], [0, 0, 1]]
    return make_camera(K, np.eye(3), np.zeros(3), W, H, 300.0, 800.0)


def test_oracle_prior_plane_fronto_parallel_kat():
    cam = _cam()
    depths = np.full((48, 64), 500.0, np.float32)
    planes, mask, prior = oracle.planar_prior(cam, depths, 200.0, 900.0, np.array([[2, 2, 40, 5, 10, 30]]))
    np.testing.assert_allclose(planes[0], [0, 0, -1, 500], rtol=0, atol=1e-4)
    assert (mask > 0).sum() > 300
    # out of [dmin, dmax]: the whole triangle is cleared
    _, mask2, prior2 = oracle.planar_prior(cam, depths, 600.0, 900.0, np.array([[2, 2, 40, 5, 10, 30]]))
    assert mask2.sum() == 0 and not prior2.any()


def test_oracle_raster_matches_float_restatement():
    """The raster loop restated with numpy float32 / Python double."""
    cam = _cam()
    depths = np.full((48, 64), 500.0, np.float32)
    t = [3, 4, 30, 9, 12, 40]
    _, mask, _ = oracle.planar_prior(cam, depths, 1.0, 1e4, np.array([t]))
    f = np.float32
    L = [np.sqrt((t[0] - t[2]) ** 2 + (t[1] - t[3]) ** 2), np.sqrt((t[0] - t[4]) ** 2 + (t[1] - t[5]) ** 2),
         np.sqrt((t[2] - t[4]) ** 2 + (t[3] - t[5]) ** 2)]
    step = f(1.0 / float(max(f(v) for v in L)))
    exp = np.zeros((48, 64), np.uint32)
    p = f(0)
    while float(p) < 1.0:
        q = f(0)
        while float(q) < 1.0 - float(p):
            x = int(float(f(p * f(t[0])) + f(q * f(t[2]))) + (1.0 - float(p) - float(q)) * t[4])
            y = int(float(f(p * f(t[1])) + f(q * f(t[3]))) + (1.0 - float(p) - float(q)) * t[5])
            exp[y, x] = 1
            q = f(q + step)
        p = f(p + step)
    np.testing.assert_array_equal(mask, exp)


def test_oracle_support_points_kat():
    costs = np.full((12, 11), 2.5, np.float32)
    costs[1, 2] = 0.05
    costs[3, 4] = 0.05      # tie: the first in (col, row) order wins
    costs[7, 9] = 0.2       # >= 0.1: not a support point
    costs[10, 1] = np.nan
    costs[11, 0] = 0.01
    pts = oracle.support_points(costs)
    np.testing.assert_array_equal(pts, [[2, 1], [0, 11]])
