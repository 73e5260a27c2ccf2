"""The N-rank simulation of tools/scale_sim.py (pure arithmetic, CPU)."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

from scale_sim import _rank_time, simulate  # noqa: E402


def _passes(n=2):
    return [{"kind": "planar" if k == 0 else "geom", "t_eff": 0.1, "t_alone": 0.15, "map_bytes": 0,
             "exchanges": 6} for k in range(n)]


HOST0 = {"load": 0.0, "jbu": 0.0, "flush": 0.0, "fusion": 0.0, "image_bytes": 0}


def test_rank_time_pairs_and_odd_view():
    assert _rank_time(6, 0.1, 0.15) == pytest.approx(0.6)
    assert _rank_time(7, 0.1, 0.15) == pytest.approx(0.75)
    assert _rank_time(0, 0.1, 0.15) == 0.0


def test_lpt_tail_caps_efficiency_at_6_125_over_7():
    """49 equal views on 8 ranks without the split: one rank runs 7 views
    (the 7th alone), the ideal is 49/8 views' throughput."""
    r = simulate(_passes(), {"planar": 0.2, "geom": 0.2}, HOST0, 49, 8, False, halo_latency_s=0.0)
    assert r["views_per_rank"] == [7, 6, 6, 6, 6, 6, 6, 6] and r["split_views"] == 0
    assert r["compute_efficiency"] == pytest.approx((49 * 0.1 / 8) / 0.75)
    assert r["compute_efficiency"] < 0.875


def test_split_tail_lifts_efficiency():
    """With the 49th view in 8 bands each rank runs 6 whole views plus one
    band (here 1/8 of the alone time + 10 % overhead)."""
    band = {"planar": 0.1375, "geom": 0.1375}
    r = simulate(_passes(), band, HOST0, 49, 8, True, halo_latency_s=0.0)
    assert r["split_views"] == 1
    per_pass = 0.6 + 0.1375 * 0.15
    assert r["compute_s"] == pytest.approx(2 * per_pass)
    assert r["compute_efficiency"] == pytest.approx((49 * 0.1 / 8) / per_pass)
    assert r["compute_efficiency"] > 0.95


def test_host_phases_and_fusion_counted():
    host = {"load": 0.8, "jbu": 0.08, "flush": 0.8, "fusion": 3.0, "image_bytes": 0}
    r = simulate(_passes(), {"planar": 0.14, "geom": 0.14}, host, 49, 8, True, halo_latency_s=0.0)
    assert r["host_s"] == pytest.approx(1.68 / 8)
    assert r["wall_s"] == pytest.approx(r["compute_s"] + r["host_s"] + 3.0)
    assert r["non_compute_share"] > r["non_compute_share_without_fusion"]
