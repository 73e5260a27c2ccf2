"""bench.py's roofline block from synthetic counter passes (no GPU): the
derived fractions follow tools/bench_pmc.py's formulas and every key the
driver reads is present."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]

import bench_pmc  # noqa: E402


def _passes():
    gui = 8.0e7                     # summed over 8 XCDs: 1e7 cycles per CU
    fetch = {"FETCH_SIZE": 1.0e6, "GRBM_GUI_ACTIVE": gui, "TD_TD_BUSY_sum": 2.048e9,
             "TA_BUFFER_READ_WAVEFRONTS_sum": 5.0e7, "SQ_INSTS_VMEM_RD": 5.2e7, "SQ_INSTS_LDS": 4.7e7,
             "SQ_WAVES": 1.5e4}
    write = {"WRITE_SIZE": 3.0e5, "GRBM_GUI_ACTIVE": gui, "TA_TA_BUSY_sum": 1.28e9, "SQ_INSTS_VMEM_WR": 1.4e6,
             "SQ_ACTIVE_INST_VALU": 1.92e9, "SQ_INSTS_VALU": 1.87e9, "TCP_TOTAL_CACHE_ACCESSES_sum": 1.8e9,
             "TA_BUFFER_READ_WAVEFRONTS_sum": 5.0e7}
    l2 = {"TCC_HIT_sum": 3.0e8, "TCC_MISS_sum": 1.0e8, "TCC_EA0_RDREQ_sum": 2.0e7, "TCC_EA0_RDREQ_128B_sum": 1.5e7,
          "TCP_TCC_READ_REQ_sum": 1.75e8, "TA_BUFFER_READ_WAVEFRONTS_sum": 5.0e7, "GRBM_GUI_ACTIVE": gui}
    per = lambda d: {k: {0: v, 1: v} for k, v in d.items()}  # two dispatches
    return {"passes": {"fetch": {"counters": per(fetch), "durations_ms": [4.0, 4.0]},
                       "write": {"counters": per(write), "durations_ms": [4.0, 4.0]},
                       "l2": {"counters": per(l2), "durations_ms": [4.0, 4.0]}}}


def test_summarize_fractions():
    s = bench_pmc.summarize(_passes())
    assert s["launches"] == 2
    assert abs(s["td_busy_frac"] - 2.048e9 / (1e7 * 256)) < 1e-12
    assert abs(s["valu_busy_frac"] - 4 * 1.92e9 / (1e7 * 256 * 4)) < 1e-12
    assert s["hbm_bytes"] == (2 * 1.0e6 + 3.0e5) * 1024
    assert abs(s["clock_ghz"] - 2.5) < 1e-12
    assert abs(s["tcp_accesses_per_gather"] - 36.0) < 1e-9
    assert abs(s["l2_hit_rate"] - 0.75) < 1e-12
    assert abs(s["l1_to_l2_reqs_per_gather"] - 3.5) < 1e-12
    assert s["ea_read_reqs"] == 2.0e7 and s["ea_read_reqs_128b"] == 1.5e7
    assert s["read_bytes_calibrated"] == 128 * 1.5e7 + 64 * 0.5e7


def test_bench_roofline_block():
    import bench
    s = bench_pmc.summarize(_passes())
    r = bench.roofline(s, 4.0, 1.0e10, 8.0, 2, 2)
    # the contract's form: algorithmic bytes / launch time against the HBM peak
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == bench.HBM_PEAK_GBS
    assert abs(r["achieved"] - 1.0e10 / 4.0e-3 / 1e9) < 0.1
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert r["traffic"] == s["hbm_bytes"]
    assert r["binding_unit"]["bound"] == "td-gather" and 0 < r["binding_unit"]["frac"] <= 1
    assert r["binding_unit"]["l1_accesses_per_gather"] == 36.0
    assert r["valu"]["bound"] == "valu" and r["valu"]["frac"] == round(s["valu_busy_frac"], 4)
    assert r["hbm_physical"]["frac"] < 1
    for k in ("achieved", "peak", "unit", "frac", "traffic"):
        assert k in r
    # frac is over algorithmic bytes; the physical fraction sits beside it
    assert r["frac_is_algorithmic"] is True
    assert r["hbm_physical_frac"] == r["hbm_physical"]["frac"]
    assert r["l2"]["hit_rate"] == 0.75 and r["l2"]["l1_to_l2_reqs_per_gather"] == 3.5


def test_bench_roofline_performed_calls():
    """the NCC calls the kernel performs (gather
    wave-instructions / waves / 36) beside the model's 14 (N-1), and the
    roofline fraction on the performed calls."""
    import bench
    s = bench_pmc.summarize(_passes())
    r = bench.roofline(s, 4.0, 1.0e10, 8.0, 2, 2, num_images=10, pixels_per_launch=960000)
    calls = 5.0e7 / 1.5e4 / 36
    assert r["ncc_calls_per_pixel_iter"] == round(calls, 2)
    assert r["ncc_calls_per_pixel_iter_model"] == 126
    perf = 960000 * ((calls * 724 + 572) + (calls * 728 + 572)) / 2
    assert r["performed_bytes_per_launch"] == round(perf)
    assert abs(r["frac_performed"] - perf / 4.0e-3 / 1e9 / bench.HBM_PEAK_GBS) < 1e-4
    # fewer calls performed than modelled: the performed fraction is the smaller
    assert r["frac_performed"] < bench.roofline(s, 4.0, 960000 * (126 * 726 + 572), 8.0, 2, 2)["frac"]


def test_view_sources_span_ranks():
    """at N > 1 every view reads sources held by other ranks;
    at N = 1 all sources are the rank's own copies (the r05 lists)."""
    import bench
    pairs = {k: [(k + d) % 10 for d in range(1, 10)] for k in range(10)}
    assert bench.view_sources(3, 0, 1, 10, pairs, 9) == pairs[3]
    for world in (2, 4, 8):
        for r in range(world):
            for k in range(10):
                src = bench.view_sources(k, r, world, 10, pairs, 9)
                assert [g % 10 for g in src] == pairs[k]
                owners = [g // 10 for g in src]
                assert owners[0] == (r + 1) % world  # the nearest source always comes from the next rank
                assert set(owners) == set(range(world))  # nine sources cover every rank of N <= 9


def test_rank_fields():
    """The N>1 attribution block: per-rank pass times, the
    depth all-gather's ms per step and the view counts, from each rank's
    [wall, photometric, all-gather, geometric, views] row summed over steps."""
    import bench
    rows = [[2.6, 1.2, 0.04, 1.3, 10.0], [2.7, 1.25, 0.02, 1.35, 10.0]]
    f = bench.rank_fields(rows, 2, "RCCL")
    assert f["world"] == 2 and f["views_per_rank"] == [10, 10]
    assert f["wall_s"] == {"min": 2.6, "max": 2.7}
    assert f["pass_s_per_step"] == {"min": 1.25, "max": 1.3}
    assert f["depth_allgather_ms_per_step"]["min"] == 10.0 and f["depth_allgather_ms_per_step"]["max"] == 20.0
    assert f["photometric_s_per_step"] == [0.6, 0.625]
    assert bench.rank_fields(rows[:1], 2, None)["depth_allgather_ms_per_step"] is None
