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
    per = lambda d: {k: {0: v, 1: v} for k, v in d.items()}  # two dispatches
    return {"passes": {"fetch": {"counters": per(fetch), "durations_ms": [4.0, 4.0]},
                       "write": {"counters": per(write), "durations_ms": [4.0, 4.0]}}}


def test_summarize_fractions():
    s = bench_pmc.summarize(_passes())
    assert s["launches"] == 2
    assert abs(s["td_busy_frac"] - 2.048e9 / (1e7 * 256)) < 1e-12
    assert abs(s["valu_busy_frac"] - 4 * 1.92e9 / (1e7 * 256 * 4)) < 1e-12
    assert s["hbm_bytes"] == (2 * 1.0e6 + 3.0e5) * 1024
    assert abs(s["clock_ghz"] - 2.5) < 1e-12
    assert abs(s["tcp_accesses_per_gather"] - 36.0) < 1e-9


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
