"""ISA guards for k_sweep (CPU tier: hipcc cross-compiles the NS 9, u8-quad
instantiation to a gfx950 listing, as `make resource-dev` does). They pin the
round-4 latency fixes, which change no result and so no parity test would
notice losing them:
- no generic (flat) loads: a flat load also counts against lgkmcnt, so every
  later scalar/LDS wait would drain it (texel() reads through the global
  address space);
- the checkerboard searches' costs are in flight together (a load inside a
  condition is sunk into its block and waited alone: one latency per step);
- no resource regression: 2 waves/SIMD for every source-count bucket (NS 9,
  16, 20, 32), scratch no larger than recorded per bucket, LDS within two
  blocks per CU.
The search-cost check reads a scheduling depth (the deepest vmcnt wait), a
property of this compiler's schedule, not of the source: it runs only under
the hipcc it was tuned on (ROCm 7.2.0) and must be re-tuned on an upgrade.
Resources and flat loads are checked under any hipcc."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "acmmp_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"

pytestmark = pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")


@pytest.fixture(scope="module")
def listing(tmp_path_factory):
    out = tmp_path_factory.mktemp("isa") / "dev_kernels.s"
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
           "-fno-slp-vectorize", "-I../../include", "-DACMMP_DEV_SUBSET", "-DACMMP_DEV_ALL_NS", "--cuda-device-only", "-S",
           "acmmp_kernels.hip", "-o", str(out), "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, cwd=CSRC, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    text = out.read_text()
    lines = text.splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_ZN5acmmp9k_sweep_fILi9ELi2EE\S*:", l))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    return lines[start:end + 1], r.stderr


def test_no_flat_loads_in_k_sweep(listing):
    body, _ = listing
    flat = [l.strip() for l in body if re.match(r"\s+flat_load", l)]
    assert not flat, flat[:5]


TUNED_HIPCC = "roc-7.2.0"  # the compiler whose schedule the vmcnt threshold was read from


def _hipcc_version():
    r = subprocess.run([HIPCC, "--version"], capture_output=True, text=True, timeout=60)
    return r.stdout + r.stderr


def test_search_costs_in_flight_together(listing):
    if TUNED_HIPCC not in _hipcc_version():
        pytest.skip(f"vmcnt depth threshold tuned on {TUNED_HIPCC}; re-tune it for this hipcc")
    body, _ = listing
    # the 72 search costs are issued before the first comparison: the
    # deepest vmcnt wait of the kernel reaches the counter's limit (63)
    depths = [int(m.group(1)) for l in body for m in [re.match(r"\s+s_waitcnt vmcnt\((\d+)\)", l)] if m]
    assert max(depths) >= 60, max(depths)


# scratch per lane of each bucket at round 5 (cost_array[8][NS] dominates)
SCRATCH_MAX = {9: 384, 16: 672, 20: 816, 32: 1264}
LDS_MAX = 160 * 1024 // 2  # two 256-thread blocks per CU (2 waves/SIMD)


@pytest.mark.parametrize("ns", sorted(SCRATCH_MAX))
def test_resources(listing, ns):
    _, remarks = listing
    tag = f"Function Name: _ZN5acmmp9k_sweep_fILi{ns}ELi2EE"
    assert tag in remarks, f"k_sweep_f<{ns}, u8> not instantiated"
    sweep = remarks[remarks.index(tag):]
    sweep = sweep[:sweep.index("Function Name:", len(tag))] if "Function Name:" in sweep[len(tag):] else sweep
    occ = int(re.search(r"Occupancy \[waves/SIMD\]: (\d+)", sweep).group(1))
    scratch = int(re.search(r"ScratchSize \[bytes/lane\]: (\d+)", sweep).group(1))
    lds = int(re.search(r"LDS Size \[bytes/block\]: (\d+)", sweep).group(1))
    assert occ == 2 and scratch <= SCRATCH_MAX[ns] and lds <= LDS_MAX, (ns, occ, scratch, lds)
