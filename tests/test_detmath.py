"""The deterministic math shared by the kernels and the oracle
(include/acmmp_detmath.h): accuracy against float64 and the published
Philox4x32-10 known-answer vectors (Random123, Salmon et al. SC'11)."""
import os
import numpy as np
import pytest

import oracle


def _ulp_err(got, ref):
    got = np.float32(got)
    ref32 = np.float32(ref)
    if np.isnan(ref32):
        return 0 if np.isnan(got) else 1e9
    if ref32 == 0:
        return abs(float(got)) / np.finfo(np.float32).tiny
    return abs(float(got) - ref) / float(np.spacing(np.abs(ref32)))


@pytest.mark.parametrize("x", list(np.linspace(-103.0, 88.0, 97)) + [-0.5, -1e-3, 0.0, 1e-6, 0.693, 2.0])
def test_expf_accuracy(x):
    x = float(np.float32(x))
    assert _ulp_err(oracle.math_fn("expf", x), np.exp(np.float64(x))) <= 2.0


def test_expf_special_values():
    assert np.isnan(oracle.math_fn("expf", float("nan")))
    assert oracle.math_fn("expf", 100.0) == float("inf")
    assert oracle.math_fn("expf", -200.0) == 0.0
    assert oracle.math_fn("expf", 0.0) == 1.0


@pytest.mark.parametrize("fn,ref", [("sinf", np.sin), ("cosf", np.cos)])
def test_sincos_accuracy(fn, ref):
    xs = np.concatenate([np.linspace(-0.2, 0.2, 81), np.linspace(-4.0, 4.0, 81)]).astype(np.float32)
    for x in xs:
        r = ref(np.float64(x))
        got = oracle.math_fn(fn, float(x))
        assert abs(got - r) <= 2 * np.spacing(np.float32(max(abs(r), 1e-30))) + 1e-9, (fn, x, got, r)


def test_acosf_accuracy_and_domain():
    for x in np.linspace(-1.0, 1.0, 201).astype(np.float32):
        r = np.arccos(np.float64(x))
        got = oracle.math_fn("acosf", float(x))
        assert abs(got - r) <= 3 * np.spacing(np.float32(max(r, 1e-7))) + 1e-7, (x, got, r)
    assert np.isnan(oracle.math_fn("acosf", 1.0000001))
    assert np.isnan(oracle.math_fn("acosf", float("nan")))


def test_philox_known_answers():
    # Random123 kat_vectors, philox4x32_10, first output word
    assert oracle.philox_x(0, 0, 0, 0, 0, 0) == 0x6627E8D5
    assert oracle.philox_x(0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF) == 0x408F276D
    assert oracle.philox_x(0xA4093822, 0x299F31D0, 0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344) == 0xD16CFE09


def test_philox4_known_answers():
    # Random123 kat_vectors, philox4x32_10, all four output words
    assert oracle.philox4(0, 0, 0, 0, 0, 0) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert oracle.philox4(0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF) == \
        [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert oracle.philox4(0xA4093822, 0x299F31D0, 0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344) == \
        [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_draws_take_the_words_of_one_block_in_turn():
    """Draw d of (pix, phase, stream) is word d mod 4 of the Philox block with
    counter (pix, d div 4, phase, stream), in curand_uniform's mapping."""
    seed, pix, phase, stream = 0x5EED, 1234, 3, 7
    for d in range(12):
        words = oracle.philox4(seed, 0, pix, d // 4, phase, stream)
        x = np.float32(words[d % 4]) * np.float32(2.3283064365386963e-10) + np.float32(2.3283064365386963e-10 / 2)
        assert oracle.uniform(seed, 0, pix, d, phase, stream) == np.float32(x)


def test_uniform_is_curand_interval():
    """curand_uniform maps to (0, 1]: x * 2^-32 + 2^-33."""
    u = np.array([oracle.uniform(0x5EED, 0, pix, d, 1, 0) for pix in range(64) for d in range(16)])
    assert (u > 0).all() and (u <= 1).all()
    assert abs(u.mean() - 0.5) < 0.03
    assert len(np.unique(u)) == u.size


# ---------------------------------------------------------------------------
# Exact shortcuts of the view selection (k_sweep Phase A, src/ACMMP.cu:1017),
# checked for EVERY float of their domain by a small C program built from the
# shared header (the product kernel uses them; the oracle keeps IEEE x / -0.18f
# and dm_expf, so parity rests on these equalities).
_EXHAUSTIVE_C = r"""
#include <stdio.h>
#include <stdint.h>
#include "acmmp_detmath.h"
#include <omp.h>
static uint64_t splitmix(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
int main(void) {
    unsigned long long bad_div = 0, bad_exp = 0;
    /* x = c * c, c in {0} U [2^-24, 2]: x in {0} U [2^-48, 4]; checked from 2^-100 */
    const long long lo = 0x0d800000LL, hi = 0x40800000LL;
    #pragma omp parallel for reduction(+:bad_div) schedule(static)
    for (long long u = lo; u <= hi; ++u) {
        const float x = dm_u2f((uint32_t)u);
        volatile float d = -0.18f;
        if (dm_f2u(x / d) != dm_f2u(dm_div_neg018(x))) bad_div++;
    }
    { volatile float d = -0.18f; if (dm_f2u(0.0f / d) != dm_f2u(dm_div_neg018(0.0f))) bad_div++; }
    /* every float in [-87, 0] (-0 included), and +0 */
    const long long m87 = (long long)dm_f2u(-87.0f);
    #pragma omp parallel for reduction(+:bad_exp) schedule(static)
    for (long long u = 0x80000000LL; u <= m87; ++u) {
        const float x = dm_u2f((uint32_t)u);
        if (dm_f2u(dm_expf(x)) != dm_f2u(dm_expf_nonpos(x))) bad_exp++;
    }
    if (dm_f2u(dm_expf(0.0f)) != dm_f2u(dm_expf_nonpos(0.0f))) bad_exp++;
    /* (the round-6 A/B variant of DESIGN §5, not the product) the NCC quotient covar / var_rs as a Markstein quotient on the
     * exactly rounded reciprocal (the device's Newton reciprocal equals IEEE
     * 1/z in its window, acmmp_selftest_reciprocal): 1.6e9 random pairs,
     * var_rs normal in [2^-20, 2^20], covar 0 or of either sign in
     * [2^-60, 2^20]; the cost 1 - q must match (and q itself) */
    unsigned long long bad_ncc = 0;
    #pragma omp parallel reduction(+:bad_ncc)
    {
        uint64_t st = 12345u + 7919u * (uint64_t)omp_get_thread_num();
        for (long i = 0; i < 200000000L; ++i) {
            uint64_t r = splitmix(&st), r2 = splitmix(&st);
            const float v = dm_u2f(((127u - 20u + (uint32_t)(r % 41u)) << 23) | ((uint32_t)(r >> 8) & 0x7fffffu));
            float cv = dm_u2f((((uint32_t)(r2 >> 40) & 1u) << 31) | ((127u - 60u + (uint32_t)(r2 % 81u)) << 23) |
                              ((uint32_t)(r2 >> 8) & 0x7fffffu));
            if ((r2 & 0xffu) == 0u) cv = 0.0f;
            volatile float one = 1.0f;
            const float y = one / v;
            const float q0 = cv * y;
            const float q = dm_fma(dm_fma(-v, q0, cv), y, q0);
            const float qi = cv / v;
            if (dm_f2u(q) != dm_f2u(qi) || dm_f2u(1.0f - q) != dm_f2u(1.0f - qi)) bad_ncc++;
        }
    }
    printf("%llu %llu %llu\n", bad_div, bad_exp, bad_ncc);
    return 0;
}
"""


@pytest.fixture(scope="module")
def exhaustive_counts(tmp_path_factory):
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("gcc not installed")
    d = tmp_path_factory.mktemp("exh")
    src, exe = d / "exh.c", d / "exh"
    src.write_text(_EXHAUSTIVE_C)
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", "-fno-fast-math", "-I" + inc, "-o", str(exe),
                    str(src), "-lm"], check=True, timeout=120)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, check=True).stdout.split()
    return int(out[0]), int(out[1]), int(out[2])


def test_div_by_neg018_matches_ieee(exhaustive_counts):
    assert exhaustive_counts[0] == 0


def test_expf_nonpos_matches_expf(exhaustive_counts):
    assert exhaustive_counts[1] == 0


def test_ncc_markstein_quotient_matches_ieee(exhaustive_counts):
    assert exhaustive_counts[2] == 0
