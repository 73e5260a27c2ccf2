"""The deterministic math shared by the kernels and the oracle
(include/acmmp_detmath.h): accuracy against float64 and the published
Philox4x32-10 known-answer vectors (Random123, Salmon et al. SC'11)."""
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


def test_uniform_is_curand_interval():
    """curand_uniform maps to (0, 1]: x * 2^-32 + 2^-33."""
    u = np.array([oracle.uniform(0x5EED, 0, pix, d, 1, 0) for pix in range(64) for d in range(16)])
    assert (u > 0).all() and (u <= 1).all()
    assert abs(u.mean() - 0.5) < 0.03
    assert len(np.unique(u)) == u.size
