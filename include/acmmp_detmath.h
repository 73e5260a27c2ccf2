/*
 * acmmp_detmath.h — deterministic float32 math shared by the HIP kernels and the
 * CPU oracle.
 *
 * Why this exists: the reference compiles src/ACMMP.cu with `--use_fast_math`
 * (src/CMakeLists.txt:19), so its transcendentals are NVIDIA hardware
 * approximations (`__expf`, `__sinf`, approximate rsqrt) whose exact bits are
 * unknowable here. PatchMatch is an argmin cascade: one ulp of difference in an
 * exp() flips accept decisions. To make the GPU path and the CPU oracle agree
 * bit-for-bit we pin every transcendental to ONE polynomial implementation
 * built only from IEEE-exact operations (+ - * /, sqrt, fma, floor, compares),
 * which gcc (x86-64) and hipcc (gfx950) both evaluate identically provided
 * both sides compile with -ffp-contract=off and without -ffast-math.
 *
 * This header is math-library plumbing (the stand-in for libm/CUDA intrinsics),
 * not part of the PatchMatch algorithm; the algorithm itself is written twice,
 * independently: oracle/acmmp_oracle.c (literal restatement) and
 * acmmp_amd/csrc/acmmp_kernels.hip (MI355X kernels).
 *
 * Accuracy: expf/sinf/cosf/acosf within ~2 ulp of the correctly rounded value
 * over the ranges PatchMatch uses (checked in tests/test_detmath.py against
 * numpy float64).
 */
#ifndef ACMMP_DETMATH_H_
#define ACMMP_DETMATH_H_

#include <stdint.h>

#if defined(__HIPCC__)
#define DM_FN static __host__ __device__ __forceinline__
#else
#define DM_FN static inline
#endif

/* bit casts without memcpy so both compilers fold them */
DM_FN uint32_t dm_f2u(float f) { union { float f; uint32_t u; } c; c.f = f; return c.u; }
DM_FN float dm_u2f(uint32_t u) { union { float f; uint32_t u; } c; c.u = u; return c.f; }

DM_FN float dm_fma(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
DM_FN float dm_sqrt(float x) { return __builtin_sqrtf(x); }          /* IEEE, correctly rounded */
DM_FN float dm_floor(float x) { return __builtin_floorf(x); }
DM_FN float dm_fabs(float x) { return dm_u2f(dm_f2u(x) & 0x7fffffffu); }

/* rsqrtf(x) in NormalizeVec3 (src/ACMMP.cu:101) is pinned to 1/sqrt(x). */
DM_FN float dm_rsqrt(float x) { return 1.0f / dm_sqrt(x); }

/* 2^k for integer k in [-126, 127] */
DM_FN float dm_pow2i(int k) { return dm_u2f((uint32_t)(k + 127) << 23); }

/* expf: Cody-Waite reduction x = k ln2 + r, |r| <= ln2/2, degree-6 minimax
 * polynomial for e^r, then scaling by 2^k in two steps so gradual underflow
 * is handled. NaN -> NaN, x > 88.73 -> +inf, x < -103.98 -> +0. */
DM_FN float dm_expf(float x) {
    if (!(x == x)) return x;                       /* NaN */
    if (x > 88.72283935546875f) return dm_u2f(0x7f800000u);
    if (x < -103.972084045410f) return 0.0f;
    const float kLog2e = 1.44269502162933349609375f;
    const float kLn2Hi = 0.693145751953125f;       /* 12 significant bits */
    const float kLn2Lo = 1.428606765330187045e-06f;
    const float kShift = 12582912.0f;              /* 1.5 * 2^23: round-to-nearest-even trick */
    float t = x * kLog2e;
    float kf = (t + kShift) - kShift;
    float r = dm_fma(-kf, kLn2Hi, x);
    r = dm_fma(-kf, kLn2Lo, r);
    /* e^r ~ 1 + r + r^2 * P(r) (Horner with fma) */
    float p = 1.9875691500e-4f;
    p = dm_fma(p, r, 1.3981999507e-3f);
    p = dm_fma(p, r, 8.3334519073e-3f);
    p = dm_fma(p, r, 4.1665795894e-2f);
    p = dm_fma(p, r, 1.6666665459e-1f);
    p = dm_fma(p, r, 5.0000001201e-1f);
    float r2 = r * r;
    float er = dm_fma(p, r2, r) + 1.0f;
    int k = (int)kf;
    /* scale in two steps: k in [-150, 128] */
    int k1 = k / 2;
    int k2 = k - k1;
    return (er * dm_pow2i(k1)) * dm_pow2i(k2);
}

/* dm_expf on x in [-87, 0], for arguments known to lie there (the view
 * selection's exp(-c^2 / 0.18), c in [0, 2]): dm_expf's common path without
 * its NaN / overflow / underflow branches, and the scaling by 2^k (k in
 * [-126, 0]) in one step, which is exact there as the two-step product is.
 * Bit-identical to dm_expf for every float in [-87, 0]: checked exhaustively
 * (tests/test_detmath.py::test_expf_nonpos_matches_expf). */
DM_FN float dm_expf_nonpos(float x) {
    const float kLog2e = 1.44269502162933349609375f;
    const float kLn2Hi = 0.693145751953125f;
    const float kLn2Lo = 1.428606765330187045e-06f;
    const float kShift = 12582912.0f;
    float t = x * kLog2e;
    float kf = (t + kShift) - kShift;
    float r = dm_fma(-kf, kLn2Hi, x);
    r = dm_fma(-kf, kLn2Lo, r);
    float p = 1.9875691500e-4f;
    p = dm_fma(p, r, 1.3981999507e-3f);
    p = dm_fma(p, r, 8.3334519073e-3f);
    p = dm_fma(p, r, 4.1665795894e-2f);
    p = dm_fma(p, r, 1.6666665459e-1f);
    p = dm_fma(p, r, 5.0000001201e-1f);
    float r2 = r * r;
    float er = dm_fma(p, r2, r) + 1.0f;
    return er * dm_pow2i((int)kf);
}

/* x / -0.18f for x in [0, 4] (the squared NCC costs of the view selection,
 * src/ACMMP.cu:1017): q = x * RN(1 / -0.18), one fma residual, one fma
 * correction (Markstein). Equal to the IEEE quotient for every float in
 * [0, 4]: checked exhaustively (tests/test_detmath.py::
 * test_div_by_neg018_matches_ieee). */
DM_FN float dm_div_neg018(float x) {
    const float r = 1.0f / -0.18f;  /* constant-folded, correctly rounded */
    const float q = x * r;
    const float e = dm_fma(0.18f, q, x);  /* x - (-0.18) q, exact */
    return dm_fma(e, r, q);
}

/* sinf/cosf: Cephes single-precision reduction by pi/4 (3-part constant) and
 * the Cephes minimax polynomials. Valid for |x| < 8192 (PatchMatch only uses
 * |x| < 0.1: perturbation angles, src/ACMMP.cu:202-211). */
DM_FN float dm_sincos_reduce(float x, int *quadrant) {
    const float kFourOverPi = 1.27323954473516f;
    const float kDP1 = 0.78515625f;
    const float kDP2 = 2.4187564849853515625e-4f;
    const float kDP3 = 3.77489497744594108e-8f;
    int j = (int)(x * kFourOverPi);
    float y = (float)j;
    if (j & 1) { j += 1; y += 1.0f; }
    *quadrant = j & 7;
    return ((x - y * kDP1) - y * kDP2) - y * kDP3;
}
DM_FN float dm_sin_poly(float z) {   /* |z| <= pi/4 */
    float zz = z * z;
    float p = dm_fma(-1.9515295891e-4f, zz, 8.3321608736e-3f);
    p = dm_fma(p, zz, -1.6666654611e-1f);
    return dm_fma(p * zz, z, z);
}
DM_FN float dm_cos_poly(float z) {   /* |z| <= pi/4 */
    float zz = z * z;
    float p = dm_fma(2.443315711809948e-5f, zz, -1.388731625493765e-3f);
    p = dm_fma(p, zz, 4.166664568298827e-2f);
    return dm_fma(p * zz, zz, dm_fma(-0.5f, zz, 1.0f));
}
DM_FN float dm_sinf(float x) {
    if (!(x == x)) return x;
    float sign = 1.0f;
    if (x < 0.0f) { x = -x; sign = -1.0f; }
    int q;
    float z = dm_sincos_reduce(x, &q);
    if (q > 3) { sign = -sign; q -= 4; }
    float v = (q == 1 || q == 2) ? dm_cos_poly(z) : dm_sin_poly(z);
    return sign * v;
}
DM_FN float dm_cosf(float x) {
    if (!(x == x)) return x;
    if (x < 0.0f) x = -x;
    int q;
    float z = dm_sincos_reduce(x, &q);
    float sign = 1.0f;
    if (q > 3) { q -= 4; sign = -sign; }
    if (q > 1) sign = -sign;
    float v = (q == 1 || q == 2) ? dm_sin_poly(z) : dm_cos_poly(z);
    return sign * v;
}

/* asinf core on [0, 1] (Cephes): returns asin(a) for a >= 0. */
DM_FN float dm_asin_pos(float a) {
    float z, x;
    int big = a > 0.5f;
    if (big) { z = 0.5f * (1.0f - a); x = dm_sqrt(z); }
    else { x = a; z = x * x; }
    float p = dm_fma(4.2163199048e-2f, z, 2.4181311049e-2f);
    p = dm_fma(p, z, 4.5470025998e-2f);
    p = dm_fma(p, z, 7.4953002686e-2f);
    p = dm_fma(p, z, 1.6666752422e-1f);
    float r = dm_fma(p * z, x, x);
    if (big) { r = r + r; r = 1.5707963267948966f - r; }
    return r;
}
/* acosf (src/ACMMP.cu:766, :1111, :1122): NaN outside [-1, 1] like CUDA acosf. */
DM_FN float dm_acosf(float x) {
    if (!(x >= -1.0f && x <= 1.0f)) return dm_u2f(0x7fc00000u);
    const float kPi = 3.14159265358979f;
    if (x < -0.5f) return kPi - 2.0f * dm_asin_pos(dm_sqrt(0.5f * (1.0f + x)));
    if (x > 0.5f) return 2.0f * dm_asin_pos(dm_sqrt(0.5f * (1.0f - x)));
    float s = (x < 0.0f) ? -dm_asin_pos(-x) : dm_asin_pos(x);
    return 1.5707963267948966f - s;
}

/* ---------------------------------------------------------------------------
 * Counter-based RNG: Philox4x32-10 (Salmon et al., SC'11), replacing the
 * reference's per-pixel curand XORWOW seeded from clock64()
 * (src/ACMMP.cu:624). Stateless: draw d of pixel `pix` in phase `phase` of
 * run `stream` is word d mod 4 of philox(key=seed, ctr={pix, d div 4, phase,
 * stream}), so one Philox block serves four consecutive draws (r06; before,
 * one block per draw, word 0 only).
 * The uniform mapping is curand_uniform's (0,1]: x * 2^-32 + 2^-33.
 * ------------------------------------------------------------------------- */
DM_FN uint32_t dm_mulhi32(uint32_t a, uint32_t b) {
    return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}
/* the four output words of one Philox4x32-10 block */
typedef struct dm_u32x4 {
    uint32_t x, y, z, w;
} dm_u32x4;
DM_FN dm_u32x4 dm_philox4(uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
    for (int r = 0; r < 10; ++r) {
        uint32_t hi0 = dm_mulhi32(M0, c0), lo0 = M0 * c0;
        uint32_t hi1 = dm_mulhi32(M1, c2), lo1 = M1 * c2;
        uint32_t n0 = hi1 ^ c1 ^ k0;
        uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += W0; k1 += W1;
    }
    dm_u32x4 o;
    o.x = c0; o.y = c1; o.z = c2; o.w = c3;
    return o;
}
DM_FN uint32_t dm_philox_x(uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1,
                           uint32_t c2, uint32_t c3) {
    return dm_philox4(k0, k1, c0, c1, c2, c3).x;
}
DM_FN float dm_uniform(uint32_t x) {
    const float kInv2Pow32 = 2.3283064365386963e-10f;
    return (float)x * kInv2Pow32 + (kInv2Pow32 / 2.0f);
}

/* Per-pixel generator handle: the counter fields and the current block. */
typedef struct dm_rng {
    uint32_t k0, k1;      /* seed */
    uint32_t pix;         /* ref-image pixel index y*W+x */
    uint32_t phase;       /* 0 = RandomInitialization, 1+i = iteration i */
    uint32_t stream;      /* RunPatchMatch call index on the engine */
    uint32_t draw;        /* running draw counter within (pix, phase) */
    dm_u32x4 blk;         /* block draw / 4 (valid from the draw that fills it) */
} dm_rng;

DM_FN float dm_rng_uniform(dm_rng *g) {
    const uint32_t w = g->draw & 3u;
    if (w == 0u) g->blk = dm_philox4(g->k0, g->k1, g->pix, g->draw >> 2, g->phase, g->stream);
    const uint32_t x = w == 0u ? g->blk.x : w == 1u ? g->blk.y : w == 2u ? g->blk.z : g->blk.w;
    g->draw += 1u;
    return dm_uniform(x);
}


/* Fidelity-study builds only (-DACMMP_CUDA_NUMERICS, tools/fidelity_study.py):
 * device code takes the reference's --use_fast_math intrinsics
 * (src/CMakeLists.txt:19) instead of the pinned functions. Such a build is
 * NOT bit-exact with the oracle and never ships. */
#if defined(ACMMP_CUDA_NUMERICS) && defined(__HIP_DEVICE_COMPILE__)
#define dm_expf(x) __expf(x)
#define dm_sinf(x) __sinf(x)
#define dm_cosf(x) __cosf(x)
#endif
#endif /* ACMMP_DETMATH_H_ */
