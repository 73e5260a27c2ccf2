/*
 * acmmp_oracle.c — CPU restatement of the reference's PatchMatch hot path.
 *
 * TEST INFRASTRUCTURE ONLY. This file is the parity oracle and the CPU
 * baseline ("kind": "port"). Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it; the product (acmmp_amd/) never
 * links, calls or falls back to it.
 *
 * PARITY UNPINNED against reference outputs: the reference engine cannot be
 * built here (nvcc/CUDA, cuRAND, OpenCV, Boost absent) and seeds its RNG from
 * clock64(), and no reference test or fixture holds PatchMatch outputs. The
 * restatement is pinned by analytic known-answer tests, the Random123
 * Philox4x32-10 vectors and fixtures the reference's own colmap2mvsnet_acm.py
 * produced (tests/test_oracle_kat.py, tests/golden/).
 *
 * What it restates (line by line, one C function per reference function):
 *   rlav440/ACMMP src/ACMMP.cu:24-1352 (device code) and :1378-1456 (RunPatchMatch).
 * With the pinned semantics of SURVEY.md Appendix A:
 *   A1 RNG: curand XORWOW seeded by clock64() (src/ACMMP.cu:624) -> stateless
 *      Philox4x32-10, counter (pixel, draw#, phase, run) — include/acmmp_detmath.h.
 *   A2 same-colour reads (near "V" searches, src/ACMMP.cu:895-988) read a
 *      snapshot taken at the start of each half-sweep.
 *   A3 uninitialised `plane_hypotheses_now` (src/ACMMP.cu:1149) is initialised
 *      to plane_hypotheses[center] as it stands at that line.
 *   A4 tex2D linear/clamp: software bilinear with fp32 weights; NaN/huge
 *      coordinates clamp to the edge texel (pin P2 below).
 *   A6 --use_fast_math transcendentals -> include/acmmp_detmath.h.
 * Arithmetic pins shared with the HIP kernels (documented in DESIGN.md §4):
 *   P1 ComputeCorrespondingPoint (src/ACMMP.cu:324-331): each homogeneous
 *      coordinate is fma(H1,y,fma(H0,x,H2)) (the inner term is constant along
 *      a patch column); the divide is 1/z then two multiplies (what
 *      --use_fast_math's x*rcp(z) does, but exactly rounded).
 *   P2 bilinear: xs=(u+0.5)-0.5, clamp to [-1,W] by compare-select (NaN->-1),
 *      x0=floor, a=xs-x0, texels clamp-to-edge, lerp = fma(a, t1-t0, t0).
 *   P4 ComputeHomography (src/ACMMP.cu:292-311): x/w, x/K[0], x/K[4] are
 *      x*(1/w), x*(1/K[0]), x*(1/K[4]) with the reciprocal exactly rounded.
 *   P3 NCC sums and moments (src/ACMMP.cu:382-430) as nvcc's default
 *      contraction (--fmad=true, implied by the reference's --use_fast_math,
 *      src/CMakeLists.txt:19) forms them: per sample row_s=fma(w,s,row_s),
 *      row_ss=fma(w*s,s,row_ss), row_rs=fma(w*r,s,row_rs), ref side likewise
 *      (row_r=fma(w,r,row_r); row_rr=fma(w*r,r,row_rr); row_w+=w); then
 *      with m=sum*inv, var=fma(sum_xx,inv,-(m*m)), covar=fma(sum_rs,inv,
 *      -(m_r*m_s)) (LLVM's fsub combine fuses the first fmul operand; the
 *      scaled moments have no other use). r01 pinned all of this unfused.
 *   Everything else is the reference expression, evaluated left to right in
 *   IEEE fp32 with no FMA contraction (-ffp-contract=off).
 *
 * Parity status: the reference cannot be built or run here (CUDA/cuRAND/OpenCV
 * absent) and ships no tests or fixtures for this path, so this
 * restatement is "parity unpinned" against reference outputs; it is pinned by
 * analytic known-answer tests (tests/test_oracle_kat.py: analytic answers, an fp64 restatement
 * of the NCC/homography/geometric cost, bit-exact init-cost aggregation) and by the
 * reference converter's cams/pair fixtures for the I/O formats.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/acmmp.h"
#include "../include/acmmp_detmath.h"

typedef struct { float x, y, z, w; } f4;
typedef struct { float x, y; } f2;
typedef struct { float x, y, z; } f3;
typedef struct { int x, y; } i2;

#define MAXSRC 32

/* ------------------------------------------------------------------ state */
typedef struct {
    const acmmp_params *prm;
    int n;                              /* num_images */
    const acmmp_camera *cams;
    const float *const *imgs;
    const float *const *depths;         /* geometric consistency maps (may be NULL) */
    const int *depth_w, *depth_h;       /* per-view depth map sizes */
    int W, H;
    int sweep_rows;                     /* rows the checkerboard grid covers */
    f4 *planes;
    float *costs;
    uint32_t *sv;
    float *pre_costs;
    const f4 *prior_planes;
    const uint32_t *masks;
    const f4 *scaled_planes;
    const f4 *seed_planes;
    /* snapshot (pin A2) */
    f4 *snap_planes;
    float *snap_costs;
} orc_state;

/* ------------------------------------------------------------ texture pins */
/* tex2D<float>(img, x+0.5f, y+0.5f) at integer (x,y): the exact texel,
 * clamp-to-edge (src/ACMMP.cu:380, :392). */
static float tex_texel(const float *img, int W, int H, int x, int y) {
    x = x < 0 ? 0 : (x > W - 1 ? W - 1 : x);
    y = y < 0 ? 0 : (y > H - 1 ? H - 1 : y);
    return img[(size_t)y * W + x];
}

/* texture_filter8 (acmmp_params): the CUDA texture unit's 1.8 fixed-point
 * fraction, rounded half-even to 1/256 (x * 256 and the scale back are exact). */
static float frac8(float a) { return rintf(a * 256.0f) * 0.00390625f; }

/* Pin P2: tex2D linear at (u+0.5, v+0.5) (src/ACMMP.cu:394); q8 = the
 * emulated 8-bit fractions of cudaFilterModeLinear instead of pin A4's fp32. */
static float tex_bilinear(const float *img, int W, int H, float u, float v, int q8) {
    float xs = (u + 0.5f) - 0.5f;
    float ys = (v + 0.5f) - 0.5f;
    float fw = (float)W, fh = (float)H;
    xs = (xs > -1.0f) ? xs : -1.0f;
    xs = (xs < fw) ? xs : fw;
    ys = (ys > -1.0f) ? ys : -1.0f;
    ys = (ys < fh) ? ys : fh;
    float fx0 = dm_floor(xs), fy0 = dm_floor(ys);
    float ax = xs - fx0, ay = ys - fy0;
    if (q8) {
        ax = frac8(ax);
        ay = frac8(ay);
    }
    int x0 = (int)fx0, y0 = (int)fy0;
    float t00 = tex_texel(img, W, H, x0, y0);
    float t10 = tex_texel(img, W, H, x0 + 1, y0);
    float t01 = tex_texel(img, W, H, x0, y0 + 1);
    float t11 = tex_texel(img, W, H, x0 + 1, y0 + 1);
    float top = dm_fma(ax, t10 - t00, t00);
    float bot = dm_fma(ax, t11 - t01, t01);
    return dm_fma(ay, bot - top, top);
}

/* tex2D(depth, (int)x + 0.5f, (int)y + 0.5f) (src/ACMMP.cu:528): truncation
 * toward zero, clamp-to-edge; NaN/huge coordinates clamp first (pin). */
static float tex_trunc(const float *img, int W, int H, float u, float v) {
    float fw = (float)W, fh = (float)H;
    u = (u > -1.0f) ? u : -1.0f;
    u = (u < fw) ? u : fw;
    v = (v > -1.0f) ? v : -1.0f;
    v = (v < fh) ? v : fh;
    return tex_texel(img, W, H, (int)u, (int)v);
}

/* --------------------------------------------------------- small helpers */
/* sort_small (src/ACMMP.cu:24-33) */
static void sort_small(float *d, const int n) {
    int j;
    for (int i = 1; i < n; i++) {
        float tmp = d[i];
        for (j = i; j >= 1 && tmp < d[j - 1]; j--) d[j] = d[j - 1];
        d[j] = tmp;
    }
}

/* FindMinCostIndex (src/ACMMP.cu:50-61): `<=`, last index wins */
static int FindMinCostIndex(const float *costs, const int n) {
    float min_cost = costs[0];
    int idx_min = 0;
    for (int idx = 1; idx < n; ++idx)
        if (costs[idx] <= min_cost) { min_cost = costs[idx]; idx_min = idx; }
    return idx_min;
}

/* FindMaxCostIndex (src/ACMMP.cu:63-74) */
static int FindMaxCostIndex(const float *costs, const int n) {
    float max_cost = costs[0];
    int idx_max = 0;
    for (int idx = 1; idx < n; ++idx)
        if (costs[idx] >= max_cost) { max_cost = costs[idx]; idx_max = idx; }
    return idx_max;
}

static void setBit(uint32_t *input, const unsigned n) { *input |= (uint32_t)(1u << n); }
static int isSet(uint32_t input, const unsigned n) { return (input >> n) & 1; }

/* Mat33DotVec3 (src/ACMMP.cu:86-91) */
static f4 Mat33DotVec3(const float m[9], const f4 v) {
    f4 r;
    r.x = m[0] * v.x + m[1] * v.y + m[2] * v.z;
    r.y = m[3] * v.x + m[4] * v.y + m[5] * v.z;
    r.z = m[6] * v.x + m[7] * v.y + m[8] * v.z;
    r.w = v.w;  /* result->w untouched in the reference: caller's value */
    return r;
}

/* Vec3DotVec3 (src/ACMMP.cu:93-96) */
static float Vec3DotVec3(const f4 a, const f4 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

/* NormalizeVec3 (src/ACMMP.cu:98-105), rsqrtf pinned to 1/sqrt */
static void NormalizeVec3(f4 *v) {
    const float n2 = v->x * v->x + v->y * v->y + v->z * v->z;
    const float inv = dm_rsqrt(n2);
    v->x *= inv;
    v->y *= inv;
    v->z *= inv;
}

/* TransformPDFToCDF (src/ACMMP.cu:107-121) */
static void TransformPDFToCDF(float *probs, const int num) {
    float sum = 0.0f;
    for (int i = 0; i < num; ++i) sum += probs[i];
    const float inv = 1.0f / sum;
    float cum = 0.0f;
    for (int i = 0; i < num; ++i) {
        const float prob = probs[i] * inv;
        cum += prob;
        probs[i] = cum;
    }
}

/* Get3DPoint (src/ACMMP.cu:123-128) */
static void Get3DPoint(const acmmp_camera *c, const i2 p, const float depth, float *X) {
    X[0] = depth * ((float)p.x - c->K[2]) / c->K[0];
    X[1] = depth * ((float)p.y - c->K[5]) / c->K[4];
    X[2] = depth;
}

/* GetViewDirection (src/ACMMP.cu:130-142) */
static f4 GetViewDirection(const acmmp_camera *c, const i2 p, const float depth) {
    float X[3];
    Get3DPoint(c, p, depth, X);
    float norm = dm_sqrt(X[0] * X[0] + X[1] * X[1] + X[2] * X[2]);
    f4 v;
    v.x = X[0] / norm;
    v.y = X[1] / norm;
    v.z = X[2] / norm;
    v.w = 0;
    return v;
}

/* GetDistance2Origin (src/ACMMP.cu:144-149) */
static float GetDistance2Origin(const acmmp_camera *c, const i2 p, const float depth, const f4 n) {
    float X[3];
    Get3DPoint(c, p, depth, X);
    return -(n.x * X[0] + n.y * X[1] + n.z * X[2]);
}

/* ComputeDepthfromPlaneHypothesis (src/ACMMP.cu:163-168) */
static float ComputeDepthfromPlaneHypothesis(const acmmp_camera *c, const f4 h, const i2 p) {
    return -h.w * c->K[0] /
           (((float)p.x - c->K[2]) * h.x + (c->K[0] / c->K[4]) * ((float)p.y - c->K[5]) * h.y +
            c->K[0] * h.z);
}

/* GenerateRandomNormal (src/ACMMP.cu:170-196). The rejection loop is capped
 * at 1000 rounds (pin; probability of reaching it < 1e-600). */
static f4 GenerateRandomNormal(const acmmp_camera *c, const i2 p, dm_rng *rs, const float depth) {
    f4 normal;
    float q1 = 1.0f, q2 = 1.0f, s = 2.0f;
    int guard = 0;
    while (s >= 1.0f && guard < 1000) {
        q1 = 2.0f * dm_rng_uniform(rs) - 1.0f;
        q2 = 2.0f * dm_rng_uniform(rs) - 1.0f;
        s = q1 * q1 + q2 * q2;
        ++guard;
    }
    const float sq = dm_sqrt(1.0f - s);
    normal.x = 2.0f * q1 * sq;
    normal.y = 2.0f * q2 * sq;
    normal.z = 1.0f - 2.0f * s;
    normal.w = 0;
    f4 vd = GetViewDirection(c, p, depth);
    float dot = normal.x * vd.x + normal.y * vd.y + normal.z * vd.z;
    if (dot > 0.0f) {
        normal.x = -normal.x;
        normal.y = -normal.y;
        normal.z = -normal.z;
    }
    NormalizeVec3(&normal);
    return normal;
}

/* GeneratePerturbedNormal (src/ACMMP.cu:198-233) */
static f4 GeneratePerturbedNormal(const acmmp_camera *c, const i2 p, const f4 normal, dm_rng *rs,
                                  const float perturbation) {
    f4 vd = GetViewDirection(c, p, 1.0f);
    const float a1 = (dm_rng_uniform(rs) - 0.5f) * perturbation;
    const float a2 = (dm_rng_uniform(rs) - 0.5f) * perturbation;
    const float a3 = (dm_rng_uniform(rs) - 0.5f) * perturbation;
    const float s1 = dm_sinf(a1), s2 = dm_sinf(a2), s3 = dm_sinf(a3);
    const float c1 = dm_cosf(a1), c2 = dm_cosf(a2), c3 = dm_cosf(a3);
    float R[9];
    R[0] = c2 * c3;
    R[1] = c3 * s1 * s2 - c1 * s3;
    R[2] = s1 * s3 + c1 * c3 * s2;
    R[3] = c2 * s3;
    R[4] = c1 * c3 + s1 * s2 * s3;
    R[5] = c1 * s2 * s3 - c3 * s1;
    R[6] = -s2;
    R[7] = c2 * s1;
    R[8] = c1 * c2;
    f4 np = Mat33DotVec3(R, normal);
    if (Vec3DotVec3(np, vd) >= 0.0f) np = normal;
    NormalizeVec3(&np);
    return np;
}

/* GenerateRandomPlaneHypothesis (src/ACMMP.cu:235-241) */
static f4 GenerateRandomPlaneHypothesis(const acmmp_camera *c, const i2 p, dm_rng *rs,
                                        const float dmin, const float dmax) {
    float depth = dm_rng_uniform(rs) * (dmax - dmin) + dmin;
    f4 h = GenerateRandomNormal(c, p, rs, depth);
    h.w = GetDistance2Origin(c, p, depth, h);
    return h;
}

/* ComputeHomography (src/ACMMP.cu:262-322), literal except pin P4. */
static void ComputeHomography(const acmmp_camera *rc, const acmmp_camera *sc, const f4 h, float *H) {
    float ref_C[3], src_C[3];
    ref_C[0] = -(rc->R[0] * rc->t[0] + rc->R[3] * rc->t[1] + rc->R[6] * rc->t[2]);
    ref_C[1] = -(rc->R[1] * rc->t[0] + rc->R[4] * rc->t[1] + rc->R[7] * rc->t[2]);
    ref_C[2] = -(rc->R[2] * rc->t[0] + rc->R[5] * rc->t[1] + rc->R[8] * rc->t[2]);
    src_C[0] = -(sc->R[0] * sc->t[0] + sc->R[3] * sc->t[1] + sc->R[6] * sc->t[2]);
    src_C[1] = -(sc->R[1] * sc->t[0] + sc->R[4] * sc->t[1] + sc->R[7] * sc->t[2]);
    src_C[2] = -(sc->R[2] * sc->t[0] + sc->R[5] * sc->t[1] + sc->R[8] * sc->t[2]);
    float Rr[9], Cr[3], tr[3];
    Rr[0] = sc->R[0] * rc->R[0] + sc->R[1] * rc->R[1] + sc->R[2] * rc->R[2];
    Rr[1] = sc->R[0] * rc->R[3] + sc->R[1] * rc->R[4] + sc->R[2] * rc->R[5];
    Rr[2] = sc->R[0] * rc->R[6] + sc->R[1] * rc->R[7] + sc->R[2] * rc->R[8];
    Rr[3] = sc->R[3] * rc->R[0] + sc->R[4] * rc->R[1] + sc->R[5] * rc->R[2];
    Rr[4] = sc->R[3] * rc->R[3] + sc->R[4] * rc->R[4] + sc->R[5] * rc->R[5];
    Rr[5] = sc->R[3] * rc->R[6] + sc->R[4] * rc->R[7] + sc->R[5] * rc->R[8];
    Rr[6] = sc->R[6] * rc->R[0] + sc->R[7] * rc->R[1] + sc->R[8] * rc->R[2];
    Rr[7] = sc->R[6] * rc->R[3] + sc->R[7] * rc->R[4] + sc->R[8] * rc->R[5];
    Rr[8] = sc->R[6] * rc->R[6] + sc->R[7] * rc->R[7] + sc->R[8] * rc->R[8];
    Cr[0] = (ref_C[0] - src_C[0]);
    Cr[1] = (ref_C[1] - src_C[1]);
    Cr[2] = (ref_C[2] - src_C[2]);
    tr[0] = sc->R[0] * Cr[0] + sc->R[1] * Cr[1] + sc->R[2] * Cr[2];
    tr[1] = sc->R[3] * Cr[0] + sc->R[4] * Cr[1] + sc->R[5] * Cr[2];
    tr[2] = sc->R[6] * Cr[0] + sc->R[7] * Cr[1] + sc->R[8] * Cr[2];

    /* pin P4: the divisions by the plane's w and by K[0], K[4] are
     * reciprocal-multiplies (what --use_fast_math compiles them to), exactly
     * rounded: inv = 1/w once, then (t*n)*inv. */
    const float inv_w = 1.0f / h.w;
    H[0] = Rr[0] - (tr[0] * h.x) * inv_w;
    H[1] = Rr[1] - (tr[0] * h.y) * inv_w;
    H[2] = Rr[2] - (tr[0] * h.z) * inv_w;
    H[3] = Rr[3] - (tr[1] * h.x) * inv_w;
    H[4] = Rr[4] - (tr[1] * h.y) * inv_w;
    H[5] = Rr[5] - (tr[1] * h.z) * inv_w;
    H[6] = Rr[6] - (tr[2] * h.x) * inv_w;
    H[7] = Rr[7] - (tr[2] * h.y) * inv_w;
    H[8] = Rr[8] - (tr[2] * h.z) * inv_w;

    const float ik0 = 1.0f / rc->K[0], ik4 = 1.0f / rc->K[4];
    float tmp[9];
    tmp[0] = H[0] * ik0;
    tmp[1] = H[1] * ik4;
    tmp[2] = ((-H[0] * rc->K[2]) * ik0 - (H[1] * rc->K[5]) * ik4) + H[2];
    tmp[3] = H[3] * ik0;
    tmp[4] = H[4] * ik4;
    tmp[5] = ((-H[3] * rc->K[2]) * ik0 - (H[4] * rc->K[5]) * ik4) + H[5];
    tmp[6] = H[6] * ik0;
    tmp[7] = H[7] * ik4;
    tmp[8] = ((-H[6] * rc->K[2]) * ik0 - (H[7] * rc->K[5]) * ik4) + H[8];

    H[0] = sc->K[0] * tmp[0] + sc->K[2] * tmp[6];
    H[1] = sc->K[0] * tmp[1] + sc->K[2] * tmp[7];
    H[2] = sc->K[0] * tmp[2] + sc->K[2] * tmp[8];
    H[3] = sc->K[4] * tmp[3] + sc->K[5] * tmp[6];
    H[4] = sc->K[4] * tmp[4] + sc->K[5] * tmp[7];
    H[5] = sc->K[4] * tmp[5] + sc->K[5] * tmp[8];
    H[6] = sc->K[8] * tmp[6];
    H[7] = sc->K[8] * tmp[7];
    H[8] = sc->K[8] * tmp[8];
}

/* ComputeCorrespondingPoint (src/ACMMP.cu:324-331), pin P1 */
static f2 ComputeCorrespondingPoint(const float *H, const i2 p) {
    const float x = (float)p.x, y = (float)p.y;
    float ptx = dm_fma(H[1], y, dm_fma(H[0], x, H[2]));
    float pty = dm_fma(H[4], y, dm_fma(H[3], x, H[5]));
    float ptz = dm_fma(H[7], y, dm_fma(H[6], x, H[8]));
    float inv = 1.0f / ptz;
    f2 r = {ptx * inv, pty * inv};
    return r;
}

/* TransformNormal cam->world (src/ACMMP.cu:333-341) */
static f4 TransformNormal(const acmmp_camera *c, f4 h) {
    f4 t;
    t.x = c->R[0] * h.x + c->R[3] * h.y + c->R[6] * h.z;
    t.y = c->R[1] * h.x + c->R[4] * h.y + c->R[7] * h.z;
    t.z = c->R[2] * h.x + c->R[5] * h.y + c->R[8] * h.z;
    t.w = h.w;
    return t;
}

/* TransformNormal2RefCam world->cam (src/ACMMP.cu:343-351) */
static f4 TransformNormal2RefCam(const acmmp_camera *c, f4 h) {
    f4 t;
    t.x = c->R[0] * h.x + c->R[1] * h.y + c->R[2] * h.z;
    t.y = c->R[3] * h.x + c->R[4] * h.y + c->R[5] * h.z;
    t.z = c->R[6] * h.x + c->R[7] * h.y + c->R[8] * h.z;
    t.w = h.w;
    return t;
}

/* ComputeBilateralWeight (src/ACMMP.cu:353-358): non-squared distances. */
static float ComputeBilateralWeight(const float xd, const float yd, const float pix,
                                    const float cpix, const float ss, const float sc) {
    const float spatial = dm_sqrt(xd * xd + yd * yd);
    const float color = dm_fabs(pix - cpix);
    return dm_expf(-spatial / (2.0f * ss * ss) - color / (2.0f * sc * sc));
}

/* Pin P3 is inferred, not measured: no reference output pins it (DESIGN.md
 * §2, "parity unpinned"). The r01 form — every product and moment rounded
 * separately, `sum += a * b` and `sum_xy * inv - m_x * m_y` unfused — stays
 * selectable in the oracle (only) for comparison against reference outputs
 * should any become available: acmmp_oracle_set_p3_fused(0). The product
 * kernels implement the fused form only. */
static int g_p3_fused = 1;
void acmmp_oracle_set_p3_fused(int fused) { g_p3_fused = fused != 0; }
int acmmp_oracle_p3_fused(void) { return g_p3_fused; }

/* ComputeBilateralNCC (src/ACMMP.cu:360-432) with pins P1-P3. */
static float ComputeBilateralNCC(const orc_state *S, int src, const i2 p, const f4 h) {
    const acmmp_params *prm = S->prm;
    const acmmp_camera *rc = &S->cams[0], *sc = &S->cams[src];
    const float *rimg = S->imgs[0], *simg = S->imgs[src];
    const int rW = rc->width, rH = rc->height, sW = sc->width, sH = sc->height;
    const float cost_max = 2.0f;
    int radius = prm->patch_size / 2;

    float H[9];
    ComputeHomography(rc, sc, h, H);
    f2 pt = ComputeCorrespondingPoint(H, p);
    if (pt.x >= (float)sW || pt.x < 0.0f || pt.y >= (float)sH || pt.y < 0.0f) return cost_max;

    float sum_ref = 0.0f, sum_ref_ref = 0.0f, sum_src = 0.0f, sum_src_src = 0.0f;
    float sum_ref_src = 0.0f, bw_sum = 0.0f;
    const float ref_center = tex_texel(rimg, rW, rH, p.x, p.y);
    for (int i = -radius; i < radius + 1; i += prm->radius_increment) {
        float r_ref = 0.0f, r_src = 0.0f, r_rr = 0.0f, r_ss = 0.0f, r_rs = 0.0f, r_w = 0.0f;
        for (int j = -radius; j < radius + 1; j += prm->radius_increment) {
            const i2 rp = {p.x + i, p.y + j};
            const float ref_pix = tex_texel(rimg, rW, rH, rp.x, rp.y);
            f2 sp = ComputeCorrespondingPoint(H, rp);
            const float src_pix = tex_bilinear(simg, sW, sH, sp.x, sp.y, prm->texture_filter8);
            float w = ComputeBilateralWeight((float)i, (float)j, ref_pix, ref_center,
                                             prm->sigma_spatial, prm->sigma_color);
            /* pin P3: nvcc's default contraction (--fmad=true, implied by the
             * reference's --use_fast_math) fuses every `sum += a * b` here */
            const float wr = w * ref_pix;
            const float ws = w * src_pix;
            if (g_p3_fused) {
                r_ref = dm_fma(w, ref_pix, r_ref);
                r_rr = dm_fma(wr, ref_pix, r_rr);
                r_src = dm_fma(w, src_pix, r_src);
                r_ss = dm_fma(ws, src_pix, r_ss);
                r_rs = dm_fma(wr, src_pix, r_rs);
            } else { /* r01: each product rounded, then added */
                r_ref += wr;
                r_rr += wr * ref_pix;
                r_src += ws;
                r_ss += ws * src_pix;
                r_rs += wr * src_pix;
            }
            r_w += w;
        }
        sum_ref += r_ref;
        sum_ref_ref += r_rr;
        sum_src += r_src;
        sum_src_src += r_ss;
        sum_ref_src += r_rs;
        bw_sum += r_w;
    }
    const float inv = 1.0f / bw_sum;
    sum_ref *= inv;
    sum_src *= inv;
    /* ... and each `sum_xy * inv - m_x * m_y` (the scaled moment being the
     * first operand) into fma(sum_xy, inv, -(m_x * m_y)). On a flat patch this
     * leaves var, covar as independent residuals instead of three equal ones,
     * which decides the kMinVar test and the cost there. */
    const float var_ref = g_p3_fused ? dm_fma(sum_ref_ref, inv, -(sum_ref * sum_ref))
                                     : sum_ref_ref * inv - sum_ref * sum_ref;
    const float var_src = g_p3_fused ? dm_fma(sum_src_src, inv, -(sum_src * sum_src))
                                     : sum_src_src * inv - sum_src * sum_src;
    const float kMinVar = 1e-5f;
    if (var_ref < kMinVar || var_src < kMinVar) return cost_max;
    const float covar = g_p3_fused ? dm_fma(sum_ref_src, inv, -(sum_ref * sum_src))
                                   : sum_ref_src * inv - sum_ref * sum_src;
    const float var_rs = dm_sqrt(var_ref * var_src);
    float c = 1.0f - covar / var_rs;
    c = (c < cost_max) ? c : cost_max;   /* min(cost_max, .) : NaN -> cost_max */
    c = (c > 0.0f) ? c : 0.0f;           /* max(0, .) */
    return c;
}

/* ComputeMultiViewInitialCostandSelectedViews (src/ACMMP.cu:434-471) */
static float ComputeMultiViewInitialCostandSelectedViews(const orc_state *S, const i2 p,
                                                         const f4 h, uint32_t *selected) {
    float cost_max = 2.0f;
    float cv[MAXSRC] = {2.0f};
    float cvc[MAXSRC] = {2.0f};
    int cost_count = 0, num_valid = 0;
    for (int i = 1; i < S->n; ++i) {
        float c = ComputeBilateralNCC(S, i, p, h);
        cv[i - 1] = c;
        cvc[i - 1] = c;
        cost_count++;
        if (c < cost_max) num_valid++;
    }
    sort_small(cv, cost_count);
    *selected = 0;
    int top_k = num_valid < S->prm->top_k ? num_valid : S->prm->top_k;
    if (top_k > 0) {
        float cost = 0.0f;
        for (int i = 0; i < top_k; ++i) cost += cv[i];
        float thr = cv[top_k - 1];
        for (int i = 0; i < S->n - 1; ++i)
            if (cvc[i] <= thr) setBit(selected, (unsigned)i);
        return cost / (float)top_k;
    }
    return cost_max;
}

/* ComputeMultiViewCostVector (src/ACMMP.cu:473-478) */
static void ComputeMultiViewCostVector(const orc_state *S, const i2 p, const f4 h, float *cv) {
    for (int i = 1; i < S->n; ++i) cv[i - 1] = ComputeBilateralNCC(S, i, p, h);
}

/* Get3DPointonWorld_cu (src/ACMMP.cu:480-504) */
static f3 Get3DPointonWorld(const float x, const float y, const float depth, const acmmp_camera *c) {
    f3 X, T, C;
    X.x = depth * (x - c->K[2]) / c->K[0];
    X.y = depth * (y - c->K[5]) / c->K[4];
    X.z = depth;
    T.x = c->R[0] * X.x + c->R[3] * X.y + c->R[6] * X.z;
    T.y = c->R[1] * X.x + c->R[4] * X.y + c->R[7] * X.z;
    T.z = c->R[2] * X.x + c->R[5] * X.y + c->R[8] * X.z;
    C.x = -(c->R[0] * c->t[0] + c->R[3] * c->t[1] + c->R[6] * c->t[2]);
    C.y = -(c->R[1] * c->t[0] + c->R[4] * c->t[1] + c->R[7] * c->t[2]);
    C.z = -(c->R[2] * c->t[0] + c->R[5] * c->t[1] + c->R[8] * c->t[2]);
    X.x = T.x + C.x;
    X.y = T.y + C.y;
    X.z = T.z + C.z;
    return X;
}

/* ProjectonCamera_cu (src/ACMMP.cu:506-516) */
static void ProjectonCamera(const f3 X, const acmmp_camera *c, f2 *pt, float *depth) {
    f3 t;
    t.x = c->R[0] * X.x + c->R[1] * X.y + c->R[2] * X.z + c->t[0];
    t.y = c->R[3] * X.x + c->R[4] * X.y + c->R[5] * X.z + c->t[1];
    t.z = c->R[6] * X.x + c->R[7] * X.y + c->R[8] * X.z + c->t[2];
    *depth = c->K[6] * t.x + c->K[7] * t.y + c->K[8] * t.z;
    pt->x = (c->K[0] * t.x + c->K[1] * t.y + c->K[2] * t.z) / *depth;
    pt->y = (c->K[3] * t.x + c->K[4] * t.y + c->K[5] * t.z) / *depth;
}

/* ComputeGeomConsistencyCost (src/ACMMP.cu:518-543) */
static float ComputeGeomConsistencyCost(const orc_state *S, int src, const f4 h, const i2 p) {
    const float max_cost = 3.0f;
    const acmmp_camera *rc = &S->cams[0], *sc = &S->cams[src];
    float depth = ComputeDepthfromPlaneHypothesis(rc, h, p);
    f3 fwd = Get3DPointonWorld((float)p.x, (float)p.y, depth, rc);
    f2 spt;
    float sd;
    ProjectonCamera(fwd, sc, &spt, &sd);
    const float src_depth = tex_trunc(S->depths[src], S->depth_w[src], S->depth_h[src], spt.x, spt.y);
    if (src_depth == 0.0f) return max_cost;
    f3 s3 = Get3DPointonWorld(spt.x, spt.y, src_depth, sc);
    f2 back;
    float rd;
    ProjectonCamera(s3, rc, &back, &rd);
    const float dc = (float)p.x - back.x;
    const float dr = (float)p.y - back.y;
    float e = dm_sqrt(dc * dc + dr * dr);
    return (e < max_cost) ? e : max_cost;  /* min(max_cost, .) */
}

/* SpatialGauss / RangeGauss (src/ACMMP.cu:151-161): pow(v,2) pinned to v*v,
 * the double `-1.0 *` kept. */
static float SpatialGauss(float x1, float y1, float x2, float y2, float sigma) {
    float dis = (x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) - 0.0f;
    return dm_expf((float)(-1.0 * (double)dis / (double)(2 * sigma * sigma)));
}
static float RangeGauss(float x, float sigma) {
    float xp = x - 0.0f;
    return dm_expf((float)(-1.0 * (double)(xp * xp) / (double)(2 * sigma * sigma)));
}

/* upscale_normal (src/ACMMP.cu:548-607) */
static f4 upscale_normal(const orc_state *S, const i2 p, const int center, const float sigmad,
                         const float sigmar, int nn, const float o_y, const float o_x,
                         const float refPix, float *cost_out) {
    const int scols = (int)S->prm->scaled_cols, srows = (int)S->prm->scaled_rows;
    float c_total = 0.0f, norm = 0.0f;
    f4 n_total = {0, 0, 0, 0};
    (void)center;
    for (int j = -nn; j <= nn; ++j) {
        int r_y = (int)(o_y + (float)j);
        r_y = (r_y > 0 ? (r_y < srows ? r_y : srows - 1) : 0);
        int r_ys = p.y + j;
        for (int i = -nn; i <= nn; ++i) {
            int r_x = (int)(o_x + (float)i);
            r_x = (r_x > 0 ? (r_x < scols ? r_x : scols - 1) : 0);
            const int sc = r_y * scols + r_x;
            const float srcPix = S->scaled_planes[sc].w;
            f4 srcNorm = S->scaled_planes[sc];
            int r_xs = p.x + i;
            const float nb = tex_texel(S->imgs[0], S->W, S->H, r_xs, r_ys);
            float sg = SpatialGauss(o_x, o_y, (float)r_x, (float)r_y, sigmad);
            float rg = RangeGauss(dm_fabs(refPix - nb), sigmar);
            float tg = sg * rg;
            norm += tg;
            c_total += srcPix * tg;
            srcNorm.x = srcNorm.x * tg;
            srcNorm.y = srcNorm.y * tg;
            srcNorm.z = srcNorm.z * tg;
            n_total.x = n_total.x + srcNorm.x;
            n_total.y = n_total.y + srcNorm.y;
            n_total.z = n_total.z + srcNorm.z;
        }
    }
    *cost_out = c_total / norm;
    n_total.x = n_total.x / norm;
    n_total.y = n_total.y / norm;
    n_total.z = n_total.z / norm;
    NormalizeVec3(&n_total);
    return n_total;
}

static dm_rng make_rng(const orc_state *S, int center, uint32_t phase) {
    dm_rng g;
    g.k0 = S->prm->seed_lo;
    g.k1 = S->prm->seed_hi;
    g.pix = (uint32_t)center;
    g.phase = phase;
    g.stream = S->prm->rng_stream;
    g.draw = 0;
    g.blk.x = g.blk.y = g.blk.z = g.blk.w = 0u;
    return g;
}

/* Double-precision constants of the reference, evaluated once. */
static float k_pert_pi(void) { return (float)((double)0.02f * M_PI); }             /* :737 */
static float k_pert3_pi(void) { return (float)((double)(3 * 0.02f) * M_PI); }     /* :649 */
static float k_angle_sigma(void) { return (float)(M_PI * (double)(5.0f / 180.0f)); } /* :715 */

/* RandomInitialization (src/ACMMP.cu:609-705) for one pixel. */
static void RandomInitialization(orc_state *S, const i2 p) {
    const acmmp_params *prm = S->prm;
    const acmmp_camera *c0 = &S->cams[0];
    const int center = p.y * S->W + p.x;
    dm_rng rs = make_rng(S, center, 0u);
    if (!prm->geom_consistency && !prm->hierarchy && !prm->seeded) {
        S->planes[center] = GenerateRandomPlaneHypothesis(c0, p, &rs, prm->depth_min, prm->depth_max);
        S->costs[center] = ComputeMultiViewInitialCostandSelectedViews(S, p, S->planes[center], &S->sv[center]);
    } else if (prm->seeded) {
        S->planes[center] = S->seed_planes[center];
        S->costs[center] = ComputeMultiViewInitialCostandSelectedViews(S, p, S->planes[center], &S->sv[center]);
    } else if (prm->planar_prior) {
        if (S->masks[center] > 0 && S->costs[center] >= 0.1f) {
            float perturbation = 0.02f;
            f4 h = S->prior_planes[center];
            float dp = h.w;
            const float dmin = (1 - 3 * perturbation) * dp;
            const float dmax = (1 + 3 * perturbation) * dp;
            dp = dm_rng_uniform(&rs) * (dmax - dmin) + dmin;
            f4 hp = GeneratePerturbedNormal(c0, p, h, &rs, k_pert3_pi());
            hp.w = dp;
            S->planes[center] = hp;
            S->costs[center] = ComputeMultiViewInitialCostandSelectedViews(S, p, S->planes[center], &S->sv[center]);
        } else {
            f4 h = S->planes[center];
            float depth = h.w;
            h.w = GetDistance2Origin(c0, p, depth, h);
            S->planes[center] = h;
            S->costs[center] = ComputeMultiViewInitialCostandSelectedViews(S, p, S->planes[center], &S->sv[center]);
        }
    } else {
        if (prm->upsample) {
            const float scale = (float)(1.0 * (double)prm->scaled_cols / (double)S->W);
            const float sigmad = 0.50f, sigmar = 25.5f;
            /* max(width / scaled_cols, height / scaled_rows) in float (:667) */
            float a = (float)S->W / prm->scaled_cols, b = (float)S->H / prm->scaled_rows;
            const int Imagescale = (int)(a > b ? a : b);
            const int WinWidth = Imagescale * Imagescale + 1;
            int nn = WinWidth / 2;
            const float o_y = (float)p.y * scale;
            const float o_x = (float)p.x * scale;
            const float refPix = tex_texel(S->imgs[0], S->W, S->H, p.x, p.y);
            float ucost;
            f4 n_total = upscale_normal(S, p, center, sigmad, sigmar, nn, o_y, o_x, refPix, &ucost);
            S->costs[center] = ucost;
            S->costs[center] = ComputeMultiViewInitialCostandSelectedViews(S, p, S->planes[center], &S->sv[center]);
            S->pre_costs[center] = S->costs[center];
            f4 h = TransformNormal2RefCam(c0, n_total);
            float depth = S->planes[center].w;
            h.w = GetDistance2Origin(c0, p, depth, h);
            S->planes[center] = h;
            S->costs[center] = ComputeMultiViewInitialCostandSelectedViews(S, p, S->planes[center], &S->sv[center]);
        } else {
            f4 h = prm->hierarchy ? S->scaled_planes[center] : S->planes[center];
            h = TransformNormal2RefCam(c0, h);
            float depth = h.w;
            h.w = GetDistance2Origin(c0, p, depth, h);
            S->planes[center] = h;
            S->costs[center] = ComputeMultiViewInitialCostandSelectedViews(S, p, S->planes[center], &S->sv[center]);
        }
    }
}

/* PlaneHypothesisRefinement (src/ACMMP.cu:707-784) */
static void PlaneHypothesisRefinement(const orc_state *S, f4 *plane, float *depth, float *cost,
                                      dm_rng *rs, const float *view_weights, const float weight_norm,
                                      float *restricted_cost, const i2 p) {
    const acmmp_params *prm = S->prm;
    const acmmp_camera *c0 = &S->cams[0];
    float perturbation = 0.02f;
    const int center = p.y * S->W + p.x;
    float gamma = 0.5f;
    float depth_sigma = (prm->depth_max - prm->depth_min) / 64.0f;
    float two_dss = 2 * depth_sigma * depth_sigma;
    float angle_sigma = k_angle_sigma();
    float two_ass = 2 * angle_sigma * angle_sigma;
    float beta = 0.18f;
    float depth_prior = 0.0f;
    float depth_rand;
    f4 plane_rand;
    const int has_prior = prm->planar_prior && S->masks[center] > 0;
    if (has_prior) {
        depth_prior = ComputeDepthfromPlaneHypothesis(c0, S->prior_planes[center], p);
        depth_rand = dm_rng_uniform(rs) * 6 * depth_sigma + (depth_prior - 3 * depth_sigma);
        plane_rand = GeneratePerturbedNormal(c0, p, S->prior_planes[center], rs, angle_sigma);
    } else {
        depth_rand = dm_rng_uniform(rs) * (prm->depth_max - prm->depth_min) + prm->depth_min;
        plane_rand = GenerateRandomNormal(c0, p, rs, *depth);
    }
    float depth_perturbed = *depth;
    const float dmin_p = (1 - perturbation) * depth_perturbed;
    const float dmax_p = (1 + perturbation) * depth_perturbed;
    do {
        depth_perturbed = dm_rng_uniform(rs) * (dmax_p - dmin_p) + dmin_p;
    } while (depth_perturbed < prm->depth_min && depth_perturbed > prm->depth_max);
    f4 plane_perturbed = GeneratePerturbedNormal(c0, p, *plane, rs, k_pert_pi());

    const int num_planes = 5;
    float depths[5] = {depth_rand, *depth, depth_rand, *depth, depth_perturbed};
    f4 normals[5] = {*plane, plane_rand, plane_rand, plane_perturbed, *plane};
    for (int i = 0; i < num_planes; ++i) {
        float cv[MAXSRC] = {2.0f};
        f4 th = normals[i];
        th.w = GetDistance2Origin(c0, p, depths[i], th);
        ComputeMultiViewCostVector(S, p, th, cv);
        float temp_cost = 0.0f;
        for (int j = 0; j < S->n - 1; ++j) {
            if (view_weights[j] > 0) {
                if (prm->geom_consistency)
                    temp_cost += view_weights[j] * (cv[j] + 0.2f * ComputeGeomConsistencyCost(S, j + 1, th, p));
                else
                    temp_cost += view_weights[j] * cv[j];
            }
        }
        temp_cost /= weight_norm;
        float depth_before = ComputeDepthfromPlaneHypothesis(c0, th, p);
        if (has_prior) {
            float dd = depths[i] - depth_prior;
            float ac = Vec3DotVec3(S->prior_planes[center], th);
            float ad = dm_acosf(ac);
            float prior = gamma + dm_expf(-dd * dd / two_dss) * dm_expf(-ad * ad / two_ass);
            float rtc = dm_expf(-temp_cost * temp_cost / beta) * prior;
            if (depth_before >= prm->depth_min && depth_before <= prm->depth_max && rtc > *restricted_cost) {
                *depth = depth_before;
                *plane = th;
                *cost = temp_cost;
                *restricted_cost = rtc;
            }
        } else {
            if (depth_before >= prm->depth_min && depth_before <= prm->depth_max && temp_cost < *cost) {
                *depth = depth_before;
                *plane = th;
                *cost = temp_cost;
            }
        }
    }
}

/* CheckerboardPropagation (src/ACMMP.cu:786-1173) for one pixel. Neighbour
 * reads come from the half-sweep snapshot (pin A2); the pixel's own state is
 * read and written live. */
static void CheckerboardPropagation(orc_state *S, const i2 p, const int iter) {
    const acmmp_params *prm = S->prm;
    const acmmp_camera *c0 = &S->cams[0];
    const int width = S->W, height = S->H;
    if (p.x >= width || p.y >= height) return;
    const f4 *sp = S->snap_planes;
    const float *sco = S->snap_costs;
    const int nsrc = S->n - 1;

    const int center = p.y * width + p.x;
    int left_near = center - 1, left_far = center - 3;
    int right_near = center + 1, right_far = center + 3;
    int up_near = center - width, up_far = center - 3 * width;
    int down_near = center + width, down_far = center + 3 * width;

    float cost_array[8][MAXSRC];
    memset(cost_array, 0, sizeof(cost_array));
    cost_array[0][0] = 2.0f;  /* `= {2.0f}` initialises only [0][0] (pin A5) */
    int flag[8] = {0};
    float costMin;
    int costMinPoint;

    if (p.y > 2) {  /* up_far */
        flag[1] = 1;
        costMin = sco[up_far];
        costMinPoint = up_far;
        for (int i = 1; i < 11; ++i) {
            if (p.y > 2 + 2 * i) {
                int pt = up_far - 2 * i * width;
                if (sco[pt] < costMin) { costMin = sco[pt]; costMinPoint = pt; }
            }
        }
        up_far = costMinPoint;
        ComputeMultiViewCostVector(S, p, sp[up_far], cost_array[1]);
    }
    if (p.y < height - 3) {  /* down_far */
        flag[3] = 1;
        costMin = sco[down_far];
        costMinPoint = down_far;
        for (int i = 1; i < 11; ++i) {
            if (p.y < height - 3 - 2 * i) {
                int pt = down_far + 2 * i * width;
                if (sco[pt] < costMin) { costMin = sco[pt]; costMinPoint = pt; }
            }
        }
        down_far = costMinPoint;
        ComputeMultiViewCostVector(S, p, sp[down_far], cost_array[3]);
    }
    if (p.x > 2) {  /* left_far */
        flag[5] = 1;
        costMin = sco[left_far];
        costMinPoint = left_far;
        for (int i = 1; i < 11; ++i) {
            if (p.x > 2 + 2 * i) {
                int pt = left_far - 2 * i;
                if (sco[pt] < costMin) { costMin = sco[pt]; costMinPoint = pt; }
            }
        }
        left_far = costMinPoint;
        ComputeMultiViewCostVector(S, p, sp[left_far], cost_array[5]);
    }
    if (p.x < width - 3) {  /* right_far: reversed comparison picks the max (:879) */
        flag[7] = 1;
        costMin = sco[right_far];
        costMinPoint = right_far;
        for (int i = 1; i < 11; ++i) {
            if (p.x < width - 3 - 2 * i) {
                int pt = right_far + 2 * i;
                if (costMin < sco[pt]) { costMin = sco[pt]; costMinPoint = pt; }
            }
        }
        right_far = costMinPoint;
        ComputeMultiViewCostVector(S, p, sp[right_far], cost_array[7]);
    }
    if (p.y > 0) {  /* up_near */
        flag[0] = 1;
        costMin = sco[up_near];
        costMinPoint = up_near;
        for (int i = 0; i < 3; ++i) {
            if (p.y > 1 + i && p.x > i) {
                int pt = up_near - (1 + i) * width - i;
                if (sco[pt] < costMin) { costMin = sco[pt]; costMinPoint = pt; }
            }
            if (p.y > 1 + i && p.x < width - 1 - i) {
                int pt = up_near - (1 + i) * width + i;
                if (sco[pt] < costMin) { costMin = sco[pt]; costMinPoint = pt; }
            }
        }
        up_near = costMinPoint;
        ComputeMultiViewCostVector(S, p, sp[up_near], cost_array[0]);
    }
    if (p.y < height - 1) {  /* down_near */
        flag[2] = 1;
        costMin = sco[down_near];
        costMinPoint = down_near;
        for (int i = 0; i < 3; ++i) {
            if (p.y < height - 2 - i && p.x > i) {
                int pt = down_near + (1 + i) * width - i;
                if (sco[pt] < costMin) { costMin = sco[pt]; costMinPoint = pt; }
            }
            if (p.y < height - 2 - i && p.x < width - 1 - i) {
                int pt = down_near + (1 + i) * width + i;
                if (sco[pt] < costMin) { costMin = sco[pt]; costMinPoint = pt; }
            }
        }
        down_near = costMinPoint;
        ComputeMultiViewCostVector(S, p, sp[down_near], cost_array[2]);
    }
    if (p.x > 0) {  /* left_near */
        flag[4] = 1;
        costMin = sco[left_near];
        costMinPoint = left_near;
        for (int i = 0; i < 3; ++i) {
            if (p.x > 1 + i && p.y > i) {
                int pt = left_near - (1 + i) - i * width;
                if (sco[pt] < costMin) { costMin = sco[pt]; costMinPoint = pt; }
            }
            if (p.x > 1 + i && p.y < height - 1 - i) {
                int pt = left_near - (1 + i) + i * width;
                if (sco[pt] < costMin) { costMin = sco[pt]; costMinPoint = pt; }
            }
        }
        left_near = costMinPoint;
        ComputeMultiViewCostVector(S, p, sp[left_near], cost_array[4]);
    }
    if (p.x < width - 1) {  /* right_near */
        flag[6] = 1;
        costMin = sco[right_near];
        costMinPoint = right_near;
        for (int i = 0; i < 3; ++i) {
            if (p.x < width - 2 - i && p.y > i) {
                int pt = right_near + (1 + i) - i * width;
                if (sco[pt] < costMin) { costMin = sco[pt]; costMinPoint = pt; }
            }
            if (p.x < width - 2 - i && p.y < height - 1 - i) {
                int pt = right_near + (1 + i) + i * width;
                if (sco[pt] < costMin) { costMin = sco[pt]; costMinPoint = pt; }
            }
        }
        right_near = costMinPoint;
        ComputeMultiViewCostVector(S, p, sp[right_near], cost_array[6]);
    }
    const int positions[8] = {up_near, up_far, down_near, down_far, left_near, left_far, right_near, right_far};

    /* Multi-hypothesis joint view selection (:994-1056) */
    float view_weights[MAXSRC] = {0.0f};
    float vsp[MAXSRC] = {0.0f};
    int nbr[4] = {center - width, center + width, center - 1, center + 1};
    for (int i = 0; i < 4; ++i) {
        if (flag[2 * i]) {
            for (int j = 0; j < nsrc; ++j) {
                if (isSet(S->sv[nbr[i]], (unsigned)j) == 1) vsp[j] += 0.9f;
                else vsp[j] += 0.1f;
            }
        }
    }
    float probs[MAXSRC] = {0.0f};
    float cost_threshold = (float)(0.8 * (double)dm_expf((float)(iter * iter) / (-90.0f)));
    for (int i = 0; i < nsrc; i++) {
        float count = 0;
        int count_false = 0;
        float tmpw = 0;
        for (int j = 0; j < 8; j++) {
            if (cost_array[j][i] < cost_threshold) {
                tmpw += dm_expf(cost_array[j][i] * cost_array[j][i] / (-0.18f));
                count++;
            }
            if (cost_array[j][i] > 1.2f) count_false++;
        }
        if (count > 2 && count_false < 3) probs[i] = tmpw / count;
        else if (count_false < 3) probs[i] = dm_expf(cost_threshold * cost_threshold / (-0.32f));
        probs[i] = probs[i] * vsp[i];
    }
    TransformPDFToCDF(probs, nsrc);
    dm_rng rs = make_rng(S, center, 1u + (uint32_t)iter);
    for (int sample = 0; sample < 15; ++sample) {
        const float rand_prob = dm_rng_uniform(&rs) - FLT_EPSILON;
        for (int image_id = 0; image_id < nsrc; ++image_id) {
            const float prob = probs[image_id];
            if (prob > rand_prob) { view_weights[image_id] += 1.0f; break; }
        }
    }
    uint32_t temp_sv = 0;
    float weight_norm = 0;
    for (int i = 0; i < nsrc; ++i) {
        if (view_weights[i] > 0) { setBit(&temp_sv, (unsigned)i); weight_norm += view_weights[i]; }
    }

    float final_costs[8] = {0.0f};
    for (int i = 0; i < 8; ++i) {
        for (int j = 0; j < nsrc; ++j) {
            if (view_weights[j] > 0) {
                if (prm->geom_consistency) {
                    if (flag[i])
                        final_costs[i] += view_weights[j] *
                            (cost_array[i][j] + 0.2f * ComputeGeomConsistencyCost(S, j + 1, sp[positions[i]], p));
                    else
                        final_costs[i] += view_weights[j] * (cost_array[i][j] + 0.1f * 3.0f);
                } else {
                    final_costs[i] += view_weights[j] * cost_array[i][j];
                }
            }
        }
        final_costs[i] /= weight_norm;
    }
    const int min_cost_idx = FindMinCostIndex(final_costs, 8);

    float cvn[MAXSRC] = {2.0f};
    ComputeMultiViewCostVector(S, p, S->planes[center], cvn);
    float cost_now = 0.0f;
    for (int i = 0; i < nsrc; ++i) {
        if (prm->geom_consistency)
            cost_now += view_weights[i] * (cvn[i] + 0.2f * ComputeGeomConsistencyCost(S, i + 1, S->planes[center], p));
        else
            cost_now += view_weights[i] * cvn[i];
    }
    cost_now /= weight_norm;
    S->costs[center] = cost_now;
    float depth_now = ComputeDepthfromPlaneHypothesis(c0, S->planes[center], p);
    float restricted_cost = 0.0f;
    if (prm->planar_prior) {
        float rfc[8] = {0.0f};
        float gamma = 0.5f;
        float depth_sigma = (prm->depth_max - prm->depth_min) / 64.0f;
        float two_dss = 2 * depth_sigma * depth_sigma;
        float angle_sigma = k_angle_sigma();
        float two_ass = 2 * angle_sigma * angle_sigma;
        float depth_prior = ComputeDepthfromPlaneHypothesis(c0, S->prior_planes[center], p);
        float beta = 0.18f;
        if (S->masks[center] > 0) {
            for (int i = 0; i < 8; i++) {
                if (flag[i]) {
                    float dn = ComputeDepthfromPlaneHypothesis(c0, sp[positions[i]], p);
                    float dd = dn - depth_prior;
                    float ac = Vec3DotVec3(S->prior_planes[center], sp[positions[i]]);
                    float ad = dm_acosf(ac);
                    float prior = gamma + dm_expf(-dd * dd / two_dss) * dm_expf(-ad * ad / two_ass);
                    rfc[i] = dm_expf(-final_costs[i] * final_costs[i] / beta) * prior;
                }
            }
            const int max_cost_idx = FindMaxCostIndex(rfc, 8);
            float dn = ComputeDepthfromPlaneHypothesis(c0, S->planes[center], p);
            float dd = dn - depth_prior;
            float ac = Vec3DotVec3(S->prior_planes[center], S->planes[center]);
            float ad = dm_acosf(ac);
            float prior = gamma + dm_expf(-dd * dd / two_dss) * dm_expf(-ad * ad / two_ass);
            float rcn = dm_expf(-cost_now * cost_now / beta) * prior;
            if (flag[max_cost_idx]) {
                float db = ComputeDepthfromPlaneHypothesis(c0, sp[positions[max_cost_idx]], p);
                if (db >= prm->depth_min && db <= prm->depth_max && rfc[max_cost_idx] > rcn) {
                    /* `depth_now = depth_before` at :1130 assigns the block-local
                     * `float depth_now` declared at :1119, which shadows the outer
                     * one: the outer depth_now (fed to the refinement) keeps the
                     * OLD plane's depth. Literal. */
                    S->planes[center] = sp[positions[max_cost_idx]];
                    S->costs[center] = final_costs[max_cost_idx];
                    restricted_cost = rfc[max_cost_idx];
                    S->sv[center] = temp_sv;
                }
            }
        } else if (flag[min_cost_idx]) {
            float db = ComputeDepthfromPlaneHypothesis(c0, sp[positions[min_cost_idx]], p);
            if (db >= prm->depth_min && db <= prm->depth_max && final_costs[min_cost_idx] < cost_now) {
                depth_now = db;
                S->planes[center] = sp[positions[min_cost_idx]];
                S->costs[center] = final_costs[min_cost_idx];
            }
        }
    }

    f4 plane_now = S->planes[center];  /* pin A3 */
    if (!prm->planar_prior && flag[min_cost_idx]) {
        float db = ComputeDepthfromPlaneHypothesis(c0, sp[positions[min_cost_idx]], p);
        if (db >= prm->depth_min && db <= prm->depth_max && final_costs[min_cost_idx] < cost_now) {
            depth_now = db;
            plane_now = sp[positions[min_cost_idx]];
            cost_now = final_costs[min_cost_idx];
            S->sv[center] = temp_sv;
        }
    }
    PlaneHypothesisRefinement(S, &plane_now, &depth_now, &cost_now, &rs, view_weights, weight_norm,
                              &restricted_cost, p);
    if (prm->hierarchy) {
        if (cost_now < S->pre_costs[center] - 0.1f) {
            S->costs[center] = cost_now;
            S->planes[center] = plane_now;
        }
    } else {
        S->costs[center] = cost_now;
        S->planes[center] = plane_now;
    }
}

/* GetDepthandNormal (src/ACMMP.cu:1199-1212) */
static void GetDepthandNormal(orc_state *S, const i2 p) {
    const int center = p.y * S->W + p.x;
    S->planes[center].w = ComputeDepthfromPlaneHypothesis(&S->cams[0], S->planes[center], p);
    S->planes[center] = TransformNormal(&S->cams[0], S->planes[center]);
}

/* CheckerboardFilter (src/ACMMP.cu:1214-1328) */
static void CheckerboardFilter(orc_state *S, const i2 p) {
    const int width = S->W, height = S->H;
    if (p.x >= width || p.y >= height) return;
    f4 *ph = S->planes;
    const int center = p.y * width + p.x;
    float filter[21];
    int index = 0;
    filter[index++] = ph[center].w;
    const int left = center - 1, leftleft = center - 3;
    const int up = center - width, upup = center - 3 * width;
    const int down = center + width, downdown = center + 3 * width;
    const int right = center + 1, rightright = center + 3;
    if (S->costs[center] < 0.001f) return;
    if (p.y > 0) filter[index++] = ph[up].w;
    if (p.y > 2) filter[index++] = ph[upup].w;
    if (p.y > 4) filter[index++] = ph[upup - width * 2].w;
    if (p.y < height - 1) filter[index++] = ph[down].w;
    if (p.y < height - 3) filter[index++] = ph[downdown].w;
    if (p.y < height - 5) filter[index++] = ph[downdown + width * 2].w;
    if (p.x > 0) filter[index++] = ph[left].w;
    if (p.x > 2) filter[index++] = ph[leftleft].w;
    if (p.x > 4) filter[index++] = ph[leftleft - 2].w;
    if (p.x < width - 1) filter[index++] = ph[right].w;
    if (p.x < width - 3) filter[index++] = ph[rightright].w;
    if (p.x < width - 5) filter[index++] = ph[rightright + 2].w;
    if (p.y > 0 && p.x < width - 2) filter[index++] = ph[up + 2].w;
    if (p.y < height - 1 && p.x < width - 2) filter[index++] = ph[down + 2].w;
    if (p.y > 0 && p.x > 1) filter[index++] = ph[up - 2].w;
    if (p.y < height - 1 && p.x > 1) filter[index++] = ph[down - 2].w;
    if (p.x > 0 && p.y > 2) filter[index++] = ph[left - width * 2].w;
    if (p.x < width - 1 && p.y > 2) filter[index++] = ph[right - width * 2].w;
    if (p.x > 0 && p.y < height - 2) filter[index++] = ph[left + width * 2].w;
    if (p.x < width - 1 && p.y < height - 2) filter[index++] = ph[right + width * 2].w;
    sort_small(filter, index);
    int m = index / 2;
    if (index % 2 == 0) ph[center].w = (filter[m - 1] + filter[m]) / 2;
    else ph[center].w = filter[m];
}

/* Rows reached by the reference's checkerboard grid: grid.y = ceil((H/2)/16)
 * blocks of 16 thread-rows, each covering 2 image rows (src/ACMMP.cu:1399,
 * :1178-1182). When H is odd and H/2 is a multiple of 16 the last row is
 * never updated or filtered (Appendix A5). */
static int checkerboard_rows(int H) {
    int gy = ((H / 2) + 16 - 1) / 16;
    int rows = gy * 32;
    return rows < H ? rows : H;
}

static int setup_state(orc_state *S, const acmmp_params *prm, int n, const acmmp_camera *cams,
                       const float *const *imgs, const float *const *depths, int *dw, int *dh,
                       float *planes, float *costs, uint32_t *sv, float *pre_costs,
                       const float *prior_planes, const uint32_t *masks,
                       const float *scaled_planes, const float *seed_planes) {
    memset(S, 0, sizeof(*S));
    if (n < 2 || n > ACMMP_MAX_IMAGES) return -1;
    S->prm = prm;
    S->n = n;
    S->cams = cams;
    S->imgs = imgs;
    S->depths = depths;
    S->W = cams[0].width;
    S->H = cams[0].height;
    S->sweep_rows = checkerboard_rows(S->H);
    S->planes = (f4 *)planes;
    S->costs = costs;
    S->sv = sv;
    S->pre_costs = pre_costs;
    S->prior_planes = (const f4 *)prior_planes;
    S->masks = masks;
    S->scaled_planes = (const f4 *)scaled_planes;
    S->seed_planes = (const f4 *)seed_planes;
    if (depths) {
        for (int i = 0; i < n; ++i) {
            if (dw[i] <= 0) dw[i] = cams[i].width;
            if (dh[i] <= 0) dh[i] = cams[i].height;
        }
    }
    S->depth_w = dw;
    S->depth_h = dh;
    return 0;
}

/* ACMMP::RunPatchMatch (src/ACMMP.cu:1378-1456), CPU. In/out: planes (float4
 * per pixel), costs; out: selected views. pre_costs: hierarchy state (in/out).
 * depth_w/depth_h may be NULL (maps sized like their views). */
int acmmp_oracle_run_patchmatch(const acmmp_params *prm, int n, const acmmp_camera *cams,
                                const float *const *imgs, const float *const *depths,
                                const int *depth_w, const int *depth_h,
                                float *planes, float *costs, uint32_t *sv, float *pre_costs,
                                const float *prior_planes, const uint32_t *masks,
                                const float *scaled_planes, const float *seed_planes,
                                int nthreads) {
    orc_state S;
    int dw[ACMMP_MAX_IMAGES], dh[ACMMP_MAX_IMAGES];
    for (int i = 0; i < ACMMP_MAX_IMAGES; ++i) {
        dw[i] = (depth_w && i < n) ? depth_w[i] : 0;
        dh[i] = (depth_h && i < n) ? depth_h[i] : 0;
    }
    if (setup_state(&S, prm, n, cams, imgs, depths, dw, dh, planes, costs, sv, pre_costs,
                    prior_planes, masks, scaled_planes, seed_planes))
        return -1;
    if (prm->geom_consistency && !depths) return -1;
    if ((prm->planar_prior) && (!prior_planes || !masks)) return -1;
    if (prm->hierarchy && !pre_costs) return -1;
    if (prm->hierarchy && !scaled_planes) return -1;
    if (prm->seeded && !seed_planes) return -1;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    const int W = S.W, H = S.H;
    const size_t P = (size_t)W * H;

    /* RandomInitialization over all pixels (16x16 grid covers the image) */
#pragma omp parallel for schedule(dynamic, 4)
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            i2 p = {x, y};
            RandomInitialization(&S, p);
        }

    S.snap_planes = (f4 *)malloc(P * sizeof(f4));
    S.snap_costs = (float *)malloc(P * sizeof(float));
    if (!S.snap_planes || !S.snap_costs) { free(S.snap_planes); free(S.snap_costs); return -2; }
    for (int it = 0; it < prm->max_iterations; ++it) {
        for (int colour = 0; colour < 2; ++colour) {  /* Black: (x+y) even; Red: odd */
            memcpy(S.snap_planes, S.planes, P * sizeof(f4));
            memcpy(S.snap_costs, S.costs, P * sizeof(float));
#pragma omp parallel for schedule(dynamic, 2)
            for (int y = 0; y < S.sweep_rows; ++y)
                for (int x = (y + colour) & 1; x < W; x += 2) {
                    i2 p = {x, y};
                    CheckerboardPropagation(&S, p, it);
                }
        }
    }
    free(S.snap_planes);
    free(S.snap_costs);
#pragma omp parallel for schedule(static)
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            i2 p = {x, y};
            GetDepthandNormal(&S, p);
        }
    for (int colour = 0; colour < 2; ++colour) {
#pragma omp parallel for schedule(static)
        for (int y = 0; y < S.sweep_rows; ++y)
            for (int x = (y + colour) & 1; x < W; x += 2) {
                i2 p = {x, y};
                CheckerboardFilter(&S, p);
            }
    }
    return 0;
}

/* T1 helpers: costs of every source view for a given per-pixel plane. */
int acmmp_oracle_eval_costs(const acmmp_params *prm, int n, const acmmp_camera *cams,
                            const float *const *imgs, const float *planes4, float *out_costs,
                            float *out_init_cost, uint32_t *out_init_views, int nthreads) {
    orc_state S;
    int dw[ACMMP_MAX_IMAGES] = {0}, dh[ACMMP_MAX_IMAGES] = {0};
    if (setup_state(&S, prm, n, cams, imgs, NULL, dw, dh, NULL, NULL, NULL, NULL, NULL, NULL,
                    NULL, NULL))
        return -1;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    const f4 *pl = (const f4 *)planes4;
    const int W = S.W, H = S.H;
#pragma omp parallel for schedule(dynamic, 4)
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            i2 p = {x, y};
            size_t c = (size_t)y * W + x;
            if (out_costs) ComputeMultiViewCostVector(&S, p, pl[c], out_costs + c * (size_t)(n - 1));
            if (out_init_cost) {
                uint32_t v = 0;
                out_init_cost[c] = ComputeMultiViewInitialCostandSelectedViews(&S, p, pl[c], &v);
                if (out_init_views) out_init_views[c] = v;
            }
        }
    return 0;
}

int acmmp_oracle_eval_geom_costs(const acmmp_params *prm, int n, const acmmp_camera *cams,
                                 const float *const *imgs, const float *const *depths,
                                 const float *planes4, float *out, int nthreads) {
    orc_state S;
    int dw[ACMMP_MAX_IMAGES] = {0}, dh[ACMMP_MAX_IMAGES] = {0};
    if (setup_state(&S, prm, n, cams, imgs, depths, dw, dh, NULL, NULL, NULL, NULL, NULL, NULL,
                    NULL, NULL))
        return -1;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    const f4 *pl = (const f4 *)planes4;
    const int W = S.W, H = S.H;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            i2 p = {x, y};
            size_t c = (size_t)y * W + x;
            for (int v = 1; v < n; ++v)
                out[c * (size_t)(n - 1) + (v - 1)] = ComputeGeomConsistencyCost(&S, v, pl[c], p);
        }
    return 0;
}

/* Single-call entry points for the analytic known-answer tests. */
float acmmp_oracle_ncc(const acmmp_params *prm, const acmmp_camera *ref, const acmmp_camera *src,
                       const float *ref_img, const float *src_img, int px, int py,
                       const float *plane4) {
    acmmp_camera cams[2] = {*ref, *src};
    const float *imgs[2] = {ref_img, src_img};
    orc_state S;
    int dw[ACMMP_MAX_IMAGES] = {0}, dh[ACMMP_MAX_IMAGES] = {0};
    setup_state(&S, prm, 2, cams, imgs, NULL, dw, dh, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL);
    i2 p = {px, py};
    f4 h = {plane4[0], plane4[1], plane4[2], plane4[3]};
    return ComputeBilateralNCC(&S, 1, p, h);
}

void acmmp_oracle_homography(const acmmp_camera *ref, const acmmp_camera *src, const float *plane4,
                             float *H9) {
    f4 h = {plane4[0], plane4[1], plane4[2], plane4[3]};
    ComputeHomography(ref, src, h, H9);
}

/* draw `draw` of (pix, phase, stream): word draw mod 4 of block draw div 4 */
float acmmp_oracle_uniform(uint32_t seed_lo, uint32_t seed_hi, uint32_t pix, uint32_t draw,
                           uint32_t phase, uint32_t stream) {
    dm_rng g;
    g.k0 = seed_lo;
    g.k1 = seed_hi;
    g.pix = pix;
    g.phase = phase;
    g.stream = stream;
    g.draw = draw & ~3u;
    g.blk.x = g.blk.y = g.blk.z = g.blk.w = 0u;
    float u = 0.0f;
    for (uint32_t d = draw & ~3u; d <= draw; ++d) u = dm_rng_uniform(&g);
    return u;
}

float acmmp_oracle_expf(float x) { return dm_expf(x); }
float acmmp_oracle_sinf(float x) { return dm_sinf(x); }
float acmmp_oracle_cosf(float x) { return dm_cosf(x); }
float acmmp_oracle_acosf(float x) { return dm_acosf(x); }

int acmmp_oracle_checkerboard_rows(int H) { return checkerboard_rows(H); }

uint32_t acmmp_oracle_philox(uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
    return dm_philox_x(k0, k1, c0, c1, c2, c3);
}

void acmmp_oracle_philox4(uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                          uint32_t *out4) {
    const dm_u32x4 o = dm_philox4(k0, k1, c0, c1, c2, c3);
    out4[0] = o.x;
    out4[1] = o.y;
    out4[2] = o.z;
    out4[3] = o.w;
}

/* JBU_cu (src/ACMMP.cu:1458-1516) with RunJBU's Imagescale
 * (src/ACMMP.cpp:1014). Returns Imagescale; writes nothing when it is 1. */
int acmmp_oracle_jbu(const float *img, int W, int H, const float *depth, int sw, int sh, float *out) {
    const int isc = (H / sh) > (W / sw) ? (H / sh) : (W / sw);
    if (isc == 1) return isc;
    const int WinWidth = isc * isc + 1;
    const int num_neighbors = WinWidth / 2;
    #pragma omp parallel for schedule(static)
    for (int py = 0; py < H; ++py) {
        for (int px = 0; px < W; ++px) {
            const float scale = 1.0 * sw / W;
            const float sigmad = 0.50;
            const float sigmar = 25.5;
            const float o_y = py * scale;
            const float o_x = px * scale;
            const float refPix = img[py * W + px];
            float total_val = 0.0, normalizing_factor = 0.0;
            for (int j = -num_neighbors; j <= num_neighbors; ++j) {
                int r_y = o_y + j;
                r_y = (r_y > 0 ? (r_y < sh ? r_y : sh - 1) : 0);
                int r_ys = py + j;
                r_ys = (r_ys > 0 ? (r_ys < H ? r_ys : H - 1) : 0);
                for (int i = -num_neighbors; i <= num_neighbors; ++i) {
                    int r_x = o_x + i;
                    r_x = (r_x > 0 ? (r_x < sw ? r_x : sw - 1) : 0);
                    const float srcPix = depth[r_y * sw + r_x];
                    int r_xs = px + i;
                    r_xs = (r_xs > 0 ? (r_xs < W ? r_xs : W - 1) : 0);
                    const float neighborPix = img[r_ys * W + r_xs];
                    const float sgauss = SpatialGauss(o_x, o_y, r_x, r_y, sigmad);
                    const float rgauss = RangeGauss(fabsf(refPix - neighborPix), sigmar);
                    const float totalgauss = sgauss * rgauss;
                    normalizing_factor += totalgauss;
                    total_val += srcPix * totalgauss;
                }
            }
            out[py * W + px] = total_val / normalizing_factor;
        }
    }
    return isc;
}
