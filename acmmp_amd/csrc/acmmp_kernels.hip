// acmmp_kernels.hip — MI355X (gfx950, CDNA4) kernels for ACMMP::RunPatchMatch.
//
// Reference semantics: rlav440/ACMMP src/ACMMP.cu:17-1352 (device code) with the
// pinned semantics of SURVEY.md Appendix A and the arithmetic pins P1-P4 listed
// in oracle/acmmp_oracle.c / DESIGN.md §4. The CPU oracle restates the
// reference literally; this file is the GPU design:
//
//  * one lane per pixel, 64-lane waves laid along a row of ONE checkerboard
//    colour (colour-split layout, acmmp_internal.h) so every state access of
//    a wave is a contiguous 256-B..1-KiB segment;
//  * the reference patch of a pixel (36 bilateral weights w and w*ref, the
//    normalised ref mean/variance) is invariant across the 14*(N-1)
//    ComputeBilateralNCC calls of a pixel-iteration: it is computed once per
//    pixel-iteration into VGPRs (exact: same operations, same order);
//  * NCC calls for views whose sampled view weight is 0 are skipped: the
//    reference multiplies their (finite, >= 0) cost by 0 and adds +0, so the
//    result is bit-identical (refinement at :751 skips them explicitly);
//  * stateless Philox RNG (no 48-B curandState traffic per pixel);
//  * all per-launch constants (cameras, homography camera terms, image
//    pointers) sit in one device struct read through scalar loads.
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include "../../include/acmmp_detmath.h"
#include "acmmp_internal.h"

namespace acmmp {

#define DEV static __device__ __forceinline__

// Patch geometry fixed by the reference defaults (patch_size 11, increment 2:
// offsets {-5,-3,-1,1,3,5}^2, src/ACMMP.h:34,37). The engine rejects others.
constexpr int kTaps = 6;

// The kernel shapes below are the measured winners of the A/B experiments
// recorded in DESIGN.md §4 (the rejected variants live in git history only):
// 16 x 16 blocks of four 8 x 8-pixel waves (lanes column-major in 4 x 4
// quarters, lane_geom_of), candidate planes staged in LDS,
// refinement items packed across lanes, two software-pipelined patch rows,
// packed-pair u8 lerps, view selection in registers, 2 waves per SIMD.
#ifndef ACMMP_WAVE_ROWS
#define ACMMP_WAVE_ROWS 8
#endif
constexpr int kWaveRows = ACMMP_WAVE_ROWS;  // rows of pixels per wave (lane_geom_of; A/B builds only)
// Geometric-cost depth fetches issued ahead of their use (A/B builds only):
// bit 0 the final candidate costs, bit 1 the current plane, bit 2 refinement.
#ifndef ACMMP_GEOM_AHEAD
#define ACMMP_GEOM_AHEAD 7
#endif
constexpr int kSweepWaves = 2; // __launch_bounds__ waves per SIMD of k_sweep
// bilateral weights from the u8-form table (KViews::wlut; A/B: 0 = computed per tap)
#ifndef ACMMP_WEIGHT_LUT
#define ACMMP_WEIGHT_LUT 1
#endif
// the view selection's exact exp / division shortcuts (A/B: 0 = the literal forms)
#ifndef ACMMP_VS_SHORTCUTS
#define ACMMP_VS_SHORTCUTS 1
#endif

// ----------------------------------------------------------------- textures
// Through the global address space: a generic (flat) load would also count
// against lgkmcnt, so every later wait for a scalar or LDS load would drain
// it too (the geometric cost's depth fetch could never overlap anything).
typedef const __attribute__((address_space(1))) float gfloat;

DEV float texel(const float *img, int pitch, int W, int H, int x, int y) {
    x = x < 0 ? 0 : (x > W - 1 ? W - 1 : x);
    y = y < 0 ? 0 : (y > H - 1 ? H - 1 : y);
    return ((gfloat *)img)[y * pitch + x];
}

// pin P2 (tex2D linear, clamp; src/ACMMP.cu:394)
DEV float bilinear(const float *img, int pitch, int W, int H, float u, float v) {
    float xs = (u + 0.5f) - 0.5f;
    float ys = (v + 0.5f) - 0.5f;
    const float fw = (float)W, fh = (float)H;
    xs = (xs > -1.0f) ? xs : -1.0f;
    xs = (xs < fw) ? xs : fw;
    ys = (ys > -1.0f) ? ys : -1.0f;
    ys = (ys < fh) ? ys : fh;
    const float fx0 = dm_floor(xs), fy0 = dm_floor(ys);
    const float ax = xs - fx0, ay = ys - fy0;
    const int x0 = (int)fx0, y0 = (int)fy0;
    const int xa = x0 < 0 ? 0 : x0;
    const int xb = (x0 + 1) > (W - 1) ? (W - 1) : (x0 + 1);
    const int ya = y0 < 0 ? 0 : y0;
    const int yb = (y0 + 1) > (H - 1) ? (H - 1) : (y0 + 1);
    const int xa2 = xa > W - 1 ? W - 1 : xa;
    const int ya2 = ya > H - 1 ? H - 1 : ya;
    const int xb2 = xb < 0 ? 0 : xb;
    const int yb2 = yb < 0 ? 0 : yb;
    const float *r0 = img + ya2 * pitch;
    const float *r1 = img + yb2 * pitch;
    const float t00 = r0[xa2], t10 = r0[xb2];
    const float t01 = r1[xa2], t11 = r1[xb2];
    const float top = dm_fma(ax, t10 - t00, t00);
    const float bot = dm_fma(ax, t11 - t01, t01);
    return dm_fma(ay, bot - top, top);
}

// tex2D(depth, (int)x + 0.5, (int)y + 0.5) (src/ACMMP.cu:528)
DEV float tex_trunc(const float *img, int pitch, int W, int H, float u, float v) {
    const float fw = (float)W, fh = (float)H;
    u = (u > -1.0f) ? u : -1.0f;
    u = (u < fw) ? u : fw;
    v = (v > -1.0f) ? v : -1.0f;
    v = (v < fh) ? v : fh;
    return texel(img, pitch, W, H, (int)u, (int)v);
}

// ------------------------------------------------------------ geometry
// Get3DPoint (src/ACMMP.cu:123-128)
DEV void get3d(const acmmp_camera &c, int px, int py, float depth, float *X) {
    X[0] = depth * ((float)px - c.K[2]) / c.K[0];
    X[1] = depth * ((float)py - c.K[5]) / c.K[4];
    X[2] = depth;
}

// GetViewDirection (src/ACMMP.cu:130-142)
DEV float4 view_direction(const acmmp_camera &c, int px, int py, float depth) {
    float X[3];
    get3d(c, px, py, depth, X);
    const float norm = dm_sqrt(X[0] * X[0] + X[1] * X[1] + X[2] * X[2]);
    return make_float4(X[0] / norm, X[1] / norm, X[2] / norm, 0.0f);
}

// GetDistance2Origin (src/ACMMP.cu:144-149)
DEV float distance_to_origin(const acmmp_camera &c, int px, int py, float depth, float4 n) {
    float X[3];
    get3d(c, px, py, depth, X);
    return -(n.x * X[0] + n.y * X[1] + n.z * X[2]);
}

// ComputeDepthfromPlaneHypothesis (src/ACMMP.cu:163-168)
DEV float plane_depth(const acmmp_camera &c, float4 h, int px, int py) {
    return -h.w * c.K[0] /
           (((float)px - c.K[2]) * h.x + (c.K[0] / c.K[4]) * ((float)py - c.K[5]) * h.y + c.K[0] * h.z);
}

// NormalizeVec3 (src/ACMMP.cu:98-105), rsqrt pinned to 1/sqrt
DEV void normalize3(float4 &v) {
    const float n2 = v.x * v.x + v.y * v.y + v.z * v.z;
    const float inv = dm_rsqrt(n2);
    v.x *= inv;
    v.y *= inv;
    v.z *= inv;
}

DEV float dot3(float4 a, float4 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

// TransformNormal cam->world (src/ACMMP.cu:333-341)
DEV float4 to_world(const acmmp_camera &c, float4 h) {
    return make_float4(c.R[0] * h.x + c.R[3] * h.y + c.R[6] * h.z,
                       c.R[1] * h.x + c.R[4] * h.y + c.R[7] * h.z,
                       c.R[2] * h.x + c.R[5] * h.y + c.R[8] * h.z, h.w);
}

// TransformNormal2RefCam world->cam (src/ACMMP.cu:343-351)
DEV float4 to_cam(const acmmp_camera &c, float4 h) {
    return make_float4(c.R[0] * h.x + c.R[1] * h.y + c.R[2] * h.z,
                       c.R[3] * h.x + c.R[4] * h.y + c.R[5] * h.z,
                       c.R[6] * h.x + c.R[7] * h.y + c.R[8] * h.z, h.w);
}

// GenerateRandomNormal (src/ACMMP.cu:170-196)
DEV float4 random_normal(const acmmp_camera &c, int px, int py, dm_rng &rs, float depth) {
    float q1 = 1.0f, q2 = 1.0f, s = 2.0f;
    int guard = 0;
    while (s >= 1.0f && guard < 1000) {
        q1 = 2.0f * dm_rng_uniform(&rs) - 1.0f;
        q2 = 2.0f * dm_rng_uniform(&rs) - 1.0f;
        s = q1 * q1 + q2 * q2;
        ++guard;
    }
    const float sq = dm_sqrt(1.0f - s);
    float4 n = make_float4(2.0f * q1 * sq, 2.0f * q2 * sq, 1.0f - 2.0f * s, 0.0f);
    const float4 vd = view_direction(c, px, py, depth);
    if (n.x * vd.x + n.y * vd.y + n.z * vd.z > 0.0f) {
        n.x = -n.x;
        n.y = -n.y;
        n.z = -n.z;
    }
    normalize3(n);
    return n;
}

// GeneratePerturbedNormal (src/ACMMP.cu:198-233)
DEV float4 perturbed_normal(const acmmp_camera &c, int px, int py, float4 normal, dm_rng &rs,
                            float perturbation) {
    const float4 vd = view_direction(c, px, py, 1.0f);
    const float a1 = (dm_rng_uniform(&rs) - 0.5f) * perturbation;
    const float a2 = (dm_rng_uniform(&rs) - 0.5f) * perturbation;
    const float a3 = (dm_rng_uniform(&rs) - 0.5f) * perturbation;
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
    float4 np = make_float4(R[0] * normal.x + R[1] * normal.y + R[2] * normal.z,
                            R[3] * normal.x + R[4] * normal.y + R[5] * normal.z,
                            R[6] * normal.x + R[7] * normal.y + R[8] * normal.z, normal.w);
    if (dot3(np, vd) >= 0.0f) np = normal;
    normalize3(np);
    return np;
}

// Exactly rounded 1/z. The IEEE division sequence (v_div_scale / v_rcp /
// 4 fma / v_div_fmas / v_div_fixup) is the pinned semantics. Inside the
// exponent window below the sample loop replaces it by v_rcp_f32 + one fma
// Newton step, which acmmp_selftest_reciprocal() proves bit-identical for
// EVERY float in that window on this hardware.
DEV float recip_newton(float z) {
    const float r = __builtin_amdgcn_rcpf(z);
    const float e = dm_fma(-z, r, 1.0f);
    return dm_fma(e, r, r);
}
DEV bool recip_fast_window(float z) {
    const float az = dm_fabs(z);
    return az >= 0x1p-125f && az < 0x1p125f;
}
DEV float recip_exact(float z) { return 1.0f / z; }


// ------------------------------------------------------ homography + NCC
// ComputeHomography (src/ACMMP.cu:262-322) with the camera-only terms
// precomputed per view (ViewRel) and pin P4.
DEV void homography(const KViews &kv, int v, float4 h, float *H) {
    const ViewRel &r = kv.rel[v];
    const acmmp_camera &rc = kv.cam[0];
    const acmmp_camera &sc = kv.cam[v];
    const float inv_w = 1.0f / h.w;
    float G[9];
    G[0] = r.Rr[0] - (r.tr[0] * h.x) * inv_w;
    G[1] = r.Rr[1] - (r.tr[0] * h.y) * inv_w;
    G[2] = r.Rr[2] - (r.tr[0] * h.z) * inv_w;
    G[3] = r.Rr[3] - (r.tr[1] * h.x) * inv_w;
    G[4] = r.Rr[4] - (r.tr[1] * h.y) * inv_w;
    G[5] = r.Rr[5] - (r.tr[1] * h.z) * inv_w;
    G[6] = r.Rr[6] - (r.tr[2] * h.x) * inv_w;
    G[7] = r.Rr[7] - (r.tr[2] * h.y) * inv_w;
    G[8] = r.Rr[8] - (r.tr[2] * h.z) * inv_w;
    const float ik0 = kv.inv_k0, ik4 = kv.inv_k4;
    float t[9];
    t[0] = G[0] * ik0;
    t[1] = G[1] * ik4;
    t[2] = ((-G[0] * rc.K[2]) * ik0 - (G[1] * rc.K[5]) * ik4) + G[2];
    t[3] = G[3] * ik0;
    t[4] = G[4] * ik4;
    t[5] = ((-G[3] * rc.K[2]) * ik0 - (G[4] * rc.K[5]) * ik4) + G[5];
    t[6] = G[6] * ik0;
    t[7] = G[7] * ik4;
    t[8] = ((-G[6] * rc.K[2]) * ik0 - (G[7] * rc.K[5]) * ik4) + G[8];
    H[0] = sc.K[0] * t[0] + sc.K[2] * t[6];
    H[1] = sc.K[0] * t[1] + sc.K[2] * t[7];
    H[2] = sc.K[0] * t[2] + sc.K[2] * t[8];
    H[3] = sc.K[4] * t[3] + sc.K[5] * t[6];
    H[4] = sc.K[4] * t[4] + sc.K[5] * t[7];
    H[5] = sc.K[4] * t[5] + sc.K[5] * t[8];
    H[6] = sc.K[8] * t[6];
    H[7] = sc.K[8] * t[7];
    H[8] = sc.K[8] * t[8];
}

// ComputeCorrespondingPoint (src/ACMMP.cu:324-331), pin P1
DEV float2 project(const float *H, float x, float y) {
    const float px = dm_fma(H[1], y, dm_fma(H[0], x, H[2]));
    const float py = dm_fma(H[4], y, dm_fma(H[3], x, H[5]));
    const float pz = dm_fma(H[7], y, dm_fma(H[6], x, H[8]));
    const float inv = recip_exact(pz);
    return make_float2(px * inv, py * inv);
}

// Texel modes of the gather kernels (template parameter TX):
//   bit 0 (kTxWide): record index by integer multiply-add (views of 2^24+
//          records), else exactly in fp32;
//   bit 1 (kTxU8):   the padded source views hold u8 texel quads (every view
//          of the problem is integer-valued in [0, 255], which 8-bit JPEG
//          input at native size is): one 4-byte record per bilinear
//          footprint instead of 16 bytes; v_cvt_f32_ubyte* restores the exact
//          fp32 texel values, so the arithmetic is unchanged.
//   bit 2 (kTxH16):  the padded source views hold f16 "difference quads"
//          (t00, t01, t10 - t00, t11 - t01) for views whose every stored value
//          is exact in f16 (8-bit input is): 8 bytes per footprint, and the
//          two row lerps are v_fma_mix_f32 straight from the f16 halves (the
//          f16 -> f32 widening is exact, the fma is the pinned fp32 fma).
//   bit 3 (kTxFrac8): acmmp_params::texture_filter8 — the bilinear fractions
//                    rounded to the CUDA texture unit's 1.8 fixed point
//                    (instantiated for the non-wide u8 and fp32 forms)
constexpr int kTxWide = 1, kTxU8 = 2, kTxH16 = 4, kTxFrac8 = 8;

// Source-image sampler: one buffer resource (SRD) per view over the padded
// copy (KViews::pad), built from wave-uniform values (the view index is a
// uniform loop counter) so the loads are index-addressed (`idxen`) buffer
// loads with the record stride in the descriptor.
struct SrcImage {
    __amdgpu_buffer_rsrc_t rsrc;
    int pitch, W, H;
    float fpitch, fp1;  // pitch and pitch + 1 as floats (exact: < 2^24)
};

template <int TX>
DEV SrcImage src_image(const KViews &kv, int v) {
    SrcImage s;
    s.pitch = kv.ppitch[v];
    s.W = kv.cam[v].width;
    s.H = kv.cam[v].height;
    // structured view, indexed loads (idxen): 8-byte records (one fp32 row
    // pair) or 4-byte records (one u8 2x2 quad)
    s.rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)kv.pad[v], (short)((TX & kTxU8) ? 4 : 8), s.pitch * (s.H + 2),
                                               0x00020000);
    s.fp1 = (float)(s.pitch + 1);
    s.fpitch = (float)s.pitch;
    return s;
}


typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// ---------------------------------------------------------- ref-image tile
// A block covers kBX colour-split columns (k0..k0+kBX-1) x kBY rows of ONE
// colour c (256 threads). Both patch offsets i, j are odd, so every
// reference sample of a colour-c pixel is itself a colour-c pixel: the
// block's whole reference footprint is a (kBX + 6) x (kBY + 10) window of the
// colour-c plane, staged once in LDS (clamp-to-edge baked in); the address
// of a sample is a compile-time offset from the lane's base.
//
// kBX = 16 colour-split columns x 16 rows packs a block's four waves (8 x 8
// colour-split pixels each, kWaveRows) 2 x 2, so they share most
// source-view rows of their patches in the CU's L1, and keeps the ragged
// last block column narrow (Wh = 800 at 1600 px: 50 x 75 blocks). cfg2, ms
// per k_sweep launch (profiles/r02_block_shape.md): 64 x 4 blocks of
// 16 x 4 waves 4.66, 32 x 8 4.41, 16 x 16 4.28, 16 x 16 of 8 x 8 waves
// 4.19, 8 x 32 4.18.
#ifndef ACMMP_KBX
#define ACMMP_KBX 16
#endif
// threads per block of the colour-split kernels (A/B builds: 512 puts a CU's
// eight waves in one block, i.e. on adjacent pixels)
#ifndef ACMMP_BLOCK_THREADS
#define ACMMP_BLOCK_THREADS 256
#endif
constexpr int kBX = ACMMP_KBX, kBY = ACMMP_BLOCK_THREADS / kBX;  // ACMMP_KBX: A/B builds only
constexpr int kTileW = kBX + 6, kTileH = kBY + 10;

DEV void load_ref_tile(const KViews &kv, float *tile, int k0, int y0, int colour) {
    const float *img = kv.img[0];
    const int pitch = kv.ipitch[0], W = kv.W, H = kv.H;
    // all of a thread's texels loaded before any is stored; a thread past the
    // end repeats the last element (same value, same address), so no load
    // sits in a conditional block waited on alone
    constexpr int kN = kTileW * kTileH, kIt = (kN + kBX * kBY - 1) / (kBX * kBY);
    float v[kIt];
    int at[kIt];
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
        int e = threadIdx.y * kBX + threadIdx.x + it * kBX * kBY;
        e = e < kN ? e : kN - 1;
        const int r = e / kTileW, kk = e - r * kTileW;
        const int yy = y0 - 5 + r;
        const int kc = k0 - 3 + kk;
        const int par = (yy + colour) & 1;
        const int xx = 2 * kc + par;
        at[it] = e;
        v[it] = texel(img, pitch, W, H, xx, yy);
    }
#pragma unroll
    for (int it = 0; it < kIt; ++it) tile[at[it]] = v[it];
}

// Reference-side invariants of ComputeBilateralNCC (src/ACMMP.cu:372-421):
// the 36 bilateral weights (ComputeBilateralWeight :353-358) and the
// normalised ref mean / variance — identical for all 14*(N-1) calls of a
// pixel-iteration, so computed once (same operations, same order).
//
// The source side of the NCC runs on PAIRS of patch columns (2p, 2p+1) held
// as packed-FP32 lanes (SoA): one v_pk_* instruction does the same IEEE
// operation for both samples of a pair, and the pair's weights come from LDS
// as one float2 (w_a, w_b), the reference pair from the tile, so no register
// shuffling is needed to feed the packed ops. LDS slot of (column pair p,
// patch row jj): jj * 3 + p, in the order the row loop reads them.
constexpr int kPairs = kTaps / 2;
constexpr int kSlots = kPairs * kTaps;
DEV int wslot(int p, int jj) { return jj * kPairs + p; }
typedef float2 WSlot;

struct PixPatch {
    WSlot *w;        // LDS: slot k of this lane at [k * kThreads]
    const float *rt; // LDS: this lane's first reference sample in the tile (tile + tb)
    int wo;          // this lane's offset into the weight array (w = wbase + wo)
    float mean;      // sum_ref * inv_bilateral_weight_sum
    float var;       // var_ref
    float inv_wsum;  // inv_bilateral_weight_sum
};

// 18 float2 rows of 256 lanes: 36 KB + the 3.9 KB tile per 256-thread block,
// so four blocks (16 waves) fit a CU's 160 KB of LDS. A wave's read of one
// slot is a conflict-free ds_read_b64 and costs no VGPRs between NCC calls;
// the matching reference pair comes from the tile (ds_read2_b32).
constexpr int kThreads = kBX * kBY;

DEV float bilateral_weight(float xd, float yd, float pix, float cpix, float ss, float sc) {
    const float spatial = dm_sqrt(xd * xd + yd * yd);
    const float color = dm_fabs(pix - cpix);
    return dm_expf(-spatial / (2.0f * ss * ss) - color / (2.0f * sc * sc));
}

// The bilateral-weight table (KViews::wlut) staged in LDS by the block
// (kernels of the u8 texel form, whose reference texels are all integers in
// [0, 255]); the caller's __syncthreads publishes it.
DEV void load_wlut(const KViews &kv, float *wl) {
    const int t = threadIdx.y * kBX + threadIdx.x;
    for (int i = t; i < kWlutClasses * 256; i += kBX * kBY) wl[i] = (&kv.wlut[0][0])[i];
}

// tb = tile index of sample (ii=0, jj=0) of this lane: ty*kTileW + tx + s.
// wlut: the LDS weight table (u8 texel form) or nullptr (weights computed).
DEV void pixel_patch(const KViews &kv, const float *tile, int tb, int s, PixPatch &pp, const float *wlut = nullptr) {
    const float ss = kv.prm.sigma_spatial, sc = kv.prm.sigma_color;
    const float center = tile[tb - s + 5 * kTileW + 3];
    float sum_ref = 0.0f, sum_rr = 0.0f, bw = 0.0f;
#pragma unroll
    for (int ii = 0; ii < kTaps; ++ii) {
        float r_ref = 0.0f, r_rr = 0.0f, r_w = 0.0f;
#pragma unroll
        for (int jj = 0; jj < kTaps; ++jj) {
            const float r = tile[tb + ii + 2 * kTileW * jj];
            // |I - I_c| of integer texels in [0, 255]: the table holds the
            // weight this expression gives for it (bit-identical)
            const float w = wlut ? wlut[wlut_class((ii < 3 ? 5 - 2 * ii : 2 * ii - 5) / 2,
                                                   (jj < 3 ? 5 - 2 * jj : 2 * jj - 5) / 2) * 256 +
                                        (int)dm_fabs(r - center)]
                                 : bilateral_weight((float)(-5 + 2 * ii), (float)(-5 + 2 * jj), r, center, ss, sc);
            const float wr = w * r;
            r_ref = dm_fma(w, r, r_ref);  // nvcc's contraction of `sum += w * r` (pin P3)
            r_rr = dm_fma(wr, r, r_rr);
            r_w += w;
            float *slot = reinterpret_cast<float *>(&pp.w[wslot(ii >> 1, jj) * kThreads]);
            slot[ii & 1] = w;
        }
        sum_ref += r_ref;
        sum_rr += r_rr;
        bw += r_w;
    }
    const float inv = 1.0f / bw;
    sum_ref *= inv;
    pp.mean = sum_ref;
    pp.var = dm_fma(sum_rr, inv, -(sum_ref * sum_ref));  // `rr * inv - m * m` contracted (pin P3)
    pp.inv_wsum = inv;
}

typedef float f2v __attribute__((ext_vector_type(2)));
// texture_filter8: a bilinear fraction in [0, 1) rounded to the texture
// unit's 1.8 fixed point (1/256 steps, 1.0 representable), exactly: x * 256
// and the scale back are exact, rint is round-half-even.
DEV f2v frac8(f2v a) {
    return f2v{__builtin_rintf(a.x * 256.0f), __builtin_rintf(a.y * 256.0f)} * 0.00390625f;
}
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// llvm.amdgcn.struct.ptr.buffer.load: the idxen form of buffer_load
// (address = base + vindex * stride + voffset); clang has no builtin for it.
__device__ u32x4 amdgcn_struct_buffer_load_b128(__amdgpu_buffer_rsrc_t rsrc, int vindex, int voffset, int soffset,
                                                int aux) __asm("llvm.amdgcn.struct.ptr.buffer.load.v4i32");
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
__device__ u32x2 amdgcn_struct_buffer_load_b64(__amdgpu_buffer_rsrc_t rsrc, int vindex, int voffset, int soffset,
                                               int aux) __asm("llvm.amdgcn.struct.ptr.buffer.load.v2i32");
__device__ unsigned amdgcn_struct_buffer_load_b32(__amdgpu_buffer_rsrc_t rsrc, int vindex, int voffset, int soffset,
                                                  int aux) __asm("llvm.amdgcn.struct.ptr.buffer.load.i32");

DEV f2v fma2(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }
DEV f2v splat(float v) { return f2v{v, v}; }

// Bilinear value of one fetched sample t = (t00, t01, t10, t11) (pin P2's
// lerp order): top = fma(ax, t10 - t00, t00), bot = fma(ax, t11 - t01, t01)
// as one packed pair, then fma(ay, bot - top, top).
DEV float lerp_sample(u32x4 t, float ax, float ay) {
    const f2v lo = f2v{__uint_as_float(t.x), __uint_as_float(t.y)};
    const f2v hi = f2v{__uint_as_float(t.z), __uint_as_float(t.w)};
    const f2v tb = fma2(splat(ax), hi - lo, lo);
    return dm_fma(ay, tb.y - tb.x, tb.x);
}

// One patch row's gathers in flight: the fetched footprints (in the form
// of TX) and the bilinear fractions of the row's 6 samples.
template <int TX>
struct RowFetch {
    u32x4 t[kTaps];   // fp32 row pairs
    unsigned q[kTaps];  // u8 quads
    u32x2 hq[kTaps];  // f16 difference quads
    f2v ax[kPairs], ay[kPairs];
};

// Projection, clamp, fractions and record index of patch row jj, and its 6
// loads issued (not waited for).
template <bool FAST, int TX>
DEV void fetch_row(const SrcImage &im, const float *H, const f2v *cx, const f2v *cy, const f2v *cz, int py, int jj,
                   RowFetch<TX> &rf) {
    constexpr bool WIDE = (TX & kTxWide) != 0, U8 = (TX & kTxU8) != 0, H16 = (TX & kTxH16) != 0;
    constexpr bool F8 = (TX & kTxFrac8) != 0;
    const f2v fw = splat((float)im.W), fh = splat((float)im.H);
    const f2v y = splat((float)(py - 5 + 2 * jj));
#pragma unroll
    for (int p = 0; p < kPairs; ++p) {
        const f2v hx = fma2(splat(H[1]), y, cx[p]);
        const f2v hy = fma2(splat(H[4]), y, cy[p]);
        const f2v hz = fma2(splat(H[7]), y, cz[p]);
        f2v inv;
        if (FAST) {  // v_rcp + one Newton step == IEEE 1/z in the window
            const f2v r = f2v{__builtin_amdgcn_rcpf(hz.x), __builtin_amdgcn_rcpf(hz.y)};
            inv = fma2(fma2(-hz, r, splat(1.0f)), r, r);
        } else {
            inv = f2v{1.0f / hz.x, 1.0f / hz.y};
        }
        f2v u = hx * inv, v = hy * inv;
        u = (u + 0.5f) - 0.5f;
        v = (v + 0.5f) - 0.5f;
        // clamp to [-1, W] x [-1, H]. FAST: every value is finite or +-inf
        // (finite homography, |hz| inside the reciprocal window), where
        // v_med3 equals max-then-min. Otherwise v_max/v_min (NaN -> -1;
        // bounds are never +-0) == the oracle's selects.
        f2v xs, ys;
        if (FAST) {
            xs = f2v{__builtin_amdgcn_fmed3f(u.x, -1.0f, fw.x), __builtin_amdgcn_fmed3f(u.y, -1.0f, fw.x)};
            ys = f2v{__builtin_amdgcn_fmed3f(v.x, -1.0f, fh.x), __builtin_amdgcn_fmed3f(v.y, -1.0f, fh.x)};
        } else {
            xs = f2v{fminf(fmaxf(u.x, -1.0f), fw.x), fminf(fmaxf(u.y, -1.0f), fw.x)};
            ys = f2v{fminf(fmaxf(v.x, -1.0f), fh.x), fminf(fmaxf(v.y, -1.0f), fh.x)};
        }
        const f2v flx = f2v{dm_floor(xs.x), dm_floor(xs.y)};
        const f2v fly = f2v{dm_floor(ys.x), dm_floor(ys.y)};
        rf.ax[p] = xs - flx;
        rf.ay[p] = ys - fly;
        if (F8) {
            rf.ax[p] = frac8(rf.ax[p]);
            rf.ay[p] = frac8(rf.ay[p]);
        }
        // record index (y0 + 1) * pitch + x0 + 1
        unsigned ia, ib;
        if (!WIDE) {
            // = fma(y0, pitch, x0 + pitch + 1): integers below 2^24, so
            // exact in fp32 (the engine selects WIDE otherwise)
            const f2v idx = fma2(fly, splat(im.fpitch), flx + im.fp1);
            ia = (unsigned)idx.x;
            ib = (unsigned)idx.y;
        } else {
            // views of 2^24 records or more: integer multiply-add (24-bit
            // operands, 32-bit result)
            const f2v q = flx + 1.0f, r = fly + 1.0f;
            ia = __umul24((unsigned)r.x, (unsigned)im.pitch) + (unsigned)q.x;
            ib = __umul24((unsigned)r.y, (unsigned)im.pitch) + (unsigned)q.y;
        }
        if (H16) {
            rf.hq[2 * p] = amdgcn_struct_buffer_load_b64(im.rsrc, (int)ia, 0, 0, 0);
            rf.hq[2 * p + 1] = amdgcn_struct_buffer_load_b64(im.rsrc, (int)ib, 0, 0, 0);
        } else if (U8) {
            rf.q[2 * p] = amdgcn_struct_buffer_load_b32(im.rsrc, (int)ia, 0, 0, 0);
            rf.q[2 * p + 1] = amdgcn_struct_buffer_load_b32(im.rsrc, (int)ib, 0, 0, 0);
        } else {
            rf.t[2 * p] = amdgcn_struct_buffer_load_b128(im.rsrc, (int)ia, 0, 0, 0);
            rf.t[2 * p + 1] = amdgcn_struct_buffer_load_b128(im.rsrc, (int)ib, 0, 0, 0);
        }
    }
}

// Bilinear values of a fetched row and their weighted sums into the
// per-column accumulators (w from the LDS weight slots, ref from the tile).
template <int TX>
DEV void reduce_row(const RowFetch<TX> &rf, const WSlot *wl, const float *rt, int wstride, int jj, f2v *acc_s,
                    f2v *acc_ss, f2v *acc_rs) {
    constexpr bool U8 = (TX & kTxU8) != 0, H16 = (TX & kTxH16) != 0;
#pragma unroll
    for (int p = 0; p < kPairs; ++p) {
        f2v sv;
        if (H16) {
            // row lerps fma(ax, t1x - t0x, t0x) as v_fma_mix_f32 on the
            // halves, then the column lerp of both samples packed (words
            // copied out first: clang's __builtin_bit_cast of a
            // vector-element lvalue reads element 0)
            const unsigned wa0 = rf.hq[2 * p].x, wa1 = rf.hq[2 * p].y;
            const unsigned wb0 = rf.hq[2 * p + 1].x, wb1 = rf.hq[2 * p + 1].y;
            const h2v ta = __builtin_bit_cast(h2v, wa0), da = __builtin_bit_cast(h2v, wa1);
            const h2v tb = __builtin_bit_cast(h2v, wb0), db = __builtin_bit_cast(h2v, wb1);
            const f2v r0 = f2v{__builtin_fmaf(rf.ax[p].x, (float)da.x, (float)ta.x),
                               __builtin_fmaf(rf.ax[p].y, (float)db.x, (float)tb.x)};
            const f2v r1 = f2v{__builtin_fmaf(rf.ax[p].x, (float)da.y, (float)ta.y),
                               __builtin_fmaf(rf.ax[p].y, (float)db.y, (float)tb.y)};
            sv = fma2(rf.ay[p], r1 - r0, r0);
        } else if (U8) {
            // lerp_sample's operations with the pair's two samples in the two
            // components (sample a in .x, b in .y, as ax / ay already are):
            // top = fma(ax, t10 - t00, t00), bot = fma(ax, t11 - t01, t01),
            // fma(ay, bot - top, top) — 6 packed ops per pair instead of 8
            const unsigned qa = rf.q[2 * p], qb = rf.q[2 * p + 1];
            const f2v t00 = f2v{(float)(qa & 0xffu), (float)(qb & 0xffu)};
            const f2v t01 = f2v{(float)((qa >> 8) & 0xffu), (float)((qb >> 8) & 0xffu)};
            const f2v t10 = f2v{(float)((qa >> 16) & 0xffu), (float)((qb >> 16) & 0xffu)};
            const f2v t11 = f2v{(float)(qa >> 24), (float)(qb >> 24)};
            const f2v top = fma2(rf.ax[p], t10 - t00, t00);
            const f2v bot = fma2(rf.ax[p], t11 - t01, t01);
            sv = fma2(rf.ay[p], bot - top, top);
        } else {
            sv = f2v{lerp_sample(rf.t[2 * p], rf.ax[p].x, rf.ay[p].x),
                     lerp_sample(rf.t[2 * p + 1], rf.ax[p].y, rf.ay[p].y)};
        }
        // w from the weight slots, ref from the tile: w * ref is the same
        // IEEE product pixel_patch formed, so re-forming it is exact
        const WSlot w = wl[wslot(p, jj) * wstride];
        const float *rr = rt + 2 * kTileW * jj + 2 * p;
        const f2v wv = f2v{w.x, w.y};
        const f2v wr = wv * f2v{rr[0], rr[1]};
        const f2v ws = wv * sv;
        acc_s[p] = fma2(wv, sv, acc_s[p]);  // `sum += w * s` contracted (pin P3)
        acc_ss[p] = fma2(ws, sv, acc_ss[p]);
        acc_rs[p] = fma2(wr, sv, acc_rs[p]);
    }
}

// Source-sample reduction of ComputeBilateralNCC (src/ACMMP.cu:382-412).
//
// Per sample: projection (pin P1, the x-terms hoisted per column), the
// coordinate clamp of pin P2, and ONE load of the 2x2 bilinear footprint
// from the padded source view (KViews::pad) at record (y0 + 1, x0 + 1).
//
// Rows are gathered one at a time (a lane's 6 samples of a row sit in the
// same one or two cache lines) and accumulated into per-column partial
// sums: within a column the rows are still added in order jj = 0..5,
// columns are summed at the end in order ii — the pinned order
// (src/ACMMP.cu:382-412). The row loop is software-pipelined: row jj + 1's
// loads are issued before row jj is reduced, so a row's gather latency
// overlaps the previous row's arithmetic.
template <bool FAST, int TX>
DEV void ncc_sums_rows(const SrcImage &im, const float *H, const WSlot *wl, const float *rt, int wstride, int px,
                       int py, float &sum_src, float &sum_ss, float &sum_rs) {
    f2v cx[kPairs], cy[kPairs], cz[kPairs];
#pragma unroll
    for (int p = 0; p < kPairs; ++p) {
        const f2v x = f2v{(float)(px - 5 + 4 * p), (float)(px - 3 + 4 * p)};
        cx[p] = fma2(splat(H[0]), x, splat(H[2]));
        cy[p] = fma2(splat(H[3]), x, splat(H[5]));
        cz[p] = fma2(splat(H[6]), x, splat(H[8]));
    }
    f2v acc_s[kPairs], acc_ss[kPairs], acc_rs[kPairs];
#pragma unroll
    for (int p = 0; p < kPairs; ++p) acc_s[p] = acc_ss[p] = acc_rs[p] = splat(0.0f);
    // two rows per trip (ping-pong fetch buffers, no register copies)
    RowFetch<TX> ra, rb;
    fetch_row<FAST, TX>(im, H, cx, cy, cz, py, 0, ra);
#pragma unroll 1
    for (int jj = 0; jj < kTaps; jj += 2) {
        fetch_row<FAST, TX>(im, H, cx, cy, cz, py, jj + 1, rb);
        reduce_row<TX>(ra, wl, rt, wstride, jj, acc_s, acc_ss, acc_rs);
        if (jj + 2 < kTaps) fetch_row<FAST, TX>(im, H, cx, cy, cz, py, jj + 2, ra);
        reduce_row<TX>(rb, wl, rt, wstride, jj + 1, acc_s, acc_ss, acc_rs);
    }
    sum_src = 0.0f;
    sum_ss = 0.0f;
    sum_rs = 0.0f;
#pragma unroll
    for (int p = 0; p < kPairs; ++p) {
        sum_src += acc_s[p].x;
        sum_src += acc_s[p].y;
        sum_ss += acc_ss[p].x;
        sum_ss += acc_ss[p].y;
        sum_rs += acc_rs[p].x;
        sum_rs += acc_rs[p].y;
    }
}

// Source-sample reduction of ComputeBilateralNCC (src/ACMMP.cu:382-412):
// returns the three weighted sums (ncc_sums_rows above).
template <bool FAST, int TX>
DEV void ncc_sums(const SrcImage &im, const float *H, const PixPatch &pp, int px, int py, float &sum_src,
                  float &sum_ss, float &sum_rs) {
    // re-read weights from LDS each call rather than caching them in VGPRs
    // (launder the integer offset, not the pointer, so the LDS address space
    // stays visible and the reads are ds_read, not flat)
    int wo = pp.wo;
    asm volatile("" : "+v"(wo));
    const WSlot *wl = pp.w - pp.wo + wo;
    ncc_sums_rows<FAST, TX>(im, H, wl, pp.rt, kThreads, px, py, sum_src, sum_ss, sum_rs);
}

// ComputeBilateralNCC (src/ACMMP.cu:360-432) for source view v (1-based,
// wave-uniform). Reference samples come from the LDS tile, source samples
// through ncc_sums.
template <int TX>
DEV float bilateral_ncc(const KViews &kv, const float *tile, int tb, const PixPatch &pp, int v, int px,
                        int py, float4 h) {
    const float cost_max = 2.0f;
    const float kMinVar = 1e-5f;
    // var_ref is invariant: when it is below kMinVar (or the centre maps
    // outside the source) every call returns cost_max.
    if (pp.var < kMinVar) return cost_max;
    const SrcImage im = src_image<TX>(kv, v);
    float H[9];
    homography(kv, v, h, H);
    const float2 pt = project(H, (float)px, (float)py);
    if (pt.x >= (float)im.W || pt.x < 0.0f || pt.y >= (float)im.H || pt.y < 0.0f) return cost_max;
    float sum_src, sum_ss, sum_rs;
    // hz is affine in the sample position, so its values over the patch lie
    // between the four corner values (up to rounding: the window test uses a
    // 2x margin). Inside the window the Newton reciprocal is bit-identical to
    // IEEE 1/z (exhaustive proof: acmmp_selftest_reciprocal).
    const float xl = (float)(px - 5), xr = (float)(px + 5), yt = (float)(py - 5), yb = (float)(py + 5);
    const float z00 = dm_fma(H[7], yt, dm_fma(H[6], xl, H[8]));
    const float z10 = dm_fma(H[7], yt, dm_fma(H[6], xr, H[8]));
    const float z01 = dm_fma(H[7], yb, dm_fma(H[6], xl, H[8]));
    const float z11 = dm_fma(H[7], yb, dm_fma(H[6], xr, H[8]));
    const float zmin = fminf(fminf(z00, z10), fminf(z01, z11));
    const float zmax = fmaxf(fmaxf(z00, z10), fmaxf(z01, z11));
    const bool fast = (zmin >= 0x1p-124f && zmax < 0x1p124f) || (zmax <= -0x1p-124f && zmin > -0x1p124f);
    if (fast) ncc_sums<true, TX>(im, H, pp, px, py, sum_src, sum_ss, sum_rs);
    else ncc_sums<false, TX>(im, H, pp, px, py, sum_src, sum_ss, sum_rs);
    sum_src *= pp.inv_wsum;
    const float var_src = dm_fma(sum_ss, pp.inv_wsum, -(sum_src * sum_src));  // pin P3
    if (var_src < kMinVar) return cost_max;
    const float covar = dm_fma(sum_rs, pp.inv_wsum, -(pp.mean * sum_src));
    const float var_rs = dm_sqrt(pp.var * var_src);
    float c = 1.0f - covar / var_rs;
    c = (c < cost_max) ? c : cost_max;
    c = (c > 0.0f) ? c : 0.0f;
    return c;
}

// ComputeMultiViewInitialCostandSelectedViews (src/ACMMP.cu:434-471)
template <int NS, int TX>
DEV float initial_cost(const KViews &kv, const float *tile, int tb, const PixPatch &pp, int px, int py,
                       float4 h, uint32_t &sel) {
    const int nsrc = kv.nsrc;
    float cv[NS];
    float cs[NS];
    int num_valid = 0;
    for (int i = 0; i < nsrc; ++i) {
        const float c = bilateral_ncc<TX>(kv, tile, tb, pp, i + 1, px, py, h);
        cv[i] = c;
        cs[i] = c;
        if (c < 2.0f) num_valid++;
    }
    for (int i = 1; i < nsrc; i++) {  // sort_small (src/ACMMP.cu:24-33)
        const float tmp = cs[i];
        int j;
        for (j = i; j >= 1 && tmp < cs[j - 1]; j--) cs[j] = cs[j - 1];
        cs[j] = tmp;
    }
    sel = 0;
    const int top_k = num_valid < kv.prm.top_k ? num_valid : kv.prm.top_k;
    if (top_k > 0) {
        float cost = 0.0f;
        for (int i = 0; i < top_k; ++i) cost += cs[i];
        const float thr = cs[top_k - 1];
        for (int i = 0; i < nsrc; ++i)
            if (cv[i] <= thr) sel |= (1u << i);
        return cost / (float)top_k;
    }
    return 2.0f;
}

// ComputeGeomConsistencyCost (src/ACMMP.cu:518-543), split so the view-
// independent half is formed once per hypothesis: geom_ref is the world
// point of the hypothesis at the pixel (ComputeDepthfromPlaneHypothesis +
// Get3DPointonWorld_cu :480-504), geom_cost_at projects it into source v,
// fetches the source depth and measures the reprojection error. Same
// operations in the same order as the unsplit function (the camera offsets
// -(R^T t) come precomputed in KViews::cw, formed by the same expression).
struct GeomRef {
    float Wp[3];
};

// -(R^T t) of camera v, component k. The product takes it from KViews::cw
// (formed on the host by the same expression: bit-identical without
// contraction); the fidelity-study build (ACMMP_CUDA_NUMERICS) forms it here
// so the device's FMA contraction and FTZ apply to it as nvcc's --fmad does
// to Get3DPointonWorld_cu (src/ACMMP.cu:490-504).
DEV float cam_offset(const KViews &kv, int v, int k) {
#ifdef ACMMP_CUDA_NUMERICS
    const acmmp_camera &c = kv.cam[v];
    return -(c.R[k] * c.t[0] + c.R[3 + k] * c.t[1] + c.R[6 + k] * c.t[2]);
#else
    return kv.cw[v][k];
#endif
}

DEV GeomRef geom_ref(const KViews &kv, float4 h, int px, int py) {
    const acmmp_camera &rc = kv.cam[0];
    const float depth = plane_depth(rc, h, px, py);
    float X[3];
    X[0] = depth * ((float)px - rc.K[2]) / rc.K[0];
    X[1] = depth * ((float)py - rc.K[5]) / rc.K[4];
    X[2] = depth;
    GeomRef g;
    g.Wp[0] = (rc.R[0] * X[0] + rc.R[3] * X[1] + rc.R[6] * X[2]) + cam_offset(kv, 0, 0);
    g.Wp[1] = (rc.R[1] * X[0] + rc.R[4] * X[1] + rc.R[7] * X[2]) + cam_offset(kv, 0, 1);
    g.Wp[2] = (rc.R[2] * X[0] + rc.R[5] * X[1] + rc.R[8] * X[2]) + cam_offset(kv, 0, 2);
    return g;
}

// geom_cost_at in two halves, so a caller can issue the source-depth
// fetches of several views (or one ahead of an NCC) before it consumes them:
// geom_fetch projects into source v and loads the depth (always in bounds:
// tex_trunc clamps, NaN included), geom_finish is the rest.
struct GeomFetch {
    float sx, sy, dep;
};

DEV GeomFetch geom_fetch(const KViews &kv, int v, const GeomRef &g) {
    const acmmp_camera &sc = kv.cam[v];
    const float *Wp = g.Wp;
    // ProjectonCamera_cu (:506-516)
    float T[3];
    T[0] = sc.R[0] * Wp[0] + sc.R[1] * Wp[1] + sc.R[2] * Wp[2] + sc.t[0];
    T[1] = sc.R[3] * Wp[0] + sc.R[4] * Wp[1] + sc.R[5] * Wp[2] + sc.t[1];
    T[2] = sc.R[6] * Wp[0] + sc.R[7] * Wp[1] + sc.R[8] * Wp[2] + sc.t[2];
    const float sd = sc.K[6] * T[0] + sc.K[7] * T[1] + sc.K[8] * T[2];
    GeomFetch f;
    f.sx = (sc.K[0] * T[0] + sc.K[1] * T[1] + sc.K[2] * T[2]) / sd;
    f.sy = (sc.K[3] * T[0] + sc.K[4] * T[1] + sc.K[5] * T[2]) / sd;
    f.dep = tex_trunc(kv.dep[v], kv.dpitch[v], kv.dw[v], kv.dh[v], f.sx, f.sy);
    return f;
}

DEV float geom_finish(const KViews &kv, int v, const GeomFetch &f, int px, int py) {
    const float max_cost = 3.0f;
    const acmmp_camera &rc = kv.cam[0];
    const acmmp_camera &sc = kv.cam[v];
    const float sx = f.sx, sy = f.sy, src_depth = f.dep;
    if (src_depth == 0.0f) return max_cost;
    float Y[3];
    Y[0] = src_depth * (sx - sc.K[2]) / sc.K[0];
    Y[1] = src_depth * (sy - sc.K[5]) / sc.K[4];
    Y[2] = src_depth;
    float Wq[3];
    Wq[0] = (sc.R[0] * Y[0] + sc.R[3] * Y[1] + sc.R[6] * Y[2]) + cam_offset(kv, v, 0);
    Wq[1] = (sc.R[1] * Y[0] + sc.R[4] * Y[1] + sc.R[7] * Y[2]) + cam_offset(kv, v, 1);
    Wq[2] = (sc.R[2] * Y[0] + sc.R[5] * Y[1] + sc.R[8] * Y[2]) + cam_offset(kv, v, 2);
    float U[3];
    U[0] = rc.R[0] * Wq[0] + rc.R[1] * Wq[1] + rc.R[2] * Wq[2] + rc.t[0];
    U[1] = rc.R[3] * Wq[0] + rc.R[4] * Wq[1] + rc.R[5] * Wq[2] + rc.t[1];
    U[2] = rc.R[6] * Wq[0] + rc.R[7] * Wq[1] + rc.R[8] * Wq[2] + rc.t[2];
    const float rd = rc.K[6] * U[0] + rc.K[7] * U[1] + rc.K[8] * U[2];
    const float bx = (rc.K[0] * U[0] + rc.K[1] * U[1] + rc.K[2] * U[2]) / rd;
    const float by = (rc.K[3] * U[0] + rc.K[4] * U[1] + rc.K[5] * U[2]) / rd;
    const float dc = (float)px - bx;
    const float dr = (float)py - by;
    const float e = dm_sqrt(dc * dc + dr * dr);
    return (e < max_cost) ? e : max_cost;
}

DEV float geom_cost_at(const KViews &kv, int v, const GeomRef &g, int px, int py) {
    return geom_finish(kv, v, geom_fetch(kv, v, g), px, py);
}

DEV float geom_cost(const KViews &kv, int v, float4 h, int px, int py) {
    return geom_cost_at(kv, v, geom_ref(kv, h, px, py), px, py);
}

DEV dm_rng make_rng(const KViews &kv, int center, uint32_t phase) {
    dm_rng g;
    g.k0 = kv.prm.seed_lo;
    g.k1 = kv.prm.seed_hi;
    g.pix = (uint32_t)center;
    g.phase = phase;
    g.stream = kv.prm.rng_stream;
    g.draw = 0;
    g.blk = dm_u32x4{0u, 0u, 0u, 0u};
    return g;
}

DEV int cs_index(const KViews &kv, int x, int y) { return y * kv.Wh + (x >> 1); }

// SpatialGauss / RangeGauss (src/ACMMP.cu:151-161), pow(v,2) pinned to v*v.
DEV float spatial_gauss(float x1, float y1, float x2, float y2, float sigma) {
    const float dis = (x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) - 0.0f;
    return dm_expf((float)(-1.0 * (double)dis / (double)(2 * sigma * sigma)));
}
DEV float range_gauss(float x, float sigma) {
    const float xp = x - 0.0f;
    return dm_expf((float)(-1.0 * (double)(xp * xp) / (double)(2 * sigma * sigma)));
}

// upscale_normal (src/ACMMP.cu:548-607)
DEV float4 upscale_normal(const KViews &kv, const KState &st, int px, int py, float sigmad,
                          float sigmar, int nn, float o_y, float o_x, float refPix, float &cost_out) {
    const int scols = (int)kv.prm.scaled_cols, srows = (int)kv.prm.scaled_rows;
    float c_total = 0.0f, norm = 0.0f;
    float4 n_total = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    for (int j = -nn; j <= nn; ++j) {
        int r_y = (int)(o_y + (float)j);
        r_y = (r_y > 0 ? (r_y < srows ? r_y : srows - 1) : 0);
        const int r_ys = py + j;
        for (int i = -nn; i <= nn; ++i) {
            int r_x = (int)(o_x + (float)i);
            r_x = (r_x > 0 ? (r_x < scols ? r_x : scols - 1) : 0);
            const float4 sn = st.scaled[r_y * scols + r_x];
            const float nb = texel(kv.img[0], kv.ipitch[0], kv.W, kv.H, px + i, r_ys);
            const float tg = spatial_gauss(o_x, o_y, (float)r_x, (float)r_y, sigmad) *
                             range_gauss(dm_fabs(refPix - nb), sigmar);
            norm += tg;
            c_total += sn.w * tg;
            n_total.x = n_total.x + sn.x * tg;
            n_total.y = n_total.y + sn.y * tg;
            n_total.z = n_total.z + sn.z * tg;
        }
    }
    cost_out = c_total / norm;
    n_total.x = n_total.x / norm;
    n_total.y = n_total.y / norm;
    n_total.z = n_total.z / norm;
    normalize3(n_total);
    return n_total;
}

// ------------------------------------------------------ colour-split lanes
// Every PatchMatch kernel maps a 64x4 block onto 64 colour-split columns x 4
// rows of ONE checkerboard colour: lane (tx, ty) of block (bx, by) handles
// pixel x = 2k + s, y, with k = 64 bx + tx, y = 4 by + ty, s = (y + colour) & 1.
struct LaneGeom {
    int k, px, py, s, tb;
};

// XCD-aware block order (cdna_hip_programming.md T1): workgroups are dealt
// round-robin to the 8 XCDs, so consecutive (x, y) blocks would land on 8
// different L2s. Remap the dispatch index so XCD j processes one contiguous
// run of blocks (a band of rows): its L2 then holds the source-image
// footprint of that band only. Bijective for any block count; affects speed
// only (dispatch placement is not guaranteed).
struct BlockXY {
    int bx, by;
};

DEV BlockXY xcd_block(int by0 = 0) {  // by0: block row of the grid's first row (row bands)
    const int gx = gridDim.x;
    const int T = gx * gridDim.y;
    const int L = blockIdx.y * gx + blockIdx.x;
    const int xcd = L & 7, i = L >> 3;
    const int q = T >> 3, r = T & 7;
    const int nl = (xcd < r) ? xcd * (q + 1) + i : r * (q + 1) + (xcd - r) * q + i;
    BlockXY b;
    b.by = nl / gx;
    b.bx = nl - b.by * gx;
    b.by += by0;
    return b;
}

// kWaveRows = R rows per wave: each wave covers 64/R columns x R rows of the
// block instead of one 64-column row, so its gathers for neighbouring patch
// rows overlap in the source image (L1 reuse within a wave).
DEV LaneGeom lane_geom_of(int colour, BlockXY b, int tid) {
    LaneGeom g;
    // waves of C columns x R rows, kBX / C of them side by side per block row
    constexpr int R = kWaveRows, C = 64 / R, WPR = kBX / C;
    static_assert(kBX % C == 0 && kBY % R == 0, "2D wave map");
    const int w = tid >> 6, l = tid & 63;
    // Which pixel of its C x R patch each lane takes. A gather costs one TD
    // cycle per L1 access, and an access serves one 64-B line for one group
    // of 8 lanes: the even or the odd lanes of a 16-lane quarter-wave
    // (profiles/r04_td_addressing.md). Default (lane map 2): a quarter is 4
    // columns x 4 rows, lanes column-major inside, so each 8-lane group is 4
    // adjacent colour-split columns of 2 rows (rows r, r + 2): 36 accesses
    // per k_sweep gather against 46 for row-major lanes (8 columns x 2 rows
    // per quarter, groups of every other column), bench +2 %
    // (profiles/r04_lanemap2_pmc.txt). ACMMP_LANE_MAP=0 restores row-major
    // lanes for A/B builds. Each lane still computes its own pixel, so the
    // map changes no result.
#ifndef ACMMP_LANE_MAP
#define ACMMP_LANE_MAP 2
#endif
    int lc, lr;  // lane -> (column, row) inside the wave's C x R pixels
    if (ACMMP_LANE_MAP == 2 && C == 8 && R == 8) {
        lc = ((l >> 2) & 3) + 4 * ((l >> 4) & 1);
        lr = (l & 3) + 4 * (l >> 5);
    } else {
        lc = l % C;
        lr = l / C;
    }
    const int tx = (w % WPR) * C + lc, ty = (w / WPR) * R + lr;
    g.k = b.bx * kBX + tx;
    g.py = b.by * kBY + ty;
    g.s = (g.py + colour) & 1;
    g.px = 2 * g.k + g.s;
    g.tb = ty * kTileW + tx + g.s;
    return g;
}

DEV LaneGeom lane_geom(int colour, BlockXY b) { return lane_geom_of(colour, b, threadIdx.y * kBX + threadIdx.x); }

// ------------------------------------------------------------------ init
// RandomInitialization (src/ACMMP.cu:609-705). Reads the row-major state,
// writes the colour-split "current" buffers. blockIdx.z = colour.
template <int NS, int TX>
__global__ __launch_bounds__(ACMMP_BLOCK_THREADS) void k_init(const KViews *__restrict__ kvp, KState st) {
    __shared__ float tile[kTileW * kTileH];
    __shared__ WSlot wlds[kSlots * kThreads];
    constexpr bool kLut = (TX & kTxU8) != 0 && ACMMP_WEIGHT_LUT;
    __shared__ float wlut[kLut ? kWlutClasses * 256 : 1];
    const KViews &kv = *kvp;
    const int colour = blockIdx.z;
    const BlockXY blk = xcd_block(st.y0 / kBY);
    load_ref_tile(kv, tile, blk.bx * kBX, blk.by * kBY, colour);
    if (kLut) load_wlut(kv, wlut);
    __syncthreads();
    const LaneGeom g = lane_geom(colour, blk);
    const int px = g.px, py = g.py;
    if (px >= kv.W || py < st.y0 || py >= st.y1) return;
    const acmmp_params &prm = kv.prm;
    const acmmp_camera &c0 = kv.cam[0];
    const int center = py * kv.W + px;
    dm_rng rs = make_rng(kv, center, 0u);
    PixPatch pp;
    pp.wo = threadIdx.y * kBX + threadIdx.x;
    pp.w = wlds + pp.wo;
    pp.rt = tile + g.tb;
    pixel_patch(kv, tile, g.tb, g.s, pp, kLut ? wlut : nullptr);
    float4 plane;
    float cost;
    uint32_t sel = 0;
    if (!prm.geom_consistency && !prm.hierarchy && !prm.seeded) {
        const float depth = dm_rng_uniform(&rs) * (prm.depth_max - prm.depth_min) + prm.depth_min;
        plane = random_normal(c0, px, py, rs, depth);
        plane.w = distance_to_origin(c0, px, py, depth, plane);
        cost = initial_cost<NS, TX>(kv, tile, g.tb, pp, px, py, plane, sel);
    } else if (prm.seeded) {
        plane = st.seed[center];
        cost = initial_cost<NS, TX>(kv, tile, g.tb, pp, px, py, plane, sel);
    } else if (prm.planar_prior) {
        if (st.mask[center] > 0 && st.rm_cost[center] >= 0.1f) {
            const float perturbation = 0.02f;
            const float4 h = st.prior[center];
            float dp = h.w;
            const float dmin = (1 - 3 * perturbation) * dp;
            const float dmax = (1 + 3 * perturbation) * dp;
            dp = dm_rng_uniform(&rs) * (dmax - dmin) + dmin;
            plane = perturbed_normal(c0, px, py, h, rs, kv.pert3_pi);
            plane.w = dp;
        } else {
            plane = st.rm_plane[center];
            plane.w = distance_to_origin(c0, px, py, plane.w, plane);
        }
        cost = initial_cost<NS, TX>(kv, tile, g.tb, pp, px, py, plane, sel);
    } else if (prm.upsample) {
        const float scale = (float)(1.0 * (double)prm.scaled_cols / (double)kv.W);
        const float sigmad = 0.50f, sigmar = 25.5f;
        const float a = (float)kv.W / prm.scaled_cols, b = (float)kv.H / prm.scaled_rows;
        const int Imagescale = (int)(a > b ? a : b);
        const int nn = (Imagescale * Imagescale + 1) / 2;
        const float o_y = (float)py * scale, o_x = (float)px * scale;
        const float refPix = texel(kv.img[0], kv.ipitch[0], kv.W, kv.H, px, py);
        float ucost;
        const float4 n_total = upscale_normal(kv, st, px, py, sigmad, sigmar, nn, o_y, o_x, refPix, ucost);
        const float4 prev = st.rm_plane[center];
        st.pre_cost[center] = initial_cost<NS, TX>(kv, tile, g.tb, pp, px, py, prev, sel);
        plane = to_cam(c0, n_total);
        plane.w = distance_to_origin(c0, px, py, prev.w, plane);
        cost = initial_cost<NS, TX>(kv, tile, g.tb, pp, px, py, plane, sel);
    } else {
        float4 h = prm.hierarchy ? st.scaled[center] : st.rm_plane[center];
        h = to_cam(c0, h);
        h.w = distance_to_origin(c0, px, py, h.w, h);
        plane = h;
        cost = initial_cost<NS, TX>(kv, tile, g.tb, pp, px, py, plane, sel);
    }
    const int ci = py * kv.Wh + g.k;
    st.plane[colour][ci] = plane;
    st.cost[colour][ci] = cost;
    st.sv[colour][ci] = sel;
}

// Packed per-view sample counts (view_weights of the reference, src/ACMMP.cu:995):
// 15 draws, so every count fits 4 bits; 32 views -> two 64-bit words.
struct ViewCounts {
    uint64_t lo = 0, hi = 0;
    __device__ __forceinline__ void add(int j) {
        if (j < 16) lo += (uint64_t)1 << (4 * j);
        else hi += (uint64_t)1 << (4 * (j - 16));
    }
    __device__ __forceinline__ int get(int j) const { return (int)(((j < 16) ? (lo >> (4 * j)) : (hi >> (4 * (j - 16)))) & 15u); }
};

// ------------------------------------------------- compacted refinement
// The candidate-plane slots (cand_lds: 8 float4 per lane, slot d of lane i at
// [d * kThreads + i]) are dead after the t = 0 accept and are reused, each
// lane only within its OWN 8 slots (waves progress independently, so a
// lane's slots may still hold live candidates of another wave's t = 0 step
// — nothing may spill across lanes of different waves):
//   slots 0..4 = the 5 refinement planes; slot 5 = results of planes 0..3;
//   slot 6 = (result of plane 4, mean, var, inv_wsum); slot 7.x = the wave's
//   owner list entry of this lane's rank.
DEV float &cmp_res(float4 *lds, int t, int lane) {
    return reinterpret_cast<float *>(lds)[4 * ((5 + (t >> 2)) * kThreads + lane) + (t & 3)];
}
DEV float &cmp_pd(float4 *lds, int k, int lane) {  // k = 1 mean, 2 var, 3 inv_wsum
    return reinterpret_cast<float *>(lds)[4 * (6 * kThreads + lane) + k];
}
DEV int &cmp_list(float4 *lds, int lane) { return reinterpret_cast<int *>(lds)[4 * (7 * kThreads + lane)]; }

DEV void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The 5 refinement hypotheses of PlaneHypothesisRefinement (src/ACMMP.cu:
// 743-783) cost sum_j w_j * (NCC_j (+ 0.2 geom_j)) over the lane's sampled
// views j. Their planes are fixed before any of them is evaluated, so all 5
// sums are formed here, view-major, and the sequential accept of the caller
// then consumes them in order t = 1..5 (same operations, same order per
// (lane, t): j ascending). Instead of one pass per (t, view with any lane
// sampling it), the wave packs the (owner lane, t) items of view j into
// ceil(5 c_j / active lanes) passes, c_j = lanes that sampled j: a lane
// evaluates another lane's item with that lane's pixel, LDS patch weights,
// tile offset and plane, and returns the cost through LDS. The view stays
// wave-uniform (scalar SRD and cameras). Result: cmp_res(t, lane) = sum_t.
template <int TX, typename RD, typename RN>
DEV void refine_costs_compact(const KViews &kv, const float *tile, WSlot *wlds, float4 *lds, const PixPatch &pp,
                              const ViewCounts &vw, int nsrc, int colour, BlockXY blk, RD ref_depth,
                              RN ref_normal, int px, int py) {
    const acmmp_camera &c0 = kv.cam[0];
    const int tid = pp.wo;
#pragma unroll
    for (int t = 0; t < 5; ++t) {
        float4 h = ref_normal(t);
        h.w = distance_to_origin(c0, px, py, ref_depth(t), h);
        lds[t * kThreads + tid] = h;
    }
    cmp_pd(lds, 1, tid) = pp.mean;
    cmp_pd(lds, 2, tid) = pp.var;
    cmp_pd(lds, 3, tid) = pp.inv_wsum;
    const int lane = tid & 63, wbase = tid & ~63;
    const uint64_t lt = (1ull << lane) - 1ull;
    const uint64_t act = __ballot(1);
    const int nact = __popcll(act), arank = __popcll(act & lt);
    float acc[5] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    wave_sync();
    for (int j = 0; j < nsrc; ++j) {
        const float wj = (float)vw.get(j);
        const uint64_t m = __ballot(wj > 0);
        if (m == 0) continue;
        const int c = __popcll(m);
        if (wj > 0) cmp_list(lds, wbase + __popcll(m & lt)) = lane;
        wave_sync();
        const int n = 5 * c;
        for (int base = 0; base < n; base += nact) {
            const int k = base + arank;
            if (k < n) {
                const int t = k / c;
                const int otid = wbase + cmp_list(lds, wbase + (k - t * c));
                const LaneGeom og = lane_geom_of(colour, blk, otid);
                PixPatch op;
                op.wo = otid;
                op.w = wlds + otid;
                op.rt = tile + og.tb;
                op.mean = cmp_pd(lds, 1, otid);
                op.var = cmp_pd(lds, 2, otid);
                op.inv_wsum = cmp_pd(lds, 3, otid);
                const float4 h = lds[t * kThreads + otid];
                if (ACMMP_GEOM_AHEAD & 4) {
                    // the geometric depth fetch goes out ahead of the NCC's gathers
                    GeomFetch gf = {};
                    if (kv.prm.geom_consistency) gf = geom_fetch(kv, j + 1, geom_ref(kv, h, og.px, og.py));
                    const float cc = bilateral_ncc<TX>(kv, tile, og.tb, op, j + 1, og.px, og.py, h);
                    cmp_res(lds, t, otid) =
                        kv.prm.geom_consistency ? cc + 0.2f * geom_finish(kv, j + 1, gf, og.px, og.py) : cc;
                } else {
                    const float cc = bilateral_ncc<TX>(kv, tile, og.tb, op, j + 1, og.px, og.py, h);
                    cmp_res(lds, t, otid) =
                        kv.prm.geom_consistency ? cc + 0.2f * geom_cost(kv, j + 1, h, og.px, og.py) : cc;
                }
            }
        }
        wave_sync();
        if (wj > 0) {
#pragma unroll
            for (int t = 0; t < 5; ++t) acc[t] += wj * cmp_res(lds, t, tid);
        }
        wave_sync();
    }
#pragma unroll
    for (int t = 0; t < 5; ++t) cmp_res(lds, t, tid) = acc[t];
    wave_sync();
}

// ------------------------------------------------------------- the sweep
// CheckerboardPropagation (src/ACMMP.cu:786-1173) for the pixels of one colour.
// Neighbour state is read from the colour-split "current" buffers (the
// half-sweep snapshot); own state lives in registers and is written to the
// "next" buffer of this colour. (A device function rather than the kernel
// body: measured 4.15 -> 4.05 ms per launch)
template <int NS, int TX>
DEV void sweep_body(const KViews *__restrict__ kvp, KState st, int colour, int iter) {
    __shared__ float tile[kTileW * kTileH];
    __shared__ WSlot wlds[kSlots * kThreads];
    __shared__ float4 cand_lds[8 * kThreads];
    constexpr bool kLut = (TX & kTxU8) != 0 && ACMMP_WEIGHT_LUT;
    __shared__ float wlut[kLut ? kWlutClasses * 256 : 1];
    const KViews &kv = *kvp;
    const BlockXY blk = xcd_block(st.y0 / kBY);
    load_ref_tile(kv, tile, blk.bx * kBX, blk.by * kBY, colour);
    if (kLut) load_wlut(kv, wlut);
    __syncthreads();
    const LaneGeom g = lane_geom(colour, blk);
    const int px = g.px, py = g.py;
    const int width = kv.W, height = kv.H;
    if (py < st.y0 || py >= st.y1 || px >= width) return;  // rows [y0, y1) of the image (a band or all)
    const int oc = colour ^ 1;
    const int Wh = kv.Wh;
    const int my = py * Wh + g.k;
    const float4 *plane_same = st.plane[colour];
    const float4 *plane_opp = st.plane[oc];
    const float *cost_same = st.cost[colour];
    const float *cost_opp = st.cost[oc];
    float4 my_plane = plane_same[my];
    float my_cost = cost_same[my];
    uint32_t my_sv = st.sv[colour][my];
    if (py >= kv.sweep_rows) {  // rows the reference grid never reaches
        st.plane_nx[colour][my] = my_plane;
        st.cost_nx[colour][my] = my_cost;
        return;
    }
    const acmmp_params &prm = kv.prm;
    const acmmp_camera &c0 = kv.cam[0];
    const int nsrc = kv.nsrc;
    const int center = py * width + px;
#define CS(x, y) ((y) * Wh + ((x) >> 1))

    // ---- adaptive checkerboard sampling (:813-991). cidx[d]: colour-split
    // index of direction d's winner; bit d of `same`: it is this colour.
    // Each search reads all its costs first, unconditionally (a step outside
    // the image reads the search's first, always valid, position instead),
    // then runs the reference's comparison chain over them in the same order
    // under the same conditions: one memory latency per search instead of
    // one per step (a load inside a condition is issued and waited alone).
    int cidx[8];
    uint32_t flags = 0, same = 0;
    // Far lines d = 0..3 (up, down, left, right; bit 2d + 1): 11 steps of 2
    // from distance 3 in the opposite colour; right_far's reversed comparison
    // keeps the max (:879). Near "V"s d = 0..3 (bit 2d): the base point is
    // the opposite colour, arm k = 2 i + side is this colour (snapshot reads,
    // pin A2). A step off the image (or a direction that does not apply)
    // reads a valid stand-in: CS(px, py) of the opposite colour, `my` of
    // this one; its value is never compared.
    auto far_valid = [&](int d, int i) -> bool {
        return d == 0 ? py > 2 + 2 * i : d == 1 ? py < height - 3 - 2 * i : d == 2 ? px > 2 + 2 * i : px < width - 3 - 2 * i;
    };
    auto far_at = [&](int d, int i) -> int {
        return d == 0 ? CS(px, py - 3 - 2 * i)
             : d == 1 ? CS(px, py + 3 + 2 * i)
             : d == 2 ? CS(px - 3 - 2 * i, py)
                      : CS(px + 3 + 2 * i, py);
    };
    auto near_valid = [&](int d, int k) -> bool {
        const int i = k >> 1, sd = k & 1;
        return d == 0 ? py > 1 + i && (sd ? px < width - 1 - i : px > i)
             : d == 1 ? py < height - 2 - i && (sd ? px < width - 1 - i : px > i)
             : d == 2 ? px > 1 + i && (sd ? py < height - 1 - i : py > i)
                      : px < width - 2 - i && (sd ? py < height - 1 - i : py > i);
    };
    auto near_at = [&](int d, int k) -> int {
        const int i = k >> 1, sd = k & 1;
        return d == 0 ? CS(sd ? px + i : px - i, py - 2 - i)
             : d == 1 ? CS(sd ? px + i : px - i, py + 2 + i)
             : d == 2 ? CS(px - 2 - i, sd ? py + i : py - i)
                      : CS(px + 2 + i, sd ? py + i : py - i);
    };
    const bool near_on[4] = {py > 0, py < height - 1, px > 0, px < width - 1};
    const int near_base[4] = {CS(px, py - 1), CS(px, py + 1), CS(px - 1, py), CS(px + 1, py)};
    // every cost of the 8 searches is loaded before any comparison: one
    // memory latency for all of them (a load inside a condition is issued
    // and waited alone)
    float cf[4][11], cn[4][6], cb[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
#pragma unroll
        for (int i = 0; i < 11; ++i) cf[d][i] = cost_opp[far_valid(d, i) ? far_at(d, i) : CS(px, py)];
        cb[d] = cost_opp[near_on[d] ? near_base[d] : CS(px, py)];
#pragma unroll
        for (int k = 0; k < 6; ++k) cn[d][k] = cost_same[near_valid(d, k) ? near_at(d, k) : my];
    }
    // the reference's comparison chains, same order, same conditions
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        if (far_valid(d, 0)) {
            flags |= 1u << (2 * d + 1);
            int b = 0;
            float m = cf[d][0];
#pragma unroll
            for (int i = 1; i < 11; ++i)
                if (far_valid(d, i) && (d == 3 ? (m < cf[d][i]) : (cf[d][i] < m))) { m = cf[d][i]; b = i; }
            cidx[2 * d + 1] = far_at(d, b);
        }
    }
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        if (near_on[d]) {
            flags |= 1u << (2 * d);
            int bi = near_base[d];
            bool bs = false;
            float m = cb[d];
#pragma unroll
            for (int k = 0; k < 6; ++k)
                if (near_valid(d, k) && cn[d][k] < m) { m = cn[d][k]; bi = near_at(d, k); bs = true; }
            cidx[2 * d] = bi;
            same |= (uint32_t)bs << (2 * d);
        }
    }
#undef CS
    // the 8 winners' planes, fetched once into this lane's LDS slots (the
    // NCC prologues then read them at LDS latency, not L2's)
    float4 *cand_slot = cand_lds + threadIdx.y * kBX + threadIdx.x;
    // (all 8 loads issued together, and stored unconditionally so none is
    // sunk into a conditional block and waited alone: an unflagged
    // direction's slot gets the own plane, and every reader of a slot
    // checks its flag first)
    float4 cpl[8];
#pragma unroll
    for (int d = 0; d < 8; ++d) {
        const bool f = (flags >> d) & 1u;
        cpl[d] = ((f && !((same >> d) & 1u)) ? plane_opp : plane_same)[f ? cidx[d] : my];
    }
#pragma unroll
    for (int d = 0; d < 8; ++d) cand_slot[d * kThreads] = cpl[d];
    auto cand = [&](int d) -> float4 { return cand_slot[d * kThreads]; };

    PixPatch pp;
    pp.wo = threadIdx.y * kBX + threadIdx.x;
    pp.w = wlds + pp.wo;
    pp.rt = tile + g.tb;
    pixel_patch(kv, tile, g.tb, g.s, pp, kLut ? wlut : nullptr);

    // cost_array[8][32] = {2.0f}: only [0][0] is 2, the rest 0 (:805)
    float cost_array[8][NS];
    // view-selection inputs (:994-1032), folded into the view-major candidate
    // loop so each view's 8 costs are consumed from registers
    float probs[NS];
    uint32_t nb[4];
    {
        const uint32_t *sv_opp = st.sv[oc];
        // (x, y+-1) are colour-split column (x >> 1); (x+-1, y) are k - 1 + s, k + s
        nb[0] = (py > 0) ? sv_opp[(py - 1) * Wh + (px >> 1)] : 0u;
        nb[1] = (py < height - 1) ? sv_opp[(py + 1) * Wh + (px >> 1)] : 0u;
        nb[2] = (px > 0) ? sv_opp[py * Wh + ((px - 1) >> 1)] : 0u;
        nb[3] = (px < width - 1) ? sv_opp[py * Wh + ((px + 1) >> 1)] : 0u;
    }
    const float cost_threshold = (float)(0.8 * (double)dm_expf((float)(iter * iter) / (-90.0f)));
    // view-major: the 8 candidates of one source view gather from nearly the
    // same footprint, back to back (results are independent)
    for (int v = 0; v < nsrc; ++v) {
        // one NCC call site: the candidate loop stays rolled (d is wave-uniform,
        // the candidate's index is picked by selects), and the sampling
        // statistics of :1013-1024 are accumulated in the same j = 0..7 order
        float count = 0;
        int count_false = 0;
        float tmpw = 0;
#pragma unroll 1
        for (int d = 0; d < 8; ++d) {
            float c;
            if ((flags >> d) & 1u) c = bilateral_ncc<TX>(kv, tile, g.tb, pp, v + 1, px, py, cand(d));
            else c = (d == 0 && v == 0) ? 2.0f : 0.0f;
            cost_array[d][v] = c;
            if (c < cost_threshold) {
                // exp(c * c / -0.18f) (:1017): c is 0 or in [2^-24, 2] (an NCC is 1 - q rounded,
                // clamped to [0, 2]), so c * c is 0 or in [2^-48, 4] and the quotient in
                // [-22.3, 0], where the Markstein quotient and dm_expf_nonpos are the IEEE
                // quotient and dm_expf bit for bit (exhaustive: tests/test_detmath.py)
#if ACMMP_VS_SHORTCUTS
                tmpw += dm_expf_nonpos(dm_div_neg018(c * c));
#else
                tmpw += dm_expf(c * c / (-0.18f));
#endif
                count++;
            }
            if (c > 1.2f) count_false++;
        }
        float vsp = 0.0f;
        for (int n = 0; n < 4; ++n)
            if ((flags >> (2 * n)) & 1u) vsp += ((nb[n] >> v) & 1u) ? 0.9f : 0.1f;
        float pr = 0.0f;
        if (count > 2 && count_false < 3) pr = tmpw / count;
        else if (count_false < 3) pr = dm_expf(cost_threshold * cost_threshold / (-0.32f));
        probs[v] = pr * vsp;
    }

    // ---- multi-hypothesis joint view selection (:994-1056)
    // CDF in registers (static indices over NS, predicated on i < nsrc): the
    // 15 draws then need no dependent scratch loads. The CDF is
    // nondecreasing (non-negative terms; once NaN it stays NaN), so the
    // reference's "first i with cdf[i] > r" (:1036-1041) is the count of
    // entries <= r, taken only if that entry is > r (a NaN or all-<= r CDF
    // selects nothing, as in the reference).
    float cdf[NS];
    {  // TransformPDFToCDF (:107-121), same operations and order
        float sum = 0.0f;
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            cdf[i] = i < nsrc ? probs[i] : 0.0f;
            if (i < nsrc) sum += cdf[i];
        }
        const float inv = 1.0f / sum;
        float cum = 0.0f;
#pragma unroll
        for (int i = 0; i < NS; ++i)
            if (i < nsrc) {
                cum += cdf[i] * inv;
                cdf[i] = cum;
            }
    }
    dm_rng rs = make_rng(kv, center, 1u + (uint32_t)iter);
    ViewCounts vw;
#pragma unroll 1
    for (int sample = 0; sample < 15; ++sample) {
        const float rand_prob = dm_rng_uniform(&rs) - FLT_EPSILON;
        int idx = 0;
        float at = cdf[0];
#pragma unroll
        for (int i = 0; i < NS; ++i) idx += (i < nsrc && cdf[i] <= rand_prob) ? 1 : 0;
#pragma unroll
        for (int i = 1; i < NS; ++i) at = idx == i ? cdf[i] : at;
        if (idx < nsrc && at > rand_prob) vw.add(idx);
    }
    uint32_t temp_sv = 0;
    float weight_norm = 0;
    for (int i = 0; i < nsrc; ++i) {
        const int c = vw.get(i);
        if (c > 0) { temp_sv |= (1u << i); weight_norm += (float)c; }
    }
    float final_costs[8];
    if (!prm.geom_consistency) {
        // photometric: the NS cost loads of a candidate issued together
        // (static offsets), unsampled views add +0 (costs are finite and
        // >= 0, fc >= +0: the same sum as skipping them)
        for (int i = 0; i < 8; ++i) {
            float fc = 0.0f;
#pragma unroll
            for (int j = 0; j < NS; ++j)
                if (j < nsrc) {
                    const float wj = (float)vw.get(j);
                    fc += wj > 0 ? wj * cost_array[i][j] : 0.0f;
                }
            final_costs[i] = fc / weight_norm;
        }
    } else if ((ACMMP_GEOM_AHEAD & 1) && NS <= 9) {
        // (the 9-view bucket only: with 16-32 views the batch of fetches
        // costs more than the latency it hides, geometric launch +0.2 / +0.6
        // / +1.1 % at nsrc 16 / 20 / 21, profiles/r05_geom_ahead_ns.jsonl;
        // those buckets take the per-view loop below)
        // views sampled by some lane of the wave (bit j; nsrc <= 32, so
        // padding slots j >= nsrc never appear)
        uint32_t wave_views = 0;
        for (int j = 0; j < nsrc; ++j) wave_views |= (__ballot(vw.get(j) > 0) != 0 ? 1u : 0u) << j;
        // geometric: a flagged candidate's source-depth fetches for all views
        // are issued before any is consumed (one memory latency per
        // candidate, not one per view); the sum is the same ops in the same
        // order, with unsampled views adding +0 as above. Only the nsrc real
        // views are fetched and read (j < nsrc is wave-uniform, so the loads
        // still go out together; padding slots j >= nsrc are never written)
        for (int i = 0; i < 8; ++i) {
            float fc = 0.0f;
            const bool fl = (flags >> i) & 1u;
            // the candidate's cost row read whole and unconditionally (one
            // batch of scratch loads, not one load and wait per sampled view)
            float ci[NS];
#pragma unroll
            for (int j = 0; j < NS; ++j) ci[j] = j < nsrc ? cost_array[i][j] : 0.0f;
            if (fl) {
                // views no lane of the wave sampled add +0 for every lane:
                // their geometric cost is not finished (wave-uniform skip;
                // the fetches stay unconditional, one batch per candidate)
                const GeomRef gi = geom_ref(kv, cand(i), px, py);
                GeomFetch gf[NS];
#pragma unroll
                for (int j = 0; j < NS; ++j) gf[j] = j < nsrc ? geom_fetch(kv, j + 1, gi) : GeomFetch{};
#pragma unroll
                for (int j = 0; j < NS; ++j)
                    if ((wave_views >> j) & 1u) {
                        const float wj = (float)vw.get(j);
                        const float gc = geom_finish(kv, j + 1, gf[j], px, py);
                        fc += wj > 0 ? wj * (ci[j] + 0.2f * gc) : 0.0f;
                    }
            } else {
#pragma unroll
                for (int j = 0; j < NS; ++j)
                    if (j < nsrc) {
                        const float wj = (float)vw.get(j);
                        fc += wj > 0 ? wj * (ci[j] + 0.1f * 3.0f) : 0.0f;
                    }
            }
            final_costs[i] = fc / weight_norm;
        }
    } else
    for (int i = 0; i < 8; ++i) {
        float fc = 0.0f;
        const bool fl = (flags >> i) & 1u;
        GeomRef gi = {};
        if (prm.geom_consistency && fl) gi = geom_ref(kv, cand(i), px, py);  // once per candidate
        for (int j = 0; j < nsrc; ++j) {
            const float wj = (float)vw.get(j);
            if (wj > 0) {
                if (prm.geom_consistency) {
                    const float cij = cost_array[i][j];
                    if (fl) fc += wj * (cij + 0.2f * geom_cost_at(kv, j + 1, gi, px, py));
                    else fc += wj * (cij + 0.1f * 3.0f);
                } else {
                    fc += wj * cost_array[i][j];
                }
            }
        }
        final_costs[i] = fc / weight_norm;
    }
    int min_cost_idx = 0;
    {
        float m = final_costs[0];
        for (int i = 1; i < 8; ++i)
            if (final_costs[i] <= m) { m = final_costs[i]; min_cost_idx = i; }
    }

    // ---- current hypothesis (:1080-1093) + refinement (:707-784): one NCC
    // site. t = 0 evaluates the current plane; t = 1..5 the refinement planes.
    const bool has_prior = prm.planar_prior && st.mask[center] > 0;
    float4 prior_plane = make_float4(0.f, 0.f, 0.f, 0.f);
    if (prm.planar_prior) prior_plane = st.prior[center];
    float cost_now = 0.0f, depth_now = 0.0f, restricted_cost = 0.0f, depth_prior = 0.0f;
    float4 plane_now = my_plane;
    // the 5 refinement hypotheses (:735-740) take their depths and normals
    // from 3 values each: (depth, normal) of t = 1..5 is
    // (rnd, now), (gen, rnd), (rnd, rnd), (gen, pert), (pert, now), with
    // gen / now the depth / plane at generation time (held apart: the
    // accepts below move depth_now and plane_now). Picked by wave-uniform
    // selects (a dynamically indexed array would live in scratch).
    float rd_rnd = 0.0f, rd_gen = 0.0f, rd_pert = 0.0f;
    float4 rn_now = my_plane, rn_rnd = my_plane, rn_pert = my_plane;
    auto ref_depth = [&](int k) -> float { return k == 4 ? rd_pert : ((k & 1) ? rd_gen : rd_rnd); };
    auto ref_normal = [&](int k) -> float4 {
        return (k == 0 || k == 4) ? rn_now : (k == 3 ? rn_pert : rn_rnd);
    };
    const float gamma = 0.5f;
    const float depth_sigma = (prm.depth_max - prm.depth_min) / 64.0f;
    const float two_dss = 2 * depth_sigma * depth_sigma;
    const float two_ass = 2 * kv.angle_sigma * kv.angle_sigma;
    const float beta = 0.18f;

    for (int t = 0; t < 6; ++t) {
        // all 5 refinement costs at once (their planes go to LDS slots 0..4)
        if (t == 1)
            refine_costs_compact<TX>(kv, tile, wlds, cand_lds, pp, vw, nsrc, colour, blk, ref_depth, ref_normal,
                                     px, py);
        float4 h;
        if (t == 0) h = my_plane;
        else h = cand_lds[(t - 1) * kThreads + pp.wo];  // stored by refine_costs_compact
        // views with a zero sampled weight contribute +0 in the reference
        // (weight 0 * finite cost), so their NCC is skipped: bit-identical
        float tc = 0.0f;
        if (t >= 1) {
            tc = cmp_res(cand_lds, t - 1, pp.wo);
        } else {
        GeomRef gnow = {};
        if (prm.geom_consistency) gnow = geom_ref(kv, h, px, py);  // once for the current plane
        for (int j = 0; j < nsrc; ++j) {
            const float wj = (float)vw.get(j);
            if (wj > 0) {
                // the geometric depth fetch goes out ahead of the NCC's gathers
                GeomFetch gf = {};
                if ((ACMMP_GEOM_AHEAD & 2) && prm.geom_consistency) gf = geom_fetch(kv, j + 1, gnow);
                const float c = bilateral_ncc<TX>(kv, tile, g.tb, pp, j + 1, px, py, h);
                if (ACMMP_GEOM_AHEAD & 2) {
                    if (prm.geom_consistency) tc += wj * (c + 0.2f * geom_finish(kv, j + 1, gf, px, py));
                    else tc += wj * c;
                } else if (prm.geom_consistency) tc += wj * (c + 0.2f * geom_cost_at(kv, j + 1, gnow, px, py));
                else tc += wj * c;
            }
        }
        }
        tc /= weight_norm;
        if (t == 0) {
            cost_now = tc;
            my_cost = cost_now;  // costs[center] = cost_now (:1092)
            depth_now = plane_depth(c0, my_plane, px, py);
            if (prm.planar_prior) {
                depth_prior = plane_depth(c0, prior_plane, px, py);
                if (st.mask[center] > 0) {
                    float rfc[8];
                    for (int i = 0; i < 8; i++) {
                        rfc[i] = 0.0f;
                        if ((flags >> i) & 1u) {
                            const float4 ci = cand(i);
                            const float dn = plane_depth(c0, ci, px, py);
                            const float dd = dn - depth_prior;
                            const float ad = dm_acosf(dot3(prior_plane, ci));
                            const float prior = gamma + dm_expf(-dd * dd / two_dss) * dm_expf(-ad * ad / two_ass);
                            rfc[i] = dm_expf(-final_costs[i] * final_costs[i] / beta) * prior;
                        }
                    }
                    int max_idx = 0;
                    {
                        float m = rfc[0];
                        for (int i = 1; i < 8; ++i)
                            if (rfc[i] >= m) { m = rfc[i]; max_idx = i; }
                    }
                    const float dn = plane_depth(c0, my_plane, px, py);
                    const float dd = dn - depth_prior;
                    const float ad = dm_acosf(dot3(prior_plane, my_plane));
                    const float prior = gamma + dm_expf(-dd * dd / two_dss) * dm_expf(-ad * ad / two_ass);
                    const float rcn = dm_expf(-cost_now * cost_now / beta) * prior;
                    if ((flags >> max_idx) & 1u) {
                        const float4 cm = cand(max_idx);
                        const float db = plane_depth(c0, cm, px, py);
                        if (db >= prm.depth_min && db <= prm.depth_max && rfc[max_idx] > rcn) {
                            // the reference assigns a shadowing local here (:1119/:1130):
                            // the outer depth_now is NOT updated
                            my_plane = cm;
                            my_cost = final_costs[max_idx];
                            restricted_cost = rfc[max_idx];
                            my_sv = temp_sv;
                        }
                    }
                } else if ((flags >> min_cost_idx) & 1u) {
                    const float4 cm = cand(min_cost_idx);
                    const float db = plane_depth(c0, cm, px, py);
                    if (db >= prm.depth_min && db <= prm.depth_max && final_costs[min_cost_idx] < cost_now) {
                        depth_now = db;
                        my_plane = cm;
                        my_cost = final_costs[min_cost_idx];
                    }
                }
            }
            plane_now = my_plane;  // pin A3
            if (!prm.planar_prior && ((flags >> min_cost_idx) & 1u)) {
                const float4 cm = cand(min_cost_idx);
                const float db = plane_depth(c0, cm, px, py);
                if (db >= prm.depth_min && db <= prm.depth_max && final_costs[min_cost_idx] < cost_now) {
                    depth_now = db;
                    plane_now = cm;
                    cost_now = final_costs[min_cost_idx];
                    my_sv = temp_sv;
                }
            }
            // PlaneHypothesisRefinement: candidate generation (:718-741)
            float depth_rand;
            float4 plane_rand;
            if (has_prior) {
                const float dpri = plane_depth(c0, prior_plane, px, py);
                depth_prior = dpri;
                depth_rand = dm_rng_uniform(&rs) * 6 * depth_sigma + (dpri - 3 * depth_sigma);
                plane_rand = perturbed_normal(c0, px, py, prior_plane, rs, kv.angle_sigma);
            } else {
                depth_rand = dm_rng_uniform(&rs) * (prm.depth_max - prm.depth_min) + prm.depth_min;
                plane_rand = random_normal(c0, px, py, rs, depth_now);
            }
            const float perturbation = 0.02f;
            float depth_perturbed = depth_now;
            const float dmin_p = (1 - perturbation) * depth_perturbed;
            const float dmax_p = (1 + perturbation) * depth_perturbed;
            do {
                depth_perturbed = dm_rng_uniform(&rs) * (dmax_p - dmin_p) + dmin_p;
            } while (depth_perturbed < prm.depth_min && depth_perturbed > prm.depth_max);
            const float4 plane_perturbed = perturbed_normal(c0, px, py, plane_now, rs, kv.pert_pi);
            rd_rnd = depth_rand;
            rd_gen = depth_now;
            rd_pert = depth_perturbed;
            rn_now = plane_now;
            rn_rnd = plane_rand;
            rn_pert = plane_perturbed;
        } else {
            const float depth_before = plane_depth(c0, h, px, py);
            if (has_prior) {
                const float dd = ref_depth(t - 1) - depth_prior;
                const float ad = dm_acosf(dot3(prior_plane, h));
                const float prior = gamma + dm_expf(-dd * dd / two_dss) * dm_expf(-ad * ad / two_ass);
                const float rtc = dm_expf(-tc * tc / beta) * prior;
                if (depth_before >= prm.depth_min && depth_before <= prm.depth_max && rtc > restricted_cost) {
                    depth_now = depth_before;
                    plane_now = h;
                    cost_now = tc;
                    restricted_cost = rtc;
                }
            } else {
                if (depth_before >= prm.depth_min && depth_before <= prm.depth_max && tc < cost_now) {
                    depth_now = depth_before;
                    plane_now = h;
                    cost_now = tc;
                }
            }
        }
    }
    // hierarchy gate (:1163-1172)
    if (prm.hierarchy) {
        if (cost_now < st.pre_cost[center] - 0.1f) {
            my_cost = cost_now;
            my_plane = plane_now;
        }
    } else {
        my_cost = cost_now;
        my_plane = plane_now;
    }
    st.plane_nx[colour][my] = my_plane;
    st.cost_nx[colour][my] = my_cost;
    st.sv[colour][my] = my_sv;
}

template <int NS, int TX>
__global__ __launch_bounds__(ACMMP_BLOCK_THREADS, kSweepWaves) void k_sweep_f(const KViews *__restrict__ kvp, KState st, int colour,
                                                              int iter) {
    sweep_body<NS, TX>(kvp, st, colour, iter);
}

// T1 kernel: costs of a given plane per pixel against every source view
// (same NCC code path as the sweep; blockIdx.z = colour).
template <int NS, int TX>
__global__ __launch_bounds__(ACMMP_BLOCK_THREADS) void k_eval_costs(const KViews *__restrict__ kvp, const float4 *planes,
                                                    float *out, float *out_init, uint32_t *out_views) {
    __shared__ float tile[kTileW * kTileH];
    __shared__ WSlot wlds[kSlots * kThreads];
    const KViews &kv = *kvp;
    const int colour = blockIdx.z;
    const BlockXY blk = xcd_block();
    load_ref_tile(kv, tile, blk.bx * kBX, blk.by * kBY, colour);
    __syncthreads();
    const LaneGeom g = lane_geom(colour, blk);
    if (g.px >= kv.W || g.py >= kv.H) return;
    const int c = g.py * kv.W + g.px;
    PixPatch pp;
    pp.wo = threadIdx.y * kBX + threadIdx.x;
    pp.w = wlds + pp.wo;
    pp.rt = tile + g.tb;
    pixel_patch(kv, tile, g.tb, g.s, pp);
    const float4 h = planes[c];
    if (out)
        for (int v = 0; v < kv.nsrc; ++v)
            out[(size_t)c * kv.nsrc + v] = bilateral_ncc<TX>(kv, tile, g.tb, pp, v + 1, g.px, g.py, h);
    if (out_init) {
        uint32_t sel = 0;
        out_init[c] = initial_cost<NS, TX>(kv, tile, g.tb, pp, g.px, g.py, h, sel);
        if (out_views) out_views[c] = sel;
    }
}

#ifndef ACMMP_TX_UNIT
// ---- non-templated kernels and every launcher: the main translation unit
// only (the texel-form units below hold the templated instantiations)
__global__ __launch_bounds__(256) void k_finalize(const KViews *__restrict__ kvp, KState st) {
    const KViews &kv = *kvp;
    const int px = blockIdx.x * 64 + threadIdx.x;
    const int py = (st.y0 / 4 + (int)blockIdx.y) * 4 + threadIdx.y;
    if (px >= kv.W || py < st.y0 || py >= st.y1) return;
    const int c = (px + py) & 1;
    const int ci = cs_index(kv, px, py);
    float4 h = st.plane[c][ci];
    h.w = plane_depth(kv.cam[0], h, px, py);
    h = to_world(kv.cam[0], h);
    const int center = py * kv.W + px;
    st.rm_plane[center] = h;
    st.rm_depth[center] = h.w;
    st.rm_cost[center] = st.cost[c][ci];
    st.rm_sv[center] = st.sv[c][ci];
}

// CheckerboardFilter (src/ACMMP.cu:1214-1328) on one colour, in place on the
// row-major planes: every read is of the opposite colour.
__global__ __launch_bounds__(256) void k_filter(const KViews *__restrict__ kvp, KState st, int colour) {
    const KViews &kv = *kvp;
    const int k = blockIdx.x * 64 + threadIdx.x;
    const int py = (st.y0 / 4 + (int)blockIdx.y) * 4 + threadIdx.y;
    const int width = kv.W, height = kv.H;
    if (py < st.y0 || py >= st.y1 || py >= kv.sweep_rows) return;
    const int px = 2 * k + ((py + colour) & 1);
    if (px >= width) return;
    // neighbours' depths from the depth plane (4 B each; the same values as
    // rm_plane[.].w, which the filter updates alongside)
    const float *ph = st.rm_depth;
    const int center = py * width + px;
    if (st.rm_cost[center] < 0.001f) return;
    float f[21];
    int n = 0;
    f[n++] = ph[center];
    const int left = center - 1, leftleft = center - 3;
    const int up = center - width, upup = center - 3 * width;
    const int down = center + width, downdown = center + 3 * width;
    const int right = center + 1, rightright = center + 3;
    if (py > 0) f[n++] = ph[up];
    if (py > 2) f[n++] = ph[upup];
    if (py > 4) f[n++] = ph[upup - width * 2];
    if (py < height - 1) f[n++] = ph[down];
    if (py < height - 3) f[n++] = ph[downdown];
    if (py < height - 5) f[n++] = ph[downdown + width * 2];
    if (px > 0) f[n++] = ph[left];
    if (px > 2) f[n++] = ph[leftleft];
    if (px > 4) f[n++] = ph[leftleft - 2];
    if (px < width - 1) f[n++] = ph[right];
    if (px < width - 3) f[n++] = ph[rightright];
    if (px < width - 5) f[n++] = ph[rightright + 2];
    if (py > 0 && px < width - 2) f[n++] = ph[up + 2];
    if (py < height - 1 && px < width - 2) f[n++] = ph[down + 2];
    if (py > 0 && px > 1) f[n++] = ph[up - 2];
    if (py < height - 1 && px > 1) f[n++] = ph[down - 2];
    if (px > 0 && py > 2) f[n++] = ph[left - width * 2];
    if (px < width - 1 && py > 2) f[n++] = ph[right - width * 2];
    if (px > 0 && py < height - 2) f[n++] = ph[left + width * 2];
    if (px < width - 1 && py < height - 2) f[n++] = ph[right + width * 2];
    for (int i = 1; i < n; i++) {  // sort_small
        const float tmp = f[i];
        int j;
        for (j = i; j >= 1 && tmp < f[j - 1]; j--) f[j] = f[j - 1];
        f[j] = tmp;
    }
    const int m = n / 2;
    const float med = (n % 2 == 0) ? (f[m - 1] + f[m]) / 2 : f[m];
    st.rm_depth[center] = med;
    st.rm_plane[center].w = med;
}

__global__ __launch_bounds__(256) void k_eval_geom(const KViews *__restrict__ kvp, const float4 *planes,
                                                   float *out) {
    const KViews &kv = *kvp;
    const int px = blockIdx.x * 64 + threadIdx.x;
    const int py = blockIdx.y * 4 + threadIdx.y;
    if (px >= kv.W || py >= kv.H) return;
    const int c = py * kv.W + px;
    for (int v = 0; v < kv.nsrc; ++v) out[(size_t)c * kv.nsrc + v] = geom_cost(kv, v + 1, planes[c], px, py);
}

// Padded copy of a source image (see KViews::pad).
// Row-paired clamp-to-edge copy of a source view for the NCC gathers:
// element (r, c), r < H + 2, c < W + 3, is the float pair
// (texel(clamp(c-1), clamp(r-1)), texel(clamp(c-1), clamp(r))); dpitch in pairs.
__global__ __launch_bounds__(256) void k_pad_image(const float *__restrict__ src, int spitch, int W, int H,
                                                   float *__restrict__ dst, int dpitch) {
    const int c = blockIdx.x * 64 + threadIdx.x;
    const int r = blockIdx.y * 4 + threadIdx.y;
    if (c >= W + 3 || r >= H + 2) return;
    const int x = min(max(c - 1, 0), W - 1);
    const int y0 = min(max(r - 1, 0), H - 1), y1 = min(r, H - 1);
    reinterpret_cast<float2 *>(dst)[(size_t)r * dpitch + c] = make_float2(src[y0 * spitch + x], src[y1 * spitch + x]);
}

hipError_t launch_pad_image(const float *src, int spitch, int W, int H, float *dst, int dpitch, hipStream_t s) {
    dim3 block(64, 4), grid((W + 3 + 63) / 64, (H + 2 + 3) / 4);
    k_pad_image<<<grid, block, 0, s>>>(src, spitch, W, H, dst, dpitch);
    return hipGetLastError();
}

// u8 quad layout: element (r, c), r < H + 2, c < W + 2, packs the texels
// (clamp(c-1), clamp(r-1)), (clamp(c-1), clamp(r)), (clamp(c), clamp(r-1)),
// (clamp(c), clamp(r)) as bytes 0..3, so the record at (y0 + 1, x0 + 1) is
// the whole bilinear footprint of (x0, y0) (same record index as the fp32
// row-paired copy). Texel (clamp(c-1), clamp(r-1)) ranges over every texel,
// so checking it checks the view: -0.0f, NaN and non-integers are not u8.
__global__ __launch_bounds__(256) void k_pad_quad(const float *__restrict__ src, int spitch, int W, int H,
                                                  uint32_t *__restrict__ dst, int dpitch, uint32_t *not_u8) {
    const int c = blockIdx.x * 64 + threadIdx.x;
    const int r = blockIdx.y * 4 + threadIdx.y;
    if (c >= W + 2 || r >= H + 2) return;
    const int xa = min(max(c - 1, 0), W - 1), xb = min(c, W - 1);
    const int ya = min(max(r - 1, 0), H - 1), yb = min(r, H - 1);
    const float t00 = src[ya * spitch + xa], t01 = src[yb * spitch + xa];
    const float t10 = src[ya * spitch + xb], t11 = src[yb * spitch + xb];
    const bool ok = t00 >= 0.0f && t00 <= 255.0f && t00 == dm_floor(t00) && (__float_as_uint(t00) >> 31) == 0u;
    if (!ok) *not_u8 = 1u;
    auto b = [](float t) -> uint32_t { return (t >= 0.0f && t <= 255.0f) ? (uint32_t)t : 0u; };
    dst[(size_t)r * dpitch + c] = b(t00) | (b(t01) << 8) | (b(t10) << 16) | (b(t11) << 24);
}

// f16 difference-quad layout: element (r, c), r < H + 2, c < W + 2, holds
// the halves (t00, t01, t10 - t00, t11 - t01) of the same clamped texels as
// the u8 quad, the differences formed in fp32 exactly as the lerp forms them
// (lerp_sample). Sets *not_h16 if any stored value is not exactly
// representable (non-finite, beyond +-65504, or more than 11 significant
// bits); the copy is then unusable and the fp32 form is built.
__global__ __launch_bounds__(256) void k_pad_h16(const float *__restrict__ src, int spitch, int W, int H,
                                                 uint2 *__restrict__ dst, int dpitch, uint32_t *not_h16) {
    const int c = blockIdx.x * 64 + threadIdx.x;
    const int r = blockIdx.y * 4 + threadIdx.y;
    if (c >= W + 2 || r >= H + 2) return;
    const int xa = min(max(c - 1, 0), W - 1), xb = min(c, W - 1);
    const int ya = min(max(r - 1, 0), H - 1), yb = min(r, H - 1);
    const float t00 = src[ya * spitch + xa], t01 = src[yb * spitch + xa];
    const float t10 = src[ya * spitch + xb], t11 = src[yb * spitch + xb];
    const float v[4] = {t00, t01, t10 - t00, t11 - t01};
    _Float16 h[4];
    bool ok = true;
    for (int i = 0; i < 4; ++i) {
        h[i] = (_Float16)v[i];
        const float back = (float)h[i];
        ok = ok && __float_as_uint(back) == __float_as_uint(v[i]) && dm_fabs(v[i]) <= 65504.0f;
    }
    if (!ok) *not_h16 = 1u;
    dst[(size_t)r * dpitch + c] = make_uint2(__builtin_bit_cast(uint32_t, h2v{h[0], h[1]}),
                                             __builtin_bit_cast(uint32_t, h2v{h[2], h[3]}));
}

hipError_t launch_pad_h16(const float *src, int spitch, int W, int H, void *dst, int dpitch, uint32_t *not_h16,
                          hipStream_t s) {
    dim3 block(64, 4), grid((W + 2 + 63) / 64, (H + 2 + 3) / 4);
    k_pad_h16<<<grid, block, 0, s>>>(src, spitch, W, H, reinterpret_cast<uint2 *>(dst), dpitch, not_h16);
    return hipGetLastError();
}

hipError_t launch_pad_quad(const float *src, int spitch, int W, int H, uint32_t *dst, int dpitch, uint32_t *not_u8,
                           hipStream_t s) {
    dim3 block(64, 4), grid((W + 2 + 63) / 64, (H + 2 + 3) / 4);
    k_pad_quad<<<grid, block, 0, s>>>(src, spitch, W, H, dst, dpitch, not_u8);
    return hipGetLastError();
}

// Exhaustive check of recip_newton against IEEE 1/z over every float32 bit
// pattern inside recip_fast_window (grid-stride over all 2^32 patterns).
__global__ __launch_bounds__(256) void k_selftest_rcp(unsigned long long *mismatch,
                                                      unsigned long long *checked) {
    unsigned long long bad = 0, n = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < (1ull << 32); u += stride) {
        const float z = __uint_as_float((uint32_t)u);
        if (!recip_fast_window(z)) continue;
        ++n;
        const float a = recip_newton(z);
        volatile float one = 1.0f;
        const float b = one / z;
        if (__float_as_uint(a) != __float_as_uint(b)) ++bad;
    }
    atomicAdd(mismatch, bad);
    atomicAdd(checked, n);
}

hipError_t launch_selftest_rcp(unsigned long long *mismatch, unsigned long long *checked, hipStream_t s) {
    k_selftest_rcp<<<4096, 256, 0, s>>>(mismatch, checked);
    return hipGetLastError();
}

// JBU_cu (src/ACMMP.cu:1458-1516): joint-bilateral upsampling of a low-res
// depth map guided by the high-res reference image; one thread per high-res
// pixel. Texture reads at integer + 0.5 are exact texels (pin A4).
__global__ __launch_bounds__(256) void k_jbu(const float *__restrict__ img, int W, int H,
                                             const float *__restrict__ depth, int sw, int sh, int image_scale,
                                             float *__restrict__ out) {
    const int px = blockIdx.x * blockDim.x + threadIdx.x;
    const int py = blockIdx.y * blockDim.y + threadIdx.y;
    if (px >= W || py >= H) return;
    const float scale = (float)(1.0 * sw / W);
    const float sigmad = 0.50f, sigmar = 25.5f;
    const int nn = (image_scale * image_scale + 1) / 2;
    const float o_y = (float)py * scale;
    const float o_x = (float)px * scale;
    const float refPix = img[(size_t)py * W + px];
    float total_val = 0.0f, normalizing_factor = 0.0f;
    for (int j = -nn; j <= nn; ++j) {
        int r_y = (int)(o_y + (float)j);
        r_y = (r_y > 0 ? (r_y < sh ? r_y : sh - 1) : 0);
        int r_ys = py + j;
        r_ys = (r_ys > 0 ? (r_ys < H ? r_ys : H - 1) : 0);
        for (int i = -nn; i <= nn; ++i) {
            int r_x = (int)(o_x + (float)i);
            r_x = (r_x > 0 ? (r_x < sw ? r_x : sw - 1) : 0);
            const float srcPix = depth[(size_t)r_y * sw + r_x];
            int r_xs = px + i;
            r_xs = (r_xs > 0 ? (r_xs < W ? r_xs : W - 1) : 0);
            const float nb = img[(size_t)r_ys * W + r_xs];
            const float tg = spatial_gauss(o_x, o_y, (float)r_x, (float)r_y, sigmad) *
                             range_gauss(dm_fabs(refPix - nb), sigmar);
            normalizing_factor += tg;
            total_val += srcPix * tg;
        }
    }
    out[(size_t)py * W + px] = total_val / normalizing_factor;
}

// ---------------------------------------------------------------- launchers
// plane_hypotheses_host[center] = (0, 0, 0, depth) for the hierarchy init
// (src/ACMMP.cpp:797-804: x, y, z never written, pinned 0)
__global__ __launch_bounds__(256) void k_depth_planes(const float *__restrict__ depth, size_t n,
                                                      float4 *__restrict__ out) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = make_float4(0.0f, 0.0f, 0.0f, depth[i]);
}

hipError_t launch_depth_planes(const float *depth, size_t n, float4 *out, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    k_depth_planes<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream>>>(depth, n, out);
    return hipGetLastError();
}

hipError_t launch_jbu(const float *img, int W, int H, const float *depth, int sw, int sh, int image_scale,
                      float *out, hipStream_t stream) {
    dim3 block(64, 4), grid((W + 63) / 64, (H + 3) / 4);
    k_jbu<<<grid, block, 0, stream>>>(img, W, H, depth, sw, sh, image_scale, out);
    return hipGetLastError();
}

#endif  // !ACMMP_TX_UNIT

// Source-view count -> array capacity of the templated kernels.
static int ns_bucket(int nsrc) {
    if (nsrc <= 4) return 4;
    if (nsrc <= 9) return 9;
    if (nsrc <= 16) return 16;
    if (nsrc <= 20) return 20;
    return 32;
}

#ifdef ACMMP_DEV_SUBSET  // resource/ISA inspection builds only: u8 quads, NS 9 (and 16/20/32 with ACMMP_DEV_ALL_NS)
#ifdef ACMMP_DEV_ALL_NS
#define ACMMP_LAUNCH_NS(KERNEL, GRID, BLOCK, STREAM, ...)                                  \
    switch (ns_bucket(h_kv.nsrc)) {                                                         \
        case 9: KERNEL<9, 2><<<GRID, BLOCK, 0, STREAM>>>(__VA_ARGS__); break;               \
        case 16: KERNEL<16, 2><<<GRID, BLOCK, 0, STREAM>>>(__VA_ARGS__); break;             \
        case 20: KERNEL<20, 2><<<GRID, BLOCK, 0, STREAM>>>(__VA_ARGS__); break;             \
        default: KERNEL<32, 2><<<GRID, BLOCK, 0, STREAM>>>(__VA_ARGS__); break;             \
    }
#else
#define ACMMP_LAUNCH_NS(KERNEL, GRID, BLOCK, STREAM, ...) KERNEL<9, 2><<<GRID, BLOCK, 0, STREAM>>>(__VA_ARGS__);
#endif
#define ACMMP_LAUNCH_INIT(GRID, STREAM, ...) ACMMP_LAUNCH_NS(k_init, GRID, dim3(kBX, kBY), STREAM, __VA_ARGS__)
#define ACMMP_LAUNCH_SWEEP(GRID, STREAM, ...) ACMMP_LAUNCH_NS(k_sweep_f, GRID, dim3(kBX, kBY), STREAM, __VA_ARGS__)
#define ACMMP_LAUNCH_EVAL(GRID, STREAM, ...) ACMMP_LAUNCH_NS(k_eval_costs, GRID, dim3(kBX, kBY), STREAM, __VA_ARGS__)
#else
// The templated kernels (k_init, k_sweep_f, k_eval_costs) are instantiated
// per texel form in their own translation unit: acmmp_kernels.hip compiled
// with -DACMMP_TX_UNIT=<form> (Makefile), 5 NS buckets each, so the build
// compiles the 8 forms in parallel. These three functions per form are the
// units' entry points; the main unit picks the form.
template <int TX> hipError_t tx_launch_init(const KViews *d_kv, int nsrc, dim3 grid, hipStream_t s, KState st);
template <int TX>
hipError_t tx_launch_sweep(const KViews *d_kv, int nsrc, dim3 grid, hipStream_t s, KState st, int colour, int iter);
template <int TX>
hipError_t tx_launch_eval(const KViews *d_kv, int nsrc, dim3 grid, hipStream_t s, const float4 *planes, float *out,
                          float *out_init, uint32_t *out_views);
#define ACMMP_TX_FORMS(X) X(0) X(1) X(2) X(3) X(4) X(5) X(8) X(10)
#define ACMMP_TX_DECL(TX)                                                                                      \
    template <> hipError_t tx_launch_init<TX>(const KViews *, int, dim3, hipStream_t, KState);                  \
    template <> hipError_t tx_launch_sweep<TX>(const KViews *, int, dim3, hipStream_t, KState, int, int);       \
    template <> hipError_t tx_launch_eval<TX>(const KViews *, int, dim3, hipStream_t, const float4 *, float *,  \
                                              float *, uint32_t *);
#ifdef ACMMP_TX_UNIT
#define ACMMP_NS_SWITCH(KERNEL, GRID, STREAM, ...)                                                         \
    switch (ns_bucket(nsrc)) {                                                                              \
        case 4: KERNEL<4, ACMMP_TX_UNIT><<<GRID, dim3(kBX, kBY), 0, STREAM>>>(__VA_ARGS__); break;          \
        case 9: KERNEL<9, ACMMP_TX_UNIT><<<GRID, dim3(kBX, kBY), 0, STREAM>>>(__VA_ARGS__); break;          \
        case 16: KERNEL<16, ACMMP_TX_UNIT><<<GRID, dim3(kBX, kBY), 0, STREAM>>>(__VA_ARGS__); break;        \
        case 20: KERNEL<20, ACMMP_TX_UNIT><<<GRID, dim3(kBX, kBY), 0, STREAM>>>(__VA_ARGS__); break;        \
        default: KERNEL<32, ACMMP_TX_UNIT><<<GRID, dim3(kBX, kBY), 0, STREAM>>>(__VA_ARGS__); break;        \
    }
template <>
hipError_t tx_launch_init<ACMMP_TX_UNIT>(const KViews *d_kv, int nsrc, dim3 grid, hipStream_t s, KState st) {
    ACMMP_NS_SWITCH(k_init, grid, s, d_kv, st);
    return hipGetLastError();
}
template <>
hipError_t tx_launch_sweep<ACMMP_TX_UNIT>(const KViews *d_kv, int nsrc, dim3 grid, hipStream_t s, KState st,
                                          int colour, int iter) {
    ACMMP_NS_SWITCH(k_sweep_f, grid, s, d_kv, st, colour, iter);
    return hipGetLastError();
}
template <>
hipError_t tx_launch_eval<ACMMP_TX_UNIT>(const KViews *d_kv, int nsrc, dim3 grid, hipStream_t s,
                                         const float4 *planes, float *out, float *out_init, uint32_t *out_views) {
    ACMMP_NS_SWITCH(k_eval_costs, grid, s, d_kv, planes, out, out_init, out_views);
    return hipGetLastError();
}
#else
ACMMP_TX_FORMS(ACMMP_TX_DECL)
// KViews::wide -> the integer record index of views with 2^24 or more
// records; KViews::texel -> the texel form; texture_filter8 -> 8-bit fractions
static int tx_form(const KViews &h_kv) {
    return (h_kv.wide ? kTxWide : 0) | (h_kv.texel == kTexelU8 ? kTxU8 : 0) |
           (h_kv.texel == kTexelH16 ? kTxH16 : 0) | (h_kv.prm.texture_filter8 ? kTxFrac8 : 0);
}
#define ACMMP_TX_CASE(FN, TX, ...) case TX: return FN<TX>(__VA_ARGS__);
#define ACMMP_TX_DISPATCH(FN, ...)                                                                   \
    switch (tx_form(h_kv)) {                                                                          \
        ACMMP_TX_CASE(FN, 0, __VA_ARGS__) ACMMP_TX_CASE(FN, 1, __VA_ARGS__) ACMMP_TX_CASE(FN, 2, __VA_ARGS__) \
        ACMMP_TX_CASE(FN, 3, __VA_ARGS__) ACMMP_TX_CASE(FN, 4, __VA_ARGS__) ACMMP_TX_CASE(FN, 5, __VA_ARGS__) \
        ACMMP_TX_CASE(FN, 8, __VA_ARGS__) ACMMP_TX_CASE(FN, 10, __VA_ARGS__)                          \
        default: return hipErrorNotSupported; /* texture_filter8 with a wide or f16 form */           \
    }
#define ACMMP_LAUNCH_INIT(GRID, STREAM, ...) ACMMP_TX_DISPATCH(tx_launch_init, d_kv, h_kv.nsrc, GRID, STREAM, st)
#define ACMMP_LAUNCH_SWEEP(GRID, STREAM, ...) \
    ACMMP_TX_DISPATCH(tx_launch_sweep, d_kv, h_kv.nsrc, GRID, STREAM, st, colour, iter)
#define ACMMP_LAUNCH_EVAL(GRID, STREAM, ...) \
    ACMMP_TX_DISPATCH(tx_launch_eval, d_kv, h_kv.nsrc, GRID, STREAM, planes, out, out_init, out_views)
#endif
#endif

#ifndef ACMMP_TX_UNIT
// Colour-split grid over image rows [st.y0, st.y1): whole blocks of kBY
// rows from the block row holding y0 (the kernels skip rows outside).
static dim3 cs_grid(const KViews &kv, const KState &st, int colours) {
    const int by0 = st.y0 / kBY;
    return dim3((kv.Wh + kBX - 1) / kBX, (st.y1 - by0 * kBY + kBY - 1) / kBY, colours);
}
// 64 x 4 grid over rows [st.y0, st.y1) and `cols` columns
static dim3 row_grid(int cols, const KState &st) {
    return dim3((cols + 63) / 64, (st.y1 - (st.y0 / 4) * 4 + 3) / 4);
}

hipError_t launch_init(const KViews *d_kv, const KViews &h_kv, const KState &st, hipStream_t stream) {
    if (st.y1 <= st.y0) return hipSuccess;
    ACMMP_LAUNCH_INIT(cs_grid(h_kv, st, 2), stream, d_kv, st);
    return hipGetLastError();
}

hipError_t launch_sweep(const KViews *d_kv, const KViews &h_kv, const KState &st, int colour, int iter,
                        hipStream_t stream) {
    if (st.y1 <= st.y0) return hipSuccess;
    ACMMP_LAUNCH_SWEEP(cs_grid(h_kv, st, 1), stream, d_kv, st, colour, iter);
    return hipGetLastError();
}

hipError_t launch_finalize(const KViews *d_kv, const KViews &h_kv, const KState &st, hipStream_t stream) {
    if (st.y1 <= st.y0) return hipSuccess;
    k_finalize<<<row_grid(h_kv.W, st), dim3(64, 4), 0, stream>>>(d_kv, st);
    return hipGetLastError();
}

hipError_t launch_filter(const KViews *d_kv, const KViews &h_kv, const KState &st, int colour,
                         hipStream_t stream) {
    if (st.y1 <= st.y0) return hipSuccess;
    k_filter<<<row_grid(h_kv.Wh, st), dim3(64, 4), 0, stream>>>(d_kv, st, colour);
    return hipGetLastError();
}

hipError_t launch_eval_costs(const KViews *d_kv, const KViews &h_kv, const float4 *planes, float *out,
                             float *out_init, uint32_t *out_views, hipStream_t stream) {
    KState all{};
    all.y1 = h_kv.H;
    ACMMP_LAUNCH_EVAL(cs_grid(h_kv, all, 2), stream, d_kv, planes, out, out_init, out_views);
    return hipGetLastError();
}

hipError_t launch_eval_geom(const KViews *d_kv, const KViews &h_kv, const float4 *planes, float *out,
                            hipStream_t stream) {
    dim3 block(64, 4), grid((h_kv.W + 63) / 64, (h_kv.H + 3) / 4);
    k_eval_geom<<<grid, block, 0, stream>>>(d_kv, planes, out);
    return hipGetLastError();
}
#endif  // !ACMMP_TX_UNIT

}  // namespace acmmp
