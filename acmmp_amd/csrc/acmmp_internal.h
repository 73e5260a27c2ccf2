// acmmp_internal.h — device-side data layout shared by the kernels
// (acmmp_kernels.hip) and the host engine (acmmp_engine.hip).
//
// HBM layout (per engine = per reference view being processed):
//   * source images: one pitched fp32 buffer per view (pitch = width rounded
//     up to 64 floats = 256 B, so every row starts on a 256-B boundary).
//   * PatchMatch state during the sweeps is stored COLOUR-SPLIT: pixel (x, y)
//     has colour c = (x + y) & 1 and lives at index y * Wh + (x >> 1) of the
//     colour-c plane, Wh = ceil(W / 2). A half-sweep of colour c reads both
//     colour planes and writes only colour c, so a wave's 64 lanes touch 64
//     consecutive elements of every array it streams (coalesced), and
//     same-colour snapshot reads (reference race) are
//     served by ping-pong buffers of the written colour with no copy.
//   * between runs the state is row-major (`rm_*`): exactly the reference's
//     plane_hypotheses_cuda / costs_cuda / selected_views_cuda, which the
//     init kernel reads and the finalize + filter kernels write.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/acmmp.h"

namespace acmmp {

// Per-view geometry derived from the two cameras, identical expressions to
// ComputeHomography's camera-only part (src/ACMMP.cu:264-290).
struct ViewRel {
    float Rr[9];   // R_relative
    float tr[3];   // t_relative
};

// Texel forms of the padded source views (KViews::texel).
enum { kTexelF32 = 0, kTexelU8 = 1, kTexelH16 = 2 };

struct KViews {
    acmmp_params prm;
    acmmp_camera cam[ACMMP_MAX_IMAGES];
    ViewRel rel[ACMMP_MAX_IMAGES];            // rel[v] for source v (1-based), rel[0] unused
    const float *img[ACMMP_MAX_IMAGES];       // pitched images
    int ipitch[ACMMP_MAX_IMAGES];             // in floats
    // Source images with clamp-to-edge baked in, so the 2x2 bilinear
    // footprint of a coordinate clamped to [-1, W] x [-1, H] is ONE load at
    // record (y0 + 1, x0 + 1), without integer clamps or selects. Either
    //  * f16 difference quads (kTexelH16): record (r, c), r < H + 2,
    //    c < W + 2, holds the halves (t00, t01, t10 - t00, t11 - t01) of
    //    texels t00 = (c-1, r-1), t01 = (c-1, r), t10 = (c, r-1),
    //    t11 = (c, r) (clamped): 8 B per footprint, when every stored value
    //    is exact in f16 (8-bit input is);
    //  * u8 quads (kTexelU8): the bytes of the same four texels, 4 B per
    //    footprint, when every view is integer-valued in [0, 255];
    //  * fp32 row pairs: record (r, c), c < W + 3, is the float pair
    //    (texel(c-1, r-1), texel(c-1, r)); a footprint is two records, 16 B.
    const float *pad[ACMMP_MAX_IMAGES];
    int ppitch[ACMMP_MAX_IMAGES];             // in records
    // -(R^T t) of every camera, the world-frame offset Get3DPointonWorld_cu
    // adds (src/ACMMP.cu:494-503), formed once on the host with the
    // kernel's float expression (same operations, same order: exact)
    float cw[ACMMP_MAX_IMAGES][3];
    const float *dep[ACMMP_MAX_IMAGES];       // pitched depth maps (geom consistency)
    int dpitch[ACMMP_MAX_IMAGES];
    int dw[ACMMP_MAX_IMAGES];
    int dh[ACMMP_MAX_IMAGES];
    int W, H, Wh, sweep_rows, nsrc;
    int wide;                                 // some view has >= 2^24 padded records
    int texel;                                // form of pad[]: kTexelF32 / kTexelU8 / kTexelH16
    float inv_k0, inv_k4;                     // 1/K[0], 1/K[4] of the ref camera (pin P4)
    float pert_pi, pert3_pi, angle_sigma;     // double-precision constants of the reference
    // Bilateral weights of ComputeBilateralWeight (src/ACMMP.cu:353-358) for
    // an 8-bit reference image (texel == kTexelU8: every texel an integer in
    // [0, 255], so |I - I_c| is one of 256 values): wlut[cls][d] =
    // expf(-spatial_cls / (2 ss^2) - d / (2 sc^2)), cls = the tap's distance
    // class (|dx|, |dy|) in {1, 3, 5}^2 up to order (kWlutClasses), formed on
    // the host by the kernel's own float expression (same operations, same
    // order: bit-identical to computing it per tap).
    float wlut[6][256];
};
constexpr int kWlutClasses = 6;
// distance class of |dx|, |dy| in {1, 3, 5}: (a, b) = ((|dx| - 1) / 2, (|dy| - 1) / 2), unordered
__host__ __device__ constexpr int wlut_class(int a, int b) {
    return a > b ? wlut_class(b, a) : (a == 0 ? b : (a == 1 ? 2 + b : 5));
}

struct KState {
    float4 *plane[2];       // colour-split current (read) planes, [colour]
    float *cost[2];
    float4 *plane_nx[2];    // colour-split next (written) planes
    float *cost_nx[2];
    uint32_t *sv[2];        // colour-split selected views (in place)
    float4 *rm_plane;       // row-major state between runs
    float *rm_cost;
    float *rm_depth;        // rm_plane[.].w as its own plane (finalize and filters)
    uint32_t *rm_sv;
    float *pre_cost;        // hierarchy (row-major)
    const float4 *prior;    // planar prior planes (row-major)
    const uint32_t *mask;   // planar prior triangle labels
    const float4 *scaled;   // hierarchy low-res planes (scaled_rows x scaled_cols)
    const float4 *seed;     // seeded priors
    int y0, y1;             // image rows [y0, y1) a launch covers (all rows, or a band; acmmp_run_patchmatch_band)
};

// Kernel launchers (acmmp_kernels.hip). All enqueue on `stream`.
hipError_t launch_init(const KViews *d_kv, const KViews &h_kv, const KState &st, hipStream_t stream);
hipError_t launch_sweep(const KViews *d_kv, const KViews &h_kv, const KState &st, int colour,
                        int iter, hipStream_t stream);
hipError_t launch_finalize(const KViews *d_kv, const KViews &h_kv, const KState &st,
                           hipStream_t stream);
hipError_t launch_filter(const KViews *d_kv, const KViews &h_kv, const KState &st, int colour,
                         hipStream_t stream);
hipError_t launch_eval_costs(const KViews *d_kv, const KViews &h_kv, const float4 *planes,
                             float *out_costs, float *out_init, uint32_t *out_views,
                             hipStream_t stream);
hipError_t launch_eval_geom(const KViews *d_kv, const KViews &h_kv, const float4 *planes,
                            float *out, hipStream_t stream);

hipError_t launch_pad_image(const float *src, int spitch, int W, int H, float *dst, int dpitch,
                            hipStream_t stream);
// f16 difference-quad copy of one view; sets *not_h16 = 1 if a stored value
// is not exact in f16 (the copy is then unusable and the fp32 form is built).
hipError_t launch_pad_h16(const float *src, int spitch, int W, int H, void *dst, int dpitch, uint32_t *not_h16,
                          hipStream_t stream);
// u8 texel-quad copy of one view; sets *not_u8 = 1 if a texel is not an
// integer in [0, 255] (the copy is then unusable and the fp32 form is built).
hipError_t launch_pad_quad(const float *src, int spitch, int W, int H, uint32_t *dst, int dpitch,
                           uint32_t *not_u8, hipStream_t stream);
hipError_t launch_depth_planes(const float *depth, size_t n, float4 *out, hipStream_t stream);
hipError_t launch_jbu(const float *img, int W, int H, const float *depth, int sw, int sh, int image_scale,
                      float *out, hipStream_t stream);
hipError_t launch_selftest_rcp(unsigned long long *mismatch, unsigned long long *checked, hipStream_t s);

// Number of checkerboard rows the reference grid reaches (src/ACMMP.cu:1399).
inline int checkerboard_rows(int H) {
    int gy = ((H / 2) + 16 - 1) / 16;
    int rows = gy * 32;
    return rows < H ? rows : H;
}

}  // namespace acmmp
