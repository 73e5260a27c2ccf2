// acmmp_planar.hip — planar-prior construction, the block of
// ProcessProblem between the first and second RunPatchMatch
// (src/acmmp_definitions.cpp:301-376):
//
//   GetSupportPoints        src/ACMMP.cpp:868-894    k_support_points (GPU)
//   DelaunayTriangulation   src/ACMMP.cpp:896-918    acmmp_delaunay.cpp (host, exact integer predicates)
//   triangle raster         acmmp_definitions.cpp:332-353   k_raster_triangles (GPU)
//   GetPriorPlaneParams     src/ACMMP.cpp:920-953    k_prior_planes (GPU)
//   GetDepthFromPlaneParam + range check  :955-958, acmmp_definitions.cpp:356-370   k_prior_range (GPU)
//   CudaPlanarPriorInitialization         src/ACMMP.cpp:811-831   (same kernel)
//
// Everything after the triangulation stays on the device: the depth map the
// planes are fitted to is the engine's resident result and the label mask /
// prior planes are written straight into the engine's prior buffers.
//
// Pins:
//  * cv::Subdiv2D is replaced by an exact Delaunay triangulation seeded with
//    Subdiv2D's own bounding triangle (3·max(w,h), src of OpenCV's
//    initDelaunay) so hull behaviour matches; co-circular ties keep the
//    existing triangulation (strict in-circle test).
//  * cv::SVD::solveZ's null vector is the cofactor vector of the 3x4 system,
//    computed in double and normalised to unit length before the reference's
//    own sign / normal normalisation (:942-951).
//  * The raster follows the reference's float/double mix literally: p and q
//    are float accumulators, 1/max_edge is formed in double and rounded to
//    float, `(1.0 - p - q) * x3` is double, the sum truncates toward zero.
//    Overlapping triangles: the later triangle wins (atomicMax of the label
//    equals the sequential overwrite order).
#include <algorithm>
#include <cstring>

#include "acmmp_ctx.h"

namespace {

constexpr int kSupportStep = 5;  // step_size (src/ACMMP.cpp:871)
constexpr int kMaxSeq = 16384;   // p/q sequence length cap = max triangle edge in px

// One thread per 5x5 block; block b = bc * nbr + br (the reference iterates
// col-major over blocks and over pixels inside a block).
__global__ void k_support_points(const float *__restrict__ cost, int W, int H, int nbr, int nblocks,
                                 int32_t *__restrict__ out) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nblocks) return;
    const int col = (b / nbr) * kSupportStep, row = (b % nbr) * kSupportStep;
    const int cb = min(W, col + kSupportStep), rb = min(H, row + kSupportStep);
    float min_cost = 2.0f;
    int px = 0, py = 0;
    for (int c = col; c < cb; ++c)
        for (int r = row; r < rb; ++r) {
            const float v = cost[(size_t)r * W + c];
            if (v < 2.0f && min_cost > v) {
                px = c;
                py = r;
                min_cost = v;
            }
        }
    out[b] = (min_cost < 0.1f) ? (py << 16) | px : -1;
}

// GetPriorPlaneParams (src/ACMMP.cpp:920-953) for triangle corners (x, y)
// with depths d: host (acmmp_prior_plane_params) and device (k_prior_planes).
__host__ __device__ inline float4 prior_plane(const acmmp_camera &cam, const int32_t *tri, const float *dk) {
    double A[3][4];
    for (int k = 0; k < 3; ++k) {
        const int x = tri[2 * k], y = tri[2 * k + 1];
        const float d = dk[k];
        // Get3DPointonRefCam (src/ACMMP.cpp:230-239)
        const float X = d * ((float)x - cam.K[2]) / cam.K[0];
        const float Y = d * ((float)y - cam.K[5]) / cam.K[4];
        A[k][0] = X;
        A[k][1] = Y;
        A[k][2] = d;
        A[k][3] = 1.0;
    }
    // null vector of A: n_j = (-1)^j det(A without column j)
    double n[4];
    for (int j = 0; j < 4; ++j) {
        const int c0 = j == 0 ? 1 : 0;
        const int c1 = j <= 1 ? 2 : 1;
        const int c2 = j <= 2 ? 3 : 2;
        const double m =
            A[0][c0] * (A[1][c1] * A[2][c2] - A[1][c2] * A[2][c1]) -
            A[0][c1] * (A[1][c0] * A[2][c2] - A[1][c2] * A[2][c0]) +
            A[0][c2] * (A[1][c0] * A[2][c1] - A[1][c1] * A[2][c0]);
        n[j] = (j & 1) ? -m : m;
    }
    const double len = sqrt(((n[0] * n[0] + n[1] * n[1]) + n[2] * n[2]) + n[3] * n[3]);
    float4 n4 = make_float4((float)(n[0] / len), (float)(n[1] / len), (float)(n[2] / len), (float)(n[3] / len));
    // :942-951 — pow(float, 2) is an exact square in double
    float norm2 = (float)sqrt(((double)n4.x * n4.x + (double)n4.y * n4.y) + (double)n4.z * n4.z);
    if (n4.w < 0) norm2 *= -1;
    n4.x /= norm2;
    n4.y /= norm2;
    n4.z /= norm2;
    n4.w /= norm2;
    return n4;
}

// GetDepthFromPlaneParam (src/ACMMP.cpp:955-958).
__host__ __device__ inline float depth_from_plane(const acmmp_camera &cam, float4 pl, int x, int y) {
    const float num = -pl.w * cam.K[0];
    const float den =
        ((float)x - cam.K[2]) * pl.x + (cam.K[0] / cam.K[4]) * ((float)y - cam.K[5]) * pl.y + cam.K[0] * pl.z;
    return num / den;
}

__global__ void k_prior_planes(const float4 *__restrict__ rm_plane, int W, acmmp_camera cam,
                               const int32_t *__restrict__ tris, int ntris, float4 *__restrict__ planes) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntris) return;
    const int32_t *tri = tris + 6 * t;
    float d[3];
    for (int k = 0; k < 3; ++k) d[k] = rm_plane[(size_t)tri[2 * k + 1] * W + tri[2 * k]].w;  // depths(y, x)
    planes[t] = prior_plane(cam, tri, d);
}

__device__ __forceinline__ float edge_len(int ax, int ay, int bx, int by) {
    // sqrt(pow(dx, 2) + pow(dy, 2)) in double, stored to float (:339-341)
    const double dx = (double)(ax - bx), dy = (double)(ay - by);
    return (float)sqrt(dx * dx + dy * dy);
}

// Triangle raster (src/acmmp_definitions.cpp:336-353), one block per triangle.
// The p and q loops run over the same float sequence s_0 = 0,
// s_k = s_{k-1} + step (while < 1.0), built once in LDS by lane 0; rows p
// are then spread over the block.
__global__ __launch_bounds__(256) void k_raster_triangles(const int32_t *__restrict__ tris, int ntris, int W,
                                                          int H, uint32_t *__restrict__ label,
                                                          int *__restrict__ overflow) {
    __shared__ float seq[kMaxSeq];
    __shared__ int nseq;
    const int t = blockIdx.x;
    if (t >= ntris) return;
    const int x1 = tris[6 * t], y1 = tris[6 * t + 1];
    const int x2 = tris[6 * t + 2], y2 = tris[6 * t + 3];
    const int x3 = tris[6 * t + 4], y3 = tris[6 * t + 5];
    if (threadIdx.x == 0) {
        const float L01 = edge_len(x1, y1, x2, y2);
        const float L02 = edge_len(x1, y1, x3, y3);
        const float L12 = edge_len(x2, y2, x3, y3);
        const float max_edge = fmaxf(L01, fmaxf(L02, L12));
        const float step = (float)(1.0 / (double)max_edge);
        int n = 0;
        for (float p = 0; p < 1.0; p += step) {
            if (n == kMaxSeq) {
                atomicAdd(overflow, 1);
                break;
            }
            seq[n++] = p;
        }
        nseq = n;
    }
    __syncthreads();
    const int n = nseq;
    const uint32_t lab = (uint32_t)t + 1u;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const float p = seq[i];
        const double lim = 1.0 - (double)p;
        for (int j = 0; j < n && (double)seq[j] < lim; ++j) {
            const float q = seq[j];
            const float fxy = p * (float)x1 + q * (float)x2;
            const float fyy = p * (float)y1 + q * (float)y2;
            const int x = (int)((double)fxy + ((1.0 - (double)p) - (double)q) * (double)x3);
            const int y = (int)((double)fyy + ((1.0 - (double)p) - (double)q) * (double)y3);
            if ((unsigned)x < (unsigned)W && (unsigned)y < (unsigned)H) atomicMax(&label[(size_t)y * W + x], lab);
        }
    }
}

// Range check of the prior depth (src/acmmp_definitions.cpp:356-370,
// GetDepthFromPlaneParam src/ACMMP.cpp:955-958) and
// CudaPlanarPriorInitialization's label -> plane expansion (:819-827).
__global__ void k_prior_range(const float4 *__restrict__ planes, acmmp_camera cam, float dmin, float dmax, int W,
                              int H, uint32_t *__restrict__ label, float4 *__restrict__ prior) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    if (x >= W || y >= H) return;
    const size_t i = (size_t)y * W + x;
    uint32_t l = label[i];
    float4 pl = make_float4(0.f, 0.f, 0.f, 0.f);
    if (l > 0) {
        pl = planes[l - 1];
        const float d = depth_from_plane(cam, pl, x, y);
        if (!(d <= dmax && d >= dmin)) {
            l = 0;
            label[i] = 0;
        }
    }
    prior[i] = l > 0 ? pl : make_float4(0.f, 0.f, 0.f, 0.f);
}

}  // namespace

extern "C" {

int acmmp_prior_plane_params(const acmmp_camera *cam, const int32_t *tri, const float *depths, float *out4) {
    if (!cam || !tri || !depths || !out4) return ACMMP_ERR_ARG;
    const float4 n4 = prior_plane(*cam, tri, depths);
    out4[0] = n4.x;
    out4[1] = n4.y;
    out4[2] = n4.z;
    out4[3] = n4.w;
    return ACMMP_OK;
}

float acmmp_depth_from_plane_param(const acmmp_camera *cam, const float *plane4, int x, int y) {
    if (!cam || !plane4) return 0.0f;
    return depth_from_plane(*cam, make_float4(plane4[0], plane4[1], plane4[2], plane4[3]), x, y);
}

int acmmp_get_support_points(acmmp_ctx *ctx, int32_t *xy, int capacity, int *count) {
    int rc = check_ready(ctx);
    if (rc) return rc;
    if (!count || capacity < 0 || (capacity > 0 && !xy)) return set_err(ctx, ACMMP_ERR_ARG, "bad output");
    if (!ctx->have_state) return set_err(ctx, ACMMP_ERR_STATE, "no results: run acmmp_run_patchmatch first");
    const int W = ctx->W, H = ctx->H;
    const int nbc = (W + kSupportStep - 1) / kSupportStep, nbr = (H + kSupportStep - 1) / kSupportStep;
    const int nblocks = nbc * nbr;
    int32_t *d_out = nullptr;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, dalloc(d_out, (size_t)nblocks));
    k_support_points<<<(nblocks + 255) / 256, 256, 0, ctx->stream>>>(ctx->d_rm_cost, W, H, nbr, nblocks, d_out);
    std::vector<int32_t> h(nblocks);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess)
        e = hipMemcpyAsync(h.data(), d_out, nblocks * sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e == hipSuccess) dfree_synced(d_out);
    else dfree(d_out);
    HIP_TRY(ctx, e);
    int n = 0;
    for (int b = 0; b < nblocks; ++b) {
        if (h[b] < 0) continue;
        if (n < capacity) {
            xy[2 * n] = h[b] & 0xffff;
            xy[2 * n + 1] = h[b] >> 16;
        }
        ++n;
    }
    *count = n;
    return n > capacity ? set_err(ctx, ACMMP_ERR_ARG, "capacity %d < %d support points", capacity, n) : ACMMP_OK;
}

int acmmp_build_planar_prior(acmmp_ctx *ctx, const int32_t *tris, int ntris, float *out_planes4,
                             uint32_t *out_mask) {
    int rc = check_ready(ctx);
    if (rc) return rc;
    if (ntris < 0 || (ntris > 0 && !tris)) return set_err(ctx, ACMMP_ERR_ARG, "bad triangle list");
    if (!ctx->have_state) return set_err(ctx, ACMMP_ERR_STATE, "no results: run acmmp_run_patchmatch first");
    const int W = ctx->W, H = ctx->H;
    const size_t P = (size_t)W * H;
    // the reference keeps only triangles whose 3 corners lie in the image
    // (:333); DelaunayTriangulation's output already satisfies it, other
    // callers' lists are filtered the same way here.
    std::vector<int32_t> kept;
    kept.reserve((size_t)ntris * 6);
    for (int t = 0; t < ntris; ++t) {
        bool in = true;
        for (int k = 0; k < 3; ++k) {
            const int x = tris[6 * t + 2 * k], y = tris[6 * t + 2 * k + 1];
            in = in && x >= 0 && x < W && y >= 0 && y < H;
        }
        if (in) kept.insert(kept.end(), tris + 6 * t, tris + 6 * t + 6);
    }
    const int nt = (int)(kept.size() / 6);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    int32_t *d_tris = nullptr;
    float4 *d_planes = nullptr;
    int *d_overflow = nullptr;
    HIP_TRY(ctx, dalloc(d_tris, kept.size() + 6));
    HIP_TRY(ctx, dalloc(d_planes, (size_t)nt + 1));
    HIP_TRY(ctx, dalloc(d_overflow, 1));
    HIP_TRY(ctx, dalloc(ctx->d_prior, P));
    HIP_TRY(ctx, dalloc(ctx->d_mask, P));
    hipStream_t s = ctx->stream;
    HIP_TRY(ctx, hipMemsetAsync(ctx->d_mask, 0, P * sizeof(uint32_t), s));
    HIP_TRY(ctx, hipMemsetAsync(d_overflow, 0, sizeof(int), s));
    if (nt > 0) {
        HIP_TRY(ctx, hipMemcpyAsync(d_tris, kept.data(), kept.size() * sizeof(int32_t), hipMemcpyHostToDevice, s));
        k_prior_planes<<<(nt + 127) / 128, 128, 0, s>>>(ctx->d_rm_plane, W, ctx->cams[0], d_tris, nt, d_planes);
        HIP_TRY(ctx, hipGetLastError());
        k_raster_triangles<<<nt, 256, 0, s>>>(d_tris, nt, W, H, ctx->d_mask, d_overflow);
        HIP_TRY(ctx, hipGetLastError());
    }
    k_prior_range<<<dim3((W + 255) / 256, H), 256, 0, s>>>(d_planes, ctx->cams[0], ctx->prm.depth_min,
                                                           ctx->prm.depth_max, W, H, ctx->d_mask, ctx->d_prior);
    HIP_TRY(ctx, hipGetLastError());
    int overflow = 0;
    HIP_TRY(ctx, hipMemcpyAsync(&overflow, d_overflow, sizeof(int), hipMemcpyDeviceToHost, s));
    if (out_planes4 && nt > 0)
        HIP_TRY(ctx, hipMemcpyAsync(out_planes4, d_planes, (size_t)nt * sizeof(float4), hipMemcpyDeviceToHost, s));
    if (out_mask) HIP_TRY(ctx, hipMemcpyAsync(out_mask, ctx->d_mask, P * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(ctx, hipStreamSynchronize(s));
    dfree_synced(d_tris);
    dfree_synced(d_planes);
    dfree_synced(d_overflow);
    if (overflow) return set_err(ctx, ACMMP_ERR_UNSUPPORTED, "%d triangles longer than %d px", overflow, kMaxSeq);
    ctx->have_prior = true;
    return ACMMP_OK;
}

int acmmp_prepare_planar_prior(acmmp_ctx *ctx, int *num_support_points, int *num_triangles) {
    int rc = check_ready(ctx);
    if (rc) return rc;
    const int cap = (ctx->W / kSupportStep + 1) * (ctx->H / kSupportStep + 1);
    std::vector<int32_t> pts((size_t)cap * 2);
    int npts = 0;
    rc = acmmp_get_support_points(ctx, pts.data(), cap, &npts);
    if (rc) return rc;
    // a planar triangulation of n points has at most 2n - 5 triangles
    const int tcap = 2 * npts + 16;
    std::vector<int32_t> tris((size_t)tcap * 6);
    int nt = 0;
    rc = acmmp_delaunay_triangulation(ctx->W, ctx->H, pts.data(), npts, tris.data(), tcap, &nt);
    if (rc) return set_err(ctx, rc, "Delaunay triangulation of %d points failed", npts);
    rc = acmmp_build_planar_prior(ctx, tris.data(), nt, nullptr, nullptr);
    if (rc) return rc;
    ctx->prm.planar_prior = 1;  // SetPlanarPriorParams (src/ACMMP.cpp:456-459)
    if (num_support_points) *num_support_points = npts;
    if (num_triangles) *num_triangles = nt;
    return ACMMP_OK;
}

}  // extern "C"
