// Two samples per gather? k_sweep gathers one u8-quad
// record (the 2x2 bilinear footprint, 4 B) per patch sample: 36 dword
// gathers per NCC call. Horizontally adjacent samples of a patch row are 2
// source texels apart, so a "pair record" of 8 B (the quads at x0 and x0 + 2)
// serves both samples of a pair with one 64-bit gather whenever the second
// sample's floor is exactly (x0 + 2, y0); the lanes where it is not need a
// dword gather of their own. This measures what that costs the texture path
// on k_sweep's own lane geometry (8 x 8 colour-split pixels per wave, lane
// map 2) under a near-identity affine map of the patch (scale 1 + e, shear):
//   mode 0  36 dword gathers per patch from quad records (the product)
//   mode 1  18 b64 gathers from pair records + a dword gather for the lanes
//           whose second sample misses the pair record (exec-masked)
//   mode 2  the 18 b64 gathers alone (mode 1's bound)
//   mode 3  the masked dword gathers of mode 1 alone
// over maps: e = 0 / 0.03 / 0.08 with shear 0.02 (the fallback share is
// printed per map). Run under rocprofv3 --pmc TD_TD_BUSY_sum
// TCP_TOTAL_CACHE_ACCESSES_sum TA_BUFFER_READ_WAVEFRONTS_sum
// (tools/microbench/run_pair.sh).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
__device__ unsigned sbl32(__amdgpu_buffer_rsrc_t r, int vindex, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.struct.ptr.buffer.load.i32");
__device__ u32x2 sbl64(__amdgpu_buffer_rsrc_t r, int vindex, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.struct.ptr.buffer.load.v2i32");

constexpr int ITERS = 16;
constexpr int PITCH = 1632;  // records per row (cfg2 u8-quad pitch)
constexpr int ROWS = 1300;

struct Map {
    float e, sh;
};

template <int MODE>
__global__ __launch_bounds__(256) void k_pair(const unsigned *quads, const u32x2 *pairs, Map m, unsigned *out,
                                              unsigned *fallback) {
    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc((void *)quads, (short)4, PITCH * ROWS, 0x00020000);
    const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc((void *)pairs, (short)8, PITCH * ROWS, 0x00020000);
    const int l = threadIdx.x & 63, wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    // lane map 2: a quarter is 4 colour-split columns x 4 rows, column-major
    const int lc = ((l >> 2) & 3) + 4 * ((l >> 4) & 1), lr = (l & 3) + 4 * (l >> 5);
    const int wx = wave % 90, wy = (wave / 90) % 140;
    const int py = 16 + wy * 8 + lr;
    const int px = 16 + 2 * (wx * 8 + lc) + (py & 1);
    unsigned acc = 0, nfb = 0;
#pragma unroll 1
    for (int it = 0; it < ITERS; ++it) {
        float off = 0.37f + 0.013f * (float)it;  // sub-texel offset, varied per iteration
        asm volatile("" : "+v"(off));
        for (int j = -5; j <= 5; j += 2) {
            const float y = (float)(py + j);
#pragma unroll
            for (int i = -5; i <= 5; i += 4) {
                const float xa = (float)(px + i), xb = (float)(px + i + 2);
                const float ua = xa * (1.0f + m.e) + y * m.sh + off, va = y * (1.0f + m.e) - xa * m.sh + off + 40.0f;
                const float ub = xb * (1.0f + m.e) + y * m.sh + off, vb = y * (1.0f + m.e) - xb * m.sh + off + 40.0f;
                const int xa0 = (int)__builtin_floorf(ua), ya0 = (int)__builtin_floorf(va);
                const int xb0 = (int)__builtin_floorf(ub), yb0 = (int)__builtin_floorf(vb);
                const int ia = (ya0 + 1) * PITCH + xa0 + 1, ib = (yb0 + 1) * PITCH + xb0 + 1;
                const bool miss = !(xb0 == xa0 + 2 && yb0 == ya0);
                nfb += miss;
                if (MODE == 0) {
                    acc += sbl32(rq, ia, 0, 0, 0);
                    acc += sbl32(rq, ib, 0, 0, 0);
                } else if (MODE == 1 || MODE == 2) {
                    const u32x2 p = sbl64(rp, ia, 0, 0, 0);
                    acc += p.x;
                    if (MODE == 1 && miss) acc += sbl32(rq, ib, 0, 0, 0);
                    else acc += p.y;
                } else {
                    if (miss) acc += sbl32(rq, ib, 0, 0, 0);
                }
            }
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
    if (MODE == 0) atomicAdd(fallback, nfb);
}

int main() {
    const size_t n = (size_t)PITCH * ROWS;
    unsigned *quads, *out, *fb;
    u32x2 *pairs;
    (void)hipMalloc(&quads, n * 4);
    (void)hipMalloc(&pairs, n * 8);
    (void)hipMalloc(&out, 4);
    (void)hipMalloc(&fb, 4);
    (void)hipMemset(quads, 1, n * 4);
    (void)hipMemset(pairs, 1, n * 8);
    const int blocks = 90 * 140 / 4;  // one wave per 8 x 8 pixel tile of a 1440 x 1120 area
    const Map maps[3] = {{0.0f, 0.02f}, {0.03f, 0.02f}, {0.08f, 0.02f}};
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int mi = 0; mi < 3; ++mi) {
        for (int mode = 0; mode < 4; ++mode) {
            for (int rep = 0; rep < 3; ++rep) {
                (void)hipMemset(fb, 0, 4);
                (void)hipEventRecord(a);
                if (mode == 0) k_pair<0><<<blocks, 256>>>(quads, pairs, maps[mi], out, fb);
                if (mode == 1) k_pair<1><<<blocks, 256>>>(quads, pairs, maps[mi], out, fb);
                if (mode == 2) k_pair<2><<<blocks, 256>>>(quads, pairs, maps[mi], out, fb);
                if (mode == 3) k_pair<3><<<blocks, 256>>>(quads, pairs, maps[mi], out, fb);
                (void)hipEventRecord(b);
                (void)hipEventSynchronize(b);
                float ms = 0;
                (void)hipEventElapsedTime(&ms, a, b);
                unsigned nfb = 0;
                (void)hipMemcpy(&nfb, fb, 4, hipMemcpyDeviceToHost);
                if (rep == 2) {
                    const double pairs_total = (double)blocks * 256 * ITERS * 18;
                    printf("map e=%.2f sh=%.2f mode %d: %.4f ms", maps[mi].e, maps[mi].sh, mode, ms);
                    if (mode == 0) printf(", second sample off the pair record: %.2f %% of lane-pairs", 100.0 * nfb / pairs_total);
                    printf("\n");
                }
            }
        }
    }
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
