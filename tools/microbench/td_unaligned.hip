// Unaligned (2-B aligned) dword buffer loads on gfx950: correctness and TD /
// L1 tag cost vs the aligned 4-B records k_sweep gathers today. A 2-B
// "column pair" record layout would put a 2x2 u8 footprint in 4 contiguous
// bytes at a 2-B aligned address, halving the bytes per footprint record.
// Patterns (ITERS loads per lane, k_sweep wave shape 8 x 8 pixels, 2-px
// lane spacing, sample walk over a 6 x 6 patch with a 2-px step):
//   0: 4-B records, idxen stride 4 (today)
//   1: 2-B records, idxen stride 2, dword load at 2-B alignment
//   2: 2-B records, byte-offset (offen) form
// Checks every loaded word of patterns 1/2 against the bytes it must hold.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ unsigned sbl32(__amdgpu_buffer_rsrc_t r, int vindex, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.struct.ptr.buffer.load.i32");
__device__ unsigned rbl32(__amdgpu_buffer_rsrc_t r, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.ptr.buffer.load.i32");

constexpr int ITERS = 576;
constexpr int PITCH = 1632;  // records per row

__global__ __launch_bounds__(256) void k_gather(const unsigned char *buf, int nbytes, int pattern, unsigned *out,
                                                unsigned *bad) {
    const int stride = pattern == 0 ? 4 : 2;
    __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)buf, (short)stride, nbytes / stride, 0x00020000);
    __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc((void *)buf, (short)0, nbytes, 0x00020000);
    const int lane = threadIdx.x & 63, wave = (blockIdx.x * 4 + (threadIdx.x >> 6));
    const int c = lane & 7, r = lane >> 3;  // 8 x 8 pixels
    int base = (wave % 64) * 8 * PITCH + 64;
    unsigned acc = 0, nbad = 0;
#pragma unroll 1
    for (int it = 0; it < ITERS; ++it) {
        const int s = it % 36;
        const int idx = base + r * PITCH + 2 * c + (s % 6) * 2 + (s / 6) * 2 * PITCH + (it / 36) % 3;
        unsigned v;
        if (pattern == 0) v = sbl32(rs, idx, 0, 0, 0);
        else if (pattern == 1) v = sbl32(rs, idx, 0, 0, 0);
        else v = rbl32(rr, 2 * idx, 0, 0);
        if (pattern != 0) {
            const size_t b = (size_t)2 * idx;
            const unsigned want = buf[b] | buf[b + 1] << 8 | buf[b + 2] << 16 | (unsigned)buf[b + 3] << 24;
            nbad += v != want;
        }
        acc += v;
    }
    if (acc == 0x12345678u) out[0] = acc;
    if (nbad) atomicAdd(bad, nbad);
}

int main() {
    const int nbytes = PITCH * 4 * 600;
    std::vector<unsigned char> h(nbytes);
    for (int i = 0; i < nbytes; ++i) h[i] = (unsigned char)(i * 131 + (i >> 8) * 7);
    unsigned char *buf;
    unsigned *out, *bad;
    (void)hipMalloc(&buf, nbytes);
    (void)hipMalloc(&out, 4);
    (void)hipMalloc(&bad, 4);
    (void)hipMemcpy(buf, h.data(), nbytes, hipMemcpyHostToDevice);
    for (int p = 0; p < 3; ++p) {
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipMemset(bad, 0, 4);
            k_gather<<<2048, 256>>>(buf, nbytes, p, out, bad);
            (void)hipDeviceSynchronize();
            unsigned nb = 0;
            (void)hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost);
            if (rep == 2) printf("pattern %d: mismatched words %u\n", p, nb);
        }
    }
    return 0;
}
