// Which lanes share one TCP (L1) cache access of a gather on gfx950? Every
// pattern places the 64 lanes of a wave on distinct dwords and differs only
// in how lanes share 64-B lines and 16-B chunks (index-addressed dword
// buffer loads, cache resident, the same per-iteration walk for all lanes).
// Run under rocprofv3 with TCP_TOTAL_CACHE_ACCESSES_sum, TD_TD_BUSY_sum and
// TA_BUFFER_READ_WAVEFRONTS_sum (tools/microbench/run_rule.sh): accesses and
// TD cycles per wave-instruction per pattern tell the coalescing rule.
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ unsigned sbl32(__amdgpu_buffer_rsrc_t r, int vindex, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.struct.ptr.buffer.load.i32");

constexpr int ITERS = 64, UNROLL = 8, NPAT = 16;

__device__ constexpr int kShare[8] = {0, 0, 2, 4, 6, 6, 8, 10};

// record (dword) of lane i; patterns documented in kName
__device__ int lane_record(int pat, int i) {
    switch (pat) {
        case 0: return i;                                 // 64 consecutive dwords: 4 lines
        case 1: return 16 * i;                            // one line per lane: 64 lines
        case 2: return 2 * i;                             // stride 8 B: 8 lines, 2 lanes per 16 B
        case 3: return 4 * i;                             // stride 16 B: 16 lines, 1 lane per 16 B
        case 4: return (i & 3) * 2 + (i >> 2) * 16;       // each quad alone in a line (8 B stride): 16 lines
        case 5: return (i & 1) * 2 + (i >> 1) * 16;       // each lane pair alone in a line: 32 lines
        case 6: return (i & 15) * 16 + (i >> 4) * 2;      // lanes i, i+16, i+32, i+48 share a line: 16 lines
        case 7: return (i & 3) * 16 + (i >> 2) * 2;       // lanes 4 apart... : line = i & 3 -> 4 lines of 16 lanes
        case 8: return (i & 7) * 2 + (i >> 3) * 16;       // 8 lanes per line (stride 8 B): 8 lines
        case 9: return (i & 15) + (i >> 4) * 16 * 8;      // 16 lanes per line, lines 512 B apart: 4 lines
        case 10: return (i & 1) + (i >> 1) * 4;           // lane pairs on adjacent dwords, pairs 16 B apart
        case 11: return (i & 31) * 16 + (i >> 5);         // lanes i, i+32 share a line: 32 lines
        // (round 5) the 8 lanes of each (quarter, parity) group on ONE pixel's
        // patch row (the shared-plane bound of DESIGN.md §5): dwords
        // {0,0,2,4,6,6,8,10} of a 512-B-apart window per group
        case 12: return ((i >> 4) * 2 + (i & 1)) * 128 + kShare[(i >> 1) & 7];       // span 0..40 B: one line
        case 13: return ((i >> 4) * 2 + (i & 1)) * 128 + 10 + kShare[(i >> 1) & 7];  // 40..84 B: two lines
        case 14: return ((i >> 4) * 2 + (i & 1)) * 128;                               // group on one dword
        default: return ((i >> 4) * 2 + (i & 1)) * 128 + ((i >> 1) & 7);             // group on 8 consecutive dwords
    }
}

__global__ __launch_bounds__(256) void k_rule(const unsigned *buf, int nrec, int pat, unsigned *out) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)buf, (short)4, nrec, 0x00020000);
    const int lane = threadIdx.x & 63, wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int rec0 = (wave % 256) * 2048 + lane_record(pat, lane);  // 64-B aligned wave base
    unsigned acc[UNROLL] = {};
#pragma unroll 1
    for (int it = 0; it < ITERS; ++it) {
        unsigned v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            int rec = rec0 + ((it * UNROLL + u) & 7) * 1024;  // uniform walk over 8 line-aligned windows
            asm volatile("" : "+v"(rec));
            v[u] = sbl32(rs, rec, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc[u] += v[u];
    }
    unsigned a = 0;
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) a ^= acc[u];
    if (a == 0x12345678u) out[0] = a;
}

int main() {
    const int nrec = 256 * 2048 + 8 * 1024 + 1024;
    unsigned *buf, *out;
    (void)hipMalloc(&buf, (size_t)nrec * 4);
    (void)hipMalloc(&out, 4);
    (void)hipMemset(buf, 1, (size_t)nrec * 4);
    const int blocks = 4096;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int p = 0; p < NPAT; ++p) {
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipEventRecord(a);
            k_rule<<<blocks, 256>>>(buf, nrec, p, out);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            if (rep == 2) {
                const double insts = (double)blocks * 4 * ITERS * UNROLL;
                printf("pattern %2d: %.3f ms, %.2f ns per inst per CU\n", p, ms, ms * 1e6 / (insts / 256));
            }
        }
    }
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
