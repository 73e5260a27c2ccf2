// TD/TA cost of index-addressed (idxen) dword buffer loads by access pattern
// on gfx950: the texture-data path that bounds k_sweep. Every
// wave issues ITERS buffer_load_dword idxen per lane with a pattern-defined
// record index into a 4-B-record buffer that stays cache resident, and sums
// the loaded words (kept live through one store). Run under
//   rocprofv3 --kernel-trace --pmc TD_TD_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE
// and compare TD busy cycles per wave-instruction per pattern.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ unsigned sbl32(__amdgpu_buffer_rsrc_t r, int vindex, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.struct.ptr.buffer.load.i32");

constexpr int ITERS = 512;
constexpr int PITCH = 1632;  // records per row (cfg2 u8-quad pitch)

__global__ __launch_bounds__(256) void k_gather(const unsigned *buf, int nrec, int pattern, unsigned *out) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)buf, (short)4, nrec, 0x00020000);
    const int lane = threadIdx.x & 63, wave = (blockIdx.x * 4 + (threadIdx.x >> 6));
    const int c = lane & 15, r = lane >> 4;
    unsigned h = (unsigned)(wave * 2654435761u) ^ (unsigned)lane * 40503u;
    int base = (wave % 64) * 8 * PITCH + 64;
    unsigned acc = 0;
#pragma unroll 1
    for (int it = 0; it < ITERS; ++it) {
        int idx;
        const int s = it & 31;  // 36-sample-like walk: offsets change per iteration
        switch (pattern) {
            case 0: idx = base + lane + 64 * (s & 7); break;                            // coalesced 256 B
            case 1: idx = base + 2 * lane + (s & 7); break;                             // stride 2, one row
            case 2: idx = base + r * PITCH + 2 * c + (s % 6) * 2 + (s / 6) * 2 * PITCH; break;  // k_sweep wave: 16 cols x 4 rows
            case 3: {                                                                  // same + per-lane jitter
                h = h * 1664525u + 1013904223u;
                idx = base + r * PITCH + 2 * c + (s % 6) * 2 + (s / 6) * 2 * PITCH + (int)((h >> 28) & 3) - 1;
            } break;
            case 4: h = h * 1664525u + 1013904223u; idx = (int)(h % (unsigned)nrec); break;  // random
            case 5: idx = base + (s & 7); break;                                        // broadcast
            case 6: idx = base + r * PITCH * 2 + 2 * c + (s % 6) * 2; break;            // rows 2 apart
            case 8: case 9: case 10: case 11:                                          // k_sweep shape, 1/4 / 1/16 / 1 lane / 1/2 active
                idx = base + r * PITCH + 2 * c + (s % 6) * 2 + (s / 6) * 2 * PITCH; break;
            case 12: h = h * 1664525u + 1013904223u; idx = (int)(h % (unsigned)nrec); break;  // random, 1/4 active
            case 13: idx = base + (lane >> 1) + 64 * (s & 7); break;                   // lane pairs share a record
            case 14: idx = base + (lane >> 2) + 64 * (s & 7); break;                   // lane quads share a record
            case 15: idx = base + 3 * lane + (s & 7); break;                            // stride 3 (12 B)
            case 16: idx = base + 8 * lane + (s & 7); break;                            // stride 8 (32 B): 4 lanes/line
            case 17: case 18: case 19: case 20: {  // k_sweep 8x8 colour-split wave: 16 px x 8 rows,
                // in a linear (17), 16x2 (18), 8x4 (19) or 4x8 (20) record-tiled layout (128-B lines)
                const int cc = lane & 7, rr = lane >> 3;
                const int x = 64 + 2 * cc + (rr & 1) + (s % 6) * 2 + (wave % 13), y = (wave % 64) * 8 + rr + (s / 6) * 2;
                const int tw = pattern == 17 ? 32 : pattern == 18 ? 16 : pattern == 19 ? 8 : 4, th = 32 / tw;
                idx = ((y / th) * (PITCH / tw) + x / tw) * 32 + (y % th) * tw + (x % tw);
            } break;
            case 21: case 22: case 23: case 24: case 25: {  // pattern 17 with the row pitch 1632 +
                // 1, 4, 8, 16, 24 records (rows no longer all start at the same offset in a 128-B line)
                const int cc = lane & 7, rr = lane >> 3;
                const int x = 64 + 2 * cc + (rr & 1) + (s % 6) * 2 + (wave % 13), y = (wave % 64) * 8 + rr + (s / 6) * 2;
                const int d = pattern == 21 ? 1 : pattern == 22 ? 4 : pattern == 23 ? 8 : pattern == 24 ? 16 : 24;
                idx = y * (PITCH + d) + x;
            } break;
            default: idx = base + lane * 33; break;                                     // one line per lane
        }
        const bool on = pattern == 8 || pattern == 12 ? (lane & 3) == 0
                        : pattern == 9                ? (lane & 15) == 0
                        : pattern == 10               ? lane == 0
                        : pattern == 11               ? (lane & 1) == 0
                                                      : true;
        if (on) acc += sbl32(rs, idx, 0, 0, 0);
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char **argv) {
    const int nrec = PITCH * 640;
    unsigned *buf, *out;
    (void)hipMalloc(&buf, (size_t)nrec * 4);
    (void)hipMalloc(&out, 4);
    (void)hipMemset(buf, 1, (size_t)nrec * 4);
    const int blocks = 2048;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int p = 0; p < 26; ++p) {
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipEventRecord(a);
            k_gather<<<blocks, 256>>>(buf, nrec, p, out);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            if (rep == 2) {
                const double insts = (double)blocks * 4 * ITERS;
                printf("pattern %d: %.3f ms, %.2f G wave-inst/s, %.1f ns per inst per CU\n", p, ms,
                       insts / (ms * 1e-3) / 1e9, ms * 1e6 / (insts / 256));
            }
        }
    }
    return 0;
}
