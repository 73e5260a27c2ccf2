// Calibration of the L2 memory-side read counters (FETCH_SIZE,
// TCC_EA0_RDREQ*) for dword gathers on gfx950 (VERDICT r4 #3,
// MI355X_MICROARCH.md §HBM: "other access widths are uncalibrated").
//
// Every pattern reads a 2 GiB buffer (8x the 256 MiB Infinity Cache, so the
// lines come from HBM) with a known number of distinct 128-B lines touched:
//   0  dwordx4 per lane, coalesced, every byte once (the guide's calibrated form)
//   1  dword per lane, coalesced, every byte once
//   2  one dword per 128-B line (lane i -> line i of the wave's 8 KiB window): every line once
//   3  one dword per 64-B half line: every half line once (two lanes per line)
//   4  one dword per 32-B sector: every sector once (four lanes per line)
//   5  k_sweep-like: one u8-quad record (dword) per lane at a random line of
//      the buffer, 1/8 of the lines (hash-scattered, lines distinct per wave)
// Run under rocprofv3 --pmc (tools/microbench/run_fetch_cal.sh). Each pattern
// is dispatched 3 times (the summary uses the last two).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr size_t kBytes = size_t(2) << 30;      // 2 GiB
constexpr size_t kDwords = kBytes / 4;
constexpr size_t kLines = kBytes / 128;

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

// one thread = one load; grid sized per pattern so the whole footprint is read once
__global__ __launch_bounds__(256) void k_cal(const unsigned *buf, int pat, unsigned *out) {
    const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
    unsigned v = 0;
    if (pat == 0) {
        const uint4 q = reinterpret_cast<const uint4 *>(buf)[t];
        v = q.x ^ q.y ^ q.z ^ q.w;
    } else if (pat == 1) {
        v = buf[t];
    } else if (pat == 2) {
        v = buf[t * 32];          // 128 B apart
    } else if (pat == 3) {
        v = buf[t * 16];          // 64 B apart
    } else if (pat == 4) {
        v = buf[t * 8];           // 32 B apart
    } else {
        // pattern 5: kLines/8 loads, each at a distinct pseudo-random line
        // (a bijection of the line index: odd multiplier mod 2^24 lines)
        const uint32_t line = (uint32_t)((t * 2654435761ull + 12345u) & (kLines - 1));
        v = buf[(size_t)line * 32 + (hash32((uint32_t)t) & 31)];
    }
    if (v == 0x9e3779b9u) out[0] = v;  // keeps the loads; the buffer never holds this value
}

int main() {
    unsigned *buf, *out;
    if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    (void)hipMemset(buf, 1, kBytes);
    (void)hipDeviceSynchronize();
    const size_t threads[6] = {kBytes / 16, kDwords, kLines, kBytes / 64, kBytes / 32, kLines / 8};
    const double lines_touched[6] = {(double)kLines, (double)kLines, (double)kLines, (double)kLines,
                                     (double)kLines, (double)(kLines / 8)};
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int p = 0; p < 6; ++p) {
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipEventRecord(a);
            k_cal<<<dim3((unsigned)(threads[p] / 256)), dim3(256)>>>(buf, p, out);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            if (rep == 2)
                printf("{\"pattern\": %d, \"loads\": %zu, \"lines_touched\": %.0f, \"line_bytes\": %.0f, \"ms\": %.3f, "
                       "\"line_GBps\": %.1f}\n",
                       p, threads[p], lines_touched[p], lines_touched[p] * 128, ms,
                       lines_touched[p] * 128 / (ms * 1e-3) / 1e9);
        }
    }
    (void)hipFree(buf);
    (void)hipFree(out);
    return 0;
}
