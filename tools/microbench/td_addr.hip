// Addressing form vs TA/TD/TCP cost of the same dword gathers on gfx950
// (is k_sweep's ~44 TD cycles per gather a per-line or a
// per-lane cost of the idxen form?). Every wave issues ITERS x UNROLL dword
// loads per lane at the SAME byte addresses in each form:
//   form 0  struct buffer load, idxen (record index, stride 4 in the SRD) — what fetch_row issues
//   form 1  raw buffer load, offen (byte offset in a VGPR)
//   form 2  flat_load_dword, 64-bit per-lane generic address
//   form 3  global_load_dword, uniform base (saddr) + 32-bit lane byte offset
//   form 4  global_load_dword, 64-bit per-lane address (vaddr, "off")
// over three lane->address shapes:
//   shape 0  coalesced: 64 consecutive records (256 B)
//   shape 1  pattern 2 of td_gather.hip: 16 colour-split columns x 4 rows (k_sweep 16x4 wave)
//   shape 2  pattern 17: 8 colour-split columns x 8 rows (k_sweep's 8x8 wave), linear rows
//   shape 3  pattern 17 with every lane's record replaced by its 8-B-aligned pair start
//            (2 lanes per 8 B: how many distinct 8-B words, not lanes, cost)
// Run under rocprofv3 (tools/microbench/run_addr.sh): TD_TD_BUSY_sum,
// TA_TA_BUSY_sum, TCP_TOTAL_CACHE_ACCESSES_sum, TCP_TCP_TA_DATA_STALL_CYCLES_sum
// per wave-instruction, dispatches in (shape, form) order, 3 reps each.
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ unsigned sbl32(__amdgpu_buffer_rsrc_t r, int vindex, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.struct.ptr.buffer.load.i32");
__device__ unsigned rbl32(__amdgpu_buffer_rsrc_t r, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.ptr.buffer.load.i32");

constexpr int ITERS = 64, UNROLL = 8;
constexpr int PITCH = 1632;  // records per row (cfg2 u8-quad pitch)

__device__ int lane_record(int shape, int lane, int wave) {
    const int base = (wave % 64) * 8 * PITCH + 64;
    switch (shape) {
        case 0: return base + lane;
        case 1: return base + (lane >> 4) * PITCH + 2 * (lane & 15);
        case 2: {
            const int cc = lane & 7, rr = lane >> 3;
            return (wave % 64) * 8 * PITCH + rr * PITCH + 64 + 2 * cc + (rr & 1) + (wave % 13);
        }
        default: {
            const int cc = lane & 7, rr = lane >> 3;
            return ((wave % 64) * 8 * PITCH + rr * PITCH + 64 + 2 * cc + (rr & 1) + (wave % 13)) & ~1;
        }
    }
}

// record offset of load u of iteration it (uniform): the 36-sample walk of
// a patch (2 columns, 2 rows apart), as td_gather.hip
__device__ int walk(int shape, int it, int u) {
    const int s = (it * UNROLL + u) & 31;
    return shape == 0 ? 64 * (s & 7) : (s % 6) * 2 + (s / 6) * 2 * PITCH;
}

template <int FORM>
__global__ __launch_bounds__(256) void k_addr(const unsigned *buf, int nrec, int shape, unsigned *out) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)buf, (short)4, nrec, 0x00020000);
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc((void *)buf, (short)0, nrec * 4, 0x00020000);
    const int lane = threadIdx.x & 63, wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int rec0 = lane_record(shape, lane, wave);
    unsigned acc[UNROLL] = {};
#pragma unroll 1
    for (int it = 0; it < ITERS; ++it) {
        unsigned v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            int rec = rec0 + walk(shape, it, u);
            asm volatile("" : "+v"(rec));  // a per-lane VGPR address, as in k_sweep
            if (FORM == 0) {
                v[u] = sbl32(rs, rec, 0, 0, 0);
            } else if (FORM == 1) {
                v[u] = rbl32(rr, rec * 4, 0, 0);
            } else if (FORM == 2) {
                const unsigned *p = buf + rec;
                asm volatile("" : "+v"(p));  // generic pointer in VGPRs: flat_load_dword
                v[u] = *p;
            } else if (FORM == 3) {
                const unsigned off = (unsigned)rec * 4u;  // zero-extended 32-bit byte offset: saddr form
                v[u] = *(const __attribute__((address_space(1))) unsigned *)((
                    const __attribute__((address_space(1))) char *)buf + off);
            } else {
                const __attribute__((address_space(1))) unsigned *p =
                    (const __attribute__((address_space(1))) unsigned *)buf + rec;
                asm volatile("" : "+v"(p));  // 64-bit VGPR address: global_load_dword v, v[a:b], off
                v[u] = *p;
            }
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
    const int nrec = PITCH * 640;
    unsigned *buf, *out;
    (void)hipMalloc(&buf, (size_t)nrec * 4);
    (void)hipMalloc(&out, 4);
    (void)hipMemset(buf, 1, (size_t)nrec * 4);
    const int blocks = 4096;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const char *fname[5] = {"idxen", "offen", "flat", "global-saddr", "global-vaddr"};
    for (int shape = 0; shape < 4; ++shape) {
        for (int form = 0; form < 5; ++form) {
            for (int rep = 0; rep < 3; ++rep) {
                (void)hipEventRecord(a);
                if (form == 0) k_addr<0><<<blocks, 256>>>(buf, nrec, shape, out);
                if (form == 1) k_addr<1><<<blocks, 256>>>(buf, nrec, shape, out);
                if (form == 2) k_addr<2><<<blocks, 256>>>(buf, nrec, shape, out);
                if (form == 3) k_addr<3><<<blocks, 256>>>(buf, nrec, shape, out);
                if (form == 4) k_addr<4><<<blocks, 256>>>(buf, nrec, shape, out);
                (void)hipEventRecord(b);
                (void)hipEventSynchronize(b);
                float ms = 0;
                (void)hipEventElapsedTime(&ms, a, b);
                if (rep == 2) {
                    const double insts = (double)blocks * 4 * ITERS * UNROLL;
                    printf("shape %d form %-12s: %.3f ms, %.2f G wave-inst/s, %.2f ns per inst per CU\n", shape,
                           fname[form], ms, insts / (ms * 1e-3) / 1e9, ms * 1e6 / (insts / 256));
                }
            }
        }
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    return 0;
}
