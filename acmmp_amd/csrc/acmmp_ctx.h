// acmmp_ctx.h — the engine object behind the opaque `acmmp_ctx *` of
// include/acmmp.h, shared by the translation units of libacmmp_amd.so
// (acmmp_engine.hip: PatchMatch runs; acmmp_planar.hip: planar-prior
// construction). Not installed, not part of the C-ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/acmmp.h"
#include "acmmp_internal.h"

using namespace acmmp;

// acmmp_texture_create: one view's padded footprint records (KViews::pad),
// built once and borrowed by any engine on the device (~ a CUDA texture
// object, src/ACMMP.cpp:640-662). The image itself stays the caller's.
struct acmmp_texture {
    int device = 0;
    const float *img = nullptr;  // borrowed, row pitch img_pitch floats
    int img_pitch = 0;
    int W = 0, H = 0;
    int form = 0;                // kTexelF32 / kTexelU8 / kTexelH16
    float *pad = nullptr;        // owned
    size_t pad_bytes = 0;        // bytes allocated at pad
    int pad_pitch = 0;           // records per row
};

struct acmmp_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    acmmp_params prm{};
    std::string err;

    int n = 0;
    int W = 0, H = 0, Wh = 0;
    acmmp_camera cams[ACMMP_MAX_IMAGES]{};

    // device buffers: images / depth maps are either owned (uploaded from the
    // host, pitched) or borrowed (caller's device pointers, zero copy)
    std::vector<float *> own_img, own_dep;
    std::vector<const float *> img, dep;
    std::vector<int> img_pitch;
    std::vector<float *> pad;          // padded source images (KViews::pad), owned
    std::vector<const float *> pad_use;  // what KViews::pad points at: pad[i] or a texture's records
    std::vector<size_t> pad_bytes;
    std::vector<int> pad_pitch;
    int pad_texel = 0;                 // form of pad[] (KViews::texel, kTexel*)
    uint32_t *d_not_u8 = nullptr;      // device flag: a view does not fit the compact form
    std::vector<int> dep_pitch, dep_w, dep_h;
    bool have_depths = false;

    float4 *d_cplane[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};  // [colour][pingpong]
    float *d_ccost[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
    uint32_t *d_csv[2] = {nullptr, nullptr};
    int cur[2] = {0, 0};
    float4 *d_rm_plane = nullptr;
    float *d_rm_cost = nullptr;
    // depth channel of d_rm_plane as its own plane (written by k_finalize and
    // the filters: the filters read 4 B per neighbour instead of a float4, and
    // the depth export is a plain copy); depth_ok: it matches d_rm_plane's .w
    // (set by a full run, cleared by every other writer of d_rm_plane)
    float *d_rm_depth = nullptr;
    bool depth_ok = false;
    uint32_t *d_rm_sv = nullptr;
    float *d_pre_cost = nullptr;
    float4 *d_prior = nullptr;
    uint32_t *d_mask = nullptr;
    float4 *d_scaled = nullptr;
    size_t scaled_count = 0;
    float4 *d_seed = nullptr;
    bool have_prior = false, have_scaled = false, have_seed = false, have_state = false;

    // Per-run constant block. A ring of pinned host / device slots so an
    // asynchronous run never has its constants overwritten by the next
    // enqueue: slot k is refilled only after its previous copy completed
    // (event), and the device copy is stream-ordered behind the kernels that
    // read it.
    static constexpr int kSlots = 4;
    KViews *d_kv_ring[kSlots] = {};
    KViews *h_kv_ring[kSlots] = {};
    hipEvent_t kv_ev[kSlots] = {};
    bool kv_used[kSlots] = {};
    int kv_slot = 0;
    KViews *d_kv = nullptr;  // slot of the current enqueue
    KViews h_kv{};

    bool timing = false;
    acmmp_timing last_timing{};
    hipEvent_t ev[8] = {};
    bool events_made = false;

    // acmmp_wait_stream: recorded on a producer stream, waited on by `stream`
    hipEvent_t wait_ev = nullptr;
};

namespace acmmp {


inline int set_err(acmmp_ctx *ctx, int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (ctx) ctx->err = buf;
    return code;
}

#define HIP_TRY(ctx, expr)                                                                   \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return set_err(ctx, ACMMP_ERR_HIP, "%s failed: %s (%s:%d)", #expr,               \
                           hipGetErrorString(e_), __FILE__, __LINE__);                       \
    } while (0)

// Device blocks (acmmp_engine.hip). hipFree synchronises the whole device —
// with two engines in flight it waits for the other one's kernels — and
// costs about a millisecond per block, so blocks freed where their engine's
// stream has just been synchronised (dfree_synced; every free of
// acmmp_destroy) go to a per-(device, size) cache that later allocations of
// the same size take from. ACMMP_DEVICE_POOL_MB caps it (default 8192; 0
// turns it off). Any other free goes to hipFree, as before.
hipError_t dev_alloc(void **p, size_t bytes);
void dev_free(void *p, bool synced);
extern thread_local bool g_frees_synced;  // set by acmmp_destroy after its stream sync

template <typename T>
inline void dfree(T *&p) {
    if (p) dev_free((void *)p, g_frees_synced);
    p = nullptr;
}

// for a block no queued work can still touch (its stream just synchronised)
template <typename T>
inline void dfree_synced(T *&p) {
    if (p) dev_free((void *)p, true);
    p = nullptr;
}

template <typename T>
inline hipError_t dalloc(T *&p, size_t count) {
    dfree(p);
    return dev_alloc((void **)&p, count * sizeof(T) > 0 ? count * sizeof(T) : 4);
}

inline int pitch_of(int w) { return (w + 63) / 64 * 64; }

inline int check_ready(acmmp_ctx *ctx) {
    if (!ctx) return ACMMP_ERR_ARG;
    if (ctx->n < 2) return set_err(ctx, ACMMP_ERR_STATE, "no images set (acmmp_set_images)");
    return ACMMP_OK;
}

// Builds the KViews constant block for the next enqueue (acmmp_engine.hip).
int upload_kv(acmmp_ctx *ctx);
KState make_state(acmmp_ctx *ctx);

}  // namespace acmmp
