// acmmp_engine.hip — host side of libacmmp_amd.so: the C-ABI declared in
// include/acmmp.h. Replaces the CUDA host code of the reference's ACMMP class
// (src/ACMMP.cpp:107-152, :638-831, src/ACMMP.cu:1378-1456) with an engine
// that owns one HIP stream, keeps all per-view state resident in HBM, enqueues
// the whole RunPatchMatch without host synchronisation between kernels, and
// reports failures as status codes instead of exit().
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "acmmp_ctx.h"
#include "../../include/acmmp_detmath.h"


thread_local bool acmmp::g_frees_synced = false;

namespace {

// the device-block cache of dev_alloc / dev_free (acmmp_ctx.h)
struct DevPool {
    std::mutex mu;
    std::unordered_map<void *, size_t> size_of;                    // every live dev_alloc block
    std::map<std::pair<int, size_t>, std::vector<void *>> free_;  // (device, bytes) -> cached blocks
    size_t cached = 0, cap = 0;
    DevPool() {
        const char *e = std::getenv("ACMMP_DEVICE_POOL_MB");
        const long long mb = e ? std::atoll(e) : 8192;
        cap = (size_t)std::max(0LL, mb) << 20;  // a negative setting means off, not a huge cap
    }
    // hipFree of every cached block of device dev (all devices: dev < 0);
    // caller holds mu. Returns the bytes given back.
    size_t release(int dev) {
        size_t n = 0;
        for (auto it = free_.begin(); it != free_.end();) {
            if (dev >= 0 && it->first.first != dev) {
                ++it;
                continue;
            }
            for (void *p : it->second) {
                (void)hipFree(p);
                n += it->first.second;
            }
            it = free_.erase(it);
        }
        cached -= n;
        return n;
    }
    size_t bytes(int dev) const {
        size_t n = 0;
        for (const auto &kv : free_)
            if (dev < 0 || kv.first.first == dev) n += kv.first.second * kv.second.size();
        return n;
    }
};
DevPool &devpool() {
    static DevPool *p = new DevPool();  // never destroyed: blocks outlive static destruction order
    return *p;
}

// the engines' pinned KViews staging blocks, cached the same way (hipHostFree
// synchronises the device too); freed only by acmmp_destroy, after its sync
std::mutex g_pinned_mu;
std::vector<KViews *> g_pinned_kv;

hipError_t pinned_kv_alloc(KViews **p) {
    {
        std::lock_guard<std::mutex> g(g_pinned_mu);
        if (devpool().cap && !g_pinned_kv.empty()) {
            *p = g_pinned_kv.back();
            g_pinned_kv.pop_back();
            return hipSuccess;
        }
    }
    return hipHostMalloc((void **)p, sizeof(KViews), hipHostMallocDefault);
}

void pinned_kv_free(KViews *p) {
    {
        std::lock_guard<std::mutex> g(g_pinned_mu);
        if (devpool().cap && g_pinned_kv.size() < 64) {
            g_pinned_kv.push_back(p);
            return;
        }
    }
    (void)hipHostFree(p);
}

// An engine's stream and events, kept for the next engine on the device when
// it is destroyed (creating and destroying them costs a few milliseconds per
// ProcessProblem); only idle handles are kept: acmmp_destroy synchronises the
// stream first. Off with the block cache (ACMMP_DEVICE_POOL_MB=0).
struct HandlePool {
    std::mutex mu;
    std::map<int, std::vector<hipStream_t>> streams;
    std::map<std::pair<int, bool>, std::vector<hipEvent_t>> events;  // (device, timed)
};
HandlePool &handles() {
    static HandlePool *p = new HandlePool();
    return *p;
}

hipError_t stream_take(int dev, hipStream_t *s) {
    if (devpool().cap) {
        std::lock_guard<std::mutex> g(handles().mu);
        auto &v = handles().streams[dev];
        if (!v.empty()) {
            *s = v.back();
            v.pop_back();
            return hipSuccess;
        }
    }
    return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}

void stream_give(int dev, hipStream_t s) {
    if (devpool().cap) {
        std::lock_guard<std::mutex> g(handles().mu);
        auto &v = handles().streams[dev];
        if (v.size() < 16) {
            v.push_back(s);
            return;
        }
    }
    (void)hipStreamDestroy(s);
}

hipError_t event_take(int dev, bool timed, hipEvent_t *e) {
    if (devpool().cap) {
        std::lock_guard<std::mutex> g(handles().mu);
        auto &v = handles().events[{dev, timed}];
        if (!v.empty()) {
            *e = v.back();
            v.pop_back();
            return hipSuccess;
        }
    }
    return timed ? hipEventCreate(e) : hipEventCreateWithFlags(e, hipEventDisableTiming);
}

void event_give(int dev, bool timed, hipEvent_t e) {
    if (devpool().cap) {
        std::lock_guard<std::mutex> g(handles().mu);
        auto &v = handles().events[{dev, timed}];
        if (v.size() < 256) {
            v.push_back(e);
            return;
        }
    }
    (void)hipEventDestroy(e);
}

}  // namespace

hipError_t acmmp::dev_alloc(void **p, size_t bytes) {
    DevPool &pool = devpool();
    int dev = 0;
    (void)hipGetDevice(&dev);
    {
        std::lock_guard<std::mutex> g(pool.mu);
        auto it = pool.free_.find({dev, bytes});
        if (it != pool.free_.end() && !it->second.empty()) {
            *p = it->second.back();
            it->second.pop_back();
            pool.cached -= bytes;
            pool.size_of[*p] = bytes;
            return hipSuccess;
        }
    }
    hipError_t e = hipMalloc(p, bytes);
    if (e == hipErrorOutOfMemory) {
        // the cache may hold what the device lacks: give this device's
        // cached blocks back and try once more
        (void)hipGetLastError();
        size_t freed = 0;
        {
            std::lock_guard<std::mutex> g(pool.mu);
            freed = pool.release(dev);
        }
        if (freed) {
            e = hipMalloc(p, bytes);
            if (e != hipSuccess) (void)hipGetLastError();
        }
    }
    if (e == hipSuccess) {
        std::lock_guard<std::mutex> g(pool.mu);
        pool.size_of[*p] = bytes;
    }
    return e;
}

void acmmp::dev_free(void *p, bool synced) {
    DevPool &pool = devpool();
    {
        std::lock_guard<std::mutex> g(pool.mu);
        auto it = pool.size_of.find(p);
        const size_t bytes = it == pool.size_of.end() ? 0 : it->second;
        if (it != pool.size_of.end()) pool.size_of.erase(it);
        if (synced && bytes && pool.cached + bytes <= pool.cap) {
            hipPointerAttribute_t a;
            int dev = 0;
            if (hipPointerGetAttributes(&a, p) == hipSuccess) dev = a.device;
            pool.free_[{dev, bytes}].push_back(p);
            pool.cached += bytes;
            return;
        }
    }
    (void)hipFree(p);
}

namespace {

void free_depths(acmmp_ctx *ctx) {
    for (auto &p : ctx->own_dep) dfree(p);
    ctx->own_dep.clear();
    ctx->dep.clear();
    ctx->dep_pitch.clear();
    ctx->dep_w.clear();
    ctx->dep_h.clear();
    ctx->have_depths = false;
}

void free_images(acmmp_ctx *ctx) {
    for (auto &p : ctx->own_img) dfree(p);
    ctx->own_img.clear();
    ctx->img.clear();
    ctx->img_pitch.clear();
    free_depths(ctx);
}

void free_state(acmmp_ctx *ctx) {
    for (int c = 0; c < 2; ++c) {
        for (int b = 0; b < 2; ++b) {
            dfree(ctx->d_cplane[c][b]);
            dfree(ctx->d_ccost[c][b]);
        }
        dfree(ctx->d_csv[c]);
    }
    dfree(ctx->d_rm_plane);
    dfree(ctx->d_rm_cost);
    dfree(ctx->d_rm_depth);
    ctx->depth_ok = false;
    dfree(ctx->d_rm_sv);
    dfree(ctx->d_pre_cost);
    dfree(ctx->d_prior);
    dfree(ctx->d_mask);
    dfree(ctx->d_scaled);
    dfree(ctx->d_seed);
    ctx->have_prior = ctx->have_scaled = ctx->have_seed = ctx->have_state = false;
}

// Camera-only part of ComputeHomography (src/ACMMP.cu:264-290), evaluated in
// the same IEEE order as the reference (this TU builds with -ffp-contract=off).
ViewRel view_rel(const acmmp_camera &rc, const acmmp_camera &sc) {
    float ref_C[3], src_C[3];
    ref_C[0] = -(rc.R[0] * rc.t[0] + rc.R[3] * rc.t[1] + rc.R[6] * rc.t[2]);
    ref_C[1] = -(rc.R[1] * rc.t[0] + rc.R[4] * rc.t[1] + rc.R[7] * rc.t[2]);
    ref_C[2] = -(rc.R[2] * rc.t[0] + rc.R[5] * rc.t[1] + rc.R[8] * rc.t[2]);
    src_C[0] = -(sc.R[0] * sc.t[0] + sc.R[3] * sc.t[1] + sc.R[6] * sc.t[2]);
    src_C[1] = -(sc.R[1] * sc.t[0] + sc.R[4] * sc.t[1] + sc.R[7] * sc.t[2]);
    src_C[2] = -(sc.R[2] * sc.t[0] + sc.R[5] * sc.t[1] + sc.R[8] * sc.t[2]);
    ViewRel r;
    r.Rr[0] = sc.R[0] * rc.R[0] + sc.R[1] * rc.R[1] + sc.R[2] * rc.R[2];
    r.Rr[1] = sc.R[0] * rc.R[3] + sc.R[1] * rc.R[4] + sc.R[2] * rc.R[5];
    r.Rr[2] = sc.R[0] * rc.R[6] + sc.R[1] * rc.R[7] + sc.R[2] * rc.R[8];
    r.Rr[3] = sc.R[3] * rc.R[0] + sc.R[4] * rc.R[1] + sc.R[5] * rc.R[2];
    r.Rr[4] = sc.R[3] * rc.R[3] + sc.R[4] * rc.R[4] + sc.R[5] * rc.R[5];
    r.Rr[5] = sc.R[3] * rc.R[6] + sc.R[4] * rc.R[7] + sc.R[5] * rc.R[8];
    r.Rr[6] = sc.R[6] * rc.R[0] + sc.R[7] * rc.R[1] + sc.R[8] * rc.R[2];
    r.Rr[7] = sc.R[6] * rc.R[3] + sc.R[7] * rc.R[4] + sc.R[8] * rc.R[5];
    r.Rr[8] = sc.R[6] * rc.R[6] + sc.R[7] * rc.R[7] + sc.R[8] * rc.R[8];
    float Cr[3];
    Cr[0] = (ref_C[0] - src_C[0]);
    Cr[1] = (ref_C[1] - src_C[1]);
    Cr[2] = (ref_C[2] - src_C[2]);
    r.tr[0] = sc.R[0] * Cr[0] + sc.R[1] * Cr[1] + sc.R[2] * Cr[2];
    r.tr[1] = sc.R[3] * Cr[0] + sc.R[4] * Cr[1] + sc.R[5] * Cr[2];
    r.tr[2] = sc.R[6] * Cr[0] + sc.R[7] * Cr[1] + sc.R[8] * Cr[2];
    return r;
}

// Rebuilds the device-side constant block from the context.
int kv_upload(acmmp_ctx *ctx) {
    KViews &kv = ctx->h_kv;
    kv.prm = ctx->prm;
    for (int i = 0; i < ctx->n; ++i) {
        kv.cam[i] = ctx->cams[i];
        kv.img[i] = ctx->img[i];
        kv.ipitch[i] = ctx->img_pitch[i];
        kv.pad[i] = ctx->pad_use[i];
        kv.ppitch[i] = ctx->pad_pitch[i];
        if (i > 0) kv.rel[i] = view_rel(ctx->cams[0], ctx->cams[i]);
        {
            const acmmp_camera &c = ctx->cams[i];
            for (int k = 0; k < 3; ++k) kv.cw[i][k] = -(c.R[k] * c.t[0] + c.R[3 + k] * c.t[1] + c.R[6 + k] * c.t[2]);
        }
        if (ctx->have_depths) {
            kv.dep[i] = ctx->dep[i];
            kv.dpitch[i] = ctx->dep_pitch[i];
            kv.dw[i] = ctx->dep_w[i];
            kv.dh[i] = ctx->dep_h[i];
        } else {
            kv.dep[i] = nullptr;
            kv.dpitch[i] = kv.dw[i] = kv.dh[i] = 0;
        }
    }
    kv.W = ctx->W;
    kv.H = ctx->H;
    kv.Wh = ctx->Wh;
    kv.sweep_rows = checkerboard_rows(ctx->H);
    kv.nsrc = ctx->n - 1;
    // fp32 record indices are exact below 2^24 records (about 4090 x 4090);
    // larger views (ETH3D high-res at native size) take the integer form.
    // ACMMP_WIDE_INDEX=1 forces it (parity tests of that path at small sizes).
    kv.wide = 0;
    for (int i = 1; i < ctx->n; ++i)
        if ((size_t)ctx->pad_pitch[i] * (ctx->cams[i].height + 2) >= (1u << 24)) kv.wide = 1;
    if (const char *e = std::getenv("ACMMP_WIDE_INDEX"))
        if (e[0] == '1') kv.wide = 1;
    kv.texel = ctx->pad_texel;
    if (kv.texel == kTexelU8) {  // bilateral weights of the 256 colour differences (KViews::wlut)
        const float ss = kv.prm.sigma_spatial, sc = kv.prm.sigma_color;
        for (int a = 0; a < 3; ++a)
            for (int b = a; b < 3; ++b) {
                const float xd = (float)(2 * a + 1), yd = (float)(2 * b + 1);
                const float spatial = dm_sqrt(xd * xd + yd * yd);
                for (int d = 0; d < 256; ++d) {
                    const float color = (float)d;
                    kv.wlut[wlut_class(a, b)][d] = dm_expf(-spatial / (2.0f * ss * ss) - color / (2.0f * sc * sc));
                }
            }
    }
    kv.inv_k0 = 1.0f / ctx->cams[0].K[0];
    kv.inv_k4 = 1.0f / ctx->cams[0].K[4];
    kv.pert_pi = (float)((double)0.02f * M_PI);            // src/ACMMP.cu:737
    kv.pert3_pi = (float)((double)(3 * 0.02f) * M_PI);     // src/ACMMP.cu:649
    kv.angle_sigma = (float)(M_PI * (double)(5.0f / 180.0f));  // src/ACMMP.cu:715
    const int k = ctx->kv_slot;
    ctx->kv_slot = (k + 1) % acmmp_ctx::kSlots;
    if (!ctx->d_kv_ring[k]) {
        HIP_TRY(ctx, dalloc(ctx->d_kv_ring[k], 1));
        HIP_TRY(ctx, pinned_kv_alloc(&ctx->h_kv_ring[k]));
        HIP_TRY(ctx, event_take(ctx->device, false, &ctx->kv_ev[k]));
    }
    if (ctx->kv_used[k]) HIP_TRY(ctx, hipEventSynchronize(ctx->kv_ev[k]));
    std::memcpy(ctx->h_kv_ring[k], &kv, sizeof(KViews));
    HIP_TRY(ctx, hipMemcpyAsync(ctx->d_kv_ring[k], ctx->h_kv_ring[k], sizeof(KViews), hipMemcpyHostToDevice,
                                ctx->stream));
    HIP_TRY(ctx, hipEventRecord(ctx->kv_ev[k], ctx->stream));
    ctx->kv_used[k] = true;
    ctx->d_kv = ctx->d_kv_ring[k];
    return ACMMP_OK;
}

// y0, y1: the image rows a launch covers (all rows by default)
KState state_of(acmmp_ctx *ctx, int y0 = 0, int y1 = -1) {
    KState st{};
    st.y0 = y0;
    st.y1 = y1 < 0 ? ctx->H : y1;
    for (int c = 0; c < 2; ++c) {
        st.plane[c] = ctx->d_cplane[c][ctx->cur[c]];
        st.cost[c] = ctx->d_ccost[c][ctx->cur[c]];
        st.plane_nx[c] = ctx->d_cplane[c][ctx->cur[c] ^ 1];
        st.cost_nx[c] = ctx->d_ccost[c][ctx->cur[c] ^ 1];
        st.sv[c] = ctx->d_csv[c];
    }
    st.rm_plane = ctx->d_rm_plane;
    st.rm_cost = ctx->d_rm_cost;
    st.rm_depth = ctx->d_rm_depth;
    st.rm_sv = ctx->d_rm_sv;
    st.pre_cost = ctx->d_pre_cost;
    st.prior = ctx->d_prior;
    st.mask = ctx->d_mask;
    st.scaled = ctx->d_scaled;
    st.seed = ctx->d_seed;
    return st;
}


int upload_pitched(acmmp_ctx *ctx, float *&dst, int &pitch, const float *src, int w, int h, bool device_src) {
    pitch = pitch_of(w);
    HIP_TRY(ctx, dalloc(dst, (size_t)pitch * (size_t)h));
    HIP_TRY(ctx, hipMemsetAsync(dst, 0, (size_t)pitch * h * sizeof(float), ctx->stream));
    HIP_TRY(ctx, hipMemcpy2DAsync(dst, (size_t)pitch * sizeof(float), src, (size_t)w * sizeof(float),
                                  (size_t)w * sizeof(float), (size_t)h,
                                  device_src ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, ctx->stream));
    return ACMMP_OK;
}

int set_depths_impl(acmmp_ctx *ctx, const float *const *depths, const int32_t *pitches, bool borrow) {
    int rc = check_ready(ctx);
    if (rc) return rc;
    if (!depths) return set_err(ctx, ACMMP_ERR_ARG, "depths is NULL");
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));  // previous run may still read the old maps
    free_depths(ctx);
    ctx->own_dep.assign(ctx->n, nullptr);
    ctx->dep.assign(ctx->n, nullptr);
    ctx->dep_pitch.assign(ctx->n, 0);
    ctx->dep_w.assign(ctx->n, 0);
    ctx->dep_h.assign(ctx->n, 0);
    for (int i = 0; i < ctx->n; ++i) {
        if (!depths[i]) return set_err(ctx, ACMMP_ERR_ARG, "depth map %d is NULL", i);
        const int w = ctx->cams[i].width, h = ctx->cams[i].height;
        if (borrow) {
            ctx->dep[i] = depths[i];
            ctx->dep_pitch[i] = pitches ? pitches[i] : w;
            if (ctx->dep_pitch[i] < w) return set_err(ctx, ACMMP_ERR_ARG, "depth pitch %d < width %d", ctx->dep_pitch[i], w);
        } else {
            rc = upload_pitched(ctx, ctx->own_dep[i], ctx->dep_pitch[i], depths[i], w, h, false);
            if (rc) return rc;
            ctx->dep[i] = ctx->own_dep[i];
        }
        ctx->dep_w[i] = w;
        ctx->dep_h[i] = h;
    }
    ctx->have_depths = true;
    if (!borrow) HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return ACMMP_OK;
}

// Records per row and bytes of one view's padded footprint records in
// `form` (128-B rows: u8 quads W + 2, f16 quads W + 2, fp32 row pairs
// W + 3; sized for the fp32 form, the largest, so one allocation serves
// every form). Non-zero: too large.
int pad_geometry(int w, int h, int form, int &pp, size_t &bytes) {
    const int pf = (w + 3 + 15) / 16 * 16;
    pp = form == kTexelU8 ? (w + 2 + 31) / 32 * 32 : form == kTexelH16 ? (w + 2 + 15) / 16 * 16 : pf;
    const size_t rec = form == kTexelU8 ? 4 : 8;
    bytes = std::max((size_t)pf * (h + 2) * 2 * sizeof(float), (size_t)pp * (h + 2) * rec);
    // the gather kernels index records with a 24x24-bit multiply into a
    // signed 32-bit record index (kv_upload picks the fp32 form below 2^24)
    return ((size_t)pf * (h + 2) >= (1u << 31) || pf >= (1 << 24) || h + 2 >= (1 << 24)) ? 1 : 0;
}

hipError_t launch_pad_form(int form, const float *img, int pitch, int w, int h, float *pad, int pp,
                           uint32_t *d_unfit, hipStream_t s) {
    if (form == kTexelF32) return launch_pad_image(img, pitch, w, h, pad, pp, s);
    if (form == kTexelU8) return launch_pad_quad(img, pitch, w, h, reinterpret_cast<uint32_t *>(pad), pp, d_unfit, s);
    return launch_pad_h16(img, pitch, w, h, pad, pp, d_unfit, s);
}

// The compact forms to try before fp32, as ACMMP_TEXEL / ACMMP_TEXEL_F32 restrict them.
int texel_tries(int tries[2]) {
    tries[0] = kTexelU8;
    tries[1] = kTexelH16;
    int ntry = 2;
    if (const char *e = std::getenv("ACMMP_TEXEL")) {
        if (!std::strcmp(e, "f32")) ntry = 0;
        else if (!std::strcmp(e, "u8")) ntry = 1;
        else if (!std::strcmp(e, "h16")) { tries[0] = kTexelH16; ntry = 1; }
    }
    if (const char *e = std::getenv("ACMMP_TEXEL_F32"))
        if (e[0] == '1') ntry = 0;
    return ntry;
}

// Shared by acmmp_set_images / acmmp_set_images_device.
int set_images_impl(acmmp_ctx *ctx, int num_images, const acmmp_camera *cams, const float *const *images,
                    const int32_t *pitches, int keep_depth_range, bool borrow,
                    const acmmp_texture *const *tex = nullptr) {
    if (!ctx) return ACMMP_ERR_ARG;
    if (num_images < 2 || num_images > ACMMP_MAX_IMAGES)
        return set_err(ctx, ACMMP_ERR_ARG, "num_images=%d outside [2, %d]", num_images, ACMMP_MAX_IMAGES);
    if (!cams || !images) return set_err(ctx, ACMMP_ERR_ARG, "cams/images NULL");
    if (ctx->prm.patch_size != 11 || ctx->prm.radius_increment != 2)
        return set_err(ctx, ACMMP_ERR_UNSUPPORTED,
                       "patch_size=%d radius_increment=%d: kernels are built for the reference "
                       "defaults 11/2 (src/ACMMP.h:34,37)",
                       ctx->prm.patch_size, ctx->prm.radius_increment);
    for (int i = 0; i < num_images; ++i) {
        if (!images[i]) return set_err(ctx, ACMMP_ERR_ARG, "image %d is NULL", i);
        if (cams[i].width < 2 || cams[i].height < 1)
            return set_err(ctx, ACMMP_ERR_ARG, "camera %d has size %dx%d (width >= 2 required)", i,
                           cams[i].width, cams[i].height);
        if (borrow && pitches && pitches[i] < cams[i].width)
            return set_err(ctx, ACMMP_ERR_ARG, "image %d pitch %d < width %d", i, pitches[i], cams[i].width);
    }
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    free_images(ctx);
    const bool resize = (ctx->W != cams[0].width || ctx->H != cams[0].height);
    ctx->n = num_images;
    for (int i = 0; i < num_images; ++i) ctx->cams[i] = cams[i];
    ctx->W = cams[0].width;
    ctx->H = cams[0].height;
    ctx->Wh = (ctx->W + 1) / 2;
    ctx->prm.num_images = num_images;
    if (!keep_depth_range) {  // InputInitialization (src/ACMMP.cpp:600-606)
        ctx->prm.depth_min = cams[0].depth_min * 0.6f;
        ctx->prm.depth_max = cams[0].depth_max * 1.2f;
        ctx->prm.disparity_min = cams[0].K[0] * ctx->prm.baseline / ctx->prm.depth_max;
        ctx->prm.disparity_max = cams[0].K[0] * ctx->prm.baseline / ctx->prm.depth_min;
    }
    ctx->own_img.assign(num_images, nullptr);
    ctx->img.assign(num_images, nullptr);
    ctx->img_pitch.assign(num_images, 0);
    for (int i = 0; i < num_images; ++i) {
        if (borrow) {
            ctx->img[i] = images[i];
            ctx->img_pitch[i] = pitches ? pitches[i] : cams[i].width;
        } else {
            int rc = upload_pitched(ctx, ctx->own_img[i], ctx->img_pitch[i], images[i], cams[i].width,
                                    cams[i].height, false);
            if (rc) return rc;
            ctx->img[i] = ctx->own_img[i];
        }
    }
    // clamp-to-edge padded copies of every view (device-side, stream ordered)
    if (ctx->pad.size() < (size_t)num_images) {
        ctx->pad.resize(num_images, nullptr);
        ctx->pad_bytes.resize(num_images, 0);
        ctx->pad_pitch.resize(num_images, 0);
        ctx->pad_use.resize(num_images, nullptr);
    }
    if (tex) {  // prebuilt records of one common form: borrowed, nothing to pad
        for (int i = 0; i < num_images; ++i) {
            ctx->pad_use[i] = tex[i]->pad;
            ctx->pad_pitch[i] = tex[i]->pad_pitch;
        }
        ctx->pad_texel = tex[0]->form;
    } else {
    // The most compact form every view fits, each attempt checked by one
    // device flag (one stream sync): u8 quads (4 B per footprint: every view
    // integer-valued in [0, 255]), then f16 difference quads (8 B: every
    // stored value exact in f16), else the fp32 row-paired form (16 B).
    // ACMMP_TEXEL=u8|h16|f32 restricts the attempt to that one form before
    // fp32 (ACMMP_TEXEL_F32=1 = f32): the parity tests of every form.
    int tries[2];
    const int ntry = texel_tries(tries);
    if (!ctx->d_not_u8) HIP_TRY(ctx, dalloc(ctx->d_not_u8, 1));
    ctx->pad_texel = -1;
    for (int k = 0; k <= ntry && ctx->pad_texel < 0; ++k) {
        const int form = k < ntry ? tries[k] : kTexelF32;
        if (form != kTexelF32) HIP_TRY(ctx, hipMemsetAsync(ctx->d_not_u8, 0, sizeof(uint32_t), ctx->stream));
        for (int i = 0; i < num_images; ++i) {
            const int w = cams[i].width, h = cams[i].height;
            int pp;
            size_t bytes;
            if (pad_geometry(w, h, form, pp, bytes))
                return set_err(ctx, ACMMP_ERR_UNSUPPORTED, "view %d is %dx%d: above the 2^31-record gather limit", i,
                               w, h);
            if (ctx->pad_bytes[i] < bytes) {
                dfree(ctx->pad[i]);
                HIP_TRY(ctx, dalloc(ctx->pad[i], bytes / sizeof(float)));
                ctx->pad_bytes[i] = bytes;
            }
            ctx->pad_pitch[i] = pp;
            ctx->pad_use[i] = ctx->pad[i];
            HIP_TRY(ctx, launch_pad_form(form, ctx->img[i], ctx->img_pitch[i], w, h, ctx->pad[i], pp, ctx->d_not_u8,
                                         ctx->stream));
        }
        if (form == kTexelF32) {
            ctx->pad_texel = kTexelF32;
        } else {
            uint32_t unfit = 1;
            HIP_TRY(ctx, hipMemcpyAsync(&unfit, ctx->d_not_u8, sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
            HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
            if (unfit == 0) ctx->pad_texel = form;
        }
    }
    }  // padded copies
    if (resize || !ctx->d_rm_plane) {
        free_state(ctx);
        const size_t P = (size_t)ctx->W * ctx->H;
        const size_t Pc = (size_t)ctx->Wh * ctx->H;
        for (int c = 0; c < 2; ++c) {
            for (int b = 0; b < 2; ++b) {
                HIP_TRY(ctx, dalloc(ctx->d_cplane[c][b], Pc));
                HIP_TRY(ctx, dalloc(ctx->d_ccost[c][b], Pc));
            }
            HIP_TRY(ctx, dalloc(ctx->d_csv[c], Pc));
        }
        HIP_TRY(ctx, dalloc(ctx->d_rm_plane, P));
        HIP_TRY(ctx, dalloc(ctx->d_rm_cost, P));
        HIP_TRY(ctx, dalloc(ctx->d_rm_depth, P));
        HIP_TRY(ctx, dalloc(ctx->d_rm_sv, P));
        HIP_TRY(ctx, dalloc(ctx->d_pre_cost, P));
        // zero-filled state (pin: the reference's never-written host fields,
        // src/ACMMP.cpp:797-804, and uninitialised pre_costs)
        HIP_TRY(ctx, hipMemsetAsync(ctx->d_rm_plane, 0, P * sizeof(float4), ctx->stream));
        HIP_TRY(ctx, hipMemsetAsync(ctx->d_rm_cost, 0, P * sizeof(float), ctx->stream));
        HIP_TRY(ctx, hipMemsetAsync(ctx->d_rm_depth, 0, P * sizeof(float), ctx->stream));
        HIP_TRY(ctx, hipMemsetAsync(ctx->d_rm_sv, 0, P * sizeof(uint32_t), ctx->stream));
        HIP_TRY(ctx, hipMemsetAsync(ctx->d_pre_cost, 0, P * sizeof(float), ctx->stream));
        for (int c = 0; c < 2; ++c) HIP_TRY(ctx, hipMemsetAsync(ctx->d_csv[c], 0, Pc * sizeof(uint32_t), ctx->stream));
    }
    if (!borrow || resize) HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return ACMMP_OK;
}

float elapsed(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return -1.f;
    return ms;
}

}  // namespace

namespace acmmp {
int upload_kv(acmmp_ctx *ctx) { return kv_upload(ctx); }
KState make_state(acmmp_ctx *ctx) { return state_of(ctx); }
}  // namespace acmmp

extern "C" {

void acmmp_default_params(acmmp_params *p) {
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    p->max_iterations = 2;
    p->patch_size = 11;
    p->num_images = 5;
    p->max_image_size = 3200;
    p->radius_increment = 2;
    p->sigma_spatial = 5.0f;
    p->sigma_color = 3.0f;
    p->top_k = 4;
    p->baseline = 0.54f;
    p->depth_min = 0.0f;
    p->depth_max = 1.0f;
    p->disparity_min = 0.0f;
    p->disparity_max = 1.0f;
    p->seed_lo = 0x5EEDu;
    p->seed_hi = 0u;
    p->rng_stream = 0u;
}

int acmmp_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int acmmp_get_texel_bits(const acmmp_ctx *ctx) {
    if (!ctx) return ACMMP_ERR_ARG;
    return ctx->pad_texel == kTexelU8 ? 8 : ctx->pad_texel == kTexelH16 ? 16 : 32;
}

const char *acmmp_version(void) {
    return "acmmp_amd 0.1 gfx950 (-O3 -ffp-contract=off, IEEE div/sqrt, pinned detmath)";
}

int acmmp_create(int device, acmmp_ctx **out) {
    if (!out) return ACMMP_ERR_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return ACMMP_ERR_HIP;
    if (device < 0 || device >= ndev) return ACMMP_ERR_ARG;
    if (hipSetDevice(device) != hipSuccess) return ACMMP_ERR_HIP;
    acmmp_ctx *ctx = new acmmp_ctx();
    ctx->device = device;
    acmmp_default_params(&ctx->prm);
    if (stream_take(device, &ctx->stream) != hipSuccess) {
        delete ctx;
        return ACMMP_ERR_HIP;
    }
    *out = ctx;
    return ACMMP_OK;
}

void acmmp_destroy(acmmp_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    // Only a stream that drained cleanly hands its blocks, staging and
    // handles on to the next engine: after a failed sync (an asynchronous
    // error, a stream that did not drain) queued work may still touch them,
    // so they are released with hipFree / hipStreamDestroy (which wait for the
    // device) instead. Work the CALLER queued on other streams that reads
    // this engine's buffers must be finished before this call (include/acmmp.h).
    const bool clean = !ctx->stream || hipStreamSynchronize(ctx->stream) == hipSuccess;
    if (!clean) (void)hipGetLastError();
    g_frees_synced = clean;  // nothing queued can touch the engine's blocks now: they go to the cache
    free_images(ctx);
    free_state(ctx);
    for (auto &p : ctx->pad) dfree(p);
    dfree(ctx->d_not_u8);
    for (int k = 0; k < acmmp_ctx::kSlots; ++k) dfree(ctx->d_kv_ring[k]);
    g_frees_synced = false;
    for (int k = 0; k < acmmp_ctx::kSlots; ++k) {
        if (ctx->h_kv_ring[k]) {
            if (clean) pinned_kv_free(ctx->h_kv_ring[k]);
            else (void)hipHostFree(ctx->h_kv_ring[k]);
        }
        if (ctx->kv_ev[k]) {
            if (clean) event_give(ctx->device, false, ctx->kv_ev[k]);
            else (void)hipEventDestroy(ctx->kv_ev[k]);
        }
    }
    if (ctx->events_made)
        for (auto &e : ctx->ev) {
            if (clean) event_give(ctx->device, true, e);
            else (void)hipEventDestroy(e);
        }
    if (ctx->wait_ev) {
        if (clean) event_give(ctx->device, false, ctx->wait_ev);
        else (void)hipEventDestroy(ctx->wait_ev);
    }
    if (ctx->stream) {
        if (clean) stream_give(ctx->device, ctx->stream);
        else (void)hipStreamDestroy(ctx->stream);
    }
    delete ctx;
}

int acmmp_release_device_cache(int device) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return ACMMP_ERR_HIP;
    if (device >= ndev || device < -1) return ACMMP_ERR_ARG;
    int cur = 0;
    (void)hipGetDevice(&cur);
    {
        DevPool &pool = devpool();
        std::lock_guard<std::mutex> g(pool.mu);
        pool.release(device);
    }
    {
        std::lock_guard<std::mutex> g(handles().mu);
        for (auto it = handles().streams.begin(); it != handles().streams.end(); ++it) {
            if (device >= 0 && it->first != device) continue;
            (void)hipSetDevice(it->first);
            for (hipStream_t s : it->second) (void)hipStreamDestroy(s);
            it->second.clear();
        }
        for (auto it = handles().events.begin(); it != handles().events.end(); ++it) {
            if (device >= 0 && it->first.first != device) continue;
            (void)hipSetDevice(it->first.first);
            for (hipEvent_t e : it->second) (void)hipEventDestroy(e);
            it->second.clear();
        }
    }
    {
        std::lock_guard<std::mutex> g(g_pinned_mu);  // host staging is not per device: released with any call
        for (KViews *p : g_pinned_kv) (void)hipHostFree(p);
        g_pinned_kv.clear();
    }
    (void)hipSetDevice(cur);
    return ACMMP_OK;
}

int64_t acmmp_device_cache_bytes(int device) {
    DevPool &pool = devpool();
    std::lock_guard<std::mutex> g(pool.mu);
    return (int64_t)pool.bytes(device);
}

const char *acmmp_last_error(const acmmp_ctx *ctx) {
    if (!ctx) return "null context";
    return ctx->err.c_str();
}

int acmmp_set_params(acmmp_ctx *ctx, const acmmp_params *p) {
    if (!ctx || !p) return ACMMP_ERR_ARG;
    ctx->prm = *p;
    if (ctx->n >= 2) ctx->prm.num_images = ctx->n;
    return ACMMP_OK;
}

int acmmp_get_params(const acmmp_ctx *ctx, acmmp_params *p) {
    if (!ctx || !p) return ACMMP_ERR_ARG;
    *p = ctx->prm;
    return ACMMP_OK;
}

int acmmp_set_geom_consistency_params(acmmp_ctx *ctx, int multi_geometry) {
    if (!ctx) return ACMMP_ERR_ARG;
    ctx->prm.geom_consistency = 1;
    ctx->prm.max_iterations = 2;  // src/ACMMP.cpp:450
    if (multi_geometry) ctx->prm.multi_geometry = 1;
    return ACMMP_OK;
}

int acmmp_set_planar_prior_params(acmmp_ctx *ctx) {
    if (!ctx) return ACMMP_ERR_ARG;
    ctx->prm.planar_prior = 1;
    return ACMMP_OK;
}

int acmmp_set_hierarchy_params(acmmp_ctx *ctx) {
    if (!ctx) return ACMMP_ERR_ARG;
    ctx->prm.hierarchy = 1;
    return ACMMP_OK;
}

int acmmp_set_images(acmmp_ctx *ctx, int num_images, const acmmp_camera *cams, const float *const *images,
                     int keep_depth_range) {
    return set_images_impl(ctx, num_images, cams, images, nullptr, keep_depth_range, false);
}

int acmmp_set_images_device(acmmp_ctx *ctx, int num_images, const acmmp_camera *cams,
                            const float *const *d_images, const int32_t *pitches, int keep_depth_range) {
    return set_images_impl(ctx, num_images, cams, d_images, pitches, keep_depth_range, true);
}

int acmmp_texture_create(int device, const float *d_image, int pitch, int width, int height, acmmp_texture **out) {
    if (!out || !d_image || width < 2 || height < 1 || pitch < width) return ACMMP_ERR_ARG;
    *out = nullptr;
    if (hipSetDevice(device) != hipSuccess) return ACMMP_ERR_HIP;
    auto *t = new (std::nothrow) acmmp_texture;
    if (!t) return ACMMP_ERR_HIP;
    t->device = device;
    t->img = d_image;
    t->img_pitch = pitch;
    t->W = width;
    t->H = height;
    hipStream_t s = nullptr;
    uint32_t *d_unfit = nullptr;
    int rc = ACMMP_OK;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc((void **)&d_unfit, sizeof(uint32_t)) != hipSuccess)
        rc = ACMMP_ERR_HIP;
    // the most compact form the image fits (the choice set_images makes per problem)
    int tries[2];
    const int ntry = texel_tries(tries);
    t->form = -1;
    for (int k = 0; rc == ACMMP_OK && k <= ntry && t->form < 0; ++k) {
        const int form = k < ntry ? tries[k] : kTexelF32;
        size_t bytes;
        if (pad_geometry(width, height, form, t->pad_pitch, bytes)) {
            rc = ACMMP_ERR_UNSUPPORTED;
            break;
        }
        if (bytes > t->pad_bytes) {  // every form's bytes, not only the first tried
            if (t->pad) (void)hipFree(t->pad);
            t->pad = nullptr;
            t->pad_bytes = 0;
            if (hipMalloc((void **)&t->pad, bytes) != hipSuccess) {
                rc = ACMMP_ERR_HIP;
                break;
            }
            t->pad_bytes = bytes;
        }
        uint32_t unfit = 0;
        if (hipMemsetAsync(d_unfit, 0, sizeof(uint32_t), s) != hipSuccess ||
            launch_pad_form(form, d_image, pitch, width, height, t->pad, t->pad_pitch, d_unfit, s) != hipSuccess ||
            hipMemcpyAsync(&unfit, d_unfit, sizeof(uint32_t), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            rc = ACMMP_ERR_HIP;
            break;
        }
        if (form == kTexelF32 || unfit == 0) t->form = form;
    }
    if (d_unfit) (void)hipFree(d_unfit);
    if (s) (void)hipStreamDestroy(s);
    if (rc != ACMMP_OK) {
        acmmp_texture_destroy(t);
        return rc;
    }
    *out = t;
    return ACMMP_OK;
}

void acmmp_texture_destroy(acmmp_texture *t) {
    if (!t) return;
    if (t->pad) {
        (void)hipSetDevice(t->device);
        (void)hipFree(t->pad);
    }
    delete t;
}

int acmmp_texture_bits(const acmmp_texture *t) {
    if (!t) return 0;
    return t->form == kTexelU8 ? 8 : t->form == kTexelH16 ? 16 : 32;
}

int acmmp_set_images_textures(acmmp_ctx *ctx, int num_images, const acmmp_camera *cams,
                              const acmmp_texture *const *textures, int keep_depth_range) {
    if (!ctx) return ACMMP_ERR_ARG;
    if (!cams || !textures || num_images < 2 || num_images > ACMMP_MAX_IMAGES)
        return set_err(ctx, ACMMP_ERR_ARG, "bad textures");
    const float *imgs[ACMMP_MAX_IMAGES];
    int32_t pitches[ACMMP_MAX_IMAGES];
    bool common = true;
    for (int i = 0; i < num_images; ++i) {
        const acmmp_texture *t = textures[i];
        if (!t) return set_err(ctx, ACMMP_ERR_ARG, "texture %d is NULL", i);
        if (t->device != ctx->device) return set_err(ctx, ACMMP_ERR_ARG, "texture %d is on device %d", i, t->device);
        if (t->W != cams[i].width || t->H != cams[i].height)
            return set_err(ctx, ACMMP_ERR_ARG, "texture %d is %dx%d, camera %dx%d", i, t->W, t->H, cams[i].width,
                           cams[i].height);
        imgs[i] = t->img;
        pitches[i] = t->img_pitch;
        common = common && t->form == textures[0]->form;
    }
    // views of different forms (one not 8-bit, say): pad per engine in the common form
    return set_images_impl(ctx, num_images, cams, imgs, pitches, keep_depth_range, true,
                           common ? textures : nullptr);
}

int acmmp_set_depth_maps(acmmp_ctx *ctx, const float *const *depths) {
    return set_depths_impl(ctx, depths, nullptr, false);
}

int acmmp_set_depth_maps_device(acmmp_ctx *ctx, const float *const *d_depths, const int32_t *pitches) {
    return set_depths_impl(ctx, d_depths, pitches, true);
}

int acmmp_set_plane_hypotheses(acmmp_ctx *ctx, const float *planes4, const float *costs) {
    int rc = check_ready(ctx);
    if (rc) return rc;
    if (!planes4 || !costs) return set_err(ctx, ACMMP_ERR_ARG, "planes/costs NULL");
    const size_t P = (size_t)ctx->W * ctx->H;
    ctx->depth_ok = false;
    HIP_TRY(ctx, hipMemcpyAsync(ctx->d_rm_plane, planes4, P * sizeof(float4), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(ctx->d_rm_cost, costs, P * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    ctx->have_state = true;
    return ACMMP_OK;
}

int acmmp_set_plane_hypotheses_device(acmmp_ctx *ctx, const float *d_planes4, const float *d_costs) {
    int rc = check_ready(ctx);
    if (rc) return rc;
    if (!d_planes4 || !d_costs) return set_err(ctx, ACMMP_ERR_ARG, "planes/costs NULL");
    const size_t P = (size_t)ctx->W * ctx->H;
    ctx->depth_ok = false;
    HIP_TRY(ctx, hipMemcpyAsync(ctx->d_rm_plane, d_planes4, P * sizeof(float4), hipMemcpyDeviceToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(ctx->d_rm_cost, d_costs, P * sizeof(float), hipMemcpyDeviceToDevice, ctx->stream));
    ctx->have_state = true;
    return ACMMP_OK;
}

int acmmp_wait_stream(acmmp_ctx *ctx, void *stream) {
    if (!ctx) return ACMMP_ERR_ARG;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    if (!ctx->wait_ev) HIP_TRY(ctx, event_take(ctx->device, false, &ctx->wait_ev));
    // hipStreamWaitEvent captures the event's state at this call, so the one
    // event is safely re-recorded by the next call
    HIP_TRY(ctx, hipEventRecord(ctx->wait_ev, (hipStream_t)stream));
    HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->wait_ev, 0));
    return ACMMP_OK;
}

int acmmp_export_results(acmmp_ctx *ctx, float *d_planes4, float *d_costs, float *d_depth) {
    int rc = check_ready(ctx);
    if (rc) return rc;
    const size_t P = (size_t)ctx->W * ctx->H;
    if (d_planes4)
        HIP_TRY(ctx, hipMemcpyAsync(d_planes4, ctx->d_rm_plane, P * sizeof(float4), hipMemcpyDeviceToDevice, ctx->stream));
    if (d_costs)
        HIP_TRY(ctx, hipMemcpyAsync(d_costs, ctx->d_rm_cost, P * sizeof(float), hipMemcpyDeviceToDevice, ctx->stream));
    if (d_depth && ctx->depth_ok)  // the depth plane the last full run wrote: a plain copy
        HIP_TRY(ctx, hipMemcpyAsync(d_depth, ctx->d_rm_depth, P * sizeof(float), hipMemcpyDeviceToDevice, ctx->stream));
    else if (d_depth)  // the .w channel: strided 2-D copy, 4 B out of every 16 B
        HIP_TRY(ctx, hipMemcpy2DAsync(d_depth, sizeof(float), (const char *)ctx->d_rm_plane + 3 * sizeof(float),
                                      sizeof(float4), sizeof(float), P, hipMemcpyDeviceToDevice, ctx->stream));
    return ACMMP_OK;
}

namespace {
int set_hierarchy_impl(acmmp_ctx *ctx, const float *scaled_planes4, int scaled_w, int scaled_h,
                       const float *upsampled_depth, bool device_src) {
    int rc = check_ready(ctx);
    if (rc) return rc;
    if (!scaled_planes4 || !upsampled_depth || scaled_w <= 0 || scaled_h <= 0)
        return set_err(ctx, ACMMP_ERR_ARG, "bad hierarchy inputs");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const size_t S = (size_t)scaled_w * scaled_h;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));  // a queued run may still read the old inputs
    HIP_TRY(ctx, dalloc(ctx->d_scaled, S));
    ctx->scaled_count = S;
    HIP_TRY(ctx, hipMemcpyAsync(ctx->d_scaled, scaled_planes4, S * sizeof(float4),
                                device_src ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, ctx->stream));
    // plane_hypotheses_host[center].w = ref_depth; x, y, z never written (pinned 0)
    const size_t P = (size_t)ctx->W * ctx->H;
    if (device_src) {
        ctx->depth_ok = false;
        HIP_TRY(ctx, launch_depth_planes(upsampled_depth, P, ctx->d_rm_plane, ctx->stream));
    } else {
        std::vector<float> tmp(P * 4, 0.0f);
        for (size_t i = 0; i < P; ++i) tmp[i * 4 + 3] = upsampled_depth[i];
        ctx->depth_ok = false;
        HIP_TRY(ctx, hipMemcpyAsync(ctx->d_rm_plane, tmp.data(), P * sizeof(float4), hipMemcpyHostToDevice,
                                    ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));  // tmp goes out of scope
    }
    // `if (width != images[0].rows || height != images[0].cols)` (src/ACMMP.cpp:766), swap included
    if (scaled_w != ctx->H || scaled_h != ctx->W) {
        ctx->prm.upsample = 1;
        ctx->prm.scaled_cols = (float)scaled_w;
        ctx->prm.scaled_rows = (float)scaled_h;
    } else {
        ctx->prm.upsample = 0;
    }
    ctx->have_scaled = true;
    return ACMMP_OK;
}
}  // namespace

int acmmp_set_hierarchy_inputs(acmmp_ctx *ctx, const float *scaled_planes4, int scaled_w, int scaled_h,
                               const float *upsampled_depth) {
    return set_hierarchy_impl(ctx, scaled_planes4, scaled_w, scaled_h, upsampled_depth, false);
}

int acmmp_set_hierarchy_inputs_device(acmmp_ctx *ctx, const float *d_scaled_planes4, int scaled_w, int scaled_h,
                                      const float *d_upsampled_depth) {
    return set_hierarchy_impl(ctx, d_scaled_planes4, scaled_w, scaled_h, d_upsampled_depth, true);
}

int acmmp_set_seed_prior(acmmp_ctx *ctx, const float *planes4) {
    int rc = check_ready(ctx);
    if (rc) return rc;
    if (!planes4) return set_err(ctx, ACMMP_ERR_ARG, "planes NULL");
    const size_t P = (size_t)ctx->W * ctx->H;
    HIP_TRY(ctx, dalloc(ctx->d_seed, P));
    HIP_TRY(ctx, hipMemcpyAsync(ctx->d_seed, planes4, P * sizeof(float4), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    ctx->prm.seeded = 1;
    ctx->have_seed = true;
    return ACMMP_OK;
}

int acmmp_set_planar_prior(acmmp_ctx *ctx, const float *plane_params4, int num_planes, const uint32_t *mask) {
    int rc = check_ready(ctx);
    if (rc) return rc;
    if (!mask || num_planes < 0 || (num_planes > 0 && !plane_params4))
        return set_err(ctx, ACMMP_ERR_ARG, "bad planar prior inputs");
    const size_t P = (size_t)ctx->W * ctx->H;
    // CudaPlanarPriorInitialization (src/ACMMP.cpp:811-831): expand the label
    // mask into a per-pixel plane array (unlabelled pixels: zero, pinned).
    std::vector<float> planes(P * 4, 0.0f);
    for (size_t i = 0; i < P; ++i) {
        const uint32_t m = mask[i];
        if (m > 0) {
            if ((int)m > num_planes)
                return set_err(ctx, ACMMP_ERR_ARG, "mask label %u exceeds %d planes", m, num_planes);
            std::memcpy(&planes[i * 4], plane_params4 + (size_t)(m - 1) * 4, 4 * sizeof(float));
        }
    }
    HIP_TRY(ctx, dalloc(ctx->d_prior, P));
    HIP_TRY(ctx, dalloc(ctx->d_mask, P));
    HIP_TRY(ctx, hipMemcpyAsync(ctx->d_prior, planes.data(), P * sizeof(float4), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(ctx->d_mask, mask, P * sizeof(uint32_t), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    ctx->have_prior = true;
    return ACMMP_OK;
}

namespace {
// The checks and constant upload every run starts with (RunPatchMatch's
// preconditions, src/ACMMP.cu:1378-1414).
int prepare_run(acmmp_ctx *ctx) {
    int rc = check_ready(ctx);
    if (rc) return rc;
    const acmmp_params &p = ctx->prm;
    if (p.geom_consistency && !ctx->have_depths)
        return set_err(ctx, ACMMP_ERR_STATE, "geom_consistency needs depth maps (acmmp_set_depth_maps)");
    if (p.planar_prior && !ctx->have_prior)
        return set_err(ctx, ACMMP_ERR_STATE, "planar_prior needs acmmp_set_planar_prior");
    if (p.hierarchy && !ctx->have_scaled)
        return set_err(ctx, ACMMP_ERR_STATE, "hierarchy needs acmmp_set_hierarchy_inputs");
    if (p.seeded && !ctx->have_seed) return set_err(ctx, ACMMP_ERR_STATE, "seeded needs acmmp_set_seed_prior");
    if (p.patch_size != 11 || p.radius_increment != 2)
        return set_err(ctx, ACMMP_ERR_UNSUPPORTED, "only patch_size 11 / radius_increment 2 are built");
    if (p.max_iterations < 0) return set_err(ctx, ACMMP_ERR_ARG, "max_iterations < 0");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    rc = kv_upload(ctx);
    if (rc) return rc;
    if (p.texture_filter8 && (ctx->pad_texel == kTexelH16 || ctx->h_kv.wide))
        return set_err(ctx, ACMMP_ERR_UNSUPPORTED, "texture_filter8 is built for the u8 / fp32 texel forms below 2^24 records");
    if (ctx->timing && !ctx->events_made) {
        for (auto &e : ctx->ev) HIP_TRY(ctx, event_take(ctx->device, true, &e));
        ctx->events_made = true;
    }
    return ACMMP_OK;
}
}  // namespace

int acmmp_run_patchmatch_async(acmmp_ctx *ctx) {
    int rc = prepare_run(ctx);
    if (rc) return rc;
    const acmmp_params &p = ctx->prm;
    hipStream_t s = ctx->stream;
    ctx->depth_ok = false;  // until this run's filters are queued (a failed run leaves the strided export)
    if (ctx->timing) HIP_TRY(ctx, hipEventRecord(ctx->ev[0], s));
    ctx->cur[0] = ctx->cur[1] = 0;
    HIP_TRY(ctx, launch_init(ctx->d_kv, ctx->h_kv, state_of(ctx), s));
    if (ctx->timing) HIP_TRY(ctx, hipEventRecord(ctx->ev[1], s));
    for (int it = 0; it < p.max_iterations; ++it) {
        for (int colour = 0; colour < 2; ++colour) {  // BlackPixelUpdate, RedPixelUpdate
            HIP_TRY(ctx, launch_sweep(ctx->d_kv, ctx->h_kv, state_of(ctx), colour, it, s));
            ctx->cur[colour] ^= 1;
        }
    }
    if (ctx->timing) HIP_TRY(ctx, hipEventRecord(ctx->ev[2], s));
    HIP_TRY(ctx, launch_finalize(ctx->d_kv, ctx->h_kv, state_of(ctx), s));
    HIP_TRY(ctx, launch_filter(ctx->d_kv, ctx->h_kv, state_of(ctx), 0, s));
    HIP_TRY(ctx, launch_filter(ctx->d_kv, ctx->h_kv, state_of(ctx), 1, s));
    ctx->depth_ok = true;  // every pixel's depth: finalize + filters over the whole image
    if (ctx->timing) HIP_TRY(ctx, hipEventRecord(ctx->ev[3], s));
    ctx->prm.rng_stream += 1u;  // a further RunPatchMatch re-seeds (clock64() in the reference)
    ctx->have_state = true;
    return ACMMP_OK;
}

int acmmp_run_patchmatch_band(acmmp_ctx *ctx, int row_lo, int row_hi, acmmp_band_exchange_fn exchange, void *user) {
    int rc = prepare_run(ctx);
    if (rc) return rc;
    const int H = ctx->H, K = ACMMP_BAND_HALO;
    if (!exchange || row_lo < 0 || row_hi > H || row_lo >= row_hi)
        return set_err(ctx, ACMMP_ERR_ARG, "band rows [%d, %d) outside [0, %d) or no exchange", row_lo, row_hi, H);
    const acmmp_params &p = ctx->prm;
    hipStream_t s = ctx->stream;
    const int lo_k = std::max(0, row_lo - K), hi_k = std::min(H, row_hi + K);
    if (ctx->timing) HIP_TRY(ctx, hipEventRecord(ctx->ev[0], s));
    ctx->cur[0] = ctx->cur[1] = 0;
    // every pixel's initial state is a function of its own inputs: computing
    // the halo rows here too means they start out valid, with no exchange
    HIP_TRY(ctx, launch_init(ctx->d_kv, ctx->h_kv, state_of(ctx, lo_k, hi_k), s));
    if (ctx->timing) HIP_TRY(ctx, hipEventRecord(ctx->ev[1], s));
    acmmp_band_halo halo{};
    halo.Wh = ctx->Wh;
    halo.stream = (void *)s;
    halo.send_up_lo = row_lo;
    halo.send_up_hi = row_lo > 0 ? std::min(row_hi, row_lo + K) : row_lo;
    halo.send_down_lo = row_hi < H ? std::max(row_lo, row_hi - K) : row_hi;
    halo.send_down_hi = row_hi;
    halo.recv_up_lo = lo_k;
    halo.recv_up_hi = row_lo;
    halo.recv_down_lo = row_hi;
    halo.recv_down_hi = hi_k;
    for (int it = 0; it < p.max_iterations; ++it) {
        for (int colour = 0; colour < 2; ++colour) {
            HIP_TRY(ctx, launch_sweep(ctx->d_kv, ctx->h_kv, state_of(ctx, row_lo, row_hi), colour, it, s));
            ctx->cur[colour] ^= 1;
            // the colour's new current state: the neighbours' rows next to
            // the band, as the next half-sweeps read them
            halo.colour = colour;
            halo.plane = ctx->d_cplane[colour][ctx->cur[colour]];
            halo.cost = ctx->d_ccost[colour][ctx->cur[colour]];
            halo.sv = ctx->d_csv[colour];
            if (const int e = exchange(user, &halo))
                return set_err(ctx, ACMMP_ERR_STATE, "band exchange failed (status %d) after iteration %d colour %d", e,
                               it, colour);
        }
    }
    if (ctx->timing) HIP_TRY(ctx, hipEventRecord(ctx->ev[2], s));
    // CheckerboardFilter reads +-5 rows (src/ACMMP.cu:1214-1328): depth /
    // normal conversion on the band +-10 rows (valid halos), the black filter
    // on the band +-5 rows (what the red filter reads), the red one on the band
    ctx->depth_ok = false;  // rows outside the band keep older depths
    HIP_TRY(ctx, launch_finalize(ctx->d_kv, ctx->h_kv, state_of(ctx, std::max(0, row_lo - 10), std::min(H, row_hi + 10)), s));
    HIP_TRY(ctx, launch_filter(ctx->d_kv, ctx->h_kv, state_of(ctx, std::max(0, row_lo - 5), std::min(H, row_hi + 5)), 0, s));
    HIP_TRY(ctx, launch_filter(ctx->d_kv, ctx->h_kv, state_of(ctx, row_lo, row_hi), 1, s));
    if (ctx->timing) HIP_TRY(ctx, hipEventRecord(ctx->ev[3], s));
    ctx->prm.rng_stream += 1u;
    ctx->have_state = true;
    return acmmp_synchronize(ctx);
}

int acmmp_synchronize(acmmp_ctx *ctx) {
    if (!ctx) return ACMMP_ERR_ARG;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (ctx->timing && ctx->events_made) {
        acmmp_timing &t = ctx->last_timing;
        t.init_ms = elapsed(ctx->ev[0], ctx->ev[1]);
        t.sweep_ms = elapsed(ctx->ev[1], ctx->ev[2]);
        t.sweep_launches = 2 * ctx->prm.max_iterations;
        t.finalize_ms = elapsed(ctx->ev[2], ctx->ev[3]);
        t.total_ms = elapsed(ctx->ev[0], ctx->ev[3]);
    }
    return ACMMP_OK;
}

int acmmp_run_patchmatch(acmmp_ctx *ctx) {
    int rc = acmmp_run_patchmatch_async(ctx);
    if (rc) return rc;
    return acmmp_synchronize(ctx);
}

int acmmp_get_plane_hypotheses(acmmp_ctx *ctx, float *planes4, size_t n) {
    int rc = check_ready(ctx);
    if (rc) return rc;
    const size_t P = (size_t)ctx->W * ctx->H;
    if (!planes4 || n < P) return set_err(ctx, ACMMP_ERR_ARG, "output capacity %zu < %zu", n, P);
    HIP_TRY(ctx, hipMemcpyAsync(planes4, ctx->d_rm_plane, P * sizeof(float4), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return ACMMP_OK;
}

int acmmp_get_costs(acmmp_ctx *ctx, float *costs, size_t n) {
    int rc = check_ready(ctx);
    if (rc) return rc;
    const size_t P = (size_t)ctx->W * ctx->H;
    if (!costs || n < P) return set_err(ctx, ACMMP_ERR_ARG, "output capacity %zu < %zu", n, P);
    HIP_TRY(ctx, hipMemcpyAsync(costs, ctx->d_rm_cost, P * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return ACMMP_OK;
}

int acmmp_get_selected_views(acmmp_ctx *ctx, uint32_t *views, size_t n) {
    int rc = check_ready(ctx);
    if (rc) return rc;
    const size_t P = (size_t)ctx->W * ctx->H;
    if (!views || n < P) return set_err(ctx, ACMMP_ERR_ARG, "output capacity %zu < %zu", n, P);
    HIP_TRY(ctx, hipMemcpyAsync(views, ctx->d_rm_sv, P * sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return ACMMP_OK;
}

int acmmp_get_device_results(acmmp_ctx *ctx, const float **d_planes4, const float **d_costs) {
    int rc = check_ready(ctx);
    if (rc) return rc;
    if (d_planes4) *d_planes4 = (const float *)ctx->d_rm_plane;
    if (d_costs) *d_costs = ctx->d_rm_cost;
    return ACMMP_OK;
}

int acmmp_get_reference_size(const acmmp_ctx *ctx, int *width, int *height) {
    if (!ctx || !width || !height) return ACMMP_ERR_ARG;
    *width = ctx->W;
    *height = ctx->H;
    return ACMMP_OK;
}

int acmmp_get_reference_image(acmmp_ctx *ctx, float *out, size_t n) {
    int rc = check_ready(ctx);
    if (rc) return rc;
    if (!out || n < (size_t)ctx->W * ctx->H) return set_err(ctx, ACMMP_ERR_ARG, "output capacity too small");
    HIP_TRY(ctx, hipMemcpy2DAsync(out, (size_t)ctx->W * sizeof(float), ctx->img[0],
                                  (size_t)ctx->img_pitch[0] * sizeof(float), (size_t)ctx->W * sizeof(float),
                                  (size_t)ctx->H, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return ACMMP_OK;
}

int acmmp_get_camera(const acmmp_ctx *ctx, int index, acmmp_camera *cam) {
    if (!ctx || !cam || index < 0 || index >= ctx->n) return ACMMP_ERR_ARG;
    *cam = ctx->cams[index];
    return ACMMP_OK;
}

int acmmp_eval_costs(acmmp_ctx *ctx, const float *planes4, float *out_costs, float *out_init_cost,
                     uint32_t *out_init_views) {
    int rc = check_ready(ctx);
    if (rc) return rc;
    if (!planes4) return set_err(ctx, ACMMP_ERR_ARG, "planes NULL");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    rc = kv_upload(ctx);
    if (rc) return rc;
    const size_t P = (size_t)ctx->W * ctx->H;
    const int ns = ctx->n - 1;
    float4 *d_pl = nullptr;
    float *d_out = nullptr, *d_init = nullptr;
    uint32_t *d_views = nullptr;
    HIP_TRY(ctx, dalloc(d_pl, P));
    if (out_costs) HIP_TRY(ctx, dalloc(d_out, P * ns));
    if (out_init_cost) HIP_TRY(ctx, dalloc(d_init, P));
    if (out_init_views) HIP_TRY(ctx, dalloc(d_views, P));
    HIP_TRY(ctx, hipMemcpyAsync(d_pl, planes4, P * sizeof(float4), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, launch_eval_costs(ctx->d_kv, ctx->h_kv, d_pl, d_out, d_init, d_views, ctx->stream));
    if (out_costs)
        HIP_TRY(ctx, hipMemcpyAsync(out_costs, d_out, P * ns * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    if (out_init_cost)
        HIP_TRY(ctx, hipMemcpyAsync(out_init_cost, d_init, P * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    if (out_init_views)
        HIP_TRY(ctx, hipMemcpyAsync(out_init_views, d_views, P * sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    dfree(d_pl);
    dfree(d_out);
    dfree(d_init);
    dfree(d_views);
    return ACMMP_OK;
}

int acmmp_eval_geom_costs(acmmp_ctx *ctx, const float *planes4, float *out) {
    int rc = check_ready(ctx);
    if (rc) return rc;
    if (!planes4 || !out) return set_err(ctx, ACMMP_ERR_ARG, "NULL argument");
    if (!ctx->have_depths) return set_err(ctx, ACMMP_ERR_STATE, "no depth maps");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    rc = kv_upload(ctx);
    if (rc) return rc;
    const size_t P = (size_t)ctx->W * ctx->H;
    const int ns = ctx->n - 1;
    float4 *d_pl = nullptr;
    float *d_out = nullptr;
    HIP_TRY(ctx, dalloc(d_pl, P));
    HIP_TRY(ctx, dalloc(d_out, P * ns));
    HIP_TRY(ctx, hipMemcpyAsync(d_pl, planes4, P * sizeof(float4), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, launch_eval_geom(ctx->d_kv, ctx->h_kv, d_pl, d_out, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(out, d_out, P * ns * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    dfree(d_pl);
    dfree(d_out);
    return ACMMP_OK;
}

int acmmp_joint_bilateral_upsample(int device, const float *image, int width, int height, const float *depth,
                                   int depth_width, int depth_height, float *out, int *image_scale) {
    if (!image || !depth || !out || width <= 0 || height <= 0 || depth_width <= 0 || depth_height <= 0)
        return ACMMP_ERR_ARG;
    // RunJBU (src/ACMMP.cpp:1012-1021): Imagescale from integer size ratios;
    // 1 means nothing to upsample and the reference writes nothing.
    const int isc = std::max(height / depth_height, width / depth_width);
    if (image_scale) *image_scale = isc;
    if (isc <= 1) return ACMMP_OK;
    if (isc > 64) return ACMMP_ERR_UNSUPPORTED;
    if (hipSetDevice(device) != hipSuccess) return ACMMP_ERR_HIP;
    const size_t P = (size_t)width * height, S = (size_t)depth_width * depth_height;
    float *d_img = nullptr, *d_dep = nullptr, *d_out = nullptr;
    // the stream and blocks come from the engines' caches and return there
    // once the stream is synchronised (hipFree would synchronise the device)
    hipStream_t s = nullptr;
    hipError_t e = stream_take(device, &s);
    if (e == hipSuccess) e = dalloc(d_img, P);
    if (e == hipSuccess) e = dalloc(d_dep, S);
    if (e == hipSuccess) e = dalloc(d_out, P);
    if (e == hipSuccess) e = hipMemcpyAsync(d_img, image, P * sizeof(float), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(d_dep, depth, S * sizeof(float), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = launch_jbu(d_img, width, height, d_dep, depth_width, depth_height, isc, d_out, s);
    if (e == hipSuccess) e = hipMemcpyAsync(out, d_out, P * sizeof(float), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e == hipSuccess) {
        dfree_synced(d_img);
        dfree_synced(d_dep);
        dfree_synced(d_out);
        stream_give(device, s);
    } else {  // a failed stream may still hold work: the plain frees
        dfree(d_img);
        dfree(d_dep);
        dfree(d_out);
        if (s) (void)hipStreamDestroy(s);
    }
    return e == hipSuccess ? ACMMP_OK : ACMMP_ERR_HIP;
}

int acmmp_joint_bilateral_upsample_device(int device, const float *d_image, int width, int height,
                                          const float *d_depth, int depth_width, int depth_height, float *d_out,
                                          int *image_scale) {
    if (!d_image || !d_depth || !d_out || width <= 0 || height <= 0 || depth_width <= 0 || depth_height <= 0)
        return ACMMP_ERR_ARG;
    const int isc = std::max(height / depth_height, width / depth_width);  // RunJBU (src/ACMMP.cpp:1012-1021)
    if (image_scale) *image_scale = isc;
    if (isc <= 1) return ACMMP_OK;
    if (isc > 64) return ACMMP_ERR_UNSUPPORTED;
    if (hipSetDevice(device) != hipSuccess) return ACMMP_ERR_HIP;
    hipStream_t s = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e == hipSuccess) e = launch_jbu(d_image, width, height, d_depth, depth_width, depth_height, isc, d_out, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (s) (void)hipStreamDestroy(s);
    return e == hipSuccess ? ACMMP_OK : ACMMP_ERR_HIP;
}

int acmmp_selftest_reciprocal(int device, uint64_t *mismatches, uint64_t *checked) {
    if (!mismatches || !checked) return ACMMP_ERR_ARG;
    if (hipSetDevice(device) != hipSuccess) return ACMMP_ERR_HIP;
    unsigned long long *d = nullptr;
    if (hipMalloc((void **)&d, 2 * sizeof(unsigned long long)) != hipSuccess) return ACMMP_ERR_HIP;
    int rc = ACMMP_OK;
    if (hipMemset(d, 0, 2 * sizeof(unsigned long long)) != hipSuccess ||
        launch_selftest_rcp(d, d + 1, nullptr) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        rc = ACMMP_ERR_HIP;
    } else {
        unsigned long long h[2] = {0, 0};
        if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) rc = ACMMP_ERR_HIP;
        *mismatches = h[0];
        *checked = h[1];
    }
    (void)hipFree(d);
    return rc;
}

int acmmp_set_timing(acmmp_ctx *ctx, int enable) {
    if (!ctx) return ACMMP_ERR_ARG;
    ctx->timing = enable != 0;
    return ACMMP_OK;
}

int acmmp_get_timing(const acmmp_ctx *ctx, acmmp_timing *t) {
    if (!ctx || !t) return ACMMP_ERR_ARG;
    *t = ctx->last_timing;
    return ACMMP_OK;
}

}  // extern "C"
