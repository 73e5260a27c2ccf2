// acmmp_fusion.cpp — RunFusion (src/acmmp_definitions.cpp:828-1043), SURVEY
// §8f rank 3: depth/normal maps of all views -> one coloured point cloud
// (<out>/ACMMP_model.ply, StoreColorPlyFileBinaryPointCloud src/ACMMP.cpp:
// 382-424).
//
// Host code, literal: the reference's fusion is order-dependent (a pixel's
// approval masks pixels of other views that later pixels then skip, and
// used_list is never reset between pixels), so approvals run sequentially in
// the reference's order with the reference's float expression order; the
// per-pixel projections and tests before them run on host threads per band
// of rows and are re-checked against the masks at approval time (exact: masks
// only ever go 0 -> 1)
// (Get3DPointonWorld / ProjectonCamera src/ACMMP.cpp:203-251, GetAngle
// :253-262). Deviations: no cv::imshow (:897-900); the PLY is written in
// point order (the reference's OpenMP-critical writes make its order
// arbitrary); a colour image whose size differs from its depth map is resized
// with a float bilinear filter (cv::resize's 8-bit fixed-point path is
// unpinned).
#include <sched.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cfloat>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/acmmp.h"
#include "acmmp_hostio.h"

namespace {

thread_local std::string f_err;

int ffail(int code, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    f_err = buf;
    return code;
}

std::string id8(int id) {
    char b[32];
    std::snprintf(b, sizeof(b), "%08d", id);
    return b;
}

struct F3 {
    float x, y, z;
};

F3 world_point(int x, int y, float depth, const acmmp_camera &c) {  // Get3DPointonWorld
    F3 p;
    p.x = depth * (x - c.K[2]) / c.K[0];
    p.y = depth * (y - c.K[5]) / c.K[4];
    p.z = depth;
    F3 t;
    t.x = c.R[0] * p.x + c.R[3] * p.y + c.R[6] * p.z;
    t.y = c.R[1] * p.x + c.R[4] * p.y + c.R[7] * p.z;
    t.z = c.R[2] * p.x + c.R[5] * p.y + c.R[8] * p.z;
    F3 C;
    C.x = -(c.R[0] * c.t[0] + c.R[3] * c.t[1] + c.R[6] * c.t[2]);
    C.y = -(c.R[1] * c.t[0] + c.R[4] * c.t[1] + c.R[7] * c.t[2]);
    C.z = -(c.R[2] * c.t[0] + c.R[5] * c.t[1] + c.R[8] * c.t[2]);
    p.x = t.x + C.x;
    p.y = t.y + C.y;
    p.z = t.z + C.z;
    return p;
}

void project(const F3 &X, const acmmp_camera &c, float &px, float &py, float &depth) {  // ProjectonCamera
    F3 t;
    t.x = c.R[0] * X.x + c.R[1] * X.y + c.R[2] * X.z + c.t[0];
    t.y = c.R[3] * X.x + c.R[4] * X.y + c.R[5] * X.z + c.t[1];
    t.z = c.R[6] * X.x + c.R[7] * X.y + c.R[8] * X.z + c.t[2];
    depth = c.K[6] * t.x + c.K[7] * t.y + c.K[8] * t.z;
    px = (c.K[0] * t.x + c.K[1] * t.y + c.K[2] * t.z) / depth;
    py = (c.K[3] * t.x + c.K[4] * t.y + c.K[5] * t.z) / depth;
}

float get_angle(const float *a, const float *b) {  // GetAngle
    const float dot = a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
    const float angle = std::acos(dot);
    if (angle != angle) return 0.0f;
    return angle;
}

// RunFusion phase 1's two arithmetic stages (see phase1 below): branch-free
// loops the vectoriser turns into AVX2 where the host has it. Each is built
// twice (target_clones: an AVX2 clone and a baseline x86-64 clone, picked by
// the loader from the running CPU), so the library never executes an AVX2
// instruction on a host without it. AVX2 without FMA, and this file builds
// with -ffp-contract=off: both clones perform the same IEEE operations, so
// the PLY does not depend on the host.
__attribute__((target_clones("avx2", "default")))
void stage_project(const F3 *X, size_t nl, const acmmp_camera &cs, int *scp, int *srp) {
    for (size_t k = 0; k < nl; ++k) {
        float ptx, pty, proj_depth;
        project(X[k], cs, ptx, pty, proj_depth);
        srp[k] = int(pty + 0.5f);
        scp[k] = int(ptx + 0.5f);
    }
}

// reprojection of candidate q's source pixel into view i (row r): error and
// relative depth difference
__attribute__((target_clones("avx2", "default")))
void stage_reproject(size_t nc, int r, const int *__restrict__ col, const int *__restrict__ scp,
                     const int *__restrict__ srp, const float *__restrict__ cd, const float *__restrict__ cr,
                     float *__restrict__ re, float *__restrict__ rd, const acmmp_camera cs, const acmmp_camera ci) {
    for (size_t q = 0; q < nc; ++q) {
        const float ref_depth = cr[q];
        float tx, ty, proj_depth;
        const F3 tmp_X = world_point(scp[q], srp[q], cd[q], cs);
        project(tmp_X, ci, tx, ty, proj_depth);
        // std::pow(v, 2) of a float v is exact in double: v * v
        const double dx = (double)(col[q] - tx), dy = (double)(r - ty);
        re[q] = (float)std::sqrt(dx * dx + dy * dy);
        rd[q] = std::fabs(proj_depth - ref_depth) / ref_depth;
    }
}

// RunFusion's threads kept on ONE last-level-cache domain (on a many-CCD
// host a view's candidate lists, written by the pool, and the masks, written
// by the walk, otherwise cross between L3s on every access; the walk, which
// is sequential, measured ~1.4 s or 5-7 s for cfg4 depending on where the
// scheduler happened to put the threads, profiles/r03_fusion_ab.jsonl):
// the calling thread is confined to the physical core it runs on, the
// workers to the rest of that core's L3 domain (within the allowed CPUs).
// Restored when RunFusion returns. ACMMP_FUSION_PIN=0 turns it off.
class CacheDomain {
  public:
    CacheDomain() : threads_(acmmp_host_threads()) {  // the budget before any pinning
        if (const char *e = std::getenv("ACMMP_FUSION_PIN"))
            if (std::atoi(e) == 0) return;
        const int cpu = sched_getcpu();
        if (cpu < 0 || sched_getaffinity(0, sizeof saved_, &saved_)) return;
        cpu_set_t l3 = cpus_of(cpu, "cache/index3/shared_cpu_list"), core = cpus_of(cpu, "topology/thread_siblings_list");
        CPU_AND(&l3, &l3, &saved_);
        CPU_AND(&core, &core, &saved_);
        if (!CPU_ISSET(cpu, &core)) return;
        CPU_XOR(&workers_, &l3, &core);  // l3 without the walk's core
        CPU_AND(&workers_, &workers_, &l3);
        if (CPU_COUNT(&workers_) < 1 || CPU_EQUAL(&l3, &saved_)) return;  // one domain already
        if (sched_setaffinity(0, sizeof core, &core)) return;
        pinned_ = true;
    }
    ~CacheDomain() {
        if (pinned_) (void)sched_setaffinity(0, sizeof saved_, &saved_);
    }
    bool pinned() const { return pinned_; }
    int threads() const { return threads_; }
    // worker threads: confine themselves (0 = no limit)
    int workers() const { return pinned_ ? CPU_COUNT(&workers_) : 0; }
    void confine_worker() const {
        if (pinned_) (void)sched_setaffinity(0, sizeof workers_, &workers_);
    }

  private:
    static cpu_set_t cpus_of(int cpu, const char *what) {
        cpu_set_t set;
        CPU_ZERO(&set);
        char path[160];
        std::snprintf(path, sizeof path, "/sys/devices/system/cpu/cpu%d/%s", cpu, what);
        FILE *f = std::fopen(path, "r");
        if (!f) return set;
        char buf[4096];
        const size_t n = std::fread(buf, 1, sizeof buf - 1, f);
        std::fclose(f);
        buf[n] = 0;
        for (char *p = buf; *p;) {  // "a-b,c,..."
            char *end = nullptr;
            const long a = std::strtol(p, &end, 10);
            if (end == p) break;
            long b = a;
            p = end;
            if (*p == '-') {
                b = std::strtol(p + 1, &end, 10);
                p = end;
            }
            for (long k = a; k <= b && k < CPU_SETSIZE; ++k)
                if (k >= 0) CPU_SET((int)k, &set);
            while (*p == ',' || *p == '\n' || *p == ' ') ++p;
        }
        return set;
    }
    int threads_;
    cpu_set_t saved_{}, workers_{};
    bool pinned_ = false;
};

// A persistent pool of acmmp_host_threads() - 1 workers: `submit` hands out
// indices 0..n-1 of a job to whichever worker is free (dynamic rows), `wait`
// blocks until a job is done. The caller's thread stays free for the
// sequential approval walk, which overlaps the next view's candidate phase.
class Pool {
  public:
    struct Job {
        std::function<void(int)> fn;
        int n = 0;
        std::atomic<int> next{0}, done{0};
    };
    explicit Pool(const CacheDomain *dom = nullptr) {
        int nw = std::max(1, (dom ? dom->threads() : acmmp_host_threads()) - 1);
        if (dom && dom->workers() > 0) nw = std::min(nw, dom->workers());
        for (int t = 0; t < nw; ++t)
            workers_.emplace_back([this, dom] {
                if (dom) dom->confine_worker();
                loop();
            });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : workers_) t.join();
    }
    int size() const { return (int)workers_.size(); }
    std::shared_ptr<Job> submit(int n, std::function<void(int)> fn) {
        auto j = std::make_shared<Job>();
        j->fn = std::move(fn);
        j->n = n;
        {
            std::lock_guard<std::mutex> g(mu_);
            jobs_.push_back(j);
        }
        cv_.notify_all();
        return j;
    }
    void wait(const std::shared_ptr<Job> &j) {
        std::unique_lock<std::mutex> g(mu_);
        done_cv_.wait(g, [&] { return j->done.load() == j->n; });
    }

  private:
    void loop() {
        for (;;) {
            std::shared_ptr<Job> j;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return stop_ || !jobs_.empty(); });
                if (stop_ && jobs_.empty()) return;
                j = jobs_.front();
            }
            int i;
            bool any = false;
            while ((i = j->next.fetch_add(1)) < j->n) {
                j->fn(i);
                any = true;
                if (j->done.fetch_add(1) + 1 == j->n) {
                    std::lock_guard<std::mutex> g(mu_);
                    done_cv_.notify_all();
                }
            }
            if (!any) {  // exhausted: retire it from the queue
                std::lock_guard<std::mutex> g(mu_);
                if (!jobs_.empty() && jobs_.front() == j) jobs_.pop_front();
            }
        }
    }
    std::vector<std::thread> workers_;
    std::deque<std::shared_ptr<Job>> jobs_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    bool stop_ = false;
};

// RunFusion's per-view masks as bitsets: a view's ~20 sources' masks then
// stay cache-resident during the approval walk (1 bit instead of 1 byte a
// pixel). The walk is their only writer; the next view's candidate phase
// reads them meanwhile (any value read is exact, see RunFusion): relaxed
// atomic words.
struct MaskBits {
    std::vector<uint64_t> w;
    void assign(size_t n) { w.assign((n + 63) / 64, 0ull); }
    bool get(size_t k) const { return (__atomic_load_n(&w[k >> 6], __ATOMIC_RELAXED) >> (k & 63)) & 1ull; }
    void set(size_t k) {  // single writer
        const uint64_t v = __atomic_load_n(&w[k >> 6], __ATOMIC_RELAXED) | (1ull << (k & 63));
        __atomic_store_n(&w[k >> 6], v, __ATOMIC_RELAXED);
    }
};

// Runs fn(0..n-1) on the pool's workers (the caller waits); returns the
// status of the lowest failing index with its message, as parallel_for does.
template <class Fn>
int pool_for(Pool &pool, int n, Fn fn) {
    std::vector<int> rc((size_t)std::max(n, 0), ACMMP_OK);
    std::vector<std::string> msg(rc.size());
    pool.wait(pool.submit(n, [&](int i) {
        rc[(size_t)i] = fn(i);
        if (rc[(size_t)i]) msg[(size_t)i] = f_err;
    }));
    for (int i = 0; i < n; ++i)
        if (rc[(size_t)i]) {
            f_err = msg[(size_t)i];
            return rc[(size_t)i];
        }
    return ACMMP_OK;
}

// Runs fn(0..n-1) on acmmp_host_threads() threads; returns the status of the lowest
// failing index with its message (what the sequential loop reports first).
template <class Fn>
int parallel_for(int n, Fn fn) {
    const int workers = std::min<int>(n, acmmp_host_threads());
    std::vector<int> rc((size_t)std::max(n, 0), ACMMP_OK);
    std::vector<std::string> msg(rc.size());
    std::atomic<int> next{0};
    auto work = [&]() {
        for (int i; (i = next.fetch_add(1)) < n;) {
            rc[(size_t)i] = fn(i);
            if (rc[(size_t)i]) msg[(size_t)i] = f_err;
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < workers; ++t) pool.emplace_back(work);
    work();
    for (auto &t : pool) t.join();
    for (int i = 0; i < n; ++i)
        if (rc[(size_t)i]) {
            f_err = msg[(size_t)i];
            return rc[(size_t)i];
        }
    return ACMMP_OK;
}

int read_dmb(const std::string &path, std::vector<float> &d, int &h, int &w, int &nb) {
    int32_t hh = 0, ww = 0, bb = 0;
    int rc = acmmp_read_dmb(path.c_str(), &hh, &ww, &bb, nullptr, 0);
    if (rc != ACMMP_OK && rc != ACMMP_ERR_ARG) return ffail(ACMMP_ERR_IO, "cannot read %s", path.c_str());
    d.resize((size_t)hh * ww * bb);
    if (acmmp_read_dmb(path.c_str(), &hh, &ww, &bb, d.data(), d.size()))
        return ffail(ACMMP_ERR_IO, "cannot read %s", path.c_str());
    h = hh;
    w = ww;
    nb = bb;
    return ACMMP_OK;
}

// Float bilinear resize of an 8-bit multi-channel image (half-pixel centres,
// edge clamp, round to nearest) — the unpinned stand-in for cv::resize.
void resize_u8(const std::vector<uint8_t> &src, int sw, int sh, int C, std::vector<uint8_t> &dst, int dw, int dh) {
    dst.resize((size_t)dw * dh * C);
    for (int y = 0; y < dh; ++y) {
        float fy = (float)((y + 0.5) * sh / dh - 0.5);
        int y0 = (int)std::floor(fy);
        float ay = fy - y0;
        if (y0 < 0) { y0 = 0; ay = 0; }
        if (y0 >= sh - 1) { y0 = sh - 1; ay = 0; }
        const int y1 = std::min(y0 + 1, sh - 1);
        for (int x = 0; x < dw; ++x) {
            float fx = (float)((x + 0.5) * sw / dw - 0.5);
            int x0 = (int)std::floor(fx);
            float ax = fx - x0;
            if (x0 < 0) { x0 = 0; ax = 0; }
            if (x0 >= sw - 1) { x0 = sw - 1; ax = 0; }
            const int x1 = std::min(x0 + 1, sw - 1);
            for (int k = 0; k < C; ++k) {
                auto at = [&](int yy, int xx) { return (float)src[((size_t)yy * sw + xx) * C + k]; };
                const float top = at(y0, x0) * (1 - ax) + at(y0, x1) * ax;
                const float bot = at(y1, x0) * (1 - ax) + at(y1, x1) * ax;
                const float v = top * (1 - ay) + bot * ay;
                dst[((size_t)y * dw + x) * C + k] = (uint8_t)std::min(255.0f, std::max(0.0f, std::nearbyint(v)));
            }
        }
    }
}

struct Point {
    F3 coord, normal, color;
};

// StoreColorPlyFileBinaryPointCloud. The 27-byte records (6 floats + r, g, b)
// are formed in chunks of 2^18 points, each written at its own offset: on
// the pool's workers when one is given (RunFusion's pool is idle by then),
// else in order on the caller. Same bytes either way. (ACMMP_PLY_CHUNK_POINTS
// sets the chunk size, so tests reach the chunk boundaries on small clouds.)
constexpr size_t kPlyRec = 6 * sizeof(float) + 3;

size_t ply_chunk_points() {
    const char *e = std::getenv("ACMMP_PLY_CHUNK_POINTS");
    const long long v = e ? std::atoll(e) : 0;
    return v > 0 ? (size_t)v : size_t(1) << 18;
}

int pwrite_all(int fd, const char *p, size_t n, off_t at) {
    while (n) {
        const ssize_t w = ::pwrite(fd, p, n, at);
        if (w <= 0) return -1;
        p += w, n -= (size_t)w, at += w;
    }
    return 0;
}

int store_ply(const std::string &path, const std::vector<Point> &pc, Pool *pool = nullptr) {
    char hdr[512];
    const int hl = std::snprintf(hdr, sizeof(hdr),
                                 "ply\nformat binary_little_endian 1.0\nelement vertex %d\n"
                                 "property float x\nproperty float y\nproperty float z\n"
                                 "property float nx\nproperty float ny\nproperty float nz\n"
                                 "property uchar red\nproperty uchar green\nproperty uchar blue\nend_header\n",
                                 (int)pc.size());
    const int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) return ffail(ACMMP_ERR_IO, "cannot write %s", path.c_str());
    const size_t per = ply_chunk_points();
    const int nchunks = (int)((pc.size() + per - 1) / per);
    auto chunk = [&](int c) -> int {
        const size_t b = (size_t)c * per, e = std::min(pc.size(), b + per);
        std::vector<char> buf((e - b) * kPlyRec);
        char *o = buf.data();
        for (size_t k = b; k < e; ++k, o += kPlyRec) {
            const Point &p = pc[k];
            F3 X = p.coord;
            if (!(X.x < FLT_MAX && X.x > -FLT_MAX) || !(X.y < FLT_MAX && X.y > -FLT_MAX) ||
                !(X.z < FLT_MAX && X.z >= -FLT_MAX)) {
                X.x = X.y = X.z = 0.0f;
            }
            const float v[6] = {X.x, X.y, X.z, p.normal.x, p.normal.y, p.normal.z};
            std::memcpy(o, v, sizeof(v));
            o[24] = (char)(int)p.color.z;  // colour is stored b, g, r; written r, g, b
            o[25] = (char)(int)p.color.y;
            o[26] = (char)(int)p.color.x;
        }
        if (pwrite_all(fd, buf.data(), buf.size(), (off_t)(hl + b * kPlyRec)))
            return ffail(ACMMP_ERR_IO, "cannot write %s", path.c_str());
        return ACMMP_OK;
    };
    int rc = pwrite_all(fd, hdr, (size_t)hl, 0) ? ffail(ACMMP_ERR_IO, "cannot write %s", path.c_str()) : ACMMP_OK;
    if (rc == ACMMP_OK && pool) rc = pool_for(*pool, nchunks, chunk);
    for (int c = 0; rc == ACMMP_OK && !pool && c < nchunks; ++c) rc = chunk(c);
    if (::close(fd) != 0 && rc == ACMMP_OK) rc = ffail(ACMMP_ERR_IO, "cannot write %s", path.c_str());
    return rc;
}

// ---- prior-aware fusion helpers (src/acmmp_definitions.cpp:443-571)
struct CInfo {  // struct c_info
    float dynamic_consistency = 0;
    int x = 0, y = 0;
    bool below_thresh = false;
    int im_num = -1;
};

struct CMetric {  // struct cmetric
    float reproj_err = 1e6, relative_depth_diff = 1e6, angle = 1e6;
};

struct FusionInputs {
    std::vector<acmmp_camera> cameras;
    std::vector<std::vector<float>> depths, normals, pdepths, pnormals;
    std::vector<int> rows, cols;
};

CMetric metric_of(const FusionInputs &in, size_t i, int r, int c, float ref_depth, const float *ref_normal, int src,
                  int src_r, int src_c, float src_depth, const float *src_normal) {
    CMetric m;
    if (src_depth > 0) {
        const F3 tmp_X = world_point(src_c, src_r, src_depth, in.cameras[src]);
        float tx, ty, proj_depth;
        project(tmp_X, in.cameras[i], tx, ty, proj_depth);
        const double dx = (double)(c - tx), dy = (double)(r - ty);  // std::pow(v, 2), exact as v * v
        m.reproj_err = (float)std::sqrt(dx * dx + dy * dy);
        m.relative_depth_diff = std::fabs(proj_depth - ref_depth) / ref_depth;
        m.angle = get_angle(ref_normal, src_normal);
    }
    return m;
}

// get_consistency_metrics (:443-516)
CInfo consistency_metrics(const FusionInputs &in, size_t i, int r, int c, float ref_depth, const float *ref_normal,
                          int src, int src_r, int src_c) {
    const size_t sp = (size_t)src_r * in.cols[src] + src_c;
    const CMetric res0 = metric_of(in, i, r, c, ref_depth, ref_normal, src, src_r, src_c, in.depths[src][sp],
                                   &in.normals[src][sp * 3]);
    const CMetric res1 = metric_of(in, i, r, c, ref_depth, ref_normal, src, src_r, src_c, in.pdepths[src][sp],
                                   &in.pnormals[src][sp * 3]);
    const bool t0 = res0.reproj_err < 2.0f && res0.relative_depth_diff < 0.01f && res0.angle < 0.174533f;
    const bool t1 = res1.reproj_err < 2.0f && res1.relative_depth_diff < 0.01f && res1.angle < 0.174533f;
    CInfo out;
    out.x = src_c;
    out.y = src_r;
    const float dc0 = std::exp(-(res0.reproj_err + 200 * res0.relative_depth_diff + res0.angle * 10));
    const float dc1 = std::exp(-(res1.reproj_err + 200 * res1.relative_depth_diff + res1.angle * 10));
    if (t0 && t1) {
        out.dynamic_consistency = std::fmax(dc0, dc1);
        out.below_thresh = true;
        out.im_num = src;
    } else if (t0) {
        out.dynamic_consistency = dc0;
        out.below_thresh = true;
        out.im_num = src;
    } else if (t1) {
        out.dynamic_consistency = dc1;
        out.below_thresh = true;
        out.im_num = src;
    }
    return out;
}

// getCandidates (:520-571)
void candidates(const FusionInputs &in, const std::vector<std::vector<uint8_t>> &masks, const std::vector<int> &srcs,
                size_t i, int r, int c, float ref_depth, const float *ref_normal, std::vector<CInfo> &out) {
    out.clear();
    for (const int s : srcs) {
        const F3 PointX = world_point(c, r, ref_depth, in.cameras[i]);
        float px, py, proj_depth;
        project(PointX, in.cameras[s], px, py, proj_depth);
        const int src_r = int(py + 0.5f);
        const int src_c = int(px + 0.5f);
        if (src_c >= 0 && src_c < in.cols[s] && src_r >= 0 && src_r < in.rows[s]) {
            if (masks[s][(size_t)src_r * in.cols[s] + src_c] == 1) continue;
            out.push_back(consistency_metrics(in, i, r, c, ref_depth, ref_normal, s, src_r, src_c));
        }
    }
}

}  // namespace


extern "C" {

const char *acmmp_fusion_last_error(void) { return f_err.c_str(); }

int acmmp_run_fusion(const char *dense_folder, const char *output_folder, const acmmp_problem *problems, int count,
                     int geom_consistency, float consistency_scalar, int con_num_thresh, const char *image_dir,
                     const char *mask_folder, int write_debug_images, int *num_points) {
    if (!dense_folder || !output_folder || !problems || count <= 0) return ffail(ACMMP_ERR_ARG, "bad args");
    const std::string dense = dense_folder, out = output_folder;
    const std::string image_folder = dense + (image_dir ? image_dir : "/images");
    const std::string cam_folder = dense + "/cams";
    const bool use_masks = mask_folder && std::string(mask_folder) != " " && mask_folder[0] != 0;
    const size_t n = (size_t)count;
    std::vector<std::vector<uint8_t>> images(n);
    std::vector<MaskBits> masks(n);
    std::vector<acmmp_camera> cameras(n);
    std::vector<std::vector<float>> depths(n), normals(n);
    std::vector<int> rows(n), cols(n);
    std::map<int, int> image_id_2_index;
    for (size_t i = 0; i < n; ++i) image_id_2_index[problems[i].ref_image_id] = (int)i;
    const bool timing = std::getenv("ACMMP_HOST_TIMING") != nullptr;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto secs = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
        return std::chrono::duration<double>(b - a).count();
    };
    const auto t_start = now();
    double t_wait = 0, t_walk = 0;
    size_t n_live = 0, n_hits = 0, n_masked = 0;
    // The threads are confined to one last-level-cache domain BEFORE the
    // loads, and the loads run on that domain's pool: the maps, images and
    // masks are then first touched (allocated) on the memory node of the
    // walk's core, which reads them. (Loaded by threads spread over the whole
    // machine, a 2-socket host put part of them on the other node, and the
    // walk measured 0.85 or 1.3 s from run to run, profiles/r05_fusion_walk_ab3.jsonl.)
    CacheDomain dom;
    Pool pool(&dom);
    // views load independently (JPEG decode, two .dmb reads, optional mask)
    int load_rc = pool_for(pool, (int)n, [&](int vi) -> int {
        const size_t i = (size_t)vi;
        const int id = problems[i].ref_image_id;
        const std::string ipath = image_folder + "/" + id8(id) + ".jpg";
        int iw = 0, ih = 0;
        std::vector<uint8_t> img;
        int rc = acmmp_internal_read_image_bgr(ipath.c_str(), img, iw, ih);
        if (rc) return ffail(rc, "cannot read image %s", ipath.c_str());
        const std::string cpath = cam_folder + "/" + id8(id) + "_cam.txt";
        if (acmmp_read_camera(cpath.c_str(), &cameras[i])) return ffail(ACMMP_ERR_IO, "cannot read %s", cpath.c_str());
        const std::string rf = out + "/2333_" + id8(id);
        int h, w, nb, h2, w2, nb2;
        rc = read_dmb(rf + (geom_consistency ? "/depths_geom.dmb" : "/depths.dmb"), depths[i], h, w, nb);
        if (!rc) rc = read_dmb(rf + "/normals.dmb", normals[i], h2, w2, nb2);
        if (rc) return rc;
        if (nb != 1 || nb2 != 3 || h2 != h || w2 != w) return ffail(ACMMP_ERR_IO, "bad maps for view %d", id);
        rows[i] = h;
        cols[i] = w;
        // RescaleImageAndCamera (src/ACMMP.cpp:181-201)
        if (w == iw && h == ih) {
            images[i] = std::move(img);
        } else {
            const float scale_x = w / static_cast<float>(iw);
            const float scale_y = h / static_cast<float>(ih);
            resize_u8(img, iw, ih, 3, images[i], w, h);
            cameras[i].K[0] *= scale_x;
            cameras[i].K[2] *= scale_x;
            cameras[i].K[4] *= scale_y;
            cameras[i].K[5] *= scale_y;
            cameras[i].width = w;
            cameras[i].height = h;
        }
        masks[i].assign((size_t)w * h);
        if (use_masks) {  // :881-905: mask = (resize(mask) < 128) / 255
            const std::string mpath = dense + "/" + mask_folder + "/" + id8(id) + ".png";
            int mw = 0, mh = 0, mc = 0, bd = 0;
            std::vector<uint16_t> m16;
            rc = acmmp_read_png(mpath.c_str(), nullptr, 0, &mw, &mh, &mc, &bd);
            if (rc == ACMMP_ERR_ARG) {
                m16.resize((size_t)mw * mh * mc);
                rc = acmmp_read_png(mpath.c_str(), m16.data(), m16.size(), &mw, &mh, &mc, &bd);
            }
            if (rc) return ffail(ACMMP_ERR_IO, "Couldn't find mask image %s", mpath.c_str());
            // cv::imread(path, -1) keeps the file's depth and channels (colour
            // as B, G, R[, A], as acmmp_read_png returns them too);
            // `(temp_mask < 128) / 255` keeps the channels,
            // and the walk reads and writes the mask with at<uchar>(r, c):
            // byte c of row r. For a 1-channel mask that is pixel (r, c); for
            // a colour one it is channel c % C of pixel c / C, reproduced here.
            // (2-channel gray+alpha masks use the gray value: unpinned.)
            const bool same = mw == w && mh == h;
            if (bd != 8 && !same)
                return ffail(ACMMP_ERR_UNSUPPORTED, "16-bit mask %s needs resizing", mpath.c_str());
            const int C = mc == 2 ? 1 : mc;
            std::vector<uint16_t> px((size_t)mw * mh * C);
            for (size_t k = 0; k < (size_t)mw * mh; ++k)
                for (int ch = 0; ch < C; ++ch) px[k * C + ch] = m16[k * mc + ch];
            std::vector<uint16_t> mr;
            if (same) {
                mr.swap(px);
            } else {
                std::vector<uint8_t> m8(px.begin(), px.end()), r8;
                resize_u8(m8, mw, mh, C, r8, w, h);
                mr.assign(r8.begin(), r8.end());
            }
            for (int r = 0; r < h; ++r)
                for (int c = 0; c < w; ++c)
                    if (mr[(size_t)r * w * C + c] < 128) masks[i].set((size_t)r * w + c);
        }
        return (int)ACMMP_OK;
    });
    if (load_rc) return load_rc;

    std::vector<std::vector<int>> src_index(n);
    for (size_t i = 0; i < n; ++i)
        for (int j = 0; j < problems[i].num_src_images; ++j) {
            auto it = image_id_2_index.find(problems[i].src_image_ids[j]);
            if (it == image_id_2_index.end())
                return ffail(ACMMP_ERR_ARG, "source %d of view %d is not a problem", problems[i].src_image_ids[j],
                             problems[i].ref_image_id);
            src_index[i].push_back(it->second);
        }
    // Two phases per view, exact to the sequential loop: (1) on the pool,
    // every pixel's per-source projections and consistency tests against
    // the masks as they stand (masks only ever go 0 -> 1, so a source or
    // pixel masked when read stays masked); (2) on this thread, in the
    // reference's pixel order, the sources that passed are re-checked
    // against the current masks and accumulated in ascending j (same exp
    // values, same sum order), then points are emitted and masks / used_list
    // updated. View i + 1's phase 1 runs while view i is walked.
    // A hit = (source slot j, source pixel sp) packed in 32 bits; its
    // exp(-tmp_index) is kept beside it, and every live pixel's sum of them
    // (ascending j, as the walk adds) is precomputed: the walk reads the
    // per-hit values only for pixels where some hit became masked.
    constexpr int kSpBits = 27;
    struct ViewHits {
        std::vector<std::vector<uint32_t>> hit;    // hits of row r, pixel order: j << kSpBits | sp
        std::vector<std::vector<float>> ex;        // their exp(-tmp_index)
        // per live pixel of row r (phase 1's order: ascending column) --
        // the walk visits only these (a pixel not live in phase 1 stays so:
        // masks only go 0 -> 1 and depths do not change)
        std::vector<std::vector<int>> live;        // its column
        std::vector<std::vector<uint16_t>> nhit;   // its number of hits
        std::vector<std::vector<float>> sum;       // sum of its hits' ex, ascending j
        std::vector<std::vector<F3>> X;            // its world point
    };
    for (size_t i = 0; i < n; ++i)
        if ((size_t)cols[i] * rows[i] > (size_t(1) << kSpBits) || problems[i].num_src_images > 32)
            return ffail(ACMMP_ERR_ARG, "view %d: fusion supports images up to 2^27 pixels and 32 sources",
                         problems[i].ref_image_id);
    // Source-major inside a row: every live pixel's world point first, then
    // one source at a time over the row (its depth/normal/mask reads follow
    // the row's projection into that source instead of hopping between 20
    // sources per pixel), then each pixel's hits in ascending j as the
    // reference adds them (same values, same order).
    struct RowScratch {
        std::vector<F3> X;
        std::vector<int> live;           // columns of the live pixels
        std::vector<uint32_t> sp;        // [live k][j]: source pixel of a hit, or kNoHit
        std::vector<float> e;            // [live k][j]: its exp(-tmp_index)
        // one source's pass over the row, in stages (see phase1)
        std::vector<int> src_c, src_r;   // [live k]: the projected source pixel
        std::vector<int> cand;           // live indices whose source pixel is in bounds, unmasked, depth > 0
        std::vector<int> ccol, csc, csr; // ... its column and source pixel
        std::vector<float> cdepth, cref; // ... its source depth and reference depth
        std::vector<float> rerr, rdiff;  // [cand q]: reprojection error, relative depth difference
    };
    constexpr uint32_t kNoHit = 0xffffffffu;
    auto phase1 = [&](size_t i, ViewHits &vh, int r) {
        thread_local RowScratch rs;
        const int W = cols[i];
        const int num_ngb = problems[i].num_src_images;
        const float depth_max = cameras[i].depth_max;
        std::vector<uint32_t> &h = vh.hit[(size_t)r];
        std::vector<float> &hx = vh.ex[(size_t)r];
        std::vector<uint16_t> &nh = vh.nhit[(size_t)r];
        std::vector<float> &sum = vh.sum[(size_t)r];
        std::vector<F3> &X = vh.X[(size_t)r];
        h.clear();
        hx.clear();
        rs.live.clear();
        rs.X.clear();
        for (int c = 0; c < W; ++c) {
            const size_t pc = (size_t)r * W + c;
            if (masks[i].get(pc)) continue;
            const float ref_depth = depths[i][pc];
            if (ref_depth <= 0.0 || ref_depth >= depth_max) continue;
            rs.live.push_back(c);
            rs.X.push_back(world_point(c, r, ref_depth, cameras[i]));
        }
        const size_t nl = rs.live.size();
        const size_t nj = (size_t)std::max(num_ngb, 1);
        rs.sp.assign(nl * nj, kNoHit);
        rs.e.resize(nl * nj);
        nh.resize(nl);
        sum.resize(nl);
        rs.src_c.resize(nl);
        rs.src_r.resize(nl);
        for (int j = 0; j < num_ngb; ++j) {
            const int s = src_index[i][j];
            const int src_cols = cols[s], src_rows = rows[s];
            // Per source, the reference's per-pixel test in four stages over
            // the row's live pixels (the same operations on the same values:
            // the two arithmetic stages are branch-free loops the compiler
            // vectorises; the gathers and the mask reads stay scalar).
            // (1) the projection into the source
            stage_project(rs.X.data(), nl, cameras[s], rs.src_c.data(), rs.src_r.data());
            // (2) in bounds, unmasked, positive source depth: the candidates,
            // with what stage 3 reads, in contiguous arrays
            rs.cand.resize(nl);
            rs.ccol.resize(nl);
            rs.csc.resize(nl);
            rs.csr.resize(nl);
            rs.cdepth.resize(nl);
            rs.cref.resize(nl);
            size_t nc = 0;
            const float *dref = depths[i].data() + (size_t)r * W;
            for (size_t k = 0; k < nl; ++k) {
                const int src_r = rs.src_r[k], src_c = rs.src_c[k];
                if (!(src_c >= 0 && src_c < src_cols && src_r >= 0 && src_r < src_rows)) continue;
                const size_t sp = (size_t)src_r * src_cols + src_c;
                if (masks[s].get(sp)) continue;
                const float src_depth = depths[s][sp];
                if (src_depth <= 0.0) continue;
                rs.cand[nc] = (int)k;
                rs.ccol[nc] = rs.live[k];
                rs.csc[nc] = src_c;
                rs.csr[nc] = src_r;
                rs.cdepth[nc] = src_depth;
                rs.cref[nc] = dref[rs.live[k]];
                ++nc;
            }
            // (3) the reprojection into view i: error and relative depth difference
            rs.rerr.resize(nc);
            rs.rdiff.resize(nc);
            stage_reproject(nc, r, rs.ccol.data(), rs.csc.data(), rs.csr.data(), rs.cdepth.data(), rs.cref.data(),
                            rs.rerr.data(), rs.rdiff.data(), cameras[s], cameras[i]);
            // (4) the reference evaluates all three before the test; acos is
            // pure, so the angle is only formed where the first two pass
            for (size_t q = 0; q < nc; ++q) {
                const float reproj_error = rs.rerr[q], relative_depth_diff = rs.rdiff[q];
                if (!(reproj_error < 2.0f && relative_depth_diff < 0.01f)) continue;
                const int k = rs.cand[q];
                const size_t pc = (size_t)r * W + rs.ccol[q];
                const size_t sp = (size_t)rs.csr[q] * src_cols + rs.csc[q];
                const float angle = get_angle(&normals[i][pc * 3], &normals[s][sp * 3]);
                if (angle < 0.174533f) {
                    const float tmp_index = reproj_error + 200 * relative_depth_diff + angle * 10;
                    rs.sp[(size_t)k * nj + (size_t)j] = (uint32_t)sp;
                    rs.e[(size_t)k * nj + (size_t)j] = std::exp(-tmp_index);
                }
            }
        }
        for (size_t k = 0; k < nl; ++k) {
            const size_t k0 = h.size();
            float total = 0;
            for (int j = 0; j < num_ngb; ++j) {
                const uint32_t sp = rs.sp[k * nj + (size_t)j];
                if (sp == kNoHit) continue;
                const float e = rs.e[k * nj + (size_t)j];
                h.push_back((uint32_t)j << kSpBits | sp);
                hx.push_back(e);
                total += e;
            }
            nh[k] = (uint16_t)(h.size() - k0);
            sum[k] = total;
        }
        // the walk emits an approved pixel's point from here (the same
        // world_point call the reference makes at approval, :1012)
        X.swap(rs.X);
        vh.live[(size_t)r].swap(rs.live);
    };
    std::vector<ViewHits> vhits(2);
    auto start_phase1 = [&](size_t i) {
        ViewHits &vh = vhits[i & 1];
        vh.hit.resize((size_t)rows[i]);
        vh.ex.resize((size_t)rows[i]);
        vh.live.resize((size_t)rows[i]);
        vh.nhit.resize((size_t)rows[i]);
        vh.sum.resize((size_t)rows[i]);
        vh.X.resize((size_t)rows[i]);
        return pool.submit(rows[i], [&, i](int r) { phase1(i, vhits[i & 1], r); });
    };
    std::vector<Point> cloud;
    {  // at most one point per pixel: reserve the address range once (pages
       // are committed as points arrive), no reallocation copies in the walk
        size_t cap = 0;
        for (size_t i = 0; i < n; ++i) cap += (size_t)cols[i] * rows[i];
        cloud.reserve(cap);
    }
    const auto t_loaded = now();
    auto job = start_phase1(0);
    for (size_t i = 0; i < n; ++i) {
        const int W = cols[i], H = rows[i];
        const int num_ngb = problems[i].num_src_images;
        std::vector<uint8_t> approved(write_debug_images ? (size_t)W * H : 0, 0);
        const auto t0 = now();
        pool.wait(job);
        const auto t1 = now();
        t_wait += secs(t0, t1);
        if (i + 1 < n) job = start_phase1(i + 1);
        const ViewHits &vh = vhits[i & 1];
        // per source: its mask words; used_list as mask indices (-1 unset)
        std::vector<uint64_t *> mw((size_t)std::max(num_ngb, 1));
        for (int j = 0; j < num_ngb; ++j) mw[(size_t)j] = masks[(size_t)src_index[i][j]].w.data();
        std::vector<int64_t> used_sp((size_t)std::max(num_ngb, 1), -1);
        uint32_t dirty = 0;  // used_sp entries written since the last approval
        auto bit = [](const uint64_t *w, size_t k) -> bool {
            return (__atomic_load_n(&w[k >> 6], __ATOMIC_RELAXED) >> (k & 63)) & 1ull;
        };
        constexpr uint32_t kSpMask = (1u << kSpBits) - 1;
        for (int r = 0; r < H; ++r) {
            const uint32_t *h = vh.hit[(size_t)r].data();
            const float *hx = vh.ex[(size_t)r].data();
            const std::vector<int> &lv = vh.live[(size_t)r];
            const uint16_t *nhr = vh.nhit[(size_t)r].data();
            const float *sumr = vh.sum[(size_t)r].data();
            const F3 *xr = vh.X[(size_t)r].data();
            const size_t nl = lv.size();
            for (size_t k = 0; k < nl; ++k) {  // the pixels live in phase 1, in column order
                const int c = lv[k];
                const size_t pc = (size_t)r * W + c;
                const int nh = nhr[k];
                const uint32_t *hp = h;
                const float *hxp = hx;
                const F3 *xp = xr + k;
                h += nh;
                hx += nh;
                // re-read: view i - 1's walk (beside view i's phase 1) and,
                // if i is its own source, view i's own approvals set bits
                if (masks[i].get(pc)) continue;
                int num_consistent = 0;
                bool masked = false;
                for (int q = 0; q < nh; ++q) {
                    const uint32_t j = hp[q] >> kSpBits, sp = hp[q] & kSpMask;
                    if (bit(mw[j], sp)) {
                        masked = true;
                        continue;
                    }
                    used_sp[j] = sp;
                    dirty |= 1u << j;
                    num_consistent++;
                }
                float dynamic_consistency = sumr[k];
                n_live++;
                n_hits += (size_t)nh;
                n_masked += masked;
                if (masked) {  // re-add the unmasked ones, ascending j
                    dynamic_consistency = 0;
                    for (int q = 0; q < nh; ++q)
                        if (!bit(mw[hp[q] >> kSpBits], hp[q] & kSpMask)) dynamic_consistency += hxp[q];
                }
                if (num_consistent >= con_num_thresh && (dynamic_consistency > consistency_scalar * num_consistent)) {
                    const float *ref_normal = &normals[i][pc * 3];
                    const uint8_t *bgr = &images[i][pc * 3];
                    Point p;
                    p.coord = *xp;  // world_point(c, r, depths[i][pc], cameras[i]), formed in phase 1
                    p.normal = F3{ref_normal[0], ref_normal[1], ref_normal[2]};
                    p.color = F3{(float)bgr[0], (float)bgr[1], (float)bgr[2]};
                    cloud.push_back(p);
                    // used_list is not reset per pixel in the reference: stale
                    // entries apply too. An entry unchanged since the last
                    // approval was set then (masks only go 0 -> 1), so only
                    // the entries written since are applied.
                    for (; dirty; dirty &= dirty - 1) {
                        const int j = __builtin_ctz(dirty);
                        const int64_t sp = used_sp[(size_t)j];
                        const int s = src_index[i][j];
                        masks[s].set((size_t)sp);
                        if (write_debug_images) {
                            // `approved` is this view's W x H image indexed by source coordinates (:1030)
                            const int ux = (int)(sp % cols[s]), uy = (int)(sp / cols[s]);
                            if (uy < H && ux < W) approved[(size_t)uy * W + ux] = 255;
                        }
                    }
                }
            }
        }
        t_walk += secs(t1, now());
        if (write_debug_images) {
            const std::string dbg = dense + "/approved_pixels_cam_" + std::to_string(i) + ".png";
            if (acmmp_internal_write_png(dbg.c_str(), W, H, 1, approved.data())) {
                if (i + 1 < n) pool.wait(job);
                return ffail(ACMMP_ERR_IO, "cannot write %s", dbg.c_str());
            }
        }
    }
    if (num_points) *num_points = (int)cloud.size();
    const auto t_walked = now();
    const int rc = store_ply(out + "/ACMMP_model.ply", cloud, &pool);
    if (timing)
        std::fprintf(stderr,
                     "[RunFusion] load=%.2fs candidates_wait=%.2fs walk=%.2fs ply=%.2fs threads=%d "
                     "walked_pixels=%zu hits=%zu pixels_with_masked_hits=%zu points=%zu pinned=%d\n",
                     secs(t_start, t_loaded), t_wait, t_walk, secs(t_walked, now()), pool.size() + 1, n_live,
                     n_hits, n_masked, cloud.size(), (int)dom.pinned());
    return rc;
}

int acmmp_run_prior_aware_fusion(const char *dense_folder, const char *output_folder, const char *fusion_folder,
                                 const acmmp_problem *problems, int count, int geom_consistency,
                                 float consistency_scalar, int num_consistent_thresh, int single_match_penalty,
                                 int *num_points) {
    if (!dense_folder || !output_folder || !fusion_folder || !problems || count <= 0)
        return ffail(ACMMP_ERR_ARG, "bad args");
    const std::string dense = dense_folder, out = output_folder, fus = fusion_folder;
    const size_t n = (size_t)count;
    FusionInputs in;
    in.cameras.resize(n);
    in.depths.resize(n);
    in.normals.resize(n);
    in.pdepths.resize(n);
    in.pnormals.resize(n);
    in.rows.resize(n);
    in.cols.resize(n);
    std::vector<std::vector<uint8_t>> images(n), masks(n);
    std::map<int, int> image_id_2_index;
    const char *suffix = geom_consistency ? "/depths_geom.dmb" : "/depths.dmb";
    for (size_t i = 0; i < n; ++i) {
        const int id = problems[i].ref_image_id;
        image_id_2_index[id] = (int)i;
        const std::string ipath = dense + "/images/" + id8(id) + ".jpg";
        int iw = 0, ih = 0;
        std::vector<uint8_t> img;
        int rc = acmmp_internal_read_image_bgr(ipath.c_str(), img, iw, ih);
        if (rc) return ffail(rc, "cannot read image %s", ipath.c_str());
        const std::string cpath = dense + "/cams/" + id8(id) + "_cam.txt";
        if (acmmp_read_camera(cpath.c_str(), &in.cameras[i]))
            return ffail(ACMMP_ERR_IO, "cannot read %s", cpath.c_str());
        // maps of the other reconstruction (fusion_folder) and of this run's (output_folder) priors
        const std::string rf = fus + "/2333_" + id8(id), pf = out + "/2333_" + id8(id);
        int h, w, nb, h2, w2, nb2, h3, w3, nb3, h4, w4, nb4;
        rc = read_dmb(rf + suffix, in.depths[i], h, w, nb);
        if (!rc) rc = read_dmb(rf + "/normals.dmb", in.normals[i], h2, w2, nb2);
        if (!rc) rc = read_dmb(pf + suffix, in.pdepths[i], h3, w3, nb3);
        if (!rc) rc = read_dmb(pf + "/normals.dmb", in.pnormals[i], h4, w4, nb4);
        if (rc) return rc;
        if (nb != 1 || nb2 != 3 || nb3 != 1 || nb4 != 3 || h2 != h || w2 != w || h3 != h || w3 != w || h4 != h ||
            w4 != w)
            return ffail(ACMMP_ERR_IO, "map sizes of view %d disagree", id);
        in.rows[i] = h;
        in.cols[i] = w;
        if (w == iw && h == ih) {
            images[i] = std::move(img);
        } else {
            const float scale_x = w / static_cast<float>(iw);
            const float scale_y = h / static_cast<float>(ih);
            resize_u8(img, iw, ih, 3, images[i], w, h);
            in.cameras[i].K[0] *= scale_x;
            in.cameras[i].K[2] *= scale_x;
            in.cameras[i].K[4] *= scale_y;
            in.cameras[i].K[5] *= scale_y;
        }
        // mask files give 255/0 here (:654-661), never the 1 the checks test:
        // only approvals mask pixels
        masks[i].assign((size_t)w * h, 0);
    }
    std::vector<Point> cloud;
    {  // at most one point per pixel (see RunFusion)
        size_t cap = 0;
        for (size_t i = 0; i < n; ++i) cap += (size_t)in.cols[i] * in.rows[i];
        cloud.reserve(cap);
    }
    Pool pool;
    // Same two-phase scheme as RunFusion: candidates (projection + metrics of
    // both maps) per band of rows on host threads against the current masks,
    // then the reference's pixel order with every approval re-checked
    // against the masks as they stand then (they only ever go 0 -> 1).
    struct Ok {  // a below-threshold candidate: the only kind that counts or masks
        int im, x, y;
        float dc;
    };
    const int band = 32;
    for (size_t i = 0; i < n; ++i) {
        const int W = in.cols[i], H = in.rows[i];
        std::vector<int> srcs;
        for (int j = 0; j < problems[i].num_src_images; ++j) {
            auto it = image_id_2_index.find(problems[i].src_image_ids[j]);
            if (it == image_id_2_index.end()) return ffail(ACMMP_ERR_ARG, "source is not a problem");
            srcs.push_back(it->second);
        }
        const int ns = std::max((int)srcs.size(), 1);
        // per pixel: bit 0 live, bit 1 map 0 evaluated, bit 2 map 1 evaluated
        std::vector<uint8_t> state((size_t)band * W);
        std::vector<uint8_t> cnt((size_t)band * W * 2);
        std::vector<Ok> oks((size_t)band * W * 2 * ns);
        for (int r0 = 0; r0 < H; r0 += band) {
            const int r1 = std::min(H, r0 + band);
            pool.wait(pool.submit(r1 - r0, [&](int rr) {
                const int r = r0 + rr;
                std::vector<CInfo> cand;
                for (int c = 0; c < W; ++c) {
                    const size_t pc = (size_t)r * W + c, q = (size_t)rr * W + c;
                    state[q] = 0;
                    if (masks[i][pc] == 1) continue;
                    const float ref_depth = in.depths[i][pc], ref_p_depth = in.pdepths[i][pc];
                    if (ref_depth <= 0.0 && ref_p_depth <= 0.0) continue;
                    uint8_t st = 1;
                    for (int b = 0; b < 2; ++b) {
                        const float d = b ? ref_p_depth : ref_depth;
                        cnt[2 * q + b] = 0;
                        if (!(d > 0.0)) continue;
                        st |= (uint8_t)(2 << b);
                        candidates(in, masks, srcs, i, r, c, d, b ? &in.pnormals[i][pc * 3] : &in.normals[i][pc * 3],
                                   cand);
                        Ok *o = &oks[(2 * q + b) * ns];
                        int k = 0;
                        for (const CInfo &ci : cand)
                            if (ci.below_thresh) o[k++] = Ok{ci.im_num, ci.x, ci.y, ci.dynamic_consistency};
                        cnt[2 * q + b] = (uint8_t)k;
                    }
                    state[q] = st;
                }
            }));
            for (int r = r0; r < r1; ++r) {
                for (int c = 0; c < W; ++c) {
                    const size_t pc = (size_t)r * W + c, q = (size_t)(r - r0) * W + c;
                    if (!state[q] || masks[i][pc] == 1) continue;
                    const float ref_depth = in.depths[i][pc], ref_p_depth = in.pdepths[i][pc];
                    const float *ref_normal = &in.normals[i][pc * 3], *ref_p_normal = &in.pnormals[i][pc * 3];
                    float d_cons[2] = {0, 0};
                    int nb[2] = {0, 0};
                    bool t[2] = {false, false};
                    for (int b = 0; b < 2; ++b) {
                        if (!(state[q] & (2 << b))) continue;
                        Ok *o = &oks[(2 * q + b) * ns];
                        int keep = 0;
                        for (int k = 0; k < cnt[2 * q + b]; ++k) {
                            if (masks[o[k].im][(size_t)o[k].y * in.cols[o[k].im] + o[k].x] == 1) continue;
                            nb[b]++;
                            d_cons[b] += o[k].dc;
                            o[keep++] = o[k];
                        }
                        cnt[2 * q + b] = (uint8_t)keep;
                        t[b] = (nb[b] >= num_consistent_thresh) && (d_cons[b] > consistency_scalar * nb[b]);
                    }
                    int pick = 0;
                    bool passing = false;
                    float g_depth = 0;
                    const float *g_normal = ref_normal;
                    if (t[0] && t[1]) {  // (:754-769)
                        passing = true;
                        pick = nb[1] >= nb[0] ? 1 : 0;
                    } else if (t[1]) {
                        passing = nb[1] >= (num_consistent_thresh + single_match_penalty);
                        pick = 1;
                    } else {
                        passing = t[0] && nb[0] >= (num_consistent_thresh + single_match_penalty);
                        pick = 0;
                    }
                    g_depth = pick ? ref_p_depth : ref_depth;
                    g_normal = pick ? ref_p_normal : ref_normal;
                    if (passing) {
                        Point p;
                        p.coord = world_point(c, r, g_depth, in.cameras[i]);
                        p.normal = F3{g_normal[0], g_normal[1], g_normal[2]};
                        const uint8_t *bgr = &images[i][pc * 3];
                        p.color = F3{(float)bgr[0], (float)bgr[1], (float)bgr[2]};
                        cloud.push_back(p);
                        const Ok *o = &oks[(2 * q + pick) * ns];
                        for (int k = 0; k < cnt[2 * q + pick]; ++k)
                            masks[o[k].im][(size_t)o[k].y * in.cols[o[k].im] + o[k].x] = 1;
                    }
                }
            }
        }
    }
    if (num_points) *num_points = (int)cloud.size();
    return store_ply(out + "/ACMMP_prior_model.ply", cloud);
}

}  // extern "C"
