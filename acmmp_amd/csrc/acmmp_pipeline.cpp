// acmmp_pipeline.cpp — the reference's pass driver around RunPatchMatch, in
// C++ over the library's own C-ABI (through include/acmmp.hpp):
//
//   GenerateSampleList          src/acmmp_definitions.cpp:179-205
//   ComputeMultiScaleSettings   src/acmmp_definitions.cpp:207-243
//   InputInitialization         src/ACMMP.cpp:525-636
//   CudaSpaceInitialization     src/ACMMP.cpp:638-809 (previous-pass loading)
//   ProcessProblem              src/acmmp_definitions.cpp:245-403
//   JointBilateralUpsampling    src/acmmp_definitions.cpp:405-438 + RunJBU src/ACMMP.cpp:1008-1087
//
// File formats and names are the reference's, so an existing output folder,
// fuse_data and later passes interoperate unchanged. Images are
// `%08d.jpg` (decoded by acmmp_image.cpp); `%08d.pgm` / `%08d.pfm` are accepted
// when no .jpg exists. Errors are status codes + acmmp_pipeline_last_error().
#include <sys/stat.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <list>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/acmmp.hpp"
#include "acmmp_hostio.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

std::string id8(int id) {
    char b[32];
    std::snprintf(b, sizeof(b), "%08d", id);
    return b;
}

bool exists(const std::string &p) {
    struct stat st;
    return ::stat(p.c_str(), &st) == 0;
}

std::string result_folder(const std::string &out, int ref_id) { return out + "/2333_" + id8(ref_id); }

std::string image_path(const std::string &dense, int id) {
    const std::string base = dense + "/images/" + id8(id);
    for (const char *ext : {".jpg", ".pgm", ".pfm"})
        if (exists(base + ext)) return base + ext;
    return base + ".jpg";
}

// Decoded-image cache. The reference re-reads and re-decodes every image of a
// problem in every pass (src/ACMMP.cpp:536-574: each view is decoded about
// N times per pass); here a decode is kept, keyed by path and the file's
// inode, size, mtime and ctime (so a rewritten file is decoded again), up to
// ACMMP_IMAGE_CACHE_MB (default 1024: one scale of a 49-view 1600x1200 DTU
// scan; 0 disables) with LRU eviction.
struct ImageCache {
    struct Entry {
        std::string key;
        acmmp::Image im;
    };
    std::mutex mu;
    std::list<Entry> lru;  // front = least recently used
    std::map<std::string, std::list<Entry>::iterator> index;
    size_t bytes = 0, cap = 0;
    ImageCache() {
        const char *e = std::getenv("ACMMP_IMAGE_CACHE_MB");
        cap = (size_t)(e ? std::max(0L, std::atol(e)) : 1024L) << 20;
    }
    bool get(const std::string &key, acmmp::Image &out) {
        std::lock_guard<std::mutex> g(mu);
        auto it = index.find(key);
        if (it == index.end()) return false;
        lru.splice(lru.end(), lru, it->second);
        out = it->second->im;
        return true;
    }
    void put(const std::string &key, const acmmp::Image &im) {
        const size_t b = im.data.size() * sizeof(float);
        std::lock_guard<std::mutex> g(mu);
        if (b > cap || index.count(key)) return;
        while (bytes + b > cap && !lru.empty()) {
            bytes -= lru.front().im.data.size() * sizeof(float);
            index.erase(lru.front().key);
            lru.pop_front();
        }
        lru.push_back(Entry{key, im});
        index[key] = std::prev(lru.end());
        bytes += b;
    }
};

ImageCache &image_cache() {
    static ImageCache c;
    return c;
}

int load_image(const std::string &path, acmmp::Image &im) {
    struct stat st;
    std::string key;
    if (::stat(path.c_str(), &st) == 0) {
        // st_ctim too: utime() cannot set it and every write changes it, so a
        // rewrite that keeps the size and restores the mtime is still seen
        char b[160];
        std::snprintf(b, sizeof(b), "|%llu|%lld|%lld.%09ld|%lld.%09ld", (unsigned long long)st.st_ino,
                      (long long)st.st_size, (long long)st.st_mtim.tv_sec, (long)st.st_mtim.tv_nsec,
                      (long long)st.st_ctim.tv_sec, (long)st.st_ctim.tv_nsec);
        key = path + b;
        if (image_cache().get(key, im)) return ACMMP_OK;
    }
    int w = 0, h = 0;
    int rc = acmmp_image_size(path.c_str(), &w, &h);
    if (rc) return fail(rc, "cannot read image %s", path.c_str());
    im.cols = w;
    im.rows = h;
    im.data.resize((size_t)w * h);
    rc = acmmp_read_image_gray(path.c_str(), im.data.data(), im.data.size(), &w, &h);
    if (rc) return fail(rc, "cannot decode image %s (baseline JPEG / PGM / PFM only)", path.c_str());
    if (!key.empty()) image_cache().put(key, im);
    return ACMMP_OK;
}

int read_dmb(const std::string &path, std::vector<float> &data, int &h, int &w, int &nb) {
    int32_t hh = 0, ww = 0, bb = 0;
    int rc = acmmp_read_dmb(path.c_str(), &hh, &ww, &bb, nullptr, 0);
    if (rc != ACMMP_OK && rc != ACMMP_ERR_ARG) return fail(ACMMP_ERR_IO, "cannot read %s", path.c_str());
    data.resize((size_t)hh * ww * bb);
    rc = acmmp_read_dmb(path.c_str(), &hh, &ww, &bb, data.data(), data.size());
    if (rc) return fail(ACMMP_ERR_IO, "cannot read %s", path.c_str());
    h = hh;
    w = ww;
    nb = bb;
    return ACMMP_OK;
}

int write_dmb(const std::string &path, int h, int w, int nb, const float *data) {
    if (acmmp_write_dmb(path.c_str(), h, w, nb, data)) return fail(ACMMP_ERR_IO, "cannot write %s", path.c_str());
    return ACMMP_OK;
}

// ---- triangulation.png (src/acmmp_definitions.cpp:310-330): the reference
// image as BGR with the triangle edges drawn in red, 1-px 8-connected lines.
int write_png8(const std::string &path, int w, int h, int channels, const uint8_t *px) {
    if (acmmp_internal_write_png(path.c_str(), w, h, channels, px))
        return fail(ACMMP_ERR_IO, "cannot write %s", path.c_str());
    return ACMMP_OK;
}

void draw_line(std::vector<uint8_t> &rgb, int w, int h, acmmp::Point a, acmmp::Point b) {
    int x0 = a.x, y0 = a.y;
    const int dx = std::abs(b.x - x0), dy = -std::abs(b.y - y0);
    const int sx = x0 < b.x ? 1 : -1, sy = y0 < b.y ? 1 : -1;
    int e = dx + dy;
    for (;;) {
        if (x0 >= 0 && x0 < w && y0 >= 0 && y0 < h) {
            uint8_t *p = &rgb[((size_t)y0 * w + x0) * 3];
            p[0] = 255;
            p[1] = 0;
            p[2] = 0;
        }
        if (x0 == b.x && y0 == b.y) break;
        const int e2 = 2 * e;
        if (e2 >= dy) {
            e += dy;
            x0 += sx;
        }
        if (e2 <= dx) {
            e += dx;
            y0 += sy;
        }
    }
}

// The triangulation picture of ProcessProblem (:301-331): the support points'
// Delaunay triangles drawn on the reference image. Returns the picture and
// the triangles (x1 y1 x2 y2 x3 y3 each), which the planar prior is built
// from too, as the reference builds both from one triangulation.
void triangulation_picture(acmmp::ACMMP &acmmp, std::vector<uint8_t> &rgb, std::vector<int32_t> &flat) {
    const int W = acmmp.GetReferenceImageWidth(), H = acmmp.GetReferenceImageHeight();
    const acmmp::Image ref = acmmp.GetReferenceImage();
    std::vector<acmmp::Point> pts;
    acmmp.GetSupportPoints(pts);
    const auto tris = acmmp.DelaunayTriangulation(W, H, pts);
    rgb.assign((size_t)W * H * 3, 0);
    for (size_t i = 0; i < (size_t)W * H; ++i) {
        const float v = std::nearbyint(std::min(255.0f, std::max(0.0f, ref.data[i])));
        rgb[3 * i] = rgb[3 * i + 1] = rgb[3 * i + 2] = (uint8_t)v;
    }
    flat.clear();
    flat.reserve(tris.size() * 6);
    for (const auto &t : tris) {
        draw_line(rgb, W, H, t.pt1, t.pt2);
        draw_line(rgb, W, H, t.pt1, t.pt3);
        draw_line(rgb, W, H, t.pt2, t.pt3);
        flat.insert(flat.end(), {t.pt1.x, t.pt1.y, t.pt2.x, t.pt2.y, t.pt3.x, t.pt3.y});
    }
}

// Runs fn(0..n-1) on acmmp_host_threads() threads. Returns the status of the lowest
// failing index and leaves its message in this thread's error slot, so the
// caller sees what the sequential loop would have reported first.
template <class Fn>
int parallel_views(int n, Fn fn) {
    const int workers = std::min<int>(n, acmmp_host_threads());
    std::vector<int> rc((size_t)n, ACMMP_OK);
    std::vector<std::string> msg((size_t)n);
    std::atomic<int> next{0};
    auto work = [&]() {
        for (int i; (i = next.fetch_add(1)) < n;) {
            rc[(size_t)i] = fn(i);
            if (rc[(size_t)i]) msg[(size_t)i] = g_err;
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < workers; ++t) pool.emplace_back(work);
    work();
    for (auto &t : pool) t.join();
    for (int i = 0; i < n; ++i)
        if (rc[(size_t)i]) {
            g_err = msg[(size_t)i];
            return rc[(size_t)i];
        }
    return ACMMP_OK;
}

// One view of InputInitialization (src/ACMMP.cpp:536-598): image + camera,
// camera size from the image, rescaled to max_image_size when larger.
int load_view(const std::string &dense, int id, int max_image_size, acmmp::Image &im, acmmp_camera &cam) {
    int rc = load_image(image_path(dense, id), im);
    if (rc) return rc;
    const std::string cam_path = dense + "/cams/" + id8(id) + "_cam.txt";
    rc = acmmp_read_camera(cam_path.c_str(), &cam);
    if (rc) return fail(rc, "cannot read camera %s", cam_path.c_str());
    cam.height = im.rows;
    cam.width = im.cols;
    if (im.cols <= max_image_size && im.rows <= max_image_size) return ACMMP_OK;
    const float factor_x = static_cast<float>(max_image_size) / im.cols;
    const float factor_y = static_cast<float>(max_image_size) / im.rows;
    const float factor = std::min(factor_x, factor_y);
    const int new_cols = (int)std::round(im.cols * factor);
    const int new_rows = (int)std::round(im.rows * factor);
    const float scale_x = new_cols / static_cast<float>(im.cols);
    const float scale_y = new_rows / static_cast<float>(im.rows);
    acmmp::Image scaled;
    scaled.cols = new_cols;
    scaled.rows = new_rows;
    scaled.data.resize((size_t)new_cols * new_rows);
    acmmp_resize_linear(im.data.data(), im.cols, im.rows, scaled.data.data(), new_cols, new_rows);
    im = std::move(scaled);
    cam.K[0] *= scale_x;
    cam.K[2] *= scale_x;
    cam.K[4] *= scale_y;
    cam.K[5] *= scale_y;
    cam.height = new_rows;
    cam.width = new_cols;
    return ACMMP_OK;
}

// ---- pSampler (src/acmmp_definitions.cpp:8-177): seeded plane priors from
// 16-bit PNG depth / normal maps under <dense>priors/{depths,normals}/%08d.png
// (the reference concatenates "priors" to dense_folder without a separator).
std::string prior_path(const std::string &dense, const char *kind, int cam) {
    return dense + "priors/" + kind + "/" + id8(cam) + ".png";
}

bool read_png(const std::string &path, std::vector<uint16_t> &px, int &w, int &h, int &c) {
    int bd = 0;
    if (acmmp_read_png(path.c_str(), nullptr, 0, &w, &h, &c, &bd) != ACMMP_ERR_ARG) return false;
    px.resize((size_t)w * h * c);
    return acmmp_read_png(path.c_str(), px.data(), px.size(), &w, &h, &c, &bd) == ACMMP_OK;
}

// depth_normal_to_plane (:72-89) with getViewDirection, normVec3 (which
// multiplies by the norm instead of dividing: kept) and distance_to_origin.
void depth_normal_to_plane(float depth, float nx, float ny, float nz, int px, int py, const acmmp_camera &cam,
                           float *out) {
    const float X0 = depth * (px - cam.K[2]) / cam.K[0];
    const float X1 = depth * (py - cam.K[5]) / cam.K[4];
    const float X2 = depth;
    const float norm = std::sqrt(X0 * X0 + X1 * X1 + X2 * X2);
    const float v0 = X0 / norm, v1 = X1 / norm, v2 = X2 / norm;
    const float dot = nx * v0 + ny * v1 + nz * v2;
    if (dot > 0.0f) {
        nx = -nx;
        ny = -ny;
        nz = -nz;
    }
    const float n2 = nx * nx + ny * ny + nz * nz;
    const float s = std::sqrt(n2);
    nx *= s;
    ny *= s;
    nz *= s;
    out[0] = nx;
    out[1] = ny;
    out[2] = nz;
    out[3] = -(nx * X0 + ny * X1 + nz * X2);
}

}  // namespace

extern "C" {

int acmmp_priors_available(const char *dense_folder, int num_cams) {
    if (!dense_folder || num_cams <= 0) return 0;
    std::vector<uint16_t> px;
    int w, h, c;
    return read_png(prior_path(dense_folder, "depths", num_cams - 1), px, w, h, c) &&
           read_png(prior_path(dense_folder, "normals", num_cams - 1), px, w, h, c);
}

int acmmp_prior_plane_estimate(const char *dense_folder, int cam_num, const acmmp_camera *cam, int rows, int cols,
                               float *planes4) {
    if (!dense_folder || !cam || rows <= 0 || cols <= 0 || !planes4) return fail(ACMMP_ERR_ARG, "bad args");
    std::vector<uint16_t> dpx, npx;
    int dw, dh, dc, nw, nh, nc;
    const std::string dp = prior_path(dense_folder, "depths", cam_num), np = prior_path(dense_folder, "normals", cam_num);
    if (!read_png(dp, dpx, dw, dh, dc) || !read_png(np, npx, nw, nh, nc))
        return fail(ACMMP_ERR_IO, "failed to load prior images: %d (%s)", cam_num, dp.c_str());
    if (nc != 3) return fail(ACMMP_ERR_UNSUPPORTED, "prior normal map %s has %d channels", np.c_str(), nc);
    // Mat::convertTo(CV_32F, alpha, beta): src * alpha + beta in float
    const float dist = cam->depth_max - cam->depth_min;
    const float range = dist / 65535.0f;
    const float nalpha = (float)(2.0 / 65536.0), nbeta = -1.0f;
    const int scale = dh / rows;  // src/acmmp_definitions.cpp:126
    for (int i = 0; i < rows; ++i)
        for (int j = 0; j < cols; ++j) {
            const int r = i * scale, c = j * scale;
            // Mat_<float>::at(r, c) on the (possibly multi-channel) depth map
            const size_t di = (size_t)r * dw * dc + c;
            const size_t ni = ((size_t)r * nw + c) * 3;
            if (r >= dh || di >= dpx.size() || r >= nh || c >= nw)
                return fail(ACMMP_ERR_ARG, "prior maps %dx%d smaller than %dx%d", dw, dh, cols, rows);
            const float base_d = (float)dpx[di] * range + cam->depth_min;
            const float nx = (float)npx[ni] * nalpha + nbeta;
            const float ny = (float)npx[ni + 1] * nalpha + nbeta;
            const float nz = (float)npx[ni + 2] * nalpha + nbeta;
            depth_normal_to_plane(base_d, nx, ny, nz, j, i, *cam, planes4 + ((size_t)i * cols + j) * 4);
        }
    return ACMMP_OK;
}

int acmmp_load_view(const char *dense_folder, int image_id, int max_image_size, float *out, size_t capacity,
                    acmmp_camera *cam) {
    if (!dense_folder || !cam || max_image_size <= 0) return fail(ACMMP_ERR_ARG, "bad args");
    acmmp::Image im;
    const int rc = load_view(dense_folder, image_id, max_image_size, im, *cam);
    if (rc) return rc;
    if (!out || capacity < im.data.size()) return ACMMP_ERR_ARG;  // *cam carries the size
    std::memcpy(out, im.data.data(), im.data.size() * sizeof(float));
    return ACMMP_OK;
}

const char *acmmp_pipeline_last_error(void) { return g_err.c_str(); }

int acmmp_generate_sample_list(const char *dense_folder, acmmp_problem *problems, int capacity, int *count) {
    if (!dense_folder || !count || capacity < 0 || (capacity > 0 && !problems)) return fail(ACMMP_ERR_ARG, "bad args");
    const std::string path = std::string(dense_folder) + "/pair.txt";
    std::ifstream file(path);
    if (!file.is_open()) return fail(ACMMP_ERR_IO, "cannot open %s", path.c_str());
    int num_images = 0;
    file >> num_images;
    if (file.fail() || num_images < 0) return fail(ACMMP_ERR_IO, "bad header in %s", path.c_str());
    *count = num_images;
    if (num_images > capacity) return fail(ACMMP_ERR_ARG, "%d problems exceed capacity %d", num_images, capacity);
    for (int i = 0; i < num_images; ++i) {
        acmmp_problem pr;
        std::memset(&pr, 0, sizeof(pr));
        pr.max_image_size = 6400;  // struct Problem defaults (src/acmmp_definitions.h:57-63)
        pr.cur_image_size = 6400;
        int num_src = 0;
        file >> pr.ref_image_id >> num_src;
        for (int j = 0; j < num_src; ++j) {
            int id = 0;
            float score = 0.0f;
            file >> id >> score;
            if (score <= 0.0f) continue;
            if (pr.num_src_images == ACMMP_MAX_IMAGES - 1)
                return fail(ACMMP_ERR_UNSUPPORTED, "view %d: more than %d sources", pr.ref_image_id,
                            ACMMP_MAX_IMAGES - 1);
            pr.src_image_ids[pr.num_src_images++] = id;
        }
        if (file.fail()) return fail(ACMMP_ERR_IO, "truncated %s", path.c_str());
        problems[i] = pr;
    }
    return ACMMP_OK;
}

int acmmp_compute_multiscale_settings(const char *dense_folder, acmmp_problem *problems, int count,
                                      int *max_num_downscale) {
    if (!dense_folder || !problems || count < 0 || !max_num_downscale) return fail(ACMMP_ERR_ARG, "bad args");
    acmmp_params pmp;
    acmmp_default_params(&pmp);
    const int size_bound = 1000;
    int best = -1;
    for (int i = 0; i < count; ++i) {
        const std::string path = image_path(dense_folder, problems[i].ref_image_id);
        int cols = 0, rows = 0;
        const int rc = acmmp_image_size(path.c_str(), &cols, &rows);
        if (rc) return fail(rc, "cannot read image %s", path.c_str());
        int max_size = std::max(rows, cols);
        if (max_size > pmp.max_image_size) max_size = pmp.max_image_size;
        problems[i].max_image_size = max_size;
        int k = 0;
        while (max_size > size_bound) {
            max_size /= 2;
            k++;
        }
        best = std::max(best, k);
        problems[i].num_downscale = k;
    }
    *max_num_downscale = best;
    return ACMMP_OK;
}

int acmmp_input_initialization(acmmp_ctx *ctx, const char *dense_folder, const char *output_folder,
                               const acmmp_problem *problems, int count, int idx) {
    if (!ctx || !dense_folder || !output_folder || !problems || idx < 0 || idx >= count)
        return fail(ACMMP_ERR_ARG, "bad args");
    const acmmp_problem &pr = problems[idx];
    const std::string dense = dense_folder;
    const int n = 1 + pr.num_src_images;
    if (n < 2 || n > ACMMP_MAX_IMAGES) return fail(ACMMP_ERR_ARG, "view %d has %d sources", pr.ref_image_id, n - 1);
    std::vector<acmmp::Image> images((size_t)n);
    std::vector<acmmp_camera> cams((size_t)n);
    // a source view uses the cur_image_size of the problem indexed by its
    // image id, as the reference does (src/ACMMP.cpp:564-568)
    for (int i = 1; i < n; ++i) {
        const int id = pr.src_image_ids[i - 1];
        if (id < 0 || id >= count)
            return fail(ACMMP_ERR_ARG, "source id %d is not a problem index (pair.txt ids must be 0..n-1)", id);
    }
    // the n decodes (+ resizes) are independent: host threads, results and
    // the first error in view order identical to the sequential loop
    int rc = parallel_views(n, [&](int i) {
        const int id = i == 0 ? pr.ref_image_id : pr.src_image_ids[i - 1];
        const int max_image_size = i == 0 ? pr.cur_image_size : problems[id].cur_image_size;
        return load_view(dense, id, max_image_size, images[(size_t)i], cams[(size_t)i]);
    });
    if (rc) return rc;
    std::vector<const float *> ptrs((size_t)n);
    for (int i = 0; i < n; ++i) ptrs[(size_t)i] = images[(size_t)i].data.data();
    rc = acmmp_set_images(ctx, n, cams.data(), ptrs.data(), 0);  // depth range x0.6 / x1.2 (:600-605)
    if (rc) return fail(rc, "%s", acmmp_last_error(ctx));
    acmmp_params p;
    acmmp_get_params(ctx, &p);
    if (p.geom_consistency) {  // :608-635
        const std::string suffix = p.multi_geometry ? "/depths_geom.dmb" : "/depths.dmb";
        std::vector<std::vector<float>> depths((size_t)n);
        rc = parallel_views(n, [&](int i) {
            const int id = i == 0 ? pr.ref_image_id : pr.src_image_ids[i - 1];
            int h = 0, w = 0, nb = 0;
            const int r = read_dmb(result_folder(output_folder, id) + suffix, depths[(size_t)i], h, w, nb);
            if (r) return r;
            if (nb != 1 || h != cams[(size_t)i].height || w != cams[(size_t)i].width)
                return fail(ACMMP_ERR_IO, "depth map of view %d is %dx%dx%d, image is %dx%d", id, w, h, nb,
                            cams[(size_t)i].width, cams[(size_t)i].height);
            return (int)ACMMP_OK;
        });
        if (rc) return rc;
        for (int i = 0; i < n; ++i) ptrs[(size_t)i] = depths[(size_t)i].data();
        rc = acmmp_set_depth_maps(ctx, ptrs.data());
        if (rc) return fail(rc, "%s", acmmp_last_error(ctx));
    }
    return ACMMP_OK;
}

int acmmp_space_initialization(acmmp_ctx *ctx, const char *output_folder, const acmmp_problem *problem) {
    if (!ctx || !output_folder || !problem) return fail(ACMMP_ERR_ARG, "bad args");
    acmmp_params p;
    acmmp_get_params(ctx, &p);
    int W = 0, H = 0;
    acmmp_get_reference_size(ctx, &W, &H);
    const std::string folder = result_folder(output_folder, problem->ref_image_id);
    if (p.geom_consistency) {  // src/ACMMP.cpp:707-742
        const std::string suffix = p.multi_geometry ? "/depths_geom.dmb" : "/depths.dmb";
        std::vector<float> d, nrm, c;
        int h = 0, w = 0, nb = 0, h2 = 0, w2 = 0, nb2 = 0, h3 = 0, w3 = 0, nb3 = 0;
        int rc = read_dmb(folder + suffix, d, h, w, nb);
        if (!rc) rc = read_dmb(folder + "/normals.dmb", nrm, h2, w2, nb2);
        if (!rc) rc = read_dmb(folder + "/costs.dmb", c, h3, w3, nb3);
        if (rc) return rc;
        if (h != H || w != W || h2 != H || w2 != W || nb2 != 3 || h3 != H || w3 != W)
            return fail(ACMMP_ERR_IO, "previous-pass maps of view %d do not match %dx%d", problem->ref_image_id, W, H);
        std::vector<float> planes((size_t)W * H * 4);
        for (size_t i = 0; i < (size_t)W * H; ++i) {
            planes[4 * i] = nrm[3 * i];
            planes[4 * i + 1] = nrm[3 * i + 1];
            planes[4 * i + 2] = nrm[3 * i + 2];
            planes[4 * i + 3] = d[i];
        }
        rc = acmmp_set_plane_hypotheses(ctx, planes.data(), c.data());
        if (rc) return fail(rc, "%s", acmmp_last_error(ctx));
    }
    if (p.hierarchy) {  // :745-808
        std::vector<float> d, nrm, c;
        int h = 0, w = 0, nb = 0, sh = 0, sw = 0, nb2 = 0, h3 = 0, w3 = 0, nb3 = 0;
        int rc = read_dmb(folder + "/depths.dmb", d, h, w, nb);
        if (!rc) rc = read_dmb(folder + "/normals.dmb", nrm, sh, sw, nb2);
        if (!rc) rc = read_dmb(folder + "/costs.dmb", c, h3, w3, nb3);
        if (rc) return rc;
        if (h != H || w != W)
            return fail(ACMMP_ERR_IO, "upsampled depth of view %d is %dx%d, image is %dx%d (run JBU first)",
                        problem->ref_image_id, w, h, W, H);
        if (nb2 != 3 || h3 != sh || w3 != sw) return fail(ACMMP_ERR_IO, "normals/costs of view %d disagree", problem->ref_image_id);
        // the upsample test with the reference's rows/cols swap (:766)
        const bool upsample = (sw != H || sh != W);
        std::vector<float> scaled((size_t)sw * sh * 4);
        for (size_t i = 0; i < (size_t)sw * sh; ++i) {
            scaled[4 * i] = nrm[3 * i];
            scaled[4 * i + 1] = nrm[3 * i + 1];
            scaled[4 * i + 2] = nrm[3 * i + 2];
            scaled[4 * i + 3] = upsample ? c[i] : (i < d.size() ? d[i] : 0.0f);
        }
        rc = acmmp_set_hierarchy_inputs(ctx, scaled.data(), sw, sh, d.data());
        if (rc) return fail(rc, "%s", acmmp_last_error(ctx));
    }
    return ACMMP_OK;
}

namespace {
// ACMMP_HOST_TIMING=1: per-phase wall times of each ProcessProblem on stderr
struct PhaseClock {
    bool on;
    std::chrono::steady_clock::time_point t;
    std::string line;
    PhaseClock() : on(std::getenv("ACMMP_HOST_TIMING") != nullptr), t(std::chrono::steady_clock::now()) {}
    void mark(const char *what) {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        char b[64];
        std::snprintf(b, sizeof(b), " %s=%.1f", what, std::chrono::duration<double, std::milli>(now - t).count());
        line += b;
        t = now;
    }
    void print(int id) {
        if (on) std::fprintf(stderr, "host_timing view %d ms:%s\n", id, line.c_str());
    }
};
}  // namespace

int acmmp_process_problem(const char *dense_folder, const char *output_folder, const acmmp_problem *problems,
                          int count, int idx, const acmmp_pass_options *opt) {
    if (!dense_folder || !output_folder || !problems || !opt || idx < 0 || idx >= count)
        return fail(ACMMP_ERR_ARG, "bad args");
    const acmmp_problem &problem = problems[idx];
    if (opt->verbose) std::printf("Processing image %s...\n", id8(problem.ref_image_id).c_str());
    const std::string folder = result_folder(output_folder, problem.ref_image_id);
    ::mkdir(folder.c_str(), 0777);
    PhaseClock clk;
    try {
        acmmp::ACMMP acmmp(opt->device);
        clk.mark("create");
        if (opt->geom_consistency) acmmp.SetGeomConsistencyParams(opt->multi_geometry != 0);
        if (opt->hierarchy) acmmp.SetHierarchyParams();
        acmmp_params p = acmmp.params();
        p.seed_lo = opt->seed_lo;
        p.seed_hi = opt->seed_hi;
        if (opt->max_iterations > 0) p.max_iterations = opt->max_iterations;
        acmmp.set_params(p);
        std::vector<acmmp::Problem> all(problems, problems + count);
        acmmp.InputInitialization(dense_folder, output_folder, all, idx);
        clk.mark("input_init");
        acmmp.CudaSpaceInitialization(output_folder, problem);
        clk.mark("space_init");
        const int width = acmmp.GetReferenceImageWidth(), height = acmmp.GetReferenceImageHeight();
        if (opt->seeded) {  // :275-281; GetCamera(idx) indexes this problem's cameras with the problem index
            const acmmp_params prm = acmmp.params();
            const acmmp::Camera cam = acmmp.GetCamera(idx < prm.num_images ? idx : 0);
            std::vector<acmmp::Float4> prior((size_t)width * height);
            const int rc = acmmp_prior_plane_estimate(dense_folder, idx, &cam, height, width, &prior[0].x);
            if (rc) return rc;
            acmmp.SetPlanarPrior(prior);
        }
        acmmp.RunPatchMatch();
        clk.mark("patchmatch");
        if (opt->planar_prior) {  // :301-379
            if (opt->verbose) std::printf("Run Planar Prior Assisted PatchMatch MVS ...\n");
            if (opt->write_triangulation) {
                // one triangulation for the picture and the prior; the PNG is
                // encoded on a helper thread while the second PatchMatch runs
                std::vector<uint8_t> rgb;
                std::vector<int32_t> tris;
                triangulation_picture(acmmp, rgb, tris);
                const int rc = acmmp_build_planar_prior(acmmp.handle(), tris.data(), (int)(tris.size() / 6), nullptr,
                                                        nullptr);
                if (rc) return fail(rc, "%s", acmmp_last_error(acmmp.handle()));
                acmmp.SetPlanarPriorParams();
                clk.mark("planar_prior");
                const std::string png_path = folder + "/triangulation.png";
                int png_rc = ACMMP_OK;  // (the error message is set on this thread, below)
                std::thread png([&] { png_rc = acmmp_internal_write_png(png_path.c_str(), width, height, 3, rgb.data()); });
                try {
                    acmmp.RunPatchMatch();
                } catch (...) {
                    png.join();
                    throw;
                }
                png.join();
                if (png_rc) return fail(ACMMP_ERR_IO, "cannot write %s", png_path.c_str());
            } else {
                acmmp.PreparePlanarPrior();  // support points, Delaunay, prior planes; SetPlanarPriorParams
                clk.mark("planar_prior");
                acmmp.RunPatchMatch();
            }
            clk.mark("patchmatch2");
        }
        const auto &planes = acmmp.GetPlaneHypotheses();
        const auto &costs = acmmp.GetCosts();
        clk.mark("fetch");
        const size_t P = (size_t)width * height;
        std::vector<float> depths(P), normals(P * 3);
        for (size_t i = 0; i < P; ++i) {
            depths[i] = planes[i].w;
            normals[3 * i] = planes[i].x;
            normals[3 * i + 1] = planes[i].y;
            normals[3 * i + 2] = planes[i].z;
        }
        const std::string suffix = opt->geom_consistency ? "/depths_geom.dmb" : "/depths.dmb";
        int rc = write_dmb(folder + suffix, height, width, 1, depths.data());
        if (!rc) rc = write_dmb(folder + "/normals.dmb", height, width, 3, normals.data());
        if (!rc) rc = write_dmb(folder + "/costs.dmb", height, width, 1, costs.data());
        if (rc) return rc;
        clk.mark("write");
    } catch (const acmmp::Error &e) {
        return fail(e.status(), "view %d: %s", problem.ref_image_id, e.what());
    }
    clk.mark("destroy");
    clk.print(problem.ref_image_id);
    if (opt->verbose) std::printf("Processing image %s done!\n", id8(problem.ref_image_id).c_str());
    return ACMMP_OK;
}

int acmmp_joint_bilateral_upsampling(const char *dense_folder, const char *output_folder,
                                     const acmmp_problem *problem, int acmmp_size, int device) {
    if (!dense_folder || !output_folder || !problem || acmmp_size <= 0) return fail(ACMMP_ERR_ARG, "bad args");
    const std::string folder = result_folder(output_folder, problem->ref_image_id);
    std::vector<float> depth;
    int dh = 0, dw = 0, nb = 0;
    int rc = read_dmb(folder + "/depths_geom.dmb", depth, dh, dw, nb);
    if (rc) return rc;
    acmmp::Image im;
    rc = load_image(image_path(dense_folder, problem->ref_image_id), im);
    if (rc) return rc;
    const float factor_x = static_cast<float>(acmmp_size) / im.cols;
    const float factor_y = static_cast<float>(acmmp_size) / im.rows;
    const float factor = std::min(factor_x, factor_y);
    const int new_cols = (int)std::round(im.cols * factor);
    const int new_rows = (int)std::round(im.rows * factor);
    std::vector<float> scaled((size_t)new_cols * new_rows);
    acmmp_resize_linear(im.data.data(), im.cols, im.rows, scaled.data(), new_cols, new_rows);
    std::vector<float> out(scaled.size());
    int isc = 0;
    rc = acmmp_joint_bilateral_upsample(device, scaled.data(), new_cols, new_rows, depth.data(), dw, dh, out.data(),
                                        &isc);
    if (rc) return fail(rc, "JBU of view %d failed", problem->ref_image_id);
    if (isc <= 1) return ACMMP_OK;  // "Image.rows = Depthmap.rows": nothing written (src/ACMMP.cpp:1016-1019)
    ::mkdir(folder.c_str(), 0777);
    return write_dmb(folder + "/depths.dmb", new_rows, new_cols, 1, out.data());
}

}  // extern "C"
