// asan_driver.cpp — sanitizer tier: drives the
// host C/C++ code of the product library (image/PNG/PNM decoders, .dmb and
// camera readers, Delaunay, resize, fusion) and the CPU oracle under
// AddressSanitizer + UndefinedBehaviorSanitizer, on valid inputs and on
// deterministic mutations of them (byte flips, truncations, header
// overwrites). Built by tests/asan/Makefile (`make -C tests/asan`, or
// `make asan` in acmmp_amd/csrc) and run by tests/test_asan.py. Test
// infrastructure only: nothing in the product links it.
//
// usage:
//   asan_driver image  <file> <iters> <seed>   JPEG / PNG / PGM / PFM readers
//   asan_driver dmb    <file> <iters> <seed>   acmmp_read_dmb / acmmp_write_dmb
//   asan_driver cam    <file> <iters> <seed>   acmmp_read_camera
//   asan_driver delaunay <iters> <seed>        acmmp_delaunay_triangulation
//   asan_driver resize <iters> <seed>          acmmp_resize_linear
//   asan_driver fusion <dense> <out> <fusion_folder | -> <ref:src,src,...>...
//                      (a fusion folder = RunPriorAwareFusion, - = RunFusion)
//   asan_driver oracle <seed>                  CPU oracle RunPatchMatch branches, JBU, planar
// Exit 0 = every call returned (any status); sanitizer findings abort.
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/acmmp.h"

extern "C" {
// oracle/acmmp_oracle.c, oracle/acmmp_oracle_planar.c
int acmmp_oracle_run_patchmatch(const acmmp_params *prm, int n, const acmmp_camera *cams, const float *const *imgs,
                                const float *const *depths, const int *depth_w, const int *depth_h, float *planes,
                                float *costs, uint32_t *sv, float *pre_costs, const float *prior_planes,
                                const uint32_t *masks, const float *scaled_planes, const float *seed_planes,
                                int nthreads);
int acmmp_oracle_eval_costs(const acmmp_params *prm, int n, const acmmp_camera *cams, const float *const *imgs,
                            const float *planes4, float *out_costs, float *out_init_cost, uint32_t *out_init_views,
                            int nthreads);
int acmmp_oracle_jbu(const float *img, int W, int H, const float *depth, int sw, int sh, float *out);
int acmmp_oracle_support_points(const float *costs, int width, int height, int32_t *xy);
}

namespace {

uint64_t g_state = 88172645463325252ull;
uint64_t rnd() {  // xorshift64
    g_state ^= g_state << 13;
    g_state ^= g_state >> 7;
    g_state ^= g_state << 17;
    return g_state;
}
int rnd_int(int n) { return n > 0 ? (int)(rnd() % (uint64_t)n) : 0; }

std::vector<uint8_t> read_all(const char *path) {
    std::vector<uint8_t> b;
    FILE *f = std::fopen(path, "rb");
    if (!f) return b;
    uint8_t tmp[65536];
    size_t n;
    while ((n = std::fread(tmp, 1, sizeof tmp, f)) > 0) b.insert(b.end(), tmp, tmp + n);
    std::fclose(f);
    return b;
}

void write_all(const std::string &path, const std::vector<uint8_t> &b) {
    FILE *f = std::fopen(path.c_str(), "wb");
    if (!f) {
        std::perror(path.c_str());
        std::exit(2);
    }
    if (!b.empty()) std::fwrite(b.data(), 1, b.size(), f);
    std::fclose(f);
}

// one of: flip bytes, truncate, overwrite a 2/4-byte field with an extreme,
// duplicate a range, insert random bytes (first 64 bytes favoured: headers)
std::vector<uint8_t> mutate(const std::vector<uint8_t> &in) {
    std::vector<uint8_t> b = in;
    if (b.empty()) return b;
    const int kind = rnd_int(5);
    auto pos = [&]() { return (size_t)(rnd_int(2) ? rnd_int((int)std::min<size_t>(b.size(), 64)) : rnd_int((int)b.size())); };
    if (kind == 0) {
        for (int k = 1 + rnd_int(8); k > 0; --k) b[pos()] ^= (uint8_t)(1u << rnd_int(8));
    } else if (kind == 1) {
        b.resize((size_t)rnd_int((int)b.size()));
    } else if (kind == 2) {
        static const uint32_t ext[] = {0u, 1u, 0x7fffu, 0xffffu, 0x7fffffffu, 0xffffffffu, 0x80000000u, 65500u};
        const uint32_t v = ext[rnd_int(8)];
        const size_t p = pos();
        const int w = rnd_int(2) ? 2 : 4;
        for (int k = 0; k < w && p + k < b.size(); ++k) b[p + k] = (uint8_t)(v >> (8 * (w - 1 - k)));
    } else if (kind == 3) {
        const size_t a = pos(), n = (size_t)rnd_int(256);
        std::vector<uint8_t> seg(b.begin() + a, b.begin() + std::min(b.size(), a + n));
        b.insert(b.begin() + pos(), seg.begin(), seg.end());
    } else {
        const size_t p = pos();
        std::vector<uint8_t> seg((size_t)rnd_int(32));
        for (auto &x : seg) x = (uint8_t)rnd();
        b.insert(b.begin() + p, seg.begin(), seg.end());
    }
    return b;
}

std::string tmp_path(const char *tag) {
    char buf[256];
    std::snprintf(buf, sizeof buf, "%s/acmmp_asan_%d_%s", std::getenv("TMPDIR") ? std::getenv("TMPDIR") : "/tmp",
                  (int)getpid(), tag);
    return buf;
}

// every image reader on one file: size probe, then exact-capacity reads
void read_image_all(const char *path) {
    int w = 0, h = 0, c = 0, bd = 0;
    if (acmmp_image_size(path, &w, &h) == ACMMP_OK && (size_t)w * h <= (64u << 20)) {
        std::vector<float> g((size_t)w * h);
        int w2 = 0, h2 = 0;
        (void)acmmp_read_image_gray(path, g.data(), g.size(), &w2, &h2);
        (void)acmmp_read_image_gray(path, nullptr, 0, &w2, &h2);
    }
    if (acmmp_read_image_bgr(path, nullptr, 0, &w, &h) == ACMMP_ERR_ARG && (size_t)w * h <= (64u << 20)) {
        std::vector<uint8_t> bgr((size_t)w * h * 3);
        (void)acmmp_read_image_bgr(path, bgr.data(), bgr.size(), &w, &h);
    }
    if (acmmp_read_png(path, nullptr, 0, &w, &h, &c, &bd) == ACMMP_ERR_ARG && (size_t)w * h * c <= (64u << 20)) {
        std::vector<uint16_t> px((size_t)w * h * c);
        (void)acmmp_read_png(path, px.data(), px.size(), &w, &h, &c, &bd);
    }
}

void read_dmb_all(const char *path) {
    int32_t h = 0, w = 0, nb = 0;
    if (acmmp_read_dmb(path, &h, &w, &nb, nullptr, 0) != ACMMP_OK) return;
    const size_t n = (size_t)h * w * nb;
    if (n > (64u << 20)) return;
    std::vector<float> d(n);
    if (acmmp_read_dmb(path, &h, &w, &nb, d.data(), d.size()) == ACMMP_OK && n > 0) {
        const std::string out = tmp_path("rewrite.dmb");
        (void)acmmp_write_dmb(out.c_str(), h, w, nb, d.data());
        std::remove(out.c_str());
    }
    std::vector<float> small(3);
    (void)acmmp_read_dmb(path, &h, &w, &nb, small.data(), small.size());  // capacity below the map
}

void read_cam_all(const char *path) {
    acmmp_camera cam;
    (void)acmmp_read_camera(path, &cam);
}

int fuzz_file(const char *path, int iters, void (*reader)(const char *)) {
    const std::vector<uint8_t> orig = read_all(path);
    if (orig.empty()) {
        std::fprintf(stderr, "empty or missing %s\n", path);
        return 2;
    }
    reader(path);
    const std::string t = tmp_path("mut");
    for (int i = 0; i < iters; ++i) {
        write_all(t, mutate(orig));
        reader(t.c_str());
    }
    std::remove(t.c_str());
    return 0;
}

int fuzz_delaunay(int iters) {
    for (int it = 0; it < iters; ++it) {
        const int W = 1 + rnd_int(400), H = 1 + rnd_int(300);
        const int n = rnd_int(it % 7 == 0 ? 2000 : 200);
        std::vector<int32_t> xy(2 * (size_t)n);
        const int mode = rnd_int(4);  // random / lattice (co-circular) / collinear / duplicates
        for (int i = 0; i < n; ++i) {
            int x = rnd_int(W), y = rnd_int(H);
            if (mode == 1) { x = (x / 5) * 5 % W; y = (y / 5) * 5 % H; }
            if (mode == 2) y = (x * 3) % H;
            if (mode == 3 && i > 0 && rnd_int(2)) { x = xy[2 * (i - 1)]; y = xy[2 * (i - 1) + 1]; }
            xy[2 * i] = x;
            xy[2 * i + 1] = y;
        }
        if (it % 11 == 5 && n > 0) xy[0] = W;  // out of range: rejected
        const int cap = rnd_int(3) == 0 ? rnd_int(4 * n + 1) : 2 * n + 8;
        std::vector<int32_t> tris(6 * (size_t)cap + 6);
        int nt = 0;
        (void)acmmp_delaunay_triangulation(W, H, xy.data(), n, tris.data(), cap, &nt);
    }
    return 0;
}

int fuzz_resize(int iters) {
    for (int it = 0; it < iters; ++it) {
        const int sw = 1 + rnd_int(300), sh = 1 + rnd_int(300), dw = 1 + rnd_int(300), dh = 1 + rnd_int(300);
        std::vector<float> src((size_t)sw * sh), dst((size_t)dw * dh);
        for (auto &v : src) v = (float)(rnd() % 256);
        (void)acmmp_resize_linear(src.data(), sw, sh, dst.data(), dw, dh);
    }
    return 0;
}

int run_fusion(int argc, char **argv) {
    if (argc < 6) return 2;
    const bool prior_aware = std::strcmp(argv[4], "-") != 0;
    std::vector<acmmp_problem> probs;
    for (int a = 5; a < argc; ++a) {
        acmmp_problem p;
        std::memset(&p, 0, sizeof p);
        p.max_image_size = p.cur_image_size = 6400;
        char *s = argv[a];
        p.ref_image_id = (int)std::strtol(s, &s, 10);
        while (*s == ':' || *s == ',') {
            ++s;
            if (p.num_src_images < ACMMP_MAX_IMAGES - 1) p.src_image_ids[p.num_src_images++] = (int)std::strtol(s, &s, 10);
        }
        probs.push_back(p);
    }
    int npts = -1, rc;
    // RunFusion / RunPriorAwareFusion with the drivers' defaults, debug images on
    if (prior_aware)
        rc = acmmp_run_prior_aware_fusion(argv[2], argv[3], argv[4], probs.data(), (int)probs.size(), 1, 0.3f, 2, 1,
                                          &npts);
    else
        rc = acmmp_run_fusion(argv[2], argv[3], probs.data(), (int)probs.size(), 1, 0.3f, 1, "/images", " ", 1,
                              &npts);
    std::printf("fusion rc=%d points=%d\n", rc, npts);
    return rc == ACMMP_OK ? 0 : 3;
}

// a small textured scene on a sideways arc for the oracle
void make_scene(int n, int W, int H, std::vector<acmmp_camera> &cams, std::vector<std::vector<float>> &imgs) {
    cams.assign(n, acmmp_camera{});
    imgs.assign(n, std::vector<float>((size_t)W * H));
    for (int i = 0; i < n; ++i) {
        acmmp_camera &c = cams[i];
        const float f = 1.2f * W;
        const float K[9] = {f, 0, 0.5f * W, 0, f, 0.5f * H, 0, 0, 1};
        std::memcpy(c.K, K, sizeof K);
        const float R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        std::memcpy(c.R, R, sizeof R);
        c.t[0] = -0.06f * i;
        c.width = W;
        c.height = H;
        c.depth_min = 2.0f;
        c.depth_max = 8.0f;
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) {
                const int xs = x + 3 * i;  // fronto-parallel plane: disparity shift
                imgs[i][(size_t)y * W + x] = (float)((xs * 37 + y * 11 + ((xs ^ y) & 15) * 9) % 256);
            }
    }
}

acmmp_params base_params(int iters) {
    acmmp_params p;
    std::memset(&p, 0, sizeof p);
    p.max_iterations = iters;
    p.patch_size = 11;
    p.max_image_size = 3200;
    p.radius_increment = 2;
    p.sigma_spatial = 5.0f;
    p.sigma_color = 3.0f;
    p.top_k = 4;
    p.baseline = 0.54f;
    p.depth_min = 2.0f;
    p.depth_max = 8.0f;
    p.seed_lo = (uint32_t)rnd();
    p.seed_hi = 7;
    return p;
}

int run_oracle() {
    const int n = 4, W = 57, H = 41;  // odd sizes: last-row / ragged paths
    std::vector<acmmp_camera> cams;
    std::vector<std::vector<float>> imgs;
    make_scene(n, W, H, cams, imgs);
    std::vector<const float *> ip(n);
    for (int i = 0; i < n; ++i) ip[i] = imgs[i].data();
    const size_t P = (size_t)W * H;
    std::vector<float> planes(4 * P, 0.0f), costs(P, 0.0f), pre(P, 0.0f);
    std::vector<uint32_t> sv(P, 0);
    acmmp_params p = base_params(2);
    p.num_images = n;
    int rc = acmmp_oracle_run_patchmatch(&p, n, cams.data(), ip.data(), nullptr, nullptr, nullptr, planes.data(),
                                         costs.data(), sv.data(), nullptr, nullptr, nullptr, nullptr, nullptr, 2);
    if (rc) return 10;
    // geometric pass from the photometric state, depth maps = its depths
    std::vector<std::vector<float>> dep(n, std::vector<float>(P));
    for (int i = 0; i < n; ++i)
        for (size_t k = 0; k < P; ++k) dep[i][k] = planes[4 * k + 3];
    std::vector<const float *> dp(n);
    for (int i = 0; i < n; ++i) dp[i] = dep[i].data();
    acmmp_params g = p;
    g.geom_consistency = 1;
    rc = acmmp_oracle_run_patchmatch(&g, n, cams.data(), ip.data(), dp.data(), nullptr, nullptr, planes.data(),
                                     costs.data(), sv.data(), nullptr, nullptr, nullptr, nullptr, nullptr, 2);
    if (rc) return 11;
    // planar prior: support points -> (no triangulation here) a flat prior on half the pixels
    std::vector<int32_t> xy(2 * P);
    (void)acmmp_oracle_support_points(costs.data(), W, H, xy.data());
    std::vector<float> prior(4 * P, 0.0f);
    std::vector<uint32_t> mask(P, 0);
    for (size_t k = 0; k < P; ++k) {
        prior[4 * k + 2] = -1.0f;
        prior[4 * k + 3] = 4.0f;
        mask[k] = (k % 3) ? 1u : 0u;
    }
    acmmp_params pl = p;
    pl.planar_prior = 1;
    rc = acmmp_oracle_run_patchmatch(&pl, n, cams.data(), ip.data(), nullptr, nullptr, nullptr, planes.data(),
                                     costs.data(), sv.data(), nullptr, prior.data(), mask.data(), nullptr, nullptr, 2);
    if (rc) return 12;
    // hierarchy from a half-resolution map (upsample branch)
    const int sw = W / 2, sh = H / 2;
    std::vector<float> scaled(4 * (size_t)sw * sh);
    for (size_t k = 0; k < (size_t)sw * sh; ++k) {
        scaled[4 * k + 0] = 0.0f;
        scaled[4 * k + 1] = 0.0f;
        scaled[4 * k + 2] = -1.0f;
        scaled[4 * k + 3] = 0.3f;
    }
    acmmp_params hi = p;
    hi.hierarchy = 1;
    hi.upsample = 1;
    hi.scaled_cols = (float)sw;
    hi.scaled_rows = (float)sh;
    rc = acmmp_oracle_run_patchmatch(&hi, n, cams.data(), ip.data(), nullptr, nullptr, nullptr, planes.data(),
                                     costs.data(), sv.data(), pre.data(), nullptr, nullptr, scaled.data(), nullptr, 2);
    if (rc) return 13;
    std::vector<float> cv(P * (n - 1)), init(P);
    std::vector<uint32_t> iv(P);
    rc = acmmp_oracle_eval_costs(&p, n, cams.data(), ip.data(), planes.data(), cv.data(), init.data(), iv.data(), 2);
    if (rc) return 14;
    std::vector<float> up(P);
    std::vector<float> low((size_t)sw * sh, 5.0f);
    (void)acmmp_oracle_jbu(imgs[0].data(), W, H, low.data(), sw, sh, up.data());
    return 0;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: see header\n");
        return 2;
    }
    const std::string cmd = argv[1];
    auto seed_at = [&](int i) {
        if (argc > i) g_state ^= std::strtoull(argv[i], nullptr, 10) * 0x9E3779B97F4A7C15ull + 1;
    };
    int rc = 2;
    if ((cmd == "image" || cmd == "dmb" || cmd == "cam") && argc >= 4) {
        seed_at(4);
        const int iters = std::atoi(argv[3]);
        rc = fuzz_file(argv[2], iters, cmd == "image" ? read_image_all : cmd == "dmb" ? read_dmb_all : read_cam_all);
    } else if (cmd == "delaunay" && argc >= 3) {
        seed_at(3);
        rc = fuzz_delaunay(std::atoi(argv[2]));
    } else if (cmd == "resize" && argc >= 3) {
        seed_at(3);
        rc = fuzz_resize(std::atoi(argv[2]));
    } else if (cmd == "fusion") {
        rc = run_fusion(argc, argv);
    } else if (cmd == "oracle") {
        seed_at(2);
        rc = run_oracle();
    }
    if (rc == 0) std::printf("%s ok\n", cmd.c_str());
    return rc;
}
