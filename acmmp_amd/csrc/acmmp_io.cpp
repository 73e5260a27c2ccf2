// acmmp_io.cpp — the reference's on-disk formats, OpenCV-free.
//   ReadCamera            src/ACMMP.cpp:154-179
//   read/writeDepthDmb    src/ACMMP.cpp:264-321
//   read/writeNormalDmb   src/ACMMP.cpp:323-380
// .dmb = int32 type(=1), h, w, nb, then h*w*nb little-endian float32 (HWC).
#include <sched.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>

#include "../../include/acmmp.h"

namespace {
// ceil(quota / period) of the cgroup CPU controller, 0 when unlimited/absent
int cgroup_cpus() {
    long long q = -1, p = 0;
    if (FILE *f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {  // cgroup v2: "max 100000" / "Q P"
        char qs[32] = {0};
        if (std::fscanf(f, "%31s %lld", qs, &p) == 2 && std::strcmp(qs, "max") != 0) q = std::atoll(qs);
        std::fclose(f);
    } else if (FILE *f1 = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {  // v1
        if (std::fscanf(f1, "%lld", &q) != 1) q = -1;
        std::fclose(f1);
        if (FILE *f2 = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
            if (std::fscanf(f2, "%lld", &p) != 1) p = 0;
            std::fclose(f2);
        }
    }
    if (q <= 0 || p <= 0) return 0;
    return (int)((q + p - 1) / p);
}
}  // namespace

extern "C" {

int acmmp_host_threads(void) {
    if (const char *e = std::getenv("ACMMP_HOST_THREADS"))
        if (std::atoi(e) > 0) return std::atoi(e);
    int n = (int)std::max(1u, std::thread::hardware_concurrency());
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof(set), &set) == 0 && CPU_COUNT(&set) > 0) n = std::min(n, (int)CPU_COUNT(&set));
    if (const int q = cgroup_cpus()) n = std::min(n, q);
    if (const char *e = std::getenv("OMP_NUM_THREADS"))
        if (std::atoi(e) > 0) n = std::min(n, std::atoi(e));
    return std::max(n, 1);
}

int acmmp_read_camera(const char *path, acmmp_camera *cam) {
    if (!path || !cam) return ACMMP_ERR_ARG;
    std::ifstream file(path);
    if (!file.is_open()) return ACMMP_ERR_IO;
    std::memset(cam, 0, sizeof(*cam));
    std::string line;
    file >> line;  // "extrinsic"
    for (int i = 0; i < 3; ++i)
        file >> cam->R[3 * i + 0] >> cam->R[3 * i + 1] >> cam->R[3 * i + 2] >> cam->t[i];
    float tmp[4];
    file >> tmp[0] >> tmp[1] >> tmp[2] >> tmp[3];  // last extrinsic row
    file >> line;                                    // "intrinsic"
    for (int i = 0; i < 3; ++i) file >> cam->K[3 * i + 0] >> cam->K[3 * i + 1] >> cam->K[3 * i + 2];
    float depth_num, interval;
    file >> cam->depth_min >> interval >> depth_num >> cam->depth_max;
    if (file.fail()) return ACMMP_ERR_IO;
    return ACMMP_OK;
}

int acmmp_read_dmb(const char *path, int32_t *h, int32_t *w, int32_t *nb, float *data, size_t cap) {
    if (!path || !h || !w || !nb) return ACMMP_ERR_ARG;
    FILE *f = std::fopen(path, "rb");
    if (!f) return ACMMP_ERR_IO;
    int32_t hdr[4] = {-1, 0, 0, 0};
    if (std::fread(hdr, sizeof(int32_t), 4, f) != 4 || hdr[0] != 1 || hdr[1] < 0 || hdr[2] < 0 || hdr[3] < 0) {
        std::fclose(f);
        return ACMMP_ERR_IO;
    }
    *h = hdr[1];
    *w = hdr[2];
    *nb = hdr[3];
    if (data) {
        size_t count = (size_t)hdr[1] * (size_t)hdr[2] * (size_t)hdr[3];
        if (count > cap) count = cap;
        if (std::fread(data, sizeof(float), count, f) != count) {
            std::fclose(f);
            return ACMMP_ERR_IO;
        }
    }
    std::fclose(f);
    return ACMMP_OK;
}

int acmmp_write_dmb(const char *path, int32_t h, int32_t w, int32_t nb, const float *data) {
    if (!path || (!data && (size_t)h * w * nb > 0) || h < 0 || w < 0 || nb < 0) return ACMMP_ERR_ARG;
    FILE *f = std::fopen(path, "wb");
    if (!f) return ACMMP_ERR_IO;
    const int32_t hdr[4] = {1, h, w, nb};
    const size_t count = (size_t)h * (size_t)w * (size_t)nb;
    bool ok = std::fwrite(hdr, sizeof(int32_t), 4, f) == 4;
    if (ok && count) ok = std::fwrite(data, sizeof(float), count, f) == count;
    std::fclose(f);
    return ok ? ACMMP_OK : ACMMP_ERR_IO;
}

}  // extern "C"
