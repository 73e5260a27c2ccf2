// acmmp_io.cpp — the reference's on-disk formats, OpenCV-free.
//   ReadCamera            src/ACMMP.cpp:154-179
//   read/writeDepthDmb    src/ACMMP.cpp:264-321
//   read/writeNormalDmb   src/ACMMP.cpp:323-380
// .dmb = int32 type(=1), h, w, nb, then h*w*nb little-endian float32 (HWC).
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>

#include "../../include/acmmp.h"

extern "C" {

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
