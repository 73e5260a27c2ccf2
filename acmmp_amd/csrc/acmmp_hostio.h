// acmmp_hostio.h — host-side helpers shared by the host modules
// (acmmp_image.cpp defines them; acmmp_pipeline.cpp and acmmp_fusion.cpp use
// them). Not part of the C-ABI.
#pragma once

#include <cstdint>
#include <vector>

// 8-bit PNG (channels 1 = gray, 3 = RGB), one IDAT, zlib at best speed.
// ACMMP_OK / ACMMP_ERR_ARG / ACMMP_ERR_IO.
int acmmp_internal_write_png(const char *path, int w, int h, int channels, const uint8_t *px);

// acmmp_read_image_bgr in one pass: decodes into `bgr` (W*H*3, BGR) and sets
// the size, without the C-ABI's size-query call (which decodes the file too).
// ACMMP_OK / ACMMP_ERR_IO / ACMMP_ERR_UNSUPPORTED.
int acmmp_internal_read_image_bgr(const char *path, std::vector<uint8_t> &bgr, int &width, int &height);
