// acmmp_image.cpp — grayscale image input for InputInitialization
// (src/ACMMP.cpp:525-601) without OpenCV:
//
//  * cv::imread(path, IMREAD_GRAYSCALE) of the reference's `%08d.jpg` inputs:
//    a baseline (SOF0/SOF1, 8-bit, Huffman) JPEG decoder that returns the
//    luminance plane exactly as libjpeg's JCS_GRAYSCALE output does — the
//    ISLOW integer IDCT with its range-limit table, Y taken without colour
//    conversion; and progressive (SOF2) files, whose spectral-selection /
//    successive-approximation scans rebuild the same coefficients libjpeg's
//    jdphuff.c does before the same IDCT (camera JPEGs reach the loader
//    unchanged: colmap2mvsnet_acm.py:453-454). Arithmetic-coded / lossless /
//    12-bit files are rejected (ACMMP_ERR_UNSUPPORTED).
//    The IDCT algorithm and its constants (the Loeffler-Ligtenberg-Moschytz
//    factorisation as laid out in jidctint.c) are the Independent JPEG
//    Group's; this file re-implements them, it contains no IJG source.
//  * binary PGM (P5, 8/16-bit) and grayscale PFM as lossless alternatives.
//  * cv::resize(..., INTER_LINEAR) of a float image (src/ACMMP.cpp:578-597),
//    including OpenCV's switch to INTER_AREA for exact 2x downscales.
#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include <zlib.h>

#include "../../include/acmmp.h"
#include "acmmp_hostio.h"

namespace {

bool read_file(const char *path, std::vector<uint8_t> &buf) {
    FILE *f = std::fopen(path, "rb");
    if (!f) return false;
    std::fseek(f, 0, SEEK_END);
    long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    if (n < 0) {
        std::fclose(f);
        return false;
    }
    buf.resize((size_t)n);
    bool ok = n == 0 || std::fread(buf.data(), 1, (size_t)n, f) == (size_t)n;
    std::fclose(f);
    return ok;
}

// ------------------------------------------------------------------ JPEG
struct Huff {
    // canonical decoding tables: maxcode[l], valptr[l], mincode[l]
    int32_t mincode[17], maxcode[18], valptr[17];
    uint8_t vals[256];
    // 8-bit lookahead: for the next 8 bits of the stream, the length (0 = the
    // code is longer than 8 bits) and symbol of the code they start with
    uint8_t look_len[256], look_sym[256];
    // AC coefficients whose code and magnitude bits fit in the next 9 bits:
    // value << 16 | run << 8 | bits consumed (0 = not covered; EOB and ZRL
    // are not covered). Derived from look_len/look_sym, so it decodes what
    // decode_huff + getbits decode from the same bits.
    int32_t fast_ac[512];
    bool present = false;
};

struct Comp {
    int id, h, v, tq;
    int td = 0, ta = 0;
    int bw = 0, bh = 0;         // blocks per line / column (component extent, padded to MCU)
    std::vector<int16_t> coef;  // only for the luminance component
    int pred = 0;
};

struct Jpeg {
    const uint8_t *p = nullptr, *end = nullptr;
    int W = 0, H = 0, ncomp = 0, hmax = 1, vmax = 1;
    Comp comp[4];
    uint16_t qt[4][64];
    bool qt_present[4] = {false, false, false, false};
    Huff dc[4], ac[4];
    int restart = 0;
    bool sof = false;
    bool progressive = false;  // SOF2
    int eobrun = 0;            // progressive AC scans: blocks left in the current end-of-band run
    // bit reader
    uint32_t bitbuf = 0;
    int bitcnt = 0;
    bool hit_marker = false;

    int err = ACMMP_OK;
};

const uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

int u16(const uint8_t *q) { return (q[0] << 8) | q[1]; }

bool build_huff(Huff &h, const uint8_t *counts, const uint8_t *symbols, int nsym) {
    if (nsym > 256) return false;
    std::memcpy(h.vals, symbols, nsym);
    int code = 0, k = 0;
    for (int l = 1; l <= 16; ++l) {
        h.valptr[l] = k;
        h.mincode[l] = code;
        code += counts[l - 1];
        k += counts[l - 1];
        h.maxcode[l] = counts[l - 1] ? code - 1 : -1;
        code <<= 1;
    }
    h.maxcode[17] = 0x7fffffff;
    std::memset(h.look_len, 0, sizeof(h.look_len));
    for (int l = 1; l <= 8; ++l) {
        // empty when maxcode[l] == -1; a code that overflows l bits, or an
        // entry a shorter code already holds, is left to the bit-serial loop
        // (which takes the shortest match, as libjpeg does)
        for (int c = h.mincode[l]; c <= h.maxcode[l] && c < (1 << l); ++c) {
            const int sym = h.vals[h.valptr[l] + c - h.mincode[l]];
            const int span = 1 << (8 - l);
            for (int e = c << (8 - l), k = 0; k < span; ++k) {
                if (h.look_len[e + k]) continue;
                h.look_len[e + k] = (uint8_t)l;
                h.look_sym[e + k] = (uint8_t)sym;
            }
        }
    }
    for (int p = 0; p < 512; ++p) {
        const int l = h.look_len[p >> 1], sym = h.look_sym[p >> 1];
        const int r = sym >> 4, t = sym & 15;
        h.fast_ac[p] = 0;
        if (!l || !t || l + t > 9) continue;
        const int v = (p >> (9 - l - t)) & ((1 << t) - 1);
        const int val = (v < (1 << (t - 1))) ? v - (1 << t) + 1 : v;  // extend()
        h.fast_ac[p] = (int32_t)((uint32_t)val << 16) | r << 8 | (l + t);
    }
    h.present = true;
    return true;
}

// Fill the bit buffer; after a marker, feed zeros (libjpeg behaviour).
inline void fill(Jpeg &j) {
    while (j.bitcnt <= 24) {
        int byte = 0;
        if (!j.hit_marker && j.p < j.end) {
            byte = *j.p;
            if (byte == 0xFF) {
                const int nx = (j.p + 1 < j.end) ? j.p[1] : 0;
                if (nx == 0x00) {
                    j.p += 2;
                } else {
                    j.hit_marker = true;  // leave the marker for the caller
                    byte = 0;
                }
            } else {
                ++j.p;
            }
        }
        j.bitbuf |= (uint32_t)byte << (24 - j.bitcnt);
        j.bitcnt += 8;
    }
}

inline int getbits(Jpeg &j, int n) {
    if (n == 0) return 0;
    fill(j);
    const int v = (int)(j.bitbuf >> (32 - n));
    j.bitbuf <<= n;
    j.bitcnt -= n;
    return v;
}

inline int decode_huff(Jpeg &j, const Huff &h) {
    fill(j);
    const int peek = (int)(j.bitbuf >> 24);
    if (const int len = h.look_len[peek]) {  // codes of up to 8 bits: one lookup
        j.bitbuf <<= len;
        j.bitcnt -= len;
        return h.look_sym[peek];
    }
    int code = 0;
    for (int l = 1; l <= 16; ++l) {
        code = (code << 1) | (int)(j.bitbuf >> 31);
        j.bitbuf <<= 1;
        j.bitcnt -= 1;
        if (h.maxcode[l] >= 0 && code <= h.maxcode[l] && code >= h.mincode[l])
            return h.vals[h.valptr[l] + code - h.mincode[l]];
    }
    j.err = ACMMP_ERR_IO;  // corrupt data
    return 0;
}

inline int extend(int v, int t) { return (t && v < (1 << (t - 1))) ? v - (1 << t) + 1 : v; }

void decode_block(Jpeg &j, Comp &c, int16_t *out) {
    const int t = decode_huff(j, j.dc[c.td]);
    if (t > 16) {
        j.err = ACMMP_ERR_IO;
        return;
    }
    const int diff = extend(getbits(j, t), t);
    c.pred += diff;
    if (out) {
        std::memset(out, 0, 64 * sizeof(int16_t));
        out[0] = (int16_t)c.pred;
    }
    const Huff &ac = j.ac[c.ta];
    for (int k = 1; k < 64;) {
        fill(j);
        if (const int32_t fa = ac.fast_ac[j.bitbuf >> 23]) {
            k += (fa >> 8) & 15;
            if (k > 63) {
                j.err = ACMMP_ERR_IO;
                return;
            }
            j.bitbuf <<= fa & 15;
            j.bitcnt -= fa & 15;
            if (out) out[kZigzag[k]] = (int16_t)(fa >> 16);
            ++k;
            continue;
        }
        const int rs = decode_huff(j, ac);
        const int r = rs >> 4, s = rs & 15;
        if (s == 0) {
            if (r != 15) break;  // EOB
            k += 16;
            continue;
        }
        k += r;
        const int v = extend(getbits(j, s), s);
        if (k > 63) {
            j.err = ACMMP_ERR_IO;
            return;
        }
        if (out) out[kZigzag[k]] = (int16_t)v;
        ++k;
    }
}

// Skip to the restart marker and reset the entropy decoder.
void handle_restart(Jpeg &j) {
    j.bitbuf = 0;
    j.bitcnt = 0;
    j.hit_marker = false;
    while (j.p + 1 < j.end && !(j.p[0] == 0xFF && j.p[1] >= 0xD0 && j.p[1] <= 0xD7)) ++j.p;
    if (j.p + 1 < j.end) j.p += 2;
    for (int c = 0; c < j.ncomp; ++c) j.comp[c].pred = 0;
    j.eobrun = 0;
}

bool decode_scan_progressive(Jpeg &j, const int *sc, int ns, int ss, int se, int ah, int al);

bool decode_scan(Jpeg &j, const uint8_t *hdr, int len) {
    const int ns = hdr[0];
    if (ns < 1 || ns > 4 || len < 1 + 2 * ns + 3) return false;
    int sc[4];
    for (int i = 0; i < ns; ++i) {
        const int cid = hdr[1 + 2 * i], tbl = hdr[2 + 2 * i];
        sc[i] = -1;
        for (int c = 0; c < j.ncomp; ++c)
            if (j.comp[c].id == cid) sc[i] = c;
        if (sc[i] < 0) return false;
        j.comp[sc[i]].td = tbl >> 4;
        j.comp[sc[i]].ta = tbl & 15;
        if (j.comp[sc[i]].td > 3 || j.comp[sc[i]].ta > 3) return false;
        // (a progressive scan needs only the table of its kind: checked there)
        if (!j.progressive && (!j.dc[j.comp[sc[i]].td].present || !j.ac[j.comp[sc[i]].ta].present)) return false;
    }
    const int ss = hdr[1 + 2 * ns], se = hdr[2 + 2 * ns], ahal = hdr[3 + 2 * ns];
    if (j.progressive) return decode_scan_progressive(j, sc, ns, ss, se, ahal >> 4, ahal & 15);
    if (ss != 0 || se != 63 || ahal != 0) return false;  // sequential
    for (int i = 0; i < ns; ++i) j.comp[sc[i]].pred = 0;
    j.bitbuf = 0;
    j.bitcnt = 0;
    j.hit_marker = false;
    int mcus_x, mcus_y;
    if (ns == 1) {
        const Comp &c = j.comp[sc[0]];
        mcus_x = (int)((j.W * (long)c.h + 8L * j.hmax - 1) / (8L * j.hmax));
        mcus_y = (int)((j.H * (long)c.v + 8L * j.vmax - 1) / (8L * j.vmax));
    } else {
        mcus_x = (j.W + 8 * j.hmax - 1) / (8 * j.hmax);
        mcus_y = (j.H + 8 * j.vmax - 1) / (8 * j.vmax);
    }
    int todo = j.restart;
    for (int my = 0; my < mcus_y; ++my) {
        for (int mx = 0; mx < mcus_x; ++mx) {
            if (j.restart && todo == 0) {
                handle_restart(j);
                todo = j.restart;
            }
            for (int i = 0; i < ns; ++i) {
                Comp &c = j.comp[sc[i]];
                const int bx_n = ns == 1 ? 1 : c.h, by_n = ns == 1 ? 1 : c.v;
                for (int by = 0; by < by_n; ++by)
                    for (int bx = 0; bx < bx_n; ++bx) {
                        const int gx = ns == 1 ? mx : mx * c.h + bx;
                        const int gy = ns == 1 ? my : my * c.v + by;
                        int16_t *dst = nullptr;
                        if (!c.coef.empty() && gx < c.bw && gy < c.bh) dst = &c.coef[((size_t)gy * c.bw + gx) * 64];
                        decode_block(j, c, dst);
                        if (j.err) return false;
                    }
            }
            if (j.restart) --todo;
        }
    }
    // continue after the entropy-coded segment
    while (j.p + 1 < j.end && !(j.p[0] == 0xFF && j.p[1] != 0x00 && !(j.p[1] >= 0xD0 && j.p[1] <= 0xD7))) ++j.p;
    return true;
}

// ---- progressive scans (ITU T.81 G.1.2; the decoding of libjpeg's
// jdphuff.c, re-implemented): DC first / DC refinement scans (possibly
// interleaved) and single-component AC first / AC refinement scans over a
// spectral band [ss, se] at bit position al. Coefficients accumulate in the
// component's coefficient array (natural order); dst == nullptr decodes a
// component whose coefficients are not kept (bits consumed all the same).
void prog_dc_first(Jpeg &j, Comp &c, int16_t *dst, int al) {
    const int t = decode_huff(j, j.dc[c.td]);
    if (t > 16) {
        j.err = ACMMP_ERR_IO;
        return;
    }
    c.pred += extend(getbits(j, t), t);
    if (dst) dst[0] = (int16_t)(int)((uint32_t)c.pred << al);
}

void prog_dc_refine(Jpeg &j, int16_t *dst, int al) {
    if (getbits(j, 1) && dst) dst[0] = (int16_t)(dst[0] | (1 << al));
}

void prog_ac_first(Jpeg &j, const Comp &c, int16_t *dst, int ss, int se, int al) {
    if (j.eobrun > 0) {
        --j.eobrun;
        return;
    }
    for (int k = ss; k <= se; ++k) {
        const int rs = decode_huff(j, j.ac[c.ta]);
        const int r = rs >> 4, sz = rs & 15;
        if (sz) {
            k += r;
            const int v = extend(getbits(j, sz), sz);
            if (k > 63) {
                j.err = ACMMP_ERR_IO;
                return;
            }
            if (dst) dst[kZigzag[k]] = (int16_t)(int)((uint32_t)v << al);
        } else if (r == 15) {
            k += 15;  // ZRL
        } else {
            j.eobrun = (1 << r) + (r ? getbits(j, r) : 0) - 1;  // this block ends the first band of the run
            return;
        }
    }
}

// one refinement bit for an already-nonzero coefficient
inline void refine_nonzero(Jpeg &j, int16_t *cf, int p1) {
    if (getbits(j, 1) && (*cf & p1) == 0) *cf = (int16_t)(*cf >= 0 ? *cf + p1 : *cf - p1);
}

void prog_ac_refine(Jpeg &j, const Comp &c, int16_t *dst, int ss, int se, int al) {
    const int p1 = 1 << al;
    int16_t scratch[64] = {0};  // a component whose coefficients are not kept: zero history
    int16_t *b = dst ? dst : scratch;
    int k = ss;
    if (j.eobrun == 0) {
        for (; k <= se; ++k) {
            const int rs = decode_huff(j, j.ac[c.ta]);
            int r = rs >> 4;
            const int sz = rs & 15;
            int v = 0;
            if (sz) {
                if (sz != 1) {  // a newly nonzero coefficient is +-1 at this bit position
                    j.err = ACMMP_ERR_IO;
                    return;
                }
                v = getbits(j, 1) ? p1 : -p1;
            } else if (r != 15) {
                j.eobrun = (1 << r) + (r ? getbits(j, r) : 0);
                break;  // the rest of this band: EOB run logic below
            }
            // skip r zero-history coefficients (refining the nonzero ones passed)
            for (; k <= se; ++k) {
                int16_t *cf = &b[kZigzag[k]];
                if (*cf != 0) {
                    refine_nonzero(j, cf, p1);
                } else if (--r < 0) {
                    break;
                }
            }
            if (v) {
                if (k > 63) {
                    j.err = ACMMP_ERR_IO;
                    return;
                }
                b[kZigzag[k]] = (int16_t)v;
            }
        }
    }
    if (j.eobrun > 0) {  // inside an EOB run: only the refinement bits of nonzero coefficients
        for (; k <= se; ++k) {
            int16_t *cf = &b[kZigzag[k]];
            if (*cf != 0) refine_nonzero(j, cf, p1);
        }
        --j.eobrun;
    }
}

bool decode_scan_progressive(Jpeg &j, const int *sc, int ns, int ss, int se, int ah, int al) {
    // T.81 G.1.1.1: DC scans cover [0, 0] (may interleave), AC scans one
    // component and a band inside [1, 63]; refinement lowers al by one
    if (ss > se || se > 63 || al > 13 || ah > 13 || (ah && ah != al + 1)) return false;
    if (ss == 0 && se != 0) return false;
    if (ss > 0 && ns != 1) return false;
    for (int i = 0; i < ns; ++i) j.comp[sc[i]].pred = 0;  // every scan starts its DC predictions at 0
    if (ns == 1 && j.comp[sc[0]].coef.empty()) {  // a component not kept: skip its entropy-coded data
        while (j.p + 1 < j.end && !(j.p[0] == 0xFF && j.p[1] != 0x00 && !(j.p[1] >= 0xD0 && j.p[1] <= 0xD7))) ++j.p;
        return true;
    }
    for (int i = 0; i < ns; ++i) {
        const Comp &c = j.comp[sc[i]];
        if (ss == 0 && ah == 0 && !j.dc[c.td].present) return false;
        if (ss > 0 && !j.ac[c.ta].present) return false;
    }
    j.bitbuf = 0;
    j.bitcnt = 0;
    j.hit_marker = false;
    j.eobrun = 0;
    int mcus_x, mcus_y;
    if (ns == 1) {  // non-interleaved: one block per MCU over the component's own extent
        const Comp &c = j.comp[sc[0]];
        mcus_x = (int)((j.W * (long)c.h + 8L * j.hmax - 1) / (8L * j.hmax));
        mcus_y = (int)((j.H * (long)c.v + 8L * j.vmax - 1) / (8L * j.vmax));
    } else {
        mcus_x = (j.W + 8 * j.hmax - 1) / (8 * j.hmax);
        mcus_y = (j.H + 8 * j.vmax - 1) / (8 * j.vmax);
    }
    int todo = j.restart;
    for (int my = 0; my < mcus_y; ++my) {
        for (int mx = 0; mx < mcus_x; ++mx) {
            if (j.restart && todo == 0) {
                handle_restart(j);
                todo = j.restart;
            }
            for (int i = 0; i < ns; ++i) {
                Comp &c = j.comp[sc[i]];
                const int bx_n = ns == 1 ? 1 : c.h, by_n = ns == 1 ? 1 : c.v;
                for (int by = 0; by < by_n; ++by)
                    for (int bx = 0; bx < bx_n; ++bx) {
                        const int gx = ns == 1 ? mx : mx * c.h + bx;
                        const int gy = ns == 1 ? my : my * c.v + by;
                        int16_t *dst = nullptr;
                        if (!c.coef.empty() && gx < c.bw && gy < c.bh) dst = &c.coef[((size_t)gy * c.bw + gx) * 64];
                        if (ss == 0) {
                            if (ah == 0) prog_dc_first(j, c, dst, al);
                            else prog_dc_refine(j, dst, al);
                        } else if (ah == 0) {
                            prog_ac_first(j, c, dst, ss, se, al);
                        } else {
                            prog_ac_refine(j, c, dst, ss, se, al);
                        }
                        if (j.err) return false;
                    }
            }
            if (j.restart) --todo;
        }
    }
    while (j.p + 1 < j.end && !(j.p[0] == 0xFF && j.p[1] != 0x00 && !(j.p[1] >= 0xD0 && j.p[1] <= 0xD7))) ++j.p;
    return true;
}

// jpeg_idct_islow (libjpeg jidctint.c): 13-bit fixed point, PASS1_BITS = 2.
constexpr int kConstBits = 13, kPass1Bits = 2;
constexpr int32_t F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373, F1175 = 9633,
                  F1501 = 12299, F1847 = 15137, F1961 = 16069, F2053 = 16819, F2562 = 20995, F3072 = 25172;

// Intermediates are 64-bit like libjpeg-turbo's JLONG on LP64 (the
// workspace is int), so out-of-range coefficients of a corrupt stream wrap
// instead of overflowing a signed int.
inline int64_t descale(int64_t x, int n) { return (x + ((int64_t)1 << (n - 1))) >> n; }

inline uint8_t range_limit(int64_t x) {
    const int idx = (int)(x & 1023);  // RANGE_MASK of the post-IDCT table (jdmaster.c)
    if (idx < 128) return (uint8_t)(idx + 128);
    if (idx < 512) return 255;
    if (idx < 896) return 0;
    return (uint8_t)(idx - 896);
}

void idct_islow(const int16_t *in, const uint16_t *q, uint8_t *out, int stride) {
    int32_t ws[64];
    for (int c = 0; c < 8; ++c) {
        const int16_t *ip = in + c;
        const uint16_t *qp = q + c;
        if (!ip[8] && !ip[16] && !ip[24] && !ip[32] && !ip[40] && !ip[48] && !ip[56]) {
            const int32_t dc = (int32_t)((uint32_t)((int32_t)ip[0] * qp[0]) << kPass1Bits);  // LEFT_SHIFT
            for (int r = 0; r < 8; ++r) ws[r * 8 + c] = dc;
            continue;
        }
        int64_t z2 = (int64_t)ip[16] * qp[16], z3 = (int64_t)ip[48] * qp[48];
        int64_t z1 = (z2 + z3) * F0541;
        int64_t tmp2 = z1 + z3 * (-F1847);
        int64_t tmp3 = z1 + z2 * F0765;
        z2 = (int64_t)ip[0] * qp[0];
        z3 = (int64_t)ip[32] * qp[32];
        int64_t tmp0 = (z2 + z3) * ((int64_t)1 << kConstBits);
        int64_t tmp1 = (z2 - z3) * ((int64_t)1 << kConstBits);
        const int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
        tmp0 = (int64_t)ip[56] * qp[56];
        tmp1 = (int64_t)ip[40] * qp[40];
        tmp2 = (int64_t)ip[24] * qp[24];
        tmp3 = (int64_t)ip[8] * qp[8];
        z1 = tmp0 + tmp3;
        z2 = tmp1 + tmp2;
        z3 = tmp0 + tmp2;
        int64_t z4 = tmp1 + tmp3;
        const int64_t z5 = (z3 + z4) * F1175;
        tmp0 *= F0298;
        tmp1 *= F2053;
        tmp2 *= F3072;
        tmp3 *= F1501;
        z1 *= -F0899;
        z2 *= -F2562;
        z3 *= -F1961;
        z4 *= -F0390;
        z3 += z5;
        z4 += z5;
        tmp0 += z1 + z3;
        tmp1 += z2 + z4;
        tmp2 += z2 + z3;
        tmp3 += z1 + z4;
        const int sh = kConstBits - kPass1Bits;
        ws[0 * 8 + c] = (int32_t)descale(tmp10 + tmp3, sh);
        ws[7 * 8 + c] = (int32_t)descale(tmp10 - tmp3, sh);
        ws[1 * 8 + c] = (int32_t)descale(tmp11 + tmp2, sh);
        ws[6 * 8 + c] = (int32_t)descale(tmp11 - tmp2, sh);
        ws[2 * 8 + c] = (int32_t)descale(tmp12 + tmp1, sh);
        ws[5 * 8 + c] = (int32_t)descale(tmp12 - tmp1, sh);
        ws[3 * 8 + c] = (int32_t)descale(tmp13 + tmp0, sh);
        ws[4 * 8 + c] = (int32_t)descale(tmp13 - tmp0, sh);
    }
    const int sh = kConstBits + kPass1Bits + 3;
    for (int r = 0; r < 8; ++r) {
        const int32_t *w = ws + r * 8;
        uint8_t *o = out + (size_t)r * stride;
        int64_t z2 = w[2], z3 = w[6];
        int64_t z1 = (z2 + z3) * F0541;
        int64_t tmp2 = z1 + z3 * (-F1847);
        int64_t tmp3 = z1 + z2 * F0765;
        // operands widened before the sum, as libjpeg-turbo's (JLONG)wsptr[0] + (JLONG)wsptr[4]
        int64_t tmp0 = ((int64_t)w[0] + w[4]) * ((int64_t)1 << kConstBits);
        int64_t tmp1 = ((int64_t)w[0] - w[4]) * ((int64_t)1 << kConstBits);
        const int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
        tmp0 = w[7];
        tmp1 = w[5];
        tmp2 = w[3];
        tmp3 = w[1];
        z1 = tmp0 + tmp3;
        z2 = tmp1 + tmp2;
        z3 = tmp0 + tmp2;
        int64_t z4 = tmp1 + tmp3;
        const int64_t z5 = (z3 + z4) * F1175;
        tmp0 *= F0298;
        tmp1 *= F2053;
        tmp2 *= F3072;
        tmp3 *= F1501;
        z1 *= -F0899;
        z2 *= -F2562;
        z3 *= -F1961;
        z4 *= -F0390;
        z3 += z5;
        z4 += z5;
        tmp0 += z1 + z3;
        tmp1 += z2 + z4;
        tmp2 += z2 + z3;
        tmp3 += z1 + z4;
        o[0] = range_limit(descale(tmp10 + tmp3, sh));
        o[7] = range_limit(descale(tmp10 - tmp3, sh));
        o[1] = range_limit(descale(tmp11 + tmp2, sh));
        o[6] = range_limit(descale(tmp11 - tmp2, sh));
        o[2] = range_limit(descale(tmp12 + tmp1, sh));
        o[5] = range_limit(descale(tmp12 - tmp1, sh));
        o[3] = range_limit(descale(tmp13 + tmp0, sh));
        o[4] = range_limit(descale(tmp13 - tmp0, sh));
    }
}

// ---- colour output (cv::imread IMREAD_COLOR = libjpeg JCS_RGB, reordered to
// BGR): chroma planes upsampled with libjpeg's default "fancy" triangle
// filters (jdsample.c h2v1 / h2v2; other ratios replicate), then the
// fixed-point YCbCr->RGB of jdcolor.c (16-bit tables, range-limited).
void h2v1_fancy(const uint8_t *in, int dw, uint8_t *out) {
    if (dw < 2) {
        out[0] = out[1] = in[0];
        return;
    }
    out[0] = in[0];
    out[1] = (uint8_t)((in[0] * 3 + in[1] + 2) >> 2);
    for (int c = 1; c < dw - 1; ++c) {
        const int v = in[c] * 3;
        out[2 * c] = (uint8_t)((v + in[c - 1] + 1) >> 2);
        out[2 * c + 1] = (uint8_t)((v + in[c + 1] + 2) >> 2);
    }
    const int c = dw - 1;
    out[2 * c] = (uint8_t)((in[c] * 3 + in[c - 1] + 1) >> 2);
    out[2 * c + 1] = in[c];
}

void h2v2_fancy_row(const uint8_t *in0, const uint8_t *in1, int dw, uint8_t *out) {
    if (dw < 2) {
        out[0] = out[1] = (uint8_t)(((in0[0] * 3 + in1[0]) * 4 + 8) >> 4);
        return;
    }
    int thiscolsum = in0[0] * 3 + in1[0];
    int nextcolsum = in0[1] * 3 + in1[1];
    out[0] = (uint8_t)((thiscolsum * 4 + 8) >> 4);
    out[1] = (uint8_t)((thiscolsum * 3 + nextcolsum + 7) >> 4);
    int lastcolsum = thiscolsum;
    thiscolsum = nextcolsum;
    for (int c = 1; c < dw - 1; ++c) {
        nextcolsum = in0[c + 1] * 3 + in1[c + 1];
        out[2 * c] = (uint8_t)((thiscolsum * 3 + lastcolsum + 8) >> 4);
        out[2 * c + 1] = (uint8_t)((thiscolsum * 3 + nextcolsum + 7) >> 4);
        lastcolsum = thiscolsum;
        thiscolsum = nextcolsum;
    }
    const int c = dw - 1;
    out[2 * c] = (uint8_t)((thiscolsum * 3 + lastcolsum + 8) >> 4);
    out[2 * c + 1] = (uint8_t)((thiscolsum * 4 + 7) >> 4);
}

// Component plane at full resolution (W x H): IDCT, then upsampling.
void component_full(const Comp &c, const uint16_t *q, int W, int H, int hmax, int vmax, std::vector<uint8_t> &out) {
    const int pw = c.bw * 8, ph = c.bh * 8;
    std::vector<uint8_t> plane((size_t)pw * ph);
    for (int by = 0; by < c.bh; ++by)
        for (int bx = 0; bx < c.bw; ++bx)
            idct_islow(&c.coef[((size_t)by * c.bw + bx) * 64], q, &plane[(size_t)by * 8 * pw + bx * 8], pw);
    const int dw = (int)(((long)W * c.h + hmax - 1) / hmax), dh = (int)(((long)H * c.v + vmax - 1) / vmax);
    const int fx = hmax / c.h, fy = vmax / c.v;
    out.assign((size_t)W * H, 0);
    std::vector<uint8_t> row((size_t)2 * dw + 2);
    for (int y = 0; y < H; ++y) {
        uint8_t *o = &out[(size_t)y * W];
        if (fx == 1 && fy == 1) {
            std::memcpy(o, &plane[(size_t)y * pw], W);
        } else if (fx == 2 && fy == 1) {
            h2v1_fancy(&plane[(size_t)y * pw], dw, row.data());
            std::memcpy(o, row.data(), W);
        } else if (fx == 2 && fy == 2) {
            const int r = y >> 1;
            const int nr = (y & 1) ? std::min(r + 1, dh - 1) : std::max(r - 1, 0);  // context rows replicate edges
            h2v2_fancy_row(&plane[(size_t)r * pw], &plane[(size_t)nr * pw], dw, row.data());
            std::memcpy(o, row.data(), W);
        } else {
            const uint8_t *src = &plane[(size_t)(y / fy) * pw];
            for (int x = 0; x < W; ++x) o[x] = src[x / fx];
        }
    }
}

inline uint8_t clamp255(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

// Parses markers up to the first SOS (size_only) or decodes the luminance
// plane into `gray` (W*H bytes), or with `bgr` the colour image (W*H*3, BGR).
int jpeg_decode(const std::vector<uint8_t> &buf, bool size_only, int &W, int &H, std::vector<uint8_t> *gray,
                std::vector<uint8_t> *bgr = nullptr) {
    Jpeg j;
    j.p = buf.data();
    j.end = buf.data() + buf.size();
    if (buf.size() < 4 || j.p[0] != 0xFF || j.p[1] != 0xD8) return ACMMP_ERR_IO;
    j.p += 2;
    bool decoded = false;
    while (j.p + 4 <= j.end) {
        if (j.p[0] != 0xFF) {
            ++j.p;
            continue;
        }
        const int m = j.p[1];
        j.p += 2;
        if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01 || m == 0xFF) {
            if (m == 0xFF) --j.p;
            continue;
        }
        if (m == 0xD9) break;  // EOI
        if (j.p + 2 > j.end) return ACMMP_ERR_IO;
        const int len = u16(j.p);
        const uint8_t *seg = j.p + 2;
        if (len < 2 || j.p + len > j.end) return ACMMP_ERR_IO;
        j.p += len;
        const int n = len - 2;
        if (m == 0xC0 || m == 0xC1 || m == 0xC2) {  // baseline / extended sequential / progressive Huffman
            j.progressive = m == 0xC2;
            if (n < 6 || seg[0] != 8) return ACMMP_ERR_UNSUPPORTED;
            j.H = u16(seg + 1);
            j.W = u16(seg + 3);
            j.ncomp = seg[5];
            if (j.ncomp < 1 || j.ncomp > 4 || n < 6 + 3 * j.ncomp || j.W <= 0 || j.H <= 0) return ACMMP_ERR_UNSUPPORTED;
            for (int c = 0; c < j.ncomp; ++c) {
                Comp &cp = j.comp[c];
                cp.id = seg[6 + 3 * c];
                cp.h = seg[7 + 3 * c] >> 4;
                cp.v = seg[7 + 3 * c] & 15;
                cp.tq = seg[8 + 3 * c];
                if (cp.h < 1 || cp.h > 4 || cp.v < 1 || cp.v > 4 || cp.tq > 3) return ACMMP_ERR_IO;
                j.hmax = std::max(j.hmax, cp.h);
                j.vmax = std::max(j.vmax, cp.v);
            }
            j.sof = true;
            W = j.W;
            H = j.H;
            if (size_only) return ACMMP_OK;
            // luminance = first component; it must carry the maximal sampling
            // factors (libjpeg's grayscale output then needs no upsampling)
            Comp &y = j.comp[0];
            if (y.h != j.hmax || y.v != j.vmax) return ACMMP_ERR_UNSUPPORTED;
            const int mcus_x = (j.W + 8 * j.hmax - 1) / (8 * j.hmax);
            const int mcus_y = (j.H + 8 * j.vmax - 1) / (8 * j.vmax);
            y.bw = mcus_x * y.h;
            y.bh = mcus_y * y.v;
            // a complete scan spends >= 2 bits per block (DC + EOB codes), so
            // a header claiming more than 8 blocks per file byte is corrupt
            // (checked before allocating from it)
            if ((size_t)mcus_x * mcus_y * j.hmax * j.vmax > 8 * buf.size() + 4096) return ACMMP_ERR_IO;
            y.coef.assign((size_t)y.bw * y.bh * 64, 0);
            if (bgr) {
                if (j.ncomp != 1 && j.ncomp != 3) return ACMMP_ERR_UNSUPPORTED;  // CMYK / YCCK
                for (int c = 1; c < j.ncomp; ++c) {
                    Comp &cp = j.comp[c];
                    if (j.hmax % cp.h || j.vmax % cp.v) return ACMMP_ERR_UNSUPPORTED;
                    cp.bw = mcus_x * cp.h;
                    cp.bh = mcus_y * cp.v;
                    cp.coef.assign((size_t)cp.bw * cp.bh * 64, 0);
                }
            }
        } else if (m >= 0xC2 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
            return ACMMP_ERR_UNSUPPORTED;  // lossless, differential, arithmetic
        } else if (m == 0xDB) {  // DQT
            int o = 0;
            while (o < n) {
                const int pq = seg[o] >> 4, tq = seg[o] & 15;
                if (tq > 3 || o + 1 + 64 * (pq + 1) > n) return ACMMP_ERR_IO;
                for (int k = 0; k < 64; ++k)
                    j.qt[tq][kZigzag[k]] = pq ? (uint16_t)u16(seg + o + 1 + 2 * k) : seg[o + 1 + k];
                j.qt_present[tq] = true;
                o += 1 + 64 * (pq + 1);
            }
        } else if (m == 0xC4) {  // DHT
            int o = 0;
            while (o < n) {
                if (o + 17 > n) return ACMMP_ERR_IO;
                const int tc = seg[o] >> 4, th = seg[o] & 15;
                int total = 0;
                for (int k = 0; k < 16; ++k) total += seg[o + 1 + k];
                if (th > 3 || tc > 1 || o + 17 + total > n) return ACMMP_ERR_IO;
                Huff &h = tc ? j.ac[th] : j.dc[th];
                if (!build_huff(h, seg + o + 1, seg + o + 17, total)) return ACMMP_ERR_IO;
                o += 17 + total;
            }
        } else if (m == 0xDD) {  // DRI
            if (n < 2) return ACMMP_ERR_IO;
            j.restart = u16(seg);
        } else if (m == 0xDA) {  // SOS
            if (!j.sof) return ACMMP_ERR_IO;
            if (!decode_scan(j, seg, n)) return j.err ? j.err : ACMMP_ERR_UNSUPPORTED;
            decoded = true;
        }
    }
    if (!j.sof) return ACMMP_ERR_IO;
    if (size_only) return ACMMP_OK;
    if (!decoded || !j.qt_present[j.comp[0].tq]) return ACMMP_ERR_IO;
    if (bgr) {
        std::vector<uint8_t> planes[3];
        for (int c = 0; c < j.ncomp; ++c) {
            if (!j.qt_present[j.comp[c].tq]) return ACMMP_ERR_IO;
            component_full(j.comp[c], j.qt[j.comp[c].tq], j.W, j.H, j.hmax, j.vmax, planes[c]);
        }
        const size_t P = (size_t)j.W * j.H;
        bgr->resize(P * 3);
        if (j.ncomp == 1) {
            for (size_t i = 0; i < P; ++i) (*bgr)[3 * i] = (*bgr)[3 * i + 1] = (*bgr)[3 * i + 2] = planes[0][i];
            return ACMMP_OK;
        }
        // jdcolor.c build_ycc_rgb_table / ycc_rgb_convert
        const int SB = 16;
        const long ONE_HALF = 1L << (SB - 1);
        auto FIX = [](double x) { return (long)(x * (1L << 16) + 0.5); };
        int cr_r[256], cb_b[256];
        long cr_g[256], cb_g[256];
        for (int i = 0, x = -128; i < 256; ++i, ++x) {
            cr_r[i] = (int)((FIX(1.40200) * x + ONE_HALF) >> SB);
            cb_b[i] = (int)((FIX(1.77200) * x + ONE_HALF) >> SB);
            cr_g[i] = (-FIX(0.71414)) * x;
            cb_g[i] = (-FIX(0.34414)) * x + ONE_HALF;
        }
        for (size_t i = 0; i < P; ++i) {
            const int yv = planes[0][i], cb = planes[1][i], cr = planes[2][i];
            (*bgr)[3 * i + 2] = clamp255(yv + cr_r[cr]);
            (*bgr)[3 * i + 1] = clamp255(yv + (int)((cb_g[cb] + cr_g[cr]) >> SB));
            (*bgr)[3 * i + 0] = clamp255(yv + cb_b[cb]);
        }
        return ACMMP_OK;
    }
    const Comp &y = j.comp[0];
    const int pw = y.bw * 8, ph = y.bh * 8;
    std::vector<uint8_t> full((size_t)pw * ph);
    for (int by = 0; by < y.bh; ++by)
        for (int bx = 0; bx < y.bw; ++bx)
            idct_islow(&y.coef[((size_t)by * y.bw + bx) * 64], j.qt[y.tq], &full[(size_t)by * 8 * pw + bx * 8], pw);
    gray->resize((size_t)j.W * j.H);
    for (int r = 0; r < j.H; ++r) std::memcpy(gray->data() + (size_t)r * j.W, &full[(size_t)r * pw], j.W);
    return ACMMP_OK;
}

// ------------------------------------------------------------- PGM / PFM
bool next_token(const std::vector<uint8_t> &b, size_t &o, std::string &tok) {
    tok.clear();
    while (o < b.size()) {
        if (b[o] == '#') {
            while (o < b.size() && b[o] != '\n') ++o;
        } else if (std::isspace(b[o])) {
            ++o;
        } else {
            break;
        }
    }
    while (o < b.size() && !std::isspace(b[o])) tok += (char)b[o++];
    return !tok.empty();
}

int pnm_decode(const std::vector<uint8_t> &b, bool size_only, int &W, int &H, std::vector<float> *out) {
    size_t o = 0;
    std::string magic, tw, th, tm;
    if (!next_token(b, o, magic) || !next_token(b, o, tw) || !next_token(b, o, th) || !next_token(b, o, tm))
        return ACMMP_ERR_IO;
    W = std::atoi(tw.c_str());
    H = std::atoi(th.c_str());
    if (W <= 0 || H <= 0) return ACMMP_ERR_IO;
    if (size_only) return ACMMP_OK;
    ++o;  // single whitespace after the header
    const size_t P = (size_t)W * H;
    if (magic == "P5") {
        const int maxv = std::atoi(tm.c_str());
        const int bps = maxv > 255 ? 2 : 1;
        if (maxv <= 0 || maxv > 65535 || o + P * bps > b.size()) return ACMMP_ERR_IO;
        out->resize(P);
        for (size_t i = 0; i < P; ++i)
            (*out)[i] = bps == 1 ? (float)b[o + i] : (float)((b[o + 2 * i] << 8) | b[o + 2 * i + 1]);
        return ACMMP_OK;
    }
    if (magic == "Pf") {  // grayscale PFM: rows bottom-to-top, scale sign = endianness
        const double scale = std::atof(tm.c_str());
        if (o + P * 4 > b.size()) return ACMMP_ERR_IO;
        out->resize(P);
        const bool little = scale < 0;
        for (int r = 0; r < H; ++r)
            for (int c = 0; c < W; ++c) {
                const uint8_t *q = &b[o + ((size_t)(H - 1 - r) * W + c) * 4];
                uint32_t u = little ? (uint32_t)q[0] | (uint32_t)q[1] << 8 | (uint32_t)q[2] << 16 | (uint32_t)q[3] << 24
                                    : (uint32_t)q[3] | (uint32_t)q[2] << 8 | (uint32_t)q[1] << 16 | (uint32_t)q[0] << 24;
                float f;
                std::memcpy(&f, &u, 4);
                (*out)[(size_t)r * W + c] = f;
            }
        return ACMMP_OK;
    }
    return ACMMP_ERR_UNSUPPORTED;
}

int decode_any(const char *path, bool size_only, int &W, int &H, std::vector<float> *out) {
    std::vector<uint8_t> buf;
    if (!path || !read_file(path, buf)) return ACMMP_ERR_IO;
    if (buf.size() >= 2 && buf[0] == 0xFF && buf[1] == 0xD8) {
        std::vector<uint8_t> g;
        const int rc = jpeg_decode(buf, size_only, W, H, size_only ? nullptr : &g);
        if (rc || size_only) return rc;
        out->resize(g.size());
        for (size_t i = 0; i < g.size(); ++i) (*out)[i] = (float)g[i];  // convertTo(CV_32FC1)
        return ACMMP_OK;
    }
    if (buf.size() >= 2 && buf[0] == 'P') return pnm_decode(buf, size_only, W, H, out);
    return ACMMP_ERR_UNSUPPORTED;
}

// ------------------------------------------------------------------ PNG
// cv::imread(path, IMREAD_UNCHANGED) of the non-interlaced 8/16-bit gray /
// RGB / RGBA PNGs the seeded-prior loader reads (src/acmmp_definitions.cpp:
// 104-106): samples as stored (16-bit big-endian -> host), colour channels
// reordered to OpenCV's BGR(A).
uint32_t be32(const uint8_t *q) { return (uint32_t)q[0] << 24 | (uint32_t)q[1] << 16 | (uint32_t)q[2] << 8 | q[3]; }

int png_decode(const std::vector<uint8_t> &b, int &W, int &H, int &C, int &depth, std::vector<uint16_t> *out) {
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    if (b.size() < 8 || std::memcmp(b.data(), sig, 8) != 0) return ACMMP_ERR_IO;
    size_t o = 8;
    int ctype = -1, interlace = 0;
    std::vector<uint8_t> z;
    while (o + 12 <= b.size()) {
        const uint32_t len = be32(&b[o]);
        if (o + 12 + (size_t)len > b.size()) return ACMMP_ERR_IO;
        const uint8_t *type = &b[o + 4], *d = &b[o + 8];
        if (!std::memcmp(type, "IHDR", 4)) {
            if (len < 13) return ACMMP_ERR_IO;
            W = (int)be32(d);
            H = (int)be32(d + 4);
            depth = d[8];
            ctype = d[9];
            interlace = d[12];
        } else if (!std::memcmp(type, "IDAT", 4)) {
            z.insert(z.end(), d, d + len);
        } else if (!std::memcmp(type, "IEND", 4)) {
            break;
        }
        o += 12 + len;
    }
    if (ctype < 0 || W <= 0 || H <= 0) return ACMMP_ERR_IO;
    if (interlace || (depth != 8 && depth != 16)) return ACMMP_ERR_UNSUPPORTED;
    C = ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 4 ? 2 : ctype == 6 ? 4 : 0;
    if (C == 0) return ACMMP_ERR_UNSUPPORTED;  // palette
    if (!out) return ACMMP_OK;
    const size_t bpp = (size_t)C * depth / 8, stride = bpp * W;
    // zlib inflates at most ~1032:1: a header implying more raw bytes than
    // that is corrupt (checked before allocating from it)
    if ((stride + 1) * (size_t)H / 1032 > z.size() + 1) return ACMMP_ERR_IO;
    std::vector<uint8_t> raw((stride + 1) * H);
    uLongf rawlen = (uLongf)raw.size();
    if (uncompress(raw.data(), &rawlen, z.data(), (uLong)z.size()) != Z_OK || rawlen != raw.size())
        return ACMMP_ERR_IO;
    std::vector<uint8_t> prev(stride, 0), cur(stride);
    out->resize((size_t)W * H * C);
    for (int y = 0; y < H; ++y) {
        const uint8_t f = raw[(stride + 1) * y];
        const uint8_t *src = &raw[(stride + 1) * y + 1];
        for (size_t i = 0; i < stride; ++i) {
            const int a = i >= bpp ? cur[i - bpp] : 0, up = prev[i], c = i >= bpp ? prev[i - bpp] : 0;
            int v = src[i];
            switch (f) {
                case 0: break;
                case 1: v += a; break;
                case 2: v += up; break;
                case 3: v += (a + up) >> 1; break;
                case 4: {
                    const int p0 = a + up - c, pa = std::abs(p0 - a), pb = std::abs(p0 - up), pc = std::abs(p0 - c);
                    v += (pa <= pb && pa <= pc) ? a : (pb <= pc ? up : c);
                    break;
                }
                default: return ACMMP_ERR_IO;
            }
            cur[i] = (uint8_t)v;
        }
        for (int x = 0; x < W; ++x)
            for (int k = 0; k < C; ++k) {
                // RGB(A) -> BGR(A), as cv::imread
                const int sk = (C >= 3 && k < 3) ? 2 - k : k;
                const size_t si = ((size_t)x * C + sk) * (depth / 8);
                (*out)[((size_t)y * W + x) * C + k] = depth == 16 ? (uint16_t)(cur[si] << 8 | cur[si + 1]) : cur[si];
            }
        prev.swap(cur);
    }
    return ACMMP_OK;
}

// ------------------------------------------------------------- resize
// cv::resize(src, dst, Size(nw, nh), 0, 0, INTER_LINEAR) for CV_32FC1: the
// exact-2x downscale takes OpenCV's INTER_AREA fast path (2x2 mean), other
// factors the separable linear filter with half-pixel centres, edge clamp,
// horizontal pass first.
void resize_linear(const float *src, int sw, int sh, float *dst, int dw, int dh) {
    const double sx = (double)sw / dw, sy = (double)sh / dh;
    const int isx = (int)std::lround(sx), isy = (int)std::lround(sy);
    if (std::fabs(sx - isx) < 2.220446049250313e-16 && std::fabs(sy - isy) < 2.220446049250313e-16 && isx == 2 &&
        isy == 2) {
        for (int y = 0; y < dh; ++y)
            for (int x = 0; x < dw; ++x) {
                const float *r0 = src + (size_t)(2 * y) * sw + 2 * x, *r1 = r0 + sw;
                dst[(size_t)y * dw + x] = ((r0[0] + r0[1]) + (r1[0] + r1[1])) * 0.25f;
            }
        return;
    }
    std::vector<int> x0(dw), x1(dw);
    std::vector<float> ax(dw);
    for (int x = 0; x < dw; ++x) {
        float fx = (float)((x + 0.5) * sx - 0.5);
        int ix = (int)std::floor(fx);
        fx -= (float)ix;
        if (ix < 0) {
            fx = 0.f;
            ix = 0;
        }
        if (ix >= sw - 1) {
            fx = 0.f;
            ix = sw - 1;
        }
        x0[x] = ix;
        x1[x] = std::min(ix + 1, sw - 1);
        ax[x] = fx;
    }
    std::vector<float> row0(dw), row1(dw);
    for (int y = 0; y < dh; ++y) {
        float fy = (float)((y + 0.5) * sy - 0.5);
        int iy = (int)std::floor(fy);
        fy -= (float)iy;
        if (iy < 0) {
            fy = 0.f;
            iy = 0;
        }
        if (iy >= sh - 1) {
            fy = 0.f;
            iy = sh - 1;
        }
        const int iy1 = std::min(iy + 1, sh - 1);
        const float *s0 = src + (size_t)iy * sw, *s1 = src + (size_t)iy1 * sw;
        for (int x = 0; x < dw; ++x) {
            row0[x] = s0[x0[x]] * (1.f - ax[x]) + s0[x1[x]] * ax[x];
            row1[x] = s1[x0[x]] * (1.f - ax[x]) + s1[x1[x]] * ax[x];
        }
        for (int x = 0; x < dw; ++x) dst[(size_t)y * dw + x] = row0[x] * (1.f - fy) + row1[x] * fy;
    }
}

// ---- 8-bit PNG writer (gray or RGB, one IDAT, filter 0), zlib at best speed
void put_chunk(std::vector<uint8_t> &png, const char *type, const std::vector<uint8_t> &data) {
    const uint32_t n = (uint32_t)data.size();
    const uint8_t len[4] = {(uint8_t)(n >> 24), (uint8_t)(n >> 16), (uint8_t)(n >> 8), (uint8_t)n};
    png.insert(png.end(), len, len + 4);
    const size_t start = png.size();
    png.insert(png.end(), type, type + 4);
    png.insert(png.end(), data.begin(), data.end());
    const uLong crc = crc32(0L, png.data() + start, (uInt)(png.size() - start));
    const uint8_t c[4] = {(uint8_t)(crc >> 24), (uint8_t)(crc >> 16), (uint8_t)(crc >> 8), (uint8_t)crc};
    png.insert(png.end(), c, c + 4);
}

int write_png8(const char *path, int w, int h, int channels, const uint8_t *px) {
    std::vector<uint8_t> raw;
    raw.reserve((size_t)h * (channels * w + 1));
    for (int y = 0; y < h; ++y) {
        raw.push_back(0);
        raw.insert(raw.end(), px + (size_t)y * channels * w, px + (size_t)(y + 1) * channels * w);
    }
    uLongf zlen = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), Z_BEST_SPEED) != Z_OK)
        return ACMMP_ERR_IO;
    z.resize(zlen);
    std::vector<uint8_t> png = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    std::vector<uint8_t> ihdr = {(uint8_t)(w >> 24), (uint8_t)(w >> 16), (uint8_t)(w >> 8), (uint8_t)w,
                                 (uint8_t)(h >> 24), (uint8_t)(h >> 16), (uint8_t)(h >> 8), (uint8_t)h,
                                 8, (uint8_t)(channels == 3 ? 2 : 0), 0, 0, 0};
    put_chunk(png, "IHDR", ihdr);
    put_chunk(png, "IDAT", z);
    put_chunk(png, "IEND", {});
    FILE *f = std::fopen(path, "wb");
    if (!f) return ACMMP_ERR_IO;
    const bool ok = std::fwrite(png.data(), 1, png.size(), f) == png.size();
    std::fclose(f);
    return ok ? ACMMP_OK : ACMMP_ERR_IO;
}

}  // namespace

// triangulation.png (acmmp_pipeline.cpp) and the fusion's debug images
int acmmp_internal_write_png(const char *path, int w, int h, int channels, const uint8_t *px) {
    if (!path || !px || w <= 0 || h <= 0 || (channels != 1 && channels != 3)) return ACMMP_ERR_ARG;
    return write_png8(path, w, h, channels, px);
}

int acmmp_internal_read_image_bgr(const char *path, std::vector<uint8_t> &bgr, int &W, int &H) {
    std::vector<uint8_t> buf;
    if (!path || !read_file(path, buf)) return ACMMP_ERR_IO;
    W = H = 0;
    if (buf.size() >= 2 && buf[0] == 0xFF && buf[1] == 0xD8) return jpeg_decode(buf, false, W, H, nullptr, &bgr);
    int C = 0, depth = 0;
    std::vector<uint16_t> px;
    const int rc = png_decode(buf, W, H, C, depth, &px);
    if (rc) return rc;
    if (depth != 8) return ACMMP_ERR_UNSUPPORTED;
    bgr.resize((size_t)W * H * 3);
    for (size_t i = 0; i < (size_t)W * H; ++i)
        for (int k = 0; k < 3; ++k) bgr[3 * i + k] = (uint8_t)px[i * C + (C >= 3 ? k : 0)];
    return ACMMP_OK;
}

extern "C" {

int acmmp_image_size(const char *path, int *width, int *height) {
    if (!width || !height) return ACMMP_ERR_ARG;
    int W = 0, H = 0;
    const int rc = decode_any(path, true, W, H, nullptr);
    if (rc) return rc;
    *width = W;
    *height = H;
    return ACMMP_OK;
}

int acmmp_read_image_gray(const char *path, float *out, size_t capacity, int *width, int *height) {
    if (!width || !height) return ACMMP_ERR_ARG;
    int W = 0, H = 0;
    std::vector<float> img;
    const int rc = decode_any(path, false, W, H, &img);
    if (rc) return rc;
    *width = W;
    *height = H;
    if (!out || capacity < img.size()) return ACMMP_ERR_ARG;
    std::memcpy(out, img.data(), img.size() * sizeof(float));
    return ACMMP_OK;
}

int acmmp_read_image_bgr(const char *path, uint8_t *out, size_t capacity, int *width, int *height) {
    if (!width || !height) return ACMMP_ERR_ARG;
    int W = 0, H = 0;
    std::vector<uint8_t> bgr;
    const int rc = acmmp_internal_read_image_bgr(path, bgr, W, H);
    if (rc) return rc;
    *width = W;
    *height = H;
    if (!out || capacity < bgr.size()) return ACMMP_ERR_ARG;
    std::memcpy(out, bgr.data(), bgr.size());
    return ACMMP_OK;
}

int acmmp_read_png(const char *path, uint16_t *out, size_t capacity, int *width, int *height, int *channels,
                   int *bit_depth) {
    if (!width || !height || !channels) return ACMMP_ERR_ARG;
    std::vector<uint8_t> buf;
    if (!path || !read_file(path, buf)) return ACMMP_ERR_IO;
    int W = 0, H = 0, C = 0, depth = 0;
    int rc = png_decode(buf, W, H, C, depth, nullptr);
    if (rc) return rc;
    *width = W;
    *height = H;
    *channels = C;
    if (bit_depth) *bit_depth = depth;
    if (!out || capacity < (size_t)W * H * C) return ACMMP_ERR_ARG;
    std::vector<uint16_t> px;
    rc = png_decode(buf, W, H, C, depth, &px);
    if (rc) return rc;
    std::memcpy(out, px.data(), px.size() * sizeof(uint16_t));
    return ACMMP_OK;
}

int acmmp_resize_linear(const float *src, int src_width, int src_height, float *dst, int dst_width,
                        int dst_height) {
    if (!src || !dst || src_width <= 0 || src_height <= 0 || dst_width <= 0 || dst_height <= 0) return ACMMP_ERR_ARG;
    resize_linear(src, src_width, src_height, dst, dst_width, dst_height);
    return ACMMP_OK;
}

}  // extern "C"
