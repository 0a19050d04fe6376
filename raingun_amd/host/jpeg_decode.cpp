// jpeg_decode.cpp — JPEG decoder for scene textures (baseline + progressive
// Huffman, 8-bit, 1 or 3 components).
//
// The reference decodes its textures with jpeg-decoder 0.1.11 through
// image::open (raingun-lib/src/material.rs:34-47).  The default flavour
// (RGH_JPEG_REFERENCE) restates that decoder's arithmetic -- a port of
// stb_image: integer IDCT with 12-bit constants, triangle chroma upsampling
// with its rounding, BT.601 YCbCr->RGB in f32 -- so the reference's golden
// renders examples/test{1,3}.png are reproduced byte for byte
// (tests/test_oracle_golden.py).  RGH_JPEG_LIBJPEG follows the IJG/libjpeg-turbo
// defaults instead (what PIL uses: ISLOW IDCT, fancy upsampling, fixed-point
// colour tables); its texels equal PIL's (tests/test_host_native.py) and it is
// the negative control of the golden-render pin.
#include "image_codec.h"

#include <array>
#include <cstring>

namespace rgh {
namespace {

constexpr int kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct Huffman {
    // canonical decoding tables (ITU T.81 F.2.2.3)
    int maxcode[18];
    int valptr[17];
    int mincode[17];
    uint8_t vals[256];
    bool present = false;
};

struct Component {
    int id = 0, h = 1, v = 1, tq = 0;
    int td = 0, ta = 0;           // current scan's tables
    int bw = 0, bh = 0;           // block grid (padded to whole MCUs)
    int dw = 0, dh = 0;           // downsampled size in samples
    int pred = 0;
    std::vector<int16_t> coef;    // bw*bh blocks * 64, natural order
};

struct Decoder {
    const uint8_t *p = nullptr, *end = nullptr;
    std::string err;
    uint16_t qt[4][64] = {};
    Huffman dc[4], ac[4];
    std::vector<Component> comps;
    int width = 0, height = 0, max_h = 1, max_v = 1, mcux = 0, mcuy = 0;
    bool progressive = false;
    int restart = 0;
    bool adobe = false;
    int adobe_transform = -1;
    // bit reader
    uint32_t bits = 0;
    int nbits = 0;
    bool hit_marker = false;
    int eobrun = 0;

    bool fail(const char *m) {
        if (err.empty()) err = m;
        return false;
    }
    int u8() { return p < end ? *p++ : (hit_marker = true, 0); }
    int u16() { int a = u8(); return (a << 8) | u8(); }

    void reset_bits() { bits = 0; nbits = 0; hit_marker = false; }
    void fill() {
        while (nbits <= 24) {
            int b = 0;
            if (!hit_marker && p < end) {
                b = *p;
                if (b == 0xFF) {
                    int nxt = p + 1 < end ? p[1] : 0;
                    if (nxt == 0x00) { p += 2; }
                    else { hit_marker = true; b = 0; }  // marker: feed zeros (IJG behaviour)
                } else {
                    ++p;
                }
            }
            bits |= (uint32_t)b << (24 - nbits);
            nbits += 8;
        }
    }
    int getbit() {
        if (nbits < 1) fill();
        int r = (int)(bits >> 31);
        bits <<= 1;
        --nbits;
        return r;
    }
    int getbits(int n) {
        if (n == 0) return 0;
        if (nbits < n) fill();
        int r = (int)(bits >> (32 - n));
        bits <<= n;
        nbits -= n;
        return r;
    }
    static int extend(int v, int t) { return v < (1 << (t - 1)) ? v - (1 << t) + 1 : v; }
    int decode(const Huffman &h) {
        int code = 0;
        for (int l = 1; l <= 16; ++l) {
            code = (code << 1) | getbit();
            if (code <= h.maxcode[l]) return h.vals[h.valptr[l] + code - h.mincode[l]];
        }
        return 0;  // corrupt data: IJG returns 0 after a warning
    }

    bool read_dqt(int len) {
        const uint8_t *stop = p + len;
        while (p < stop) {
            int pq = u8(), tq = pq & 15;
            if (tq > 3) return fail("bad DQT");
            for (int i = 0; i < 64; ++i) qt[tq][kZigzag[i]] = (uint16_t)((pq >> 4) ? u16() : u8());
        }
        return true;
    }
    bool read_dht(int len) {
        const uint8_t *stop = p + len;
        while (p < stop) {
            int tc = u8(), th = tc & 15;
            if (th > 3) return fail("bad DHT");
            Huffman &h = (tc >> 4) ? ac[th] : dc[th];
            int counts[17] = {0};
            int total = 0;
            for (int l = 1; l <= 16; ++l) { counts[l] = u8(); total += counts[l]; }
            if (total > 256) return fail("bad DHT count");
            for (int i = 0; i < total; ++i) h.vals[i] = (uint8_t)u8();
            int code = 0, k = 0;
            for (int l = 1; l <= 16; ++l) {
                h.valptr[l] = k;
                h.mincode[l] = code;
                code += counts[l];
                k += counts[l];
                h.maxcode[l] = counts[l] ? code - 1 : -1;
                code <<= 1;
            }
            h.maxcode[17] = 0x7fffffff;
            h.present = true;
        }
        return true;
    }
    bool read_sof(int len, bool prog) {
        progressive = prog;
        if (u8() != 8) return fail("only 8-bit JPEG is supported");
        height = u16();
        width = u16();
        int nc = u8();
        if (width <= 0 || height <= 0 || (nc != 1 && nc != 3)) return fail("unsupported JPEG geometry/components");
        comps.resize(nc);
        for (auto &c : comps) {
            c.id = u8();
            int hv = u8();
            c.h = hv >> 4;
            c.v = hv & 15;
            c.tq = u8() & 3;
            if (c.h < 1 || c.h > 4 || c.v < 1 || c.v > 4) return fail("bad sampling factors");
            max_h = std::max(max_h, c.h);
            max_v = std::max(max_v, c.v);
        }
        (void)len;
        mcux = (width + 8 * max_h - 1) / (8 * max_h);
        mcuy = (height + 8 * max_v - 1) / (8 * max_v);
        for (auto &c : comps) {
            c.bw = mcux * c.h;
            c.bh = mcuy * c.v;
            c.dw = (width * c.h + max_h - 1) / max_h;
            c.dh = (height * c.v + max_v - 1) / max_v;
            c.coef.assign((size_t)c.bw * c.bh * 64, 0);
        }
        return true;
    }

    // ---- block decoders (ITU T.81 F.2 / G.1.2; libjpeg jdhuff.c / jdphuff.c)
    void block_baseline(Component &c, int16_t *blk) {
        int t = decode(dc[c.td]);
        int diff = t ? extend(getbits(t), t) : 0;
        c.pred += diff;
        blk[0] = (int16_t)c.pred;
        for (int k = 1; k < 64;) {
            int rs = decode(ac[c.ta]);
            int r = rs >> 4, s = rs & 15;
            if (s) {
                k += r;
                if (k > 63) break;
                blk[kZigzag[k]] = (int16_t)extend(getbits(s), s);
                ++k;
            } else {
                if (r != 15) break;
                k += 16;
            }
        }
    }
    void block_dc_first(Component &c, int16_t *blk, int al) {
        int t = decode(dc[c.td]);
        int diff = t ? extend(getbits(t), t) : 0;
        c.pred += diff;
        blk[0] = (int16_t)(c.pred * (1 << al));
    }
    void block_dc_refine(int16_t *blk, int al) {
        if (getbit()) blk[0] = (int16_t)(blk[0] | (1 << al));
    }
    void block_ac_first(Component &c, int16_t *blk, int ss, int se, int al) {
        if (eobrun > 0) { --eobrun; return; }
        for (int k = ss; k <= se; ++k) {
            int rs = decode(ac[c.ta]);
            int r = rs >> 4, s = rs & 15;
            if (s) {
                k += r;
                if (k > 63) break;
                blk[kZigzag[k]] = (int16_t)(extend(getbits(s), s) * (1 << al));
            } else {
                if (r < 15) {
                    eobrun = (1 << r) - 1;
                    if (r) eobrun += getbits(r);
                    break;
                }
                k += 15;
            }
        }
    }
    void refine_nonzero(int16_t *c, int p1, int m1) {
        if (getbit() && (*c & p1) == 0) *c = (int16_t)(*c >= 0 ? *c + p1 : *c + m1);
    }
    void block_ac_refine(Component &c, int16_t *blk, int ss, int se, int al) {
        const int p1 = 1 << al, m1 = -1 * (1 << al);
        int k = ss;
        if (eobrun == 0) {
            for (; k <= se; ++k) {
                int rs = decode(ac[c.ta]);
                int r = rs >> 4, s = rs & 15;
                if (s) {
                    s = getbit() ? p1 : m1;
                } else if (r != 15) {
                    eobrun = 1 << r;
                    if (r) eobrun += getbits(r);
                    break;
                }
                do {
                    int16_t *cp = blk + kZigzag[k];
                    if (*cp != 0) refine_nonzero(cp, p1, m1);
                    else if (--r < 0) break;
                    ++k;
                } while (k <= se);
                if (s && k <= 63) blk[kZigzag[k]] = (int16_t)s;
            }
        }
        if (eobrun > 0) {
            for (; k <= se; ++k) {
                int16_t *cp = blk + kZigzag[k];
                if (*cp != 0) refine_nonzero(cp, p1, m1);
            }
            --eobrun;
        }
    }

    bool read_restart_marker() {
        // align to a byte, then expect RSTn
        nbits = 0;
        bits = 0;
        hit_marker = false;
        while (p + 1 < end && !(p[0] == 0xFF && p[1] >= 0xD0 && p[1] <= 0xD7)) ++p;
        if (p + 1 < end) p += 2;
        for (auto &c : comps) c.pred = 0;
        eobrun = 0;
        return true;
    }

    bool read_sos() {
        int ns = u16();
        (void)ns;
        int n = u8();
        if (n < 1 || n > 4) return fail("bad SOS");
        std::vector<Component *> sc;
        for (int i = 0; i < n; ++i) {
            int id = u8(), t = u8();
            Component *cp = nullptr;
            for (auto &c : comps)
                if (c.id == id) cp = &c;
            if (!cp) return fail("SOS names an unknown component");
            cp->td = t >> 4;
            cp->ta = t & 15;
            sc.push_back(cp);
        }
        int ss = u8(), se = u8(), a = u8();
        int ah = a >> 4, al = a & 15;
        if (!progressive) { ss = 0; se = 63; ah = al = 0; }
        reset_bits();
        eobrun = 0;
        for (auto *c : sc) c->pred = 0;
        int restarts_left = restart;
        auto do_block = [&](Component &c, int bx, int by) {
            int16_t *blk = c.coef.data() + ((size_t)by * c.bw + bx) * 64;
            if (!progressive) block_baseline(c, blk);
            else if (ss == 0) { if (ah == 0) block_dc_first(c, blk, al); else block_dc_refine(blk, al); }
            else if (ah == 0) block_ac_first(c, blk, ss, se, al);
            else block_ac_refine(c, blk, ss, se, al);
        };
        auto restart_tick = [&]() {
            if (restart) {
                if (restarts_left == 0) { read_restart_marker(); restarts_left = restart; }
                --restarts_left;
            }
        };
        if (sc.size() == 1) {
            // non-interleaved: the component's own block grid, unpadded (T.81 A.2.2)
            Component &c = *sc[0];
            int cbw = (c.dw + 7) / 8, cbh = (c.dh + 7) / 8;
            for (int by = 0; by < cbh; ++by)
                for (int bx = 0; bx < cbw; ++bx) {
                    restart_tick();
                    do_block(c, bx, by);
                }
        } else {
            for (int my = 0; my < mcuy; ++my)
                for (int mx = 0; mx < mcux; ++mx) {
                    restart_tick();
                    for (auto *cp : sc)
                        for (int v = 0; v < cp->v; ++v)
                            for (int h = 0; h < cp->h; ++h) do_block(*cp, mx * cp->h + h, my * cp->v + v);
                }
        }
        // skip to the next marker
        while (p + 1 < end && !(p[0] == 0xFF && p[1] != 0x00 && !(p[1] >= 0xD0 && p[1] <= 0xD7))) ++p;
        return true;
    }
};

// ---- ISLOW inverse DCT (IJG jidctint.c algorithm: LL&M, CONST_BITS 13, PASS1_BITS 2)
constexpr int CONST_BITS = 13, PASS1_BITS = 2;
constexpr int32_t F_0_298631336 = 2446, F_0_390180644 = 3196, F_0_541196100 = 4433, F_0_765366865 = 6270,
                  F_0_899976223 = 7373, F_1_175875602 = 9633, F_1_501321110 = 12299, F_1_847759065 = 15137,
                  F_1_961570560 = 16069, F_2_053119869 = 16819, F_2_562915447 = 20995, F_3_072711026 = 25172;
inline int32_t descale(int64_t x, int n) { return (int32_t)((x + ((int64_t)1 << (n - 1))) >> n); }

// post-IDCT range limit: index & 1023, values -512..511 -> clamp(v + 128) (IJG prepare_range_limit_table)
struct RangeLimit {
    uint8_t t[1024];
    RangeLimit() {
        for (int i = 0; i < 1024; ++i) {
            int v = i < 512 ? i : i - 1024;
            int o = v + 128;
            t[i] = (uint8_t)(o < 0 ? 0 : o > 255 ? 255 : o);
        }
        // IJG's table maps [128, 511] to 255 and [512, 895] to 0, as above
    }
};
const RangeLimit kRange;

void idct_islow(const int16_t *in, const uint16_t *q, uint8_t *out, int stride) {
    int32_t ws[64];
    for (int col = 0; col < 8; ++col) {
        const int16_t *ip = in + col;
        const uint16_t *qp = q + col;
        int32_t *wp = ws + col;
        if (ip[8] == 0 && ip[16] == 0 && ip[24] == 0 && ip[32] == 0 && ip[40] == 0 && ip[48] == 0 && ip[56] == 0) {
            int32_t dc = ((int32_t)ip[0] * qp[0]) * (1 << PASS1_BITS);
            for (int r = 0; r < 8; ++r) wp[8 * r] = dc;
            continue;
        }
        int64_t z2 = (int64_t)ip[16] * qp[16], z3 = (int64_t)ip[48] * qp[48];
        int64_t z1 = (z2 + z3) * F_0_541196100;
        int64_t tmp2 = z1 + z3 * (-F_1_847759065);
        int64_t tmp3 = z1 + z2 * F_0_765366865;
        z2 = (int64_t)ip[0] * qp[0];
        z3 = (int64_t)ip[32] * qp[32];
        int64_t tmp0 = (z2 + z3) * (1 << CONST_BITS);
        int64_t tmp1 = (z2 - z3) * (1 << CONST_BITS);
        int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
        tmp0 = (int64_t)ip[56] * qp[56];
        tmp1 = (int64_t)ip[40] * qp[40];
        tmp2 = (int64_t)ip[24] * qp[24];
        tmp3 = (int64_t)ip[8] * qp[8];
        z1 = tmp0 + tmp3;
        z2 = tmp1 + tmp2;
        z3 = tmp0 + tmp2;
        int64_t z4 = tmp1 + tmp3;
        int64_t z5 = (z3 + z4) * F_1_175875602;
        tmp0 *= F_0_298631336;
        tmp1 *= F_2_053119869;
        tmp2 *= F_3_072711026;
        tmp3 *= F_1_501321110;
        z1 *= -F_0_899976223;
        z2 *= -F_2_562915447;
        z3 *= -F_1_961570560;
        z4 *= -F_0_390180644;
        z3 += z5;
        z4 += z5;
        tmp0 += z1 + z3;
        tmp1 += z2 + z4;
        tmp2 += z2 + z3;
        tmp3 += z1 + z4;
        const int sh = CONST_BITS - PASS1_BITS;
        wp[0] = descale(tmp10 + tmp3, sh);
        wp[56] = descale(tmp10 - tmp3, sh);
        wp[8] = descale(tmp11 + tmp2, sh);
        wp[48] = descale(tmp11 - tmp2, sh);
        wp[16] = descale(tmp12 + tmp1, sh);
        wp[40] = descale(tmp12 - tmp1, sh);
        wp[24] = descale(tmp13 + tmp0, sh);
        wp[32] = descale(tmp13 - tmp0, sh);
    }
    for (int row = 0; row < 8; ++row) {
        const int32_t *wp = ws + 8 * row;
        uint8_t *op = out + (size_t)row * stride;
        const int sh = CONST_BITS + PASS1_BITS + 3;
        if (wp[1] == 0 && wp[2] == 0 && wp[3] == 0 && wp[4] == 0 && wp[5] == 0 && wp[6] == 0 && wp[7] == 0) {
            uint8_t v = kRange.t[descale(wp[0], PASS1_BITS + 3) & 1023];
            for (int i = 0; i < 8; ++i) op[i] = v;
            continue;
        }
        int64_t z2 = wp[2], z3 = wp[6];
        int64_t z1 = (z2 + z3) * F_0_541196100;
        int64_t tmp2 = z1 + z3 * (-F_1_847759065);
        int64_t tmp3 = z1 + z2 * F_0_765366865;
        int64_t tmp0 = ((int64_t)wp[0] + wp[4]) * (1 << CONST_BITS);
        int64_t tmp1 = ((int64_t)wp[0] - wp[4]) * (1 << CONST_BITS);
        int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
        tmp0 = wp[7];
        tmp1 = wp[5];
        tmp2 = wp[3];
        tmp3 = wp[1];
        z1 = tmp0 + tmp3;
        z2 = tmp1 + tmp2;
        z3 = tmp0 + tmp2;
        int64_t z4 = tmp1 + tmp3;
        int64_t z5 = (z3 + z4) * F_1_175875602;
        tmp0 *= F_0_298631336;
        tmp1 *= F_2_053119869;
        tmp2 *= F_3_072711026;
        tmp3 *= F_1_501321110;
        z1 *= -F_0_899976223;
        z2 *= -F_2_562915447;
        z3 *= -F_1_961570560;
        z4 *= -F_0_390180644;
        z3 += z5;
        z4 += z5;
        tmp0 += z1 + z3;
        tmp1 += z2 + z4;
        tmp2 += z2 + z3;
        tmp3 += z1 + z4;
        op[0] = kRange.t[descale(tmp10 + tmp3, sh) & 1023];
        op[7] = kRange.t[descale(tmp10 - tmp3, sh) & 1023];
        op[1] = kRange.t[descale(tmp11 + tmp2, sh) & 1023];
        op[6] = kRange.t[descale(tmp11 - tmp2, sh) & 1023];
        op[2] = kRange.t[descale(tmp12 + tmp1, sh) & 1023];
        op[5] = kRange.t[descale(tmp12 - tmp1, sh) & 1023];
        op[3] = kRange.t[descale(tmp13 + tmp0, sh) & 1023];
        op[4] = kRange.t[descale(tmp13 - tmp0, sh) & 1023];
    }
}

// ---- upsampling to full resolution (IJG jdsample.c)
std::vector<uint8_t> upsample(const std::vector<uint8_t> &plane, int pw, int dw, int dh, int hf, int vf, int W,
                              int H) {
    std::vector<uint8_t> out((size_t)W * H);
    auto at = [&](int x, int y) -> int {
        y = y < 0 ? 0 : (y >= dh ? dh - 1 : y);  // context rows replicate the edge rows (jdmainct.c)
        return plane[(size_t)y * pw + x];
    };
    if (hf == 1 && vf == 1) {
        for (int y = 0; y < H; ++y) std::memcpy(&out[(size_t)y * W], &plane[(size_t)y * pw], W);
        return out;
    }
    const bool fancy = dw > 2;
    if (hf == 2 && vf == 1 && fancy) {  // h2v1_fancy_upsample
        std::vector<uint8_t> row(2 * dw);
        for (int y = 0; y < H; ++y) {
            const uint8_t *in = &plane[(size_t)y * pw];
            uint8_t *o = row.data();
            int v = in[0];
            *o++ = (uint8_t)v;
            *o++ = (uint8_t)((v * 3 + in[1] + 2) >> 2);
            for (int x = 1; x < dw - 1; ++x) {
                v = in[x] * 3;
                *o++ = (uint8_t)((v + in[x - 1] + 1) >> 2);
                *o++ = (uint8_t)((v + in[x + 1] + 2) >> 2);
            }
            v = in[dw - 1];
            *o++ = (uint8_t)((v * 3 + in[dw - 2] + 1) >> 2);
            *o++ = (uint8_t)v;
            std::memcpy(&out[(size_t)y * W], row.data(), W);
        }
        return out;
    }
    if (hf == 2 && vf == 2 && fancy) {  // h2v2_fancy_upsample
        std::vector<uint8_t> row(2 * dw);
        for (int oy = 0; oy < H; ++oy) {
            const int iy = oy >> 1;
            const int ny = (oy & 1) ? iy + 1 : iy - 1;  // next-nearest input row
            uint8_t *o = row.data();
            int thiscol = at(0, iy) * 3 + at(0, ny);
            int nextcol = at(1, iy) * 3 + at(1, ny);
            *o++ = (uint8_t)((thiscol * 4 + 8) >> 4);
            *o++ = (uint8_t)((thiscol * 3 + nextcol + 7) >> 4);
            int lastcol = thiscol;
            thiscol = nextcol;
            for (int x = 2; x < dw; ++x) {
                nextcol = at(x, iy) * 3 + at(x, ny);
                *o++ = (uint8_t)((thiscol * 3 + lastcol + 8) >> 4);
                *o++ = (uint8_t)((thiscol * 3 + nextcol + 7) >> 4);
                lastcol = thiscol;
                thiscol = nextcol;
            }
            *o++ = (uint8_t)((thiscol * 3 + lastcol + 8) >> 4);
            *o++ = (uint8_t)((thiscol * 4 + 7) >> 4);
            std::memcpy(&out[(size_t)oy * W], row.data(), W);
        }
        return out;
    }
    // other factors: pixel replication (IJG int_upsample / h2v2_upsample)
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) out[(size_t)y * W + x] = plane[(size_t)(y / vf) * pw + x / hf];
    return out;
}


// ---- jpeg-decoder 0.1.11 flavour (the reference's decoder, Cargo.lock:400-406).
// That crate's idct.rs / upsampler.rs are ports of stb_image's
// stbi__idct_block / resample_row_*; its colour conversion is BT.601 in f32.
inline int32_t f2f(float x) { return (int32_t)(x * 4096.0f + 0.5f); }
inline uint8_t clamp_u8(int32_t x) { return (uint8_t)(x < 0 ? 0 : x > 255 ? 255 : x); }

struct Idct1D {
    int32_t t0, t1, t2, t3, x0, x1, x2, x3;
    Idct1D(int32_t s0, int32_t s1, int32_t s2, int32_t s3, int32_t s4, int32_t s5, int32_t s6, int32_t s7) {
        int32_t p2 = s2, p3 = s6;
        int32_t p1 = (int32_t)((uint32_t)(p2 + p3) * (uint32_t)f2f(0.5411961f));
        t2 = p1 + p3 * f2f(-1.847759065f);
        t3 = p1 + p2 * f2f(0.765366865f);
        p2 = s0;
        p3 = s4;
        t0 = (p2 + p3) * 4096;
        t1 = (p2 - p3) * 4096;
        x0 = t0 + t3;
        x3 = t0 - t3;
        x1 = t1 + t2;
        x2 = t1 - t2;
        t0 = s7;
        t1 = s5;
        t2 = s3;
        t3 = s1;
        p3 = t0 + t2;
        int32_t p4 = t1 + t3;
        p1 = t0 + t3;
        p2 = t1 + t2;
        int32_t p5 = (p3 + p4) * f2f(1.175875602f);
        t0 = t0 * f2f(0.298631336f);
        t1 = t1 * f2f(2.053119869f);
        t2 = t2 * f2f(3.072711026f);
        t3 = t3 * f2f(1.501321110f);
        p1 = p5 + p1 * f2f(-0.899976223f);
        p2 = p5 + p2 * f2f(-2.562915447f);
        p3 = p3 * f2f(-1.961570560f);
        p4 = p4 * f2f(-0.390180644f);
        t3 += p1 + p4;
        t2 += p2 + p3;
        t1 += p2 + p4;
        t0 += p1 + p3;
    }
};

void idct_stb(const int16_t *in, const uint16_t *q, uint8_t *out, int stride) {
    int32_t v[64];
    int32_t d[64];
    for (int i = 0; i < 64; ++i) d[i] = (int32_t)in[i] * (int32_t)q[i];
    for (int i = 0; i < 8; ++i) {
        const int32_t *c = d + i;
        if (c[8] == 0 && c[16] == 0 && c[24] == 0 && c[32] == 0 && c[40] == 0 && c[48] == 0 && c[56] == 0) {
            for (int r = 0; r < 8; ++r) v[i + 8 * r] = c[0] * 4;
            continue;
        }
        Idct1D k(c[0], c[8], c[16], c[24], c[32], c[40], c[48], c[56]);
        k.x0 += 512; k.x1 += 512; k.x2 += 512; k.x3 += 512;
        v[i + 0] = (k.x0 + k.t3) >> 10;
        v[i + 56] = (k.x0 - k.t3) >> 10;
        v[i + 8] = (k.x1 + k.t2) >> 10;
        v[i + 48] = (k.x1 - k.t2) >> 10;
        v[i + 16] = (k.x2 + k.t1) >> 10;
        v[i + 40] = (k.x2 - k.t1) >> 10;
        v[i + 24] = (k.x3 + k.t0) >> 10;
        v[i + 32] = (k.x3 - k.t0) >> 10;
    }
    for (int r = 0; r < 8; ++r) {
        const int32_t *w = v + 8 * r;
        uint8_t *o = out + (size_t)r * stride;
        Idct1D k(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7]);
        const int32_t bias = 65536 + (128 << 17);
        k.x0 += bias; k.x1 += bias; k.x2 += bias; k.x3 += bias;
        o[0] = clamp_u8((k.x0 + k.t3) >> 17);
        o[7] = clamp_u8((k.x0 - k.t3) >> 17);
        o[1] = clamp_u8((k.x1 + k.t2) >> 17);
        o[6] = clamp_u8((k.x1 - k.t2) >> 17);
        o[2] = clamp_u8((k.x2 + k.t1) >> 17);
        o[5] = clamp_u8((k.x2 - k.t1) >> 17);
        o[3] = clamp_u8((k.x3 + k.t0) >> 17);
        o[4] = clamp_u8((k.x3 - k.t0) >> 17);
    }
}

// stb resample_row_h_2 / resample_row_v_2 / resample_row_hv_2; the "far" row is
// the previous input row for even output rows and the next one for odd rows,
// clamped to the component's real rows.
std::vector<uint8_t> upsample_stb(const std::vector<uint8_t> &plane, int pw, int dw, int dh, int hf, int vf, int W,
                                  int H) {
    std::vector<uint8_t> out((size_t)W * H);
    std::vector<uint8_t> row((size_t)dw * hf + 8);
    for (int oy = 0; oy < H; ++oy) {
        const int iy = oy / vf;
        const uint8_t *near = &plane[(size_t)iy * pw];
        if (hf == 1 && vf == 1) {
            std::memcpy(&out[(size_t)oy * W], near, W);
            continue;
        }
        uint8_t *o = row.data();
        if (hf == 2 && vf == 1) {
            if (dw == 1) {
                o[0] = o[1] = near[0];
            } else {
                o[0] = near[0];
                o[1] = (uint8_t)((near[0] * 3 + near[1] + 2) >> 2);
                for (int i = 1; i < dw - 1; ++i) {
                    int n = 3 * near[i] + 2;
                    o[2 * i] = (uint8_t)((n + near[i - 1]) >> 2);
                    o[2 * i + 1] = (uint8_t)((n + near[i + 1]) >> 2);
                }
                o[2 * (dw - 1)] = (uint8_t)((near[dw - 1] * 3 + near[dw - 2] + 2) >> 2);
                o[2 * (dw - 1) + 1] = near[dw - 1];
            }
        } else if (vf == 2 && (hf == 1 || hf == 2)) {
            int fy = (oy & 1) ? iy + 1 : iy - 1;
            fy = fy < 0 ? 0 : (fy > dh - 1 ? dh - 1 : fy);
            const uint8_t *far = &plane[(size_t)fy * pw];
            if (hf == 1) {
                for (int i = 0; i < dw; ++i) o[i] = (uint8_t)((3 * near[i] + far[i] + 2) >> 2);
            } else if (dw == 1) {
                o[0] = o[1] = (uint8_t)((3 * near[0] + far[0] + 2) >> 2);
            } else {
                int t1 = 3 * near[0] + far[0];
                o[0] = (uint8_t)((t1 + 2) >> 2);
                for (int i = 1; i < dw; ++i) {
                    int t0 = t1;
                    t1 = 3 * near[i] + far[i];
                    o[2 * i - 1] = (uint8_t)((3 * t0 + t1 + 8) >> 4);
                    o[2 * i] = (uint8_t)((3 * t1 + t0 + 8) >> 4);
                }
                o[2 * dw - 1] = (uint8_t)((t1 + 2) >> 2);
            }
        } else {
            for (int x = 0; x < W; ++x) o[x] = near[x / hf];
        }
        std::memcpy(&out[(size_t)oy * W], o, W);
    }
    return out;
}

}  // namespace

bool decode_jpeg(const uint8_t *data, size_t size, Image &img, std::string &err, JpegFlavor flavor) {
    const bool stb = flavor == JpegFlavor::Reference;
    Decoder d;
    d.p = data;
    d.end = data + size;
    if (size < 4 || data[0] != 0xFF || data[1] != 0xD8) { err = "not a JPEG file"; return false; }
    d.p += 2;
    bool sof = false;
    while (d.p < d.end) {
        if (*d.p != 0xFF) { ++d.p; continue; }
        while (d.p < d.end && *d.p == 0xFF) ++d.p;
        if (d.p >= d.end) break;
        int m = *d.p++;
        if (m == 0xD9) break;                       // EOI
        if (m >= 0xD0 && m <= 0xD7) continue;       // stray RST
        int len = d.u16() - 2;
        if (len < 0 || d.p + len > d.end) { err = "truncated JPEG segment"; return false; }
        const uint8_t *next = d.p + len;
        bool ok = true;
        switch (m) {
        case 0xDB: ok = d.read_dqt(len); break;
        case 0xC4: ok = d.read_dht(len); break;
        case 0xC0: case 0xC1: ok = d.read_sof(len, false); sof = true; break;
        case 0xC2: ok = d.read_sof(len, true); sof = true; break;
        case 0xDD: d.restart = d.u16(); break;
        case 0xDA:
            if (!sof) { err = "SOS before SOF"; return false; }
            d.p -= 2;  // read_sos reads the length itself
            ok = d.read_sos();
            next = d.p;
            break;
        case 0xEE:  // Adobe APP14
            if (len >= 12 && std::memcmp(d.p, "Adobe", 5) == 0) { d.adobe = true; d.adobe_transform = d.p[11]; }
            break;
        default:
            if ((m >= 0xC3 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC)) {
                err = "unsupported JPEG process (arithmetic/lossless/hierarchical)";
                return false;
            }
            break;
        }
        if (!ok) { err = d.err; return false; }
        d.p = next;
    }
    if (!sof) { err = "no frame header"; return false; }
    // dequantise + IDCT into padded component planes
    std::vector<std::vector<uint8_t>> planes(d.comps.size());
    for (size_t ci = 0; ci < d.comps.size(); ++ci) {
        Component &c = d.comps[ci];
        const int pw = c.bw * 8;
        planes[ci].assign((size_t)pw * c.bh * 8, 0);
        for (int by = 0; by < c.bh; ++by)
            for (int bx = 0; bx < c.bw; ++bx)
                (stb ? idct_stb : idct_islow)(c.coef.data() + ((size_t)by * c.bw + bx) * 64, d.qt[c.tq],
                                              planes[ci].data() + (size_t)by * 8 * pw + bx * 8, pw);
    }
    const int W = d.width, H = d.height;
    std::vector<std::vector<uint8_t>> full(d.comps.size());
    for (size_t ci = 0; ci < d.comps.size(); ++ci) {
        Component &c = d.comps[ci];
        full[ci] = (stb ? upsample_stb : upsample)(planes[ci], c.bw * 8, c.dw, c.dh, d.max_h / c.h, d.max_v / c.v, W, H);
    }
    img.width = (uint32_t)W;
    img.height = (uint32_t)H;
    img.rgba.assign((size_t)W * H * 4, 255);
    if (d.comps.size() == 1) {
        for (size_t i = 0; i < (size_t)W * H; ++i) img.rgba[4 * i] = img.rgba[4 * i + 1] = img.rgba[4 * i + 2] = full[0][i];
        return true;
    }
    const bool ycc = !(d.adobe && d.adobe_transform == 0);  // JFIF / Adobe transform 1: YCbCr
    if (!ycc) {
        for (size_t i = 0; i < (size_t)W * H; ++i)
            for (int k = 0; k < 3; ++k) img.rgba[4 * i + k] = full[k][i];
        return true;
    }
    if (stb) {
        // jpeg-decoder 0.1.11 ycbcr_to_rgb: f32 BT.601, (v + 0.5) as i32, clamp
        for (size_t i = 0; i < (size_t)W * H; ++i) {
            const float y = (float)full[0][i], cb = (float)full[1][i] - 128.0f, cr = (float)full[2][i] - 128.0f;
            const float r = y + 1.40200f * cr;
            const float g = y - 0.34414f * cb - 0.71414f * cr;
            const float b = y + 1.77200f * cb;
            img.rgba[4 * i + 0] = clamp_u8((int32_t)(r + 0.5f));
            img.rgba[4 * i + 1] = clamp_u8((int32_t)(g + 0.5f));
            img.rgba[4 * i + 2] = clamp_u8((int32_t)(b + 0.5f));
        }
        return true;
    }
    // IJG jdcolor.c ycc_rgb_convert (SCALEBITS 16)
    static int cr_r[256], cb_b[256], cr_g[256], cb_g[256];
    static bool init = false;
    if (!init) {
        const int ONE_HALF = 1 << 15;
        for (int i = 0; i < 256; ++i) {
            int x = i - 128;
            cr_r[i] = (int)((91881 * x + ONE_HALF) >> 16);
            cb_b[i] = (int)((116130 * x + ONE_HALF) >> 16);
            cr_g[i] = -46802 * x;
            cb_g[i] = -22554 * x + ONE_HALF;
        }
        init = true;
    }
    auto clamp8 = [](int v) -> uint8_t { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); };
    for (size_t i = 0; i < (size_t)W * H; ++i) {
        int y = full[0][i], cb = full[1][i], cr = full[2][i];
        img.rgba[4 * i + 0] = clamp8(y + cr_r[cr]);
        img.rgba[4 * i + 1] = clamp8(y + ((cb_g[cb] + cr_g[cr]) >> 16));
        img.rgba[4 * i + 2] = clamp8(y + cb_b[cb]);
    }
    return true;
}

}  // namespace rgh
