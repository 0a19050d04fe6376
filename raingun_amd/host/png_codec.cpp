// png_codec.cpp — PNG read (textures, golden images) and write (rendered
// frames) for the C++ host, on the system zlib.
//
// Reading covers what image 0.12's PNG path hands the reference
// (material.rs:34-47 via image::open): bit depths 1-16, greyscale, grey+alpha,
// RGB, RGBA and palette (+tRNS), Adam7 interlacing; 16-bit samples keep their
// high byte.  Writing is the frame output of render.rs:58 (image.save): 8-bit
// RGBA, one filter byte per row, zlib level 6.
#include <zlib.h>

#include <cstring>

#include "image_codec.h"

namespace rgh {
namespace {

uint32_t be32(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
void put32(std::vector<uint8_t> &o, uint32_t v) {
    o.push_back((uint8_t)(v >> 24));
    o.push_back((uint8_t)(v >> 16));
    o.push_back((uint8_t)(v >> 8));
    o.push_back((uint8_t)v);
}

bool inflate_all(const std::vector<uint8_t> &in, std::vector<uint8_t> &out, size_t expect) {
    out.resize(expect);
    z_stream zs;
    std::memset(&zs, 0, sizeof zs);
    if (inflateInit(&zs) != Z_OK) return false;
    zs.next_in = const_cast<Bytef *>(in.data());
    zs.avail_in = (uInt)in.size();
    zs.next_out = out.data();
    zs.avail_out = (uInt)out.size();
    int r = inflate(&zs, Z_FINISH);
    size_t got = zs.total_out;
    inflateEnd(&zs);
    return (r == Z_STREAM_END || r == Z_BUF_ERROR || r == Z_OK) && got == expect;
}

int paeth(int a, int b, int c) {
    int p = a + b - c, pa = p > a ? p - a : a - p, pb = p > b ? p - b : b - p, pc = p > c ? p - c : c - p;
    if (pa <= pb && pa <= pc) return a;
    return pb <= pc ? b : c;
}

// Undo the filters of one (sub)image of w x h pixels stored at `src`; returns bytes consumed.
bool unfilter(const uint8_t *src, size_t avail, uint32_t w, uint32_t h, int bpp_bits, std::vector<uint8_t> &rows,
              size_t *used) {
    const size_t stride = ((size_t)w * bpp_bits + 7) / 8;
    const int bpp = (bpp_bits + 7) / 8;
    if ((stride + 1) * h > avail) return false;
    rows.assign(stride * h, 0);
    std::vector<uint8_t> zero(stride, 0);
    for (uint32_t y = 0; y < h; ++y) {
        const uint8_t *in = src + (stride + 1) * y;
        int ft = in[0];
        ++in;
        uint8_t *o = &rows[stride * y];
        const uint8_t *up = y ? &rows[stride * (y - 1)] : zero.data();
        for (size_t x = 0; x < stride; ++x) {
            int a = x >= (size_t)bpp ? o[x - bpp] : 0, b = up[x], c = x >= (size_t)bpp ? up[x - bpp] : 0, v;
            switch (ft) {
            case 0: v = in[x]; break;
            case 1: v = in[x] + a; break;
            case 2: v = in[x] + b; break;
            case 3: v = in[x] + ((a + b) >> 1); break;
            case 4: v = in[x] + paeth(a, b, c); break;
            default: return false;
            }
            o[x] = (uint8_t)v;
        }
    }
    *used = (stride + 1) * h;
    return true;
}

}  // namespace

bool decode_png(const uint8_t *data, size_t size, Image &img, std::string &err) {
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
    if (size < 8 || std::memcmp(data, sig, 8) != 0) { err = "not a PNG file"; return false; }
    size_t p = 8;
    uint32_t W = 0, H = 0;
    int depth = 0, ctype = -1, interlace = 0;
    std::vector<uint8_t> idat, plte, trns;
    while (p + 12 <= size) {
        uint32_t len = be32(data + p);
        const uint8_t *type = data + p + 4;
        if (p + 12 + (size_t)len > size) { err = "truncated PNG chunk"; return false; }
        const uint8_t *body = data + p + 8;
        if (!std::memcmp(type, "IHDR", 4) && len >= 13) {
            W = be32(body);
            H = be32(body + 4);
            depth = body[8];
            ctype = body[9];
            interlace = body[12];
        } else if (!std::memcmp(type, "PLTE", 4)) {
            plte.assign(body, body + len);
        } else if (!std::memcmp(type, "tRNS", 4)) {
            trns.assign(body, body + len);
        } else if (!std::memcmp(type, "IDAT", 4)) {
            idat.insert(idat.end(), body, body + len);
        } else if (!std::memcmp(type, "IEND", 4)) {
            break;
        }
        p += 12 + (size_t)len;
    }
    static const int chans_of[7] = {1, 0, 3, 1, 2, 0, 4};
    if (W == 0 || H == 0 || ctype < 0 || ctype > 6 || chans_of[ctype] == 0 ||
        !(depth == 1 || depth == 2 || depth == 4 || depth == 8 || depth == 16)) {
        err = "unsupported PNG header";
        return false;
    }
    if (ctype == 3 && plte.empty()) { err = "PNG palette missing"; return false; }
    const int chans = chans_of[ctype], bits = chans * depth;
    // raw size over the 7 Adam7 passes (or the one image)
    static const int ax0[7] = {0, 4, 0, 2, 0, 1, 0}, ay0[7] = {0, 0, 4, 0, 2, 0, 1}, adx[7] = {8, 8, 4, 4, 2, 2, 1},
                     ady[7] = {8, 8, 8, 4, 4, 2, 2};
    auto pass_dims = [&](int k, uint32_t &pw, uint32_t &ph) {
        pw = W > (uint32_t)ax0[k] ? (W - ax0[k] + adx[k] - 1) / adx[k] : 0;
        ph = H > (uint32_t)ay0[k] ? (H - ay0[k] + ady[k] - 1) / ady[k] : 0;
    };
    size_t expect = 0;
    const int npass = interlace ? 7 : 1;
    for (int k = 0; k < npass; ++k) {
        uint32_t pw = W, ph = H;
        if (interlace) pass_dims(k, pw, ph);
        if (pw && ph) expect += (((size_t)pw * bits + 7) / 8 + 1) * ph;
    }
    std::vector<uint8_t> raw;
    if (!inflate_all(idat, raw, expect)) { err = "corrupt PNG image data"; return false; }
    img.width = W;
    img.height = H;
    img.rgba.assign((size_t)W * H * 4, 255);
    size_t off = 0;
    std::vector<uint8_t> rows;
    for (int k = 0; k < npass; ++k) {
        uint32_t pw = W, ph = H;
        if (interlace) pass_dims(k, pw, ph);
        if (!pw || !ph) continue;
        size_t used = 0;
        if (!unfilter(raw.data() + off, raw.size() - off, pw, ph, bits, rows, &used)) {
            err = "corrupt PNG filter data";
            return false;
        }
        off += used;
        const size_t stride = ((size_t)pw * bits + 7) / 8;
        for (uint32_t y = 0; y < ph; ++y) {
            const uint8_t *r = &rows[stride * y];
            for (uint32_t x = 0; x < pw; ++x) {
                uint32_t v[4] = {0, 0, 0, 255};
                uint32_t raw16[4] = {0, 0, 0, 0};
                for (int c = 0; c < chans; ++c) {
                    uint32_t s;
                    if (depth == 8) s = r[(size_t)x * chans + c];
                    else if (depth == 16) {
                        const uint8_t *q = r + ((size_t)x * chans + c) * 2;
                        raw16[c] = (uint32_t)q[0] << 8 | q[1];
                        s = q[0];
                    } else {
                        size_t bit = ((size_t)x * chans + c) * depth;
                        s = (r[bit / 8] >> (8 - depth - bit % 8)) & ((1u << depth) - 1);
                    }
                    v[c] = s;
                }
                uint8_t px[4];
                const uint32_t maxv = (1u << (depth > 8 ? 8 : depth)) - 1;
                auto scale = [&](uint32_t s) -> uint8_t { return (uint8_t)(depth >= 8 ? s : s * 255 / maxv); };
                auto sample = [&](int c) -> uint32_t { return depth == 16 ? raw16[c] : v[c]; };
                switch (ctype) {
                case 0: {
                    px[0] = px[1] = px[2] = scale(v[0]);
                    px[3] = (trns.size() >= 2 && sample(0) == ((uint32_t)trns[0] << 8 | trns[1])) ? 0 : 255;
                    break;
                }
                case 2: {
                    px[0] = scale(v[0]); px[1] = scale(v[1]); px[2] = scale(v[2]);
                    bool t = trns.size() >= 6 && sample(0) == ((uint32_t)trns[0] << 8 | trns[1]) &&
                             sample(1) == ((uint32_t)trns[2] << 8 | trns[3]) && sample(2) == ((uint32_t)trns[4] << 8 | trns[5]);
                    px[3] = t ? 0 : 255;
                    break;
                }
                case 3: {
                    uint32_t i = v[0];
                    if (3 * i + 2 >= plte.size()) { err = "PNG palette index out of range"; return false; }
                    px[0] = plte[3 * i]; px[1] = plte[3 * i + 1]; px[2] = plte[3 * i + 2];
                    px[3] = i < trns.size() ? trns[i] : 255;
                    break;
                }
                case 4: px[0] = px[1] = px[2] = scale(v[0]); px[3] = scale(v[1]); break;
                default: px[0] = scale(v[0]); px[1] = scale(v[1]); px[2] = scale(v[2]); px[3] = scale(v[3]); break;
                }
                uint32_t X = interlace ? ax0[k] + x * adx[k] : x, Y = interlace ? ay0[k] + y * ady[k] : y;
                std::memcpy(&img.rgba[((size_t)Y * W + X) * 4], px, 4);
            }
        }
    }
    return true;
}

std::vector<uint8_t> encode_png(const uint8_t *rgba, uint32_t width, uint32_t height) {
    std::vector<uint8_t> out = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
    auto chunk = [&](const char *tag, const uint8_t *body, size_t len) {
        put32(out, (uint32_t)len);
        size_t st = out.size();
        out.insert(out.end(), tag, tag + 4);
        out.insert(out.end(), body, body + len);
        put32(out, (uint32_t)crc32(0, out.data() + st, (uInt)(len + 4)));
    };
    uint8_t ihdr[13];
    const uint32_t wv = width, hv = height;
    for (int i = 0; i < 4; ++i) { ihdr[i] = (uint8_t)(wv >> (24 - 8 * i)); ihdr[4 + i] = (uint8_t)(hv >> (24 - 8 * i)); }
    ihdr[8] = 8; ihdr[9] = 6; ihdr[10] = 0; ihdr[11] = 0; ihdr[12] = 0;
    chunk("IHDR", ihdr, 13);
    const size_t stride = (size_t)width * 4;
    std::vector<uint8_t> raw((stride + 1) * height);
    for (uint32_t y = 0; y < height; ++y) {
        raw[(stride + 1) * y] = 0;
        std::memcpy(&raw[(stride + 1) * y + 1], rgba + stride * y, stride);
    }
    uLongf zlen = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(zlen);
    compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6);
    chunk("IDAT", z.data(), zlen);
    chunk("IEND", nullptr, 0);
    return out;
}

bool decode_image(const uint8_t *data, size_t size, Image &out, std::string &err, JpegFlavor flavor) {
    if (size >= 8 && data[0] == 0x89 && data[1] == 'P') return decode_png(data, size, out, err);
    if (size >= 3 && data[0] == 0xFF && data[1] == 0xD8) return decode_jpeg(data, size, out, err, flavor);
    err = "The image format could not be determined (only JPEG and PNG textures are supported)";
    return false;
}

}  // namespace rgh
