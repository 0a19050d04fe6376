// image_codec.h — texture decoding and PNG output for the C++ host
// (jpeg_decode.cpp, png_codec.cpp).
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace rgh {

struct Image {
    uint32_t width = 0, height = 0;
    std::vector<uint8_t> rgba;  // row-major RGBA8, alpha 255
};

// Which decoder's rounding to reproduce: the reference's (jpeg-decoder 0.1.11:
// stb_image IDCT + upsampling, f32 YCbCr) or IJG libjpeg's (ISLOW + fancy).
enum class JpegFlavor { Reference = 0, Libjpeg = 1 };

// Baseline or progressive Huffman JPEG, 8-bit, greyscale or 3-component.
bool decode_jpeg(const uint8_t *data, size_t size, Image &out, std::string &err,
                 JpegFlavor flavor = JpegFlavor::Reference);

// 8-bit PNG (greyscale, grey+alpha, RGB, RGBA, palette; non-interlaced), zlib via inflate below.
bool decode_png(const uint8_t *data, size_t size, Image &out, std::string &err);

// Encode RGBA8 as PNG (filter 0 per row, stored/fixed-Huffman deflate).
std::vector<uint8_t> encode_png(const uint8_t *rgba, uint32_t width, uint32_t height);

// Decode any of the above by signature.
bool decode_image(const uint8_t *data, size_t size, Image &out, std::string &err,
                  JpegFlavor flavor = JpegFlavor::Reference);

}  // namespace rgh
