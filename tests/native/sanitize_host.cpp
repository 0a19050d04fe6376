// sanitize_host.cpp — host-code sanitizer harness (built with
// -fsanitize=address,undefined by tests/test_sanitizers.py, CPU only).
//
// Drives every parser of the native host layer and the CPU restatement over
// the reference's own fixtures and over corrupted copies of them:
//   * YAML scene loader (raingun_amd/host/yaml.cpp, scene_loader.cpp):
//     examples/test{1,2,3}.yml, then truncations and byte flips;
//   * JPEG decoder (jpeg_decode.cpp, both rounding flavours) and PNG codec
//     (png_codec.cpp): the reference's textures and golden PNGs, then
//     truncations and byte flips; PNG encode -> decode round trips;
//   * the CPU restatement (oracle/raingun_oracle.c): a small render of every
//     example scene through rgo_render (2 threads).
// Corrupted inputs may be rejected (any status); what must not happen is an
// out-of-bounds access, use-after-free, leak or undefined behaviour -- the
// sanitizers abort the process on the first one.
//   usage: sanitize_host <golden dir> [mutations per file]
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "../../include/raingun.h"
#include "../../include/raingun_host.h"

extern "C" int32_t rgo_render(const rg_scene_desc *s, uint32_t w, uint32_t h, const rg_tiling *tiling, uint8_t *rgba,
                              float *rgb, rg_ray_counts *counts, int32_t nthreads, int64_t *error_pixel);

namespace {

std::vector<uint8_t> read_file(const std::string &path) {
    std::ifstream f(path, std::ios::binary);
    return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

uint64_t splitmix(uint64_t &s) {  // deterministic mutations
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Truncations at fractions of the length, then `n` copies with 1-8 random byte changes.
template <class F>
void mutate(const std::vector<uint8_t> &orig, int n, uint64_t seed, F &&use) {
    for (int k = 0; k <= 16; ++k) {
        std::vector<uint8_t> t(orig.begin(), orig.begin() + (long)(orig.size() * k / 16));
        use(t);
    }
    uint64_t s = seed;
    for (int i = 0; i < n; ++i) {
        std::vector<uint8_t> m = orig;
        const int flips = 1 + (int)(splitmix(s) % 8);
        for (int j = 0; j < flips && !m.empty(); ++j) m[splitmix(s) % m.size()] = (uint8_t)splitmix(s);
        use(m);
    }
}

int decode(const std::vector<uint8_t> &b, int flavor) {
    uint32_t w = 0, h = 0;
    uint8_t *px = nullptr;
    const int32_t st = rgh_image_decode(b.data(), b.size(), flavor, &w, &h, &px);
    if (st == 0 && px) {
        volatile uint32_t sum = 0;  // touch every byte of the output
        for (size_t i = 0; i < (size_t)w * h * 4; ++i) sum += px[i];
        (void)sum;
    }
    rgh_free(px);
    return st;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <golden dir> [mutations]\n", argv[0]);
        return 2;
    }
    const std::string g = argv[1];
    const int n = argc > 2 ? std::atoi(argv[2]) : 200;
    int ok_files = 0, rejected = 0, accepted = 0;

    // images: the reference's textures and golden renders
    const char *images[] = {"textures/clay-ground-seamless.jpg", "textures/land_ocean_ice_cloud_2048.jpg",
                            "textures/tile1/color.jpg", "examples/test1.png", "examples/test2.png", "examples/test3.png"};
    for (const char *rel : images) {
        const std::vector<uint8_t> b = read_file(g + "/" + rel);
        if (b.empty()) {
            std::fprintf(stderr, "missing fixture %s\n", rel);
            return 3;
        }
        for (int flavor : {RGH_JPEG_REFERENCE, RGH_JPEG_LIBJPEG}) {
            if (decode(b, flavor) != 0) {
                std::fprintf(stderr, "fixture %s did not decode\n", rel);
                return 4;
            }
        }
        ++ok_files;
        // big textures: fewer mutations (each decode of a 2048x1024 progressive JPEG takes a while under ASan)
        const int m = b.size() > (1u << 20) ? n / 10 : n;
        mutate(b, m, 0x5EED ^ b.size(), [&](const std::vector<uint8_t> &x) {
            (decode(x, RGH_JPEG_REFERENCE) == 0 ? accepted : rejected)++;
        });
    }

    // PNG round trips (odd sizes, the encoder's filters and the decoder's)
    for (uint32_t w : {1u, 3u, 17u, 64u}) {
        for (uint32_t h : {1u, 2u, 9u}) {
            std::vector<uint8_t> px((size_t)w * h * 4);
            uint64_t s = w * 131 + h;
            for (auto &v : px) v = (uint8_t)splitmix(s);
            uint8_t *png = nullptr;
            size_t size = 0;
            if (rgh_png_encode(px.data(), w, h, &png, &size) != 0) return 5;
            uint32_t w2 = 0, h2 = 0;
            uint8_t *back = nullptr;
            if (rgh_image_decode(png, size, RGH_JPEG_REFERENCE, &w2, &h2, &back) != 0 || w2 != w || h2 != h ||
                std::memcmp(back, px.data(), px.size()) != 0)
                return 6;
            rgh_free(back);
            rgh_free(png);
        }
    }

    // scenes: load, render a small frame with the CPU restatement, then corrupted YAML
    for (const char *name : {"test1.yml", "test2.yml", "test3.yml"}) {
        const std::vector<uint8_t> y = read_file(g + "/examples/" + name);
        rgh_scene *sc = nullptr;
        if (rgh_scene_load_string((const char *)y.data(), y.size(), g.c_str(), &sc) != 0) {
            std::fprintf(stderr, "scene %s did not load: %s\n", name, rgh_last_error());
            return 7;
        }
        const uint32_t W = 64, H = 48;
        std::vector<uint8_t> rgba((size_t)W * H * 4);
        std::vector<float> rgb((size_t)W * H * 3);
        rg_ray_counts counts;
        int64_t err = -1;
        rg_tiling whole = {H, 1, 0};
        if (rgo_render(rgh_scene_desc(sc), W, H, &whole, rgba.data(), rgb.data(), &counts, 2, &err) != 0) return 8;
        rg_tiling shard = {5, 3, 1};  // a sharded tiling with a partial last tile
        if (rgo_render(rgh_scene_desc(sc), W, H, &shard, rgba.data(), nullptr, &counts, 2, &err) != 0) return 9;
        rgh_scene_free(sc);
        ++ok_files;
        mutate(y, n, 0xABCD ^ y.size(), [&](const std::vector<uint8_t> &x) {
            rgh_scene *m = nullptr;
            // no texture root: corrupted paths must fail cleanly, not open arbitrary files
            const int32_t st = rgh_scene_load_string((const char *)x.data(), x.size(), "/nonexistent", &m);
            if (st == 0) {
                ++accepted;
                rgh_scene_free(m);
            } else {
                ++rejected;
                (void)rgh_last_error();
            }
        });
    }
    std::printf("{\"fixtures\": %d, \"mutants_accepted\": %d, \"mutants_rejected\": %d}\n", ok_files, accepted,
                rejected);
    return 0;
}
