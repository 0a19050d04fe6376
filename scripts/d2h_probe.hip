// d2h_probe.hip — device-to-host bandwidth of the ways a rendered frame can
// reach host memory (the host-visible rg_render_image path):
//   sdma1     one hipMemcpyAsync of the whole frame
//   sdmaN     the frame in N chunks on N streams (several copy engines)
//   kernel    a blit kernel storing 16 B per lane straight into page-locked host
//             memory (hipHostMalloc'd or hipHostRegister'd), PCIe writes issued by the CUs
// Build: hipcc -O3 --offload-arch=gfx950 -o scripts/bin/d2h_probe scripts/d2h_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                      \
        }                                                                      \
    } while (0)

typedef unsigned v4u __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void blit(const uint4 *src, uint4 *dst, size_t n16) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * 256;
    const v4u *s = reinterpret_cast<const v4u *>(src);
    v4u *d = reinterpret_cast<v4u *>(dst);
    for (; i < n16; i += stride) __builtin_nontemporal_store(s[i], &d[i]);
}

__global__ __launch_bounds__(256) void blit_plain(const uint4 *src, uint4 *dst, size_t n16) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * 256;
    for (; i < n16; i += stride) dst[i] = src[i];
}

// Framebuffer-shaped stores straight into host memory: one wave per TWxTH pixel
// tile (TW*TH = 64, lane = pixel, 4 B per lane), image width W pixels: each
// wave store is TH row segments of TW*4 bytes (the render kernel's 8x8 tiles
// give 8 x 32 B).
// SCATTER: tiles in a scrambled order (t * 7919 mod ntiles), as a render's
// tiles finish -- neighbouring tiles' stores no longer arrive together.
template <int TW, bool SCATTER = false>
__global__ __launch_bounds__(256) void tile_store(const uint32_t *src, uint32_t *dst, uint32_t W, uint32_t H) {
    constexpr int TH = 64 / TW;
    const uint32_t tiles_x = W / TW, ntiles = tiles_x * (H / TH);
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t t0 = blockIdx.x * 4 + (threadIdx.x >> 6); t0 < ntiles; t0 += gridDim.x * 4) {
        const uint32_t t = SCATTER ? (uint32_t)(((unsigned long long)t0 * 7919u) % ntiles) : t0;
        const uint32_t x = (t % tiles_x) * TW + lane % TW, y = (t / tiles_x) * TH + lane / TW;
        dst[(size_t)y * W + x] = src[(size_t)y * W + x];
    }
}

int main(int argc, char **argv) {
    const size_t bytes = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : (size_t)3840 * 2160 * 4;
    const int reps = 20;
    void *d = nullptr;
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(d, 0x5a, bytes));
    void *hm = nullptr;
    CK(hipHostMalloc(&hm, bytes, hipHostMallocDefault));
    void *hr = std::aligned_alloc(4096, (bytes + 4095) / 4096 * 4096);
    std::memset(hr, 0, bytes);
    CK(hipHostRegister(hr, bytes, hipHostRegisterDefault));
    void *hr_dev = nullptr;
    CK(hipHostGetDevicePointer(&hr_dev, hr, 0));
    hipStream_t s[8];
    for (auto &x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char *name, auto &&body) {
        body();  // warm
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, s[0]));
        for (int r = 0; r < reps; ++r) body();
        for (int k = 1; k < 8; ++k) {  // join every stream into s[0]
            hipEvent_t j;
            CK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
            CK(hipEventRecord(j, s[k]));
            CK(hipStreamWaitEvent(s[0], j, 0));
            CK(hipEventDestroy(j));
        }
        CK(hipEventRecord(e1, s[0]));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("{\"probe\": \"%s\", \"bytes\": %zu, \"ms\": %.4f, \"GBps\": %.2f}\n", name, bytes, ms / reps,
                    bytes / (ms / reps * 1e-3) / 1e9);
        std::fflush(stdout);
    };
    for (void *h : {hm, hr}) {
        const char *tag = h == hm ? "hostmalloc" : "registered";
        void *hdev = h == hm ? hm : hr_dev;
        char nm[64];
        std::snprintf(nm, sizeof nm, "sdma1_%s", tag);
        run(nm, [&] { CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s[0])); });
        for (int n : {2, 4, 8}) {
            std::snprintf(nm, sizeof nm, "sdma%d_%s", n, tag);
            run(nm, [&] {
                const size_t c = (bytes / n + 4095) / 4096 * 4096;
                for (int k = 0; k < n; ++k) {
                    const size_t off = (size_t)k * c;
                    if (off >= bytes) break;
                    const size_t len = off + c > bytes ? bytes - off : c;
                    CK(hipMemcpyAsync((char *)h + off, (char *)d + off, len, hipMemcpyDeviceToHost, s[k]));
                }
            });
        }
        for (int blocks : {64, 256, 1024}) {
            std::snprintf(nm, sizeof nm, "kernel_nt%d_%s", blocks, tag);
            run(nm, [&] {
                hipLaunchKernelGGL(blit, dim3(blocks), dim3(256), 0, s[0], (const uint4 *)d, (uint4 *)hdev, bytes / 16);
            });
            std::snprintf(nm, sizeof nm, "kernel%d_%s", blocks, tag);
            run(nm, [&] {
                hipLaunchKernelGGL(blit_plain, dim3(blocks), dim3(256), 0, s[0], (const uint4 *)d, (uint4 *)hdev,
                                   bytes / 16);
            });
        }
        const uint32_t W = 3840, H = (uint32_t)(bytes / 4 / W) / 64 * 64;
        std::snprintf(nm, sizeof nm, "tile8x8_%s", tag);
        run(nm, [&] { hipLaunchKernelGGL(tile_store<8>, dim3(2048), dim3(256), 0, s[0], (const uint32_t *)d, (uint32_t *)hdev, W, H); });
        std::snprintf(nm, sizeof nm, "tile16x4_%s", tag);
        run(nm, [&] { hipLaunchKernelGGL(tile_store<16>, dim3(2048), dim3(256), 0, s[0], (const uint32_t *)d, (uint32_t *)hdev, W, H); });
        std::snprintf(nm, sizeof nm, "tile32x2_%s", tag);
        run(nm, [&] { hipLaunchKernelGGL(tile_store<32>, dim3(2048), dim3(256), 0, s[0], (const uint32_t *)d, (uint32_t *)hdev, W, H); });
        std::snprintf(nm, sizeof nm, "scatter8x8_%s", tag);
        run(nm, [&] { hipLaunchKernelGGL((tile_store<8, true>), dim3(2048), dim3(256), 0, s[0], (const uint32_t *)d, (uint32_t *)hdev, W, H); });
        std::snprintf(nm, sizeof nm, "scatter16x4_%s", tag);
        run(nm, [&] { hipLaunchKernelGGL((tile_store<16, true>), dim3(2048), dim3(256), 0, s[0], (const uint32_t *)d, (uint32_t *)hdev, W, H); });
        std::snprintf(nm, sizeof nm, "scatter32x2_%s", tag);
        run(nm, [&] { hipLaunchKernelGGL((tile_store<32, true>), dim3(2048), dim3(256), 0, s[0], (const uint32_t *)d, (uint32_t *)hdev, W, H); });
        std::snprintf(nm, sizeof nm, "scatter64x1_%s", tag);
        run(nm, [&] { hipLaunchKernelGGL((tile_store<64, true>), dim3(2048), dim3(256), 0, s[0], (const uint32_t *)d, (uint32_t *)hdev, W, H); });
        std::snprintf(nm, sizeof nm, "tile64x1_%s", tag);
        run(nm, [&] { hipLaunchKernelGGL(tile_store<64>, dim3(2048), dim3(256), 0, s[0], (const uint32_t *)d, (uint32_t *)hdev, W, H); });
    }
    // correctness of the last blit
    const unsigned char *p = (const unsigned char *)hr;
    for (size_t i = 0; i < bytes; i += 4099)
        if (p[i] != 0x5a) {
            std::printf("{\"error\": \"blit mismatch at %zu\"}\n", i);
            return 1;
        }
    CK(hipHostUnregister(hr));
    std::free(hr);
    CK(hipHostFree(hm));
    CK(hipFree(d));
    return 0;
}
