// Does the runtime throttle how many waves of ONE dispatch with scratch
// (private memory) run at once?  (round-4 diagnostic)
//
// spin<S>: every one-wave block waits ~T us on the wall clock (s_sleep loop,
// nothing else busy); S > 0 also touches an S-dword private array with a
// dynamic index, so the kernel has S*4 bytes of scratch per lane.  Launch
// n = 1024 .. 8192 blocks; without throttling every n that fits the GPU's wave
// slots takes ~T, with a per-dispatch scratch-wave limit the time grows with n.
//   hipcc --offload-arch=gfx950 -O2 scratch_probe.hip -o scratch_probe && ./scratch_probe
#include <hip/hip_runtime.h>

#include <cstdio>

template <int S>
__global__ __launch_bounds__(64) void spin(unsigned *out, unsigned idx, unsigned long long ticks) {
    const unsigned long long t0 = wall_clock64();
    unsigned acc = threadIdx.x;
    if constexpr (S > 0) {
        volatile unsigned arr[S];
        for (int i = 0; i < S; ++i) arr[i] = i + threadIdx.x;
        while (wall_clock64() - t0 < ticks) {
            acc += arr[(acc + idx) % S];
            __builtin_amdgcn_s_sleep(8);
        }
    } else {
        while (wall_clock64() - t0 < ticks) {
            acc += idx;
            __builtin_amdgcn_s_sleep(8);
        }
    }
    if (acc == 0xFFFFFFFFu) out[blockIdx.x] = acc;
}

template <int S>
static float run(unsigned *d, unsigned n, unsigned long long ticks) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(spin<S>, dim3(n), dim3(64), 0, 0, d, 3u, ticks);  // warm
    hipEventRecord(a, 0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(spin<S>, dim3(n), dim3(64), 0, 0, d, 3u, ticks);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / 5;
}

int main() {
    unsigned *d = nullptr;
    if (hipMalloc(&d, 1 << 20) != hipSuccess) return 1;
    const unsigned long long ticks = 2000;  // 20 us at the 100 MHz wall clock
    for (unsigned n : {1024u, 2048u, 4096u, 8192u, 16384u}) {
        const float t0 = run<0>(d, n, ticks), t1 = run<16>(d, n, ticks), t2 = run<184>(d, n, ticks);
        printf("{\"blocks\": %u, \"no_scratch_ms\": %.4f, \"scratch_64B_ms\": %.4f, \"scratch_736B_ms\": %.4f}\n", n, t0,
               t1, t2);
    }
    hipFree(d);
    return 0;
}
