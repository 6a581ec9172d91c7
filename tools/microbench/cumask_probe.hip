// CU-mask probe (gfx950): the blend's one-wave workgroups keep every freed wave slot, so a
// second queue's 256-thread workgroups (the geometry chain) are placed only as the blend
// drains (dispatch_probe.hip, chain_probe.hip).  If the blend's stream is created with a CU
// mask that leaves R CUs out, do a chain's workgroups on an unmasked stream get placed on
// those CUs at once, and what does the busy kernel lose?
//   hipcc --offload-arch=gfx950 -O3 -o cumask_probe cumask_probe.hip && ./cumask_probe
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));         \
            return 1;                                                                         \
        }                                                                                     \
    } while (0)

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }

// Busy: one-wave workgroups of 5-40 us of dependent FMAs (100 MHz ticks).
__global__ __launch_bounds__(64) void k_busy(unsigned long long* t, float* sink) {
    const uint64_t t0 = now();
    if (blockIdx.x == 0 && threadIdx.x == 0) t[0] = t0;
    const uint32_t h = blockIdx.x * 2654435761u;
    const uint64_t dur = 500 + (h >> 20) % 3500;
    float a = threadIdx.x, b = a + 1.0f, c = a + 2.0f, d = a + 3.0f;
    while (now() - t0 < dur) {
#pragma unroll
        for (int i = 0; i < 64; i++) {
            a = fmaf(a, 1.0001f, 0.5f);
            b = fmaf(b, 1.0001f, 0.5f);
            c = fmaf(c, 1.0001f, 0.5f);
            d = fmaf(d, 1.0001f, 0.5f);
        }
    }
    if (a + b + c + d == 1.2345f) sink[threadIdx.x] = a;
    if (threadIdx.x == 0) atomicMax(&t[1], (unsigned long long)now());
}

// Probe: 256-thread workgroups of ~2 us, start/end stamps.
__global__ __launch_bounds__(256) void k_probe(unsigned long long* st, float* sink) {
    const uint64_t t0 = now();
    float a = threadIdx.x;
    while (now() - t0 < 200) a = fmaf(a, 1.0001f, 0.5f);
    if (a == 1.2345f) sink[threadIdx.x] = a;
    if (threadIdx.x == 0) {
        st[2 * blockIdx.x] = t0;
        st[2 * blockIdx.x + 1] = now();
    }
}

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int ncu = p.multiProcessorCount;
    unsigned long long *t, *st;
    float* sink;
    CHECK(hipMalloc(&t, 16));
    CHECK(hipMalloc(&st, 16 * 8 * 1024));
    CHECK(hipMalloc(&sink, 4096));
    hipStream_t sb;
    CHECK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    const int G = 64, chain = 8;
    printf("%d CUs; busy: 20 rounds of one-wave workgroups of 5-40 us on a stream masked to leave R CUs out\n"
           "(every (%d/R)-th CU); probe: a chain of %d kernels x %d workgroups of 256 threads (~2 us each)\n"
           "on an unmasked stream, launched 100 us later; times in us from the busy kernel's first wave\n",
           ncu, ncu, chain, G);
    for (int rep = 0; rep < 2; rep++)
        for (int R : {0, 8, 16, 32, 64}) {
            std::vector<uint32_t> mask((ncu + 31) / 32, 0);
            for (int c = 0; c < ncu; c++) {
                const bool out = R > 0 && (c % (ncu / R)) == (ncu / R) - 1;
                if (!out) mask[c / 32] |= 1u << (c % 32);
            }
            hipStream_t sa;
            CHECK(hipExtStreamCreateWithCUMask(&sa, (uint32_t)mask.size(), mask.data()));
            CHECK(hipMemset(t, 0, 16));
            CHECK(hipDeviceSynchronize());
            const int busy_groups = ncu * 32 * 20;
            hipLaunchKernelGGL(k_busy, dim3(busy_groups), dim3(64), 0, sa, t, sink);
            std::this_thread::sleep_for(std::chrono::microseconds(100));
            for (int c = 0; c < chain; c++)
                hipLaunchKernelGGL(k_probe, dim3(G), dim3(256), 0, sb, st + 2 * (size_t)c * G, sink);
            CHECK(hipGetLastError());
            CHECK(hipDeviceSynchronize());
            unsigned long long ht[2];
            std::vector<unsigned long long> hs(2 * (size_t)G * chain);
            CHECK(hipMemcpy(ht, t, 16, hipMemcpyDeviceToHost));
            CHECK(hipMemcpy(hs.data(), st, hs.size() * 8, hipMemcpyDeviceToHost));
            unsigned long long mn = ~0ull, mx = 0;
            for (size_t g = 0; g < hs.size() / 2; g++) {
                mn = std::min(mn, hs[2 * g]);
                mx = std::max(mx, hs[2 * g + 1]);
            }
            printf("rep %d  R %2d  busy end %7.1f | chain first start %7.1f  last end %7.1f  span %7.1f us\n", rep, R,
                   (ht[1] - ht[0]) / 100.0, (mn - ht[0]) / 100.0, (mx - ht[0]) / 100.0, (mx - mn) / 100.0);
            CHECK(hipStreamDestroy(sa));
        }
    return 0;
}
