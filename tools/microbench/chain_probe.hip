// Chain probe (gfx950): how fast does a chain of dependent small kernels (the
// geometry of the next frame in flight) progress while a blend-like kernel holds
// the GPU, against the same work as ONE resident kernel with grid barriers
// between its phases?  And what does each cost the blend-like kernel?
//
// blend-like: 32,640 one-wave workgroups (the config-2 blend's grid), 6 KB of LDS
// each (~26 per CU resident, like the blend), 20-100 us of dependent FMAs each.
// chain: 16 phases; each phase streams a 4 MB slice (read + write) over G
// workgroups of 256 threads (or 4 G one-wave workgroups).  "kernels": one launch per phase on a second stream;
// "resident": one launch of G workgroups, a grid barrier between phases (bounded
// spin: a barrier that waits too long sets an error flag and the kernel exits).
//   hipcc --offload-arch=gfx950 -O3 -o chain_probe chain_probe.hip && ./chain_probe
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdlib>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }

// t[0] = first wave start, t[1] = last wave end (100 MHz ticks)
__global__ __launch_bounds__(64) void k_blendlike(unsigned long long* t, float* sink) {
    __shared__ float pad[1536];
    const uint64_t t0 = now();
    if (threadIdx.x == 0) atomicMin(&t[0], (unsigned long long)t0);
    const uint32_t h = blockIdx.x * 2654435761u;
    const uint64_t dur = 2000 + (h >> 16) % 8000;
    pad[threadIdx.x] = (float)threadIdx.x;
    float a = pad[(threadIdx.x + 1) & 63], b = a + 1.0f, c = a + 2.0f, d = a + 3.0f;
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

constexpr int kPhases = 16;
constexpr size_t kSlice = 1u << 20;   // floats per phase slice (4 MB)

__device__ __forceinline__ void phase_work(const float* in, float* out, int phase, int g, int G) {
    const size_t per = kSlice / G;
    const size_t b = (size_t)g * per;
    const float* src = in + (size_t)phase * kSlice;
    float* dst = out + (size_t)phase * kSlice;
    for (size_t i = b + threadIdx.x; i < b + per; i += 256) dst[i] = src[i] * 1.5f + 1.0f;
}

template <int TPB>
__global__ __launch_bounds__(TPB) void k_phase(const float* in, float* out, int phase, unsigned long long* t) {
    __builtin_amdgcn_s_setprio(3);
    if (phase == 0 && threadIdx.x == 0) atomicMin(&t[2], (unsigned long long)now());
    if (threadIdx.x == 0) atomicMin(&t[4 + 2 * phase], (unsigned long long)now());   // per-phase first start
    // TPB threads per workgroup: the same slice per phase, split over gridDim.x workgroups
    const size_t per = kSlice / gridDim.x;
    const size_t b = (size_t)blockIdx.x * per;
    const float* src = in + (size_t)phase * kSlice;
    float* dst = out + (size_t)phase * kSlice;
    for (size_t i = b + threadIdx.x; i < b + per; i += TPB) dst[i] = src[i] * 1.5f + 1.0f;
    if (phase == kPhases - 1 && threadIdx.x == 0) atomicMax(&t[3], (unsigned long long)now());
    if (threadIdx.x == 0) atomicMax(&t[5 + 2 * phase], (unsigned long long)now());   // per-phase last end
}

__global__ __launch_bounds__(256) void k_resident(const float* in, float* out, unsigned* ctr, unsigned* err,
                                                  unsigned long long* t) {
    __builtin_amdgcn_s_setprio(3);
    if (threadIdx.x == 0) atomicMin(&t[2], (unsigned long long)now());
    const unsigned G = gridDim.x;
    for (int p = 0; p < kPhases; p++) {
        phase_work(in, out, p, blockIdx.x, G);
        if (p == kPhases - 1) break;
        __threadfence();
        __syncthreads();
        if (threadIdx.x == 0) {
            __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned target = G * (unsigned)(p + 1);
            unsigned spins = 0;
            while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1u << 22)) {
                    atomicOr(err, 1u);
                    break;
                }
            }
        }
        __syncthreads();
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    }
    if (threadIdx.x == 0) atomicMax(&t[3], (unsigned long long)now());
}

int main() {
    // CHAIN_FIRST=1: the chain's stream is created before the blend-like one (HIP hands
    // out hardware queues in creation order; does the queue order decide who waits?)
    hipStream_t sa, sb;
    const char* cf = getenv("CHAIN_FIRST");
    if (cf && cf[0] == '1') {
        CHECK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
        CHECK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    } else {
        CHECK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
        CHECK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    }
    unsigned long long* t;
    unsigned *ctr, *err;
    float *in, *out, *sink;
    CHECK(hipMalloc(&t, 8 * (4 + 2 * kPhases)));
    CHECK(hipMalloc(&ctr, 4));
    CHECK(hipMalloc(&err, 4));
    CHECK(hipMalloc(&in, kPhases * kSlice * 4));
    CHECK(hipMalloc(&out, kPhases * kSlice * 4));
    CHECK(hipMalloc(&sink, 4096));
    CHECK(hipMemset(in, 0, kPhases * kSlice * 4));
    const int blend_groups = 32640;
    printf("blend-like: %d one-wave workgroups, 20-100 us each; chain: %d phases of a 4 MB slice (read+write)\n"
           "times in us; 'chain' counts from the chain's first wave to its last\n", blend_groups, kPhases);
    unsigned long long init[4 + 2 * kPhases];
    for (int i = 0; i < 4 + 2 * kPhases; i++) init[i] = (i % 2 == 0) ? ~0ull : 0ull;
    for (int rep = 0; rep < 2; rep++) {
        // mode 0: blend-like alone; 1: kernels alone; 2: resident alone; 3: blend + kernels; 4: blend + resident;
        // 5: one-wave-workgroup kernels alone; 6: blend + one-wave-workgroup kernels
        for (int G : {256, 512, 1024}) {
            for (int mode = 0; mode < 7; mode++) {
                if (mode == 0 && G != 256) continue;
                if ((mode == 2 || mode == 4) && G > 512) continue;   // resident: at most 2 workgroups per CU
                CHECK(hipMemcpy(t, init, sizeof init, hipMemcpyHostToDevice));
                CHECK(hipMemset(ctr, 0, 4));
                CHECK(hipMemset(err, 0, 4));
                CHECK(hipDeviceSynchronize());
                const bool blend = mode == 0 || mode == 3 || mode == 4 || mode == 6;
                if (blend) hipLaunchKernelGGL(k_blendlike, dim3(blend_groups), dim3(64), 0, sa, t, sink);
                if (blend && mode != 0) std::this_thread::sleep_for(std::chrono::microseconds(50));
                if (mode == 1 || mode == 3)
                    for (int p = 0; p < kPhases; p++)
                        hipLaunchKernelGGL(k_phase<256>, dim3(G), dim3(256), 0, sb, in, out, p, t);
                if (mode == 5 || mode == 6)   // one-wave workgroups, 4x as many (same threads)
                    for (int p = 0; p < kPhases; p++)
                        hipLaunchKernelGGL(k_phase<64>, dim3(4 * G), dim3(64), 0, sb, in, out, p, t);
                if (mode == 2 || mode == 4) hipLaunchKernelGGL(k_resident, dim3(G), dim3(256), 0, sb, in, out, ctr, err, t);
                CHECK(hipGetLastError());
                CHECK(hipDeviceSynchronize());
                unsigned long long h[4 + 2 * kPhases];
                unsigned herr;
                CHECK(hipMemcpy(h, t, sizeof h, hipMemcpyDeviceToHost));
                CHECK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
                const char* names[] = {"blend alone", "kernels alone", "resident alone", "blend + kernels",
                                       "blend + resident", "64-thr kernels alone", "blend + 64-thr kernels"};
                printf("rep %d G %4d %-22s", rep, G, names[mode]);
                if (blend) printf("  blend %7.1f", (h[1] - h[0]) / 100.0);
                if (mode) printf("  chain %7.1f", (h[3] - h[2]) / 100.0);
                if (blend && mode) printf("  (chain start %+7.1f, end %+7.1f vs blend start)",
                                          ((double)h[2] - (double)h[0]) / 100.0, ((double)h[3] - (double)h[0]) / 100.0);
                if (herr) printf("  BARRIER TIMEOUT");
                printf("\n");
                if (blend && (mode == 3 || mode == 6) && G == 256) {   // per-phase [start, end] vs blend start
                    printf("      phases:");
                    for (int p = 0; p < kPhases; p++)
                        printf(" [%.0f,%.0f]", ((double)h[4 + 2 * p] - (double)h[0]) / 100.0,
                               ((double)h[5 + 2 * p] - (double)h[0]) / 100.0);
                    printf("\n");
                }
            }
        }
    }
    return 0;
}
