// Dispatch probe (gfx950): while a long kernel of one-wave (or 256-thread) workgroups fills every
// wave slot (the blend's shape), how soon do the workgroups of a small kernel on a
// second stream get placed, as a function of their size (64 vs 256 threads) and of
// the LDS they ask for?  Answers whether the frames-in-flight geometry chain starves
// because its 256-thread workgroups cannot find room while blend waves refill
// every freed slot.
//   hipcc --offload-arch=gfx950 -O3 -o dispatch_probe dispatch_probe.hip && ./dispatch_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>
#include <algorithm>

#define CHECK(x)                                                                 \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                            \
        }                                                                        \
    } while (0)

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }

// Busy: each one-wave workgroup runs dependent FMAs for 5-40 us (100 MHz ticks).
__global__ __launch_bounds__(256) void k_busy(unsigned long long* t, float* sink) {
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

// Probe: records each workgroup's start and end; ~2 us of work; optional LDS.
template <int LDS_WORDS>
__global__ void k_probe(unsigned long long* st, float* sink, int prio) {
    if (prio) __builtin_amdgcn_s_setprio(3);
    const uint64_t t0 = now();
    __shared__ float s[LDS_WORDS > 0 ? LDS_WORDS : 1];
    float a = threadIdx.x;
    s[threadIdx.x % (LDS_WORDS > 0 ? LDS_WORDS : 1)] = a;
    __syncthreads();
    while (now() - t0 < 200) a = fmaf(a, 1.0001f, s[(threadIdx.x + 1) % (LDS_WORDS > 0 ? LDS_WORDS : 1)]);
    if (a == 1.2345f) sink[threadIdx.x] = a;
    if (threadIdx.x == 0) {
        st[2 * blockIdx.x] = t0;
        st[2 * blockIdx.x + 1] = now();
    }
}

static int run(hipStream_t sa, hipStream_t sb, unsigned long long* t, unsigned long long* st, float* sink,
               int busy_threads, int threads, int G, int lds, int prio, int chain, const char* tag) {
    CHECK(hipMemset(t, 0, 16));
    CHECK(hipDeviceSynchronize());
    const int busy_groups = busy_threads ? 256 * 32 * 20 * 64 / busy_threads : 0;
    if (busy_threads) hipLaunchKernelGGL(k_busy, dim3(busy_groups), dim3(busy_threads), 0, sa, t, sink);
    std::this_thread::sleep_for(std::chrono::microseconds(100));
    // a chain of dependent probe kernels on one stream; each writes its own records
    for (int c = 0; c < chain; c++) {
        unsigned long long* sc = st + 2 * (size_t)c * G;
        if (lds == 0)
            hipLaunchKernelGGL(k_probe<0>, dim3(G), dim3(threads), 0, sb, sc, sink, prio);
        else
            hipLaunchKernelGGL(k_probe<8192>, dim3(G), dim3(threads), 0, sb, sc, sink, prio);
    }
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
    const double base = busy_threads ? (double)ht[0] : (double)mn;
    printf("%-6s busy %3d thr (end %7.1f) | probe %3d thr x %4d wg%s%s x %d kernels: first start %7.1f  last end %7.1f"
           "  span %7.1f us\n",
           tag, busy_threads, busy_threads ? (ht[1] - ht[0]) / 100.0 : 0.0, threads, G, lds ? ", 32 KB LDS" : "",
           prio ? ", prio 3" : "", chain, (mn - base) / 100.0, (mx - base) / 100.0, (mx - mn) / 100.0);
    return 0;
}

int main() {
    hipStream_t sa, sb;
    CHECK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    unsigned long long *t, *st;
    float* sink;
    CHECK(hipMalloc(&t, 16));
    CHECK(hipMalloc(&st, 16 * 8 * 1024));
    CHECK(hipMalloc(&sink, 4096));
    printf("busy: one long kernel (20 rounds of 5-40 us workgroups, 64 or 256 threads); probe: workgroups of\n"
           "~2 us on a second stream, launched ~100 us later (a chain: dependent kernels on that stream);\n"
           "times in us from the busy kernel's first wave\n");
    struct P { int threads, G, lds, prio, chain; };
    const P ps[] = {{64, 64, 0, 0, 1},   {64, 256, 0, 0, 1},  {64, 1024, 0, 0, 1}, {256, 64, 0, 0, 1},
                    {256, 256, 0, 0, 1}, {64, 256, 1, 0, 1},  {64, 64, 0, 0, 8},   {256, 16, 0, 0, 8},
                    {64, 64, 0, 1, 8},   {256, 64, 0, 0, 8}};
    for (int rep = 0; rep < 2; rep++)
        for (int bt : {64, 256})
            for (const P& p : ps)
                if (run(sa, sb, t, st, sink, bt, p.threads, p.G, p.lds, p.prio, p.chain, rep ? "rep1" : "rep0")) return 1;
    for (const P& p : ps)
        if (run(sa, sb, t, st, sink, 0, p.threads, p.G, p.lds, p.prio, p.chain, "alone")) return 1;
    return 0;
}
