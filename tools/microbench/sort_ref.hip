// sort_ref.hip — analysis tool (not product): times rocPRIM's device radix sort on
// the depth sort's workload, as a yardstick for our hand-written passes.
// Items are u64 (key << 32 | index) with keys spread over `span_bits` bits above a
// base (the preprocess key -Z * 1e6 of a frame), sorted on bits [32, 32 + span_bits).
//   hipcc -O3 --offload-arch=gfx950 -o sort_ref sort_ref.hip
//   ./sort_ref [n_millions=1,2,5] [span_bits=24]
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

static void run(size_t n, int span_bits) {
    std::vector<unsigned long long> h(n);
    std::mt19937_64 rng(7);
    const unsigned long long base = 3000000ull;
    for (size_t i = 0; i < n; i++) {
        const unsigned long long key = base + (rng() & ((1ull << span_bits) - 1ull));
        h[i] = (key << 32) | (unsigned long long)i;
    }
    unsigned long long *in = nullptr, *out = nullptr;
    CK(hipMalloc(&in, n * 8));
    CK(hipMalloc(&out, n * 8));
    CK(hipMemcpy(in, h.data(), n * 8, hipMemcpyHostToDevice));
    // key bits that differ: [32, 32 + span_bits + 1) covers base + span
    const unsigned begin = 32, end = 32 + span_bits + 2;
    size_t tmp_bytes = 0;
    CK(rocprim::radix_sort_keys(nullptr, tmp_bytes, in, out, n, begin, end));
    void* tmp = nullptr;
    CK(hipMalloc(&tmp, tmp_bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 5; w++) CK(rocprim::radix_sort_keys(tmp, tmp_bytes, in, out, n, begin, end));
    const int reps = 50;
    CK(hipEventRecord(a, 0));
    for (int r = 0; r < reps; r++) CK(rocprim::radix_sort_keys(tmp, tmp_bytes, in, out, n, begin, end));
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<unsigned long long> o(n);
    CK(hipMemcpy(o.data(), out, n * 8, hipMemcpyDeviceToHost));
    bool ok = true;
    for (size_t i = 1; i < n; i++) ok &= o[i - 1] <= o[i];
    std::printf("rocprim radix_sort_keys n=%zu bits=[%u,%u) %.1f us/sort sorted=%d\n", n, begin, end,
                1000.0 * ms / reps, (int)ok);
    CK(hipFree(tmp));
    CK(hipFree(in));
    CK(hipFree(out));
}

int main(int argc, char** argv) {
    const int span = argc > 2 ? std::atoi(argv[2]) : 24;
    if (argc > 1) {
        run((size_t)(std::atof(argv[1]) * 1e6), span);
        return 0;
    }
    for (double m : {1.0, 2.0, 5.0}) run((size_t)(m * 1e6), span);
    return 0;
}
