// Streaming-bandwidth yardstick (gfx950): what a plain coalesced kernel reaches on
// this HBM3E — read-only (sum), copy, write-only, and a 38-stream read shaped like
// k_preprocess (one thread per element, one 4-B load from each of 38 arrays) — so
// the geometry kernels' GB/s can be set against the practical rate, not only the
// 8 TB/s spec.  Sizes: 1 GiB per array pass (larger than the 256 MB MALL).
//   hipcc --offload-arch=gfx950 -O3 -o stream_rate stream_rate.hip && ./stream_rate
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

__global__ __launch_bounds__(256) void k_read(const float4* __restrict__ a, size_t n, float* out) {
    float s = 0.0f;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1.2345f) out[0] = s;
}

__global__ __launch_bounds__(256) void k_copy(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) b[i] = a[i];
}

__global__ __launch_bounds__(256) void k_write(float4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        b[i] = make_float4(1.0f, 2.0f, 3.0f, 4.0f);
}

// 38 arrays of n floats, one thread per element (the preprocess's access shape), all
// loads issued before use; writes one 16-B word per element (its record's shape).
template <bool NT = false>
__global__ __launch_bounds__(256) void k_soa38(const float* __restrict__ a, size_t stride, size_t n,
                                               float4* __restrict__ rec) {
    const size_t i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= n) return;
    float v[38];
#pragma unroll
    for (int k = 0; k < 38; k++) v[k] = NT ? __builtin_nontemporal_load(a + k * stride + i) : a[k * stride + i];
    float s0 = 0, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
    for (int k = 0; k < 38; k += 4) {
        s0 += v[k];
        if (k + 1 < 38) s1 += v[k + 1];
        if (k + 2 < 38) s2 += v[k + 2];
        if (k + 3 < 38) s3 += v[k + 3];
    }
    rec[i] = make_float4(s0, s1, s2, s3);
}

// The same bytes with 16 B per lane: each thread loads a float4 of every array (4 elements)
// and writes four 16-B words -- the access shape an LDS-staged preprocess would have.
__global__ __launch_bounds__(256) void k_soa38_v4(const float* __restrict__ a, size_t stride, size_t n,
                                                  float4* __restrict__ rec) {
    const size_t i4 = blockIdx.x * 256ull + threadIdx.x;   // float4 index
    if (4 * i4 >= n) return;
    float4 s = make_float4(0, 0, 0, 0);
    float4 v[38];
#pragma unroll
    for (int k = 0; k < 38; k++) v[k] = reinterpret_cast<const float4*>(a + k * stride)[i4];
#pragma unroll
    for (int k = 0; k < 38; k++) {
        s.x += v[k].x;
        s.y += v[k].y;
        s.z += v[k].z;
        s.w += v[k].w;
    }
    rec[4 * i4] = s;
    rec[4 * i4 + 1] = s;
    rec[4 * i4 + 2] = s;
    rec[4 * i4 + 3] = s;
}

// 38 arrays staged through LDS by float4 loads (wave w loads arrays w, w + 4, ...), then one
// element per thread read from LDS: the preprocess's one-thread-per-Gaussian shape with
// 16-B-per-lane global loads.
__global__ __launch_bounds__(256) void k_soa38_lds(const float* __restrict__ a, size_t stride, size_t n,
                                                   float4* __restrict__ rec) {
    __shared__ float4 s_v[38][64];   // 38 arrays x 256 elements
    const size_t i0 = blockIdx.x * 256ull;
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    for (int k = (int)w; k < 38; k += 4)
        s_v[k][lane] = reinterpret_cast<const float4*>(a + k * stride + i0)[lane];
    __syncthreads();
    const float* sf = reinterpret_cast<const float*>(s_v);
    float s0 = 0, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
    for (int k = 0; k < 38; k += 4) {
        s0 += sf[k * 256 + t];
        if (k + 1 < 38) s1 += sf[(k + 1) * 256 + t];
        if (k + 2 < 38) s2 += sf[(k + 2) * 256 + t];
        if (k + 3 < 38) s3 += sf[(k + 3) * 256 + t];
    }
    if (i0 + t < n) rec[i0 + t] = make_float4(s0, s1, s2, s3);
}

// Plain read with four 16-B loads in flight per thread (the one-load loop above is
// bound by its round trip, not by HBM).
__global__ __launch_bounds__(256) void k_read4(const float4* __restrict__ a, size_t n, float* out) {
    float s = 0.0f;
    const size_t st = (size_t)gridDim.x * 256;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i + 3 * st < n; i += 4 * st) {
        const float4 v0 = a[i], v1 = a[i + st], v2 = a[i + 2 * st], v3 = a[i + 3 * st];
        s += v0.x + v1.y + v2.z + v3.w;
    }
    if (s == 1.2345f) out[0] = s;
}

// The preprocess's load shape over a blocked layout: BLK elements x 38 arrays contiguous
// per block ([n / BLK][38][BLK] floats), so a workgroup's 38 loads fall in one ~38 KB
// region instead of 38 streams 20 MB apart.  NT: nontemporal loads.
template <int BLK, bool NT>
__global__ __launch_bounds__(256) void k_blk38(const float* __restrict__ a, size_t n, float4* __restrict__ rec) {
    const size_t i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= n) return;
    const float* base = a + (i / BLK) * (38ull * BLK) + (i % BLK);
    float v[38];
#pragma unroll
    for (int k = 0; k < 38; k++) v[k] = NT ? __builtin_nontemporal_load(base + k * BLK) : base[k * BLK];
    float s0 = 0, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
    for (int k = 0; k < 38; k += 4) {
        s0 += v[k];
        if (k + 1 < 38) s1 += v[k + 1];
        if (k + 2 < 38) s2 += v[k + 2];
        if (k + 3 < 38) s3 += v[k + 3];
    }
    rec[i] = make_float4(s0, s1, s2, s3);
}

int main() {
    const size_t bytes = 1ull << 30, n4 = bytes / 16;
    float4 *a, *b;
    float* out;
    CHECK(hipMalloc(&a, bytes));
    CHECK(hipMalloc(&b, bytes));
    CHECK(hipMalloc(&out, 64));
    CHECK(hipMemset(a, 0, bytes));
    CHECK(hipMemset(b, 0, bytes));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int grids[] = {1024, 2048, 4096, 8192};
    for (int g : grids) {
        float best[3] = {1e9f, 1e9f, 1e9f};
        for (int rep = 0; rep < 5; rep++) {
            for (int k = 0; k < 3; k++) {
                CHECK(hipEventRecord(e0));
                if (k == 0) hipLaunchKernelGGL(k_read, dim3(g), dim3(256), 0, 0, a, n4, out);
                if (k == 1) hipLaunchKernelGGL(k_copy, dim3(g), dim3(256), 0, 0, a, b, n4 / 2);
                if (k == 2) hipLaunchKernelGGL(k_write, dim3(g), dim3(256), 0, 0, b, n4);
                CHECK(hipEventRecord(e1));
                CHECK(hipEventSynchronize(e1));
                float ms;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < best[k]) best[k] = ms;
            }
        }
        printf("grid %5d x 256: read %.0f GB/s  copy (half read, half write) %.0f GB/s  write %.0f GB/s\n", g,
               bytes / (best[0] * 1e6), bytes / (best[1] * 1e6), bytes / (best[2] * 1e6));
    }
    // preprocess shape at config 3 size: 5M elements x 38 arrays (760 MB) + 80 MB of 16-B writes
    const size_t n = 5000000, stride = (n + 63) / 64 * 64;
    float best = 1e9f;
    for (int rep = 0; rep < 5; rep++) {
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_soa38<false>, dim3((n + 255) / 256), dim3(256), 0, 0, reinterpret_cast<const float*>(a), stride,
                           n, b);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    const double mb = (38.0 * 4 * n + 16.0 * n) / 1e6;
    printf("38-array SoA read + 16-B write, 5M elements (%.0f MB): %.1f us, %.0f GB/s\n", mb, best * 1e3,
           mb / (best * 1e3) * 1e3);
    for (int variant = 0; variant < 2; variant++) {
        float bv = 1e9f;
        for (int rep = 0; rep < 5; rep++) {
            CHECK(hipEventRecord(e0));
            if (variant == 0)
                hipLaunchKernelGGL(k_soa38_v4, dim3((n / 4 + 255) / 256), dim3(256), 0, 0,
                                   reinterpret_cast<const float*>(a), stride, n, b);
            else
                hipLaunchKernelGGL(k_soa38_lds, dim3((n + 255) / 256), dim3(256), 0, 0,
                                   reinterpret_cast<const float*>(a), stride, n, b);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < bv) bv = ms;
        }
        const double mbv = variant == 0 ? (38.0 * 4 * n + 64.0 * n) / 1e6 : mb;
        printf("%s: %.1f us, %.0f GB/s\n",
               variant == 0 ? "38-array SoA read, float4 per lane + 64-B writes per 4 elements"
                            : "38-array SoA read staged through LDS by float4 loads + 16-B write",
               bv * 1e3, mbv / (bv * 1e3) * 1e3);
    }
    {   // four loads in flight per thread
        float b4 = 1e9f;
        for (int rep = 0; rep < 5; rep++) {
            CHECK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_read4, dim3(4096), dim3(256), 0, 0, a, n4, out);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < b4) b4 = ms;
        }
        printf("read, 4 x 16-B loads in flight per thread, grid 4096: %.0f GB/s\n", bytes / (b4 * 1e6));
    }
    for (int variant = 0; variant < 8; variant++) {
        float bv = 1e9f;
        for (int rep = 0; rep < 5; rep++) {
            CHECK(hipEventRecord(e0));
            const float* af = reinterpret_cast<const float*>(a);
            const dim3 g((n + 255) / 256);
            if (variant == 0) hipLaunchKernelGGL((k_blk38<256, false>), g, dim3(256), 0, 0, af, n, b);
            if (variant == 1) hipLaunchKernelGGL((k_blk38<64, false>), g, dim3(256), 0, 0, af, n, b);
            if (variant == 2) hipLaunchKernelGGL((k_blk38<1024, false>), g, dim3(256), 0, 0, af, n, b);
            if (variant == 3) hipLaunchKernelGGL((k_blk38<256, true>), g, dim3(256), 0, 0, af, n, b);
            if (variant == 4) hipLaunchKernelGGL(k_soa38<false>, g, dim3(256), 0, 0, af, stride, n, b);
            if (variant == 5) hipLaunchKernelGGL(k_soa38<true>, g, dim3(256), 0, 0, af, stride, n, b);
            if (variant == 6) hipLaunchKernelGGL((k_blk38<64, true>), g, dim3(256), 0, 0, af, n, b);
            if (variant == 7) hipLaunchKernelGGL((k_blk38<1024, true>), g, dim3(256), 0, 0, af, n, b);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < bv) bv = ms;
        }
        static const char* names[] = {"blocked 256 x 38", "blocked 64 x 38", "blocked 1024 x 38",
                                      "blocked 256 x 38, nontemporal loads", "SoA 38 arrays (again)",
                                      "SoA 38 arrays, nontemporal loads", "blocked 64 x 38, nontemporal loads",
                                      "blocked 1024 x 38, nontemporal loads"};
        printf("%s read + 16-B write, 5M elements: %.1f us, %.0f GB/s\n", names[variant], bv * 1e3,
               mb / (bv * 1e3) * 1e3);
    }
    return 0;
}
