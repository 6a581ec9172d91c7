// Is v_exp_f32 (2^t) correctly rounded on gfx950?  Over every float t in [T_LO, T_HI):
// compare the hardware result with 2^t computed in double precision and rounded to
// float (exact except within ~1e-16 of a rounding midpoint; such cases are counted
// apart).  Prints the mismatches, the largest difference in ulps, and examples.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <cmath>

__device__ __forceinline__ uint32_t fkey(float f) { uint32_t b = __float_as_uint(f); return (b & 0x80000000u) ? ~b : (b | 0x80000000u); }
__device__ __forceinline__ float kfloat(uint32_t k) { return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k); }

__global__ void probe(uint32_t klo, uint32_t khi, unsigned long long* cnt, unsigned int* maxulp, float* ex) {
    const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
    unsigned long long bad = 0, hard = 0, n = 0;
    unsigned int mu = 0;
    for (uint64_t k = klo + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < khi; k += nthr) {
        const float t = kfloat((uint32_t)k);
        const float h = __builtin_amdgcn_exp2f(t);
        const double d = exp2((double)t);
        const float r = (float)d;
        n++;
        if (h != r) {
            // near a midpoint? distance of d from the midpoint between r and its neighbour toward d
            const float nb = d > (double)r ? nextafterf(r, INFINITY) : nextafterf(r, -INFINITY);
            const double mid = 0.5 * ((double)r + (double)nb);
            if (fabs(d - mid) < 1e-15 * fabs(d)) hard++;
            else {
                bad++;
                const unsigned int u = (unsigned int)abs((int)__float_as_uint(h) - (int)__float_as_uint(r));
                mu = max(mu, u);
                if (bad == 1 && atomicAdd(cnt + 3, 1ull) < 4) {
                    const unsigned long long s = atomicAdd(cnt + 4, 1ull);
                    if (s < 4) { ex[3 * s] = t; ex[3 * s + 1] = h; ex[3 * s + 2] = r; }
                }
            }
        }
    }
    atomicAdd(cnt, bad); atomicAdd(cnt + 1, hard); atomicAdd(cnt + 2, n); atomicMax(maxulp, mu);
}

static uint32_t hkey(float f) { uint32_t b; memcpy(&b, &f, 4); return (b & 0x80000000u) ? ~b : (b | 0x80000000u); }

int main(int argc, char** argv) {
    const float ranges[][2] = {{-12.0f, 1.0f}, {-126.0f, -12.0f}, {1.0f, 127.0f}};
    unsigned long long* dc; unsigned int* dm; float* de;
    hipMalloc(&dc, 5 * 8); hipMalloc(&dm, 4); hipMalloc(&de, 12 * 4);
    for (auto& rg : ranges) {
        hipMemset(dc, 0, 40); hipMemset(dm, 0, 4); hipMemset(de, 0, 48);
        hipLaunchKernelGGL(probe, dim3(16384), dim3(256), 0, 0, hkey(rg[0]), hkey(rg[1]), dc, dm, de);
        unsigned long long c[5]; unsigned int m; float e[12];
        hipMemcpy(c, dc, 40, hipMemcpyDeviceToHost); hipMemcpy(&m, dm, 4, hipMemcpyDeviceToHost);
        hipMemcpy(e, de, 48, hipMemcpyDeviceToHost);
        printf("t in [%g, %g): %llu floats, %llu not correctly rounded (max %u ulp), %llu near-midpoint (undecided)\n",
               rg[0], rg[1], c[2], c[0], m, c[1]);
        for (int s = 0; s < 4 && s < (int)c[4]; s++) printf("   e.g. t=%a hw=%a rn=%a\n", e[3 * s], e[3 * s + 1], e[3 * s + 2]);
    }
    return 0;
}
