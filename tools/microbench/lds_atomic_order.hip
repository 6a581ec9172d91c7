// LDS atomic order probe (gfx950): does ds_add_rtn_u32 from one wave64 instruction
// return old values in LANE order when several lanes hit the same address?  If so,
// a stable counting-sort rank is `atomicAdd(&count[digit], 1)` (one LDS op) instead
// of ballot-based digit matching (~4 VALU per digit bit).  Every lane compares the
// value it got with its stable rank computed by ballot matching; mismatches are
// counted over many waves, iterations and digit distributions.  Also times both.
//   hipcc --offload-arch=gfx950 -O3 -o lds_atomic_order lds_atomic_order.hip && ./lds_atomic_order
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

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

// digits in [0, ndig); `skew` > 0 concentrates them (many lanes on few digits)
__global__ __launch_bounds__(256) void k_check(int iters, uint32_t ndig, int skew, uint32_t seed,
                                               unsigned long long* bad, unsigned long long* total) {
    __shared__ uint32_t cnt[4][256];
    const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63u;
    cnt[w][lane] = 0;
    cnt[w][lane + 64] = 0;
    cnt[w][lane + 128] = 0;
    cnt[w][lane + 192] = 0;
    __syncthreads();
    uint32_t expect_base[1];
    (void)expect_base;
    unsigned long long nbad = 0;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (int it = 0; it < iters; it++) {
        uint32_t h = hash32(seed ^ (blockIdx.x * 7919u + it * 104729u + lane * 31u + w * 1000003u));
        uint32_t d = h % ndig;
        if (skew == 1) d = (h >> 8) % 3 == 0 ? 0u : d;                 // a third of the lanes on digit 0
        if (skew == 2) d = (uint32_t)(lane >> 4) % ndig;                // runs of 16 lanes
        if (skew == 3) d = ((h >> 4) & 1) ? (lane * 5u) % ndig : 1u;   // interleaved
        const bool valid = ((h >> 20) & 7u) != 0u;                       // ~1/8 of the lanes idle
        // stable rank by ballot matching over 8 digit bits
        uint64_t peers = __ballot(valid);
        for (int b = 0; b < 8; b++) {
            const bool bit = (d >> b) & 1u;
            const uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        uint32_t before = 0;
        if (valid) before = cnt[w][d];
        // make sure every lane's read happens before any lane's atomic of this iteration
        __builtin_amdgcn_wave_barrier();
        uint32_t got = 0;
        if (valid) got = atomicAdd(&cnt[w][d], 1u);
        __builtin_amdgcn_wave_barrier();
        if (valid) {
            const uint32_t want = before + (uint32_t)__popcll(peers & lt);
            nbad += got != want;
        }
    }
    atomicAdd(bad, nbad);
    if (t == 0) atomicAdd(total, (unsigned long long)iters * 256ull);
}

int main() {
    unsigned long long *bad, *total;
    CHECK(hipMalloc(&bad, 8));
    CHECK(hipMalloc(&total, 8));
    const uint32_t digs[] = {1, 2, 4, 16, 128, 256};
    unsigned long long all_bad = 0, all_total = 0;
    for (int skew = 0; skew < 4; skew++)
        for (uint32_t nd : digs)
            for (uint32_t seed = 1; seed <= 3; seed++) {
                CHECK(hipMemset(bad, 0, 8));
                CHECK(hipMemset(total, 0, 8));
                hipLaunchKernelGGL(k_check, dim3(4096), dim3(256), 0, 0, 200, nd, skew, seed * 0x9E3779B9u, bad, total);
                CHECK(hipGetLastError());
                CHECK(hipDeviceSynchronize());
                unsigned long long hb, ht;
                CHECK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
                CHECK(hipMemcpy(&ht, total, 8, hipMemcpyDeviceToHost));
                all_bad += hb;
                all_total += ht;
                if (hb) printf("skew %d digits %u seed %u: %llu of %llu lane-ops out of lane order\n", skew, nd, seed, hb, ht);
            }
    printf("ds_add_rtn lane order: %llu mismatches in %llu lane-ops (%s)\n", all_bad, all_total,
           all_bad ? "NOT in lane order" : "all in lane order");
    return 0;
}
