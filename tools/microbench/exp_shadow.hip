// Does independent VALU work issue in the shadow of v_exp_f32 (gfx950)?  Each step of
// the loop is E v_exp_f32 (E = 0 or 2, independent chains) plus F v_fma_f32 spread over 8
// independent chains, as in the blend's pair loop (two exps per pair among ~34 other
// VALU).  Printed: SIMD-cycles per step at 2.4 GHz, with 8 waves per SIMD (256 CUs x 32
// waves).  If the exps overlap the fmas, cycles(E=2, F) ~ max(cycles(0, F), cycles(2, 0))
// rather than the sum; that tells whether cutting non-exp VALU from the loop can pay.
//   hipcc --offload-arch=gfx950 -O3 -o exp_shadow exp_shadow.hip && ./exp_shadow
#include <hip/hip_runtime.h>
#include <cstdio>

#define STEPS 32

template <int E, int F>
__global__ __launch_bounds__(256) void k(float* out, int iters) {
    float a[8];
#pragma unroll
    for (int c = 0; c < 8; c++) a[c] = threadIdx.x + c;
    float e0 = threadIdx.x * 1e-3f, e1 = e0 + 1e-4f;
    const float b = 1.0001f, cc = 0.5f;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int s = 0; s < STEPS; s++) {
            if (E >= 1) asm volatile("v_exp_f32 %0, %0" : "+v"(e0));
#pragma unroll
            for (int f = 0; f < F / 2; f++) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[f & 7]) : "v"(b), "v"(cc));
            if (E >= 2) asm volatile("v_exp_f32 %0, %0" : "+v"(e1));
#pragma unroll
            for (int f = F / 2; f < F; f++) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[f & 7]) : "v"(b), "v"(cc));
        }
    }
    float r = e0 + e1;
#pragma unroll
    for (int c = 0; c < 8; c++) r += a[c];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int E, int F>
void run(float* out, int blocks, int iters) {
    hipEvent_t t0, t1;
    (void)hipEventCreate(&t0);
    (void)hipEventCreate(&t1);
    hipLaunchKernelGGL((k<E, F>), dim3(blocks), dim3(256), 0, 0, out, 2);
    (void)hipEventRecord(t0, 0);
    hipLaunchKernelGGL((k<E, F>), dim3(blocks), dim3(256), 0, 0, out, iters);
    (void)hipEventRecord(t1, 0);
    (void)hipEventSynchronize(t1);
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, t0, t1);
    const double waves_per_simd = blocks * 4.0 / (256 * 4.0);
    const double steps = (double)iters * STEPS * waves_per_simd;   // steps each SIMD runs
    const double cycles = ms * 1e-3 * 2.4e9 / steps;
    printf("exp %d  fma %2d  : %6.2f SIMD-cycles per step  (%.2f per VALU instruction)\n", E, F, cycles,
           (E + F) ? cycles / (E + F) : 0.0);
}

int main() {
    float* out = nullptr;
    if (hipMalloc(&out, 256 * 8 * 256 * sizeof(float)) != hipSuccess) return 1;
    const int blocks = 256 * 8, iters = 100;
    run<2, 0>(out, blocks, iters);
    run<0, 8>(out, blocks, iters);
    run<2, 8>(out, blocks, iters);
    run<0, 16>(out, blocks, iters);
    run<2, 16>(out, blocks, iters);
    run<0, 24>(out, blocks, iters);
    run<2, 24>(out, blocks, iters);
    run<0, 34>(out, blocks, iters);
    run<2, 34>(out, blocks, iters);
    run<2, 32>(out, blocks, iters);
    run<2, 30>(out, blocks, iters);
    (void)hipFree(out);
    return 0;
}
