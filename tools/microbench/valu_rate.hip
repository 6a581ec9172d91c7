// VALU issue-rate microbenchmark (gfx950): wave64 instructions per SIMD-cycle
// for v_fma_f32, v_pk_fma_f32, v_exp_f32, v_cndmask_b32 and v_readlane_b32, with
// 8 independent chains per lane and 8 waves per SIMD (256 CUs x 32 waves).
//   hipcc --offload-arch=gfx950 -O3 -o valu_rate valu_rate.hip && ./valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP 256
template <int OP>
__global__ __launch_bounds__(256) void k(float* out, int iters) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
          a7 = a0 + 7;
    const float b = 1.0001f, c = 0.5f;
    double p0 = a0, p1 = a1, p2 = a2, p3 = a3;
    const double pb = 1.0;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int r = 0; r < REP / 8; r++) {
            if (OP == 0) {
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a0) : "v"(b), "v"(c));
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a1) : "v"(b), "v"(c));
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a2) : "v"(b), "v"(c));
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a3) : "v"(b), "v"(c));
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a4) : "v"(b), "v"(c));
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a5) : "v"(b), "v"(c));
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a6) : "v"(b), "v"(c));
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a7) : "v"(b), "v"(c));
            } else if (OP == 1) {
                // four independent 64-bit register pairs, two packed fmas per lane each
                asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p0) : "v"(pb));
                asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p1) : "v"(pb));
                asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p2) : "v"(pb));
                asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p3) : "v"(pb));
                asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p0) : "v"(pb));
                asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p1) : "v"(pb));
                asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p2) : "v"(pb));
                asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p3) : "v"(pb));
            } else if (OP == 2) {
                asm volatile("v_exp_f32 %0, %0" : "+v"(a0));
                asm volatile("v_exp_f32 %0, %0" : "+v"(a1));
                asm volatile("v_exp_f32 %0, %0" : "+v"(a2));
                asm volatile("v_exp_f32 %0, %0" : "+v"(a3));
                asm volatile("v_exp_f32 %0, %0" : "+v"(a4));
                asm volatile("v_exp_f32 %0, %0" : "+v"(a5));
                asm volatile("v_exp_f32 %0, %0" : "+v"(a6));
                asm volatile("v_exp_f32 %0, %0" : "+v"(a7));
            } else if (OP == 3) {
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(a0) : "v"(b));
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(a1) : "v"(b));
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(a2) : "v"(b));
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(a3) : "v"(b));
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(a4) : "v"(b));
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(a5) : "v"(b));
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(a6) : "v"(b));
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(a7) : "v"(b));
            }
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + (float)(p0 + p1 + p2 + p3);
}

template <int OP>
double run(float* out, int blocks, int iters, int instr_per_rep) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, 2);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, iters);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double waves = blocks * 4.0;
    const double instrs = waves * iters * (double)instr_per_rep;   // wave-instructions
    const double simds = 256 * 4.0;
    const double cycles = ms * 1e-3 * 2.4e9;
    return instrs / simds / cycles;   // wave-instructions per SIMD per cycle (at 2.4 GHz)
}

int main() {
    float* out;
    hipMalloc(&out, 256 * 8 * 256 * 4 * sizeof(float));
    const int blocks = 256 * 8, iters = 200;
    printf("v_fma_f32     %.3f wave-instr/SIMD/cycle\n", run<0>(out, blocks, iters, REP));
    printf("v_pk_fma_f32  %.3f wave-instr/SIMD/cycle (each = 2 fma per lane)\n", run<1>(out, blocks, iters, REP));
    printf("v_exp_f32     %.3f wave-instr/SIMD/cycle\n", run<2>(out, blocks, iters, REP));
    printf("v_add_f32     %.3f wave-instr/SIMD/cycle\n", run<3>(out, blocks, iters, REP));
    return 0;
}
