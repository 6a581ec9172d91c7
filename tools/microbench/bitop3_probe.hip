// bitop3_probe.hip — analysis tool: prints v_bitop3_b32(0xF0, 0xCC, 0xAA, T) for a few
// truth tables T; the result byte equals T iff the table index is S0*4 + S1*2 + S2.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* o, const unsigned* in) {
    const unsigned a = in[0], b = in[1], c = in[2];
    o[0] = __builtin_amdgcn_bitop3_b32(a, b, c, 0x41);
    o[1] = __builtin_amdgcn_bitop3_b32(a, b, c, 0x90);
    o[2] = __builtin_amdgcn_bitop3_b32(a, b, c, 0x82);
    o[3] = __builtin_amdgcn_bitop3_b32(a, b, c, 0x01);
}
int main() {
    unsigned h[3] = {0xF0u, 0xCCu, 0xAAu}, r[4];
    unsigned *din, *dout;
    (void)hipMalloc(&din, 12);
    (void)hipMalloc(&dout, 16);
    (void)hipMemcpy(din, h, 12, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dout, din);
    (void)hipMemcpy(r, dout, 16, hipMemcpyDeviceToHost);
    std::printf("bitop3 T=0x41 -> 0x%x, T=0x90 -> 0x%x, T=0x82 -> 0x%x, T=0x01 -> 0x%x\n", r[0], r[1], r[2], r[3]);
    return 0;
}
