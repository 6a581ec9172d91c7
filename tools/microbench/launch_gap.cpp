// Cost of a dependent kernel launch on one stream (gfx950): chains of K
// kernels that do nothing, read one flag then exit, or write 1 KB per
// workgroup, at the grid sizes the pipeline uses.  Prints us per kernel.
//   hipcc --offload-arch=gfx950 -O3 -o launch_gap launch_gap.cpp && ./launch_gap
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty() {}
__global__ void k_flag(const unsigned* f) {
    if (*f == 12345u) asm volatile("s_nop 0");
}
__global__ void k_write(float* o) { o[blockIdx.x * 256 + threadIdx.x] = 1.0f; }

template <typename F>
float chain(F launch, int K) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 10; i++) launch();
    hipEventRecord(a, 0);
    for (int i = 0; i < K; i++) launch();
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms * 1e3f / K;
}

int main() {
    unsigned* f;
    float* o;
    hipMalloc(&f, 4);
    hipMemset(f, 0, 4);
    hipMalloc(&o, 8192 * 256 * 4);
    const int K = 200;
    for (int g : {1, 256, 489, 1024, 8160}) {
        const float e = chain([&] { hipLaunchKernelGGL(k_empty, dim3(g), dim3(256), 0, 0); }, K);
        const float fl = chain([&] { hipLaunchKernelGGL(k_flag, dim3(g), dim3(256), 0, 0, f); }, K);
        const float w = chain([&] { hipLaunchKernelGGL(k_write, dim3(g), dim3(256), 0, 0, o); }, K);
        printf("grid %5d: empty %.2f us  read-flag %.2f us  write 1KB/WG %.2f us\n", g, e, fl, w);
    }
    return 0;
}
