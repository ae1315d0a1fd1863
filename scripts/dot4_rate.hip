#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(256) void k(unsigned* out, unsigned seed, int iters) {
    unsigned a[8], b = seed + threadIdx.x;
    for (int i = 0; i < 8; ++i) a[i] = seed * (i + 1);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = __builtin_amdgcn_udot4(b, a[i] ^ b, a[i], false);
    }
    unsigned s = 0;
    for (int i = 0; i < 8; ++i) s += a[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void kadd(unsigned* out, unsigned seed, int iters) {
    unsigned a[8], b = seed + threadIdx.x;
    for (int i = 0; i < 8; ++i) a[i] = seed * (i + 1);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = (a[i] ^ b) + a[i];
    }
    unsigned s = 0;
    for (int i = 0; i < 8; ++i) s += a[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
    unsigned* d; hipMalloc(&d, 4 << 20);
    const int blocks = 256 * 8, iters = 4096;
    for (int v = 0; v < 2; ++v) {
        hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
        auto launch = [&]() { if (v == 0) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 7u, iters);
                              else hipLaunchKernelGGL(kadd, dim3(blocks), dim3(256), 0, 0, d, 7u, iters); };
        launch(); hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        const double ops = (double)blocks * 256 * iters * 8;
        printf("%s: %.3f ms  %.1f Tops/s (lane-ops, 2 VALU per op for the add variant)\n", v == 0 ? "dot4(+xor)" : "xor+add", ms, ops / ms / 1e9);
    }
}
