// Probe: __builtin_amdgcn_global_load_lds (4-byte) places lane l's dword at LDS base + 4*l, from a per-lane
// global address; the LDS base is wave-uniform.  build: hipcc --offload-arch=gfx950 -O3 -o build/probe_glds scripts/probe_glds.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef __attribute__((address_space(3))) void* lds_vp;
typedef __attribute__((address_space(1))) void* gbl_vp;

__global__ void k(const uint32_t* src, uint32_t* out) {
    __shared__ uint32_t buf[2][64 * 4];
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = 0; i < 4; ++i) {
        const uint32_t* g = src + ((l * 7 + 3 * i + w) & 255);          // per-lane scattered source
        __builtin_amdgcn_global_load_lds((gbl_vp)g, (lds_vp)(&buf[w][64 * i]), 4, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = 0; i < 4; ++i) out[w * 256 + 64 * i + l] = buf[w][64 * i + l];
}

int main() {
    uint32_t h[256], *d, *o, ho[512];
    for (int i = 0; i < 256; ++i) h[i] = 0x1000 + i;
    (void)hipMalloc(&d, sizeof h); (void)hipMalloc(&o, sizeof ho);
    (void)hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(128), 0, 0, d, o);
    (void)hipMemcpy(ho, o, sizeof ho, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int w = 0; w < 2; ++w)
        for (int i = 0; i < 4; ++i)
            for (int l = 0; l < 64; ++l)
                if (ho[w * 256 + 64 * i + l] != h[(l * 7 + 3 * i + w) & 255]) ++bad;
    printf("global_load_lds dword lane placement: %s (%d/512 wrong)\n", bad ? "WRONG" : "OK", bad);
    return bad ? 1 : 0;
}
