// Probes two gfx950 facts the MFMA correlation relies on (exact integer data, asymmetric operands):
//  1. v_mfma_i32_16x16x64_i8 operand map: lane l holds A[l&15][16*(l>>4) + j] and B[16*(l>>4) + j][l&15]
//     (j = 0..15, 4 VGPRs); D: col = l&15, row = 4*(l>>4) + r.
//  2. ds_read_b128 at byte-unaligned LDS addresses returns the bytes at that address.
// build: hipcc --offload-arch=gfx950 -O3 -o build/probe scripts/probe_mfma_lds.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void k_mfma(const int8_t* A, const int8_t* B, int32_t* D) {
    const int l = threadIdx.x;
    v4i a, b;
    int8_t* pa = (int8_t*)&a;
    int8_t* pb = (int8_t*)&b;
    for (int j = 0; j < 16; ++j) {
        pa[j] = A[(l & 15) * 64 + 16 * (l >> 4) + j];
        pb[j] = B[(16 * (l >> 4) + j) * 16 + (l & 15)];
    }
    v4i c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

__global__ void k_lds(uint32_t* out, int base) {
    __shared__ __attribute__((aligned(16))) uint8_t s[1024];
    for (int i = threadIdx.x; i < 1024; i += 64) s[i] = (uint8_t)(i * 7 + 3);
    __syncthreads();
    const int off = base + threadIdx.x;          // every byte offset
    const uint4 v = *(const uint4*)(s + off);
    out[threadIdx.x * 4 + 0] = v.x; out[threadIdx.x * 4 + 1] = v.y;
    out[threadIdx.x * 4 + 2] = v.z; out[threadIdx.x * 4 + 3] = v.w;
}

int main() {
    int8_t hA[16 * 64], hB[64 * 16];
    srand(5);
    for (int i = 0; i < 16 * 64; ++i) hA[i] = (int8_t)(rand() % 256 - 128);
    for (int i = 0; i < 64 * 16; ++i) hB[i] = (int8_t)(rand() % 256 - 128);
    int8_t *dA, *dB;
    int32_t* dD;
    (void)hipMalloc(&dA, sizeof hA); (void)hipMalloc(&dB, sizeof hB); (void)hipMalloc(&dD, 16 * 16 * 4);
    (void)hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_mfma, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    int32_t hD[256];
    (void)hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
            int32_t ref = 0;
            for (int k = 0; k < 64; ++k) ref += (int32_t)hA[i * 64 + k] * hB[k * 16 + j];
            if (ref != hD[i * 16 + j]) ++bad;
        }
    printf("mfma_i32_16x16x64_i8 layout: %s (%d/256 mismatches)\n", bad ? "MISMATCH" : "OK", bad);

    uint32_t* dO;
    (void)hipMalloc(&dO, 64 * 16);
    int lbad = 0;
    for (int base = 0; base < 4; ++base) {
        hipLaunchKernelGGL(k_lds, dim3(1), dim3(64), 0, 0, dO, base * 64 + 1);
        uint32_t hO[256];
        (void)hipMemcpy(hO, dO, sizeof hO, hipMemcpyDeviceToHost);
        for (int t = 0; t < 64; ++t) {
            const int off = base * 64 + 1 + t;
            for (int b = 0; b < 16; ++b) {
                const uint8_t got = (uint8_t)(hO[t * 4 + b / 4] >> (8 * (b % 4)));
                if (got != (uint8_t)((off + b) * 7 + 3)) { ++lbad; break; }
            }
        }
    }
    printf("unaligned ds_read_b128: %s (%d/256 lanes wrong)\n", lbad ? "WRONG" : "OK", lbad);
    return (bad || lbad) ? 1 : 0;
}
