// Issue cost of the integer VALU instructions the bilinear taps use, at full occupancy (8 independent chains per
// lane, 2048 workgroups of 256 threads): cycles per wave64 instruction per SIMD from s_memtime around the loop.
// build: hipcc --offload-arch=gfx950 -O3 -o build/valu_rate scripts/valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

#define BODY8(INS)                                                                                          \
    asm volatile(INS " %0, %0, %8, %9\n\t" INS " %1, %1, %8, %9\n\t" INS " %2, %2, %8, %9\n\t" INS          \
                     " %3, %3, %8, %9\n\t" INS " %4, %4, %8, %9\n\t" INS " %5, %5, %8, %9\n\t" INS          \
                     " %6, %6, %8, %9\n\t" INS " %7, %7, %8, %9"                                           \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)            \
                 : "v"(b), "v"(c))
#define BODY8_2(INS)                                                                                        \
    asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS " %3, %3, %8\n\t" INS  \
                     " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS " %6, %6, %8\n\t" INS " %7, %7, %8"         \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)            \
                 : "v"(b))

template <int OP>
__global__ __launch_bounds__(256) void k(unsigned* out, unsigned long long* cyc, unsigned seed, int iters) {
    unsigned a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17,
             a7 = a0 * 19, b = seed ^ threadIdx.x, c = seed * 31;
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int it = 0; it < iters; ++it) {
        if (OP == 0) BODY8_2("v_add_u32");
        if (OP == 1) BODY8_2("v_mul_u32_u24");
        if (OP == 2) BODY8("v_mad_u32_u24");
        if (OP == 3) BODY8_2("v_mul_lo_u32");
        if (OP == 4) BODY8("v_bfe_u32");
        if (OP == 5) BODY8("v_alignbyte_b32");
        if (OP == 6) BODY8("v_dot4_u32_u8");
        if (OP == 7) BODY8("v_perm_b32");
        if (OP == 8) BODY8("v_lshl_or_b32");
        if (OP == 9) BODY8("v_add3_u32");
        if (OP == 10) BODY8("v_mad_i32_i24");
        if (OP == 11) BODY8_2("v_ashrrev_i32");
        if (OP == 12) BODY8("v_pk_mad_u16");
        if (OP == 13) BODY8("v_dot2_u32_u16");
        if (OP == 14) BODY8_2("v_pk_sub_i16");
        if (OP == 15) BODY8("v_lshl_add_u32");
        if (OP == 16) BODY8_2("v_sub_u32");
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    const char* names[] = {"v_add_u32", "v_mul_u32_u24", "v_mad_u32_u24", "v_mul_lo_u32", "v_bfe_u32",
                           "v_alignbyte_b32", "v_dot4_u32_u8", "v_perm_b32", "v_lshl_or_b32", "v_add3_u32",
                           "v_mad_i32_i24", "v_ashrrev_i32", "v_pk_mad_u16", "v_dot2_u32_u16",
                           "v_pk_sub_i16", "v_lshl_add_u32", "v_sub_u32"};
    const int blocks = 2048, iters = 2048;
    unsigned* d;
    unsigned long long* dc;
    CK(hipMalloc(&d, blocks * 256 * 4));
    CK(hipMalloc(&dc, blocks * 8));
    auto run = [&](int op) -> double {
        hipEvent_t e0, e1;
        hipEventCreate(&e0); hipEventCreate(&e1);
        auto launch = [&]() {
            switch (op) {
                case 0: hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, d, dc, 7u, iters); break;
                case 1: hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, d, dc, 7u, iters); break;
                case 2: hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, d, dc, 7u, iters); break;
                case 3: hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, d, dc, 7u, iters); break;
                case 4: hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, d, dc, 7u, iters); break;
                case 5: hipLaunchKernelGGL(k<5>, dim3(blocks), dim3(256), 0, 0, d, dc, 7u, iters); break;
                case 6: hipLaunchKernelGGL(k<6>, dim3(blocks), dim3(256), 0, 0, d, dc, 7u, iters); break;
                case 7: hipLaunchKernelGGL(k<7>, dim3(blocks), dim3(256), 0, 0, d, dc, 7u, iters); break;
                case 8: hipLaunchKernelGGL(k<8>, dim3(blocks), dim3(256), 0, 0, d, dc, 7u, iters); break;
                case 9: hipLaunchKernelGGL(k<9>, dim3(blocks), dim3(256), 0, 0, d, dc, 7u, iters); break;
                case 10: hipLaunchKernelGGL(k<10>, dim3(blocks), dim3(256), 0, 0, d, dc, 7u, iters); break;
                case 11: hipLaunchKernelGGL(k<11>, dim3(blocks), dim3(256), 0, 0, d, dc, 7u, iters); break;
                case 12: hipLaunchKernelGGL(k<12>, dim3(blocks), dim3(256), 0, 0, d, dc, 7u, iters); break;
                case 13: hipLaunchKernelGGL(k<13>, dim3(blocks), dim3(256), 0, 0, d, dc, 7u, iters); break;
                case 14: hipLaunchKernelGGL(k<14>, dim3(blocks), dim3(256), 0, 0, d, dc, 7u, iters); break;
                case 15: hipLaunchKernelGGL(k<15>, dim3(blocks), dim3(256), 0, 0, d, dc, 7u, iters); break;
                default: hipLaunchKernelGGL(k<16>, dim3(blocks), dim3(256), 0, 0, d, dc, 7u, iters); break;
            }
        };
        launch();
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        return ms / 5;
    };
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const double simds = prop.multiProcessorCount * 4.0;
    const double instr = (double)blocks * 4 * iters * 8;   // wave-instructions
    double base = 0;
    for (int op = 0; op < 17; ++op) {
        const double ms = run(op);
        // cycles per wave-instruction per SIMD at an assumed 2.4 GHz (relative numbers are what matter)
        const double cpi = ms * 1e-3 * 2.4e9 / (instr / simds);
        if (op == 0) base = ms;
        printf("%-18s %8.3f ms  %5.2f cyc/wave-instr/SIMD @2.4GHz  %.2fx v_add\n", names[op], ms, cpi, ms / base);
    }
    return 0;
}
