// pyr_walk.hip — profiling harness (not part of the product): the source pyramid's level-0 pass against the HBM
// copy ceiling.  Times (a) float4 copy / read kernels in the guide's form (MI355X_MICROARCH.md: 6.29 TB/s float4
// copy), (b) the product k_pyr_down_s at level 0 -> 1 of nsrc Src7-sized sources in the engine's layout, and (c) a
// barrier-free wave-walker form of cv::pyrDown (no LDS: a wave owns a strip of output columns and walks down its
// rows; vertical [1 4 6 4 1] in packed u16 accumulators as the rows stream in, horizontal by v_dot2 on the finished
// output row with the halo pairs from the neighbouring lanes by DPP wave shifts), checked byte for byte against (b).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/pyr_walk.hip -o build/pyr_walk
#include "../fastest_image_pattern_matching_amd/csrc/fpm_kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace fpm;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

// ---- ceilings -------------------------------------------------------------------------------------------------
template <int U>
__global__ __launch_bounds__(256) void k_copy4(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
    const size_t stride = (size_t)gridDim.x * 256 * U;
    for (size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x; i < n16; i += stride) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = i + 256 * u < n16 ? src[i + 256 * u] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < U; ++u) if (i + 256 * u < n16) dst[i + 256 * u] = v[u];
    }
}
template <int U>
__global__ __launch_bounds__(256) void k_read4(const uint4* __restrict__ src, size_t n16, uint32_t* out) {
    const size_t stride = (size_t)gridDim.x * 256 * U;
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x; i < n16; i += stride) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = i + 256 * u < n16 ? src[i + 256 * u] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u].x + v[u].y + v[u].z + v[u].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}
// a 4:1 "copy" with the pyramid's byte ratio (read 4 bytes, write 1): the level-0 pass's own ceiling
template <int U>
__global__ __launch_bounds__(256) void k_read4_write1(const uint4* __restrict__ src, uint32_t* __restrict__ dst, size_t n16) {
    const size_t stride = (size_t)gridDim.x * 256 * U;
    for (size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x; i < n16; i += stride) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = i + 256 * u < n16 ? src[i + 256 * u] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < U; ++u) if (i + 256 * u < n16) dst[i + 256 * u] = v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
}

// ---- the wave walker --------------------------------------------------------------------------------------------
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as16(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t as32(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }

// units = (image, strip, chunk of CH output rows); wave g of G takes the contiguous range [U g / G, U (g + 1) / G) and
// walks it (consecutive chunks of one strip continue without re-reading).  A strip = m output lanes (lanes 1 .. m, 8
// output columns each) plus halo lanes 0 and m + 1 (they load and sum their columns, store nothing).
template <int PF>
__global__ __launch_bounds__(256) void k_pyr_walk(const uint8_t* __restrict__ src0, int sw, int sh, int sp,
                                                  size_t s_img, uint8_t* __restrict__ dst0, int dw, int dh, int dp,
                                                  size_t d_img, int nimg, int m, int CH) {
    const int lane = threadIdx.x & 63;
    const int ns = (dw + 8 * m - 1) / (8 * m), chunks = (dh + CH - 1) / CH;
    const long U = (long)ns * chunks * nimg;
    const int G = gridDim.x * 4;
    const int g = xcd_remap(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6);
    long u = U * g / G;
    const long u_end = U * (g + 1) / G;
    while (u < u_end) {
        const long strip = u / chunks;
        const int c0 = (int)(u - strip * chunks);
        const int run = (int)min(u_end - u, (long)(chunks - c0));
        u += run;
        const int bx = (int)(strip % ns), bz = (int)(strip / ns);
        const uint8_t* src = src0 + (size_t)bz * s_img;
        uint8_t* dst = dst0 + (size_t)bz * d_img;
        const int oy_b = c0 * CH, oy_e = min(dh, (c0 + run) * CH);
        const int cx = 16 * (m * bx + lane - 1);               // this lane's first input column
        const bool ld = lane <= m + 1 && cx >= 0 && cx < sp;
        const bool out_lane = lane >= 1 && lane <= m && cx < sw;
        const int ox = cx >> 1;
        // borders (reflect-101): only output column 0 reads columns -2, -1 (its left pair becomes (col 2, col 1)), and
        // only the last output column dw - 1 reads columns >= sw -- it is lane `rlane`'s output jl (uniform), with
        // weights folded onto the columns the reflection maps to: sw even: [1 4 6 4 | +1 on col sw - 2]; sw odd:
        // cols sw - 3, sw - 2, sw - 1 weighted 2, 8, 6
        const bool left_lane = cx == 0;
        const int xl = dw - 1, jl = xl & 7;
        const bool rwave = xl >= 8 * m * bx && xl < 8 * m * (bx + 1);
        const bool rlane = out_lane && (xl >> 3) == (ox >> 3);
        const bool sw_odd = sw & 1;
        auto srow = [&](int y) {
            y = y < 0 ? -y : y;
            y = y >= sh ? 2 * sh - 2 - y : y;
            return y < 0 ? 0 : (y >= sh ? sh - 1 : y);
        };
        const int r_first = 2 * oy_b - 2, r_last = 2 * oy_e;
        auto load_row = [&](int y) -> uint4 {
            uint4 v = make_uint4(0, 0, 0, 0);
            if (y <= r_last) {   // (uniform) the row's offset in SGPRs, the lane's column in a VGPR
                const uint8_t* rp = src + (size_t)__builtin_amdgcn_readfirstlane(srow(y)) * sp;
                if (ld) v = *(const uint4*)(rp + cx);
            }
            return v;
        };
        u16x2 P[8], Q[8], R[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) P[k] = Q[k] = R[k] = u16x2{0, 0};
        uint4 buf[PF];
#pragma unroll
        for (int i = 0; i < PF; ++i) buf[i] = load_row(r_first + i);
        auto emit = [&](int oy) {   // P holds the vertical sums of output row oy at columns cx .. cx + 15
            uint32_t L = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)as32(P[7]), 0x138, 0xf, 0xf, false);
            const uint32_t Rr = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)as32(P[0]), 0x130, 0xf, 0xf, false);
            if (left_lane) L = __builtin_amdgcn_perm(as32(P[0]), as32(P[1]), 0x07060100u);
            uint32_t o[8];
            if (!rwave) {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const u16x2 pl = j == 0 ? as16(L) : P[j - 1];
                    const u16x2 pr = j == 7 ? as16(Rr) : P[j + 1];
                    uint32_t a = __builtin_amdgcn_udot2(pl, u16x2{1, 4}, 128u, false);
                    a = __builtin_amdgcn_udot2(P[j], u16x2{6, 4}, a, false);
                    o[j] = a + pr.x;
                }
            } else {   // the strip holding the last output column (uniform branch)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const u16x2 pl = j == 0 ? as16(L) : P[j - 1];
                    const u16x2 pr = j == 7 ? as16(Rr) : P[j + 1];
                    u16x2 k1 = {1, 4}, k2 = {6, 4};
                    uint32_t last = pr.x;
                    if (j == jl && rlane) {
                        if (sw_odd) { k1 = u16x2{2, 8}; k2 = u16x2{6, 0}; last = 0; }
                        else last = P[j].x;
                    }
                    uint32_t a = __builtin_amdgcn_udot2(pl, k1, 128u, false);
                    a = __builtin_amdgcn_udot2(P[j], k2, a, false);
                    o[j] = a + last;
                }
            }
            if (!out_lane) return;
            const uint32_t lo = __builtin_amdgcn_perm(__builtin_amdgcn_perm(o[3], o[2], 0x0c0c0501u),
                                                      __builtin_amdgcn_perm(o[1], o[0], 0x0c0c0501u), 0x05040100u);
            const uint32_t hi = __builtin_amdgcn_perm(__builtin_amdgcn_perm(o[7], o[6], 0x0c0c0501u),
                                                      __builtin_amdgcn_perm(o[5], o[4], 0x0c0c0501u), 0x05040100u);
            uint8_t* d = dst + (size_t)oy * dp + ox;
            if (ox + 8 <= dw) {
                *(uint2*)d = make_uint2(lo, hi);
            } else {
                for (int j = 0; j < dw - ox; ++j) d[j] = (uint8_t)((j < 4 ? lo : hi) >> (8 * (j & 3)));
            }
        };
        int r = r_first;
        while (r <= r_last) {
#pragma unroll
            for (int i = 0; i < PF; ++i) {
                if (r > r_last) break;
                const uint4 v = buf[i];
                buf[i] = load_row(r + PF);
                const uint32_t w[4] = {v.x, v.y, v.z, v.w};
                u16x2 vv[8];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    vv[2 * k] = as16(__builtin_amdgcn_perm(0u, w[k], 0x0c010c00u));
                    vv[2 * k + 1] = as16(__builtin_amdgcn_perm(0u, w[k], 0x0c030c02u));
                }
                if ((i & 1) == 0) {   // even row 2k: last tap of output k - 1, centre of k, first of k + 1
                    const int k = (r >> 1);
#pragma unroll
                    for (int q = 0; q < 8; ++q) P[q] += vv[q];
                    if (k - 1 >= oy_b) emit(k - 1);
#pragma unroll
                    for (int q = 0; q < 8; ++q) { Q[q] += vv[q] * (unsigned short)6; R[q] = vv[q]; }
                } else {              // odd row 2k + 1: outputs k and k + 1, weight 4 each
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        Q[q] += vv[q] * (unsigned short)4;
                        R[q] += vv[q] * (unsigned short)4;
                        P[q] = Q[q];
                        Q[q] = R[q];
                    }
                }
                ++r;
            }
        }
    }
}

void launch_pyr_walk(int pf, const uint8_t* src, int sw, int sh, int sp, size_t s_img, uint8_t* dst, int dw, int dh,
                     int dp, size_t d_img, int nimg, int m, int ch, int waves) {
    const int ns = (dw + 8 * m - 1) / (8 * m), chunks = (dh + ch - 1) / ch;
    const long U = (long)ns * chunks * nimg;
    const long w = std::min((long)waves, U);
    const int blocks = (int)((w + 3) / 4);
    if (pf == 8)
        hipLaunchKernelGGL(k_pyr_walk<8>, dim3(blocks), dim3(256), 0, 0, src, sw, sh, sp, s_img, dst, dw, dh, dp, d_img, nimg, m, ch);
    else if (pf == 4)
        hipLaunchKernelGGL(k_pyr_walk<4>, dim3(blocks), dim3(256), 0, 0, src, sw, sh, sp, s_img, dst, dw, dh, dp, d_img, nimg, m, ch);
    else
        hipLaunchKernelGGL(k_pyr_walk<6>, dim3(blocks), dim3(256), 0, 0, src, sw, sh, sp, s_img, dst, dw, dh, dp, d_img, nimg, m, ch);
}

__global__ void k_fill(uint8_t* p, size_t n, uint32_t seed) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
        p[i] = (uint8_t)(h >> 7);
    }
}

int main(int argc, char** argv) {
    const int nsrc = argc > 1 ? atoi(argv[1]) : 43;
    const int reps = 20;
    auto timeit = [&](auto fn, const char* name, double bytes) {
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        fn();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) fn();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1000.0 / reps;
        printf("%-44s %8.1f us  %7.0f GB/s\n", name, us, bytes / us / 1e3);
        return us;
    };
    // ceilings on 512 MiB (twice the Infinity Cache)
    {
        const size_t bytes = (size_t)512 << 20, n16 = bytes / 16;
        uint8_t *a, *b; uint32_t* o;
        CK(hipMalloc(&a, bytes)); CK(hipMalloc(&b, bytes)); CK(hipMalloc(&o, 64));
        hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, a, bytes, 1u);
        for (int grid : {1024, 2048, 4096, 8192, 16384}) {
            char name[64];
            snprintf(name, sizeof name, "copy4 U1 g%d (r+w)", grid);
            timeit([&] { hipLaunchKernelGGL(k_copy4<1>, dim3(grid), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, n16); }, name, 2.0 * bytes);
            snprintf(name, sizeof name, "copy4 U4 g%d (r+w)", grid);
            timeit([&] { hipLaunchKernelGGL(k_copy4<4>, dim3(grid), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, n16); }, name, 2.0 * bytes);
        }
        for (int grid : {2048, 8192}) {
            char name[64];
            snprintf(name, sizeof name, "read4 U4 g%d", grid);
            timeit([&] { hipLaunchKernelGGL(k_read4<4>, dim3(grid), dim3(256), 0, 0, (const uint4*)a, n16, o); }, name, (double)bytes);
            snprintf(name, sizeof name, "read4 write1 U4 g%d (r+w)", grid);
            timeit([&] { hipLaunchKernelGGL(k_read4_write1<4>, dim3(grid), dim3(256), 0, 0, (const uint4*)a, (uint32_t*)b, n16); }, name, 1.25 * bytes);
        }
        CK(hipFree(a)); CK(hipFree(b)); CK(hipFree(o));
    }
    // level 0 -> 1 of nsrc Src7-sized sources, the engine's layout (pitch round_up(w + 4, 64), one spare row)
    const int W = 4024, H = 3036, dw = (W + 1) / 2, dh = (H + 1) / 2;
    const int sp = (W + 4 + 63) & ~63, dp = (dw + 4 + 63) & ~63;
    const size_t s_img = (size_t)sp * (H + 1), d_img = (size_t)dp * (dh + 1);
    uint8_t *s, *d0, *d1;
    CK(hipMalloc(&s, s_img * nsrc)); CK(hipMalloc(&d0, d_img * nsrc)); CK(hipMalloc(&d1, d_img * nsrc));
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, s, s_img * nsrc, 7u);
    CK(hipMemset(d0, 0, d_img * nsrc));
    const double bytes = (double)nsrc * ((double)W * H + (double)dw * dh);
    printf("level 0 -> 1, %d sources: %.1f MB algorithmic\n", nsrc, bytes / 1e6);
    timeit([&] { launch_pyr_down(s, W, H, sp, s_img, d0, dw, dh, dp, d_img, nsrc, 0); }, "product k_pyr_down_s", bytes);
    std::vector<uint8_t> ref(d_img * nsrc), got(d_img * nsrc);
    CK(hipMemcpy(ref.data(), d0, ref.size(), hipMemcpyDeviceToHost));
    for (int pf : {4, 6, 8})
        for (int m : {48, 51, 62})
            for (int ch : {16, 32})
                for (int waves : {4096, 8192, 16384}) {
                    CK(hipMemset(d1, 0, d_img * nsrc));
                    char name[96];
                    snprintf(name, sizeof name, "walk pf%d m%d ch%d waves%d", pf, m, ch, waves);
                    timeit([&] { launch_pyr_walk(pf, s, W, H, sp, s_img, d1, dw, dh, dp, d_img, nsrc, m, ch, waves); }, name, bytes);
                    CK(hipMemcpy(got.data(), d1, got.size(), hipMemcpyDeviceToHost));
                    size_t bad = 0;
                    for (int k = 0; k < nsrc; ++k)
                        for (int y = 0; y < dh; ++y)
                            for (int x = 0; x < dw; ++x)
                                bad += ref[k * d_img + (size_t)y * dp + x] != got[k * d_img + (size_t)y * dp + x];
                    if (bad) printf("   MISMATCH: %zu bytes differ\n", bad);
                }
    // small odd sizes against the product (borders, partial strips)
    for (int t = 0; t < 12; ++t) {
        const int w = 5 + (t * 397) % 1500, h = 3 + (t * 211) % 700;
        const int w1 = (w + 1) / 2, h1 = (h + 1) / 2, p = (w + 4 + 63) & ~63, p1 = (w1 + 4 + 63) & ~63;
        const size_t si = (size_t)p * (h + 1), di = (size_t)p1 * (h1 + 1);
        hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, s, si * 2, 11u + t);
        CK(hipMemset(d0, 0, di * 2)); CK(hipMemset(d1, 0, di * 2));
        launch_pyr_down(s, w, h, p, si, d0, w1, h1, p1, di, 2, 0);
        launch_pyr_walk(8, s, w, h, p, si, d1, w1, h1, p1, di, 2, 51, 16, 8192);
        CK(hipDeviceSynchronize());
        std::vector<uint8_t> a(di * 2), b(di * 2);
        CK(hipMemcpy(a.data(), d0, a.size(), hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), d1, b.size(), hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (int k = 0; k < 2; ++k)
            for (int y = 0; y < h1; ++y)
                for (int x = 0; x < w1; ++x) bad += a[k * di + (size_t)y * p1 + x] != b[k * di + (size_t)y * p1 + x];
        printf("check %dx%d: %s\n", w, h, bad ? "FAIL" : "OK");
    }
    return 0;
}
