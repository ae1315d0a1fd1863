// fpm_kernels.hip — MI355X (gfx950) kernels of the NCC template-matching hot path.
//
//   K1  k_pyr_down_s  cv::pyrDown, one level per launch    (TemplateMatcher.cpp:55, :124)
//       k_pyr_down2   two levels per launch (small inputs)
//   K2  k_warp        cv::warpAffine INTER_LINEAR          (TemplateMatcher.cpp:175, :1089)
//   K3+K4 k_ncc_map   matchTemplate(TM_CCORR) + CCOEFF_Denominator   (:177 -> :514, :523, :527-598)
//   K5  k_nms         minMaxLoc + getNextMaxLoc / s_BlockMax (:179-210, :1196-1221, DataStructures.h:118-246)
//       k_cand_init   top candidate -> ptLT                (:262-266)
//   K6-K8 refinement  getRotatedROI + IM_Conv_SIMD fold + CCOEFF_Denominator + minMaxLoc + 3x3
//                     (:309-328, :461-512, :527-598): k_roi_tables / k_roi_warp / k_roi_corr (i8 MFMA) / k_roi_eval
//                     for large templates, k_roi_small (the ROI sampled into LDS, never stored) for small ones
//       k_cand_step   best-of-3 / early break / back-mapping (:331-366) after k_roi_small (small batches: after
//                     the last of consecutive small layers, the earlier steps in k_roi_small's prologue);
//                     k_cand_step_tab / k_roi_eval also write the next layer's k_roi_tables output (RoiArgs::nt_tab)
//       k_overlap_pairs filterWithRotatedRect's pair tests (:1133-1194), decisions replayed on the host
//
// Numerics contract: built with -ffp-contract=off, no fast-math; integer sums are exact; the per-row
// int32 -> f32 fold is sequential in template-row order; the normalisation is IEEE f64 in the reference's
// operation order.  Results are bit-identical to oracle/fpm_oracle.cpp.
#include <float.h>
#include <stdio.h>
#include <stdlib.h>
#include <limits.h>

#include <map>
#include <mutex>
#include <type_traits>
#include <utility>

#include "fpm_kernels.h"
#include "fpm_rrect.h"

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) is per device: remember, per (device, kernel), the largest dynamic
// LDS already allowed, under a mutex (contexts on several devices / host threads launch concurrently)
static void ensure_lds_attr(const void* fn, size_t bytes) {
    if (bytes <= 65536) return;
    int dev = 0;
    (void)hipGetDevice(&dev);
    static std::mutex mu;
    static std::map<std::pair<int, const void*>, size_t> done;
    std::lock_guard<std::mutex> lock(mu);
    size_t& cur = done[std::make_pair(dev, fn)];
    if (bytes <= cur) return;
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    cur = bytes;
}

namespace fpm {

__device__ __forceinline__ int rint_i(double v) { return (int)__builtin_rint(v); }
__device__ __forceinline__ int sat_s16(int v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }
__device__ __forceinline__ int reflect101(int p, int n) {
    if (n == 1) return 0;
    while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
    return p;
}
__device__ __forceinline__ double dmax0(double a) { return a < 0.0 ? 0.0 : a; }     // std::max(a, 0.0)
__device__ __forceinline__ double dmin(double a, double b) { return b < a ? b : a; }  // std::min(a, b)

// One bilinear tap set of cv::remap (remapBilinear<FixedPtCast<int,uchar,15>>), BORDER_CONSTANT = cval.
// X, Y are the fixed-point coordinates at INTER_BITS precision: (X0 + adelta) >> (AB_BITS - INTER_BITS).
__device__ __forceinline__ int warp_tap(const uint8_t* __restrict__ src, int sw, int sh, int sp, int X, int Y,
                                        int cval) {
    const int sx = sat_s16(X >> kInterBits), sy = sat_s16(Y >> kInterBits);
    const int fx = X & (kInterTab - 1), fy = Y & (kInterTab - 1);
    const int w0 = (kInterTab - fy) * (kInterTab - fx) * 32, w1 = (kInterTab - fy) * fx * 32;
    const int w2 = fy * (kInterTab - fx) * 32, w3 = fy * fx * 32;
    int v0, v1, v2, v3;
    if ((unsigned)sx < (unsigned)(sw > 1 ? sw - 1 : 0) && (unsigned)sy < (unsigned)(sh > 1 ? sh - 1 : 0)) {
        const uint8_t* p = src + (size_t)sy * sp + sx;
        v0 = p[0]; v1 = p[1]; v2 = p[sp]; v3 = p[sp + 1];
    } else if (sx >= sw || sx + 1 < 0 || sy >= sh || sy + 1 < 0) {
        return cval;
    } else {
        const bool x0 = sx >= 0 && sx < sw, x1 = sx + 1 >= 0 && sx + 1 < sw;
        const bool y0 = sy >= 0 && sy < sh, y1 = sy + 1 >= 0 && sy + 1 < sh;
        const uint8_t* r0 = src + (size_t)sy * sp;
        const uint8_t* r1 = r0 + sp;
        v0 = x0 && y0 ? r0[sx] : cval;
        v1 = x1 && y0 ? r0[sx + 1] : cval;
        v2 = x0 && y1 ? r1[sx] : cval;
        v3 = x1 && y1 ? r1[sx + 1] : cval;
    }
    return (v0 * w0 + v1 * w1 + v2 * w2 + v3 * w3 + (1 << 14)) >> 15;
}

// CCOEFF_Denominator's per-position body (TemplateMatcher.cpp:567-595).
__device__ __forceinline__ float ccoeff(double num, double wsum, double wsq, double mean0, double tnorm,
                                        double inv_area) {
    double wndMean2 = 0, wndSum2 = 0, t;
    t = wsum;
    wndMean2 += t * t;
    num -= t * mean0;
    wndMean2 *= inv_area;
    t = wsq;
    wndSum2 += t;
    const double diff2 = dmax0(wndSum2 - wndMean2);
    if (diff2 <= dmin(0.5, (double)(10 * FLT_EPSILON) * wndSum2))
        t = 0;
    else
        t = __builtin_sqrt(diff2) * tnorm;
    if (__builtin_fabs(num) < t)
        num /= t;
    else if (__builtin_fabs(num) < t * 1.125)
        num = num > 0 ? 1 : -1;
    else
        num = 0;
    return (float)num;
}

// ============================================================================================== K1
// pyrDown, LDS-tiled: a 256-thread workgroup produces a 128 x 32 output tile.  Its 288 x 68 input tile (source
// columns 2*ox0-16 .. +287, rows 2*oy0-2 .. +67, rows reflected at load time) is fetched with 16-byte loads that
// are all issued before the first use; columns outside the image are then patched in LDS with reflect-101.
// Horizontal [1 4 6 4 1]: h = dot4(0x04060401, 4 bytes) + 5th byte with v_dot4_u32_u8; vertical sum of 5 rows,
// (v + 128) >> 8, four output bytes per dword store.  Exact integer arithmetic.
// XCD-aware work placement (cdna_hip_programming.md T1; a speed choice only, never a correctness one): blocks that
// share an XCD (the same blockIdx % 8 group) take neighbouring work units, so the source lines that neighbouring
// units share are fetched into one L2 instead of up to eight.
// xcd_remap: bijection of [0, n) placing each group's blocks on one contiguous range of virtual ids.
__device__ __forceinline__ int xcd_remap(int b, int n) {
    const int q = n >> 3, r = n & 7, x = b & 7;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}
// xcd_split: the n work units of a 1-D grid-stride loop cut into one contiguous range per group, in proportion to the
// group's block count; this block is block k of nk in its group.
struct XcdSplit { int lo, hi, k, nk; };
__device__ __forceinline__ XcdSplit xcd_split(int n) {
    const int G = gridDim.x, b = blockIdx.x, x = b & 7, q = G >> 3, r = G & 7;
    const int nk = q + (x < r ? 1 : 0);
    const int first = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;   // group's first virtual block
    XcdSplit s;
    s.lo = (int)((int64_t)n * first / G);
    s.hi = (int)((int64_t)n * (first + nk) / G);
    s.k = b >> 3;
    s.nk = nk;
    return s;
}


constexpr int PD_OW = 128, PD_OH = 32;
constexpr int PD_IW = 2 * PD_OW + 32, PD_IH = 2 * PD_OH + 4;   // 288 x 68 bytes
constexpr uint32_t PD_K = 0x04060401u;                         // bytes {1, 4, 6, 4}

// ABL (profiling builds only): 1 = stop after the loads, 2 = after the LDS tile, 3 = after the horizontal pass
template <int ABL>
__global__ __launch_bounds__(256) void k_pyr_down(const uint8_t* __restrict__ src, int sw, int sh, int sp,
                                                  size_t s_img, uint8_t* __restrict__ dst, int dw, int dh,
                                                  int dp, size_t d_img) {
    __shared__ __attribute__((aligned(16))) uint8_t tin[PD_IH][PD_IW];
    __shared__ __attribute__((aligned(16))) uint16_t hs[PD_IH][PD_OW];
    // tiles in row-major order per image, XCD groups on contiguous tile ranges (horizontal neighbours share the
    // 16-byte halo columns' cache lines)
    const int gx = gridDim.x, gy = gridDim.y;
    const int t = xcd_remap(blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z), gx * gy * gridDim.z);
    const int bx = t % gx, byz = t / gx, by = byz % gy, bz = byz / gy;
    src += (size_t)bz * s_img;
    dst += (size_t)bz * d_img;
    const int tid = threadIdx.x;
    const int ox0 = bx * PD_OW, oy0 = by * PD_OH;
    const int ix0 = 2 * ox0 - 16;   // tin column 0 <-> source column ix0 (16-byte aligned)
    const int iy0 = 2 * oy0 - 2;    // tin row 0    <-> source row iy0 (reflected)
    constexpr int Q = PD_IW / 16;   // 18 uint4 per row
    constexpr int NLD = (PD_IH * Q + 255) / 256;
    // rows: one reflection covers every row an output needs (-2 .. sh+1); rows past that are clamped (unused)
    auto srow = [&](int r) {
        int y = iy0 + r;
        y = y < 0 ? -y : y;
        y = y >= sh ? 2 * sh - 2 - y : y;
        return y < 0 ? 0 : (y >= sh ? sh - 1 : y);
    };
    uint4 v[NLD];
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
        const int i = tid + 256 * k;
        const int r = i / Q, c = i - r * Q;
        const int x = ix0 + 16 * c;
        v[k] = make_uint4(0, 0, 0, 0);
        if (i < PD_IH * Q && x >= 0 && x + 16 <= sp) v[k] = *(const uint4*)(src + (size_t)srow(r) * sp + x);
    }
    if (ABL == 1) {
        uint32_t x = 0;
        for (int k = 0; k < NLD; ++k) x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
        if (x == 0x9e3779b9u) dst[tid] = (uint8_t)x;
        return;
    }
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
        const int i = tid + 256 * k;
        if (i < PD_IH * Q) {
            const int r = i / Q, c = i - r * Q;
            *(uint4*)&tin[r][16 * c] = v[k];
        }
    }
    // columns outside [0, sw) that an output of this tile reads (at most 2 on each side): reflect-101
    const int xlo = 2 * ox0 - 2, xhi = min(2 * (ox0 + PD_OW - 1) + 2, 2 * (dw - 1) + 2);
    if (xlo < 0 || xhi >= sw) {          // uniform per workgroup
        __syncthreads();                 // the 16-byte tile stores above cover the patched bytes
        for (int i = tid; i < PD_IH * 4; i += 256) {
            const int r = i >> 2, k = i & 3;
            const int x = k < 2 ? xlo + k : xhi - (k - 2);   // xlo, xlo+1, xhi, xhi-1
            if ((x < 0 && k < 2) || (x >= sw && k >= 2))
                tin[r][x - ix0] = src[(size_t)srow(r) * sp + reflect101(x, sw)];
        }
    }
    __syncthreads();
    if (ABL == 2) { if (tin[tid & 63][tid >> 2] == 0x5a && tid == 999) dst[0] = 1; return; }
    // horizontal: 4 consecutive outputs per item, tin columns 2*oc + 14 .. 2*oc + 24
    constexpr int NH = PD_IH * (PD_OW / 4);
#pragma unroll
    for (int k = 0; k < (NH + 255) / 256; ++k) {
        const int i = tid + 256 * k;
        if (i >= NH) break;
        const int r = i / (PD_OW / 4), g = i - r * (PD_OW / 4);
        const uint32_t* w = (const uint32_t*)&tin[r][8 * g + 12];   // bytes 8g+12 .. 8g+27
        const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3];
        // output 4g+j uses tin bytes 8g + 2j + 14 .. +18  (= w-relative 2j + 2 .. 2j + 6)
        const uint32_t h0 = __builtin_amdgcn_udot4(PD_K, __builtin_amdgcn_alignbyte(w1, w0, 2), 0, false) + ((w1 >> 16) & 0xff);
        const uint32_t h1 = __builtin_amdgcn_udot4(PD_K, w1, 0, false) + (w2 & 0xff);
        const uint32_t h2 = __builtin_amdgcn_udot4(PD_K, __builtin_amdgcn_alignbyte(w2, w1, 2), 0, false) + ((w2 >> 16) & 0xff);
        const uint32_t h3 = __builtin_amdgcn_udot4(PD_K, w2, 0, false) + (w3 & 0xff);
        uint2 o;
        o.x = h0 | (h1 << 16);
        o.y = h2 | (h3 << 16);
        *(uint2*)&hs[r][4 * g] = o;
    }
    __syncthreads();
    if (ABL == 3) { if (hs[tid & 63][tid >> 1] == 0x5a5a && tid == 999) dst[0] = 1; return; }
    // vertical: 4 consecutive outputs of one row per item
#pragma unroll
    for (int k = 0; k < PD_OH * (PD_OW / 4) / 256; ++k) {
        const int i = tid + 256 * k;
        const int orow = i / (PD_OW / 4), g = i - orow * (PD_OW / 4);
        const int oy = oy0 + orow, ox = ox0 + 4 * g;
        if (oy >= dh || ox >= dw) continue;
        uint32_t acc[4] = {128, 128, 128, 128};
        const int kw[5] = {1, 4, 6, 4, 1};
#pragma unroll
        for (int t = 0; t < 5; ++t) {
            const uint2 q = *(const uint2*)&hs[2 * orow + t][4 * g];
            acc[0] += kw[t] * (q.x & 0xffff); acc[1] += kw[t] * (q.x >> 16);
            acc[2] += kw[t] * (q.y & 0xffff); acc[3] += kw[t] * (q.y >> 16);
        }
        uint8_t* d = dst + (size_t)oy * dp + ox;
        if (ox + 4 <= dw) {
            *(uint32_t*)d = (acc[0] >> 8) | ((acc[1] >> 8) << 8) | ((acc[2] >> 8) << 16) | ((acc[3] >> 8) << 24);
        } else {
            for (int j = 0; j < dw - ox; ++j) d[j] = (uint8_t)(acc[j] >> 8);
        }
    }
}

// ---- K1, streaming form (the product's): one workgroup = a strip of PD_OW output columns x a run of output
// rows, walked down in chunks of PD_OH output rows.  The 4 input rows two chunks share are carried as horizontal
// sums (no re-read), and the next chunk's 64 input rows are loaded into registers while the current chunk is
// filtered and stored, so every workgroup keeps its loads in flight for its whole life instead of one burst per
// tile (the one-tile form above reaches 3.2-4.2 TB/s: its workgroups wait for their single burst).  Same integer
// arithmetic as k_pyr_down, exact.
typedef unsigned short fpm_u16x2 __attribute__((ext_vector_type(2)));

// OH: output rows per chunk (window 2 OH + 4 input rows; 16-byte loads per thread for it: 5 at OH 32, 3 at OH 16)
template <int OH>
__global__ __launch_bounds__(256) void k_pyr_down_s(const uint8_t* __restrict__ src0, int sw, int sh, int sp,
                                                    size_t s_img, uint8_t* __restrict__ dst0, int dw, int dh,
                                                    int dp, size_t d_img, int nimg, int32_t* zero, int nzero) {
    constexpr int IH = 2 * OH + 4;
    constexpr int PS_NL = (IH * (PD_IW / 16) + 255) / 256;
    __shared__ __attribute__((aligned(16))) uint8_t tin[IH][PD_IW];
    if (blockIdx.x == 0)
        for (int i = threadIdx.x; i < nzero; i += 256) zero[i] = 0;
    __shared__ __attribute__((aligned(16))) uint16_t hs[IH][PD_OW];
    // work units = (image, strip, chunk) in row-major order; workgroup w takes the contiguous range
    // [U*w/G, U*(w+1)/G) (equal shares: no tail round of a few workgroups), split where it crosses a strip; XCD
    // groups take contiguous ranges of workgroups (neighbouring strips share the halo columns' lines)
    const int gx = (dw + PD_OW - 1) / PD_OW, chunks = (dh + OH - 1) / OH;
    const long U = (long)gx * chunks * nimg;
    const int w = xcd_remap(blockIdx.x, gridDim.x);
    long u = U * w / gridDim.x;
    const long u_end = U * (w + 1) / gridDim.x;
    const int tid = threadIdx.x;
    while (u < u_end) {
        const long strip = u / chunks;
        const int c0 = (int)(u - strip * chunks);
        const int run = (int)min(u_end - u, (long)(chunks - c0));
        u += run;
        const int bx = (int)(strip % gx), bz = (int)(strip / gx);
        const uint8_t* src = src0 + (size_t)bz * s_img;
        uint8_t* dst = dst0 + (size_t)bz * d_img;
        const int ox0 = bx * PD_OW;
        const int oy_begin = c0 * OH, oy_end = min(dh, (c0 + run) * OH);
        __syncthreads();   // the previous run is done with tin / hs
        const int ix0 = 2 * ox0 - 16;     // tin column 0 <-> source column ix0 (16-byte aligned)
        constexpr int Q = PD_IW / 16;     // 18 uint4 per row
        auto srow = [&](int y) {          // one reflection covers every row an output needs (-2 .. sh+1)
            y = y < 0 ? -y : y;
            y = y >= sh ? 2 * sh - 2 - y : y;
            return y < 0 ? 0 : (y >= sh ? sh - 1 : y);
        };
        uint4 v[PS_NL];
        // window rows [roff, roff + nrows) <- input rows iy .. iy + nrows - 1, element i = tid + 256k -> (i / Q, i % Q)
        auto issue = [&](int iy, int nrows) {
#pragma unroll
            for (int k = 0; k < PS_NL; ++k) {
                const int i = tid + 256 * k;
                const int r = i / Q, c = i - r * Q;
                const int x = ix0 + 16 * c;
                v[k] = make_uint4(0, 0, 0, 0);
                if (r < nrows && x >= 0 && x + 16 <= sp) v[k] = *(const uint4*)(src + (size_t)srow(iy + r) * sp + x);
            }
        };
        auto commit = [&](int roff, int nrows) {
#pragma unroll
            for (int k = 0; k < PS_NL; ++k) {
                const int i = tid + 256 * k;
                const int r = i / Q, c = i - r * Q;
                if (r < nrows) *(uint4*)&tin[roff + r][16 * c] = v[k];
            }
        };
        // columns outside [0, sw) that an output of this strip reads (at most 2 on each side): reflect-101
        const int xlo = 2 * ox0 - 2, xhi = min(2 * (ox0 + PD_OW - 1) + 2, 2 * (dw - 1) + 2);
        const bool edge = xlo < 0 || xhi >= sw;   // uniform per workgroup
        issue(2 * oy_begin - 2, IH);
        for (int oyc = oy_begin; oyc < oy_end; oyc += OH) {
            const bool first = oyc == oy_begin;
            const int roff = first ? 0 : 4, nrows = first ? IH : 2 * OH;
            const int iy = 2 * oyc - 2 + roff;
            commit(roff, nrows);
            if (edge) {
                __syncthreads();   // the 16-byte tile stores above cover the patched bytes
                for (int i = tid; i < nrows * 4; i += 256) {
                    const int r = i >> 2, k = i & 3;
                    const int x = k < 2 ? xlo + k : xhi - (k - 2);   // xlo, xlo+1, xhi, xhi-1
                    if ((x < 0 && k < 2) || (x >= sw && k >= 2))
                        tin[roff + r][x - ix0] = src[(size_t)srow(iy + r) * sp + reflect101(x, sw)];
                }
            }
            __syncthreads();
            // the next chunk's 64 new input rows (its window rows 4..67) are in flight while this chunk is filtered
            if (oyc + OH < oy_end) issue(2 * oyc + 2 * OH + 2, 2 * OH);
            // horizontal [1 4 6 4 1] of the new window rows: 4 consecutive outputs per item (as k_pyr_down; the 5th tap
            // enters the v_dot4 as its accumulator)
            const int nh = nrows * (PD_OW / 4);
            for (int i = tid; i < nh; i += 256) {
                const int r = roff + i / (PD_OW / 4), g = i % (PD_OW / 4);
                const uint32_t* w = (const uint32_t*)&tin[r][8 * g + 12];
                const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3];
                const uint32_t h0 = __builtin_amdgcn_udot4(PD_K, __builtin_amdgcn_alignbyte(w1, w0, 2), (w1 >> 16) & 0xff, false);
                const uint32_t h1 = __builtin_amdgcn_udot4(PD_K, w1, w2 & 0xff, false);
                const uint32_t h2 = __builtin_amdgcn_udot4(PD_K, __builtin_amdgcn_alignbyte(w2, w1, 2), (w2 >> 16) & 0xff, false);
                const uint32_t h3 = __builtin_amdgcn_udot4(PD_K, w2, w3 & 0xff, false);
                uint2 o;
                o.x = h0 | (h1 << 16);
                o.y = h2 | (h3 << 16);
                *(uint2*)&hs[r][4 * g] = o;
            }
            __syncthreads();
            // vertical: 4 consecutive outputs of one row per item, two per register in packed u16 arithmetic — exact:
            // a horizontal sum is <= 16 * 255, so 128 + sum_t k_t * h_t <= 65408 fits 16 bits, and (v >> 8) is the
            // half's high byte, gathered by one v_perm
#pragma unroll
            for (int k = 0; k < OH * (PD_OW / 4) / 256; ++k) {
                const int i = tid + 256 * k;
                const int orow = i / (PD_OW / 4), g = i - orow * (PD_OW / 4);
                const int oy = oyc + orow, ox = ox0 + 4 * g;
                if (oy >= oy_end || ox >= dw) continue;
                fpm_u16x2 a01 = {128, 128}, a23 = {128, 128};
                constexpr unsigned short kw[5] = {1, 4, 6, 4, 1};
#pragma unroll
                for (int tt = 0; tt < 5; ++tt) {
                    const uint2 q = *(const uint2*)&hs[2 * orow + tt][4 * g];
                    a01 += __builtin_bit_cast(fpm_u16x2, q.x) * kw[tt];
                    a23 += __builtin_bit_cast(fpm_u16x2, q.y) * kw[tt];
                }
                const uint32_t packed = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, a23),
                                                              __builtin_bit_cast(uint32_t, a01), 0x07050301u);
                uint8_t* d = dst + (size_t)oy * dp + ox;
                if (ox + 4 <= dw) {
                    *(uint32_t*)d = packed;
                } else {
                    for (int j = 0; j < dw - ox; ++j) d[j] = (uint8_t)(packed >> (8 * j));
                }
            }
            __syncthreads();
            // carry: window rows 2 OH .. 2 OH + 3 (input rows 2 * (oyc + OH) - 2 .. + 1) are the next window's rows 0..3
            ((uint32_t*)hs[tid >> 6])[tid & 63] = ((uint32_t*)hs[2 * OH + (tid >> 6)])[tid & 63];
            __syncthreads();
        }
    }
}

static const int kPyrWGs = [] {   // FPM_PYR_WGS: profiling override
    const char* e = getenv("FPM_PYR_WGS");
    return e && atoi(e) > 0 ? atoi(e) : 4096;
}();
static const int kPyrOH = [] {   // FPM_PYR_OH (16 or 32): profiling override of the chunk height
    const char* e = getenv("FPM_PYR_OH");
    return e && atoi(e) == 16 ? 16 : 32;
}();
void launch_pyr_down(const uint8_t* src, int sw, int sh, int sp, size_t s_img, uint8_t* dst, int dw, int dh,
                     int dp, size_t d_img, int nimg, hipStream_t st, int seg_chunks, int32_t* zero, int nzero) {
    // equal shares of the (image, strip, chunk) units over kPyrWGs workgroups (4 rounds of 4 per CU; measured
    // 2048 / 4096 / 8192: 37.1 / 35.7 / 36.0 µs per launch averaged over the Src7 levels), or
    // seg_chunks units each
    if (dw <= 0 || dh <= 0 || nimg <= 0) return;
    const int oh = kPyrOH;
    const int gx = (dw + PD_OW - 1) / PD_OW, chunks = (dh + oh - 1) / oh;
    const long units = (long)gx * chunks * nimg;
    const long g = seg_chunks > 0 ? (units + seg_chunks - 1) / seg_chunks : std::min(units, (long)kPyrWGs);
    if (oh == 16)
        hipLaunchKernelGGL(k_pyr_down_s<16>, dim3((unsigned)g), dim3(256), 0, st, src, sw, sh, sp, s_img, dst, dw, dh,
                           dp, d_img, nimg, zero, nzero);
    else
        hipLaunchKernelGGL(k_pyr_down_s<32>, dim3((unsigned)g), dim3(256), 0, st, src, sw, sh, sp, s_img, dst, dw, dh,
                           dp, d_img, nimg, zero, nzero);
}

// ---- K1, two levels per launch (round 4; the engine uses it where a level pair's input is small): a workgroup walks a
// strip of PD2_OWC columns of level l+2 down in chunks.  A chunk first filters PD2_OHB rows of level l+1 over the
// PD2_OWB columns around the ones the strip's level-(l+2) outputs read -- its own 2 PD2_OWC columns, stored to memory,
// plus halo columns on each side that the neighbouring strips own (4, of which 2 are read, so the own columns are whole
// dword groups) -- from a level-l window exactly as k_pyr_down_s does, and keeps them in an LDS ring after
// the 4 rows the previous chunk left there.  It then applies level l+1's own reflect-101 border to the ring (cv::pyrDown
// pads its input, so a level-(l+1) column or row outside the image is a copy of one of its pixels, not a filtered
// level-l value) and filters the PD2_OHB / 2 level-(l+2) rows the ring now completes.  Level l+1 is written once and
// never read back (the one-level kernel re-reads it for the next level), and a search's pyramid takes half the
// launches.  A run of chunks that does not start at the top of its strip first rebuilds the 4 ring rows the chunk
// above would have carried (a 76-row level-l window instead of 68).  Same integer arithmetic as k_pyr_down on both
// levels: exact.  The next chunk's 64 level-l rows are in flight while a chunk is filtered.
constexpr int PD2_OWC = 64;                       // level-(l+2) columns per strip
constexpr int PD2_OWB = 2 * PD2_OWC + 8;          // 136 level-(l+1) columns per strip: 4-column halos (2 read), so
constexpr int PD2_GB = PD2_OWB / 4;               // the own columns are groups 1 .. 32 of the 34 (dword stores)
constexpr int PD2_BP = 136;                       // ring row pitch (bytes) = level-(l+1) horizontal-sum pitch (u16)
// PD2_OHB: level-(l+1) rows per chunk (32: window 76 rows at a run start, 68 after it; ring 4 carried + 32 + 2 rows
// reflected past the bottom row)
template <int PD2_OHB>
__global__ __launch_bounds__(256) void k_pyr_down2(const uint8_t* __restrict__ src0, int sw, int sh, int sp,
                                                   size_t s_img, uint8_t* __restrict__ b0, int bw, int bh, int bpp,
                                                   size_t b_img, uint8_t* __restrict__ c0, int cw, int ch, int cpp,
                                                   size_t c_img, int nimg, int32_t* zero, int nzero) {
    constexpr int PD2_IH = 2 * (PD2_OHB + 4) + 4, PD2_RING = PD2_OHB + 6;
    __shared__ __attribute__((aligned(16))) uint8_t tin[PD2_IH][PD_IW];
    __shared__ __attribute__((aligned(16))) uint16_t hs[PD2_IH][PD2_BP];
    __shared__ __attribute__((aligned(16))) uint8_t ring[PD2_RING][PD2_BP];
    __shared__ __attribute__((aligned(16))) uint16_t hc[PD2_RING][PD2_OWC];
    if (blockIdx.x == 0)
        for (int i = threadIdx.x; i < nzero; i += 256) zero[i] = 0;
    // work units = (image, strip, chunk), contiguous ranges per workgroup, XCD groups on neighbouring ranges (as
    // k_pyr_down_s)
    const int gx = (cw + PD2_OWC - 1) / PD2_OWC, chunks = (bh + PD2_OHB - 1) / PD2_OHB;
    const long U = (long)gx * chunks * nimg;
    const int w = xcd_remap(blockIdx.x, gridDim.x);
    long u = U * w / gridDim.x;
    const long u_end = U * (w + 1) / gridDim.x;
    const int tid = threadIdx.x;
    constexpr int Q = PD_IW / 16;                    // 18 uint4 per window row
    constexpr int NL = (PD2_IH * Q + 255) / 256;     // 6 loads per thread for a 76-row window
    constexpr unsigned short kw[5] = {1, 4, 6, 4, 1};
    auto srow = [&](int y) {   // level-l rows: one reflection covers -2 .. sh + 1; rows past that are clamped (unused)
        y = y < 0 ? -y : y;
        y = y >= sh ? 2 * sh - 2 - y : y;
        return y < 0 ? 0 : (y >= sh ? sh - 1 : y);
    };
    while (u < u_end) {
        const long strip = u / chunks;
        const int k_begin = (int)(u - strip * chunks);
        const int k_end = k_begin + (int)min(u_end - u, (long)(chunks - k_begin));
        u += k_end - k_begin;
        const int sx = (int)(strip % gx), bz = (int)(strip / gx);
        const uint8_t* src = src0 + (size_t)bz * s_img;
        uint8_t* bdst = b0 + (size_t)bz * b_img;
        uint8_t* cdst = c0 + (size_t)bz * c_img;
        const int cx0 = sx * PD2_OWC;
        const int bx0 = 2 * cx0 - 4;   // ring column 0 <-> level-(l+1) column bx0
        const int ix0 = 4 * cx0 - 16;  // tin column 0 <-> level-l column ix0 (16-byte aligned)
        // level-l columns outside [0, sw) that the strip's in-image level-(l+1) columns read: reflect-101 patches
        const int xlo = 2 * max(bx0, 0) - 2, xhi = 2 * min(bx0 + PD2_OWB - 1, bw - 1) + 2;
        const bool edge = xlo < 0 || xhi >= sw;                      // uniform per workgroup
        const bool bedge = bx0 < 0 || bx0 + PD2_OWB > bw;            // level-(l+1) columns to reflect in the ring
        uint4 v[NL];
        auto issue = [&](int iy, int nrows) {   // window rows [.., + nrows) <- level-l rows iy ..
#pragma unroll
            for (int q = 0; q < NL; ++q) {
                const int i = tid + 256 * q;
                const int r = i / Q, c = i - r * Q;
                const int x = ix0 + 16 * c;
                v[q] = make_uint4(0, 0, 0, 0);
                if (r < nrows && x >= 0 && x + 16 <= sp) v[q] = *(const uint4*)(src + (size_t)srow(iy + r) * sp + x);
            }
        };
        __syncthreads();   // the previous run is done with the LDS
        // a run start: level-(l+1) rows 32 k - 4 .. 32 k + 31, i.e. level-l rows 64 k - 10 .. 64 k + 65
        issue(2 * (PD2_OHB * k_begin - 4) - 2, PD2_IH);
        for (int k = k_begin; k < k_end; ++k) {
            const bool start = k == k_begin;
            const int roff = start ? 0 : 4, nrows = start ? PD2_IH : 2 * PD2_OHB;
            const int by_first = start ? PD2_OHB * k - 4 : PD2_OHB * k;   // first level-(l+1) row filtered
            const int nb = PD2_OHB * (k + 1) - by_first;                   // 36 or 32 rows
            const int iy = 2 * by_first - 2 + roff;                        // level-l row of window row roff
            const int rb0 = PD2_OHB * k - 4;                               // level-(l+1) row of ring row 0
#pragma unroll
            for (int q = 0; q < NL; ++q) {
                const int i = tid + 256 * q;
                const int r = i / Q, c = i - r * Q;
                if (r < nrows) *(uint4*)&tin[roff + r][16 * c] = v[q];
            }
            if (edge) {
                __syncthreads();   // the 16-byte stores above cover the patched bytes
                for (int i = tid; i < nrows * 4; i += 256) {
                    const int r = i >> 2, q = i & 3;
                    const int x = q < 2 ? xlo + q : xhi - (q - 2);   // xlo, xlo + 1, xhi, xhi - 1
                    if ((x < 0 && q < 2) || (x >= sw && q >= 2))
                        tin[roff + r][x - ix0] = src[(size_t)srow(iy + r) * sp + reflect101(x, sw)];
                }
            }
            __syncthreads();
            if (k + 1 < k_end) issue(2 * PD2_OHB * (k + 1) + 2, 2 * PD2_OHB);
            // level l+1, horizontal [1 4 6 4 1] of the new window rows: ring column p = 4g + j reads level-l columns
            // 2 (bx0 + p) - 2 .. + 4 = tin bytes 8g + 2j + 6 .. + 10
            for (int i = tid; i < nrows * PD2_GB; i += 256) {
                const int r = roff + i / PD2_GB, g = i % PD2_GB;
                const uint32_t* wp = (const uint32_t*)&tin[r][8 * g + 4];
                const uint32_t w0 = wp[0], w1 = wp[1], w2 = wp[2], w3 = wp[3];
                const uint32_t h0 = __builtin_amdgcn_udot4(PD_K, __builtin_amdgcn_alignbyte(w1, w0, 2), (w1 >> 16) & 0xff, false);
                const uint32_t h1 = __builtin_amdgcn_udot4(PD_K, w1, w2 & 0xff, false);
                const uint32_t h2 = __builtin_amdgcn_udot4(PD_K, __builtin_amdgcn_alignbyte(w2, w1, 2), (w2 >> 16) & 0xff, false);
                const uint32_t h3 = __builtin_amdgcn_udot4(PD_K, w2, w3 & 0xff, false);
                uint2 o;
                o.x = h0 | (h1 << 16);
                o.y = h2 | (h3 << 16);
                *(uint2*)&hs[r][4 * g] = o;
            }
            __syncthreads();
            // level l+1, vertical: rows by_first .. + nb - 1 into ring rows by - rb0; the strip's own in-image columns
            // (ring columns 4 .. 2 PD2_OWC + 3, groups 1 .. 32) and rows (>= 32 k: the rebuilt carry rows belong to the
            // chunk above) go to memory as dwords
            for (int i = tid; i < nb * PD2_GB; i += 256) {
                const int orow = i / PD2_GB, g = i - orow * PD2_GB;
                fpm_u16x2 a01 = {128, 128}, a23 = {128, 128};
#pragma unroll
                for (int tt = 0; tt < 5; ++tt) {
                    const uint2 q = *(const uint2*)&hs[2 * orow + tt][4 * g];
                    a01 += __builtin_bit_cast(fpm_u16x2, q.x) * kw[tt];
                    a23 += __builtin_bit_cast(fpm_u16x2, q.y) * kw[tt];
                }
                const uint32_t packed = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, a23),
                                                              __builtin_bit_cast(uint32_t, a01), 0x07050301u);
                const int by = by_first + orow;
                *(uint32_t*)&ring[by - rb0][4 * g] = packed;
                if (by < PD2_OHB * k || by >= bh) continue;
                const int bx = bx0 + 4 * g;
                if (g < 1 || g > PD2_OWC / 2 || bx >= bw) continue;
                uint8_t* d = bdst + (size_t)by * bpp + bx;
                if (bx + 4 <= bw) {
                    *(uint32_t*)d = packed;
                } else {
                    for (int j = 0; j < bw - bx; ++j) d[j] = (uint8_t)(packed >> (8 * j));
                }
            }
            __syncthreads();
            // level l+1's reflect-101 border in the ring: rows -2, -1 (first chunk), bh, bh + 1 (last chunk; ring rows
            // <= 37), then columns -2, -1, bw, bw + 1 where they fall in the strip (corners from the reflected rows)
            const bool top = k == 0, bottom = k == chunks - 1;
            if (top || bottom) {
                for (int i = tid; i < 4 * PD2_OWB; i += 256) {
                    const int e = i / PD2_OWB, c = i - e * PD2_OWB;
                    if ((e < 2 && !top) || (e >= 2 && !bottom)) continue;
                    const int r = e < 2 ? e - 2 : bh + (e - 2);
                    ring[r - rb0][c] = ring[reflect101(r, bh) - rb0][c];
                }
                if (bedge) __syncthreads();
            }
            if (bedge) {
                for (int i = tid; i < PD2_RING * 4; i += 256) {
                    const int r = i >> 2, q = i & 3;
                    const int bx = q < 2 ? q - 2 : bw + (q - 2);
                    const int p = bx - bx0;
                    if (p >= 0 && p < PD2_OWB) ring[r][p] = ring[r][reflect101(bx, bw) - bx0];
                }
            }
            if (top || bottom || bedge) __syncthreads();
            // level l+2: the rows this chunk completes, [lo, hi): row c reads level-(l+1) rows 2c - 2 .. 2c + 2
            const int lo = top ? 0 : PD2_OHB / 2 * k - 1;
            const int hi = bottom ? ch : min(ch, PD2_OHB / 2 * (k + 1) - 1);
            const int r_lo = 2 * lo - 2 - rb0, nr = 2 * (hi - lo) + 3;   // ring rows read
            // horizontal: output cx0 + 4g + j reads ring columns 8g + 2j + 2 .. + 6
            for (int i = tid; i < nr * (PD2_OWC / 4); i += 256) {
                const int r = r_lo + i / (PD2_OWC / 4), g = i % (PD2_OWC / 4);
                const uint32_t* wp = (const uint32_t*)&ring[r][8 * g];
                const uint32_t w0 = wp[0], w1 = wp[1], w2 = wp[2], w3 = wp[3];
                const uint32_t h0 = __builtin_amdgcn_udot4(PD_K, __builtin_amdgcn_alignbyte(w1, w0, 2), (w1 >> 16) & 0xff, false);
                const uint32_t h1 = __builtin_amdgcn_udot4(PD_K, w1, w2 & 0xff, false);
                const uint32_t h2 = __builtin_amdgcn_udot4(PD_K, __builtin_amdgcn_alignbyte(w2, w1, 2), (w2 >> 16) & 0xff, false);
                const uint32_t h3 = __builtin_amdgcn_udot4(PD_K, w2, w3 & 0xff, false);
                uint2 o;
                o.x = h0 | (h1 << 16);
                o.y = h2 | (h3 << 16);
                *(uint2*)&hc[r][4 * g] = o;
            }
            __syncthreads();
            // carries for the next chunk (nothing reads them before the barrier below): ring rows 32 .. 35 (level-(l+1)
            // rows 32 k + 28 .. + 31) -> 0 .. 3, and the window's last 4 horizontal-sum rows (level-l rows 64 k + 62 ..
            // + 65) -> 0 .. 3
            for (int i = tid; i < 4 * (PD2_BP / 4); i += 256)
                ((uint32_t*)ring[i / (PD2_BP / 4)])[i % (PD2_BP / 4)] = ((uint32_t*)ring[PD2_OHB + i / (PD2_BP / 4)])[i % (PD2_BP / 4)];
            const int hlast = roff + nrows - 4;
            for (int i = tid; i < 4 * (PD2_BP / 2); i += 256)
                ((uint32_t*)hs[i / (PD2_BP / 2)])[i % (PD2_BP / 2)] = ((uint32_t*)hs[hlast + i / (PD2_BP / 2)])[i % (PD2_BP / 2)];
            // vertical: 4 consecutive outputs of one row per item
            for (int i = tid; i < (hi - lo) * (PD2_OWC / 4); i += 256) {
                const int crow = lo + i / (PD2_OWC / 4), g = i % (PD2_OWC / 4);
                const int cx = cx0 + 4 * g;
                if (cx >= cw) continue;
                const int r0 = 2 * crow - 2 - rb0;
                fpm_u16x2 a01 = {128, 128}, a23 = {128, 128};
#pragma unroll
                for (int tt = 0; tt < 5; ++tt) {
                    const uint2 q = *(const uint2*)&hc[r0 + tt][4 * g];
                    a01 += __builtin_bit_cast(fpm_u16x2, q.x) * kw[tt];
                    a23 += __builtin_bit_cast(fpm_u16x2, q.y) * kw[tt];
                }
                const uint32_t packed = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, a23),
                                                              __builtin_bit_cast(uint32_t, a01), 0x07050301u);
                uint8_t* d = cdst + (size_t)crow * cpp + cx;
                if (cx + 4 <= cw) {
                    *(uint32_t*)d = packed;
                } else {
                    for (int j = 0; j < cw - cx; ++j) d[j] = (uint8_t)(packed >> (8 * j));
                }
            }
            __syncthreads();
        }
    }
}

// FPM_PYR2_OH (16 or 32): profiling override of the two-level chunk height (32 is faster at the sizes the engine
// uses the kernel for: one Src7 source, levels 0-2, 11.3 vs 13.2 us; 16 at 43 sources, 217 vs 237 us)
// Unset: 32, or 16 where the 32-row chunks would give fewer units than the chip has CUs (the small level pairs of a
// lone search, whose workgroups each run one unit: half the rows on each workgroup's serial path).
static const int kPyr2OH = [] {
    const char* e = getenv("FPM_PYR2_OH");
    return e ? (atoi(e) == 16 ? 16 : 32) : 0;
}();
// one launch for pyramid levels l+1 and l+2 of nimg images (the units shared over kPyrWGs workgroups as
// launch_pyr_down; seg_chunks > 0: that many units per workgroup, so runs start mid-strip -- tests; chunk_rows 16 /
// 32 forces the level-(l+1) chunk height, 0 chooses it as above)
void launch_pyr_down2(const uint8_t* src, int sw, int sh, int sp, size_t s_img, uint8_t* bdst, int bw, int bh, int bp,
                      size_t b_img, uint8_t* cdst, int cw, int ch, int cp, size_t c_img, int nimg, hipStream_t st,
                      int seg_chunks, int32_t* zero, int nzero, int chunk_rows) {
    if (bw <= 0 || bh <= 0 || cw <= 0 || ch <= 0 || nimg <= 0) return;
    const int gx = (cw + PD2_OWC - 1) / PD2_OWC;
    // chunk_rows 16 / 32: forced (parity tests of both ring carries); else the env override or the rule above
    const int ohb = chunk_rows == 16 || chunk_rows == 32 ? chunk_rows
                    : kPyr2OH ? kPyr2OH : ((long)gx * ((bh + 31) / 32) * nimg < 256 ? 16 : 32);
    const int chunks = (bh + ohb - 1) / ohb;
    const long units = (long)gx * chunks * nimg;
    const long g = seg_chunks > 0 ? (units + seg_chunks - 1) / seg_chunks : std::min(units, (long)kPyrWGs);
    if (ohb == 16)
        hipLaunchKernelGGL(k_pyr_down2<16>, dim3((unsigned)g), dim3(256), 0, st, src, sw, sh, sp, s_img, bdst, bw, bh,
                           bp, b_img, cdst, cw, ch, cp, c_img, nimg, zero, nzero);
    else
        hipLaunchKernelGGL(k_pyr_down2<32>, dim3((unsigned)g), dim3(256), 0, st, src, sw, sh, sp, s_img, bdst, bw, bh,
                           bp, b_img, cdst, cw, ch, cp, c_img, nimg, zero, nzero);
}

// ============================================================================================== K2
__global__ __launch_bounds__(256) void k_warp(const WarpJob* __restrict__ jobs, int32_t* zero, int nzero) {
    if (blockIdx.x == 0 && blockIdx.y == 0)
        for (int i = threadIdx.x; i < nzero; i += 256) zero[i] = 0;
    const WarpJob& j = jobs[blockIdx.y];
    const int total = j.dw * j.dh;
    for (int idx = blockIdx.x * 256 + threadIdx.x; idx < total; idx += gridDim.x * 256) {
        const int y = idx / j.dw, x = idx - y * j.dw;
        const int X0 = rint_i((j.M[1] * y + j.M[2]) * kAbScale) + kRoundDelta;
        const int Y0 = rint_i((j.M[4] * y + j.M[5]) * kAbScale) + kRoundDelta;
        const int ad = rint_i(j.M[0] * x * kAbScale), bd = rint_i(j.M[3] * x * kAbScale);
        const int X = (X0 + ad) >> (kAbBits - kInterBits), Y = (Y0 + bd) >> (kAbBits - kInterBits);
        j.dst[(size_t)y * j.dp + x] = (uint8_t)warp_tap(j.src, j.sw, j.sh, j.sp, X, Y, j.border);
    }
}

void launch_warp(const WarpJob* jobs, int njobs, int max_pixels, hipStream_t st, int32_t* zero, int nzero) {
    if (njobs <= 0 || (max_pixels <= 0 && nzero <= 0)) return;
    int gx = max_pixels > 0 ? (max_pixels + 255) / 256 : 1;
    if (gx > 1024) gx = 1024;
    hipLaunchKernelGGL(k_warp, dim3(gx, njobs), dim3(256), 0, st, jobs, zero, nzero);
}

// ============================================================================================== K3+K4
__global__ __launch_bounds__(256) void k_ncc_map(const NccJob* __restrict__ jobs, int tmpl_in_lds) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const NccJob& j = jobs[blockIdx.y];
    const uint8_t* T = j.tmpl;
    int tp = j.tp;
    if (tmpl_in_lds) {
        for (int i = threadIdx.x; i < j.tw * j.th; i += 256) smem[i] = j.tmpl[(size_t)(i / j.tw) * j.tp + i % j.tw];
        __syncthreads();
        T = smem;
        tp = j.tw;
    }
    const int total = j.ow * j.oh;
    for (int idx = blockIdx.x * 256 + threadIdx.x; idx < total; idx += gridDim.x * 256) {
        if (j.equal1) { j.out[idx] = 1.f; continue; }
        const int y = idx / j.ow, x = idx - y * j.ow;
        uint64_t sI = 0, sQ = 0, accI = 0;
        float accF = 0.f;
        for (int r = 0; r < j.th; ++r) {
            const uint8_t* ir = j.img + (size_t)(y + r) * j.ip + x;
            const uint8_t* tr = T + (size_t)r * tp;
            uint32_t d = 0, s1 = 0, s2 = 0;
            for (int c = 0; c < j.tw; ++c) {
                const uint32_t v = ir[c], t = tr[c];
                d += v * t; s1 += v; s2 += v * v;
            }
            if (j.fold) accF = accF + (float)(int)d;   // TemplateMatcher.cpp:507
            else accI += d;
            sI += s1; sQ += s2;
        }
        const double num = j.fold ? (double)accF : (double)(float)(double)accI;
        j.out[idx] = ccoeff(num, (double)sI, (double)sQ, j.mean, j.norm, j.inv_area);
    }
}

// LDS-tiled NCC for small templates (the top layer: area <= MinReduceArea by construction).  A 256-thread
// workgroup computes a 64 x 16 tile of one map; its canvas window ((16 + th - 1) rows x (64 + 4*ntw + 4) bytes)
// and the template (rows of ntw words, zero beyond tw) are staged in LDS.  The window sums of I and I^2 depend on
// the canvas row and the output column only, so they are formed once per staged row (h1 / h2: sums over the
// template width, v_dot4_u32_u8 with a byte mask) and summed over th rows per output.  A thread owns 4 adjacent
// outputs of one row: per template word it funnel-shifts two canvas words into the 4 byte alignments and
// accumulates the correlation with one v_dot4_u32_u8 each.  Exact u32 row sums, then the same f32 fold /
// TM_CCORR rounding and f64 normalisation as k_ncc_map.  Dynamic LDS: ncc_tile_lds(tw, th).
constexpr int NT_W = 64, NT_H = 16;
constexpr int NT_MAXW = 32;                 // template words per row (tw <= 128)
constexpr int NT_MAXH = 64;                 // template rows

static size_t ncc_tile_lds(int tw, int th) {
    const int ntw = (tw + 3) >> 2, iwq = NT_W / 4 + ntw + 1, irows = NT_H + th - 1;
    return (size_t)4 * (th * ntw + ntw + irows * iwq) + (size_t)8 * irows * NT_W;
}

__global__ __launch_bounds__(256) void k_ncc_tile(const NccJob* __restrict__ jobs, int tiles_x) {
    extern __shared__ __attribute__((aligned(16))) uint32_t nt_lds[];
    const NccJob& j = jobs[blockIdx.y];
    const int tx0 = (blockIdx.x % tiles_x) * NT_W, ty0 = (blockIdx.x / tiles_x) * NT_H;
    if (tx0 >= j.ow || ty0 >= j.oh) return;   // uniform: this map has fewer tiles
    const int tw = j.tw, th = j.th, ntw = (tw + 3) >> 2;
    const int iwq = NT_W / 4 + ntw + 1;        // canvas words per staged row
    const int irows = NT_H + th - 1;
    uint32_t* H1 = nt_lds;                     // [irows][64] window row sums of I (16-byte aligned: first)
    uint32_t* H2 = H1 + irows * NT_W;          // [irows][64] of I^2
    uint32_t* Tw = H2 + irows * NT_W;          // [th][ntw]
    uint32_t* Mw = Tw + th * ntw;              // [ntw] byte masks of the template width
    uint32_t* Iw = Mw + ntw;                   // [irows][iwq]
    const int tid = threadIdx.x;
    for (int i = tid; i < th * ntw; i += 256) {
        const int r = i / ntw, k = i - r * ntw;
        uint32_t w = 0;
        for (int b = 0; b < 4; ++b) {
            const int c = 4 * k + b;
            if (c < tw) w |= (uint32_t)j.tmpl[(size_t)r * j.tp + c] << (8 * b);
        }
        Tw[r * ntw + k] = w;
    }
    if (tid < ntw) {
        uint32_t m = 0;
        for (int b = 0; b < 4; ++b)
            if (4 * tid + b < tw) m |= 1u << (8 * b);
        Mw[tid] = m;
    }
    for (int i = tid; i < irows * iwq; i += 256) {
        const int r = i / iwq, k = i - r * iwq;
        const int y = ty0 + r, x = tx0 + 4 * k;
        Iw[r * iwq + k] = (y < j.ih && x + 4 <= j.ip) ? *(const uint32_t*)(j.img + (size_t)y * j.ip + x) : 0u;
    }
    __syncthreads();
    if (j.equal1) {
        for (int i = tid; i < NT_W * NT_H; i += 256) {
            const int y = ty0 + i / NT_W, x = tx0 + i % NT_W;
            if (x < j.ow && y < j.oh) j.out[(size_t)y * j.ow + x] = 1.f;
        }
        return;
    }
    // window row sums: item (staged row r, 4 output columns q)
    for (int it = tid; it < irows * (NT_W / 4); it += 256) {
        const int r = it >> 4, q = it & 15;
        const uint32_t* ir = Iw + r * iwq + q;
        uint32_t s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
        uint32_t w0 = ir[0];
        for (int k = 0; k < ntw; ++k) {
            const uint32_t w1 = ir[k + 1];
            const uint32_t m = Mw[k], mff = m * 0xffu;
            const uint32_t sh[4] = {w0, __builtin_amdgcn_alignbyte(w1, w0, 1), __builtin_amdgcn_alignbyte(w1, w0, 2),
                                    __builtin_amdgcn_alignbyte(w1, w0, 3)};
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                s1[u] = __builtin_amdgcn_udot4(m, sh[u], s1[u], false);
                s2[u] = __builtin_amdgcn_udot4(sh[u] & mff, sh[u], s2[u], false);
            }
            w0 = w1;
        }
        *(uint4*)(H1 + r * NT_W + 4 * q) = make_uint4(s1[0], s1[1], s1[2], s1[3]);
        *(uint4*)(H2 + r * NT_W + 4 * q) = make_uint4(s2[0], s2[1], s2[2], s2[3]);
    }
    __syncthreads();
    const int ly = tid >> 4, lx = (tid & 15) * 4;   // outputs (tx0 + lx .. +3, ty0 + ly)
    float accF[4] = {0.f, 0.f, 0.f, 0.f};
    uint64_t accI[4] = {0, 0, 0, 0};
    uint32_t sI[4] = {0, 0, 0, 0}, sQ[4] = {0, 0, 0, 0};
    for (int r = 0; r < th; ++r) {
        const uint32_t* ir = Iw + (ly + r) * iwq + (lx >> 2);
        const uint32_t* tr = Tw + r * ntw;
        uint32_t d[4] = {0, 0, 0, 0};
        uint32_t w0 = ir[0];
        for (int k = 0; k < ntw; ++k) {
            const uint32_t w1 = ir[k + 1];
            const uint32_t t = tr[k];
            d[0] = __builtin_amdgcn_udot4(t, w0, d[0], false);
            d[1] = __builtin_amdgcn_udot4(t, __builtin_amdgcn_alignbyte(w1, w0, 1), d[1], false);
            d[2] = __builtin_amdgcn_udot4(t, __builtin_amdgcn_alignbyte(w1, w0, 2), d[2], false);
            d[3] = __builtin_amdgcn_udot4(t, __builtin_amdgcn_alignbyte(w1, w0, 3), d[3], false);
            w0 = w1;
        }
        const uint4 h1 = *(const uint4*)(H1 + (ly + r) * NT_W + lx), h2 = *(const uint4*)(H2 + (ly + r) * NT_W + lx);
        sI[0] += h1.x; sI[1] += h1.y; sI[2] += h1.z; sI[3] += h1.w;
        sQ[0] += h2.x; sQ[1] += h2.y; sQ[2] += h2.z; sQ[3] += h2.w;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (j.fold) accF[q] = accF[q] + (float)(int)d[q];   // TemplateMatcher.cpp:507
            else accI[q] += d[q];
        }
    }
    const int y = ty0 + ly;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int x = tx0 + lx + q;
        if (x < j.ow && y < j.oh) {
            const double num = j.fold ? (double)accF[q] : (double)(float)(double)accI[q];
            j.out[(size_t)y * j.ow + x] = ccoeff(num, (double)sI[q], (double)sQ[q], j.mean, j.norm, j.inv_area);
        }
    }
}

void launch_ncc_map(const NccJob* jobs, int njobs, int max_out, int tmpl_bytes, hipStream_t st) {
    if (njobs <= 0 || max_out <= 0) return;
    int gx = (max_out + 255) / 256;
    if (gx > 2048) gx = 2048;
    const int in_lds = tmpl_bytes <= 32768 ? 1 : 0;
    hipLaunchKernelGGL(k_ncc_map, dim3(gx, njobs), dim3(256), in_lds ? tmpl_bytes : 0, st, jobs, in_lds);
}

bool ncc_tile_fits(int tw, int th) { return tw <= 4 * NT_MAXW && th <= NT_MAXH; }

void launch_ncc_tile(const NccJob* jobs, int njobs, int max_ow, int max_oh, int tw, int th, hipStream_t st) {
    if (njobs <= 0 || max_ow <= 0 || max_oh <= 0) return;
    const int tiles_x = (max_ow + NT_W - 1) / NT_W, tiles_y = (max_oh + NT_H - 1) / NT_H;
    const size_t lds = ncc_tile_lds(tw, th);
    if (lds > 65536) ensure_lds_attr((const void*)k_ncc_tile, ncc_tile_lds(4 * NT_MAXW, NT_MAXH));
    hipLaunchKernelGGL(k_ncc_tile, dim3(tiles_x * tiles_y, njobs), dim3(256), lds, st, jobs, tiles_x);
}

// ============================================================================================== K5
__device__ __forceinline__ void better(float& v, int& i, float ov, int oi) {
    if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
}

// workgroup argmax with first-occurrence (lowest index) tie-break; result broadcast to every thread
__device__ void wg_argmax(float& v, int& i, float* sv, int* si) {
    for (int off = 32; off > 0; off >>= 1) {
        const float ov = __shfl_xor(v, off);
        const int oi = __shfl_xor(i, off);
        better(v, i, ov, oi);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sv[w] = v; si[w] = i; }
    __syncthreads();
    if (threadIdx.x == 0)
        for (int k = 1; k < (int)(blockDim.x >> 6); ++k) better(sv[0], si[0], sv[k], si[k]);
    __syncthreads();
    v = sv[0];
    i = si[0];
    __syncthreads();
}

// minMaxLoc over a sub-rectangle: first max in row-major order
__device__ __forceinline__ void rect_max(const float* m, int mw, int x0, int y0, int w, int h, float* bv, int* bi) {
    float best = m[(size_t)y0 * mw + x0];
    int bx = 0, by = 0;
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            const float v = m[(size_t)(y0 + y) * mw + x0 + x];
            if (v > best) { best = v; bx = x; by = y; }
        }
    *bv = best;
    *bi = (y0 + by) * mw + x0 + bx;
}

// s_BlockMax block layout of one map.  Qt (DataStructures.h:150-213): blocks of the template size, grid row-major, right
// strip, bottom strip, corner.  MFC (MatchTool/MatchToolDlg.h:108-175, fpm_params.semantics): blocks of twice the
// template size, no blocks at all when the map holds no whole block (the peaks then come from full-map scans), then
// right + bottom strips, the right strip alone, or else the full-width bottom strip (empty without any residue).
struct BlockGeom {
    int bw, bh, ncol, nrow, rw, rh, nb, mfc;
    __host__ __device__ void init(int mw, int mh, int tw, int th, int mfc_ = 0) {
        mfc = mfc_;
        bw = mfc ? 2 * tw : tw; bh = mfc ? 2 * th : th;
        ncol = mw / bw; nrow = mh / bh;
        rw = mw - ncol * bw; rh = mh - nrow * bh;
        if (!mfc) nb = ncol * nrow + (rw > 0) + (rh > 0) + (rw > 0 && rh > 0);
        else nb = (ncol == 0 || nrow == 0) ? 0 : ncol * nrow + ((rw > 0 && rh > 0) ? 2 : 1);
    }
    __host__ __device__ void rect(int b, int mw, int mh, int& x, int& y, int& w, int& h) const {
        if (b < ncol * nrow) { x = (b % ncol) * bw; y = (b / ncol) * bh; w = bw; h = bh; return; }
        b -= ncol * nrow;
        if (mfc) {
            if (rw > 0 && b == 0) { x = ncol * bw; y = 0; w = rw; h = mh; return; }
            if (rw > 0 && rh > 0) { x = 0; y = nrow * bh; w = ncol * bw; h = rh; return; }
            x = 0; y = nrow * bh; w = mw; h = rh;   // the full-width bottom strip (h = 0 without any residue)
            return;
        }
        if (rw > 0) { if (b == 0) { x = ncol * bw; y = 0; w = rw; h = mh; return; } --b; }
        if (rh > 0) { if (b == 0) { x = 0; y = nrow * bh; w = ncol * bw; h = rh; return; } --b; }
        x = ncol * bw; y = nrow * bh; w = rw; h = rh;
    }
    // k_nms_blocks' work items: the regular blocks, then each strip block (the right / bottom residue strips span
    // the whole map height / width) cut into chunks of one regular block's area, scanned by separate waves
    __host__ __device__ int nreg() const { return nb > 0 ? ncol * nrow : 0; }
    __host__ __device__ int chunks(int b, int mw, int mh) const {
        int x, y, w, h;
        rect(b, mw, mh, x, y, w, h);
        const long n = (long)w * h, e = (long)bw * bh;
        return n <= e ? 1 : (int)((n + e - 1) / e);
    }
    __host__ __device__ int items(int mw, int mh) const {
        int it = nreg();
        for (int b = nreg(); b < nb; ++b) it += chunks(b, mw, mh);
        return it;
    }
};
int nms_block_items(int mw, int mh, int tw, int th, int mfc) {
    BlockGeom g;
    g.init(mw, mh, tw, th, mfc);
    return g.items(mw, mh);
}

// wave argmax (value, key) with lowest-key tie-break, by DPP steps (no LDS round trip per step): quad swaps, row
// half-mirror, row mirror, then row_bcast15 / row_bcast31 fold the rows into lane 63, read back to every lane
template <int CTRL, int ROWS>
__device__ __forceinline__ void dpp_better(float& v, int& b) {
    const float ov = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(-INFINITY), __float_as_int(v), CTRL,
                                                                ROWS, 0xf, false));
    const int ob = __builtin_amdgcn_update_dpp(INT_MAX, b, CTRL, ROWS, 0xf, false);
    better(v, b, ov, ob);
}
__device__ __forceinline__ void wave_better_reduce(float& v, int& b) {
    dpp_better<0xb1, 0xf>(v, b);    // quad_perm [1,0,3,2]
    dpp_better<0x4e, 0xf>(v, b);    // quad_perm [2,3,0,1]
    dpp_better<0x141, 0xf>(v, b);   // row_half_mirror
    dpp_better<0x140, 0xf>(v, b);   // row_mirror
    dpp_better<0x142, 0xa>(v, b);   // row_bcast15 into rows 1 and 3
    dpp_better<0x143, 0xc>(v, b);   // row_bcast31 into rows 2 and 3
    v = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
    b = __builtin_amdgcn_readlane(b, 63);
}

__device__ __forceinline__ int empty_loc(int b) { return -1 - b; }

// minMaxLoc over a sub-rectangle by one wave: first max in row-major order (rect_max), result in every lane.  An empty
// rectangle (a zero-width or zero-height s_BlockMax strip) gives cv::minMaxLoc's answer for an empty array, 0 at
// (-1, -1) relative to the strip: bi = -1 here, which callers store as the block's empty marker (empty_loc)
__device__ __forceinline__ void wave_rect_max(const float* m, int mw, int x0, int y0, int w, int h, int lane,
                                              float& bv, int& bi) {
    const int n = w * h;
    if (n <= 0) {
        bv = 0.f;
        bi = -1;
        return;
    }
    float v = -INFINITY;
    int i = INT_MAX;
    int r = lane / w, c = lane - (lane / w) * w;   // element e = lane + 64k -> (r, c), advanced incrementally
    const int dr = 64 / w, dc = 64 - (64 / w) * w;
#pragma unroll 4
    for (int e = lane; e < n; e += 64) {
        const int idx = (y0 + r) * mw + x0 + c;
        const float x = m[idx];
        if (x > v) { v = x; i = idx; }   // a lane visits increasing indices: strict > keeps the first
        r += dr;
        c += dc;
        if (c >= w) { c -= w; ++r; }
    }
    wave_better_reduce(v, i);
    bv = v;
    bi = i;
}

// K5a: the s_BlockMax constructor (DataStructures.h:150-213) for every top-layer map at once, one wave per block;
// with a.cand it also lists the map's pixels >= thr (the only ones the peak loop can accept), each pixel once (the
// corner block, which repeats the right strip's pixels, emits none)
// s_BlockMax maxima of a key-combined strip chunk: the order-preserving u32 of a float (non-NaN), high word; the
// complement of the map index, low word — a u64 atomicMax then keeps the largest value and, among equal values,
// the first index (cv::minMaxLoc's rule); +-0 compare equal, so -0 enters as +0
__device__ __forceinline__ uint64_t blockmax_key(float v, int i) {
    uint32_t u = __float_as_uint(v == 0.f ? 0.f : v);
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return ((uint64_t)u << 32) | (uint32_t)(0xffffffffu - (uint32_t)i);
}

// one wave: maximum (first-max rule) of the elements [e0, e1) of a w-wide rectangle at (x, y) in row-major order,
// and (cand) the pixels >= the top-layer score appended to the map's list in the same loads (k_nms_greedy sorts
// the list, so its order is free)
__device__ __forceinline__ void nms_scan(const NmsArgs& a, const NmsJob& j, int32_t* cand, int x, int y, int w,
                                         int e0, int e1, int lane, float& bv, int& bi) {
    float v = -INFINITY;
    int i = INT_MAX;
    const int e = e0 + lane;
    int r = e / w, c = e - (e / w) * w;
    const int dr = 64 / w, dc = 64 - (64 / w) * w;
    constexpr int U = 8;   // wave-instructions of loads in flight before the first use
    int ncand = 0;
    for (int f0 = e0; f0 < e1; f0 += 64 * U) {
        int idx[U];
        float xv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            idx[u] = (y + r) * j.mw + x + c;
            xv[u] = f0 + 64 * u + lane < e1 ? j.map[idx[u]] : -INFINITY;
            r += dr;
            c += dc;
            if (c >= w) { c -= w; ++r; }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool in = f0 + 64 * u + lane < e1;
            if (in && xv[u] > v) { v = xv[u]; i = idx[u]; }   // a lane visits increasing indices: strict > keeps the first
            if (cand) ncand += __popcll(__ballot(in && (double)xv[u] >= a.thr));
        }
    }
    wave_better_reduce(v, i);
    if (ncand > 0) {   // one atomic per wave for its pixels >= the score, then (rare) a second pass writes them
        int base = 0;
        if (lane == 0) base = atomicAdd(&a.cand_cnt[blockIdx.y], ncand);
        base = __shfl(base, 0);
        int rr = e / w, cc = e - (e / w) * w;
        for (int f0 = e0; f0 < e1; f0 += 64) {
            const int id2 = (y + rr) * j.mw + x + cc;
            const bool take = f0 + lane < e1 && (double)j.map[id2] >= a.thr;
            const uint64_t mk = __ballot(take);
            const int pos = base + __popcll(mk & ((1ull << lane) - 1));
            if (take && pos < a.cand_cap) cand[pos] = id2;
            base += __popcll(mk);
            rr += dr;
            cc += dc;
            if (cc >= w) { cc -= w; ++rr; }
        }
    }
    bv = v;
    bi = i;
}

__global__ __launch_bounds__(256) void k_nms_blocks(NmsArgs a) {
    const NmsJob& j = a.jobs[blockIdx.y];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (a.cand && a.cand_cnt[blockIdx.y] < 0) return;   // taken by k_nms_greedy from k_top_mma's list (no map)
    BlockGeom g;
    g.init(j.mw, j.mh, a.tw, a.th, a.mfc);
    if (j.mw <= 0 || j.mh <= 0) return;
    const int corner = (!g.mfc && g.rw > 0 && g.rh > 0) ? g.nb - 1 : -1;   // (MFC has no corner block)
    int32_t* cand = a.cand ? a.cand + (size_t)blockIdx.y * a.cand_cap : nullptr;
    const int nreg = g.nreg();
    int ch[3] = {0, 0, 0}, nitems = nreg;
    for (int s = 0; s < g.nb - nreg && s < 3; ++s) {   // (no key scratch: every strip by one wave)
        ch[s] = a.skey ? g.chunks(nreg + s, j.mw, j.mh) : 1;
        nitems += ch[s];
    }
    for (int item = blockIdx.x * 4 + wv; item < nitems; item += gridDim.x * 4) {
        int b = item, k = 0, nk = 1, s = 0;
        if (item >= nreg) {
            int t = item - nreg;
            while (t >= ch[s]) { t -= ch[s]; ++s; }
            b = nreg + s; k = t; nk = ch[s];
        }
        int x, y, w, h;
        g.rect(b, j.mw, j.mh, x, y, w, h);
        const int n = w * h;
        float v = 0.f;
        int i = -1;   // an empty rectangle: cv::minMaxLoc's 0 at (-1, -1) (wave_rect_max)
        if (n > 0) {
            const int e0 = nk == 1 ? 0 : k * g.bw * g.bh, e1 = nk == 1 ? n : min(n, e0 + g.bw * g.bh);
            nms_scan(a, j, (cand && b != corner) ? cand : nullptr, x, y, w, e0, e1, lane, v, i);
        }
        if (nk == 1) {
            if (lane == 0) { j.bmax[b] = v; j.bloc[b] = i >= 0 ? i : empty_loc(b); }
            continue;
        }
        if (lane == 0) {   // a strip chunk: combine by key; the last chunk to finish writes the block's maximum
            uint64_t* key = a.skey + (size_t)blockIdx.y * 3 + s;
            atomicMax((unsigned long long*)key, (unsigned long long)blockmax_key(v, i));
            __threadfence();
            if (atomicAdd(a.sdone + (size_t)blockIdx.y * 3 + s, 1) == nk - 1) {
                const uint64_t fin = atomicMax((unsigned long long*)key, 0ull);
                const int fi = (int)(0xffffffffu - (uint32_t)fin);
                j.bmax[b] = fi == INT_MAX ? -INFINITY : j.map[fi];
                j.bloc[b] = fi;
            }
        }
    }
}

// argmax over the block maxima, broadcast to every thread: GetMaxValueLoc, Qt max_element (first block on ties,
// DataStructures.h:232-245) or MFC's '>=' scan (the last block on ties, MatchToolDlg.h:194-210)
__device__ __forceinline__ void block_argmax(const float* bm, const int* bl, int nb, bool last, float* sv, int* si,
                                             float& v, int& i) {
    v = -INFINITY;
    i = INT_MAX;
    for (int b = threadIdx.x; b < nb; b += 256) better(v, i, bm[b], last ? nb - 1 - b : b);
    wg_argmax(v, i, sv, si);
    i = bl[last ? nb - 1 - i : i];
}

// a block location: a map index, or empty_loc(b) for the empty strip b, whose minMaxLoc answer is (x0 - 1, y0 - 1)
__device__ __forceinline__ void block_loc_xy(const BlockGeom& g, int loc, int mw, int mh, int& px, int& py) {
    if (loc >= 0) { px = loc % mw; py = loc / mw; return; }
    int x, y, w, h;
    g.rect(-1 - loc, mw, mh, x, y, w, h);
    px = x - 1;
    py = y - 1;
}

// K5: peak extraction of one map per workgroup: getNextMaxLoc (plain: painted rectangle + full-map argmax) or its
// s_BlockMax form when k_nms_fast's LDS cannot hold the map's blocks (block maxima from k_nms_blocks in global
// scratch; after each painted rectangle the intersecting blocks are re-scanned one wave per block,
// TemplateMatcher.cpp:1208-1221, DataStructures.h:215-246)
// k_cand_init's work for the cap candidate slots of one job, done by the workgroup that found the job's cnt peaks
// (spk, in LDS): the same CandState per slot; the job's live candidates take one contiguous range of the live list
// (one atomic per job; the list's order never reaches a result: records are indexed by candidate id).
// mode 1: states only (no refinement), 2: live, 3: live and the first refinement layer is layer 0.  Workgroup-
// uniform call.
__device__ void cand_init_job(const CandInitArgs& c, int mode, int job, int cnt, const Peak* spk, int* sbase) {
    const int tid = threadIdx.x;
    if (tid == 0) *sbase = (mode >= 2 && cnt > 0) ? atomicAdd(c.live_count, cnt) : 0;
    __syncthreads();
    const int ang = job % c.nang, base = *sbase;
    for (int r = tid; r < c.cap; r += 256) {
        const int id = job * c.cap + r;
        CandState s;
        s.lt = f2(0.f, 0.f);
        s.node = ang;
        s.alive = 0;
        s.reached0 = 0;
        s.pad = 0;
        if (r < cnt) {
            const Peak pk = spk[r];
            // s_MatchParameter(Point2f(ptMaxLoc.x - fTranslationX, ...)) (TemplateMatcher.cpp:186/193/201/208),
            // ptRotatePt2f(pt, ptCenter, -angle * D2R) (:265-266)
            const F2 pt = f2((float)pk.x - c.angles[ang].tx, (float)pk.y - c.angles[ang].ty);
            s.lt = rotate_pt(pt, c.center, c.top_nodes[ang].cn, c.top_nodes[ang].sn);
            if (mode >= 2) {
                s.alive = 1;
                s.reached0 = mode == 3 ? 1 : 0;
                c.live[base + r] = id;
            }
        }
        c.state[id] = s;
    }
}

constexpr int kNmsPlainBlk = 4096;   // plain path: 64-pixel block maxima kept in LDS (maps up to 256 K pixels)
constexpr long kNmsBlkMinWork = 1 << 16;   // ... used when peak slots x map pixels reach this
constexpr size_t kNmsPlainBlkLds = (size_t)8 * kNmsPlainBlk;   // dynamic LDS of k_nms's block maxima
// ci_mode 0: peaks only; 1-3: also the job's candidate slots (cand_init_job; plain path, cap <= kNmsInitCap).
// blk_lds: the launch carries kNmsPlainBlkLds of dynamic LDS for the plain path's block maxima (launch_nms gives it
// only where some job can take that path, so the other launches keep their occupancy)
__global__ __launch_bounds__(256) void k_nms(NmsArgs a, CandInitArgs ci, int ci_mode, int blk_lds) {
    __shared__ float sv[4];
    __shared__ int si[4];
    __shared__ int naff;
    __shared__ int aff[256];
    __shared__ Peak spk[kNmsInitCap];
    __shared__ int sbase;
    extern __shared__ __attribute__((aligned(16))) uint8_t nms_dyn[];
    float* const pbv = (float*)nms_dyn;
    int* const pbi = (int*)(nms_dyn + 4 * kNmsPlainBlk);
    const NmsJob& j = a.jobs[blockIdx.x];
    if (a.cand && a.cand_cnt[blockIdx.x] < 0) return;   // taken by k_nms_greedy
    float* m = j.map;
    const int mw = j.mw, mh = j.mh, n = mw * mh, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    Peak* out = a.peaks + (size_t)blockIdx.x * a.cap;
    const double ov = a.overlap;
    BlockGeom g;
    g.init(mw, mh, a.tw, a.th, a.mfc);
    const bool blocks = a.by_block && g.nb > 0;   // (an MFC map without a whole block: full-map scans)
    const bool last = g.mfc != 0;
    float v = -INFINITY;
    int i = INT_MAX;
    if (n <= 0) {
        if (tid == 0) a.counts[blockIdx.x] = 0;
        if (ci_mode) cand_init_job(ci, ci_mode, blockIdx.x, 0, spk, &sbase);
        return;
    }
    float* bm = j.bmax;
    int* bl = j.bloc;
    // plain path on maps of up to kNmsPlainBlk blocks of 64 pixels: the first maximum of every block in LDS; after a
    // painted rectangle only the blocks it touches are re-scanned, and the workgroup argmax of the block maxima (largest
    // value, lowest index) is the map's first maximum -- the same answer as a full-map scan (round 4: the README Test4
    // search, 43 peak slots on a 373 x 284 map, spent 545 us in full scans)
    const int nb64 = (n + 63) >> 6;
    // (small loops keep the full-map scan: a lone Src7 search's 41 maps of ~2 K pixels and 8 peak slots ran 10.8 us
    // that way, 15.0 us with the block maxima's extra barriers, profiles/r04_end)
    const bool chunked = blk_lds && !blocks && nb64 <= kNmsPlainBlk && (long)a.cap * n >= kNmsBlkMinWork;
    const bool m16 = ((uintptr_t)m & 15) == 0;
    auto scan_blk = [&](int b) {   // first maximum of block b: its 16 loads in flight, compared in index order
        const int k0 = b << 6, k1 = min(n, k0 + 64);
        float tv = -INFINITY;
        int ti = INT_MAX;
        if (m16 && k1 - k0 == 64) {
            float4 x[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) x[u] = *(const float4*)(m + k0 + 4 * u);
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                if (x[u].x > tv) { tv = x[u].x; ti = k0 + 4 * u; }
                if (x[u].y > tv) { tv = x[u].y; ti = k0 + 4 * u + 1; }
                if (x[u].z > tv) { tv = x[u].z; ti = k0 + 4 * u + 2; }
                if (x[u].w > tv) { tv = x[u].w; ti = k0 + 4 * u + 3; }
            }
        } else {
            for (int k = k0; k < k1; ++k) { const float x = m[k]; if (x > tv) { tv = x; ti = k; } }
        }
        pbv[b] = tv;
        pbi[b] = ti;
    };
    auto blocks_argmax = [&]() {
        v = -INFINITY;
        i = INT_MAX;
        for (int b = tid; b < nb64; b += 256) better(v, i, pbv[b], pbi[b]);
        wg_argmax(v, i, sv, si);
    };
    if (blocks) {
        block_argmax(bm, bl, g.nb, last, sv, si, v, i);
    } else if (chunked) {
        for (int b = tid; b < nb64; b += 256) scan_blk(b);
        __syncthreads();
        blocks_argmax();
    } else {
        for (int k = tid; k < n; k += 256) { const float x = m[k]; if (x > v) { v = x; i = k; } }
        wg_argmax(v, i, sv, si);
    }
    if ((double)v < a.thr) {
        if (tid == 0) a.counts[blockIdx.x] = 0;
        if (ci_mode) cand_init_job(ci, ci_mode, blockIdx.x, 0, spk, &sbase);
        return;
    }
    int cnt = 0;
    int px, py;
    block_loc_xy(g, i, mw, mh, px, py);
    if (tid == 0) {
        out[0].x = px; out[0].y = py; out[0].score = v;
        if (ci_mode) { spk[0].x = px; spk[0].y = py; spk[0].score = v; }
    }
    ++cnt;
    for (int it = 0; it < a.cap - 1; ++it) {
        // rect of getNextMaxLoc (TemplateMatcher.cpp:1198-1201 / :1211-1214): int truncation of f64
        const int sx = (int)(px - a.tw * (1 - ov)), sy = (int)(py - a.th * (1 - ov));
        const int rw = (int)(2 * a.tw * (1 - ov)), rh = (int)(2 * a.th * (1 - ov));
        if (rw > 0 && rh > 0) {
            const int x1 = sx > 0 ? sx : 0, y1 = sy > 0 ? sy : 0;
            const int x2 = min(sx + rw - 1, mw - 1), y2 = min(sy + rh - 1, mh - 1);
            const int cw = x2 - x1 + 1, ch = y2 - y1 + 1;
            if (cw > 0 && ch > 0)
                for (int k = tid; k < cw * ch; k += 256) m[(size_t)(y1 + k / cw) * mw + x1 + k % cw] = -1.f;
        }
        if (tid == 0) naff = 0;
        __syncthreads();
        if (blocks) {
            // blocks whose rectangle intersects the painted one (UpdateMax), listed, then re-scanned per wave
            for (int b = tid; b < g.nb; b += 256) {
                int x, y, w, h;
                g.rect(b, mw, mh, x, y, w, h);
                const int ix1 = max(x, sx), iy1 = max(y, sy);
                const int iw = min(x + w, sx + rw) - ix1, ih = min(y + h, sy + rh) - iy1;
                if (iw > 0 && ih > 0) {
                    const int k = atomicAdd(&naff, 1);
                    if (k < 256) aff[k] = b;
                }
            }
            __syncthreads();
            const int na = naff;
            if (na <= 256) {
                for (int k = wv; k < na; k += 4) {
                    const int b = aff[k];
                    int x, y, w, h;
                    g.rect(b, mw, mh, x, y, w, h);
                    float bv;
                    int bi;
                    wave_rect_max(m, mw, x, y, w, h, lane, bv, bi);
                    if (lane == 0) { bm[b] = bv; bl[b] = bi; }
                }
            } else {   // (a painted rectangle spanning > 256 blocks: overlap < 0 with tiny blocks) one per thread
                for (int b = tid; b < g.nb; b += 256) {
                    int x, y, w, h;
                    g.rect(b, mw, mh, x, y, w, h);
                    const int ix1 = max(x, sx), iy1 = max(y, sy);
                    const int iw = min(x + w, sx + rw) - ix1, ih = min(y + h, sy + rh) - iy1;
                    if (iw > 0 && ih > 0) rect_max(m, mw, x, y, w, h, &bm[b], &bl[b]);
                }
            }
            __syncthreads();
            block_argmax(bm, bl, g.nb, last, sv, si, v, i);
        } else if (chunked) {
            // the blocks the painted rectangle (rows y1 .. y2, columns x1 .. x2, as painted above) touches: row y's
            // segment covers blocks (y mw + x1) >> 6 .. (y mw + x2) >> 6, at most per_row of them (a block two rows share
            // is re-scanned twice, to the same values)
            if (rw > 0 && rh > 0) {
                const int x1 = sx > 0 ? sx : 0, y1 = sy > 0 ? sy : 0;
                const int x2 = min(sx + rw - 1, mw - 1), y2 = min(sy + rh - 1, mh - 1);
                if (x1 <= x2 && y1 <= y2) {
                    const int per_row = ((x2 - x1) >> 6) + 2;
                    for (int q = tid; q < (y2 - y1 + 1) * per_row; q += 256) {
                        const int y = y1 + q / per_row, b = ((y * mw + x1) >> 6) + q % per_row;
                        if (b <= ((y * mw + x2) >> 6)) scan_blk(b);
                    }
                }
            }
            __syncthreads();
            blocks_argmax();
        } else {
            v = -INFINITY;
            i = INT_MAX;
            for (int k = tid; k < n; k += 256) { const float x = m[k]; if (x > v) { v = x; i = k; } }
            wg_argmax(v, i, sv, si);
        }
        if ((double)v < a.thr) break;
        block_loc_xy(g, i, mw, mh, px, py);
        if (tid == 0) {
            out[cnt].x = px; out[cnt].y = py; out[cnt].score = v;
            if (ci_mode) { spk[cnt].x = px; spk[cnt].y = py; spk[cnt].score = v; }
        }
        ++cnt;
    }
    if (tid == 0) a.counts[blockIdx.x] = cnt;
    if (ci_mode) cand_init_job(ci, ci_mode, blockIdx.x, cnt, spk, &sbase);
}

// K5 (s_BlockMax, fast form): the same sequence of peaks as k_nms's block mode with the map left untouched.  A
// pixel inside an accepted peak's rectangle reads as -1 (the value getNextMaxLoc paints), so an iteration is: the
// blocks the new rectangle intersects (from the grid arithmetic, UpdateMax), their maxima re-scanned one wave per
// block, the maxima of their 64-block groups, and one wave's argmax over the group maxima (GetMaxValueLoc: first
// block on ties).  Block / group maxima and the accepted peaks live in LDS.  Sparse mode (thr > -1 and the
// map's candidate list fits): a block's maximum only matters while it is >= thr, and every pixel >= thr is in
// the candidate list, so a block re-scan reads its few candidates from LDS instead of the map (a block left with
// none reads -inf: the loop then stops exactly where the reference's maximum drops below thr).

// s_BlockMax block(s) holding map pixel (x, y): grid block or strip; b2 = the corner block (repeats the right strip)
__device__ __forceinline__ int nms_block_of(const BlockGeom& g, int x, int y, int tw, int th, int& b2) {
    const int gw = g.ncol * tw, gh = g.nrow * th, base = g.ncol * g.nrow;
    b2 = -1;
    if (x < gw && y < gh) return (y / th) * g.ncol + x / tw;
    if (x >= gw) {
        if (y >= gh) b2 = base + 2;   // rw > 0 and rh > 0: right strip, bottom strip, corner
        return base;
    }
    return base + (g.rw > 0 ? 1 : 0);
}

// the MFC block holding map pixel (x, y) (MatchToolDlg.h:108-175: grid, then right strip, then bottom strip)
__device__ __forceinline__ int nms_block_of_mfc(const BlockGeom& g, int x, int y) {
    const int gw = g.ncol * g.bw, gh = g.nrow * g.bh, base = g.ncol * g.nrow;
    if (x < gw && y < gh) return (y / g.bh) * g.ncol + x / g.bw;
    if (x >= gw) return base;
    return base + (g.rw > 0 ? 1 : 0);
}

__global__ __launch_bounds__(256) void k_nms_fast(NmsArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t nms_lds[];
    __shared__ int wsum[4];
    __shared__ int sparse_s;
    const NmsJob& j = a.jobs[blockIdx.x];
    const float* m = j.map;
    const int mw = j.mw, mh = j.mh, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    Peak* out = a.peaks + (size_t)blockIdx.x * a.cap;
    if (a.cand && a.cand_cnt[blockIdx.x] < 0) return;   // taken by k_nms_greedy
    if (mw <= 0 || mh <= 0) { if (tid == 0) a.counts[blockIdx.x] = 0; return; }
    const bool stamp = a.stamps && blockIdx.x == 0 && tid == 0;
    uint64_t st_t = stamp ? __builtin_readcyclecounter() : 0, st_acc[6] = {0, 0, 0, 0, 0, 0};
    auto STAMP = [&](int k) {
        if (stamp) { const uint64_t t = __builtin_readcyclecounter(); st_acc[k] += t - st_t; st_t = t; }
    };
    const double ov = a.overlap;
    const int tw = a.tw, th = a.th;
    BlockGeom g;
    g.init(mw, mh, tw, th);
    const int nb = g.nb, ng = (nb + 63) >> 6, LB = a.lds_blocks;
    // positions are kept as keys (y << 16) | x (maps are < 65536 wide and high): key order = row-major order, so
    // ties resolve exactly as on map indices, and no division is needed in the loop
    float* bm = (float*)nms_lds;                  // [LB] block maxima
    int* bl = (int*)(bm + LB);                    // [LB] their keys
    int* st = bl + LB;                            // [LB + 1] candidate ranges (sparse mode)
    float* gm = (float*)(st + LB + 1);            // [LB / 64 + 1] group maxima
    int* gb = (int*)(gm + (LB >> 6) + 1);         // their block indices
    float* cv = (float*)(gb + (LB >> 6) + 1);     // [cand_lds] candidate values, grouped by block
    int* ci = (int*)(cv + a.cand_lds);            // [cand_lds] candidate keys
    for (int b = tid; b < nb; b += 256) {
        const int idx = j.bloc[b];
        bm[b] = j.bmax[b];
        bl[b] = ((idx / mw) << 16) | (idx % mw);
    }
    // ---- sparse mode setup: counting sort of the candidate list by block into LDS
    const int K = a.cand ? a.cand_cnt[blockIdx.x] : 0;
    bool sparse = a.cand && a.thr > -1.0 && K <= a.cand_cap && K <= a.cand_lds;
    if (sparse) {
        const int32_t* cand = a.cand + (size_t)blockIdx.x * a.cand_cap;
        for (int b = tid; b <= nb; b += 256) st[b] = 0;
        __syncthreads();
        for (int k = tid; k < K; k += 256) {
            const int idx = cand[k];
            int b2;
            const int b = nms_block_of(g, idx % mw, idx / mw, tw, th, b2);
            atomicAdd(&st[b], 1);
            if (b2 >= 0) atomicAdd(&st[b2], 1);
        }
        __syncthreads();
        // exclusive scan of st[0 .. nb): per-thread chunk sums, wave prefix by shuffles, wave totals, chunk re-walk
        const int chunk = (nb + 255) / 256, c0 = tid * chunk, c1 = min(nb, c0 + chunk);
        int sum = 0;
        for (int b = c0; b < c1; ++b) sum += st[b];
        int incl = sum;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(incl, off);
            if (lane >= off) incl += y;
        }
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        int run = incl - sum;
        for (int w = 0; w < wv; ++w) run += wsum[w];
        if (tid == 255) sparse_s = run + sum <= a.cand_lds;   // the corner's repeats must fit too
        for (int b = c0; b < c1; ++b) { const int x = st[b]; st[b] = run; run += x; }
        __syncthreads();
        sparse = sparse_s != 0;
        if (sparse) {
            for (int k = tid; k < K; k += 256) {   // scatter; afterwards st[b] = end of block b = start of b + 1
                const int idx = cand[k];
                const float val = m[idx];
                const int x = idx % mw, y = idx / mw, key = (y << 16) | x;
                int b2;
                const int b = nms_block_of(g, x, y, tw, th, b2);
                const int p = atomicAdd(&st[b], 1);
                cv[p] = val; ci[p] = key;
                if (b2 >= 0) { const int p2 = atomicAdd(&st[b2], 1); cv[p2] = val; ci[p2] = key; }
            }
        }
    }
    __syncthreads();
    auto group_max = [&](int gi) {   // one wave
        const int b = gi * 64 + lane;
        float v = b < nb ? bm[b] : -INFINITY;
        int bb = b < nb ? b : INT_MAX;
        wave_better_reduce(v, bb);
        if (lane == 0) { gm[gi] = v; gb[gi] = bb; }
    };
    for (int gi = wv; gi < ng; gi += 4) group_max(gi);
    __syncthreads();
    // the peak loop runs in wave 0 alone (no barriers): the state is in LDS and the work per peak is a few blocks
    if (wv != 0) return;
    int nres = 0;   // (profiling) blocks re-scanned
    auto final_max = [&](float& v, int& key) {
        float fv = -INFINITY;
        int bb = INT_MAX;
        for (int k = lane; k < ng; k += 64) better(fv, bb, gm[k], gb[k]);
        wave_better_reduce(fv, bb);
        v = fv;
        key = bl[bb];
    };
    float v;
    int key;
    final_max(v, key);
    STAMP(0);   // setup
    // rectangle of getNextMaxLoc (TemplateMatcher.cpp:1198-1201 / :1211-1214): int truncation of f64
    const int rw = (int)(2 * tw * (1 - ov)), rh = (int)(2 * th * (1 - ov));
    const int gw = g.ncol * tw, gh = g.nrow * th, ngrid = g.ncol * g.nrow;
    int qx[4] = {0, 0, 0, 0}, qy[4] = {0, 0, 0, 0};   // accepted rectangles' origins: rectangle k in lane k % 64
    int cnt = 0;
    for (;;) {
        if ((double)v < a.thr) break;
        const int px = key & 0xffff, py = key >> 16;
        const int sx = (int)(px - tw * (1 - ov)), sy = (int)(py - th * (1 - ov));
        if (lane == 0) { out[cnt].x = px; out[cnt].y = py; out[cnt].score = v; }
        if (lane == (cnt & 63)) {
            const int hw = cnt >> 6;
            if (hw == 0) { qx[0] = sx; qy[0] = sy; }
            else if (hw == 1) { qx[1] = sx; qy[1] = sy; }
            else if (hw == 2) { qx[2] = sx; qy[2] = sy; }
            else { qx[3] = sx; qy[3] = sy; }
        }
        ++cnt;
        if (cnt >= a.cap) break;
        if (rw <= 0 || rh <= 0) continue;   // nothing painted: the same peak again (as the reference finds it)
        // blocks intersecting [sx, sx + rw) x [sy, sy + rh) (UpdateMax), one candidate per lane: lanes 0-8 the <= 3x3
        // grid blocks, lanes 9-11 the right strip, bottom strip and corner
        int lb = -1, lx = 0, ly = 0, lw = 0, lh = 0;
        if (lane < 9) {
            if (g.ncol > 0 && g.nrow > 0 && sx < gw && sx + rw > 0 && sy < gh && sy + rh > 0) {
                const int c0 = max(sx, 0) / tw, c1 = min(sx + rw - 1, gw - 1) / tw;
                const int r0 = max(sy, 0) / th, r1 = min(sy + rh - 1, gh - 1) / th;
                const int r = r0 + lane / 3, c = c0 + lane % 3;
                if (r <= r1 && c <= c1) { lb = r * g.ncol + c; lx = c * tw; ly = r * th; lw = tw; lh = th; }
            }
        } else if (lane == 9) {
            if (g.rw > 0) { lb = ngrid; lx = gw; ly = 0; lw = g.rw; lh = mh; }
        } else if (lane == 10) {
            if (g.rh > 0) { lb = ngrid + (g.rw > 0 ? 1 : 0); lx = 0; ly = gh; lw = gw; lh = g.rh; }
        } else if (lane == 11) {
            if (g.rw > 0 && g.rh > 0) { lb = ngrid + 2; lx = gw; ly = gh; lw = g.rw; lh = g.rh; }
        }
        bool upd = lb >= 0 && min(lx + lw, sx + rw) - max(lx, sx) > 0 && min(ly + lh, sy + rh) - max(ly, sy) > 0;
        // painting only lowers values: a block whose current maximum lies outside the new rectangle keeps it (value
        // and first position), so only blocks whose maximum was painted are re-scanned
        if (upd) {
            const int k = bl[lb], kx = k & 0xffff, ky = k >> 16;
            upd = kx >= sx && kx < sx + rw && ky >= sy && ky < sy + rh;
        }
        const uint64_t umask = __ballot(upd);
        STAMP(1);   // enumeration + the painted-maximum test
        for (uint64_t mk = umask; mk;) {
            const int l = __builtin_ctzll(mk);
            mk &= mk - 1;
            const int b = __builtin_amdgcn_readlane(lb, l);
            const int x = __builtin_amdgcn_readlane(lx, l), y = __builtin_amdgcn_readlane(ly, l);
            const int w = __builtin_amdgcn_readlane(lw, l), h = __builtin_amdgcn_readlane(lh, l);
            // accepted rectangles that meet this block
            uint64_t hit[4];
#pragma unroll
            for (int hw = 0; hw < 4; ++hw) {
                const int k = hw * 64 + lane;
                hit[hw] = __ballot(k < cnt && min(x + w, qx[hw] + rw) > max(x, qx[hw]) &&
                                   min(y + h, qy[hw] + rh) > max(y, qy[hw]));
            }
            auto painted = [&](int X, int Y) {
                bool p = false;
#pragma unroll
                for (int hw = 0; hw < 4; ++hw) {
                    uint64_t hm = hit[hw];
                    while (hm) {
                        const int hl = __builtin_ctzll(hm);
                        hm &= hm - 1;
                        const int ax = __builtin_amdgcn_readlane(qx[hw], hl), ay = __builtin_amdgcn_readlane(qy[hw], hl);
                        p |= X >= ax && X < ax + rw && Y >= ay && Y < ay + rh;
                    }
                }
                return p;
            };
            float bv = -INFINITY;
            int bk = INT_MAX;
            if (sparse) {
                const int e0 = b == 0 ? 0 : st[b - 1], e1 = st[b];
                for (int e = e0 + lane; e < e1; e += 64) {
                    const int ck = ci[e];
                    const float cval = cv[e];
                    if (!painted(ck & 0xffff, ck >> 16)) better(bv, bk, cval, ck);
                }
                wave_better_reduce(bv, bk);
                if (bk == INT_MAX) bk = (y << 16) | x;   // no candidate left: below thr (any valid position)
            } else {
                const int n = w * h;
                int r = lane / w, cc = lane - (lane / w) * w;
                const int dr = 64 / w, dc = 64 - (64 / w) * w;
                for (int e = lane; e < n; e += 64) {
                    const int X = x + cc, Y = y + r;
                    const float val = painted(X, Y) ? -1.f : m[Y * mw + X];
                    if (val > bv) { bv = val; bk = (Y << 16) | X; }
                    r += dr;
                    cc += dc;
                    if (cc >= w) { cc -= w; ++r; }
                }
                wave_better_reduce(bv, bk);   // ties: lowest key = first in the block's row-major order
            }
            if (lane == 0) { bm[b] = bv; bl[b] = bk; }
            ++nres;
        }
        STAMP(2);   // block re-scans
        // the re-scanned blocks' 64-block groups (unique)
        const int lg = upd ? (lb >> 6) : -1;
        bool first = upd;
        for (int u = 0; u < 12; ++u) {
            const int gu = __builtin_amdgcn_readlane(lg, u);
            if (u < lane && gu == lg) first = false;
        }
        for (uint64_t gmask = __ballot(first); gmask;) {
            const int l = __builtin_ctzll(gmask);
            gmask &= gmask - 1;
            group_max(__builtin_amdgcn_readlane(lg, l));
        }
        STAMP(3);   // group maxima
        final_max(v, key);
        STAMP(4);   // final argmax
    }
    if (tid == 0) a.counts[blockIdx.x] = cnt;
    if (stamp) {
        for (int k = 0; k < 5; ++k) a.stamps[k] = st_acc[k];
        a.stamps[5] = (uint64_t)cnt;
        a.stamps[6] = (uint64_t)(sparse ? 1 : 0);
        a.stamps[7] = (uint64_t)nres;
    }
}

// K5 (s_BlockMax, greedy form).  With every painted rectangle the reference takes the maximum of the remaining
// pixels, ordered by value (descending), then block (first in s_BlockMax order: max_element), then row-major
// position inside the block (minMaxLoc).  Only pixels >= thr can be taken and the values never change except by
// painting, so the peak sequence is the greedy pass over the pixels >= thr sorted by that key: a pixel is taken
// iff no earlier taken pixel's rectangle covers it.  Here: bitonic sort of the candidate list in LDS, then one
// wave walks it 64 candidates at a time; coverage is looked up in per-cell lists (cells of template size) of the
// taken rectangles.  Maps this form does not take (candidate list too long, thr <= -1, an empty painted
// rectangle, a zero-width strip) are left to k_nms_fast; a taken map is marked by cand_cnt = -1.
constexpr int kGreedyMax = 4096;   // candidates sorted in LDS
constexpr int kCellIds = 6;        // taken rectangles listed per cell before the cell falls back to a full scan

__device__ __forceinline__ bool greedy_before(float va, uint64_t ka, float vb, uint64_t kb) {
    return va > vb || (va == vb && ka < kb);
}

// Also the plain getNextMaxLoc loop (a.by_block == 0, TemplateMatcher.cpp:197-212 / :1196-1206): with every painted
// rectangle the reference takes the first maximum of the map in row-major order, so the key is the position alone
// (block 0 for every pixel), and the same greedy pass gives its peaks.  a.cand_val: the candidates' values come with the
// list (k_top_mma, which never writes the map); ci_mode != 0 (plain path, cap <= kNmsInitCap): the candidate init of
// the jobs this kernel takes (cand_init_job, as k_nms does); a.reset_untaken: a job it does not take gets cand_cnt = 0,
// so k_nms_blocks can list that job's pixels again from the fallback map.
__global__ __launch_bounds__(256) void k_nms_greedy(NmsArgs a, CandInitArgs ci, int ci_mode) {
    extern __shared__ __attribute__((aligned(16))) uint8_t nms_lds[];
    __shared__ Peak spk[kNmsInitCap];
    __shared__ int sbase, scnt;
    const NmsJob& j = a.jobs[blockIdx.x];
    const float* m = j.map;
    const int mw = j.mw, mh = j.mh, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const double ov = a.overlap;
    const int tw = a.tw, th = a.th;
    const int rw = (int)(2 * tw * (1 - ov)), rh = (int)(2 * th * (1 - ov));
    const bool plain = !a.by_block;
    BlockGeom g;
    g.init(mw, mh, tw, th, a.mfc);
    const int K = a.cand_cnt[blockIdx.x];
    const int cxn = (mw + tw - 1) / tw, cyn = (mh + th - 1) / th, ncell = cxn * cyn;
    const int GC = a.greedy_cap > 0 ? a.greedy_cap : kGreedyMax;   // sort capacity of this launch's LDS (power of 2)
    if (!(mw > 0 && mh > 0 && (plain || (g.ncol > 0 && g.nrow > 0)) && rw > 0 && rh > 0 && a.thr > -1.0 && K >= 0 &&
          K <= a.cand_cap && K <= GC && ncell <= a.lds_blocks)) {
        if (a.reset_untaken && tid == 0 && K >= 0) a.cand_cnt[blockIdx.x] = 0;
        return;
    }
    int P = 64;
    while (P < K) P <<= 1;
    uint64_t* sk = (uint64_t*)nms_lds;                 // [GC] (block << 32) | (y << 16) | x
    float* sv = (float*)(sk + GC);                     // [GC] values
    uint8_t* ccnt = (uint8_t*)(sv + GC);               // [cells] taken rectangles per cell
    uint8_t* cids = ccnt + a.lds_blocks;               // [cells][kCellIds]
    int* accx = (int*)(cids + (size_t)a.lds_blocks * kCellIds + 16 - ((a.lds_blocks * (1 + kCellIds)) & 15));
    int* accy = accx + 256;
    const int32_t* cand = a.cand + (size_t)blockIdx.x * a.cand_cap;
    for (int i = tid; i < P; i += 256) {
        if (i < K) {
            const int idx = cand[i], x = idx % mw, y = idx / mw;
            int b2;
            // MFC: the last block wins equal maxima, so the block part of the key counts down
            const int b = plain ? 0 : g.mfc ? g.nb - 1 - nms_block_of_mfc(g, x, y) : nms_block_of(g, x, y, tw, th, b2);
            sv[i] = a.cand_val ? a.cand_val[(size_t)blockIdx.x * a.cand_cap + i] : m[idx];
            sk[i] = ((uint64_t)b << 32) | (uint32_t)((y << 16) | x);
        } else {
            sv[i] = -INFINITY;
            sk[i] = ~0ull;
        }
    }
    for (int c = tid; c < ncell; c += 256) ccnt[c] = 0;
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1)   // bitonic sort into greedy order
        for (int jj = k >> 1; jj > 0; jj >>= 1) {
            for (int i = tid; i < P; i += 256) {
                const int l = i ^ jj;
                if (l > i) {
                    const float vi = sv[i], vl = sv[l];
                    const uint64_t ki = sk[i], kl = sk[l];
                    const bool asc = (i & k) == 0;
                    if (asc ? greedy_before(vl, kl, vi, ki) : greedy_before(vi, ki, vl, kl)) {
                        sv[i] = vl; sv[l] = vi; sk[i] = kl; sk[l] = ki;
                    }
                }
            }
            __syncthreads();
        }
    Peak* out = a.peaks + (size_t)blockIdx.x * a.cap;
    int cnt = 0;
    if (wv == 0) {
    for (int base = 0; base < K && cnt < a.cap; base += 64) {
        const int i = base + lane;
        const bool valid = i < K;
        const uint32_t pk = valid ? (uint32_t)sk[i] : 0u;
        const int x = pk & 0xffff, y = pk >> 16;
        const float v = valid ? sv[i] : -INFINITY;
        bool covered = !valid;
        if (valid) {
            const int c = (y / th) * cxn + x / tw;
            const int nc = ccnt[c];
            if (nc <= kCellIds) {
                for (int r = 0; r < nc; ++r) {
                    const int id = cids[c * kCellIds + r];
                    const int qx = accx[id], qy = accy[id];
                    covered |= x >= qx && x < qx + rw && y >= qy && y < qy + rh;
                }
            } else {
                for (int id = 0; id < cnt; ++id) {
                    const int qx = accx[id], qy = accy[id];
                    covered |= x >= qx && x < qx + rw && y >= qy && y < qy + rh;
                }
            }
        }
        uint64_t fre = __ballot(!covered);
        while (fre && cnt < a.cap) {
            const int l = __builtin_ctzll(fre);
            const int tx = __builtin_amdgcn_readlane(x, l), ty = __builtin_amdgcn_readlane(y, l);
            const float tv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
            const int sx = (int)(tx - tw * (1 - ov)), sy = (int)(ty - th * (1 - ov));
            if (!(tx >= sx && tx < sx + rw && ty >= sy && ty < sy + rh)) {
                // (uniform) a painted rectangle that misses its own peak (e.g. MaxOverlap 0.8 on a 5-row template:
                // int(2 * 5 * 0.2) = 1 row, starting a row above): the peak stays the map's maximum, so the reference
                // takes it again with every remaining getNextMaxLoc call
                if (lane == 0)
                    for (int k = cnt; k < a.cap; ++k) {
                        out[k].x = tx; out[k].y = ty; out[k].score = tv;
                        if (ci_mode && k < kNmsInitCap) { spk[k].x = tx; spk[k].y = ty; spk[k].score = tv; }
                    }
                cnt = a.cap;
                break;
            }
            if (lane == 0) {
                out[cnt].x = tx; out[cnt].y = ty; out[cnt].score = tv;
                accx[cnt] = sx; accy[cnt] = sy;
                if (ci_mode && cnt < kNmsInitCap) { spk[cnt].x = tx; spk[cnt].y = ty; spk[cnt].score = tv; }
            }
            // register the rectangle in the <= 3 x 3 cells it covers (lanes 0-8)
            const int cx0 = max(sx, 0) / tw, cx1 = min(sx + rw - 1, mw - 1) / tw;
            const int cy0 = max(sy, 0) / th, cy1 = min(sy + rh - 1, mh - 1) / th;
            if (lane < 9) {
                const int cx = cx0 + lane % 3, cy = cy0 + lane / 3;
                if (cx <= cx1 && cy <= cy1 && sx + rw > 0 && sy + rh > 0) {
                    const int c = cy * cxn + cx;
                    const int nc = ccnt[c];
                    if (nc < kCellIds) cids[c * kCellIds + nc] = (uint8_t)cnt;
                    ccnt[c] = (uint8_t)(nc < 255 ? nc + 1 : 255);
                }
            }
            ++cnt;
            // this chunk's later candidates: covered by the new rectangle?
            const bool hit = lane > l && x >= sx && x < sx + rw && y >= sy && y < sy + rh;
            fre &= ~__ballot(hit);
            fre &= fre - 1;   // lane l taken
        }
    }
    if (lane == 0) {
        a.counts[blockIdx.x] = cnt;
        a.cand_cnt[blockIdx.x] = -1;   // taken by this form: k_nms_fast / k_nms / k_top_mma's fallback skip the map
        scnt = cnt;
    }
    }   // wave 0
    if (ci_mode) {   // workgroup-uniform: every wave reaches it
        __syncthreads();
        cand_init_job(ci, ci_mode, blockIdx.x, scnt, spk, &sbase);
    }
}

static size_t nms_greedy_lds(int cells, int gcap = kGreedyMax) {
    return (size_t)12 * gcap + (size_t)cells * (1 + kCellIds) + 16 + 8 * 256;
}

// LDS bytes of k_nms_fast for a block capacity, peak capacity and candidate capacity
static size_t nms_fast_lds(int blocks, int /*cap*/, int cands) {
    return (size_t)12 * blocks + 4 + (size_t)8 * ((blocks >> 6) + 1) + (size_t)8 * cands;
}

constexpr int kNmsLdsBlocksMax = 12 * 1024;   // block maxima kept in LDS up to this many blocks
constexpr int kNmsLdsBytes = 160 * 1024 - 4096;   // k_nms_fast dynamic LDS budget (statics take the rest)

void launch_nms(const NmsArgs& a0, int njobs, int max_blocks, int max_map_dim, int max_cells, hipStream_t st,
                int max_items, const CandInitArgs* ci, long max_map_px) {
    if (njobs <= 0) return;
    NmsArgs a = a0;
    CandInitArgs cz{};
    // k_nms's block maxima (its plain path on maps where peak slots x pixels >= kNmsBlkMinWork): LDS only if some map
    // can take that path (max_map_px < 0: unknown, always)
    const int blk = max_map_px < 0 || (long)a.cap * max_map_px >= kNmsBlkMinWork;
    const size_t blds = blk ? kNmsPlainBlkLds : 0;
    if (!a.by_block && ci && a.cap <= kNmsInitCap) {   // plain path with the candidate init fused
        hipLaunchKernelGGL(k_nms, dim3(njobs), dim3(256), blds, st, a, *ci,
                           ci->refine == 0 ? 1 : (ci->refine == 2 ? 3 : 2), blk);
        return;
    }
    if (a.by_block && max_blocks > 0) {
        const int items = max_items > max_blocks ? max_items : max_blocks;
        hipLaunchKernelGGL(k_nms_blocks, dim3((items + 3) / 4 < 16384 ? (items + 3) / 4 : 16384, njobs),
                           dim3(256), 0, st, a);
        // the greedy form takes what it can (thr > 0: an empty strip's stale 0 is never a peak); k_nms the rest
        const bool greedy = a.cand && !a.stamps && a.thr > 0.0 && max_map_dim < 65536 && a.cap <= 256 &&
                            nms_greedy_lds(max_cells) <= (size_t)kNmsLdsBytes;
        if (greedy) ensure_lds_attr((const void*)k_nms_greedy, kNmsLdsBytes);
        if (a.mfc) {   // MFC block semantics: greedy form + k_nms (k_nms_fast is Qt-only)
            if (greedy) {
                NmsArgs gA = a;
                gA.lds_blocks = max_cells;
                hipLaunchKernelGGL(k_nms_greedy, dim3(njobs), dim3(256), nms_greedy_lds(max_cells), st, gA, cz, 0);
            }
            a.lds_blocks = 0;
            hipLaunchKernelGGL(k_nms, dim3(njobs), dim3(256), blds, st, a, cz, 0, blk);
            return;
        }
        const size_t fixed = nms_fast_lds(max_blocks, a.cap, 0);
        if (max_blocks <= kNmsLdsBlocksMax && a.cap <= 256 && a.overlap >= 0.0 && max_map_dim < 65536 &&
            a.thr > 0.0 && fixed <= (size_t)kNmsLdsBytes) {
            a.lds_blocks = max_blocks;
            const long room = ((long)kNmsLdsBytes - (long)fixed) / 8;
            a.cand_lds = a.cand ? (int)(room < kNmsCandCap ? room : kNmsCandCap) : 0;
            const size_t lds = nms_fast_lds(max_blocks, a.cap, a.cand_lds);
            ensure_lds_attr((const void*)k_nms_fast, kNmsLdsBytes);
            if (greedy) {
                NmsArgs gA = a;
                gA.lds_blocks = max_cells;
                hipLaunchKernelGGL(k_nms_greedy, dim3(njobs), dim3(256), nms_greedy_lds(max_cells), st, gA, cz, 0);
            }
            hipLaunchKernelGGL(k_nms_fast, dim3(njobs), dim3(256), lds, st, a);
            return;
        }
    }
    a.lds_blocks = 0;
    hipLaunchKernelGGL(k_nms, dim3(njobs), dim3(256), blds, st, a, cz, 0, blk);
}

// ============================================================================================== init
__global__ __launch_bounds__(256) void k_cand_init(CandInitArgs a, int mark_reached0) {
    const int id = blockIdx.x * 256 + threadIdx.x;
    if (id >= a.total) return;
    const int job = id / a.cap, r = id - job * a.cap, ang = job % a.nang;
    CandState s;
    s.lt = f2(0.f, 0.f);
    s.node = ang;
    s.alive = 0;
    s.reached0 = 0;
    s.pad = 0;
    if (r < a.counts[job]) {
        const Peak pk = a.peaks[id];
        // s_MatchParameter(Point2f(ptMaxLoc.x - fTranslationX, ...)) (TemplateMatcher.cpp:186/193/201/208)
        const F2 pt = f2((float)pk.x - a.angles[ang].tx, (float)pk.y - a.angles[ang].ty);
        // ptRotatePt2f(pt, ptCenter, -angle * D2R) (:265-266)
        s.lt = rotate_pt(pt, a.center, a.top_nodes[ang].cn, a.top_nodes[ang].sn);
        if (a.refine) {
            s.alive = 1;
            s.reached0 = mark_reached0;
            const int slot = atomicAdd(a.live_count, 1);
            a.live[slot] = id;
        }
    }
    a.state[id] = s;
}

void launch_cand_init(const CandInitArgs& a, hipStream_t st) {
    if (a.total <= 0) return;
    // mark_reached0 is folded into refine: refine == 2 means the first refinement layer is layer 0
    CandInitArgs b = a;
    const int mark = a.refine == 2 ? 1 : 0;
    if (b.refine) b.refine = 1;
    hipLaunchKernelGGL(k_cand_init, dim3((a.total + 255) / 256), dim3(256), 0, st, b, mark);
}

// ============================================================================================== K2-K5 fused
// The top layer of a small-canvas search (the Src7 case: ~80 x 80 canvases, a 12 x 9 template, plain
// getNextMaxLoc) as ONE workgroup per (source, angle): the rotated canvas (k_warp's fixed-point warp, same
// integers), its NCC map (k_ncc_tile's exact integer sums per 4 outputs by v_dot4 on funnel-shifted words, same
// TM_CCORR rounding and f64 CCOEFF) and the peak loop (k_nms's plain path: painted rectangle + first-max argmax)
// all in LDS -- no canvas or map round trip through HBM and two launches fewer per search.  The engine uses it when
// the plain peak path applies and the largest canvas + map fit top_fused_lds() <= top_fused_lds_limit(); block 0 zeroes the
// search's counters (as k_warp does on the split path).  Src7, 43 sources (1763 jobs): 75.5 us per launch against
// 106.4 for k_warp + k_ncc_tile + k_nms; round-3 ablations (a profiling build, since removed from the product) put
// 21 us in the taps, 19 in the correlation, 3 in the peak loop.
constexpr int kTopThreads = 256;   // k_top_fused workgroup (measured: 512 threads per job no faster)
// one (source, angle) job of k_top_fused (returns when the job is done; the caller separates jobs by a barrier)
__device__ __forceinline__ void top_fused_job(int job, const WarpJob* __restrict__ wjobs,
                                              const NccJob* __restrict__ njobs, const NmsArgs& a,
                                              const CandInitArgs& ci, int ci_mode, uint32_t* tf_lds, float* sv,
                                              int* si, Peak* spk, int* sbase_p) {
    int& sbase = *sbase_p;
    const int tid = threadIdx.x;
    const WarpJob& w = wjobs[job];
    const NccJob& j = njobs[job];
    const int dw = w.dw, dh = w.dh, cpw = ((dw + 3) >> 2) + 1;   // canvas words per row (+1: the funnel reads)
    const int tw = j.tw, th = j.th, ntw = (tw + 3) >> 2, ow = j.ow, oh = j.oh, n = ow * oh;
    if (n <= 0) {   // uniform: no map for this angle (TemplateMatcher.cpp:176-178)
        if (tid == 0) a.counts[job] = 0;
        if (ci_mode) cand_init_job(ci, ci_mode, job, 0, spk, &sbase);
        return;
    }
    uint32_t* Cw = tf_lds;                        // [dh][cpw] canvas, zero past dw
    float* Mp = (float*)(Cw + dh * cpw);          // [oh][ow] map
    uint32_t* Tw = (uint32_t*)(Mp + n);           // [th][ntw] template, zero past tw
    uint32_t* Mw = Tw + th * ntw;                 // [ntw] byte masks of the template width
    int32_t* tab = (int32_t*)(Mw + ntw);          // warpAffine's tables: adelta, bdelta [dw], X0, Y0 [dh]

    for (int x = tid; x < dw; x += kTopThreads) {
        tab[x] = rint_i(w.M[0] * x * kAbScale);
        tab[dw + x] = rint_i(w.M[3] * x * kAbScale);
    }
    for (int y = tid; y < dh; y += kTopThreads) {
        tab[2 * dw + y] = rint_i((w.M[1] * y + w.M[2]) * kAbScale) + kRoundDelta;
        tab[2 * dw + dh + y] = rint_i((w.M[4] * y + w.M[5]) * kAbScale) + kRoundDelta;
    }
    __syncthreads();
    // K2: the rotated canvas, four pixels (one word) per item
    for (int i = tid; i < dh * cpw; i += kTopThreads) {
        const int y = i / cpw, k = i - y * cpw;
        const int X0 = tab[2 * dw + y], Y0 = tab[2 * dw + dh + y];
        uint32_t word = 0;
        for (int b = 0; b < 4; ++b) {   // (measured: branch-free taps with clamped loads are slower, 75 -> 80 us:
            const int x = 4 * k + b;    // the canvas corners outside the image then load too)
            if (x >= dw) break;
            const int ad = tab[x], bd = tab[dw + x];
            const int X = (X0 + ad) >> (kAbBits - kInterBits), Y = (Y0 + bd) >> (kAbBits - kInterBits);
            word |= (uint32_t)warp_tap(w.src, w.sw, w.sh, w.sp, X, Y, w.border) << (8 * b);
        }
        Cw[i] = word;
    }
    for (int i = tid; i < th * ntw; i += kTopThreads) {
        const int r = i / ntw, k = i - r * ntw;
        uint32_t t = 0;
        for (int b = 0; b < 4; ++b)
            if (4 * k + b < tw) t |= (uint32_t)j.tmpl[(size_t)r * j.tp + 4 * k + b] << (8 * b);
        Tw[i] = t;
    }
    if (tid < ntw) {
        uint32_t m = 0;
        for (int b = 0; b < 4; ++b)
            if (4 * tid + b < tw) m |= 1u << (8 * b);
        Mw[tid] = m;
    }
    __syncthreads();
    // K3+K4: 4 adjacent outputs per item, the window sums alongside the correlation (measured: sharing them per
    // band of rows through LDS costs the occupancy it saves in VALU, 75 -> 108 us per 43-source launch); exact u32
    // sums (<= 128 * 64 * 255^2 < 2^32)
    const int ngx = (ow + 3) >> 2;
    for (int it = tid; it < oh * ngx; it += kTopThreads) {
        const int y = it / ngx, q = it - y * ngx;
        uint32_t d[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
        for (int r = 0; r < th; ++r) {
            const uint32_t* ir = Cw + (y + r) * cpw + q;
            const uint32_t* tr = Tw + r * ntw;
            uint32_t w0 = ir[0];
            for (int k = 0; k < ntw; ++k) {
                const uint32_t w1 = ir[k + 1], t = tr[k], m = Mw[k], mff = m * 0xffu;
                const uint32_t sh[4] = {w0, __builtin_amdgcn_alignbyte(w1, w0, 1),
                                        __builtin_amdgcn_alignbyte(w1, w0, 2), __builtin_amdgcn_alignbyte(w1, w0, 3)};
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    d[u] = __builtin_amdgcn_udot4(t, sh[u], d[u], false);
                    s1[u] = __builtin_amdgcn_udot4(m, sh[u], s1[u], false);
                    s2[u] = __builtin_amdgcn_udot4(sh[u] & mff, sh[u], s2[u], false);
                }
                w0 = w1;
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int x = 4 * q + u;
            if (x >= ow) break;
            const double num = (double)(float)(double)(uint64_t)d[u];   // TM_CCORR's f32 result (fold == 0)
            Mp[y * ow + x] = j.equal1 ? 1.f : ccoeff(num, (double)s1[u], (double)s2[u], j.mean, j.norm, j.inv_area);
        }
    }
    __syncthreads();
    // K5 (plain getNextMaxLoc, TemplateMatcher.cpp:197-212 / :1196-1206) on the LDS map
    Peak* out = a.peaks + (size_t)job * a.cap;
    const double ov = a.overlap;
    float v = -INFINITY;
    int i = INT_MAX;
    for (int k = tid; k < n; k += kTopThreads) { const float x = Mp[k]; if (x > v) { v = x; i = k; } }
    wg_argmax(v, i, sv, si);
    if ((double)v < a.thr) {
        if (tid == 0) a.counts[job] = 0;
        if (ci_mode) cand_init_job(ci, ci_mode, job, 0, spk, &sbase);
        return;
    }
    int cnt = 0;
    int px = i % ow, py = i / ow;
    if (tid == 0) {
        out[0].x = px; out[0].y = py; out[0].score = v;
        if (ci_mode) { spk[0].x = px; spk[0].y = py; spk[0].score = v; }
    }
    ++cnt;
    for (int itn = 0; itn < a.cap - 1; ++itn) {
        const int sx = (int)(px - a.tw * (1 - ov)), sy = (int)(py - a.th * (1 - ov));
        const int rw = (int)(2 * a.tw * (1 - ov)), rh = (int)(2 * a.th * (1 - ov));
        if (rw > 0 && rh > 0) {
            const int x1 = sx > 0 ? sx : 0, y1 = sy > 0 ? sy : 0;
            const int x2 = min(sx + rw - 1, ow - 1), y2 = min(sy + rh - 1, oh - 1);
            const int cw = x2 - x1 + 1, ch = y2 - y1 + 1;
            if (cw > 0 && ch > 0)
                for (int k = tid; k < cw * ch; k += kTopThreads) Mp[(y1 + k / cw) * ow + x1 + k % cw] = -1.f;
        }
        __syncthreads();
        v = -INFINITY;
        i = INT_MAX;
        for (int k = tid; k < n; k += kTopThreads) { const float x = Mp[k]; if (x > v) { v = x; i = k; } }
        wg_argmax(v, i, sv, si);
        if ((double)v < a.thr) break;
        px = i % ow;
        py = i / ow;
        if (tid == 0) {
            out[cnt].x = px; out[cnt].y = py; out[cnt].score = v;
            if (ci_mode) { spk[cnt].x = px; spk[cnt].y = py; spk[cnt].score = v; }
        }
        ++cnt;
    }
    if (tid == 0) a.counts[job] = cnt;
    if (ci_mode) cand_init_job(ci, ci_mode, job, cnt, spk, &sbase);
}

// jobs k = blockIdx.x, + gridDim.x, ... in `order` (the grid may be smaller than the job count: FPM_GRID_TOP)
__global__ __launch_bounds__(kTopThreads) void k_top_fused(const WarpJob* __restrict__ wjobs,
                                                           const NccJob* __restrict__ njobs,
                                                           NmsArgs a, int32_t* zero, int nzero,
                                                           CandInitArgs ci, int ci_mode, const int32_t* order,
                                                           int njobs_n) {
    extern __shared__ __attribute__((aligned(16))) uint32_t tf_lds[];
    __shared__ float sv[kTopThreads / 64];
    __shared__ int si[kTopThreads / 64];
    __shared__ Peak spk[kNmsInitCap];   // ci_mode != 0: the job's peaks for cand_init_job
    __shared__ int sbase;
    if (blockIdx.x == 0)
        for (int i = threadIdx.x; i < nzero; i += kTopThreads) zero[i] = 0;
    for (int k = blockIdx.x; k < njobs_n; k += gridDim.x) {
        if (k != (int)blockIdx.x) __syncthreads();   // the previous job is done with the LDS
        top_fused_job(order ? order[k] : k, wjobs, njobs, a, ci, ci_mode, tf_lds, sv, si, spk, &sbase);
    }
}

size_t top_fused_lds(int bw, int bh, int tw, int th) {
    const int cpw = ((bw + 3) >> 2) + 1, ntw = (tw + 3) >> 2;
    const size_t map = (size_t)std::max(bw - tw + 1, 0) * std::max(bh - th + 1, 0);
    return 4 * ((size_t)bh * cpw + map + (size_t)th * ntw + ntw + 2 * ((size_t)bw + bh));
}

// The dynamic LDS a k_top_fused job may use without raising the kernel's 64 KB default launch limit: 64 KB minus
// the kernel's static LDS (peak list, reduction slots), read from the code object once per device
size_t top_fused_lds_limit() {
    int dev = 0;
    (void)hipGetDevice(&dev);
    static std::mutex mu;
    static std::map<int, size_t> lim;
    std::lock_guard<std::mutex> lock(mu);
    auto it = lim.find(dev);
    if (it != lim.end()) return it->second;
    hipFuncAttributes fa{};
    size_t stat = 8192;   // conservative if the query fails
    if (hipFuncGetAttributes(&fa, (const void*)k_top_fused) == hipSuccess) stat = fa.sharedSizeBytes;
    const size_t l = stat < 65536 ? 65536 - stat : 0;
    lim[dev] = l;
    return l;
}

void launch_top_fused(const WarpJob* wjobs, const NccJob* njobs, const NmsArgs& a, int njobs_n, size_t lds,
                      int32_t* zero, int nzero, hipStream_t st, const CandInitArgs* ci, const int32_t* order) {
    if (njobs_n <= 0) return;
    CandInitArgs cz{};
    const bool fuse = ci && a.cap <= kNmsInitCap;
    const int mode = !fuse ? 0 : (ci->refine == 0 ? 1 : (ci->refine == 2 ? 3 : 2));
    if (fuse && zero && nzero > 0 && mode != 1) {
        // block 0's clearing would race the other blocks' live-count atomics: the counters must be zeroed by an
        // earlier launch (the engine passes zero = nullptr then)
        std::fprintf(stderr, "fpm: launch_top_fused contract violated (counter zeroing with candidate-init mode %d)\n",
                     mode);
        std::abort();
    }
    // FPM_GRID_TOP: workgroup cap (a scheduling knob: the jobs loop; read when a search is recorded), 0 / unset: one
    // workgroup per job
    const char* gte = getenv("FPM_GRID_TOP");
    const int grid_cap = gte && atoi(gte) > 0 ? atoi(gte) : 0;
    const int grid = grid_cap > 0 && njobs_n > grid_cap ? grid_cap : njobs_n;
    hipLaunchKernelGGL(k_top_fused, dim3(grid), dim3(kTopThreads), lds, st, wjobs, njobs, a, zero, nzero,
                       fuse ? *ci : cz, mode, order, njobs_n);
}

// ============================================================================================== K6+K7+K8
// Refinement ROIs (getRotatedROI + MatchTemplate(bUseSIMD) + minMaxLoc, TemplateMatcher.cpp:309-328), per layer
// as four kernels over the device-compacted list of live (candidate, angle) ROIs:
//   k_roi_tables  per ROI: the fixed-point warp tables (adelta/bdelta per column, X0/Y0 per row) and one
//                 descriptor per 32x32 tile (source footprint box, interior flag)
//   k_roi_warp    per 32x32 ROI tile and wave: LDS-staged footprint + bilinear gathers -> ROI bytes in HBM
//   k_roi_corr    per (ROI, band of 32 template rows): exact row dot products for all 49 offsets on the matrix
//                 cores + window sums
//   k_roi_eval    per live candidate: ordered f32 fold (:505-508), CCOEFF, argmax, 3x3, candidate step
// (A single fused kernel per layer was measured slower: at its LDS/VGPR footprint the latency-bound sampling
// loses the occupancy it needs; see DESIGN.md.)
// ---- geometry of the refinement scratch ----------------------------------------------------------------------
constexpr int ROI_RC = kMmaRows;     // template rows per correlation chunk
constexpr int ROI_T = 32;            // warp tile: 32 x 32 ROI pixels per wave task
constexpr int ROI_FT = 4096;         // per-wave LDS footprint buffer (bytes) >= worst-case rotated tile bbox
// k_roi_warp's footprint row pitch in LDS: one fixed odd number of dwords (row-strided byte gathers spread over the
// banks) and a compile-time constant, so a tap's second row is the same ds_read's immediate offset and the byte address
// is one multiply-add with a constant; boxes up to 16 dwords wide and ROI_FT / 68 = 60 rows stage into LDS
constexpr int kFtPitch = 68;
// The per-ROI warp tables in HBM (k_roi_tables) carry OpenCV's AB_BITS fixed point scaled by 2^kTabShift: 16
// fractional bits, so in a sum of a row and a column entry the integer coordinate is the high half-word (read by the
// samplers' SDWA word selects, no shift) and OpenCV's INTER_BITS coordinate is the sum >> kTapShift (the scaling is
// exact: (a << 6) + (b << 6) = (a + b) << 6, and every rounding below the 5 kept fraction bits is a floor either way).
constexpr int kTabShift = 6;
constexpr int kTabFrac = kAbBits + kTabShift;           // 16
constexpr int kTapShift = kTabFrac - kInterBits;        // 11
// The ROI scratch holds every sampled byte XOR 0x80 (u8 -> the i8 the matrix cores take, x ^ 0x80 = x - 128): the
// samplers write it flipped (one bit-op per 4 pixels), so k_roi_corr stages rows into LDS as they are
constexpr uint32_t kRoiFlip = 0x80808080u;

int roi_pick_rc(int /*tw*/, int th) { return th < ROI_RC ? th : ROI_RC; }

// ROI row pitch: >= RW + 16 (look-ahead of the 16-byte B reads at shift <= 6) and >= 64*ceil(tw/64) + 22 (the
// MFMA k range), pitch/16 odd (spreads the LDS banks of row-strided 16-byte reads)
__host__ __device__ inline int roi_pitch_calc(int tw) {
    const int need_a = tw + 6 + 16, need_b = 64 * ((tw + 63) / 64) + 22;
    int q = ((need_a > need_b ? need_a : need_b) + 15) / 16;   // in 16-byte units
    if ((q & 1) == 0) ++q;
    return q * 16;
}
int roi_pitch_for(int tw) { return roi_pitch_calc(tw); }
int roi_tab_rows(int th) { return (th + 6 + ROI_T - 1) / ROI_T * ROI_T; }
// Position of ROI row y in a ROI's X0 / Y0 tables: inside each 32-row tile block, rows y, y + 8, y + 16, y + 24 are
// adjacent (k_roi_warp's lane of rows lr + 8i reads its four row origins as one 16-byte load)
__host__ __device__ inline int roi_tab_row_pos(int y) { return (y & ~31) | ((y & 7) << 2) | ((y >> 3) & 3); }
size_t roi_tiles_bytes(int tw, int th) {   // tile-major ROI scratch of one (tw+6) x (th+6) ROI
    return (size_t)((tw + 6 + ROI_T - 1) / ROI_T) * ((th + 6 + ROI_T - 1) / ROI_T) * ROI_T * ROI_T;
}

// LDS row pitch of the staged i8 template rows: >= tp8, pitch/16 odd (conflict-free row-strided b128 reads)
__host__ __device__ inline int tmpl_lds_pitch(int tp8) {
    int q = tp8 / 16;
    if ((q & 1) == 0) ++q;
    return q * 16;
}

size_t roi_corr_lds(int roi_pitch, int tw, int /*rc*/, bool ga) {
    constexpr int src_rows = 2 * kMmaRows + 6;
    const int tp8 = 64 * ((tw + 63) / 64);
    return (size_t)src_rows * roi_pitch + (ga ? 0 : (size_t)2 * kMmaRows * tmpl_lds_pitch(tp8)) +
           sizeof(uint32_t) * (2 * src_rows + 2 * 7 * src_rows + 2 * kMmaRows + 2 * kMmaRows * 49) + 64;
}

// bilinear tap from global memory (fallback when a footprint does not fit the LDS buffer);
// (sum_i w_i v_i + 2^14) >> 15 evaluated as t = 32*h0 + fy*(h1 - h0), h = 32*va + fx*(vb - va) ->
// (t + 512) >> 10: the same integer with fewer multiplies
__device__ __forceinline__ int roi_tap(const uint8_t* __restrict__ src, int sw, int sh, int sp, int X, int Y) {
    const int sx = sat_s16(X >> kInterBits), sy = sat_s16(Y >> kInterBits);
    const int fx = X & (kInterTab - 1), fy = Y & (kInterTab - 1);
    int v0, v1, v2, v3;
    if ((unsigned)sx < (unsigned)(sw - 1) && (unsigned)sy < (unsigned)(sh - 1)) {
        const uint8_t* p = src + (size_t)sy * sp + sx;
        v0 = p[0]; v1 = p[1]; v2 = p[sp]; v3 = p[sp + 1];
    } else if (sx >= sw || sx + 1 < 0 || sy >= sh || sy + 1 < 0) {
        return 0;
    } else {
        const bool x0 = sx >= 0 && sx < sw, x1 = sx + 1 >= 0 && sx + 1 < sw;
        const bool y0 = sy >= 0 && sy < sh, y1 = sy + 1 >= 0 && sy + 1 < sh;
        const uint8_t* r0 = src + (size_t)sy * sp;
        const uint8_t* r1 = r0 + sp;
        v0 = x0 && y0 ? r0[sx] : 0;
        v1 = x1 && y0 ? r0[sx + 1] : 0;
        v2 = x0 && y1 ? r1[sx] : 0;
        v3 = x1 && y1 ? r1[sx + 1] : 0;
    }
    const int h0 = 32 * v0 + fx * (v1 - v0), h1 = 32 * v2 + fx * (v3 - v2);
    return (32 * h0 + fy * (h1 - h0) + 512) >> 10;
}

// a * b + c on the 24-bit multiplier (|a|, |b| < 2^23): written out because the compiler otherwise re-associates
// such footprint offsets into the quarter-rate v_mad_u64_u32
__device__ __forceinline__ int mad24(int a, int b, int c) {
    int d;
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

// interior bilinear tap from an LDS footprint FT (16-byte aligned; tap (sx, sy) at byte offset off, row pitch
// ftw): per tap row one aligned dword pair (ds_read2_b32) funnel-shifted to the tap's byte (v_alignbyte uses the
// offset's low two bits; unaligned 32-bit DS reads measured 2.5x slower than byte gathers), the horizontal passes
// as u8 dot products with the per-axis weights (32 - fx, fx, 0, 0), the vertical pass as 24-bit multiply-adds:
// the same integer as roi_tap's (32*h0 + fy*(h1 - h0) + 512) >> 10.  The footprint buffers carry >= 4 bytes of
// slack after their last row (the pair's second dword).
__device__ __forceinline__ int ft_tap_interior(const uint8_t* FT, int off, int ftw, int X, int Y) {
    const uint32_t fx = X & (kInterTab - 1), fy = Y & (kInterTab - 1);
    const uint32_t* F = (const uint32_t*)FT;
    const int off1 = off + ftw;
    const uint32_t* q0 = F + (off >> 2);
    const uint32_t* q1 = F + (off1 >> 2);
    const uint32_t r0 = __builtin_amdgcn_alignbyte(q0[1], q0[0], (uint32_t)off);
    const uint32_t r1 = __builtin_amdgcn_alignbyte(q1[1], q1[0], (uint32_t)off1);
    const uint32_t wx = 32u + fx * 255u;
    const uint32_t h0 = __builtin_amdgcn_udot4(r0, wx, 0u, false), h1 = __builtin_amdgcn_udot4(r1, wx, 0u, false);
    return (int)((__umul24(32u - fy, h0) + __umul24(fy, h1) + 512u) >> 10);
}

// the same tap by four byte gathers (p = tap (sx, sy))
__device__ __forceinline__ int ft_tap_bytes(const uint8_t* FT, int off, int ftw, int X, int Y) {
    const int fx = X & (kInterTab - 1), fy = Y & (kInterTab - 1);
    const uint8_t* p = FT + off;
    const int v0 = p[0], v1 = p[1], v2 = p[ftw], v3 = p[ftw + 1];
    const int h0 = 32 * v0 + __mul24(fx, v1 - v0), h1 = 32 * v2 + __mul24(fx, v3 - v2);
    return (32 * h0 + __mul24(fy, h1 - h0) + 512) >> 10;
}

// Interior taps addressed directly in the LDS address space: the caller offsets the fixed-point row coordinates by
// whole multiples of 2^10 per tile so that (X0 + ad) >> 10 is the tap's column inside the wave's footprint plus the
// footprint's LDS byte offset and (Y0 + bd) >> 10 its footprint row; the byte address is then one 24-bit
// multiply-add and every ds_read carries its own offset (no base adds), fractions untouched.
typedef __attribute__((address_space(3))) const uint8_t fpm_lds_u8;
__device__ __forceinline__ uint32_t lds_offset_of(const uint8_t* p) { return (uint32_t)(size_t)(fpm_lds_u8*)p; }
// the four taps of one pixel: (p, p + 1) and (p + ftw, p + ftw + 1)
__device__ __forceinline__ void lds_taps(uint32_t off, int ftw, int v[4]) {
    fpm_lds_u8* p = (fpm_lds_u8*)(size_t)off;
    fpm_lds_u8* q = (fpm_lds_u8*)(size_t)(off + ftw);
    v[0] = p[0]; v[1] = p[1]; v[2] = q[0]; v[3] = q[1];
}
// (32*h0 + fy*(h1 - h0) + 512) >> 10 with h = 32*va + fx*(vb - va), on the 24-bit multiplier only
__device__ __forceinline__ int bilerp24(const int v[4], int fx, int fy) {
    const int h0 = mad24(fx, v[1] - v[0], v[0] << 5), h1 = mad24(fx, v[3] - v[2], v[2] << 5);
    return mad24(fy, h1 - h0, (h0 << 5) + 512) >> 10;
}
// The same integers for the four pixels of one output row, packed into a dword (pixel u in byte u), in 7 VALU per
// pixel + 3 per row instead of 12 per pixel (k_roi_warp's row: 64 VALU instead of 77): the two tap rows' horizontal passes run as one pair of 16-bit lanes (h = 32 va + fx (vb - va)
// <= 8160; lane arithmetic mod 2^16, exact since the true value fits), fx taken from the low half of its register by
// op_sel (no splat), the vertical pass as one u16 dot product with the weights (64 (32 - fy), 64 fy) plus 64 * 512:
// 64 * (32 h0 + fy (h1 - h0) + 512) < 2^24, so the result byte is bits 16..23 and two byte permutes + one bitwise op
// pack the row.  Taps must be zero-extended bytes (lds_taps16).  (Reading the taps straight into the lane pairs with
// ds_read_u8_d16 / _d16_hi does not work on gfx950: with SRAM ECC the D16 loads zero the other half of the register
// instead of preserving it -- found by the GPU suite, round 4 -- so the two halves would need an OR: no saving.)
typedef unsigned short fpm_u16x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t bilerp_row4(const int v[4][4], const int fx[4], const int fy[4]) {
    uint32_t r[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const uint32_t a02 = __builtin_amdgcn_perm((uint32_t)v[u][2], (uint32_t)v[u][0], 0x0c040c00u);   // (v0, v2)
        const uint32_t a13 = __builtin_amdgcn_perm((uint32_t)v[u][3], (uint32_t)v[u][1], 0x0c040c00u);   // (v1, v3)
        const fpm_u16x2v d = __builtin_bit_cast(fpm_u16x2v, a13) - __builtin_bit_cast(fpm_u16x2v, a02);
        const fpm_u16x2v b = __builtin_bit_cast(fpm_u16x2v, a02) << (fpm_u16x2v)5;
        uint32_t h;
        asm("v_pk_mad_u16 %0, %1, %2, %3 op_sel_hi:[0,1,1]"
            : "=v"(h) : "v"(fx[u]), "v"(__builtin_bit_cast(uint32_t, d)), "v"(__builtin_bit_cast(uint32_t, b)));
        const uint32_t wy = (uint32_t)mad24(fy[u], 64 * 0x10000 - 64, 64 * 32);   // (64 (32 - fy), 64 fy)
        r[u] = __builtin_amdgcn_udot2(__builtin_bit_cast(fpm_u16x2v, h), __builtin_bit_cast(fpm_u16x2v, wy), 64u * 512u,
                                      false);
    }
    return __builtin_amdgcn_perm(r[1], r[0], 0x0c0c0602u) | __builtin_amdgcn_perm(r[3], r[2], 0x06020c0cu);
}
// The 16 taps of one output row (4 pixels x 2 rows x 2 columns) at a compile-time pitch, all issued before any use:
// explicit ds_read_u8 (zero-extending; the compiler's own form re-masks every result with 0xff when it feeds 16-bit
// lanes) and one lgkmcnt(0) that the results depend on.  Half as many reads as ds_read_u16 pairs (each tap row's two
// columns, at byte-aligned addresses) give the same bytes but ran 4.2x slower (k_roi_warp3 layer-0 microbenchmark
// 1689 vs 399 us, round 3): the LDS serves unaligned halfwords, slowly.
template <int PITCH>
__device__ __forceinline__ void lds_taps16(const uint32_t off[4], int v[4][4]) {
    // one statement: the 16 reads and the wait they end with (no compiler-placed copy of a result register can
    // come between a read and its wait)
    asm volatile("ds_read_u8 %0, %16\n\tds_read_u8 %1, %16 offset:1\n\tds_read_u8 %2, %16 offset:%20\n\t"
                 "ds_read_u8 %3, %16 offset:%21\n\t"
                 "ds_read_u8 %4, %17\n\tds_read_u8 %5, %17 offset:1\n\tds_read_u8 %6, %17 offset:%20\n\t"
                 "ds_read_u8 %7, %17 offset:%21\n\t"
                 "ds_read_u8 %8, %18\n\tds_read_u8 %9, %18 offset:1\n\tds_read_u8 %10, %18 offset:%20\n\t"
                 "ds_read_u8 %11, %18 offset:%21\n\t"
                 "ds_read_u8 %12, %19\n\tds_read_u8 %13, %19 offset:1\n\tds_read_u8 %14, %19 offset:%20\n\t"
                 "ds_read_u8 %15, %19 offset:%21\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&v"(v[0][0]), "=&v"(v[0][1]), "=&v"(v[0][2]), "=&v"(v[0][3]), "=&v"(v[1][0]), "=&v"(v[1][1]),
                   "=&v"(v[1][2]), "=&v"(v[1][3]), "=&v"(v[2][0]), "=&v"(v[2][1]), "=&v"(v[2][2]), "=&v"(v[2][3]),
                   "=&v"(v[3][0]), "=&v"(v[3][1]), "=&v"(v[3][2]), "=&v"(v[3][3])
                 : "v"(off[0]), "v"(off[1]), "v"(off[2]), "v"(off[3]), "i"(PITCH), "i"(PITCH + 1)
                 : "memory");
}

// One bilinear ROI pixel from a staged footprint, BORDER_CONSTANT(0) rules of remapBilinear (general path).
__device__ __forceinline__ int ft_tap_general(const uint8_t* FT, int ftw, int bxa, int by0, int W, int H, int X, int Y) {
    const int sx = sat_s16(X >> kInterBits), sy = sat_s16(Y >> kInterBits);
    const int fx = X & (kInterTab - 1), fy = Y & (kInterTab - 1);
    const uint8_t* p = FT + (sy - by0) * ftw + (sx - bxa);
    int v0, v1, v2, v3;
    if ((unsigned)sx < (unsigned)(W - 1) && (unsigned)sy < (unsigned)(H - 1)) {
        v0 = p[0]; v1 = p[1]; v2 = p[ftw]; v3 = p[ftw + 1];
    } else if (sx >= W || sx + 1 < 0 || sy >= H || sy + 1 < 0) {
        return 0;
    } else {
        const bool x0 = sx >= 0 && sx < W, x1 = sx + 1 >= 0 && sx + 1 < W;
        const bool y0 = sy >= 0 && sy < H, y1 = sy + 1 >= 0 && sy + 1 < H;
        v0 = x0 && y0 ? p[0] : 0;
        v1 = x1 && y0 ? p[1] : 0;
        v2 = x0 && y1 ? p[ftw] : 0;
        v3 = x1 && y1 ? p[ftw + 1] : 0;
    }
    const int h0 = 32 * v0 + fx * (v1 - v0), h1 = 32 * v2 + fx * (v3 - v2);
    return (32 * h0 + fy * (h1 - h0) + 512) >> 10;
}

// this launch's live ROIs [slot_base, slot_base + count) (the host's rounds of whole candidates)
__device__ __forceinline__ int roi_base(const RoiArgs& a) { return a.slot_base; }
__device__ __forceinline__ void roi_slot(const RoiArgs& a, int slot, int& id, int& jj) {
    const int ri = roi_base(a) + slot;
    const int li = ri / a.n3;
    jj = ri - li * a.n3;
    id = a.live[li];
}

__device__ __forceinline__ int roi_count(const RoiArgs& a) {
    int rois = *a.live_count * a.n3 - roi_base(a);
    return rois < 0 ? 0 : (rois > a.slot_cap ? a.slot_cap : rois);
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Global -> LDS staging with several loads in flight per thread (a load-then-store loop would otherwise wait one
// full memory round trip per iteration).
// (a) footprint rows of a tile: lane -> word column lane & 15 (< wpr), rows (lane >> 4) + 4i
template <int B>
__device__ __forceinline__ void stage_footprint(uint8_t* FT, int ftw, int wpr, int fth, const uint8_t* gsrc,
                                                size_t gpitch, int gx0, int gP, int lane) {
    const int c = lane & 15;
    if (c >= wpr) return;
    const int gx = gx0 + 4 * c;
    const bool inb = gx < gP;
    const uint8_t* gp = gsrc + 4 * c + (size_t)(lane >> 4) * gpitch;
    uint8_t* lp = FT + 4 * c + (lane >> 4) * ftw;
    const size_t gstep = 4 * gpitch;
    const int lstep = 4 * ftw;
    for (int r0 = lane >> 4; r0 < fth; r0 += 4 * B) {   // B rows' loads in flight (VGPRs vs occupancy)
        uint32_t v[B];
#pragma unroll
        for (int i = 0; i < B; ++i) v[i] = (inb && r0 + 4 * i < fth) ? *(const uint32_t*)(gp + i * gstep) : 0u;
#pragma unroll
        for (int i = 0; i < B; ++i)
            if (r0 + 4 * i < fth) *(uint32_t*)(lp + i * lstep) = v[i];
        gp += B * gstep;
        lp += B * lstep;
    }
}
// (a') the same footprint through LDS-DMA (global_load_lds_dword): dword L of the row-major footprint (pitch wpr
// words) comes from lane L % 64 of instruction L / 64, whose LDS destination is the wave-uniform FT + 4*64*(L/64);
// every load of the tile is in flight at once and no VGPR holds data.  Columns past the image edge read the
// row's pitch slack / next row (never sampled: the box already carries the +2 tap margin).
typedef __attribute__((address_space(3))) void* fpm_lds_vp;
typedef __attribute__((address_space(1))) void* fpm_gbl_vp;
__device__ __forceinline__ void stage_footprint_dma(uint8_t* FT, int wpr, int fth, const uint8_t* gsrc,
                                                    size_t gpitch, int lane) {
    const int total = wpr * fth;
    int r = lane / wpr, c = lane - r * wpr;
    const int dr = 64 / wpr, dc = 64 - dr * wpr;
    for (int i0 = 0; i0 < total; i0 += 64) {
        if (i0 + lane < total)
            __builtin_amdgcn_global_load_lds((fpm_gbl_vp)(gsrc + (size_t)r * gpitch + 4 * c), (fpm_lds_vp)(FT + 4 * i0), 4, 0, 0);
        r += dr;
        c += dc;
        if (c >= wpr) { c -= wpr; ++r; }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// (b) a rows x q16 block of 16-byte vectors (workgroup-wide, nthr threads): dst pitch dp, src pitch sp
__device__ __forceinline__ void stage_block16(uint8_t* dst, int dp, const uint8_t* src, size_t sp, int rows, int q16,
                                              int tid, int nthr) {
    const int total = rows * q16;
    int r = tid / q16, c = tid - (tid / q16) * q16;     // (r, c) of element tid, advanced by nthr per step
    const int dr = nthr / q16, dc = nthr - dr * q16;
    for (int i0 = tid; i0 < total; i0 += 4 * nthr) {
        uint4 v[4];
        int rr[4], cc[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            rr[k] = r; cc[k] = c;
            v[k] = (i0 + k * nthr < total) ? *(const uint4*)(src + (size_t)r * sp + 16 * c) : make_uint4(0, 0, 0, 0);
            r += dr; c += dc;
            if (c >= q16) { c -= q16; ++r; }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (i0 + k * nthr < total) *(uint4*)(dst + (size_t)rr[k] * dp + 16 * cc[k]) = v[k];
    }
}
// (c) a rows x wpr block of dwords (workgroup-wide), zero where the source column gx0 + 4c >= gP
__device__ __forceinline__ void stage_block4(uint8_t* dst, int dp, const uint8_t* src, size_t sp, int rows, int wpr,
                                             int gx0, int gP, int tid, int nthr) {
    const int total = rows * wpr;
    int r = tid / wpr, c = tid - (tid / wpr) * wpr;
    const int dr = nthr / wpr, dc = nthr - dr * wpr;
    for (int i0 = tid; i0 < total; i0 += 8 * nthr) {
        uint32_t v[8];
        int rr[8], cc[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            rr[k] = r; cc[k] = c;
            v[k] = (i0 + k * nthr < total && gx0 + 4 * c < gP) ? *(const uint32_t*)(src + (size_t)r * sp + 4 * c) : 0u;
            r += dr; c += dc;
            if (c >= wpr) { c -= wpr; ++r; }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (i0 + k * nthr < total) *(uint32_t*)(dst + (size_t)rr[k] * dp + 4 * cc[k]) = v[k];
    }
}

// ---- K6a: per-ROI fixed-point warp tables (getRotatedROI -> warpAffine's adelta/bdelta/X0/Y0) and, from them,
// one descriptor per 32x32 ROI tile: the tile's source footprint box (corner samples +-1 px: the fixed-point map
// is two roundings of a linear map, so every pixel's tap lies within the corners' range +-1) and flags
// (bit0: footprint non-empty, bit1: fits the per-wave LDS buffer, bit2: every tap inside the image) with the ROI's
// source index above them (bits 8 and up: k_roi_warp then needs neither the candidate id nor a division per task).
constexpr int kTileAny = 1, kTileLds = 2, kTileInterior = 4, kTileSrcShift = 8;
int roi_tiles_for(int tw, int th) { return ((tw + 6 + ROI_T - 1) / ROI_T) * ((th + 6 + ROI_T - 1) / ROI_T); }

// The tables and descriptors of one ROI (slot) from its candidate's ptLT and angle node, by threads t0, t0 + nt, ...
// of the caller.  The descriptors' corner samples recompute the same fixed-point rows and columns (pure functions of
// M), so the threads need no LDS copy of the tables and no barrier.  Used by k_roi_tables and, for the next layer's
// survivors, by the steps in k_roi_eval / k_cand_step_tab (RoiArgs::nt_tab).
__device__ void roi_tables_fill(int32_t* tab, int4* tdesc, int tdesc_stride, int tabw, int tabh, int tw, int th,
                                int W, int H, int slot, F2 lt, const AngleNode& nd, int src_bits, int t0, int nt) {
    const int RW = tw + 6, RH = th + 6;
    const int txn = (RW + ROI_T - 1) / ROI_T, tyn = (RH + ROI_T - 1) / ROI_T;
    double M[6];
    roi_matrix(W, H, f2(lt.x * 2, lt.y * 2), nd.c, nd.s, M);
    int32_t* t = tab + (size_t)slot * 2 * (tabw + tabh);
    for (int x = t0; x < tabw; x += nt) {
        const int ad = rint_i(M[0] * x * kAbScale), bd = rint_i(M[3] * x * kAbScale);
        t[x] = ad * (1 << kTabShift); t[tabw + x] = bd * (1 << kTabShift);
    }
    for (int y = t0; y < tabh; y += nt) {
        // rows past the ROI (the last tile block's padding) repeat its last row: k_roi_warp reads them unclamped
        const int yc = min(y, RH - 1);
        const int x0 = rint_i((M[1] * yc + M[2]) * kAbScale) + kRoundDelta;
        const int y0 = rint_i((M[4] * yc + M[5]) * kAbScale) + kRoundDelta;
        const int q = roi_tab_row_pos(y);
        t[2 * tabw + q] = x0 * (1 << kTabShift); t[2 * tabw + tabh + q] = y0 * (1 << kTabShift);
    }
    for (int i = t0; i < txn * tyn; i += nt) {
        const int ty = i / txn, tx = i - ty * txn;
        const int cx0 = tx * ROI_T, cx1 = min(cx0 + ROI_T, RW) - 1;
        const int ry0 = ty * ROI_T, ry1 = min(ry0 + ROI_T, RH) - 1;
        int bx0 = INT_MAX, bx1 = INT_MIN, by0 = INT_MAX, by1 = INT_MIN;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int c = (k & 1) ? cx1 : cx0, r = (k & 2) ? ry1 : ry0;
            const int ad = rint_i(M[0] * c * kAbScale), bd = rint_i(M[3] * c * kAbScale);
            const int x0 = rint_i((M[1] * r + M[2]) * kAbScale) + kRoundDelta;
            const int y0 = rint_i((M[4] * r + M[5]) * kAbScale) + kRoundDelta;
            const int X = (x0 + ad) >> (kAbBits - kInterBits);
            const int Y = (y0 + bd) >> (kAbBits - kInterBits);
            bx0 = min(bx0, X >> kInterBits); bx1 = max(bx1, X >> kInterBits);
            by0 = min(by0, Y >> kInterBits); by1 = max(by1, Y >> kInterBits);
        }
        const bool interior = bx0 - 1 >= 0 && bx1 + 1 <= W - 2 && by0 - 1 >= 0 && by1 + 1 <= H - 2;
        bx0 = max(bx0 - 1, 0); by0 = max(by0 - 1, 0);
        bx1 = min(bx1 + 2, W - 1); by1 = min(by1 + 2, H - 1);
        const bool any = bx0 <= bx1 && by0 <= by1;
        const int bxa = bx0 & ~3;
        const int wpr = any ? (bx1 - bxa + 4) >> 2 : 0;   // dwords per footprint row
        const int fth = any ? by1 - by0 + 1 : 0;
        const bool in_lds = wpr <= 16 && kFtPitch * fth <= ROI_FT;
        tdesc[(size_t)slot * tdesc_stride + i] =
            make_int4(bxa, by0, wpr | (fth << 16),
                      (any ? kTileAny : 0) | (in_lds ? kTileLds : 0) | (interior ? kTileInterior : 0) | src_bits);
    }
}

__global__ __launch_bounds__(256) void k_roi_tables(RoiArgs a) {
    const int rois = roi_count(a);
    for (int slot = blockIdx.x; slot < rois; slot += gridDim.x) {
        int id, jj;
        roi_slot(a, slot, id, jj);
        const CandState st = a.state[id];
        const AngleNode nd = a.nodes[st.node * a.n3 + jj];
        roi_tables_fill(a.tab, a.tdesc, a.tdesc_stride, a.tabw, a.tabh, a.tw, a.th, a.W, a.H, slot, st.lt, nd,
                        (id / a.per_source) << kTileSrcShift, threadIdx.x, 256);
    }
}

// ---- K6b: ROI sampling.  One wave = one 32x32 ROI tile at a time: the tile's source footprint is staged into
// wave-private LDS with dword loads; every lane produces 4 rows x 4 pixels by gathering the bilinear taps from LDS and
// stores them as dwords.  Interior tiles take a branch-free path; others follow remapBilinear's BORDER_CONSTANT(0)
// rules per pixel.  No workgroup barrier.
// The task bookkeeping is wave-uniform and stays off the VALU: the task index is made uniform (readfirstlane of the
// wave id), so its decode into (slot, tile row, tile column) and the per-ROI data (source level, table base) run on
// the scalar unit; footprint loads and ROI stores address a uniform base plus 32-bit lane offsets.  (Round 2's form
// decoded every task with integer divisions on the VALU and built 64-bit addresses per lane: ~180 of the ~630 VALU
// instructions a layer-0 tile cost, in a kernel that is VALU-issue bound.)
// loads / stores at a wave-uniform base + a 32-bit lane byte offset (the saddr + voffset form: no 64-bit address
// arithmetic per lane)
template <typename T>
__device__ __forceinline__ T ld_at(const void* base, uint32_t byte_off) {
    return *(const T*)((const char*)base + (size_t)byte_off);
}
template <typename T>
__device__ __forceinline__ void st_at(void* base, uint32_t byte_off, T v) {
    *(T*)((char*)base + (size_t)byte_off) = v;
}

// the footprint box of a tile: dword column lane & 15 (< wpr), rows (lane >> 4) + 4k for k < ceil(fth / 4), B rows in
// flight; gsrc is the wave-uniform box origin in the source level (pitch gpitch).  Every condition is wave-uniform
// (the row count per lane is ceil(fth / 4) for all lanes; a lane group whose last row lies past the box re-stages
// row fth - 1, the same bytes to the same place), so the loop is straight-line code with scalar branches only.
template <int B, int PITCH>
__device__ __forceinline__ void stage_footprint32(uint8_t* FT, int wpr, int fth, const uint8_t* gsrc, int gpitch,
                                                  int lane) {
    const int c = lane & 15;
    if (c >= wpr) return;
    // columns past the box read the row's pitch slack or the next row (the level images carry one spare row): those
    // bytes land in footprint columns no tap reads (the box already holds the +2 tap margin)
    const int rl = lane >> 4, rlast = fth - 1, n = (fth + 3) >> 2;
    fpm_lds_u8* ft = (fpm_lds_u8*)(size_t)(lds_offset_of(FT) + 4u * c);
    for (int k0 = 0; k0 < n; k0 += B) {
        uint32_t v[B];
        int r[B];
#pragma unroll
        for (int i = 0; i < B; ++i) {
            r[i] = min(rl + 4 * (k0 + i), rlast);
            if (k0 + i < n) v[i] = ld_at<uint32_t>(gsrc, (uint32_t)mad24(r[i], gpitch, 4 * c));
        }
#pragma unroll
        for (int i = 0; i < B; ++i)
            if (k0 + i < n) *(__attribute__((address_space(3))) uint32_t*)(ft + mad24(r[i], PITCH, 0)) = v[i];
    }
}

// FB: footprint rows in flight per lane (0 = LDS-DMA).  ABL (profiling ablations, product 0): 1 = no footprint
// staging, 2 = no gathers (stores zeros), 3 = tables + descriptor only, 4 = dot-product interior taps (ft_tap_interior),
// 5 = no ROI stores (interior rows computed, a never-true store kept), 6 = neither staging nor stores, 7 = as 6 with
// synthetic taps (no LDS reads), 8 = as 6 with the taps XOR-folded (no bilinear arithmetic), 9 = as 6 with two tap
// reads per pixel (the other two taps copied: LDS instruction count halved, arithmetic unchanged)
template <int FB, int ABL = 0, int WPE = 7>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_roi_warp(RoiArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t ft_all[4 * ROI_FT + 16];   // + slack for ft_tap_interior
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t* FT = ft_all + wv * ROI_FT;
    const int RW = a.tw + 6, RH = a.th + 6, W = a.W, H = a.H;
    const int txn = (RW + ROI_T - 1) / ROI_T, tyn = (RH + ROI_T - 1) / ROI_T;
    const int per_roi = txn * tyn;
    const int tasks = roi_count(a) * per_roi;
    const int lr = lane >> 3, lg = lane & 7;   // lane -> rows lr + 8i, columns 4*lg .. 4*lg+3
    // XCD groups take contiguous task ranges (a tile's neighbours and the candidate's other angle ROIs -- nearly the
    // same source region -- are staged through one L2), and inside a group the workgroups sweep that range together
    // (task = lo + 4 k + wave, stride 4 nk): at any time the group works on one window of neighbouring tiles.
    // (Measured: one contiguous run per wave instead loses that shared window, 241 -> 278 us per 43-source launch.)
    const XcdSplit xs = xcd_split(tasks);
    const int tstride = xs.nk * 4;
    const uint32_t st_lane = 4u * lg + 32u * lr;   // the lane's byte offset in a 1 KB ROI tile (row lr, column 4*lg)
    int task = xs.lo + xs.k * 4 + wv;
    if (task >= xs.hi) return;
    // The next task's tile descriptor (footprint box, flags, source index) is loaded one task ahead, during the current
    // task's gathers: the footprint loads then start as soon as a task begins instead of after a dependent global round
    // trip.  Wave-uniform values, carried in 4 VGPRs.
    int4 nd;
    auto prefetch = [&](int t) {
        const int s_ = t / per_roi;
        nd = a.tdesc[(size_t)s_ * a.tdesc_stride + (t - s_ * per_roi)];
    };
    prefetch(task);
    for (; task < xs.hi; task += tstride) {
        // wave-uniform, so on the scalar unit
        const int slot = task / per_roi;
        const int rem = task - slot * per_roi;
        const int ty = rem / txn, tx = rem - ty * txn;
        const int32_t* tb = a.tab + (size_t)slot * 2 * (a.tabw + a.tabh);   // this ROI's warp tables
        const int cx0 = tx * ROI_T, cx1 = min(cx0 + ROI_T, RW) - 1;
        const int ry0 = ty * ROI_T, ry1 = min(ry0 + ROI_T, RH) - 1;
        const int c0 = cx0 + 4 * lg;
        const int4 dsc = nd;
        const int flags = __builtin_amdgcn_readfirstlane(dsc.w);
        const bool in_lds = (flags & kTileLds) != 0;
        const int cc = min(c0, cx1 & ~3);   // tables are read in bounds even for idle lanes
        const int4 A = ld_at<int4>(tb, 4u * cc);
        const int4 B = ld_at<int4>(tb, 4u * (a.tabw + cc));
        const int adv[4] = {A.x, A.y, A.z, A.w}, bdv[4] = {B.x, B.y, B.z, B.w};
        // the lane's rows ry0 + lr + 8i: one 16-byte load each for X0 and Y0 (roi_tab_row_pos; rows past the ROI hold
        // its last row)
        const int4 X4 = ld_at<int4>(tb, 4u * (2 * a.tabw + ry0 + 4 * lr));
        const int4 Y4 = ld_at<int4>(tb, 4u * (2 * a.tabw + a.tabh + ry0 + 4 * lr));
        const int X0r[4] = {X4.x, X4.y, X4.z, X4.w}, Y0r[4] = {Y4.x, Y4.y, Y4.z, Y4.w};
        uint8_t* tile = a.roi + (size_t)slot * a.roi_stride + ((size_t)rem << 10);   // tile-major: (ty, tx) = rem

        const int bxa = __builtin_amdgcn_readfirstlane(dsc.x), by0 = __builtin_amdgcn_readfirstlane(dsc.y);
        const int dz = __builtin_amdgcn_readfirstlane(dsc.z);
        const int wpr = dz & 0xffff, fth = dz >> 16;
        const uint8_t* lvl = a.level + (size_t)(flags >> kTileSrcShift) * a.level_stride;   // its source level
        constexpr int ftw = kFtPitch;
        wave_sync();   // previous task's gathers are done with FT
        if (ABL != 1 && ABL != 3 && ABL < 6 && (flags & kTileAny) && in_lds) {
            if constexpr (FB == 0) stage_footprint_dma(FT, wpr, fth, lvl + (size_t)by0 * a.P + bxa, a.P, lane);
            else stage_footprint32<FB, kFtPitch>(FT, wpr, fth, lvl + (size_t)by0 * a.P + bxa, a.P, lane);
        }
        if (task + tstride < xs.hi) prefetch(task + tstride);
        wave_sync();
        if (c0 > cx1) continue;
        // tile-major ROI scratch: tile (ty, tx) is a contiguous 32 x 32 block, so one store instruction of the wave
        // (8 rows x 8 lanes x 4 bytes) writes 256 contiguous bytes
        if (ABL == 3) continue;
        if (ABL == 2) {
            for (int i = 0; i < 4; ++i)
                if (ry0 + lr + 8 * i <= ry1) st_at<uint32_t>(tile, st_lane + 256u * i, (uint32_t)(X0r[i] ^ Y0r[i] ^ adv[0] ^ bdv[3]));
            continue;
        }
        if (ABL == 0 && !(flags & kTileAny)) {   // footprint outside the level: zeros, stored flipped (as k_roi_warp3)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (ry0 + lr + 8 * i <= ry1) st_at<uint32_t>(tile, st_lane + 256u * i, kRoiFlip);
            continue;
        }
        if ((flags & kTileInterior) && in_lds && ABL == 4) {
            const int obase = by0 * ftw + bxa;
            const int nvalid = RW - c0;
            const uint32_t colmask = nvalid >= 4 ? 0xffffffffu : (1u << (8 * nvalid)) - 1u;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (ry0 + lr + 8 * i > ry1) break;
                uint32_t pk = 0;
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int X = (X0r[i] + adv[u]) >> kTapShift;
                    const int Y = (Y0r[i] + bdv[u]) >> kTapShift;
                    const int off = mad24(Y >> kInterBits, ftw, (X >> kInterBits) - obase);
                    pk |= (uint32_t)ft_tap_interior(FT, off, ftw, X, Y) << (8 * u);
                }
                st_at<uint32_t>(tile, st_lane + 256u * i, (pk & colmask) ^ kRoiFlip);
            }
            continue;
        }
        if ((flags & kTileInterior) && in_lds) {
            // columns past the ROI's right edge are zero: one byte mask per lane instead of a select per pixel
            const int nvalid = RW - c0;
            const uint32_t colmask = nvalid >= 4 ? 0xffffffffu : (1u << (8 * nvalid)) - 1u;
            const int xo = ((int)lds_offset_of(FT) - bxa) << kTabFrac, yo = -(by0 << kTabFrac);
            // one output row (4 pixels) at a time: all 16 tap reads issued before any arithmetic (measured: 126.8 ->
            // 113.1 us per Src7 layer-0 launch at 8 sources with the folded addressing, scripts/warp_exp.hip; rows
            // past the tile repeat its last row's coordinates and are not stored)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int x0r = X0r[i] + xo, y0r = Y0r[i] + yo;
                uint32_t off[4];
                int fxv[4], fyv[4], v[4][4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int sxv = x0r + adv[u], syv = y0r + bdv[u];
                    fxv[u] = __builtin_amdgcn_ubfe(sxv, kTapShift, kInterBits);
                    fyv[u] = __builtin_amdgcn_ubfe(syv, kTapShift, kInterBits);
                    off[u] = (uint32_t)mad24(syv >> kTabFrac, ftw, sxv >> kTabFrac);
                }
                // the 16 reads together ahead of the arithmetic (measured: the compiler's scheduling otherwise
                // interleaves them with waits, 241 -> 280 us per launch)
                if constexpr (ABL == 7) {
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        for (int k = 0; k < 4; ++k) v[u][k] = (off[u] >> (2 * k)) & 0xff;
                } else if constexpr (ABL == 9) {
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        asm volatile("ds_read_u8 %0, %2\n\tds_read_u8 %1, %2 offset:%3" : "=&v"(v[u][0]), "=&v"(v[u][2]) : "v"(off[u]), "i"(kFtPitch));
                    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0][0]), "+v"(v[0][2]), "+v"(v[1][0]), "+v"(v[1][2]), "+v"(v[2][0]), "+v"(v[2][2]), "+v"(v[3][0]), "+v"(v[3][2]) :: "memory");
#pragma unroll
                    for (int u = 0; u < 4; ++u) { v[u][1] = v[u][0]; v[u][3] = v[u][2]; }
                } else {
                    lds_taps16<kFtPitch>(off, v);
                }
                uint32_t pk;
                if constexpr (ABL == 8) {
                    pk = 0;
#pragma unroll
                    for (int u = 0; u < 4; ++u) pk ^= (uint32_t)(v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3]) << u;
                } else {
                    pk = bilerp_row4(v, fxv, fyv);
                }
                if (ABL >= 5) {
                    if ((pk & colmask) == 0x9e3779b9u && (lane ^ bxa) == 977) st_at<uint32_t>(tile, st_lane, pk);
                } else if (ry0 + lr + 8 * i <= ry1) {
                    st_at<uint32_t>(tile, st_lane + 256u * i, (pk & colmask) ^ kRoiFlip);
                }
            }
            continue;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (ry0 + lr + 8 * i > ry1) break;
            uint32_t pk = 0;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int X = (X0r[i] + adv[u]) >> kTapShift;
                const int Y = (Y0r[i] + bdv[u]) >> kTapShift;
                int v;
                if (in_lds) {
                    const int sx = sat_s16(X >> kInterBits), sy = sat_s16(Y >> kInterBits);
                    const int fx = X & (kInterTab - 1), fy = Y & (kInterTab - 1);
                    const uint8_t* p = FT + (sy - by0) * ftw + (sx - bxa);
                    int v0, v1, v2, v3;
                    if ((unsigned)sx < (unsigned)(W - 1) && (unsigned)sy < (unsigned)(H - 1)) {
                        v0 = p[0]; v1 = p[1]; v2 = p[ftw]; v3 = p[ftw + 1];
                    } else if (sx >= W || sx + 1 < 0 || sy >= H || sy + 1 < 0) {
                        v0 = v1 = v2 = v3 = 0;
                    } else {
                        const bool x0 = sx >= 0 && sx < W, x1 = sx + 1 >= 0 && sx + 1 < W;
                        const bool y0 = sy >= 0 && sy < H, y1 = sy + 1 >= 0 && sy + 1 < H;
                        v0 = x0 && y0 ? p[0] : 0;
                        v1 = x1 && y0 ? p[1] : 0;
                        v2 = x0 && y1 ? p[ftw] : 0;
                        v3 = x1 && y1 ? p[ftw + 1] : 0;
                    }
                    const int h0 = 32 * v0 + fx * (v1 - v0), h1 = 32 * v2 + fx * (v3 - v2);
                    v = (32 * h0 + fy * (h1 - h0) + 512) >> 10;
                } else {
                    v = roi_tap(lvl, W, H, a.P, X, Y);
                }
                if (c0 + u >= RW) v = 0;
                pk |= (uint32_t)v << (8 * u);
            }
            st_at<uint32_t>(tile, st_lane + 256u * i, pk ^ kRoiFlip);
        }
    }
}

// The LDS byte address of a tap from two folded 16-fraction-bit coordinates: row (high half of y) * pitch + byte column
// (high half of x), as two SDWA word-select instructions (instead of two shifts and a multiply-add)
__device__ __forceinline__ uint32_t tap_lds_addr(uint32_t x, uint32_t y, uint32_t pitch) {
    uint32_t t, r;
    asm("v_mul_u32_u24_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD"
        : "=v"(t) : "v"(y), "v"(pitch));
    asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD"
        : "=v"(r) : "v"(x), "v"(t));
    return r;
}
// a raw buffer over a footprint box (gfx9 dword 3), so its rows load with the row offset in an SGPR (soffset) and the
// lane's offset in a VGPR fixed for the kernel: no VALU per staged row
__device__ __forceinline__ __amdgpu_buffer_rsrc_t box_rsrc(const uint8_t* base) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 0x7fffffff, 0x00020000);
}

// ---- K6b over a candidate's three angle ROIs at once (n3 == 3): the three ROIs of one candidate sample nearly the
// same source region (their angles differ by the layer's angle step, a fraction of a degree), so a task is one tile
// position of all three: their footprint boxes' union is staged into LDS once (when it fits the wave's buffer) and
// the three tiles are sampled from it one after the other -- the same taps, addressed from the union's origin, so
// the same bytes as k_roi_warp.  A union that does not fit falls back to staging each ROI's own box.
// Round 4, the VALU budget (the kernel is VALU-issue bound):
//  * staging in 16-byte pieces: a lane's global offset (row lane >> 2, chunk lane & 3) and LDS address are kernel
//    constants, every LDS store carries its row group as the instruction's immediate offset, and all of a box's rows
//    (<= 4 loads per lane) are in flight together; whole 16-row groups are staged, so up to 15 rows past the box are
//    read (the level slab carries slack rows for that); rows past the wave's buffer are dropped (never sampled);
//  * PITCH: the footprint's LDS row pitch.  The product's 68 bytes (17 dwords) puts the 8 sampled rows of a wave's
//    4 x 8-pixel block on distinct banks; at 64 bytes (one b128 store per 16-byte piece instead of 4 b32) rows r and
//    r + 4 share banks and the tap reads conflict: 465 vs 384 us at layer 0 (43 sources, scripts/roi_microbench.hip,
//    profiles/r04/mbw_r04f.txt; the round-3 form with per-row staging: 397 us).  STG 1 = the round-3 per-row staging;
//  * per task, not per ROI: the lane's table offsets, the column mask and the row masks (the three ROIs share them);
//  * the interior pixel: the tables' 16-fraction-bit scale (kTabShift) puts the integer tap coordinate in the high
//    half-word, read by SDWA word selects, and the 16 tap reads and their wait are one asm statement.
// ABL (profiling ablations, scripts/roi_microbench.hip; the product uses 0): 1 = no footprint staging, 2 = interior
// taps read but not interpolated (XOR-folded), 3 = interior addressing only (no tap reads), 4 = no ROI stores (a
// never-true store kept), 5 = no interior rows (staging, tables and border tiles only), 6 = as 5 without staging,
// 7 = as 6 without the table loads, 8 = as 7 without border tiles (descriptor loads and the task loop only)
// PFT: the next ROI's tables are requested before this ROI's rows are sampled (16 more VGPRs); SLD: descriptors by
// scalar loads
template <int WPE, int PITCH = 64, int STG = 0, int ABL = 0, bool PFT = false, bool SLD = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_roi_warp3(RoiArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t ft_all[4 * ROI_FT + 16];
    constexpr int ftw = PITCH;   // footprint row pitch
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t* FT = ft_all + wv * ROI_FT;
    const uint32_t ft_lds = lds_offset_of(FT);
    const int RW = a.tw + 6, RH = a.th + 6, W = a.W, H = a.H, P = a.P;
    const int txn = (RW + ROI_T - 1) / ROI_T, tyn = (RH + ROI_T - 1) / ROI_T;
    const int per_roi = txn * tyn;
    const int tasks = roi_count(a) / 3 * per_roi;
    const int lr = lane >> 3, lg = lane & 7;
    const XcdSplit xs = xcd_split(tasks);
    const int tstride = xs.nk * 4;
    const uint32_t st_lane = 4u * lg + 32u * lr;
    // footprint staging: lane -> 16-byte chunk lane & 3 of rows lane >> 2 (+ 16 k): a box's full 64-byte width (columns
    // past it read the row's slack / the next row and are never sampled), <= 4 dwordx4 loads per lane all in flight,
    // then 16-byte LDS stores at the row's immediate offset
    const uint32_t stage_goff = (uint32_t)((lane >> 2) * P + 16 * (lane & 3));
    const uint32_t stage_lds = ft_lds + (uint32_t)((lane >> 2) * ftw + 16 * (lane & 3));
    const size_t tab_stride = (size_t)2 * (a.tabw + a.tabh);
    const uint32_t pitch_v = __builtin_amdgcn_readfirstlane(ftw);   // the LDS pitch as an SDWA operand
    auto stage = [&](int wpr, int fth, const uint8_t* gsrc) {
        if (ABL == 1 || ABL >= 6) return;
        if (STG == 1) {
            stage_footprint32<12, PITCH>(FT, wpr, fth, gsrc, P, lane);
            return;
        }
        const int n = (fth + 15) >> 4;   // wave-uniform, <= 4
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (k < n) v[k] = ld_at<u32x4>(gsrc + (size_t)k * 16 * P, stage_goff);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (k >= n) continue;
            if (PITCH % 16 == 0) {
                *(__attribute__((address_space(3))) u32x4*)(size_t)(stage_lds + 16 * ftw * k) = v[k];
            } else if ((lane >> 2) + 16 * k < ROI_FT / PITCH) {   // rows past the buffer are never sampled
                __attribute__((address_space(3))) uint32_t* d =
                    (__attribute__((address_space(3))) uint32_t*)(size_t)(stage_lds + 16 * ftw * k);
                d[0] = v[k].x; d[1] = v[k].y; d[2] = v[k].z; d[3] = v[k].w;
            }
        }
    };
    for (int task = xs.lo + xs.k * 4 + wv; task < xs.hi; task += tstride) {
        const int cand = task / per_roi;
        const int rem = task - cand * per_roi;
        const int ty = rem / txn, tx = rem - ty * txn;
        const int cx0 = tx * ROI_T, cx1 = min(cx0 + ROI_T, RW) - 1;
        const int ry0 = ty * ROI_T, ry1 = min(ry0 + ROI_T, RH) - 1;
        const int c0 = cx0 + 4 * lg;
        int bx[3], by[3], wp[3], fh[3], fl[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            // the descriptor through the scalar cache (a uniform address in the constant address space: one
            // s_load_dwordx4, no vector load and no readfirstlane; k_roi_tables wrote it in an earlier launch)
            int4 d;
            if (SLD) {
                typedef int sv4 __attribute__((ext_vector_type(4)));
                const sv4 q = *(const __attribute__((address_space(4))) sv4*)(size_t)(a.tdesc + (size_t)(3 * cand + j) * a.tdesc_stride + rem);
                d = make_int4(q.x, q.y, q.z, q.w);
            } else {
                d = a.tdesc[(size_t)(3 * cand + j) * a.tdesc_stride + rem];
            }
            bx[j] = __builtin_amdgcn_readfirstlane(d.x);
            by[j] = __builtin_amdgcn_readfirstlane(d.y);
            const int dz = __builtin_amdgcn_readfirstlane(d.z);
            wp[j] = dz & 0xffff;
            fh[j] = dz >> 16;
            fl[j] = __builtin_amdgcn_readfirstlane(d.w);
        }
        const uint8_t* lvl = a.level + (size_t)(fl[0] >> kTileSrcShift) * a.level_stride;   // one candidate, one source
        // union of the boxes that stage into LDS
        int ux0 = INT_MAX, uy0 = INT_MAX, ux1 = INT_MIN, uy1 = INT_MIN;
#pragma unroll
        for (int j = 0; j < 3; ++j)
            if ((fl[j] & kTileAny) && (fl[j] & kTileLds)) {
                ux0 = min(ux0, bx[j]); uy0 = min(uy0, by[j]);
                ux1 = max(ux1, bx[j] + 4 * wp[j]); uy1 = max(uy1, by[j] + fh[j]);
            }
        const bool any_lds = ux0 != INT_MAX;
        const int uwpr = any_lds ? (ux1 - ux0) >> 2 : 0, ufth = any_lds ? uy1 - uy0 : 0;
        const bool uni = any_lds && uwpr <= 16 && ftw * ufth <= ROI_FT;
        // per task: the lane's table offsets (columns c0 .. c0 + 3, rows ry0 + lr + 8i), column mask, row masks
        const int cc = min(c0, cx1 & ~3);   // tables are read in bounds even for idle lanes
        const uint32_t oA = 4u * cc, oB = 4u * (a.tabw + cc), oX = 4u * (2 * a.tabw + ry0 + 4 * lr),
                       oY = oX + 4u * a.tabh;
        const int nvalid = RW - c0;
        const uint32_t colmask = nvalid >= 4 ? 0xffffffffu : (1u << (8 * max(nvalid, 0))) - 1u;
        int4 tA, tB, tX, tY, nA, nB, nX, nY;
        bool nxt_ok = false;   // (PFT) nA .. nY hold the next non-empty ROI's tables
        auto load_next = [&](int slot_) {
            const int32_t* tb = a.tab + (size_t)slot_ * tab_stride;
            nA = ld_at<int4>(tb, oA);
            nB = ld_at<int4>(tb, oB);
            nX = ld_at<int4>(tb, oX);
            nY = ld_at<int4>(tb, oY);
        };
        auto load_tabs = [&](int slot_) {
            if (ABL >= 7) {
                tA = tB = tX = tY = make_int4(slot_, 0, 0, 0);
                return;
            }
            const int32_t* tb = a.tab + (size_t)slot_ * tab_stride;
            tA = ld_at<int4>(tb, oA);
            tB = ld_at<int4>(tb, oB);
            tX = ld_at<int4>(tb, oX);
            tY = ld_at<int4>(tb, oY);
        };
        load_tabs(3 * cand);   // the first ROI's tables share the staging's round trip
        if (uni) {
            wave_sync();   // previous task's gathers are done with FT
            stage(uwpr, ufth, lvl + (size_t)uy0 * P + ux0);
            wave_sync();
        }
#pragma unroll 1
        for (int j = 0; j < 3; ++j) {
            const int slot = 3 * cand + j;
            const int flags = fl[j];
            const bool in_lds = (flags & kTileLds) != 0;
            int bxa = bx[j], by0 = by[j];
            if (uni) {
                bxa = ux0; by0 = uy0;
            } else {
                wave_sync();
                if ((flags & kTileAny) && in_lds) stage(wp[j], fh[j], lvl + (size_t)by0 * P + bxa);
                wave_sync();
            }
            if (j > 0 && (flags & kTileAny)) {   // (an empty tile needs no tables)
                if (PFT && nxt_ok) {
                    tA = nA; tB = nB; tX = nX; tY = nY;
                } else {
                    load_tabs(slot);
                }
            }
            nxt_ok = false;
            if (PFT && j + 1 < 3 && (fl[j + 1] & kTileAny)) {
                load_next(slot + 1);
                nxt_ok = true;
            }
            const uint32_t adv[4] = {(uint32_t)tA.x, (uint32_t)tA.y, (uint32_t)tA.z, (uint32_t)tA.w};
            const uint32_t bdv[4] = {(uint32_t)tB.x, (uint32_t)tB.y, (uint32_t)tB.z, (uint32_t)tB.w};
            const uint32_t X0r[4] = {(uint32_t)tX.x, (uint32_t)tX.y, (uint32_t)tX.z, (uint32_t)tX.w};
            const uint32_t Y0r[4] = {(uint32_t)tY.x, (uint32_t)tY.y, (uint32_t)tY.z, (uint32_t)tY.w};
            uint8_t* tile = a.roi + (size_t)slot * a.roi_stride + ((size_t)rem << 10);
            if (c0 > cx1) continue;
            if (!(flags & kTileAny)) {
                // the tile's footprint lies entirely outside the level: every tap is BORDER_CONSTANT 0, so the tile is
                // zeros (stored flipped) -- no taps (18 % of the layer-0 tiles of the Src7 bench: ROIs reaching past
                // the image; they took the per-pixel border path before, round 4)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (ry0 + lr + 8 * i <= ry1) st_at<uint32_t>(tile, st_lane + 256u * i, kRoiFlip);
                continue;
            }
            if (ABL == 8 && !((flags & kTileInterior) && in_lds)) {
                if (X0r[0] == 0x9e3779b9u) st_at<uint32_t>(tile, st_lane, adv[0]);
                continue;
            }
            if ((flags & kTileInterior) && in_lds) {
                // folded coordinates: (X0 + adv + xo) >> 16 is the tap's LDS byte column (footprint base included),
                // (Y0 + bdv + yo) >> 16 its footprint row; both lie in [0, 2^15), so the high half-words are exact
                const uint32_t xo = (ft_lds - (uint32_t)bxa) << kTabFrac, yo = 0u - ((uint32_t)by0 << kTabFrac);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t x0r = X0r[i] + xo, y0r = Y0r[i] + yo;
                    uint32_t off[4];
                    int fxv[4], fyv[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const uint32_t sxv = x0r + adv[u], syv = y0r + bdv[u];
                        off[u] = tap_lds_addr(sxv, syv, pitch_v);
                        fxv[u] = (int)((sxv >> kTapShift) & (kInterTab - 1));
                        fyv[u] = (int)((syv >> kTapShift) & (kInterTab - 1));
                    }
                    if (ABL >= 5) continue;
                    uint32_t pk;
                    if (ABL == 3) {
                        pk = off[0] ^ off[1] ^ off[2] ^ off[3] ^ (uint32_t)(fxv[0] + fxv[1] + fxv[2] + fxv[3]) ^
                             (uint32_t)(fyv[0] + fyv[1] + fyv[2] + fyv[3]);
                    } else {
                        int v[4][4];
                        lds_taps16<ftw>(off, v);
                        if (ABL == 2) {
                            pk = 0;
#pragma unroll
                            for (int u = 0; u < 4; ++u) pk ^= (uint32_t)(v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3]) << (8 * u);
                        } else {
                            pk = bilerp_row4(v, fxv, fyv);
                        }
                    }
                    if (ABL == 4 ? pk == 0x9e3779b9u && c0 < 0 : ry0 + lr + 8 * i <= ry1)
                        st_at<uint32_t>(tile, st_lane + 256u * i, (pk & colmask) ^ kRoiFlip);
                }
                continue;
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (ry0 + lr + 8 * i > ry1) break;
                uint32_t pk = 0;
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int X = (int)(X0r[i] + adv[u]) >> kTapShift;
                    const int Y = (int)(Y0r[i] + bdv[u]) >> kTapShift;
                    int v;
                    if (in_lds) {
                        const int sx = sat_s16(X >> kInterBits), sy = sat_s16(Y >> kInterBits);
                        const int fx = X & (kInterTab - 1), fy = Y & (kInterTab - 1);
                        const uint8_t* p = FT + (sy - by0) * ftw + (sx - bxa);
                        int v0, v1, v2, v3;
                        if ((unsigned)sx < (unsigned)(W - 1) && (unsigned)sy < (unsigned)(H - 1)) {
                            v0 = p[0]; v1 = p[1]; v2 = p[ftw]; v3 = p[ftw + 1];
                        } else if (sx >= W || sx + 1 < 0 || sy >= H || sy + 1 < 0) {
                            v0 = v1 = v2 = v3 = 0;
                        } else {
                            const bool x0 = sx >= 0 && sx < W, x1 = sx + 1 >= 0 && sx + 1 < W;
                            const bool y0 = sy >= 0 && sy < H, y1 = sy + 1 >= 0 && sy + 1 < H;
                            v0 = x0 && y0 ? p[0] : 0;
                            v1 = x1 && y0 ? p[1] : 0;
                            v2 = x0 && y1 ? p[ftw] : 0;
                            v3 = x1 && y1 ? p[ftw + 1] : 0;
                        }
                        const int h0 = 32 * v0 + fx * (v1 - v0), h1 = 32 * v2 + fx * (v3 - v2);
                        v = (32 * h0 + fy * (h1 - h0) + 512) >> 10;
                    } else {
                        v = roi_tap(lvl, W, H, a.P, X, Y);
                    }
                    if (c0 + u >= RW) v = 0;
                    pk |= (uint32_t)v << (8 * u);
                }
                st_at<uint32_t>(tile, st_lane + 256u * i, pk ^ kRoiFlip);
            }
        }
    }
}

// ---- K7: per-row exact correlation on the matrix cores.  For one ROI, the 49 per-row dot products
// R[t][dy][dx] = sum_c T[t][c] * I[t+dy][c+dx] (IM_Conv_SIMD's int32 row results, TemplateMatcher.cpp:487-512)
// are, for each shift dx, a banded GEMM  D_dx[t][s] = sum_c T[t][c] * I[s][c+dx]  kept where 0 <= s - t < 7:
// A = template rows (M = 16), B = source rows (N = 16), K = columns, 64 per v_mfma_i32_16x16x64_i8.
// A work item is a band of 32 template rows (2 M tiles) and its 38 source rows (3 N tiles); wave w takes the
// (M, N) tile pair (w & 1, (w & 1) + (w >> 1)) and all 7 shifts, so a shift is uniform per instruction: B
// fragments are aligned 16 + 8 byte LDS reads funnel-shifted by a constant (v_alignbyte), A fragments aligned
// 16-byte loads of the i8 template.  u8 operands enter the signed MFMA as x ^ 0x80 = x - 128; the exact value
// is restored with integer corrections  sum T*I = sum T'I' + 128*(W[s][dx] + TS[t]) - 16384*tw  (W = window row
// sum of I, TS = template row sum; mod 2^32, true value < 2^31).  The item also produces the rows' exact window
// sums of I and I^2 and the per-16-row-chunk window-sum partials used by the normalisation.
typedef int fpm_v4i __attribute__((ext_vector_type(4)));
constexpr int kBandRows = 2 * kMmaRows;       // template rows per work item
constexpr int kBandSrc = kBandRows + 6;       // source rows per work item
constexpr int kStageRows = (kBandSrc + 3) / 4;   // staged rows per wave
constexpr int kStageBatch = 5;                  // of which loaded together

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += (uint32_t)__shfl_xor((int)v, m, 64);
    return v;
}

__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, int sh) {
    return sh == 0 ? lo : __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// The 7 shifted banded GEMM tiles of one wave: acc[d] += A(16 template rows) x B_d(16 ROI rows shifted by d) over
// nk k-steps of 64 bytes.  ap / bp: this lane's A row / B row at byte 16*(lane >> 4) of k-step 0 (16-byte aligned).
__device__ __forceinline__ void band_mfma(const uint8_t* ap, const uint8_t* bp, int nk, fpm_v4i acc[7]) {
    fpm_v4i c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0, c4 = c0, c5 = c0, c6 = c0;
    for (int k = 0; k < nk; ++k) {
        const fpm_v4i av = *(const fpm_v4i*)__builtin_assume_aligned(ap + 64 * k, 16);
        const uint8_t* bk = (const uint8_t*)__builtin_assume_aligned(bp + 64 * k, 16);
        const uint4 lo = *(const uint4*)bk;
        const uint2 hi = *(const uint2*)(bk + 16);
        const uint32_t w0 = lo.x, w1 = lo.y, w2 = lo.z, w3 = lo.w, w4 = hi.x, w5 = hi.y;
        // shift d: bytes [d, d + 16) of w0..w5 (d >> 2 whole words, then alignbyte by d & 3)
        const uint32_t a10 = __builtin_amdgcn_alignbyte(w1, w0, 1), a21 = __builtin_amdgcn_alignbyte(w2, w1, 1),
                       a32 = __builtin_amdgcn_alignbyte(w3, w2, 1), a43 = __builtin_amdgcn_alignbyte(w4, w3, 1),
                       a54 = __builtin_amdgcn_alignbyte(w5, w4, 1);
        const uint32_t b10 = __builtin_amdgcn_alignbyte(w1, w0, 2), b21 = __builtin_amdgcn_alignbyte(w2, w1, 2),
                       b32 = __builtin_amdgcn_alignbyte(w3, w2, 2), b43 = __builtin_amdgcn_alignbyte(w4, w3, 2),
                       b54 = __builtin_amdgcn_alignbyte(w5, w4, 2);
        const uint32_t e10 = __builtin_amdgcn_alignbyte(w1, w0, 3), e21 = __builtin_amdgcn_alignbyte(w2, w1, 3),
                       e32 = __builtin_amdgcn_alignbyte(w3, w2, 3), e43 = __builtin_amdgcn_alignbyte(w4, w3, 3);
        c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, fpm_v4i{(int)w0, (int)w1, (int)w2, (int)w3}, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, fpm_v4i{(int)a10, (int)a21, (int)a32, (int)a43}, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, fpm_v4i{(int)b10, (int)b21, (int)b32, (int)b43}, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, fpm_v4i{(int)e10, (int)e21, (int)e32, (int)e43}, c3, 0, 0, 0);
        c4 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, fpm_v4i{(int)w1, (int)w2, (int)w3, (int)w4}, c4, 0, 0, 0);
        c5 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, fpm_v4i{(int)a21, (int)a32, (int)a43, (int)a54}, c5, 0, 0, 0);
        c6 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, fpm_v4i{(int)b21, (int)b32, (int)b43, (int)b54}, c6, 0, 0, 0);
    }
    acc[0] = c0; acc[1] = c1; acc[2] = c2; acc[3] = c3; acc[4] = c4; acc[5] = c5; acc[6] = c6;
}

// The same with the A fragments read from the global i8 slab (L2-resident, shared by every ROI of the layer):
// two k-steps of A in flight; the empty asm keeps the compiler from sinking the prefetch to its use.
// The slab carries >= 256 bytes of slack past its last row.
__device__ __forceinline__ void band_mfma_ga(const int8_t* ap, const uint8_t* bp, int nk, fpm_v4i acc[7]) {
    fpm_v4i c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0, c4 = c0, c5 = c0, c6 = c0;
    fpm_v4i p0 = *(const fpm_v4i*)ap, p1 = *(const fpm_v4i*)(ap + 64);
    for (int k = 0; k < nk; ++k) {
        const fpm_v4i av = p0;
        p0 = p1;
        p1 = *(const fpm_v4i*)(ap + 64 * (k + 2));
        asm volatile("" ::: "memory");
        const uint8_t* bk = (const uint8_t*)__builtin_assume_aligned(bp + 64 * k, 16);
        const uint4 lo = *(const uint4*)bk;
        const uint2 hi = *(const uint2*)(bk + 16);
        const uint32_t w0 = lo.x, w1 = lo.y, w2 = lo.z, w3 = lo.w, w4 = hi.x, w5 = hi.y;
        const uint32_t a10 = __builtin_amdgcn_alignbyte(w1, w0, 1), a21 = __builtin_amdgcn_alignbyte(w2, w1, 1),
                       a32 = __builtin_amdgcn_alignbyte(w3, w2, 1), a43 = __builtin_amdgcn_alignbyte(w4, w3, 1),
                       a54 = __builtin_amdgcn_alignbyte(w5, w4, 1);
        const uint32_t b10 = __builtin_amdgcn_alignbyte(w1, w0, 2), b21 = __builtin_amdgcn_alignbyte(w2, w1, 2),
                       b32 = __builtin_amdgcn_alignbyte(w3, w2, 2), b43 = __builtin_amdgcn_alignbyte(w4, w3, 2),
                       b54 = __builtin_amdgcn_alignbyte(w5, w4, 2);
        const uint32_t e10 = __builtin_amdgcn_alignbyte(w1, w0, 3), e21 = __builtin_amdgcn_alignbyte(w2, w1, 3),
                       e32 = __builtin_amdgcn_alignbyte(w3, w2, 3), e43 = __builtin_amdgcn_alignbyte(w4, w3, 3);
        c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, fpm_v4i{(int)w0, (int)w1, (int)w2, (int)w3}, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, fpm_v4i{(int)a10, (int)a21, (int)a32, (int)a43}, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, fpm_v4i{(int)b10, (int)b21, (int)b32, (int)b43}, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, fpm_v4i{(int)e10, (int)e21, (int)e32, (int)e43}, c3, 0, 0, 0);
        c4 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, fpm_v4i{(int)w1, (int)w2, (int)w3, (int)w4}, c4, 0, 0, 0);
        c5 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, fpm_v4i{(int)a21, (int)a32, (int)a43, (int)a54}, c5, 0, 0, 0);
        c6 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, fpm_v4i{(int)b21, (int)b32, (int)b43, (int)b54}, c6, 0, 0, 0);
    }
    acc[0] = c0; acc[1] = c1; acc[2] = c2; acc[3] = c3; acc[4] = c4; acc[5] = c5; acc[6] = c6;
}

// The same with this wave's A fragments held in registers (k_roi_corr's register-A form): the loop reads only LDS.
template <int NK>
__device__ __forceinline__ void band_mfma_regs(const fpm_v4i* A, const uint8_t* bp, int nk, fpm_v4i acc[7]) {
    fpm_v4i c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0, c4 = c0, c5 = c0, c6 = c0;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
        if (k >= nk) continue;
        const fpm_v4i av = A[k];
        const uint8_t* bk = (const uint8_t*)__builtin_assume_aligned(bp + 64 * k, 16);
        const uint4 lo = *(const uint4*)bk;
        const uint2 hi = *(const uint2*)(bk + 16);
        const uint32_t w0 = lo.x, w1 = lo.y, w2 = lo.z, w3 = lo.w, w4 = hi.x, w5 = hi.y;
        const uint32_t a10 = __builtin_amdgcn_alignbyte(w1, w0, 1), a21 = __builtin_amdgcn_alignbyte(w2, w1, 1),
                       a32 = __builtin_amdgcn_alignbyte(w3, w2, 1), a43 = __builtin_amdgcn_alignbyte(w4, w3, 1),
                       a54 = __builtin_amdgcn_alignbyte(w5, w4, 1);
        const uint32_t b10 = __builtin_amdgcn_alignbyte(w1, w0, 2), b21 = __builtin_amdgcn_alignbyte(w2, w1, 2),
                       b32 = __builtin_amdgcn_alignbyte(w3, w2, 2), b43 = __builtin_amdgcn_alignbyte(w4, w3, 2),
                       b54 = __builtin_amdgcn_alignbyte(w5, w4, 2);
        const uint32_t e10 = __builtin_amdgcn_alignbyte(w1, w0, 3), e21 = __builtin_amdgcn_alignbyte(w2, w1, 3),
                       e32 = __builtin_amdgcn_alignbyte(w3, w2, 3), e43 = __builtin_amdgcn_alignbyte(w4, w3, 3);
        c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, fpm_v4i{(int)w0, (int)w1, (int)w2, (int)w3}, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, fpm_v4i{(int)a10, (int)a21, (int)a32, (int)a43}, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, fpm_v4i{(int)b10, (int)b21, (int)b32, (int)b43}, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, fpm_v4i{(int)e10, (int)e21, (int)e32, (int)e43}, c3, 0, 0, 0);
        c4 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, fpm_v4i{(int)w1, (int)w2, (int)w3, (int)w4}, c4, 0, 0, 0);
        c5 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, fpm_v4i{(int)a21, (int)a32, (int)a43, (int)a54}, c5, 0, 0, 0);
        c6 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, fpm_v4i{(int)b21, (int)b32, (int)b43, (int)b54}, c6, 0, 0, 0);
    }
    acc[0] = c0; acc[1] = c1; acc[2] = c2; acc[3] = c3; acc[4] = c4; acc[5] = c5; acc[6] = c6;
}

// MODE (profiling ablations in scripts/roi_microbench.hip; the product uses 0): 2 = no MFMA loop, 3 = no staging
// (slot-major form only), 4 = no window-edge phase, 5 = no row-result stores, 6 = no window partials, 7 = no row sums
// GA: A operand read from the global i8 slab (no template rows in LDS); WPE: register cap (waves per SIMD);
// NK > 0: register-A form (A fragments of nk <= NK k-steps held per wave, band-major item runs; needs GA)
// PFR (register-A form): prefetch the next item's rows (false: load this item's rows at its start, fewer VGPRs)
// RS: 1 = row statistics in one phase (a quad of lanes per row: its I / I^2 totals reduced by DPP, then the edge pixels
// of each window subtracted by the same lanes; the window partials split over lane pairs), 0 = the earlier form (row
// totals by LDS atomics, a separate edge phase, one thread per partial), 2 = as 1 with the partials before the GEMM
// SE: the band's row results are written into LDS by the epilogue and copied to HBM as 16-byte runs during the next
// item's staging (after the loads of its rows are issued, so waiting for those loads does not wait for these stores)
// DMA (register-A form, no row prefetch): the item's ROI rows go global -> LDS by LDS-DMA (one global_load_lds_dwordx4
// per row and wave, the scratch already flipped): no staging registers and no VALU per staged row
// DB (with DMA): two row buffers; the next item's rows are issued into the other buffer once this item's are in LDS,
// so an item waits for rows requested one item earlier (the LDS holds a second kBandSrc x SBp buffer after the rest)
// wave priority of the GEMM phase (s_setprio): 1 = the banded GEMM and its row-result epilogue at priority 1 (the
// product: the item's matrix work is not held behind the co-resident waves' staging and statistics VALU; Src7 kernel
// pass 196.5 -> 185.7 us per k_roi_corr launch averaged over the layers, profiles/r06_prio/), 2 = the GEMM alone,
// 0 = none
#ifndef FPM_CORR_PRIO
#define FPM_CORR_PRIO 1
#endif
template <int MODE, bool GA, int WPE, int NK = 0, bool PFR = true, int RS = 1, bool SE = false, bool DMA = false,
          bool DB = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_roi_corr(RoiArgs a) {
    static_assert(!DMA || (NK > 0 && !PFR), "LDS-DMA staging replaces the register staging of the register-A form");
    static_assert(!DB || DMA, "the double buffer is filled by LDS-DMA");
    static_assert(NK == 0 || (GA && MODE != 3), "the register-A form stages no template rows");
    static_assert(!SE || NK > 0, "the staged epilogue is flushed in the register-A form's staging phase");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tw = a.tw, th = a.th, RW = tw + 6;
    const int SBp = a.roi_pitch;
    const int TBp = tmpl_lds_pitch(a.tp8);
    uint8_t* const SB0 = smem;                                 // kBandSrc rows x SBp, bytes ^ 0x80
    uint8_t* SB = SB0;
    uint8_t* TB = SB + (size_t)kBandSrc * SBp;                 // kBandRows template rows (i8) x TBp (!GA)
    uint32_t* rall = (uint32_t*)(TB + (GA ? 0 : (size_t)kBandRows * TBp)); // full-row sums of I
    uint32_t* rallq = rall + kBandSrc;                         // full-row sums of I^2
    uint32_t* wi = rallq + kBandSrc;                           // [row][dx] window sums of I
    uint32_t* wq = wi + kBandSrc * 7;                          // [row][dx] window sums of I^2
    uint32_t* lts = wq + kBandSrc * 7;                         // the band's template-row sums (16-byte aligned)
    uint32_t* rsb = lts + 2 * kMmaRows;                        // (SE) the band's [rb][49] row results (16-byte aligned)
    uint8_t* const SB1 = (uint8_t*)(((uintptr_t)(rsb + 2 * kMmaRows * 49) + 64 + 15) & ~(uintptr_t)15);   // (DB)
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int nband = (th + kBandRows - 1) / kBandRows;
    const int rois = roi_count(a), items = rois * nband;
    const int q4 = SBp >> 4;                                   // 16-byte columns per row
    const int nwr = (RW + 3) >> 2;                             // words holding ROI pixels
    const int g = lane >> 4, n = lane & 15;
    const int mt = wv & 1, nt = mt + (wv >> 1);                // this wave's (M, N) tile pair
    const int txn = (RW + ROI_T - 1) / ROI_T;
    const XcdSplit xs = xcd_split(items);   // the XCD group's contiguous range of items
    // NK = 0: items slot-major (an ROI's bands, which share rows, on one XCD group), grid-stride over the range.
    // NK > 0 (register-A form): items band-major (item = band * rois + slot) and each workgroup takes one
    // contiguous run of its group's range, so consecutive items share their template band: the wave loads its A
    // fragments once per band and the MFMA loop reads only LDS; the next item's ROI rows are loaded into
    // registers while the current item computes, so staging costs one LDS store per item.
    int it_lo = xs.lo + xs.k, it_hi = xs.hi, it_step = xs.nk;
    if (NK > 0) {
        const int64_t span = xs.hi - xs.lo;
        it_lo = xs.lo + (int)(span * xs.k / xs.nk);
        it_hi = xs.lo + (int)(span * (xs.k + 1) / xs.nk);
        it_step = 1;
    }
    constexpr int NA = NK > 0 ? NK : 1;
    fpm_v4i Areg[NA];
#pragma unroll
    for (int k = 0; k < NA; ++k) Areg[k] = fpm_v4i{0, 0, 0, 0};
    int a_band = -1;
    uint4 pv[kStageRows];
    const int lc = min(lane, 2 * txn - 1);   // an in-bounds chunk for lanes past the ROI width (zeroed when stored)
    auto load_rows = [&](int it) {           // unconditional loads: rows past the band repeat its last row
        const int bd = it / rois, sl = it - bd * rois;
        const int T0n = bd * kBandRows, nsn = min(kBandRows, th - T0n) + 6;
        const uint8_t* rsrc = a.roi + (size_t)sl * a.roi_stride;
        // row indices wave-uniform (scalar), the lane's column offset recomputed per call (opaque): no per-row
        // address registers kept across the item loop
        const int wvu = __builtin_amdgcn_readfirstlane(wv);
        int lcv = lc;
        asm volatile("" : "+v"(lcv));
        const uint32_t lane_off = ((uint32_t)(lcv >> 1) << 10) + 16u * (uint32_t)(lcv & 1);
#pragma unroll
        for (int i = 0; i < kStageRows; ++i) {
            const int R = T0n + min(wvu + 4 * i, nsn - 1);
            pv[i] = *(const uint4*)(rsrc + ((size_t)((R >> 5) * txn) << 10) + (R & 31) * ROI_T + lane_off);
        }
    };
    if (NK > 0 && PFR && it_lo < it_hi) load_rows(it_lo);
    // (SE) the previous item's row results: LDS -> its [rb][49] range of the ROI's series, 16-byte stores (the range
    // starts 16-byte aligned: slot stride and T0 * 49 are multiples of 4 words), the < 4-word tail by single words
    int pv_slot = -1, pv_T0 = 0, pv_rb = 0;
    auto flush = [&]() {
        if (!SE || pv_slot < 0) return;
        uint32_t* dst = a.rowsum + (((size_t)th * 49 + 3) & ~(size_t)3) * pv_slot + (size_t)pv_T0 * 49;
        const int nw = pv_rb * 49, n16 = nw >> 2;
        for (int i = tid; i < n16; i += 256) *(uint4*)(dst + 4 * i) = *(const uint4*)(rsb + 4 * i);
        if (tid < (nw & 3)) dst[4 * n16 + tid] = rsb[4 * n16 + tid];
    };
    // (DMA) item it's ROI rows wv + 4i -> buffer buf: SGPR row address, the lane's 16-byte chunk of it (lanes past the
    // ROI width idle: the LDS chunks past the ROI are multiplied by the template's zero padding and never summed)
    auto dma_rows = [&](int it, uint8_t* buf) {
        const int bd = it / rois, sl = it - bd * rois;
        const int T0n = bd * kBandRows, nsn = min(kBandRows, th - T0n) + 6;
        const uint8_t* rsrc = a.roi + (size_t)sl * a.roi_stride;
        const uint32_t lane_off = ((uint32_t)(lane >> 1) << 10) + 16u * (uint32_t)(lane & 1);
        const int wvu = __builtin_amdgcn_readfirstlane(wv);
        const bool in_roi = lane < 2 * txn;
#pragma unroll
        for (int i = 0; i < kStageRows; ++i) {
            const int r = wvu + 4 * i;
            if (r < nsn && in_roi) {
                const int R = T0n + r;
                const uint8_t* gp = rsrc + ((size_t)((R >> 5) * txn) << 10) + (R & 31) * ROI_T + lane_off;
                const uint32_t ldsa = __builtin_amdgcn_readfirstlane(lds_offset_of(buf + (size_t)r * SBp));
                uint32_t keep;
                asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
                             "s_mov_b32 m0, %0"
                             : "=&s"(keep) : "v"(gp), "s"(ldsa) : "memory");
            }
        }
    };
    for (int item = it_lo; item < it_hi; item += it_step) {
        int slot, band;
        if (NK > 0) { band = item / rois; slot = item - band * rois; }
        else { slot = item / nband; band = item - slot * nband; }
        SB = DB && ((item - it_lo) & 1) ? SB1 : SB0;
        const int T0 = band * kBandRows, rb = min(kBandRows, th - T0), nsrc = rb + 6;
        __syncthreads();   // previous item done with SB / rall / wi
        if (RS == 0 && tid < kBandSrc) { rall[tid] = 0; rallq[tid] = 0; }
        if (NK > 0) {
            // this item's rows (loaded during the previous item) ^ 0x80 into LDS; this wave's A fragments when the
            // band changes (workgroup-uniform); then the next item's row loads
            const bool in_roi = lane < 2 * txn;
            if (DB) {
                // this item's rows were issued during the previous item (the first item's now); wait, then start the
                // previous item's row-result stores
                if (item == it_lo) dma_rows(item, SB);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                flush();
            } else if (DMA) {
                dma_rows(item, SB);
                flush();
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            } else {
            if (!PFR) load_rows(item);
            flush();
#pragma unroll
            for (int i = 0; i < kStageRows; ++i) {
                const int r = wv + 4 * i;
                // the scratch is stored flipped (kRoiFlip); columns past the ROI: flipped zeros
                if (r < nsrc && lane < q4)
                    *(uint4*)(SB + (size_t)r * SBp + 16 * lane) = in_roi ? pv[i] : make_uint4(kRoiFlip, kRoiFlip, kRoiFlip, kRoiFlip);
            }
            }
            if (band != a_band) {
                a_band = band;
                if (tid < kBandRows) lts[tid] = tid < rb ? (uint32_t)a.tsum[T0 + tid] : 0u;
                if (kMmaRows * mt < rb) {
                    const int8_t* ap = a.tmpl8 + (size_t)(T0 + kMmaRows * mt + n) * a.tp8 + 16 * g;
#pragma unroll
                    for (int k = 0; k < NA; ++k)
                        if (k < a.nk) Areg[k] = *(const fpm_v4i*)(ap + 64 * k);
                }
            }
            if (PFR && item + 1 < it_hi) load_rows(item + 1);
        } else if (MODE != 3) {   // stage: wave wv stages rows wv + 4i (kStageBatch rows' loads in flight), ^ 0x80
            if (tid < kBandRows) lts[tid] = tid < rb ? (uint32_t)a.tsum[T0 + tid] : 0u;
            // tile-major ROI scratch (k_roi_warp): row R, 16-byte chunk c lives in tile (R >> 5, c >> 1)
            const uint8_t* rsrc = a.roi + (size_t)slot * a.roi_stride;
            for (int c0 = 0; c0 < q4; c0 += 64) {
                const int c = c0 + lane;
                for (int i0 = 0; i0 < kStageRows; i0 += kStageBatch) {
                    uint4 v[kStageBatch];
#pragma unroll
                    for (int i = 0; i < kStageBatch; ++i) {
                        const int r = wv + 4 * (i0 + i);
                        const int R = T0 + r;
                        v[i] = (r < nsrc && c < 2 * txn)
                                   ? *(const uint4*)(rsrc + ((size_t)((R >> 5) * txn + (c >> 1)) << 10) + (R & 31) * ROI_T + 16 * (c & 1))
                                   : make_uint4(kRoiFlip, kRoiFlip, kRoiFlip, kRoiFlip);
                    }
#pragma unroll
                    for (int i = 0; i < kStageBatch; ++i) {
                        const int r = wv + 4 * (i0 + i);
                        if (r < nsrc && c < q4) *(uint4*)(SB + (size_t)r * SBp + 16 * c) = v[i];
                    }
                }
            }
        }
        __syncthreads();
        if (DB && item + 1 < it_hi) dma_rows(item + 1, SB == SB0 ? SB1 : SB0);   // every wave is past the other buffer
        if (RS >= 1 && MODE != 7 && tid < 4 * nsrc) {
            // row r's statistics by the quad of lanes 4r .. 4r + 3 (whole quads: DPP within the quad): exact full-row
            // sums of I and I^2 over the row's words (pixels past RW are zero), then each lane subtracts the window's
            // edge pixels for its dx (qq and qq + 4): window [dx, dx + tw) = row minus bytes [0, dx) and [dx + tw, RW)
            const int r = tid >> 2, qq = tid & 3;
            const int per = (nwr + 3) >> 2, k0 = qq * per, k1 = min(nwr, k0 + per);
            const uint32_t* row = (const uint32_t*)(SB + (size_t)r * SBp);
            uint32_t s1 = 0, s2 = 0;
            int k = k0;
            for (; k + 8 <= k1; k += 8) {
                uint32_t x[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) x[u] = row[k + u] ^ 0x80808080u;
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    s1 = __builtin_amdgcn_udot4(x[u], 0x01010101u, s1, false);
                    s2 = __builtin_amdgcn_udot4(x[u], x[u], s2, false);
                }
            }
            for (; k < k1; ++k) {
                const uint32_t x = row[k] ^ 0x80808080u;
                s1 = __builtin_amdgcn_udot4(x, 0x01010101u, s1, false);
                s2 = __builtin_amdgcn_udot4(x, x, s2, false);
            }
            // left edge bytes 0..5 (words 0, 1) and right edge bytes tw .. tw + 5 (funnel-shifted from 3 words)
            const uint32_t l0 = row[0] ^ 0x80808080u, l1 = row[1] ^ 0x80808080u;
            const int wr = tw >> 2;
            const uint32_t x0 = row[wr], x1 = row[wr + 1], x2 = row[wr + 2];
            const uint32_t e0 = __builtin_amdgcn_alignbyte(x1, x0, (uint32_t)tw) ^ 0x80808080u;
            const uint32_t e1 = __builtin_amdgcn_alignbyte(x2, x1, (uint32_t)tw) ^ 0x80808080u;
            s1 += (uint32_t)__builtin_amdgcn_mov_dpp((int)s1, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
            s2 += (uint32_t)__builtin_amdgcn_mov_dpp((int)s2, 0xB1, 0xF, 0xF, false);
            s1 += (uint32_t)__builtin_amdgcn_mov_dpp((int)s1, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
            s2 += (uint32_t)__builtin_amdgcn_mov_dpp((int)s2, 0x4E, 0xF, 0xF, false);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int dx = qq + 4 * h;
                if (dx < 7) {
                    // left: bytes c < dx of (l0, l1); right: bytes i >= dx of (e0, e1[0..1])
                    const uint32_t ml0 = dx >= 4 ? 0xffffffffu : (1u << (8 * dx)) - 1u;
                    const uint32_t ml1 = dx <= 4 ? 0u : (1u << (8 * (dx - 4))) - 1u;
                    const uint32_t mr0 = dx >= 4 ? 0u : ~((1u << (8 * dx)) - 1u);
                    const uint32_t mr1 = dx <= 4 ? 0xffffu : dx == 5 ? 0xff00u : 0u;
                    const uint32_t a0 = l0 & ml0, a1 = l1 & ml1, b0 = e0 & mr0, b1 = e1 & mr1;
                    uint32_t q1 = __builtin_amdgcn_udot4(a0, 0x01010101u, 0u, false);
                    q1 = __builtin_amdgcn_udot4(a1, 0x01010101u, q1, false);
                    q1 = __builtin_amdgcn_udot4(b0, 0x01010101u, q1, false);
                    q1 = __builtin_amdgcn_udot4(b1, 0x01010101u, q1, false);
                    uint32_t q2 = __builtin_amdgcn_udot4(a0, a0, 0u, false);
                    q2 = __builtin_amdgcn_udot4(a1, a1, q2, false);
                    q2 = __builtin_amdgcn_udot4(b0, b0, q2, false);
                    q2 = __builtin_amdgcn_udot4(b1, b1, q2, false);
                    wi[r * 7 + dx] = s1 - q1;
                    wq[r * 7 + dx] = s2 - q2;
                }
            }
        }
        if (RS == 0 && MODE != 7 && tid < 4 * nsrc) {   // exact full-row sums of I and I^2: thread (row, quarter of the row's words)
            const int r = tid >> 2, qq = tid & 3;
            const int per = (nwr + 3) >> 2, k0 = qq * per, k1 = min(nwr, k0 + per);
            const uint32_t* row = (const uint32_t*)(SB + (size_t)r * SBp);
            uint32_t s1 = 0, s2 = 0;
            int k = k0;
            for (; k + 8 <= k1; k += 8) {
                uint32_t x[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) x[u] = row[k + u] ^ 0x80808080u;
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    s1 = __builtin_amdgcn_udot4(x[u], 0x01010101u, s1, false);
                    s2 = __builtin_amdgcn_udot4(x[u], x[u], s2, false);
                }
            }
            for (; k < k1; ++k) {
                const uint32_t x = row[k] ^ 0x80808080u;
                s1 = __builtin_amdgcn_udot4(x, 0x01010101u, s1, false);
                s2 = __builtin_amdgcn_udot4(x, x, s2, false);
            }
            atomicAdd(&rall[r], s1);
            atomicAdd(&rallq[r], s2);
        }
        if (!GA) {   // template rows T0 .. T0 + 16*ceil(rb/16) - 1 of the i8 slab
            const int trows = (rb + kMmaRows - 1) / kMmaRows * kMmaRows;
            stage_block16(TB, TBp, (const uint8_t*)a.tmpl8 + (size_t)T0 * a.tp8, a.tp8, trows, a.tp8 >> 4, tid, 256);
        }
        if (RS == 0) __syncthreads();
        for (int i = tid; RS == 0 && MODE != 4 && i < nsrc * 7; i += 256) {   // window [dx, dx + tw): full row minus <= 6 edge pixels
            const int r = i / 7, dx = i - r * 7;
            const uint8_t* sbr = SB + (size_t)r * SBp;
            uint32_t q1 = rall[r], q2 = rallq[r];
            for (int c = 0; c < dx; ++c) { const uint32_t v = sbr[c] ^ 0x80u; q1 -= v; q2 -= v * v; }
            for (int c = dx + tw; c < RW; ++c) { const uint32_t v = sbr[c] ^ 0x80u; q1 -= v; q2 -= v * v; }
            wi[i] = q1;
            wq[i] = q2;
        }
        __syncthreads();
        // per-16-row-chunk partials of the window sums, 8 rows per lane (lane pairs, combined by DPP within the quad;
        // the 8 rows' LDS reads all in flight)
        auto partials = [&]() {
            if (MODE == 6 || tid >= 4 * 49) return;
            const int pr = tid >> 1, half = tid & 1;
            const int h = pr / 49, k = pr - h * 49;
            const int chunk = (T0 >> 4) + h;
            const int tlo = kMmaRows * h, thi = min(tlo + kMmaRows, rb);
            const bool ok = chunk < a.nchunk && tlo < thi;   // the same for both lanes of the pair
            const int pdy = k / 7, ddx = k - pdy * 7;
            const int t0 = tlo + 8 * half, n8 = ok ? min(8, thi - t0) : 0;
            uint32_t s1 = 0, x[8], y[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = (t0 + u + pdy) * 7 + ddx;
                x[u] = u < n8 ? wi[i] : 0u;
                y[u] = u < n8 ? wq[i] : 0u;
            }
            uint64_t s2 = 0;
#pragma unroll
            for (int u = 0; u < 8; ++u) { s1 += x[u]; s2 += y[u]; }
            s1 += (uint32_t)__builtin_amdgcn_mov_dpp((int)s1, 0xB1, 0xF, 0xF, false);
            const uint32_t lo = (uint32_t)s2, hi = (uint32_t)(s2 >> 32);
            s2 += (uint64_t)(uint32_t)__builtin_amdgcn_mov_dpp((int)lo, 0xB1, 0xF, 0xF, false) |
                  ((uint64_t)(uint32_t)__builtin_amdgcn_mov_dpp((int)hi, 0xB1, 0xF, 0xF, false) << 32);
            if (ok && half == 0) {
                // 32-bit index recomputed per item (opaque k): a loop-invariant 64-bit address kept across the item
                // loop was spilled, and its reload's vmcnt(0) waited for every row-result store of the item
                uint32_t kk = (uint32_t)k;
                asm volatile("" : "+v"(kk));
                const uint32_t wo = ((uint32_t)slot * (uint32_t)a.nchunk + (uint32_t)chunk) * 49u + kk;
                a.wsum[wo] = s1;
                a.wsq[wo] = s2;
            }
        };
        if (RS == 2) partials();   // before the banded GEMM (the same wave's MFMA work follows)
        const bool active = kMmaRows * mt < rb && kMmaRows * nt < nsrc;   // wave-uniform
        if (FPM_CORR_PRIO == 1) __builtin_amdgcn_s_setprio(1);   // the GEMM and its epilogue
        if (MODE != 2 && active) {
            int sr = kMmaRows * nt + n;
            if (sr >= nsrc) sr = 0;   // column outside the band: computed, never stored
            const uint8_t* bp = SB + (size_t)sr * SBp + 16 * g;
            fpm_v4i acc[7];
            if (FPM_CORR_PRIO == 2) __builtin_amdgcn_s_setprio(1);
            if (NK > 0)
                band_mfma_regs<NA>(Areg, bp, a.nk, acc);
            else if (GA)
                band_mfma_ga(a.tmpl8 + (size_t)(T0 + kMmaRows * mt + n) * a.tp8 + 16 * g, bp, a.nk, acc);
            else
                band_mfma(TB + (size_t)(kMmaRows * mt + n) * TBp + 16 * g, bp, a.nk, acc);
            if (FPM_CORR_PRIO == 2) __builtin_amdgcn_s_setprio(0);
            // D_dx: col = lane & 15 -> source row 16*nt + n, row = 4*(lane >> 4) + r -> template row 16*mt + 4g + r
            uint32_t* rs_out = a.rowsum + (((size_t)th * 49 + 3) & ~(size_t)3) * slot + (size_t)T0 * 49;   // uniform
            const uint32_t kFix = 16384u * (uint32_t)tw;
            // the lane's row offsets as 32-bit values recomputed per item (opaque t0): kept across the item loop as
            // 64-bit addresses they were spilled, and each reload's vmcnt(0) waited for the previous rows' stores
            int t0 = kMmaRows * mt + 4 * g;
            asm volatile("" : "+v"(t0));
            const int s_ = kMmaRows * nt + n;
            // the template-row sums of the lane's 4 output rows from LDS (staged with the band; read from global memory
            // here, each row's load also waited for the previous row's stores: 4 memory round trips per item)
            const uint4 ts4 = *(const uint4*)(lts + t0);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int t = t0 + r, dy = s_ - t;
                if (t < rb && s_ < nsrc && dy >= 0 && dy < 7) {
                    const uint32_t ts = r == 0 ? ts4.x : r == 1 ? ts4.y : r == 2 ? ts4.z : ts4.w;
                    if (MODE == 5) {   // ablation: keep the MFMA results live, store nothing
                        uint32_t x = ts;
#pragma unroll
                        for (int d = 0; d < 7; ++d) x += (uint32_t)acc[d][r];
                        if (x == 0x9e3779b9u && a.W < 0) rs_out[t] = x;
                        continue;
                    }
                    const uint32_t o = (uint32_t)(t * 49 + dy * 7);
                    if (SE) {
#pragma unroll
                        for (int d = 0; d < 7; ++d) rsb[o + d] = (uint32_t)acc[d][r] + 128u * (wi[s_ * 7 + d] + ts) - kFix;
                        continue;
                    }
#pragma unroll
                    for (int d = 0; d < 7; ++d) rs_out[o + d] = (uint32_t)acc[d][r] + 128u * (wi[s_ * 7 + d] + ts) - kFix;
                }
            }
        }
        if (FPM_CORR_PRIO == 1) __builtin_amdgcn_s_setprio(0);
        if (RS == 1) partials();
        if (RS == 0 && MODE != 6 && tid < 2 * 49) {   // per-16-row-chunk partials of the window sums
            const int h = tid / 49, k = tid - h * 49;
            const int chunk = (T0 >> 4) + h;
            const int tlo = kMmaRows * h, thi = min(tlo + kMmaRows, rb);
            if (chunk < a.nchunk && tlo < thi) {
                const int pdy = k / 7, ddx = k - pdy * 7;
                uint32_t s1 = 0;
                uint64_t s2 = 0;
                for (int t = tlo; t < thi; ++t) {
                    s1 += wi[(t + pdy) * 7 + ddx];
                    s2 += wq[(t + pdy) * 7 + ddx];
                }
                a.wsum[((size_t)slot * a.nchunk + chunk) * 49 + k] = s1;
                a.wsq[((size_t)slot * a.nchunk + chunk) * 49 + k] = s2;
            }
        }
        if (SE) { pv_slot = slot; pv_T0 = T0; pv_rb = rb; }
    }
    if (SE && pv_slot >= 0) {   // the last item's row results
        __syncthreads();
        flush();
    }
}

#ifdef FPM_EXPERIMENTAL   // measured slower (bench 33.02k vs 34.10k searches/s): scripts/corr16_bench.hip only
// ---- K7, round 5: the register-A / LDS-DMA correlation with items of ONE 16-row M tile (k_roi_corr's band is two).
// A k_roi_corr item waits for its 38 ROI rows (one LDS-DMA round trip) and two barriers before its matrix work, and
// its 40 KB of LDS allow 4 items in flight per CU.  Here an item is (ROI, 16 template rows = one window-sum chunk):
// 22 ROI rows (18 KB), a 2-wave workgroup (wave w takes the N tile of ROI rows 16 w .. 16 w + 15, both waves the
// band's A fragments), about 22 KB of LDS, so 7 items are in flight per CU at the same waves per SIMD.  The price is
// 22 / 16 staged rows per template row instead of 38 / 32, and the same banded MFMA count (two N tiles per M tile).
// Outputs are k_roi_corr's exactly: the row dot products [t][49] (exact u32, through LDS as 16-byte runs during the
// next item, SE), and the window-sum partial of the item's chunk (one 16-row chunk per item).
constexpr int kB16Rows = kMmaRows, kB16Src = kB16Rows + 6;
__host__ __device__ inline size_t roi_corr16_lds(int roi_pitch) {
    return (size_t)kB16Src * roi_pitch + sizeof(uint32_t) * (2 * 7 * kB16Src + kB16Rows + kB16Rows * 49) + 64;
}
template <int NK, int WPE>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(WPE))) void k_roi_corr16(RoiArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int NT = 128;
    const int tw = a.tw, th = a.th, RW = tw + 6;
    const int SBp = a.roi_pitch;
    uint8_t* const SB = smem;                                   // kB16Src rows x SBp, bytes ^ 0x80
    uint32_t* wi = (uint32_t*)(SB + (size_t)kB16Src * SBp);     // [row][dx] window sums of I
    uint32_t* wq = wi + kB16Src * 7;                            // [row][dx] window sums of I^2
    uint32_t* lts = wq + kB16Src * 7;                           // the band's template-row sums
    uint32_t* rsb = lts + kB16Rows;                             // the band's [t][49] row results (16-byte aligned)
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int nband = (th + kB16Rows - 1) / kB16Rows;
    const int rois = roi_count(a), items = rois * nband;
    const int nwr = (RW + 3) >> 2;
    const int g = lane >> 4, n = lane & 15;
    const int txn = (RW + ROI_T - 1) / ROI_T;
    const XcdSplit xs = xcd_split(items);
    const int64_t span = xs.hi - xs.lo;
    const int it_lo = xs.lo + (int)(span * xs.k / xs.nk), it_hi = xs.lo + (int)(span * (xs.k + 1) / xs.nk);
    fpm_v4i Areg[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) Areg[k] = fpm_v4i{0, 0, 0, 0};
    int a_band = -1;
    int pv_slot = -1, pv_T0 = 0, pv_rb = 0;
    auto flush = [&]() {   // the previous item's row results: LDS -> its [rb][49] range of the ROI's series
        if (pv_slot < 0) return;
        uint32_t* dst = a.rowsum + (((size_t)th * 49 + 3) & ~(size_t)3) * pv_slot + (size_t)pv_T0 * 49;
        const int nw = pv_rb * 49, n16 = nw >> 2;
        for (int i = tid; i < n16; i += NT) *(uint4*)(dst + 4 * i) = *(const uint4*)(rsb + 4 * i);
        if (tid < (nw & 3)) dst[4 * n16 + tid] = rsb[4 * n16 + tid];
    };
    // item it's ROI rows wv + 2 i -> SB by LDS-DMA (one global_load_lds_dwordx4 per row and wave; lanes past the ROI
    // width idle: those LDS chunks meet the template's zero padding only)
    auto dma_rows = [&](int it) {
        const int bd = it / rois, sl = it - bd * rois;
        const int T0n = bd * kB16Rows, nsn = min(kB16Rows, th - T0n) + 6;
        const uint8_t* rsrc = a.roi + (size_t)sl * a.roi_stride;
        const uint32_t lane_off = ((uint32_t)(lane >> 1) << 10) + 16u * (uint32_t)(lane & 1);
        const int wvu = __builtin_amdgcn_readfirstlane(wv);
        const bool in_roi = lane < 2 * txn;
#pragma unroll
        for (int i = 0; i < (kB16Src + 1) / 2; ++i) {
            const int r = wvu + 2 * i;
            if (r < nsn && in_roi) {
                const int R = T0n + r;
                const uint8_t* gp = rsrc + ((size_t)((R >> 5) * txn) << 10) + (R & 31) * ROI_T + lane_off;
                const uint32_t ldsa = __builtin_amdgcn_readfirstlane(lds_offset_of(SB + (size_t)r * SBp));
                uint32_t keep;
                asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
                             "s_mov_b32 m0, %0"
                             : "=&s"(keep) : "v"(gp), "s"(ldsa) : "memory");
            }
        }
    };
    for (int item = it_lo; item < it_hi; ++item) {
        const int band = item / rois, slot = item - band * rois;
        const int T0 = band * kB16Rows, rb = min(kB16Rows, th - T0), nsrc = rb + 6;
        __syncthreads();   // the previous item is done with SB / wi / rsb
        dma_rows(item);
        flush();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (band != a_band) {   // this band's A fragments (both waves: the item's one M tile) and template-row sums
            a_band = band;
            if (tid < kB16Rows) lts[tid] = tid < rb ? (uint32_t)a.tsum[T0 + tid] : 0u;
            const int8_t* ap = a.tmpl8 + (size_t)(T0 + n) * a.tp8 + 16 * g;
#pragma unroll
            for (int k = 0; k < NK; ++k)
                if (k < a.nk) Areg[k] = *(const fpm_v4i*)(ap + 64 * k);
        }
        __syncthreads();
        if (tid < 4 * nsrc) {
            // row r's window sums by the quad of lanes 4r .. 4r + 3 (k_roi_corr's RS 1 form): full-row sums of I and I^2
            // reduced by DPP within the quad, each lane subtracting the edge pixels of its windows dx = q, q + 4
            const int r = tid >> 2, qq = tid & 3;
            const int per = (nwr + 3) >> 2, k0 = qq * per, k1 = min(nwr, k0 + per);
            const uint32_t* row = (const uint32_t*)(SB + (size_t)r * SBp);
            uint32_t s1 = 0, s2 = 0;
            int k = k0;
            for (; k + 8 <= k1; k += 8) {
                uint32_t x[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) x[u] = row[k + u] ^ 0x80808080u;
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    s1 = __builtin_amdgcn_udot4(x[u], 0x01010101u, s1, false);
                    s2 = __builtin_amdgcn_udot4(x[u], x[u], s2, false);
                }
            }
            for (; k < k1; ++k) {
                const uint32_t x = row[k] ^ 0x80808080u;
                s1 = __builtin_amdgcn_udot4(x, 0x01010101u, s1, false);
                s2 = __builtin_amdgcn_udot4(x, x, s2, false);
            }
            const uint32_t l0 = row[0] ^ 0x80808080u, l1 = row[1] ^ 0x80808080u;
            const int wr = tw >> 2;
            const uint32_t x0 = row[wr], x1 = row[wr + 1], x2 = row[wr + 2];
            const uint32_t e0 = __builtin_amdgcn_alignbyte(x1, x0, (uint32_t)tw) ^ 0x80808080u;
            const uint32_t e1 = __builtin_amdgcn_alignbyte(x2, x1, (uint32_t)tw) ^ 0x80808080u;
            s1 += (uint32_t)__builtin_amdgcn_mov_dpp((int)s1, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
            s2 += (uint32_t)__builtin_amdgcn_mov_dpp((int)s2, 0xB1, 0xF, 0xF, false);
            s1 += (uint32_t)__builtin_amdgcn_mov_dpp((int)s1, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
            s2 += (uint32_t)__builtin_amdgcn_mov_dpp((int)s2, 0x4E, 0xF, 0xF, false);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int dx = qq + 4 * h;
                if (dx < 7) {
                    const uint32_t ml0 = dx >= 4 ? 0xffffffffu : (1u << (8 * dx)) - 1u;
                    const uint32_t ml1 = dx <= 4 ? 0u : (1u << (8 * (dx - 4))) - 1u;
                    const uint32_t mr0 = dx >= 4 ? 0u : ~((1u << (8 * dx)) - 1u);
                    const uint32_t mr1 = dx <= 4 ? 0xffffu : dx == 5 ? 0xff00u : 0u;
                    const uint32_t a0 = l0 & ml0, a1 = l1 & ml1, b0 = e0 & mr0, b1 = e1 & mr1;
                    uint32_t q1 = __builtin_amdgcn_udot4(a0, 0x01010101u, 0u, false);
                    q1 = __builtin_amdgcn_udot4(a1, 0x01010101u, q1, false);
                    q1 = __builtin_amdgcn_udot4(b0, 0x01010101u, q1, false);
                    q1 = __builtin_amdgcn_udot4(b1, 0x01010101u, q1, false);
                    uint32_t q2 = __builtin_amdgcn_udot4(a0, a0, 0u, false);
                    q2 = __builtin_amdgcn_udot4(a1, a1, q2, false);
                    q2 = __builtin_amdgcn_udot4(b0, b0, q2, false);
                    q2 = __builtin_amdgcn_udot4(b1, b1, q2, false);
                    wi[r * 7 + dx] = s1 - q1;
                    wq[r * 7 + dx] = s2 - q2;
                }
            }
        }
        __syncthreads();
        if (kMmaRows * wv < nsrc) {   // wave-uniform: wave 1's N tile exists
            int sr = kMmaRows * wv + n;
            if (sr >= nsrc) sr = 0;   // column outside the band: computed, never stored
            const uint8_t* bp = SB + (size_t)sr * SBp + 16 * g;
            fpm_v4i acc[7];
            band_mfma_regs<NK>(Areg, bp, a.nk, acc);
            const uint32_t kFix = 16384u * (uint32_t)tw;
            int t0 = 4 * g;
            asm volatile("" : "+v"(t0));
            const int s_ = kMmaRows * wv + n;
            const uint4 ts4 = *(const uint4*)(lts + t0);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int t = t0 + r, dy = s_ - t;
                if (t < rb && s_ < nsrc && dy >= 0 && dy < 7) {
                    const uint32_t ts = r == 0 ? ts4.x : r == 1 ? ts4.y : r == 2 ? ts4.z : ts4.w;
                    const uint32_t o = (uint32_t)(t * 49 + dy * 7);
#pragma unroll
                    for (int d = 0; d < 7; ++d) rsb[o + d] = (uint32_t)acc[d][r] + 128u * (wi[s_ * 7 + d] + ts) - kFix;
                }
            }
        }
        // the item's chunk partial of the window sums (positions k by lane pairs, 8 rows each, combined by DPP)
        if (tid < 2 * 49) {
            const int k = tid >> 1, half = tid & 1;
            const int chunk = T0 >> 4;
            const int pdy = k / 7, ddx = k - pdy * 7;
            const int t0 = 8 * half, n8 = min(8, rb - t0);
            uint32_t s1 = 0, x[8], y[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = (t0 + u + pdy) * 7 + ddx;
                x[u] = u < n8 ? wi[i] : 0u;
                y[u] = u < n8 ? wq[i] : 0u;
            }
            uint64_t s2 = 0;
#pragma unroll
            for (int u = 0; u < 8; ++u) { s1 += x[u]; s2 += y[u]; }
            s1 += (uint32_t)__builtin_amdgcn_mov_dpp((int)s1, 0xB1, 0xF, 0xF, false);
            const uint32_t lo = (uint32_t)s2, hi = (uint32_t)(s2 >> 32);
            s2 += (uint64_t)(uint32_t)__builtin_amdgcn_mov_dpp((int)lo, 0xB1, 0xF, 0xF, false) |
                  ((uint64_t)(uint32_t)__builtin_amdgcn_mov_dpp((int)hi, 0xB1, 0xF, 0xF, false) << 32);
            if (half == 0 && chunk < a.nchunk) {
                uint32_t kk = (uint32_t)k;
                asm volatile("" : "+v"(kk));
                const uint32_t wo = ((uint32_t)slot * (uint32_t)a.nchunk + (uint32_t)chunk) * 49u + kk;
                a.wsum[wo] = s1;
                a.wsq[wo] = s2;
            }
        }
        pv_slot = slot; pv_T0 = T0; pv_rb = rb;
    }
    if (pv_slot >= 0) {   // the last item's row results
        __syncthreads();
        flush();
    }
}

#endif   // FPM_EXPERIMENTAL (k_roi_corr16)

#ifdef FPM_EXPERIMENTAL   // measurement-only kernel (scripts/fused_bench.hip); the product Makefile never defines it
// ---- K6+K7 fused (templates too large for k_roi_small): the ROI never leaves the CU.  A work unit is one ROI and
// one run of consecutive 32-row template bands; a workgroup walks its run band by band:
//   the band's new ROI rows are sampled straight into an LDS ring of kBandSrc rows (32x32 tiles: the tile's
//   source footprint staged in wave-private LDS, the bilinear taps gathered from it — K6b's sampler, with the
//   warp tables computed in LDS instead of read from HBM), their exact row sums of I and I^2 reduced on the fly;
//   the 6 rows a band shares with the next stay in the ring (ring slot = ROI row mod kBandSrc);
//   then K7's banded GEMM on the matrix cores (A fragments of the band in registers, loaded during the sampling)
//   and its epilogue: the exact per-row dot products and the per-16-row window-sum partials, exactly k_roi_corr's
//   outputs, so K8 (k_roi_eval) folds them unchanged.
// Only the first band of a run samples its 6 leading rows again (runs of ~3.5 bands: ~4.5 % extra sampling), the
// ~0.4 MB sampled ROI of a layer-0 Src7 candidate is neither written to nor re-read from HBM, and the per-ROI warp
// tables / tile descriptors need no kernel of their own.
constexpr int kFuseFt = 3072;                  // per-wave footprint: any <= 32x32 interior tile box is <= 56 x 49 B
constexpr int kFuseFtStride = kFuseFt + 64;    // + over-read slack
constexpr int kFuseWgs = 256 * 3;              // 3 workgroups per CU (LDS ~52 KB, <= 168 VGPRs at layer 0)

struct FuseLayout {
    int sbp, ft, tab, rt, sums, mat, total;
};
__host__ __device__ inline FuseLayout fuse_layout(int tw) {
    FuseLayout L;
    const int txn = (tw + 6 + ROI_T - 1) / ROI_T;
    L.sbp = roi_pitch_calc(tw);
    L.ft = kBandSrc * L.sbp;                   // ring of kBandSrc ROI rows (i8: I ^ 0x80), pitch sbp
    L.tab = L.ft + 4 * kFuseFtStride;          // ad[32 txn], bd[32 txn] (int32)
    L.rt = L.tab + 8 * ROI_T * txn;            // x0[32], y0[32] of the row block being sampled
    L.sums = L.rt + 8 * ROI_T;                 // rall, rallq [kBandSrc], wi, wq [kBandSrc][7] (ring slots)
    L.mat = L.sums + 4 * 16 * kBandSrc;        // the ROI's affine map (6 doubles)
    L.total = L.mat + 8 * 6;
    return L;
}
bool roi_fused_fits(int tw) { return (tw + 63) / 64 <= 16 && 3 * (size_t)fuse_layout(tw).total <= 160 * 1024; }
int roi_fused_parts(int th) {
    const int nband = (th + kBandRows - 1) / kBandRows;
    const int p = (2 * nband + 3) / 7;         // runs of ~3.5 bands
    return p < 1 ? 1 : p;
}

// sum over each aligned group of 8 lanes, in every lane of the group: quad_perm [1,0,3,2], [2,3,0,1], then
// row_half_mirror (lane i <-> 7 - i of the 8) — three DPP adds, no LDS traffic
__device__ __forceinline__ uint32_t sum8_dpp(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);
    return v;
}

template <int NK>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void k_roi_fused(RoiArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tw = a.tw, th = a.th, RW = tw + 6, W = a.W, H = a.H;
    const FuseLayout LY = fuse_layout(tw);
    const int SBp = LY.sbp;
    const int txn = (RW + ROI_T - 1) / ROI_T;
    uint8_t* SB = smem;
    int32_t* lad = (int32_t*)(smem + LY.tab);
    int32_t* lbd = lad + ROI_T * txn;
    int32_t* lx0 = (int32_t*)(smem + LY.rt);
    int32_t* ly0 = lx0 + ROI_T;
    uint32_t* rall = (uint32_t*)(smem + LY.sums);
    uint32_t* rallq = rall + kBandSrc;
    uint32_t* wi = rallq + kBandSrc;
    uint32_t* wq = wi + kBandSrc * 7;
    double* lM = (double*)(smem + LY.mat);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    uint8_t* FT = smem + LY.ft + wv * kFuseFtStride;
    const int nband = (th + kBandRows - 1) / kBandRows;
    const int nparts = a.nparts;
    const int units = roi_count(a) * nparts;
    const int g = lane >> 4, n = lane & 15;
    const int mt = wv & 1, nt = mt + (wv >> 1);   // this wave's (M, N) tile pair (k_roi_corr)
    const int lr = lane >> 3, lg = lane & 7;      // sampling: rows lr + 8i, columns 4 lg .. 4 lg + 3 of a tile
    const uint32_t kFix = 16384u * (uint32_t)tw;
    auto ring = [](int r) { return r % kBandSrc; };
    const XcdSplit xs = xcd_split(units);         // an XCD group takes a contiguous run of units (an ROI's runs
                                                  // and the candidate's other angles share source lines in L2)
    for (int u = xs.lo + xs.k; u < xs.hi; u += xs.nk) {
        const int slot = u / nparts, part = u - slot * nparts;
        const int b0 = part * nband / nparts, b1 = (part + 1) * nband / nparts;
        int id, jj;
        roi_slot(a, slot, id, jj);
        const uint8_t* lvl = a.level + (size_t)(id / a.per_source) * a.level_stride;
        __syncthreads();   // the previous unit is done with every LDS array
        {
            double M[6];
            const CandState st = a.state[id];
            const AngleNode nd = a.nodes[st.node * a.n3 + jj];
            roi_matrix(W, H, f2(st.lt.x * 2, st.lt.y * 2), nd.c, nd.s, M);   // getRotatedROI :1074-1090
            for (int x = tid; x < ROI_T * txn; x += 256) {   // warpAffine's adelta / bdelta (k_roi_tables)
                lad[x] = rint_i(M[0] * x * kAbScale);
                lbd[x] = rint_i(M[3] * x * kAbScale);
            }
            if (tid < 6) lM[tid] = M[tid];   // the row terms are computed per row block (below)
        }
        uint32_t* rs_out = a.rowsum + (((size_t)th * 49 + 3) & ~(size_t)3) * slot;
        for (int b = b0; b < b1; ++b) {
            const int T0 = b * kBandRows, rb = min(kBandRows, th - T0), nsrc = rb + 6;
            const int rlo = b == b0 ? 0 : 6;       // ring rows T0 .. T0 + 5 carried from the previous band
            // new rows T0 + rlo .. T0 + nsrc - 1, in row blocks of <= 32 (one tile row each)
            for (int rb0 = rlo; rb0 < nsrc; rb0 += ROI_T) {
                const int nr = min(ROI_T, nsrc - rb0), R0 = T0 + rb0;   // ROI rows R0 .. R0 + nr - 1
                __syncthreads();   // the previous block's sampling is done with x0 / y0; (first block) the previous
                                   // band's MFMA is done with the ring rows and window sums overwritten here
                if (tid < nr) {
                    const int y = R0 + tid;
                    lx0[tid] = rint_i((lM[1] * y + lM[2]) * kAbScale) + kRoundDelta;
                    ly0[tid] = rint_i((lM[4] * y + lM[5]) * kAbScale) + kRoundDelta;
                    rall[ring(y)] = 0u;
                    rallq[ring(y)] = 0u;
                }
                __syncthreads();
                for (int tx = wv; tx < txn; tx += 4) {
                    const int cx0 = tx * ROI_T, cx1 = min(cx0 + ROI_T, RW) - 1;
                    // the tile's source footprint box from its corner samples (+-1 px, see k_roi_tables)
                    int bx0 = INT_MAX, bx1 = INT_MIN, by0 = INT_MAX, by1 = INT_MIN;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int c = (k & 1) ? cx1 : cx0, r = (k & 2) ? nr - 1 : 0;
                        const int X = (lx0[r] + lad[c]) >> (kAbBits - kInterBits);
                        const int Y = (ly0[r] + lbd[c]) >> (kAbBits - kInterBits);
                        bx0 = min(bx0, X >> kInterBits); bx1 = max(bx1, X >> kInterBits);
                        by0 = min(by0, Y >> kInterBits); by1 = max(by1, Y >> kInterBits);
                    }
                    const bool interior = bx0 - 1 >= 0 && bx1 + 1 <= W - 2 && by0 - 1 >= 0 && by1 + 1 <= H - 2;
                    bx0 = max(bx0 - 1, 0); by0 = max(by0 - 1, 0);
                    bx1 = min(bx1 + 2, W - 1); by1 = min(by1 + 2, H - 1);
                    const bool any = bx0 <= bx1 && by0 <= by1;
                    const int bxa = bx0 & ~3;
                    int ftw = any ? ((bx1 - bxa + 4) & ~3) : 0;
                    if (((ftw >> 2) & 1) == 0) ftw += 4;    // odd dword pitch: spread gather banks
                    const int fth = any ? by1 - by0 + 1 : 0;
                    const int wpr = ftw >> 2;
                    const bool in_lds = wpr <= 16 && ftw * fth <= kFuseFt;
                    wave_sync();   // the previous tile's gathers are done with FT
                    if (any && in_lds) stage_footprint<2>(FT, ftw, wpr, fth, lvl + (size_t)by0 * a.P + bxa, a.P, bxa, a.P, lane);
                    wave_sync();
                    const int c0 = cx0 + 4 * lg;
                    int adv[4], bdv[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) { adv[q] = lad[c0 + q]; bdv[q] = lbd[c0 + q]; }
                    const int nvalid = RW - c0;
                    const uint32_t colmask = nvalid >= 4 ? 0xffffffffu : (nvalid <= 0 ? 0u : (1u << (8 * nvalid)) - 1u);
                    const int xo = ((int)lds_offset_of(FT) - bxa) << kAbBits, yo = -(by0 << kAbBits);
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int rr = lr + 8 * i;
                        const int rc = rr < nr ? rr : nr - 1;   // rows past the block repeat its last row, unstored
                        uint32_t pk = 0;
                        if (interior && in_lds) {   // folded LDS addressing, the row's 16 tap reads before arithmetic
                            const int x0r = lx0[rc] + xo, y0r = ly0[rc] + yo;
                            uint32_t off[4];
                            int fxv[4], fyv[4], v[4][4];
#pragma unroll
                            for (int q = 0; q < 4; ++q) {
                                const int sxv = x0r + adv[q], syv = y0r + bdv[q];
                                fxv[q] = __builtin_amdgcn_ubfe(sxv, kAbBits - kInterBits, kInterBits);
                                fyv[q] = __builtin_amdgcn_ubfe(syv, kAbBits - kInterBits, kInterBits);
                                off[q] = (uint32_t)mad24(syv >> kAbBits, ftw, sxv >> kAbBits);
                            }
#pragma unroll
                            for (int q = 0; q < 4; ++q) lds_taps(off[q], ftw, v[q]);
#pragma unroll
                            for (int q = 0; q < 4; ++q) pk |= (uint32_t)bilerp24(v[q], fxv[q], fyv[q]) << (8 * q);
                        } else {
#pragma unroll
                            for (int q = 0; q < 4; ++q) {
                                const int X = (lx0[rc] + adv[q]) >> (kAbBits - kInterBits);
                                const int Y = (ly0[rc] + bdv[q]) >> (kAbBits - kInterBits);
                                const int v = !any ? 0 : in_lds ? ft_tap_general(FT, ftw, bxa, by0, W, H, X, Y)
                                                                : roi_tap(lvl, W, H, a.P, X, Y);
                                pk |= (uint32_t)v << (8 * q);
                            }
                        }
                        pk &= colmask;
                        // exact row sums of I and I^2 over the row's 32 tile columns (8 lanes), one LDS atomic each
                        uint32_t s1 = __builtin_amdgcn_udot4(pk, 0x01010101u, 0u, false);
                        uint32_t s2 = __builtin_amdgcn_udot4(pk, pk, 0u, false);
                        s1 = sum8_dpp(s1);
                        s2 = sum8_dpp(s2);
                        if (rr < nr) {
                            const int slotr = ring(R0 + rr);
                            *(uint32_t*)(SB + (size_t)slotr * SBp + c0) = pk ^ 0x80808080u;
                            if (lg == 0) {
                                atomicAdd(&rall[slotr], s1);
                                atomicAdd(&rallq[slotr], s2);
                            }
                        }
                    }
                }
            }
            __syncthreads();   // the band's rows and row sums are complete
            // this band's A fragments (L2-resident slab; rows past the template are the slab's zero padding), in
            // flight during the edge sums
            fpm_v4i Areg[NK];
            {
                const int8_t* ap = a.tmpl8 + (size_t)(T0 + kMmaRows * mt + n) * a.tp8 + 16 * g;
#pragma unroll
                for (int k = 0; k < NK; ++k)
                    Areg[k] = k < a.nk ? *(const fpm_v4i*)(ap + 64 * k) : fpm_v4i{0, 0, 0, 0};
            }
            for (int i = tid; i < (nsrc - rlo) * 7; i += 256) {   // window [dx, dx + tw): full row minus edges
                const int r = ring(T0 + rlo + i / 7), dx = i % 7;
                const uint8_t* sbr = SB + (size_t)r * SBp;
                uint32_t q1 = rall[r], q2 = rallq[r];
                for (int c = 0; c < dx; ++c) { const uint32_t v = sbr[c] ^ 0x80u; q1 -= v; q2 -= v * v; }
                for (int c = dx + tw; c < RW; ++c) { const uint32_t v = sbr[c] ^ 0x80u; q1 -= v; q2 -= v * v; }
                wi[r * 7 + dx] = q1;
                wq[r * 7 + dx] = q2;
            }
            __syncthreads();
            if (kMmaRows * mt < rb && kMmaRows * nt < nsrc) {   // wave-uniform
                int sr = kMmaRows * nt + n;
                if (sr >= nsrc) sr = 0;   // column outside the band: computed, never stored
                const uint8_t* bp = SB + (size_t)ring(T0 + sr) * SBp + 16 * g;
                const uint4 ts4 = ld_at<uint4>(a.tsum, 4u * (T0 + kMmaRows * mt + 4 * g));   // (see k_roi_corr)
                fpm_v4i acc[7];
                band_mfma_regs<NK>(Areg, bp, a.nk, acc);
                // D_dx: col = lane & 15 -> source row 16*nt + n, row = 4*(lane >> 4) + r -> template row 16*mt + 4g + r
                const int s_ = kMmaRows * nt + n;
                const uint32_t* wr = wi + ring(T0 + (s_ < nsrc ? s_ : 0)) * 7;
                // element (template row tb + r, dy = s_ - tb - r, dx = d) of the band's [t][49] block sits at
                // ob[42 r + d]: one pointer per lane, immediate offsets
                const int tb = kMmaRows * mt + 4 * g;
                uint32_t* ob = rs_out + (size_t)(T0 + tb) * 49 + (s_ - tb) * 7;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int t = tb + r, dy = s_ - t;
                    if (t < rb && s_ < nsrc && dy >= 0 && dy < 7) {
                        const uint32_t ts = r == 0 ? ts4.x : r == 1 ? ts4.y : r == 2 ? ts4.z : ts4.w;
#pragma unroll
                        for (int d = 0; d < 7; ++d) ob[42 * r + d] = (uint32_t)acc[d][r] + 128u * (wr[d] + ts) - kFix;
                    }
                }
            }
            if (tid < 2 * 49) {   // per-16-row-chunk partials of the window sums (k_roi_corr)
                const int h = tid / 49, k = tid - h * 49;
                const int chunk = (T0 >> 4) + h;
                const int tlo = kMmaRows * h, thi = min(tlo + kMmaRows, rb);
                if (chunk < a.nchunk && tlo < thi) {
                    const int pdy = k / 7, ddx = k - pdy * 7;
                    uint32_t s1 = 0;
                    uint64_t s2 = 0;
                    for (int t = tlo; t < thi; ++t) {
                        const int r = ring(T0 + t + pdy) * 7 + ddx;
                        s1 += wi[r];
                        s2 += wq[r];
                    }
                    a.wsum[((size_t)slot * a.nchunk + chunk) * 49 + k] = s1;
                    a.wsq[((size_t)slot * a.nchunk + chunk) * 49 + k] = s2;
                }
            }
        }
    }
}
#endif   // FPM_EXPERIMENTAL

// candidate step of :329-366 as a pure function of the state and the n3 records (k_cand_step, k_roi_eval, the
// k_roi_small prologue)
// next_nodes != nullptr: also loads the stepped candidate's next-layer node of angle jj into *next_nd (issued with the
// child's own node, off the dependent-load chain of a k_roi_small prologue)
__device__ __forceinline__ CandState cand_step_state(CandState s, int n3, const AngleNode* nodes, double thr, int W,
                                                     int H, int mark_reached0, const float* score, const int* mx,
                                                     const int* my, const AngleNode* next_nodes = nullptr,
                                                     int jj = 0, AngleNode* next_nd = nullptr, int nnext = 1) {
    int imax = 0;
    double big = -1;
    for (int k = 0; k < n3; ++k)
        if ((double)score[k] > big) { imax = k; big = score[k]; }
    if ((double)score[imax] < thr) {   // :331-332
        s.alive = 0;
        return s;
    }
    const int child = s.node * n3 + imax;
    const AngleNode nd = nodes[child];
    if (next_nodes)
        for (int k = 0; k < nnext; ++k) next_nd[k] = next_nodes[child * n3 + jj + k];
    const F2 sc = f2((W - 1) / 2.0f, (H - 1) / 2.0f);
    const F2 r0 = rotate_pt(f2(s.lt.x * 2, s.lt.y * 2), sc, nd.c, nd.s);   // :350-353
    const F2 pad = f2(r0.x - 3, r0.y - 3);
    F2 p = f2((float)((double)mx[imax] + pad.x), (float)((double)my[imax] + pad.y));
    p = rotate_pt(p, sc, nd.cn, nd.sn);
    s.lt = p;          // :366
    s.node = child;    // :363
    s.reached0 = mark_reached0;
    return s;
}

// ---- K6-K8 for small templates: one workgroup per ROI does the whole refinement of the ROI in LDS (tables,
// 32x32-tile sampling from wave footprints, exact row / window sums, the band-by-band banded GEMM on the matrix
// cores, the ordered f32 fold, CCOEFF, argmax, 3x3) and writes its RoiRecord; k_cand_step then steps the
// candidates.  Used where the ROI, the template and one band of row sums fit the LDS budget (upper layers), so a
// layer costs two launches instead of four and no scratch leaves the CU.
struct SmallLayout {
    int sbp, tbp, rh, u, tab, sum, rs, sc, ts, total;
};
// The U region holds, one after the other: the ROI's whole source footprint or (when that does not fit) one 32x32
// tile's footprint per wave, then the template rows.  A pure rotation keeps the footprint's box within the ROI's
// diagonal D (+ the sampling margins and alignment of k_roi_small: width <= D + 14, height <= D + 4), so where that
// box is smaller than the per-wave tile buffers U is sized to it and the tile path is never taken (it then reads
// its taps from global memory, should it be).  nw = waves per workgroup.
// (integer arithmetic only: host and device must size the LDS regions identically, so no sqrtf whose rounding could
// differ between the two compilations; isqrt_ceil = the smallest d with d * d >= n)
__host__ __device__ inline int isqrt_ceil(int n) {
    int d = 0;
    while ((d + 1) * (d + 1) <= n) ++d;   // floor(sqrt(n)) (n < 2^21 here: a ROI diagonal, at most ~1500 steps)
    return d * d == n ? d : d + 1;
}
__host__ __device__ inline int small_footprint_bound(int rw, int rh) {
    const int d = isqrt_ceil((rw - 1) * (rw - 1) + (rh - 1) * (rh - 1)) + 2;
    return ((d + 16) * (d + 6) + 15) & ~15;
}
__host__ __device__ inline SmallLayout small_layout(int tw, int th, int nw = 4) {
    SmallLayout L;
    L.sbp = roi_pitch_calc(tw);
    L.tbp = tmpl_lds_pitch(64 * ((tw + 63) / 64));
    L.rh = th + 6;
    const int th16 = (th + kMmaRows - 1) / kMmaRows * kMmaRows;
    L.u = ((L.rh + 16) * L.sbp + 15) & ~15;       // SB rows + slack rows read by the last band's N tiles
    const int fb = small_footprint_bound(tw + 6, th + 6);
    const int fp = fb < nw * ROI_FT ? fb : nw * ROI_FT;
    const int ub = th16 * L.tbp > fp ? th16 * L.tbp : fp;
    L.tab = L.u + ub;
    L.sum = L.tab + 4 * (2 * L.sbp + 2 * ((L.rh + 3) & ~3));
    // the band's row sums live only in the band phase, when the footprints (U) and the warp tables (tab) are dead and U
    // holds the template rows: placed after those rows when they fit there (Src7 layer 3: 46.1 -> 39.8 KB per
    // workgroup, 3 -> 4 workgroups per CU), else after the window sums
    const int rs_size = 4 * kBandRows * 49;
    const int after_sums = L.sum + 4 * (2 * L.rh + 2 * 7 * L.rh) + 8 * 49 * 2;
    if (th16 * L.tbp + rs_size <= L.sum - L.u) {
        L.rs = L.u + th16 * L.tbp;
        L.sc = after_sums;
    } else {
        L.rs = after_sums;
        L.sc = L.rs + rs_size;
    }
    L.ts = L.sc + 4 * 64;
    L.total = L.ts + 4 * th16;
    return L;
}
constexpr int kSmallLdsMax = 72 * 1024;
bool roi_small_fits(int tw, int th) { return th <= 256 && small_layout(tw, th).total <= kSmallLdsMax; }
size_t roi_small_lds(int tw, int th) { return (size_t)small_layout(tw, th).total; }

// MODE (profiling ablations in scripts/roi_microbench.hip; the product uses 0): 1 = tables + sampling only,
// 2 = + row / window sums, 3 = + bands without the fold, 5 = full with byte-gather taps, 9 = full with per-phase
// s_memtime stamps (a.stamps)
// PROL: the previous layer's candidate step in the prologue (a.prev_rec set; a separate instantiation: its registers
// would cost the plain form spills, 11 -> 33 VGPRs at 4 waves, k_roi_small 178 -> 207 us per 43-source pass)
// NT: threads per workgroup (256; 128: two waves per ROI, so twice the ROIs per CU where the waves and not the LDS
// bound the residency, the four MFMA tile pairs of a band then in two passes per wave; 512: eight waves per ROI for
// layers with fewer ROIs than CUs, the sampling and staging spread over twice the lanes); needs RW <= 4 NT
template <int MODE, int WPE = 3, bool PROL = false, int NT = 256>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(WPE))) void k_roi_small(RoiArgs a) {
    constexpr int NW = NT / 64;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tw = a.tw, th = a.th, RW = tw + 6, RH = th + 6, W = a.W, H = a.H;
    const SmallLayout LY = small_layout(tw, th, NW);
    const int SBp = LY.sbp, TBp = LY.tbp;
    uint8_t* SB = smem;                                  // RH ROI rows x SBp (u8, then ^ 0x80)
    uint8_t* TB = smem + LY.u;                           // template rows (i8) x TBp
    uint8_t* FTall = smem + LY.u;                        // (sampling phase) 4 wave footprints
    int32_t* lad = (int32_t*)(smem + LY.tab);
    int32_t* lbd = lad + SBp;
    int32_t* lx0 = lbd + SBp;
    int32_t* ly0 = lx0 + ((RH + 3) & ~3);
    uint32_t* rall = (uint32_t*)(smem + LY.sum);
    uint32_t* rallq = rall + RH;
    uint32_t* wi = rallq + RH;                           // [row][dx]
    uint32_t* wq = wi + RH * 7;
    uint64_t* tot = (uint64_t*)(((uintptr_t)(wq + RH * 7) + 7) & ~(uintptr_t)7);   // [2][49] window totals
    uint32_t* rs = (uint32_t*)(smem + LY.rs);            // kBandRows x 49 row sums of the current band
    float* sc = (float*)(smem + LY.sc);
    uint32_t* lts = (uint32_t*)(smem + LY.ts);            // template-row sums, 16-row padded
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int rois = roi_count(a);
    const int q4 = SBp >> 4, nwr = (RW + 3) >> 2;
    const int txn = (RW + ROI_T - 1) / ROI_T, tyn = (RH + ROI_T - 1) / ROI_T;
    const int g = lane >> 4, n = lane & 15;
    const int lr = lane >> 3, lg = lane & 7;
    auto STAMP = [&](int k) {
        if (MODE == 9 && tid == 0 && blockIdx.x < 64) a.stamps[blockIdx.x * 16 + k] = __builtin_readcyclecounter();
    };
    for (int slot = blockIdx.x; slot < rois; slot += gridDim.x) {
        STAMP(0);
        int id, jj;
        roi_slot(a, slot, id, jj);
        const uint8_t* lvl = a.level + (size_t)(id / a.per_source) * a.level_stride;
        CandState st = a.state[id];
        AngleNode nd;
        if (PROL) {   // the previous layer's candidate step (same inputs, same result in every thread)
            if (st.alive) {
                const RoiRecord* r = a.prev_rec + (size_t)id * a.n3;
                float score[3];
                int mx[3], my[3];
                for (int k = 0; k < a.n3; ++k) { score[k] = r[k].score; mx[k] = r[k].mx; my[k] = r[k].my; }
                st = cand_step_state(st, a.n3, a.prev_nodes, a.prev_thr, a.prev_W, a.prev_H, 0, score, mx, my, a.nodes,
                                     jj, &nd);
                if (jj == 0 && tid == 0 && st.alive) atomicAdd(a.live_out_count, 1);   // live entering this layer
            }
            if (jj == 0 && tid == 0) a.state_out[id] = st;
            if (!st.alive) continue;   // uniform over the workgroup
        } else {
            nd = a.nodes[st.node * a.n3 + jj];
        }
        __syncthreads();
        {   // warpAffine tables of this ROI (getRotatedROI :1074-1090)
            double M[6];
            roi_matrix(W, H, f2(st.lt.x * 2, st.lt.y * 2), nd.c, nd.s, M);
            for (int x = tid; x < RW; x += NT) {
                lad[x] = rint_i(M[0] * x * kAbScale);
                lbd[x] = rint_i(M[3] * x * kAbScale);
            }
            for (int y = tid; y < RH; y += NT) {
                lx0[y] = rint_i((M[1] * y + M[2]) * kAbScale) + kRoundDelta;
                ly0[y] = rint_i((M[4] * y + M[5]) * kAbScale) + kRoundDelta;
            }
        }
        __syncthreads();
        STAMP(1);
        // the ROI's whole source footprint (corner samples +-1 px, see k_roi_tables) if it fits the U region
        int gbx0 = INT_MAX, gbx1 = INT_MIN, gby0 = INT_MAX, gby1 = INT_MIN;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int c = (k & 1) ? RW - 1 : 0, r = (k & 2) ? RH - 1 : 0;
            const int X = (lx0[r] + lad[c]) >> (kAbBits - kInterBits);
            const int Y = (ly0[r] + lbd[c]) >> (kAbBits - kInterBits);
            gbx0 = min(gbx0, X >> kInterBits); gbx1 = max(gbx1, X >> kInterBits);
            gby0 = min(gby0, Y >> kInterBits); gby1 = max(gby1, Y >> kInterBits);
        }
        const bool g_interior = gbx0 - 1 >= 0 && gbx1 + 1 <= W - 2 && gby0 - 1 >= 0 && gby1 + 1 <= H - 2;
        gbx0 = max(gbx0 - 1, 0); gby0 = max(gby0 - 1, 0);
        gbx1 = min(gbx1 + 2, W - 1); gby1 = min(gby1 + 2, H - 1);
        const bool g_any = gbx0 <= gbx1 && gby0 <= gby1;
        const int gbxa = gbx0 & ~3;
        const int gftw = g_any ? ((gbx1 - gbxa + 4) & ~3) + 4 : 4;   // +4: odd-ish pitch vs banks
        const int gfth = g_any ? gby1 - gby0 + 1 : 0;
        const int gobase = gby0 * gftw + gbxa;
        if (g_any && gftw * gfth <= LY.tab - LY.u) {   // wave-uniform (same values in every thread)
            uint8_t* FT = FTall;
            const int wpr = gftw >> 2;
            stage_block4(FT, gftw, lvl + (size_t)gby0 * a.P + gbxa, a.P, gfth, wpr, gbxa, a.P, tid, NT);
            __syncthreads();
            STAMP(8);
            // thread -> one fixed group of 4 columns (its column table entries held in registers) and every
            // nrl-th row: no per-item division, 2 table reads per 4 pixels instead of 10
            const int ngrp = (RW + 3) >> 2;
            const int nrl = NT / ngrp;                    // row lanes (>= 1: RW <= 4 NT for this kernel)
            const int rl = tid / ngrp, c0 = 4 * (tid - rl * ngrp);
            int ad4[4], bd4[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) { ad4[u] = lad[c0 + u]; bd4[u] = lbd[c0 + u]; }
            if (g_interior && MODE != 5) {   // folded LDS addressing, a row's 16 tap reads before its arithmetic
                const int xo = ((int)lds_offset_of(FT) - gbxa) << kAbBits, yo = -(gby0 << kAbBits);
                const int nvalid = RW - c0;
                const uint32_t colmask = nvalid >= 4 ? 0xffffffffu : (nvalid <= 0 ? 0u : (1u << (8 * nvalid)) - 1u);
                for (int r = rl < nrl ? rl : RH; r < RH; r += nrl) {
                    const int x0r = lx0[r] + xo, y0r = ly0[r] + yo;
                    uint32_t off[4];
                    int fxv[4], fyv[4], v[4][4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int sxv = x0r + ad4[u], syv = y0r + bd4[u];
                        fxv[u] = __builtin_amdgcn_ubfe(sxv, kAbBits - kInterBits, kInterBits);
                        fyv[u] = __builtin_amdgcn_ubfe(syv, kAbBits - kInterBits, kInterBits);
                        off[u] = (uint32_t)mad24(syv >> kAbBits, gftw, sxv >> kAbBits);
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) lds_taps(off[u], gftw, v[u]);
                    uint32_t pk = 0;
#pragma unroll
                    for (int u = 0; u < 4; ++u) pk |= (uint32_t)bilerp24(v[u], fxv[u], fyv[u]) << (8 * u);
                    *(uint32_t*)(SB + r * SBp + c0) = pk & colmask;
                }
            } else {
                for (int r = rl < nrl ? rl : RH; r < RH; r += nrl) {
                    const int X0 = lx0[r], Y0 = ly0[r];
                    uint32_t pk = 0;
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int X = (X0 + ad4[u]) >> (kAbBits - kInterBits);
                        const int Y = (Y0 + bd4[u]) >> (kAbBits - kInterBits);
                        int v;
                        if (g_interior) {
                            const int off = mad24(Y >> kInterBits, gftw, (X >> kInterBits) - gobase);
                            v = ft_tap_bytes(FT, off, gftw, X, Y);
                        } else {
                            v = ft_tap_general(FT, gftw, gbxa, gby0, W, H, X, Y);
                        }
                        if (c0 + u >= RW) v = 0;
                        pk |= (uint32_t)v << (8 * u);
                    }
                    *(uint32_t*)(SB + r * SBp + c0) = pk;
                }
            }
            STAMP(9);
        } else if (!g_any) {   // the ROI lies entirely outside the image: all zero (BORDER_CONSTANT 0)
            for (int i = tid; i < RH * (SBp >> 2); i += NT) ((uint32_t*)SB)[i] = 0u;
        } else {   // footprint too large: one 32x32 tile per wave at a time (in LDS where U holds a buffer per wave)
            const bool tile_bufs = NW * ROI_FT <= LY.tab - LY.u;
            uint8_t* FT = FTall + wv * ROI_FT;
            for (int task = wv; task < txn * tyn; task += NW) {
                const int ty = task / txn, tx = task - ty * txn;
                const int cx0 = tx * ROI_T, cx1 = min(cx0 + ROI_T, RW) - 1;
                const int ry0 = ty * ROI_T, ry1 = min(ry0 + ROI_T, RH) - 1;
                int bx0 = INT_MAX, bx1 = INT_MIN, by0 = INT_MAX, by1 = INT_MIN;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int c = (k & 1) ? cx1 : cx0, r = (k & 2) ? ry1 : ry0;
                    const int X = (lx0[r] + lad[c]) >> (kAbBits - kInterBits);
                    const int Y = (ly0[r] + lbd[c]) >> (kAbBits - kInterBits);
                    bx0 = min(bx0, X >> kInterBits); bx1 = max(bx1, X >> kInterBits);
                    by0 = min(by0, Y >> kInterBits); by1 = max(by1, Y >> kInterBits);
                }
                const bool interior = bx0 - 1 >= 0 && bx1 + 1 <= W - 2 && by0 - 1 >= 0 && by1 + 1 <= H - 2;
                bx0 = max(bx0 - 1, 0); by0 = max(by0 - 1, 0);
                bx1 = min(bx1 + 2, W - 1); by1 = min(by1 + 2, H - 1);
                const bool any = bx0 <= bx1 && by0 <= by1;
                const int bxa = bx0 & ~3;
                int ftw = any ? ((bx1 - bxa + 4) & ~3) : 0;
                if (((ftw >> 2) & 1) == 0) ftw += 4;
                const int fth = any ? by1 - by0 + 1 : 0;
                const int wpr = ftw >> 2;
                const bool in_lds = tile_bufs && wpr <= 16 && ftw * fth <= ROI_FT;
                wave_sync();
                if (any && in_lds) stage_footprint<4>(FT, ftw, wpr, fth, lvl + (size_t)by0 * a.P + bxa, a.P, bxa, a.P, lane);
                wave_sync();
                const int c0 = cx0 + 4 * lg;
                if (c0 > cx1) continue;
                for (int i = 0; i < 4; ++i) {
                    const int r = ry0 + lr + 8 * i;
                    if (r > ry1) break;
                    const int X0 = lx0[r], Y0 = ly0[r];
                    uint32_t pk = 0;
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int X = (X0 + lad[c0 + u]) >> (kAbBits - kInterBits);
                        const int Y = (Y0 + lbd[c0 + u]) >> (kAbBits - kInterBits);
                        int v;
                        if (interior && in_lds) {
                            const int off = mad24(Y >> kInterBits, ftw, (X >> kInterBits) - (by0 * ftw + bxa));
                            v = MODE == 5 ? ft_tap_bytes(FT, off, ftw, X, Y) : ft_tap_interior(FT, off, ftw, X, Y);
                        } else {
                            v = in_lds ? ft_tap_general(FT, ftw, bxa, by0, W, H, X, Y) : roi_tap(lvl, W, H, a.P, X, Y);
                        }
                        if (c0 + u >= RW) v = 0;
                        pk |= (uint32_t)v << (8 * u);
                    }
                    *(uint32_t*)(SB + r * SBp + c0) = pk;
                }
            }
        }
        __syncthreads();
        if (MODE == 1) continue;
        STAMP(2);
        for (int r = tid; r < RH; r += NT) {   // exact full-row sums of I and I^2, one thread per row
            const uint32_t* row = (const uint32_t*)(SB + (size_t)r * SBp);
            uint32_t s1 = 0, s2 = 0;
            int k = 0;
            for (; k + 8 <= nwr; k += 8) {
                uint32_t x[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) x[u] = row[k + u];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    s1 = __builtin_amdgcn_udot4(x[u], 0x01010101u, s1, false);
                    s2 = __builtin_amdgcn_udot4(x[u], x[u], s2, false);
                }
            }
            for (; k < nwr; ++k) {
                const uint32_t x = row[k];
                s1 = __builtin_amdgcn_udot4(x, 0x01010101u, s1, false);
                s2 = __builtin_amdgcn_udot4(x, x, s2, false);
            }
            rall[r] = s1;
            rallq[r] = s2;
        }
        __syncthreads();
        for (int i = tid; i < RH * q4; i += NT) {   // bytes flipped to the signed MFMA operand
            uint4* v = (uint4*)SB + i;   // rows are contiguous (pitch SBp = 16 * q4)
            uint4 x = *v;
            x.x ^= 0x80808080u; x.y ^= 0x80808080u; x.z ^= 0x80808080u; x.w ^= 0x80808080u;
            *v = x;
        }
        {   // all template rows (padded to 16) of the i8 slab
            const int trows = (th + kMmaRows - 1) / kMmaRows * kMmaRows;
            stage_block16(TB, TBp, (const uint8_t*)a.tmpl8, a.tp8, trows, a.tp8 >> 4, tid, NT);
            // and the template-row sums (trows <= 256) for the band epilogues (3 waves per SIMD: 82.9 -> 81.0 us per
            // Src7 layer-3 launch; the 4-wave form reads them from global memory there, as its registers spill more)
            if (WPE < 4)
                for (int i = tid; i < (NT >= 256 ? min(trows, NT) : trows); i += NT) lts[i] = (uint32_t)a.tsum[i];
        }
        __syncthreads();
        STAMP(3);
        for (int r = tid; r < RH; r += NT) {    // windows [dx, dx + tw) of a row: full row minus <= 6 edge pixels,
            const uint8_t* sbr = SB + (size_t)r * SBp;   // the row's 12 edge bytes read once by one thread
            uint32_t lv[6], rv[6];
#pragma unroll
            for (int c = 0; c < 6; ++c) { lv[c] = sbr[c] ^ 0x80u; rv[c] = sbr[tw + c] ^ 0x80u; }
            uint32_t q1 = rall[r], q2 = rallq[r];
#pragma unroll
            for (int c = 0; c < 6; ++c) { q1 -= rv[c]; q2 -= rv[c] * rv[c]; }   // dx = 0: columns tw .. tw + 5
#pragma unroll
            for (int dx = 0; dx < 7; ++dx) {
                if (dx > 0) {   // column dx - 1 leaves on the left, column tw + dx - 1 enters on the right
                    q1 += rv[dx - 1] - lv[dx - 1];
                    q2 += rv[dx - 1] * rv[dx - 1] - lv[dx - 1] * lv[dx - 1];
                }
                wi[r * 7 + dx] = q1;
                wq[r * 7 + dx] = q2;
            }
        }
        if (tid < 98) tot[tid] = 0;   // (NT >= 128)
        __syncthreads();
        STAMP(4);
        // window totals of the 49 positions (exact): 4 threads per position, u64 LDS adds (NT < 196: a loop)
#pragma unroll 1
        for (int q = tid; q < (NT >= 4 * 49 ? (tid < 4 * 49 ? tid + 1 : 0) : 4 * 49); q += NT) {
            const int part = q / 49, k = q - part * 49, pdy = k / 7, ddx = k - pdy * 7;
            const int t0 = part * th / 4, t1 = (part + 1) * th / 4;
            uint64_t s1 = 0, s2 = 0;
            int t = t0;
            for (; t + 8 <= t1; t += 8) {   // 8 LDS reads of each in flight
                uint32_t x[8], y[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) { x[u] = wi[(t + u + pdy) * 7 + ddx]; y[u] = wq[(t + u + pdy) * 7 + ddx]; }
#pragma unroll
                for (int u = 0; u < 8; ++u) { s1 += x[u]; s2 += y[u]; }
            }
            for (; t < t1; ++t) { s1 += wi[(t + pdy) * 7 + ddx]; s2 += wq[(t + pdy) * 7 + ddx]; }
            atomicAdd((unsigned long long*)&tot[k], (unsigned long long)s1);
            atomicAdd((unsigned long long*)&tot[49 + k], (unsigned long long)s2);
        }
        if (MODE == 2) continue;
        STAMP(5);
        float accF = 0.f;
        uint64_t accI = 0;
        const uint32_t kFix = 16384u * (uint32_t)tw;
        for (int T0 = 0; T0 < th; T0 += kBandRows) {   // bands in row order: MFMA -> LDS row sums -> fold
            const int rb = min(kBandRows, th - T0), nsrc = rb + 6;
            // the band's four (M, N) tile pairs (t, s) = (0, 0), (1, 1), (0, 1), (1, 2): pair p on wave p % NW (NW = 8:
            // waves 4-7 have none)
#pragma unroll
            for (int pass = 0; pass < (4 + NW - 1) / NW; ++pass) {
            const int p = wv + pass * NW, mt = p & 1, nt = mt + (p >> 1);
            if (p < 4 && kMmaRows * mt < rb && kMmaRows * nt < nsrc) {
                const uint8_t* ap = TB + (size_t)(T0 + kMmaRows * mt + n) * TBp + 16 * g;
                const uint8_t* bp = SB + (size_t)(T0 + kMmaRows * nt + n) * SBp + 16 * g;   // slack rows cover sr >= RH
                fpm_v4i acc[7];
                band_mfma(ap, bp, a.nk, acc);
                const int s_ = kMmaRows * nt + n;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int t = kMmaRows * mt + 4 * g + r, dy = s_ - t;
                    if (t < rb && s_ < nsrc && dy >= 0 && dy < 7) {
                        const uint32_t ts = WPE < 4 ? lts[T0 + t] : (uint32_t)a.tsum[T0 + t];
#pragma unroll
                        for (int d = 0; d < 7; ++d)
                            rs[t * 49 + dy * 7 + d] = (uint32_t)acc[d][r] + 128u * (wi[(T0 + s_) * 7 + d] + ts) - kFix;
                    }
                }
            }
            }
            __syncthreads();
            if (MODE != 3 && tid < 49) {
                if (a.fold) {
                    int t = 0;
                    for (; t + 8 <= rb; t += 8) {   // 8 LDS reads in flight, adds in row order (:507)
                        uint32_t x[8];
#pragma unroll
                        for (int u = 0; u < 8; ++u) x[u] = rs[(t + u) * 49 + tid];
#pragma unroll
                        for (int u = 0; u < 8; ++u) accF = accF + (float)(int)x[u];
                    }
                    for (; t < rb; ++t) accF = accF + (float)(int)rs[t * 49 + tid];
                } else {
                    for (int t = 0; t < rb; ++t) accI += rs[t * 49 + tid];
                }
            }
            __syncthreads();
        }
        if (tid < 49) {
            const double num = a.fold ? (double)accF : (double)(float)(double)accI;
            sc[tid] = ccoeff(num, (double)tot[tid], (double)tot[49 + tid], a.mean, a.norm, a.inv_area);
        }
        __syncthreads();
        STAMP(6);
        if (wv == 0) {   // cv::minMaxLoc: first maximum in row-major order, as a wave reduction
            float v = lane < 49 ? sc[lane] : -INFINITY;
            int bi = lane < 49 ? lane : 64;
            if (v != v) { v = -INFINITY; bi = 64 + lane; }   // a NaN never beats the running maximum
            wave_better_reduce(v, bi);                        // largest value, lowest index among equals
            const float s0 = sc[0];
            if (s0 != s0 || bi >= 64) bi = 0;                 // the scan starts at sc[0]: a NaN there stays
            const float best = sc[bi];
            const int mx = bi % 7, my = bi / 7;
            RoiRecord r;
            r.score = best;
            r.mx = (int16_t)mx;
            r.my = (int16_t)my;
            const int border = (mx == 0 || my == 0 || mx == 6 || my == 6) ? 1 : 0;
            r.on_border = border;
            for (int x = -1; x <= 1; ++x)
                for (int y = -1; y <= 1; ++y) r.vec[(x + 1) * 3 + (y + 1)] = border ? 0.f : sc[(my + y) * 7 + (mx + x)];
            // (the candidate step follows in k_cand_step: fusing it here as a last-arriver hand-off between
            // workgroups, system-coherent stores + one agent-scope atomic per record, cost 30 us per layer at 32
            // sources: every workgroup then waits for its write-through stores; measured r02)
            if (lane == 0) a.rec[(size_t)id * a.n3 + jj] = r;
        }
        STAMP(7);
    }
}

// candidate step of :329-366 from the scores and 7x7 argmax positions of a candidate's n3 records: best of the
// angles, early break below vecLayerScore, back-mapping of ptLT, append to the next live list
// returns the survivor's position in the next live list (-1: dead) and its stepped state in *so
// nn != nullptr (with a.nt_tab): also the survivor's n3 next-layer nodes, loaded beside its own child node
__device__ int cand_step_one(const RoiArgs& a, int id, const float* score, const int* mx, const int* my,
                             CandState* so = nullptr, AngleNode* nn = nullptr) {
    CandState* out = a.state_out ? a.state_out : a.state;
    CandState s = a.state[id];
    if (!s.alive) {   // a hole of a prologue-stepped run (k_roi_small prev_rec): dead before this layer
        out[id] = s;
        return -1;
    }
    s = cand_step_state(s, a.n3, a.nodes, a.thr, a.W, a.H, a.mark_reached0, score, mx, my, nn ? a.nt_nodes : nullptr,
                        0, nn, a.n3);
    out[id] = s;
    if (so) *so = s;
    if (!s.alive) return -1;
    const int p = atomicAdd(a.live_out_count, 1);
    a.live_out[p] = id;
    return p;
}

// the next layer's tables of a survivor at live position p (RoiArgs::nt_tab; wave j <-> refinement angle j)
__device__ __forceinline__ void cand_next_tables(const RoiArgs& a, int id, int p, const CandState& s,
                                                 const AngleNode& nd, int j, int lane) {
    roi_tables_fill(a.nt_tab, a.tdesc, a.tdesc_stride, a.nt_tabw, a.nt_tabh, a.nt_tw, a.nt_th, a.nt_W, a.nt_H,
                    p * a.n3 + j, s.lt, nd, (id / a.per_source) << kTileSrcShift, lane, 64);
}

// the candidate step as its own launch over the live list (after k_roi_small's equal1 records)
__global__ __launch_bounds__(256) void k_cand_step(RoiArgs a) {
    const int n = *a.live_count;
    for (int li = blockIdx.x * 256 + threadIdx.x; li < n; li += gridDim.x * 256) {
        const int id = a.live[li];
        const RoiRecord* r = a.rec + (size_t)id * a.n3;
        float score[3];
        int mx[3], my[3];
        for (int k = 0; k < a.n3; ++k) { score[k] = r[k].score; mx[k] = r[k].mx; my[k] = r[k].my; }
        cand_step_one(a, id, score, mx, my);
    }
}

// the candidate step with the next layer's tables (RoiArgs::nt_tab): one workgroup per live candidate, thread 0
// steps, wave j writes the tables of the survivor's angle j (saves the next layer's k_roi_tables launch)
__global__ __launch_bounds__(192) void k_cand_step_tab(RoiArgs a) {
    __shared__ int pos;
    __shared__ CandState ns;
    __shared__ AngleNode nn[3];
    const int n = *a.live_count;
    const int lane = threadIdx.x & 63, j = threadIdx.x >> 6;
    for (int li = blockIdx.x; li < n; li += gridDim.x) {
        const int id = a.live[li];
        __syncthreads();   // previous candidate's pos / ns consumed
        if (threadIdx.x == 0) {
            const RoiRecord* r = a.rec + (size_t)id * a.n3;
            float score[3];
            int mx[3], my[3];
            for (int k = 0; k < a.n3; ++k) { score[k] = r[k].score; mx[k] = r[k].mx; my[k] = r[k].my; }
            CandState s;
            pos = cand_step_one(a, id, score, mx, my, &s, a.nt_tab ? nn : nullptr);
            ns = s;
        }
        __syncthreads();
        if (pos >= 0 && j < a.n3) cand_next_tables(a, id, pos, ns, nn[j], j, lane);
    }
}

// ---- K8: per live candidate (one wave per refinement angle j): ordered f32 fold of the ROI's 49 row-sum series
// (:505-508), window sums, CCOEFF, argmax, border, 3x3 -> RoiRecord; then (layers > 0) the candidate step of
// :329-366: best of the n3 angles, early break below vecLayerScore, back-mapping of ptLT, append to the next live
// list.  Each wave streams its [th][49] series through wave-private LDS in blocks of kEvalRows rows, the next
// block's loads in flight while 49 lanes fold the current one in row order.  No workgroup barrier in the loop.
// Blocks of ROWS rows: 40 for batches (8 loads per lane, 48 KB of LDS per three-wave workgroup, so three workgroups per
// CU -- 768 candidates at once, which holds the bench's 64-source context passes (<= 704 candidates per layer) in one
// round; 48-row blocks: 10 loads, 61 KB, two per CU, the same time per launch when one round holds the layer, round
// 4), 48 for a lone search (fewer blocks, so fewer LDS-DMA round trips in each wave's chain)
template <int ROWS>
struct EvalBlk {
    static_assert(ROWS * 49 % 4 == 0, "a block is whole uint4 of the [th][49] series");
    static constexpr int dma = (ROWS * 49 / 4 + 63) / 64;   // 16-byte LDS-DMA loads per lane per block
    static constexpr int buf = dma * 1024;                  // bytes per block buffer
};

template <int ROWS>
__device__ void eval_roi(const RoiArgs& a, int slot, int lane, uint8_t* blk, float* sc, RoiRecord* out,
                         RoiRecord* keep) {
    constexpr int kEvalRows = ROWS, kEvalDma = EvalBlk<ROWS>::dma, kEvalBuf = EvalBlk<ROWS>::buf;
    const int th = a.th;
    if (a.equal1) {   // CCOEFF_Denominator: matResult = 1 everywhere (:529-533)
        if (lane == 0) {
            RoiRecord r;
            r.score = 1.f; r.mx = 0; r.my = 0; r.on_border = 1;
            for (int k = 0; k < 9; ++k) r.vec[k] = 0.f;
            *out = r;
            *keep = r;
        }
        return;
    }
    const size_t total4 = ((size_t)th * 49 + 3) >> 2;   // uint4 per ROI series (slot stride 4 * total4)
    const uint4* rs = (const uint4*)(a.rowsum + (size_t)slot * total4 * 4);
    uint64_t s1 = 0, s2 = 0;
    if (lane < 49) {   // window sums over the chunk partials
        const uint32_t* ws = a.wsum + (size_t)slot * a.nchunk * 49 + lane;
        const uint64_t* wq = a.wsq + (size_t)slot * a.nchunk * 49 + lane;
        int c = 0;
        for (; c + 8 <= a.nchunk; c += 8) {
            uint32_t x[8];
            uint64_t y[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) { x[u] = ws[(size_t)(c + u) * 49]; y[u] = wq[(size_t)(c + u) * 49]; }
#pragma unroll
            for (int u = 0; u < 8; ++u) { s1 += x[u]; s2 += y[u]; }
        }
        for (; c < a.nchunk; ++c) { s1 += ws[(size_t)c * 49]; s2 += wq[(size_t)c * 49]; }
    }
    // the series streams through two wave-private LDS buffers by LDS-DMA: block b + 1 (exactly kEvalDma
    // 16-byte loads per lane, padded with dummy loads so a counted vmcnt is exact) is in flight while block b folds
    constexpr int BQ = kEvalRows * 49 / 4;   // uint4 per block
    const int nblk = (th + kEvalRows - 1) / kEvalRows;
    auto issue_block = [&](int b, uint8_t* buf) {
#pragma unroll
        for (int i = 0; i < kEvalDma; ++i) {
            size_t q = (size_t)b * BQ + 64 * i + lane;
            if (64 * i + lane >= BQ || q >= total4) q = 0;   // dummy: lands past the rows that are read
            // inline asm: the compiler does not track this LDS-DMA, so it inserts no vmcnt(0) before the fold's
            // LDS reads; the counted waits below order them (the guide's documented recipe)
            uint32_t keep;
            const uint32_t ldsa = (uint32_t)(uintptr_t)(fpm_lds_vp)(buf + 1024 * i);
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep) : "v"(rs + q), "s"(__builtin_amdgcn_readfirstlane(ldsa)) : "memory");
        }
    };
    float accF = 0.f;
    uint64_t accI = 0;
    issue_block(0, blk);
    for (int b = 0; b < nblk; ++b) {
        const uint32_t* cb = (const uint32_t*)(blk + (b & 1) * kEvalBuf);
        if (b + 1 < nblk) {
            issue_block(b + 1, blk + ((b + 1) & 1) * kEvalBuf);
            asm volatile("s_waitcnt vmcnt(%0)" :: "i"(kEvalDma) : "memory");   // block b + 1's loads may stay in flight
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        wave_sync();
        const int rows = min(kEvalRows, th - b * kEvalRows);
        if (lane < 49) {
            if (a.fold) {
                int t = 0;
                for (; t + 8 <= rows; t += 8) {   // 8 LDS reads in flight, adds in row order (:507)
                    uint32_t x[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) x[u] = cb[(t + u) * 49 + lane];
#pragma unroll
                    for (int u = 0; u < 8; ++u) accF = accF + (float)(int)x[u];
                }
                for (; t < rows; ++t) accF = accF + (float)(int)cb[t * 49 + lane];
            } else {
                for (int t = 0; t < rows; ++t) accI += cb[t * 49 + lane];
            }
        }
        wave_sync();   // block b folded before its buffer is refilled with block b + 2
    }
    if (lane < 49) {
        const double num = a.fold ? (double)accF : (double)(float)(double)accI;
        sc[lane] = ccoeff(num, (double)s1, (double)s2, a.mean, a.norm, a.inv_area);
    }
    wave_sync();
    if (lane == 0) {   // cv::minMaxLoc: first maximum in row-major order
        float best = sc[0];
        int bi = 0;
        for (int k = 1; k < 49; ++k)
            if (sc[k] > best) { best = sc[k]; bi = k; }
        const int mx = bi % 7, my = bi / 7;
        RoiRecord r;
        r.score = best;
        r.mx = (int16_t)mx;
        r.my = (int16_t)my;
        const int border = (mx == 0 || my == 0 || mx == 6 || my == 6) ? 1 : 0;
        r.on_border = border;
        for (int x = -1; x <= 1; ++x)
            for (int y = -1; y <= 1; ++y) r.vec[(x + 1) * 3 + (y + 1)] = border ? 0.f : sc[(my + y) * 7 + (mx + x)];
        *out = r;
        *keep = r;
    }
}

template <int ROWS>
__global__ __launch_bounds__(192) void k_roi_eval(RoiArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t blk_all[3][2 * EvalBlk<ROWS>::buf];
    __shared__ float sc_all[3][64];
    __shared__ RoiRecord recs[3];
    __shared__ int pos;
    __shared__ CandState ns;
    __shared__ AngleNode nn[3];
    const int lane = threadIdx.x & 63, j = threadIdx.x >> 6;   // wave j <-> refinement angle j
    const int rois = roi_count(a);
    const int base = roi_base(a);
    const int c_lo = base / a.n3, c_hi = (base + rois) / a.n3;   // rounds hold whole candidates
    for (int li = c_lo + blockIdx.x; li < c_hi; li += gridDim.x) {
        const int id = a.live[li];
        const int slot = li * a.n3 + j - base;
        __syncthreads();   // previous candidate's records consumed
        eval_roi<ROWS>(a, slot, lane, blk_all[j], sc_all[j], a.rec + (size_t)id * a.n3 + j, &recs[j]);
        if (!a.step) continue;
        __syncthreads();
        if (threadIdx.x == 0) {   // TemplateMatcher.cpp:329-366
            float score[3];
            int mx[3], my[3];
            for (int k = 0; k < a.n3; ++k) { score[k] = recs[k].score; mx[k] = recs[k].mx; my[k] = recs[k].my; }
            CandState s;
            pos = cand_step_one(a, id, score, mx, my, &s, a.nt_tab ? nn : nullptr);
            ns = s;
        }
        if (!a.nt_tab) continue;
        __syncthreads();
        if (pos >= 0) cand_next_tables(a, id, pos, ns, nn[j], j, lane);   // the next layer's tables (no k_roi_tables)
    }
}

void launch_roi_tables(const RoiArgs& a, hipStream_t st) {
    if (a.slot_cap <= 0 || a.equal1) return;
    const int grid = a.slot_cap < 4096 ? a.slot_cap : 4096;
    hipLaunchKernelGGL(k_roi_tables, dim3(grid), dim3(256), 0, st, a);
}

// footprint rows in flight per lane and waves per SIMD: each staging round trip is one memory latency per wave, so
// more rows in flight pay until the registers cost occupancy.  Src7 layer-0 microbenchmark at the bench's 43 sources
// per pass (1419 ROIs, 579 K tiles): round 3 before the uniform staging loop, batch 2 509 us, 4 486, 8 479, 16 557-580
// (5-6 waves); with it (61 VGPRs at batch 8), batch 8 at 7 waves 458, batch 4 / 8 / 12 at 8 waves 448 / 450 / 446
// (scripts/gpu_kpass_mb.sh, profiles/r03_i)
constexpr int kWarpFootBatch = 12, kWarpWaves = 8;
// Workgroup caps of the looping kernels (every one of them loops over its work, so the results do not depend on the
// grid).  With several contexts in flight (the bench: three HIP streams), a grid of one workgroup per work item keeps
// the kernel's queue ahead of the other streams' kernels for its whole run; a persistent grid of the kernel's own
// residency leaves the slots its workgroups free at the end to the other contexts.  Measured on the bench (128
// Src7 sources over 3 contexts, one box, profiles/r05c, r05d): k_roi_small capped at its residency 33.27-33.52k ->
// 33.93-34.23k searches/s.  The sampler at its residency (7 per CU) gained +0.3-1.2 % at 128 sources per step
// (profiles/r05f) but nothing at the bench's 192 (34.58k / 34.59k vs 34.56k / 34.54k uncapped, 34.61k / 34.66k at
// 2688, alternated, profiles/r05j), while its static task ranges make each launch 7 % slower on its own (239 vs
// 222 us at 64 sources): uncapped by default.  FPM_GRID_WARP / FPM_GRID_CORR /
// FPM_GRID_SMALL (read when a search is recorded): N > 0 caps the kernel at N workgroups, 0 lifts the cap (the
// uncapped grids of round 4), unset: the defaults at each launch below.
static int grid_cap_env(const char* v, int dflt) { return v ? (atoi(v) > 0 ? atoi(v) : 0) : dflt; }
static int capped(int grid, int cap) { return cap > 0 && grid > cap ? cap : grid; }
// the device's compute units (hipDeviceProp_t::multiProcessorCount, read once per device; 256 on MI355X): the
// persistent grids and the lone-search rules below scale with it
static int device_cus() {
    int dev = 0;
    (void)hipGetDevice(&dev);
    static std::mutex mu;
    static std::map<int, int> cus;
    std::lock_guard<std::mutex> lock(mu);
    auto it = cus.find(dev);
    if (it != cus.end()) return it->second;
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
    return n;
}
void launch_roi_warp(const RoiArgs& a, hipStream_t st) {
    if (a.slot_cap <= 0 || a.equal1) return;
    const long tiles = (long)a.slot_cap * ((a.th + 6 + ROI_T - 1) / ROI_T) * ((a.tw + 6 + ROI_T - 1) / ROI_T);
    if (tiles > INT_MAX) return;   // the engine bounds slot_cap far below this
    const long want = (tiles + 3) / 4;
    const int grid = (int)(want < 16384 ? want : 16384);
    // a candidate's three angle ROIs from one staged union footprint (k_roi_warp3; Src7 kernel pass at 43 sources:
    // layer 0 395 -> 329 us, layer 1 114 -> 99, bench 28.07k -> 29.62k searches/s, profiles/r03_r); FPM_WARP3=0 keeps
    // one ROI per task (measurement)
    const char* w3e = getenv("FPM_WARP3");   // read when the search is recorded (once per plan)
    const int warp3 = w3e ? atoi(w3e) : 1;
    if (warp3 && a.n3 == 3 && a.slot_base % 3 == 0 && a.slot_cap % 3 == 0) {
        const long want3 = (tiles / 3 + 3) / 4;
        // 7 waves per SIMD with the first ROI's tables requested before the staging (8 would spill them): microbenchmark
        // 405.5 / 406.3 -> 400.6 / 402.0 us (round 3)
        // batches of at most two sources (a lone search) run at the residency: the grid is sized for the plan's candidate
        // capacity, mostly idle workgroups there, and fewer dispatches take a lone Src7 search's layer 0 from 19.5 to
        // 15.1 us (profiles/r05m vs r05_end lat_*.txt); larger batches keep the full grid (its dynamic balance beats the
        // persistent grid's static task ranges, r05j)
        const int srcs = a.slot_cap / std::max(1, a.per_source * a.n3);
        const int dflt_cap = srcs <= 2 ? 7 * device_cus() : 0;
        hipLaunchKernelGGL((k_roi_warp3<7, kFtPitch, 0>), dim3(capped((int)(want3 < 16384 ? want3 : 16384), grid_cap_env(getenv("FPM_GRID_WARP"), dflt_cap))),
                           dim3(256), 0, st, a);
        return;
    }
    hipLaunchKernelGGL((k_roi_warp<kWarpFootBatch, 0, kWarpWaves>), dim3(grid), dim3(256), 0, st, a);
}

constexpr size_t kLdsPerCu = 160 * 1024;   // MI355X (gfx950) LDS per CU
constexpr bool kCorrGlobalA = true;   // measured in scripts/roi_microbench.hip
constexpr int kCorrWaves = 3;
// register-A form at 13-16 k-steps: 2 waves per SIMD (A fragments + prefetched rows: 221 VGPRs), one workgroup per
// resident slot (MI355X: 256 CUs)
constexpr int kCorrRunWaves = 2;
template <int NK>
static void launch_corr_regs(const RoiArgs& a, long items, size_t lds, hipStream_t st) {
    if constexpr (NK <= 12) {
        // up to 12 k-steps the A fragments fit 3 waves per SIMD (166 VGPRs) without the row prefetch; measured
        // faster than the prefetching 2-wave form (occupancy hides the staging latency better)
        // at 4 k-steps 4 waves per SIMD pay despite a 28-byte spill (Src7 layer 2: 68.2 -> 58.0 us per 43-source
        // launch); at 8 / 12 k-steps the larger spills lose (136.5 -> 145.2, 301.1 -> 403.2 us)
        // ... and at 8 k-steps since the load addressing is scalar (136 VGPRs at 3 waves, 4 spilled at 4 waves: Src7
        // layer 1 107.7 -> 99.4 us per 43-source microbenchmark launch, profiles/r03_y)
        if (NK == 4 && lds * 4 <= kLdsPerCu) {
            const int grid = capped((int)std::min<long>(items, 4L * device_cus()), grid_cap_env(getenv("FPM_GRID_CORR"), 0));
            hipLaunchKernelGGL((k_roi_corr<0, true, 4, NK, false, 1, true>), dim3(grid), dim3(256), lds, st, a);
            return;
        }
        // at 8 and 12 k-steps the source rows staged by LDS-DMA (no staging VGPRs) make room for 4 waves per SIMD
        // (43 Src7 sources: layer 0 269.8 -> 241.1 us, profiles/r04/mb_r04e.txt; layer 1 103.0 -> 93.5 us,
        // profiles/r04/mbl1_r04g.txt; host-checked)
        if ((NK == 8 || NK == 12) && lds * 4 <= kLdsPerCu) {
            const int grid = capped((int)std::min<long>(items, 4L * device_cus()), grid_cap_env(getenv("FPM_GRID_CORR"), 0));
            hipLaunchKernelGGL((k_roi_corr<0, true, 4, NK, false, 1, true, true>), dim3(grid), dim3(256), lds, st, a);
            return;
        }
        // row results staged in LDS and flushed during the next item's staging (SE; Src7 microbenchmark at 43 sources:
        // layer 0 293.6 -> 264.4 us, layer 1 124.2 -> 115.4, bit-identical)
        const int grid = capped((int)std::min<long>(items, (long)kCorrWaves * device_cus()), grid_cap_env(getenv("FPM_GRID_CORR"), 0));
        hipLaunchKernelGGL((k_roi_corr<0, true, kCorrWaves, NK, false, 1, true>), dim3(grid), dim3(256), lds, st, a);
    } else {
        const int grid = (int)std::min<long>(items, (long)kCorrRunWaves * device_cus());
        hipLaunchKernelGGL((k_roi_corr<0, true, kCorrRunWaves, NK>), dim3(grid), dim3(256), lds, st, a);
    }
}
#ifdef FPM_EXPERIMENTAL
// k_roi_corr16 (16-row items, 2-wave workgroups): as many workgroups as the LDS holds per CU, persistent
bool launch_roi_corr16(const RoiArgs& a, hipStream_t st) {
    if (a.nk > 12 || (a.roi_pitch >> 4) > 64) return false;
    const size_t lds = roi_corr16_lds(a.roi_pitch);
    const int per_cu = (int)std::min<size_t>(8, kLdsPerCu / lds);
    if (per_cu < 1) return false;
    const long items = (long)a.slot_cap * ((a.th + kB16Rows - 1) / kB16Rows);
    const int grid = capped((int)std::min<long>(items, (long)per_cu * device_cus()), grid_cap_env(getenv("FPM_GRID_CORR"), 0));
    if (a.nk <= 4) hipLaunchKernelGGL((k_roi_corr16<4, 4>), dim3(grid), dim3(128), lds, st, a);
    else if (a.nk <= 8) hipLaunchKernelGGL((k_roi_corr16<8, 4>), dim3(grid), dim3(128), lds, st, a);
    else hipLaunchKernelGGL((k_roi_corr16<12, 4>), dim3(grid), dim3(128), lds, st, a);
    return true;
}

#endif

void launch_roi_corr(const RoiArgs& a, hipStream_t st) {
    if (a.slot_cap <= 0 || a.equal1) return;
    const size_t lds = roi_corr_lds(a.roi_pitch, a.tw, a.rc, kCorrGlobalA);
    // register-A form where its staged rows fit one 64-lane pass and A fits 16 k-steps (templates <= 1024 wide);
    // the slot-major form below serves wider templates
    if ((a.roi_pitch >> 4) <= 64 && a.nk <= 16 && lds <= 65536) {
        const long items = (long)a.slot_cap * ((a.th + kBandRows - 1) / kBandRows);
        if (a.nk <= 4) launch_corr_regs<4>(a, items, lds, st);
        else if (a.nk <= 8) launch_corr_regs<8>(a, items, lds, st);
        else if (a.nk <= 12) launch_corr_regs<12>(a, items, lds, st);
        else launch_corr_regs<16>(a, items, lds, st);
        return;
    }
    ensure_lds_attr((const void*)k_roi_corr<0, kCorrGlobalA, kCorrWaves>, lds);
    const long items = (long)a.slot_cap * ((a.th + kBandRows - 1) / kBandRows);
    const int grid = (int)(items < 16384 ? items : 16384);
    hipLaunchKernelGGL((k_roi_corr<0, kCorrGlobalA, kCorrWaves>), dim3(grid), dim3(256), lds, st, a);
}

#ifdef FPM_EXPERIMENTAL
void launch_roi_fused(const RoiArgs& a, hipStream_t st) {
    if (a.slot_cap <= 0 || a.equal1) return;
    const size_t lds = (size_t)fuse_layout(a.tw).total;
    const long units = (long)a.slot_cap * a.nparts;
    const int grid = (int)(units < kFuseWgs ? units : kFuseWgs);
    if (a.nk <= 4) hipLaunchKernelGGL(k_roi_fused<4>, dim3(grid), dim3(256), lds, st, a);
    else if (a.nk <= 8) hipLaunchKernelGGL(k_roi_fused<8>, dim3(grid), dim3(256), lds, st, a);
    else if (a.nk <= 12) hipLaunchKernelGGL(k_roi_fused<12>, dim3(grid), dim3(256), lds, st, a);
    else hipLaunchKernelGGL(k_roi_fused<16>, dim3(grid), dim3(256), lds, st, a);
}
#endif

void launch_roi_eval(const RoiArgs& a, hipStream_t st) {
    if (a.slot_cap <= 0) return;
    const int cands = (a.slot_cap + a.n3 - 1) / a.n3;
    const int grid = cands < 4096 ? cands : 4096;
    const int srcs = a.slot_cap / std::max(1, a.per_source * a.n3);   // (batches of <= 2 sources: a lone search)
    if (srcs <= 2) hipLaunchKernelGGL(k_roi_eval<48>, dim3(grid), dim3(64 * a.n3), 0, st, a);
    else hipLaunchKernelGGL(k_roi_eval<40>, dim3(grid), dim3(64 * a.n3), 0, st, a);
}

void launch_roi_small(const RoiArgs& a, hipStream_t st) {
    if (a.slot_cap <= 0) return;
    if (a.equal1) {   // records of ones (CCOEFF_Denominator :529-533); the step follows in k_cand_step
        RoiArgs b = a;
        b.step = 0;
        launch_roi_eval(b, st);
        return;
    }
    // two-wave workgroups at 4 waves per SIMD (8 per CU) where that holds more ROIs per CU than the four-wave form, i.e.
    // where the waves and not the LDS bound the residency (Src7 layers 4 and 5: 8 ROIs per CU instead of 4, with the
    // U region sized to the footprint bound): k_roi_small 22.1 -> 21.1 ms per 100 bench steps, bench 34.62k / 34.75k
    // -> 35.06k / 35.05k alternated (profiles/r05l; at 3 waves per SIMD: 35.01k).  FPM_SMALL_NT=256 keeps the
    // four-wave form (read when a search is recorded).
    const char* nte = getenv("FPM_SMALL_NT");
    // eight-wave workgroups (one per CU) for a lone search's layers: batches of at most two sources whose plan holds at
    // most 1024 ROIs (a lone Src7 search: 936, 99 live), so each ROI's chain of phases is the time -- not a search with
    // thousands of candidates (Src10 +-180, TargetNum 100: 14.8 K), whose ROIs need the residency of the smaller forms.
    // FPM_SMALL_NT=512 forces them, another value keeps them off.
    const int srcs = a.slot_cap / std::max(1, a.per_source * a.n3);
    const int kCUs = device_cus();
    if (nte ? atoi(nte) == 512 : (srcs <= 2 && a.slot_cap <= 4 * kCUs)) {
        const size_t lds8 = (size_t)small_layout(a.tw, a.th, 8).total;
        const int grid = capped(a.slot_cap < 8192 ? a.slot_cap : 8192, grid_cap_env(getenv("FPM_GRID_SMALL"), kCUs));
        if (a.prev_rec) {
            ensure_lds_attr((const void*)k_roi_small<0, 2, true, 512>, lds8);
            hipLaunchKernelGGL((k_roi_small<0, 2, true, 512>), dim3(grid), dim3(512), lds8, st, a);
        } else {
            ensure_lds_attr((const void*)k_roi_small<0, 2, false, 512>, lds8);
            hipLaunchKernelGGL((k_roi_small<0, 2, false, 512>), dim3(grid), dim3(512), lds8, st, a);
        }
        return;
    }
    const size_t lds2 = (size_t)small_layout(a.tw, a.th, 2).total, lds4 = (size_t)small_layout(a.tw, a.th).total;
    const int per_cu2 = (int)std::min<size_t>(8, kLdsPerCu / std::max<size_t>(lds2, 1));
    const int per_cu4 = (int)std::min<size_t>((size_t)(lds4 * 4 <= kLdsPerCu ? 4 : 3), kLdsPerCu / std::max<size_t>(lds4, 1));
    // (only where the layer has more ROIs than the four-wave form holds at once: with fewer, as in a lone search, each
    // ROI's chain of phases is what counts, and two waves take longer over it: 10.7 -> 13.2 us, r05_end2)
    // FPM_SMALL_NT=128 forces the two-wave form wherever it applies, 256 never uses it
    const int nt_env = nte ? atoi(nte) : 0;
    if (!a.prev_rec && a.tw + 6 <= 512 && per_cu2 > per_cu4 && nt_env != 256 &&
        (nt_env == 128 || a.slot_cap > per_cu4 * kCUs)) {
        // (5 waves per SIMD, 10 workgroups per CU -- layers 4-5 in one round at 64 sources -- spill 172 bytes: 21.1 ->
        // 23.3 ms per 100 bench steps, profiles/r05n)
        const int grid = capped(a.slot_cap < 16384 ? a.slot_cap : 16384,
                                grid_cap_env(getenv("FPM_GRID_SMALL"), per_cu2 * kCUs));
        ensure_lds_attr((const void*)k_roi_small<0, 4, false, 128>, lds2);
        hipLaunchKernelGGL((k_roi_small<0, 4, false, 128>), dim3(grid), dim3(128), lds2, st, a);
        return;
    }
    const size_t lds = lds4;
    // default cap: the kernel's residency (workgroups per CU: its waves per SIMD, or fewer where the LDS runs out)
    const int wpe = a.prev_rec ? 3 : (lds * 4 <= kLdsPerCu ? 4 : 3);
    const int per_cu = (int)std::min<size_t>((size_t)wpe, kLdsPerCu / std::max<size_t>(lds, 1));
    const int grid = capped(a.slot_cap < 8192 ? a.slot_cap : 8192,
                            grid_cap_env(getenv("FPM_GRID_SMALL"), std::max(per_cu, 1) * kCUs));
    // 4 waves per SIMD where 4 workgroups' LDS fit a CU (Src7 layers 5 and 4: 46.8 -> 42.4 and 54.7 -> 47.4 us per
    // 43-source launch despite a 48-byte spill; 5 waves spill 176 bytes and measured slower), else 3
    if (a.prev_rec) {   // small batches only (the engine's rule): occupancy matters less than spills (3 vs 28 VGPRs)
        ensure_lds_attr((const void*)k_roi_small<0, 3, true>, lds);
        hipLaunchKernelGGL((k_roi_small<0, 3, true>), dim3(grid), dim3(256), lds, st, a);
        return;
    }
    if (lds * 4 <= kLdsPerCu) {
        ensure_lds_attr((const void*)k_roi_small<0, 4>, lds);
        hipLaunchKernelGGL((k_roi_small<0, 4>), dim3(grid), dim3(256), lds, st, a);
        return;
    }
    ensure_lds_attr((const void*)k_roi_small<0>, lds);
    hipLaunchKernelGGL(k_roi_small<0>, dim3(grid), dim3(256), lds, st, a);
}

void launch_cand_step(const RoiArgs& a, int max_items, hipStream_t st) {
    if (max_items <= 0 || !a.step) return;
    if (a.nt_tab) {
        const int grid = max_items < 2048 ? max_items : 2048;
        hipLaunchKernelGGL(k_cand_step_tab, dim3(grid), dim3(192), 0, st, a);
        return;
    }
    int grid = (max_items + 255) / 256;
    if (grid > 1024) grid = 1024;
    hipLaunchKernelGGL(k_cand_step, dim3(grid), dim3(256), 0, st, a);
}

// ============================================================================================== K2-K5 on the matrix cores
// The top layer of a search whose canvases or angle count are large (BASELINE configs[3] at 1 deg: 361 angles of
// ~150 x 150 maps per source; configs[2] at +-180: 47 maps of ~1150 x 1150), TemplateMatcher.cpp:162-211.  One kernel
// per search does, for every (source, angle) job, the rotated canvas (cv::warpAffine, the same fixed-point tables and
// taps as k_warp), TM_CCORR and CCOEFF_Denominator (the exact integer correlation rounded once to f32, the f64
// normalisation of k_ncc_tile), without writing the canvas or the map: the only pixels the peak loop can ever take are
// those with a score >= the top-layer score (k_nms_greedy's argument), so the kernel lists those (index, score) per
// job and k_nms_greedy (plain or s_BlockMax key) takes the peaks from the list.  A job whose list overflows (or that the
// greedy form cannot take) gets its full map from a second launch of this kernel (mode 1) and the split peak kernels.
//
// Work unit: one job's strip of sw output columns, walked down in bands of 16 output rows.  Per band:
//   sampling  the band's new canvas rows (sw + tw - 1 columns) into an LDS ring of three i8 planes: I' = I - 128,
//             and the low (flipped) and high bytes of I'^2 (<= 16384), 8 pixels per lane, the taps from the wave's
//             staged source footprint;
//   MFMA      per 16 x 16 output tile and wave: D += A B on v_mfma_i32_16x16x64_i8 with A = canvas rows (the 16 output
//             rows; K = 64 = two template rows x 32 columns, or one row x 64 columns for templates 18-49 wide) and B =
//             the template row Toeplitz-banded over the 16 output columns (B[c][n] = T'[r][c - n], zero outside
//             0 <= c - n < tw), so sum_slots D = sum T'I' exactly; three more MFMAs with B = the band of ones give the
//             window sums of I' and of the two byte planes of I'^2.  Exact: sum T I = sum T'I' + 128 (sum I + sum T) -
//             16384 area, sum I^2 = 256 (sum hi + sum I') + sum lo' + 16512 area;
//   epilogue  a conservative f32 bound (nf^2 >= thr^2 norm^2 area df, nf = area ccorr - sum I sum T, df = area sum I^2 -
//             (sum I)^2, with an absolute slack E on the two f32 terms) and, where it passes, the exact f64 score.
// Exactness of the bound (prefilter): for area <= 258 every integer term is < 2^24 (exact in f32); the two products
// carry at most 512 of rounding each (E = 1024), and thrK includes a 1e-5 relative margin over the f64 evaluation's
// and the f32 score rounding's relative errors (<= 1e-6), so no output with (double)score >= thr is ever rejected.
constexpr int TM_BH = 16;            // output rows per band (one MFMA M block)
// ring row pitch (bytes): the A fragments of the two-row layout read columns <= sw + 15 and the samples reach
// sw + tw + 6 (<= 215); the one-row layout's reach sw + 63.  Both are +-2 x 16 B mod 256 B (56 / 72 words), so the 16
// lanes of every ds_read_b128 lane group (rows ln at two 16-byte column blocks) and of every ds_write_b64 group (4
// rows x 4 words) hit disjoint banks
constexpr int TM_CP2 = 224, TM_CP1 = 288;
constexpr int TM_FTP = 44;           // sampling footprint buffer: row pitch (bytes; an odd word count spreads the
constexpr int TM_FTB = 44 * 40;      // taps over the banks) and size per wave (a 16 x 32 tile of a rotation covers at
                                     // most 37 x 37 source pixels + taps)
// TOPMMA_ABL (measurement builds only, scripts/gpu_abl.sh; the product is 0): 1 = no sampling, 3 = no MFMA loop, 4 = no
// epilogue, 5 = no staging loads, 6 = no gather (1, 5 and 6 leave garbage in the ring: their exact paths run far more)
#ifndef TOPMMA_ABL
#define TOPMMA_ABL 0
#endif
// wave priorities (s_setprio) of the band's phases: 4 = the tiles (MFMA loop and epilogue) at priority 1, the sampling
// at 0 (the product: a wave's matrix instructions are not held behind the other waves' sampling VALU on its SIMD;
// configs[3] 735.6 -> 677-678 us per launch, profiles/r06_prio/), 1 = the MFMA loop only (678-689), 2 = the
// sampling at 1 instead (721.7), 3 = MFMA loop 2 / sampling 1 (681), 0 = none (735.6; measurement builds)
#ifndef TOPMMA_PRIO
#define TOPMMA_PRIO 4
#endif

bool top_mma_fits(int tw, int th) { return tw >= 1 && th >= 1 && ((tw <= 17 && th <= 32) || (tw <= 49 && th <= 16)); }

// the loop bounds every lane runs unrolled (NQM MFMA slots; a slot beyond the template is masked, not branched
// around, so all of the loop's LDS reads are issued before the first use) and the ring's rows (RR, a power of two
// >= 16 + th - 1): <8, 32> for templates up to 17 x 16 (BASELINE configs[2] and [3]), <16, 64> for every other shape
static bool top_mma_small(const TopMmaArgs& a) { return a.R == 2 && a.th <= 16; }

void top_mma_layout(TopMmaArgs& a, int sw, int max_rows) {
    a.sw = sw;
    a.R = a.tw <= 17 ? 2 : 1;
    a.nq = a.R == 2 ? (a.th + 1) / 2 : a.th;
    a.cp = top_mma_small(a) ? TM_CP2 : TM_CP1;
    a.rr = top_mma_small(a) ? 32 : 64;
    a.ct = (sw + a.tw - 1 + 8 + 3) & ~3;             // canvas columns (+ the 8-pixel reads past the last one)
    a.rt = max_rows + a.th;                          // canvas rows of the tallest unit
    a.o_colt = 3 * a.rr * a.cp;                      // the ring's three planes
    a.o_rowt = a.o_colt + 8 * a.ct;
    a.o_bf = (a.o_rowt + 8 * a.rt + 15) & ~15;
    a.nqm = top_mma_small(a) ? 8 : 16;               // B slots in LDS (zero beyond nq)
    a.o_ft = a.o_bf + 1024 * a.nqm;                  // the 4 waves' sampling footprint buffers
}
size_t top_mma_lds(const TopMmaArgs& a) { return (size_t)a.o_ft + 4 * TM_FTB; }

typedef short fpm_s2 __attribute__((ext_vector_type(2)));

// 24-bit multiply-adds as single full-rate instructions (a plain int multiply whose operands the compiler cannot
// bound becomes the quarter-rate v_mul_lo_u32, and it drops __mul24's sign extension when it proves it redundant)
__device__ __forceinline__ int tm_mad_i24(int a, int b, int c) {
    int r;
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ int tm_mad_u24(int a, int b, int c) {
    int r;
    asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "i"(b), "v"(c));
    return r;
}

// the three ring words of 4 canvas pixels from two pairs of 16-bit pixel values (p0 = pixels 0, 1; p1 = 2, 3):
// I' (flipped bytes), the low bytes of I'^2 (flipped) and the high bytes (packed 16-bit squares, byte permutes)
__device__ __forceinline__ void tm_planes(uint32_t p0, uint32_t p1, uint32_t& wi, uint32_t& wl, uint32_t& wh) {
    const fpm_s2 k128 = {128, 128};
    const fpm_s2 d0 = __builtin_bit_cast(fpm_s2, p0) - k128, d1 = __builtin_bit_cast(fpm_s2, p1) - k128;
    const uint32_t q0 = __builtin_bit_cast(uint32_t, d0 * d0), q1 = __builtin_bit_cast(uint32_t, d1 * d1);
    wi = __builtin_amdgcn_perm(p1, p0, 0x06040200u) ^ kRoiFlip;
    wl = __builtin_amdgcn_perm(q1, q0, 0x06040200u) ^ kRoiFlip;
    wh = __builtin_amdgcn_perm(q1, q0, 0x07050301u);
}

// TH > 0: the template height as a compile-time constant (two-row slots, NQM = (TH + 1) / 2, every slot exact: no
// masks); TH == 0: any height up to the form's bounds, rows past th masked
// MODE 0: the candidate lists (kernel k_top_mma); MODE 1: the full maps of the jobs the lists left (k_top_map).
template <int NQM, int RR, int TM_CP, int TH, int MODE>
__device__ __forceinline__ void top_mma_body(const TopMmaArgs& a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t tm_lds[];
    constexpr int PS = RR * TM_CP;   // plane stride of the ring: I', lo(I'^2) ^ 0x80, hi(I'^2)
    uint8_t* const ring = tm_lds;
    int32_t* const cad = (int32_t*)(tm_lds + a.o_colt);   // adelta [ct], bdelta [ct] of the unit's canvas columns
    int32_t* const rxy = (int32_t*)(tm_lds + a.o_rowt);   // X0 [rt], Y0 [rt] of its canvas rows
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int ln = lane & 15, lg = lane >> 4;
    const int tw = a.tw, th = TH > 0 ? TH : a.th, mask = RR - 1;
    // the B fragments (correlation) staged once into LDS, zero past slot nq; the band of ones (window sum of I') in
    // registers: byte i of lane (n, g) is k = 16 g + i
    fpm_v4i* const bl = (fpm_v4i*)(tm_lds + a.o_bf);
    uint8_t* const ftb = tm_lds + a.o_ft;
    for (int i = tid; i < NQM * 64; i += 256)
        bl[i] = i < a.nq * 64 ? *(const fpm_v4i*)(a.bfrag + (size_t)i * 16) : fpm_v4i{0, 0, 0, 0};
    fpm_v4i ones;
    {
        const int c0 = a.R == 2 ? 16 * (lg & 1) : 16 * lg;
        uint32_t w[4] = {0, 0, 0, 0};
        for (int i = 0; i < 16; ++i) {
            const int c = c0 + i - ln;
            if (c >= 0 && c < tw) w[i >> 2] |= 1u << (8 * (i & 3));
        }
        ones = fpm_v4i{(int)w[0], (int)w[1], (int)w[2], (int)w[3]};
    }
    const fpm_v4i zero4 = {0, 0, 0, 0};
    const uint32_t area = (uint32_t)a.area;
    const float areaf = (float)a.area, tsumf = (float)a.tsum;
    const int co = a.R == 2 ? 16 * (lg & 1) : 16 * lg;   // the lane's A / B column offset in a slot
    // XCD-aware order (mode 0, one unit per workgroup): consecutive workgroups go to the 8 XCDs in turn, so XCD x
    // takes the x-th contiguous eighth of the unit list (the units of a few sources: their top levels stay in its L2)
    int u0 = blockIdx.x;
    if (MODE == 0 && (int)gridDim.x == a.nunits) {
        const int x = blockIdx.x & 7, q = a.nunits >> 3, r = a.nunits & 7;
        u0 = x * q + min(x, r) + (blockIdx.x >> 3);
    }
    for (int u = u0; u < a.nunits; u += gridDim.x) {
        const TopUnit U = a.units[u];
        if (MODE == 1 && a.cand_cnt[U.job] < 0) continue;   // (uniform) taken from its list: no map needed
        const WarpJob& W = a.wjobs[U.job];
        const NccJob& NJ = a.njobs[U.job];
        const int mw = NJ.ow;
        const int swu = min(a.sw, mw - U.x0);                 // output columns of this strip
        const int ncols = swu + tw - 1;                       // canvas columns it reads (<= dw - x0)
        const int nrows = min(U.y1 + th - 1, W.dh) - U.y0;    // canvas rows of the unit
        const uint8_t* src = W.src;
        const int sw = W.sw, sh = W.sh, sp = W.sp, border = W.border;
        __syncthreads();   // the previous unit is done with the LDS
        for (int i = tid; i < ncols; i += 256) {
            const int x = U.x0 + i;
            cad[i] = rint_i(W.M[0] * x * kAbScale);
            cad[a.ct + i] = rint_i(W.M[3] * x * kAbScale);
        }
        for (int i = tid; i < nrows; i += 256) {
            const int y = U.y0 + i;
            rxy[i] = rint_i((W.M[1] * y + W.M[2]) * kAbScale) + kRoundDelta;
            rxy[a.rt + i] = rint_i((W.M[4] * y + W.M[5]) * kAbScale) + kRoundDelta;
        }
        const int nbu = (swu + 15) >> 4;
        for (int yb = U.y0; yb < U.y1; yb += TM_BH) {
            const int rs = yb == U.y0 ? yb : yb + th - 1;
            const int re = min(yb + TM_BH + th - 1, U.y0 + nrows);
            __syncthreads();   // tables ready / the previous band's tiles are done with the ring rows replaced now
            if (TOPMMA_PRIO == 2 || TOPMMA_PRIO == 3) __builtin_amdgcn_s_setprio(1);
            if (TOPMMA_PRIO == 4) __builtin_amdgcn_s_setprio(0);
            // ---- the band's new canvas rows (cv::warpAffine with k_warp's integers), flipped to i8.  One wave per
            // sampling tile of 16 rows x 32 columns: the tile's source footprint (the box of its clamped tap coordinates:
            // the fixed-point coordinates are monotone in x and y, so the corners bound it; coordinates clamped into
            // [-2, w] x [-2, h], where every tap outside the level reads the border value) is staged from the level into
            // the wave's LDS buffer, the border value filling what lies outside, and the 4 taps of each pixel are read
            // from there (a clamped tap outside the image reads the border value exactly as warp_tap's per-tap rule
            // does, and four border values interpolate to the border value)
            {
                const int nrw = re - rs, ntc = (ncols + 31) >> 5, ntr = (nrw + 15) >> 4;
                uint8_t* const ft = ftb + wv * TM_FTB;
                for (int t = wv; t < (TOPMMA_ABL == 1 ? 0 : ntr * ntc); t += 4) {
                    const int tr = t / ntc, tc = t - tr * ntc;
                    const int ty0 = rs + 16 * tr, ty1 = min(ty0 + 16, re), tx0 = 32 * tc, tx1 = min(tx0 + 32, ncols);
                    const int r0 = ty0 - U.y0, r1 = ty1 - 1 - U.y0;
                    const int Xa = rxy[r0] + cad[tx0], Xb = rxy[r0] + cad[tx1 - 1];
                    const int Xc = rxy[r1] + cad[tx0], Xd = rxy[r1] + cad[tx1 - 1];
                    const int Ya = rxy[a.rt + r0] + cad[a.ct + tx0], Yb = rxy[a.rt + r0] + cad[a.ct + tx1 - 1];
                    const int Yc = rxy[a.rt + r1] + cad[a.ct + tx0], Yd = rxy[a.rt + r1] + cad[a.ct + tx1 - 1];
                    // the tile's raw tap box (wave-uniform): wholly outside the level (every tap reads the border
                    // value), wholly inside (no clamping, no border), or across the edge (clamped into the frame)
                    const int rx0 = __builtin_amdgcn_readfirstlane(min(min(Xa, Xb), min(Xc, Xd)) >> kAbBits);
                    const int rx1 = __builtin_amdgcn_readfirstlane(max(max(Xa, Xb), max(Xc, Xd)) >> kAbBits);
                    const int ry0 = __builtin_amdgcn_readfirstlane(min(min(Ya, Yb), min(Yc, Yd)) >> kAbBits);
                    const int ry1 = __builtin_amdgcn_readfirstlane(max(max(Ya, Yb), max(Yc, Yd)) >> kAbBits);
                    const int y = ty0 + (lane >> 2), xq = tx0 + 8 * (lane & 3);   // this lane's 8 pixels
                    const bool mine = y < ty1 && xq < tx1;
                    if (rx1 + 1 < 0 || rx0 >= sw || ry1 + 1 < 0 || ry0 >= sh) {
                        if (mine) {
                            const uint32_t bp = (uint32_t)border * 0x10001u;
                            uint32_t wi, wl, wh;
                            tm_planes(bp, bp, wi, wl, wh);
                            uint8_t* const rp = ring + (y & mask) * TM_CP + xq;
                            *(uint2*)rp = make_uint2(wi, wi);
                            *(uint2*)(rp + PS) = make_uint2(wl, wl);
                            *(uint2*)(rp + 2 * PS) = make_uint2(wh, wh);
                        }
                        continue;   // (uniform; the buffer was not touched)
                    }
                    const bool inner = rx0 >= 0 && rx1 + 1 < sw && ry0 >= 0 && ry1 + 1 < sh;
                    const int bx0 = min(max(rx0, -2), sw), bx1 = min(max(rx1, -2), sw) + 1;
                    const int by0 = min(max(ry0, -2), sh), by1 = min(max(ry1, -2), sh) + 1;
                    // staged columns: the aligned words of source columns [bx0 & ~3, bx1] (the box's first column sits
                    // at byte bx0 & 3 of the buffer row)
                    const int cx0 = bx0 & ~3, nwd = ((bx1 - cx0) >> 2) + 1, nr = by1 - by0 + 1;
                    // (a pure rotation of a 16 x 32 tile covers at most 35 x 35 source pixels + the tap neighbours and the
                    // word alignment: nr <= 37 <= TM_FTB / TM_FTP, nwd <= 10 <= TM_FTP / 4 -- top_mma_fits' matrices)
                    {
                        // lane -> word column lane & 15 (< nwd) of rows (lane >> 4) + 4 i: every load of the box in flight
                        // at once (<= 10 per lane), no division; an inner box's words are all inside the level's rows
                        // (whose pitch holds >= 4 bytes past the width)
                        const uint32_t bw4 = 0x01010101u * (uint32_t)border;
                        const int wc = lane & 15, c = cx0 + 4 * wc;
                        const bool col_in = wc < nwd, full = inner || (c >= 0 && c + 4 <= sw);
                        uint32_t wds[TM_FTB / TM_FTP / 4];
#pragma unroll
                        for (int u = 0; u < TM_FTB / TM_FTP / 4; ++u) {
                            const int r = (lane >> 4) + 4 * u, yy = by0 + r;
                            const bool in = col_in && r < nr && full && (inner || (yy >= 0 && yy < sh));
                            wds[u] = (in && TOPMMA_ABL != 5) ? *(const uint32_t*)(src + (size_t)yy * sp + c) : bw4;
                        }
#pragma unroll
                        for (int u = 0; u < TM_FTB / TM_FTP / 4; ++u) {
                            const int r = (lane >> 4) + 4 * u, yy = by0 + r;
                            if (col_in && r < nr) {
                                uint32_t w = wds[u];
                                if (!full && yy >= 0 && yy < sh) {   // a word the level's edge cuts (boundary tiles)
#pragma unroll
                                    for (int b = 0; b < 4; ++b) {
                                        const int x = c + b;
                                        const uint32_t v = (x >= 0 && x < sw) ? src[(size_t)yy * sp + x] : (uint32_t)border;
                                        w = (w & ~(0xffu << (8 * b))) | (v << (8 * b));
                                    }
                                }
                                *(uint32_t*)(ft + r * TM_FTP + 4 * wc) = w;
                            }
                        }
                        wave_sync();
                    }
                    if (mine && TOPMMA_ABL != 6) {
                        const int ry = y - U.y0;
                        // the footprint origin folded into the row's fixed-point start (exact: a whole-pixel shift)
                        const int X0 = rxy[ry] - (cx0 << kAbBits), Y0 = rxy[a.rt + ry] - (by0 << kAbBits);
                        const int4 a0 = *(const int4*)(cad + xq), a1 = *(const int4*)(cad + xq + 4);
                        const int4 b0 = *(const int4*)(cad + a.ct + xq), b1 = *(const int4*)(cad + a.ct + xq + 4);
                        const int adv[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
                        const int bdv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
                        const int xlo = -2 - cx0, xhi = sw - cx0, ylo = -2 - by0, yhi = sh - by0;
                        uint32_t pv[4] = {0, 0, 0, 0};
                        // (inner is wave-uniform: two copies of the loop, the inner one without the clamps)
                        auto gather = [&](auto inner_c) {
#pragma unroll
                            for (int b = 0; b < 8; ++b) {
                                const int X = X0 + adv[b], Y = Y0 + bdv[b];
                                const int fx = (X >> (kAbBits - kInterBits)) & (kInterTab - 1);
                                const int fy = (Y >> (kAbBits - kInterBits)) & (kInterTab - 1);
                                int sx = X >> kAbBits, sy = Y >> kAbBits;
                                if (!decltype(inner_c)::value) {
                                    sx = min(max(sx, xlo), xhi);
                                    sy = min(max(sy, ylo), yhi);
                                }
                                const uint8_t* p = ft + tm_mad_u24(sy, TM_FTP, sx);   // (0 <= sy, sx < TM_FTP)
                                const int v0 = p[0], v1 = p[1], v2 = p[TM_FTP], v3 = p[TM_FTP + 1];
                                const int h0 = tm_mad_i24(v1 - v0, fx, v0 << kInterBits);
                                const int h1 = tm_mad_i24(v3 - v2, fx, v2 << kInterBits);
                                const int v = tm_mad_i24(h1 - h0, fy, (h0 << kInterBits) + 512) >> 10;
                                pv[b >> 1] |= (uint32_t)v << (16 * (b & 1));
                            }
                        };
                        if (inner) gather(std::true_type{});
                        else gather(std::false_type{});
                        uint32_t wi0, wl0, wh0, wi1, wl1, wh1;
                        tm_planes(pv[0], pv[1], wi0, wl0, wh0);
                        tm_planes(pv[2], pv[3], wi1, wl1, wh1);
                        uint8_t* const rp = ring + (y & mask) * TM_CP + xq;
                        *(uint2*)rp = make_uint2(wi0, wi1);
                        *(uint2*)(rp + PS) = make_uint2(wl0, wl1);
                        *(uint2*)(rp + 2 * PS) = make_uint2(wh0, wh1);
                    }
                    wave_sync();   // the buffer is reused by the wave's next tile
                }
            }
            if (TOPMMA_PRIO == 2 || TOPMMA_PRIO == 3) __builtin_amdgcn_s_setprio(0);
            __syncthreads();
            // ---- the band's 16 x 16 output tiles, one wave each: NQM slots unrolled (A and B of every slot requested
            // before the first MFMA; slots >= nq read zero B)
            for (int nb = wv; nb < nbu; nb += 4) {
                fpm_v4i acc = zero4, acc1 = zero4, accl = zero4, acch = zero4;
                if (TOPMMA_PRIO == 1 || TOPMMA_PRIO == 4) __builtin_amdgcn_s_setprio(1);
                if (TOPMMA_PRIO == 3) __builtin_amdgcn_s_setprio(2);
                if (TOPMMA_ABL != 3) {
                    // slot q's fragments (three planes) are requested two slots ahead of its MFMAs
                    const uint8_t* abase = ring + 16 * nb + co;
                    const int rstep = a.R == 2 ? 2 : 1, r0 = yb + ln + (a.R == 2 ? (lg >> 1) : 0);
                    fpm_v4i av[3][3], bv[3];
#pragma unroll
                    for (int q = 0; q < 2; ++q) {
                        const uint8_t* ap = abase + ((r0 + q * rstep) & mask) * TM_CP;
#pragma unroll
                        for (int pl = 0; pl < 3; ++pl) av[q][pl] = *(const fpm_v4i*)(ap + pl * PS);
                        bv[q] = bl[q * 64 + lane];
                    }
#pragma unroll
                    for (int q = 0; q < NQM; ++q) {
                        if (q + 2 < NQM) {
                            const uint8_t* ap = abase + ((r0 + (q + 2) * rstep) & mask) * TM_CP;
#pragma unroll
                            for (int pl = 0; pl < 3; ++pl) av[(q + 2) % 3][pl] = *(const fpm_v4i*)(ap + pl * PS);
                            bv[(q + 2) % 3] = bl[(q + 2) * 64 + lane];
                        }
                        fpm_v4i* const A = av[q % 3];
                        // a template row past th (the odd row of the last two-row slot, or a slot past nq): its canvas
                        // row enters no sum (the correlation's B is zero there, the window sums' A are zeroed)
                        if (TH == 0 && q >= a.nq - 1) {   // (uniform) only the last slot can hold such a row
                            const int ro = a.R == 2 ? 2 * q + (lg >> 1) : q;
                            if (ro >= th) A[0] = A[1] = A[2] = zero4;
                        }
                        acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[0], bv[q % 3], acc, 0, 0, 0);
                        acc1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[0], ones, acc1, 0, 0, 0);
                        accl = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[1], ones, accl, 0, 0, 0);
                        acch = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[2], ones, acch, 0, 0, 0);
                    }
                }
                if (TOPMMA_PRIO == 1 || TOPMMA_PRIO == 3) __builtin_amdgcn_s_setprio(0);
                if (TOPMMA_ABL == 4) {
                    if (acc[0] == 0x12345 && acc1[1] == 0x777) a.cand_cnt[0] = acc[2] + acc1[3] + accl[0] + acch[1];
                    continue;
                }
                // D: column ln = output column 16 nb + ln, rows 4 lg + i = output rows yb + 4 lg + i
                const int xo = 16 * nb + ln, yo0 = yb + 4 * lg;
                // the cheap part for the lane's 4 outputs: exact integer sums and the prefilter (pairs of outputs in
                // packed f32 lanes)
                uint32_t ccv[4], wsv[4], wq[4], dfi[4];
                const uint32_t ccofs = 128u * a.tsum - 16384u * area, qofs = 16512u * area;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    wsv[i] = (uint32_t)acc1[i] + 128u * area;
                    ccv[i] = (uint32_t)acc[i] + (wsv[i] << 7) + ccofs;
                    wq[i] = (((uint32_t)acch[i] + (uint32_t)acc1[i]) << 8) + (uint32_t)accl[i] + qofs;
                    // df = area sum I^2 - (sum I)^2 exactly (mod 2^32: its value is < 2^32 for area <= 257; 24-bit
                    // factors); 0 is a flat window, whose score is 0 (CCOEFF's t = 0 branch)
                    dfi[i] = __umul24(area, wq[i]) - __umul24(wsv[i], wsv[i]);
                }
                uint32_t pm = 0;
                const bool colok = xo < swu;
                if (MODE == 0 && a.prefilter) {
                    typedef float f2_t __attribute__((ext_vector_type(2)));
                    const f2_t ar2 = {areaf, areaf}, ts2 = {tsumf, tsumf}, e2 = {a.E, a.E}, k2 = {a.thrK, a.thrK};
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int i0 = 2 * h, i1 = 2 * h + 1;
                        const f2_t ws = {(float)wsv[i0], (float)wsv[i1]}, cc = {(float)ccv[i0], (float)ccv[i1]};
                        const f2_t df = {(float)dfi[i0], (float)dfi[i1]};
                        const f2_t nfp = __builtin_elementwise_fma(ar2, cc, -(ws * ts2)) + e2;
                        const f2_t lhs = nfp * nfp, rhs = k2 * df;
                        if (colok && yo0 + i0 < U.y1 && dfi[i0] != 0u && nfp.x > 0.f && lhs.x >= rhs.x) pm |= 1u << i0;
                        if (colok && yo0 + i1 < U.y1 && dfi[i1] != 0u && nfp.y > 0.f && lhs.y >= rhs.y) pm |= 1u << i1;
                    }
                } else {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if (colok && yo0 + i < U.y1) pm |= 1u << i;
                }
                // the exact f64 score where the bound passed (rare in mode 0; every valid output in mode 1), one
                // instance of ccoeff in a data-dependent loop (the register budget of the MFMA loop stays small)
                float sv0 = 0.f, sv1 = 0.f, sv2 = 0.f, sv3 = 0.f;
                uint32_t tk = 0;
                while (pm) {
                    const int i = __builtin_ctz(pm);
                    pm &= pm - 1;
                    const uint32_t cc = i == 0 ? ccv[0] : i == 1 ? ccv[1] : i == 2 ? ccv[2] : ccv[3];
                    const uint32_t ws = i == 0 ? wsv[0] : i == 1 ? wsv[1] : i == 2 ? wsv[2] : wsv[3];
                    const uint32_t qs = i == 0 ? wq[0] : i == 1 ? wq[1] : i == 2 ? wq[2] : wq[3];
                    const double num = (double)(float)(double)cc;   // TM_CCORR's f32 result
                    const float sc = ccoeff(num, (double)ws, (double)qs, a.mean, a.norm, a.inv_area);
                    if (MODE == 1) {
                        NJ.out[(size_t)(yo0 + i) * mw + U.x0 + xo] = sc;
                    } else if ((double)sc >= a.thr) {
                        tk |= 1u << i;
                        if (i == 0) sv0 = sc; else if (i == 1) sv1 = sc; else if (i == 2) sv2 = sc; else sv3 = sc;
                    }
                }
                if (MODE == 0 && __ballot(tk != 0)) {   // (wave-uniform; rare)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const bool take = (tk >> i) & 1u;
                        const uint64_t mk = __ballot(take);
                        if (mk) {   // one atomic per wave and output row
                            int base = 0;
                            if (lane == 0) base = atomicAdd(&a.cand_cnt[U.job], __popcll(mk));
                            base = __shfl(base, 0);
                            if (take) {
                                const int pos = base + __popcll(mk & ((1ull << lane) - 1));
                                if (pos < a.cand_cap) {
                                    a.cand[(size_t)U.job * a.cand_cap + pos] = (yo0 + i) * mw + U.x0 + xo;
                                    a.cand_val[(size_t)U.job * a.cand_cap + pos] =
                                        i == 0 ? sv0 : i == 1 ? sv1 : i == 2 ? sv2 : sv3;
                                }
                            }
                        }
                    }
                }
            }
        }
    }
}

// The exact-height two-row forms (<= 40 KB of LDS at the BASELINE shapes) are held to 128 registers: 4 workgroups
// per CU.
template <int NQM, int RR, int TM_CP, int TH = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RR == 32 && TH > 0 ? 4 : 1)))
void k_top_mma(TopMmaArgs a) {
    top_mma_body<NQM, RR, TM_CP, TH, 0>(a);
}
template <int NQM, int RR, int TM_CP, int TH = 0>
__global__ __launch_bounds__(256) void k_top_map(TopMmaArgs a) {
    top_mma_body<NQM, RR, TM_CP, TH, 1>(a);
}

template <int NQM, int RR, int CP, int TH = 0>
static void launch_top_form(const TopMmaArgs& a, int grid, size_t lds, hipStream_t st) {
    if (a.mode == 0) {
        ensure_lds_attr((const void*)k_top_mma<NQM, RR, CP, TH>, lds);
        hipLaunchKernelGGL((k_top_mma<NQM, RR, CP, TH>), dim3(grid), dim3(256), lds, st, a);
    } else {
        ensure_lds_attr((const void*)k_top_map<NQM, RR, CP, TH>, lds);
        hipLaunchKernelGGL((k_top_map<NQM, RR, CP, TH>), dim3(grid), dim3(256), lds, st, a);
    }
}

void launch_top_mma(const TopMmaArgs& a, hipStream_t st) {
    if (a.nunits <= 0) return;
    const size_t lds = top_mma_lds(a);
    // mode 1 touches only the jobs left by the greedy form (usually none): a small grid walks the unit list
    const int grid = a.mode == 1 ? std::min(a.nunits, 4 * device_cus()) : a.nunits;
    // exact-height forms for the two-row layout's common top templates (16 rows: a square template at MinReduceArea
    // 256, BASELINE configs[3]; 14: configs[2]), the masked small form for other heights up to 16
    if (top_mma_small(a) && a.th == 16) launch_top_form<8, 32, TM_CP2, 16>(a, grid, lds, st);
    else if (top_mma_small(a) && a.th == 14) launch_top_form<7, 32, TM_CP2, 14>(a, grid, lds, st);
    else if (top_mma_small(a)) launch_top_form<8, 32, TM_CP2>(a, grid, lds, st);
    else launch_top_form<16, 64, TM_CP1>(a, grid, lds, st);
}

void launch_top_greedy(const NmsArgs& a0, int njobs, int max_cells, hipStream_t st, const CandInitArgs* ci) {
    if (njobs <= 0) return;
    NmsArgs a = a0;
    a.lds_blocks = max_cells;
    CandInitArgs cz{};
    const bool fuse = ci && !a.by_block && a.cap <= kNmsInitCap;
    const int mode = !fuse ? 0 : (ci->refine == 0 ? 1 : (ci->refine == 2 ? 3 : 2));
    // sort capacity: the lists' capacity (a power of 2, at most kGreedyMax), so short lists need little LDS and many
    // workgroups fit a CU (most of them end after reading their count)
    int gc = 64;
    while (gc < a.cand_cap && gc < kGreedyMax) gc <<= 1;
    a.greedy_cap = gc;
    const size_t lds = nms_greedy_lds(max_cells, gc);
    ensure_lds_attr((const void*)k_nms_greedy, lds);
    hipLaunchKernelGGL(k_nms_greedy, dim3(njobs), dim3(256), lds, st, a, fuse ? *ci : cz, mode);
}

// ============================================================================================== pack
__global__ __launch_bounds__(256) void k_pack(PackArgs a) {
    const int tid = blockIdx.x * 256 + threadIdx.x, nthr = gridDim.x * 256;
    int32_t* hc = (int32_t*)(a.host + a.o_counts);
    for (int i = tid; i < a.J; i += nthr) hc[i] = a.counts[i];
    // only the slots below each job's peak count (the host reads no others): at Src7's top layer ~1 slot in 10, the
    // rest of the 16-byte slots need not cross PCIe
    int4* hp = (int4*)(a.host + a.o_peaks);
    const int cap = a.cap;   // peak slots per job (P.cap; the host checks C == J * cap before the launch)
    for (int i = tid; i < a.C; i += nthr) {
        const int job = i / cap;
        if (i - job * cap < a.counts[job]) hp[i] = *(const int4*)(a.peaks + i);
    }
    int32_t* hl = (int32_t*)(a.host + a.o_live);
    for (int i = tid; i < a.nlive; i += nthr) hl[i] = a.livecnt[i];
    if (a.live0) {
        const int n0 = *a.live0_count;
        int32_t* hi = (int32_t*)(a.host + a.o_live0);
        CandState* hs = (CandState*)(a.host + a.o_state0);
        for (int li = tid; li < n0; li += nthr) {
            const int id = a.live0[li];
            hi[li] = id;
            hs[li] = a.state[id];
        }
        uint32_t* hr = (uint32_t*)(a.host + a.o_rec0);
        constexpr int RW = sizeof(RoiRecord) / 4;
        for (int i = tid; i < n0 * a.n3 * RW; i += nthr) {
            const int q = i / RW, w = i - q * RW, li = q / a.n3, j = q - li * a.n3;
            hr[i] = ((const uint32_t*)(a.rec + (size_t)a.live0[li] * a.n3 + j))[w];
        }
    }
    // The one visibility rule for the kernels that write mapped pinned host memory (k_pack, k_overlap_pairs): plain
    // stores, no fence in the kernel; the host reads the buffer only after hipStreamSynchronize on the kernel's stream,
    // which (HIP's synchronisation semantics for host-pinned memory) makes the completed kernel's stores visible to it.
    // (A system-scope fence per workgroup writes its XCD's L2 back each time: +80 us on the Src10 +-180 tail when
    // k_overlap_pairs had one, profiles/r05b.)  tests/test_gpu_overlap.py::test_device_filter_twice_in_one_context
    // and every search's results (read through this buffer) check it.
}

void launch_pack(const PackArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(k_pack, dim3(16), dim3(256), 0, st, a);
}

// ---- filterWithRotatedRect pair decisions (launch_overlap_pairs).  One wave per rectangle i: the lanes sweep j > i in
// chunks of 64 with the box prefilter and compact the overlapping partners into the wave's LDS list (ballot + prefix,
// ascending j), then run the exact pair test on them 64 at a time; one atomic per wave reserves the output range.
__global__ __launch_bounds__(256) void k_overlap_pairs(const OvRect* __restrict__ r, const float4* __restrict__ box,
                                                       int n, double max_overlap, int32_t* lists, int list_cap,
                                                       int32_t* offcnt, int32_t* meta) {
    __shared__ int32_t cand[4][kOverlapMaxCand];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (int i = blockIdx.x * 4 + wv; i < n; i += gridDim.x * 4) {
        const OvRect ri = r[i];
        const float4 bi = box[i];
        int nc = 0;   // wave-uniform
        bool over = false;
        // four 64-rectangle chunks' boxes in flight per round (the sweep of the first rectangles is the kernel's
        // critical path: ~n / 64 dependent load round trips otherwise), then the chunks in ascending order
        for (int j0 = i + 1; j0 < n && !over; j0 += 256) {
            float4 bj[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int j = j0 + 64 * u + lane;
                bj[u] = j < n ? box[j] : make_float4(INFINITY, -INFINITY, INFINITY, -INFINITY);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int j = j0 + 64 * u + lane;
                const bool ov = j < n && !(bj[u].x > bi.z || bj[u].z < bi.x || bj[u].y > bi.w || bj[u].w < bi.y);
                const uint64_t m = __ballot(ov);
                const int c = __popcll(m);
                if (nc + c > kOverlapMaxCand) { over = true; break; }
                if (ov) cand[wv][nc + __popcll(m & below)] = j;
                nc += c;
            }
        }
        if (over) {
            if (lane == 0) atomicOr(&meta[1], 1);
            if (lane == 0) { offcnt[2 * i] = 0; offcnt[2 * i + 1] = 0; }
            continue;
        }
        __builtin_amdgcn_wave_barrier();
        // exact tests: lane k of round t decides partner cand[64 t + k]; verdicts replace the entries (j: drop, ~j:
        // undecided, INT_MIN: no drop)
        for (int k0 = 0; k0 < nc; k0 += 64) {
            const int k = k0 + lane;
            if (k < nc) {
                const int j = cand[wv][k];
                const OvRect rj = r[j];
                F2 pts[24];
                int np = 0;
                const int kind = rrect_isect_pts<false>(ri.w, ri.h, rj.w, rj.h, ri.c, rj.c, pts, &np);
                int verdict = INT_MIN;
                if (kind < 0) {   // more than 8 intersection points after the near-duplicate pass: the host decides
                    verdict = ~j;
                } else if (kind == 2) {
                    verdict = j;
                } else if (kind == 1 && np >= 3) {
                    if (!sort_pts_fast(pts, np)) verdict = ~j;
                    else if (contour_area_pts(pts, np) / (ri.w * ri.h) > max_overlap) verdict = j;
                }
                cand[wv][k] = verdict;
            }
        }
        __builtin_amdgcn_wave_barrier();
        // compact the drops / undecided pairs (ascending j) into the output
        int nd = 0;
        for (int k0 = 0; k0 < nc; k0 += 64) {
            const int k = k0 + lane;
            const bool keep = k < nc && cand[wv][k] != INT_MIN;
            nd += __popcll(__ballot(keep));
        }
        int base = 0;
        if (lane == 0 && nd > 0) base = atomicAdd(&meta[0], nd);
        base = __shfl(base, 0, 64);
        if (base + nd > list_cap) {
            if (lane == 0) { atomicOr(&meta[1], 2); offcnt[2 * i] = 0; offcnt[2 * i + 1] = 0; }
            continue;
        }
        int w = 0;
        for (int k0 = 0; k0 < nc; k0 += 64) {
            const int k = k0 + lane;
            const bool keep = k < nc && cand[wv][k] != INT_MIN;
            const uint64_t m = __ballot(keep);
            if (keep) lists[base + w + __popcll(m & below)] = cand[wv][k];
            w += __popcll(m);
        }
        if (lane == 0) { offcnt[2 * i] = base; offcnt[2 * i + 1] = nd; }
    }
    // lists / offcnt live in mapped pinned host memory: k_pack's visibility rule (no fence; the host reads after
    // hipStreamSynchronize)
}

void launch_overlap_pairs(const OvRect* r, const float4* box, int n, double max_overlap, int32_t* lists, int list_cap,
                          int32_t* offcnt, int32_t* meta, hipStream_t st) {
    if (n <= 0) return;
    const int grid = std::min((n + 3) / 4, 65535);
    hipLaunchKernelGGL(k_overlap_pairs, dim3(grid), dim3(256), 0, st, r, box, n, max_overlap, lists, list_cap, offcnt,
                       meta);
}

}  // namespace fpm
