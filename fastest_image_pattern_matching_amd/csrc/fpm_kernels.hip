// fpm_kernels.hip — MI355X (gfx950) kernels of the NCC template-matching hot path.
//
//   K1  k_pyr_down    cv::pyrDown                          (TemplateMatcher.cpp:55, :124)
//   K2  k_warp        cv::warpAffine INTER_LINEAR          (TemplateMatcher.cpp:175, :1089)
//   K3+K4 k_ncc_map   matchTemplate(TM_CCORR) + CCOEFF_Denominator   (:177 -> :514, :523, :527-598)
//   K5  k_nms         minMaxLoc + getNextMaxLoc / s_BlockMax (:179-210, :1196-1221, DataStructures.h:118-246)
//       k_cand_init   top candidate -> ptLT                (:262-266)
//   K6+K7+K8 k_roi_corr  getRotatedROI + IM_Conv_SIMD fold + CCOEFF_Denominator + minMaxLoc + 3x3
//                     (:309-328, :461-512, :527-598) fused: the ROI is sampled into LDS, never stored
//       k_cand_step   best-of-3 / early break / back-mapping (:331-366) for layers > 0
//
// Numerics contract: built with -ffp-contract=off, no fast-math; integer sums are exact; the per-row
// int32 -> f32 fold is sequential in template-row order; the normalisation is IEEE f64 in the reference's
// operation order.  Results are bit-identical to oracle/fpm_oracle.cpp.
#include <float.h>
#include <limits.h>

#include "fpm_kernels.h"

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
// Output tile 64 x 32 per 256-thread workgroup; input tile (132 + 4) x 68 bytes in LDS.  Interior tiles
// load aligned dwords; border tiles apply reflect-101 per byte.  Exact integer arithmetic.
constexpr int PYR_OW = 64, PYR_OH = 32, PYR_IW = 2 * PYR_OW + 8, PYR_IH = 2 * PYR_OH + 4;

__global__ __launch_bounds__(256) void k_pyr_down(const uint8_t* __restrict__ src, int sw, int sh, int sp,
                                                  size_t s_img, uint8_t* __restrict__ dst, int dw, int dh,
                                                  int dp, size_t d_img) {
    __shared__ __attribute__((aligned(16))) uint8_t tin[PYR_IH][PYR_IW];
    __shared__ uint16_t hs[PYR_IH][PYR_OW];
    src += (size_t)blockIdx.z * s_img;
    dst += (size_t)blockIdx.z * d_img;
    const int tid = threadIdx.x;
    const int ox0 = blockIdx.x * PYR_OW, oy0 = blockIdx.y * PYR_OH;
    const int ix0 = 2 * ox0 - 4;  // tin column 0 <-> source column ix0 (4-byte aligned)
    const int iy0 = 2 * oy0 - 2;  // tin row 0    <-> source row iy0
    const bool interior = ix0 >= 0 && ix0 + PYR_IW <= sw && iy0 >= 0 && iy0 + PYR_IH <= sh;
    if (interior) {
        constexpr int WPR = PYR_IW / 4;  // 34 dwords per row
        for (int i = tid; i < PYR_IH * WPR; i += 256) {
            const int r = i / WPR, c = i - r * WPR;
            *(uint32_t*)&tin[r][4 * c] = *(const uint32_t*)(src + (size_t)(iy0 + r) * sp + ix0 + 4 * c);
        }
    } else {
        for (int i = tid; i < PYR_IH * (PYR_IW - 4); i += 256) {
            const int r = i / (PYR_IW - 4), c = 2 + (i - r * (PYR_IW - 4));
            tin[r][c] = src[(size_t)reflect101(iy0 + r, sh) * sp + reflect101(ix0 + c, sw)];
        }
    }
    __syncthreads();
    // horizontal [1 4 6 4 1]: output column oc uses tin columns 2*oc + 2 .. 2*oc + 6
    for (int i = tid; i < PYR_IH * PYR_OW; i += 256) {
        const int r = i >> 6, oc = i & 63;
        const uint8_t* p = &tin[r][2 * oc + 2];
        hs[r][oc] = (uint16_t)(p[0] + 4 * p[1] + 6 * p[2] + 4 * p[3] + p[4]);
    }
    __syncthreads();
    const int oc = tid & 63;
    const int ox = ox0 + oc;
    for (int orow = tid >> 6; orow < PYR_OH; orow += 4) {
        const int oy = oy0 + orow;
        if (ox < dw && oy < dh) {
            const int v = hs[2 * orow][oc] + 4 * hs[2 * orow + 1][oc] + 6 * hs[2 * orow + 2][oc] +
                          4 * hs[2 * orow + 3][oc] + hs[2 * orow + 4][oc];
            dst[(size_t)oy * dp + ox] = (uint8_t)((v + 128) >> 8);
        }
    }
}

void launch_pyr_down(const uint8_t* src, int sw, int sh, int sp, size_t s_img, uint8_t* dst, int dw, int dh,
                     int dp, size_t d_img, int nimg, hipStream_t st) {
    dim3 grid((dw + PYR_OW - 1) / PYR_OW, (dh + PYR_OH - 1) / PYR_OH, nimg);
    hipLaunchKernelGGL(k_pyr_down, grid, dim3(256), 0, st, src, sw, sh, sp, s_img, dst, dw, dh, dp, d_img);
}

// ============================================================================================== K2
__global__ __launch_bounds__(256) void k_warp(const WarpJob* __restrict__ jobs) {
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

void launch_warp(const WarpJob* jobs, int njobs, int max_pixels, hipStream_t st) {
    if (njobs <= 0 || max_pixels <= 0) return;
    int gx = (max_pixels + 255) / 256;
    if (gx > 1024) gx = 1024;
    hipLaunchKernelGGL(k_warp, dim3(gx, njobs), dim3(256), 0, st, jobs);
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

void launch_ncc_map(const NccJob* jobs, int njobs, int max_out, int tmpl_bytes, hipStream_t st) {
    if (njobs <= 0 || max_out <= 0) return;
    int gx = (max_out + 255) / 256;
    if (gx > 2048) gx = 2048;
    const int in_lds = tmpl_bytes <= 32768 ? 1 : 0;
    hipLaunchKernelGGL(k_ncc_map, dim3(gx, njobs), dim3(256), in_lds ? tmpl_bytes : 0, st, jobs, in_lds);
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

struct BlockGeom {
    int ncol, nrow, rw, rh, nb;
    __device__ void init(int mw, int mh, int tw, int th) {
        ncol = mw / tw; nrow = mh / th;
        rw = mw - ncol * tw; rh = mh - nrow * th;
        nb = ncol * nrow + (rw > 0) + (rh > 0) + (rw > 0 && rh > 0);
    }
    // s_BlockMax block order (DataStructures.h:150-213): grid row-major, right strip, bottom strip, corner
    __device__ void rect(int b, int mw, int mh, int tw, int th, int& x, int& y, int& w, int& h) const {
        if (b < ncol * nrow) { x = (b % ncol) * tw; y = (b / ncol) * th; w = tw; h = th; return; }
        b -= ncol * nrow;
        if (rw > 0) { if (b == 0) { x = ncol * tw; y = 0; w = rw; h = mh; return; } --b; }
        if (rh > 0) { if (b == 0) { x = 0; y = nrow * th; w = ncol * tw; h = rh; return; } --b; }
        x = ncol * tw; y = nrow * th; w = rw; h = rh;
    }
};

__global__ __launch_bounds__(256) void k_nms(NmsArgs a) {
    __shared__ float sv[4];
    __shared__ int si[4];
    const NmsJob& j = a.jobs[blockIdx.x];
    float* m = j.map;
    const int mw = j.mw, mh = j.mh, n = mw * mh, tid = threadIdx.x;
    Peak* out = a.peaks + (size_t)blockIdx.x * a.cap;
    const double ov = a.overlap;
    BlockGeom g;
    g.init(mw, mh, a.tw, a.th);
    float v = -INFINITY;
    int i = INT_MAX;
    if (n <= 0) { if (tid == 0) a.counts[blockIdx.x] = 0; return; }
    if (a.by_block) {
        for (int b = tid; b < g.nb; b += 256) {
            int x, y, w, h;
            g.rect(b, mw, mh, a.tw, a.th, x, y, w, h);
            rect_max(m, mw, x, y, w, h, &j.bmax[b], &j.bloc[b]);
        }
        __syncthreads();
        for (int b = tid; b < g.nb; b += 256) better(v, i, j.bmax[b], b);
        wg_argmax(v, i, sv, si);
        i = j.bloc[i];
    } else {
        for (int k = tid; k < n; k += 256) { const float x = m[k]; if (x > v) { v = x; i = k; } }
        wg_argmax(v, i, sv, si);
    }
    if ((double)v < a.thr) { if (tid == 0) a.counts[blockIdx.x] = 0; return; }
    int cnt = 0;
    if (tid == 0) { out[0].x = i % mw; out[0].y = i / mw; out[0].score = v; }
    ++cnt;
    for (int it = 0; it < a.cap - 1; ++it) {
        const int px = i % mw, py = i / mw;
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
        __syncthreads();
        v = -INFINITY;
        i = INT_MAX;
        if (a.by_block) {
            for (int b = tid; b < g.nb; b += 256) {
                int x, y, w, h;
                g.rect(b, mw, mh, a.tw, a.th, x, y, w, h);
                const int ix1 = max(x, sx), iy1 = max(y, sy);
                const int iw = min(x + w, sx + rw) - ix1, ih = min(y + h, sy + rh) - iy1;
                if (iw > 0 && ih > 0) rect_max(m, mw, x, y, w, h, &j.bmax[b], &j.bloc[b]);
            }
            __syncthreads();
            for (int b = tid; b < g.nb; b += 256) better(v, i, j.bmax[b], b);
            wg_argmax(v, i, sv, si);
            i = j.bloc[i];
        } else {
            for (int k = tid; k < n; k += 256) { const float x = m[k]; if (x > v) { v = x; i = k; } }
            wg_argmax(v, i, sv, si);
        }
        if ((double)v < a.thr) break;
        if (tid == 0) { out[cnt].x = i % mw; out[cnt].y = i / mw; out[cnt].score = v; }
        ++cnt;
    }
    if (tid == 0) a.counts[blockIdx.x] = cnt;
}

void launch_nms(const NmsArgs& a, int njobs, int /*max_map*/, hipStream_t st) {
    if (njobs <= 0) return;
    hipLaunchKernelGGL(k_nms, dim3(njobs), dim3(256), 0, st, a);
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

// ============================================================================================== K6+K7+K8
// One workgroup per refinement ROI (candidate, angle j).  Per chunk of RC template rows:
//   sample ROI rows [t0, t0+rc+6) of the rotated (w+6)x(h+6) ROI straight from the pyramid level into LDS,
//   stage template rows [t0, t0+rc) into LDS, per-row int32 dot products for all 49 (dy,dx) offsets with
//   v_dot4_u32_u8 (thread = (template row, dy), 7 dx accumulators via v_alignbyte), then 49 threads fold
//   the chunk's rows into f32 in row order and add exact window sums.  Finally CCOEFF normalisation in f64,
//   first-occurrence argmax over the 7x7 map, border flag and 3x3 neighbourhood.
constexpr int ROI_MAXRC = 32;

struct RoiLayout {
    int RW, RH, ntw, SBp, TBp;
    size_t o_ad, o_bd, o_x0, o_y0, o_ra, o_rq, o_rs, o_sc, o_sb, o_tb, total;
    __host__ __device__ void make(int tw, int th, int rc) {
        RW = tw + 6; RH = th + 6;
        ntw = (tw + 3) / 4;
        SBp = 4 * ntw + 12; if (SBp < RW) SBp = (RW + 3) & ~3;
        if (((SBp >> 2) & 1) == 0) SBp += 4;
        TBp = 4 * ntw; if (((TBp >> 2) & 1) == 0) TBp += 4;
        size_t o = 0;
        auto take = [&](size_t bytes) { size_t r = o; o += (bytes + 15) & ~(size_t)15; return r; };
        o_ad = take(sizeof(int) * RW);
        o_bd = take(sizeof(int) * RW);
        o_x0 = take(sizeof(int) * (rc + 6));
        o_y0 = take(sizeof(int) * (rc + 6));
        o_ra = take(sizeof(int) * (rc + 6));
        o_rq = take(sizeof(int) * (rc + 6));
        o_rs = take(sizeof(uint32_t) * rc * 49);
        o_sc = take(sizeof(float) * 64);
        o_sb = take((size_t)(rc + 6) * SBp);
        o_tb = take((size_t)rc * TBp);
        total = o;
    }
};

size_t roi_lds_bytes(int tw, int th, int rc) {
    RoiLayout l;
    l.make(tw, th, rc);
    return l.total;
}

int roi_pick_rc(int tw, int th) {
    int rc = th < ROI_MAXRC ? th : ROI_MAXRC;
    while (rc > 1 && roi_lds_bytes(tw, th, rc) > 150 * 1024) --rc;
    return rc;
}

__global__ __launch_bounds__(256) void k_roi_corr(RoiArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    RoiLayout L;
    L.make(a.tw, a.th, a.rc);
    int* ad = (int*)(smem + L.o_ad);
    int* bd = (int*)(smem + L.o_bd);
    int* x0r = (int*)(smem + L.o_x0);
    int* y0r = (int*)(smem + L.o_y0);
    int* rall = (int*)(smem + L.o_ra);
    int* rallq = (int*)(smem + L.o_rq);
    uint32_t* rs = (uint32_t*)(smem + L.o_rs);
    float* sc = (float*)(smem + L.o_sc);
    uint8_t* SB = smem + L.o_sb;
    uint8_t* TB = smem + L.o_tb;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int RW = L.RW, tw = a.tw, th = a.th;
    const int items = *a.live_count * a.n3;

    for (int item = blockIdx.x; item < items; item += gridDim.x) {
        const int li = item / a.n3, jj = item - li * a.n3;
        const int id = a.live[li];
        const CandState st = a.state[id];
        const AngleNode nd = a.nodes[st.node * a.n3 + jj];
        RoiRecord* out = a.rec + (size_t)id * a.n3 + jj;
        if (a.equal1) {   // CCOEFF_Denominator: matResult = 1 everywhere (:529-533)
            if (tid == 0) {
                out->score = 1.f; out->mx = 0; out->my = 0; out->on_border = 1;
                for (int k = 0; k < 9; ++k) out->vec[k] = 0.f;
            }
            continue;
        }
        const int src = id / a.per_source;
        const uint8_t* lvl = a.level + (size_t)src * a.level_stride;
        double M[6];
        roi_matrix(a.W, a.H, f2(st.lt.x * 2, st.lt.y * 2), nd.c, nd.s, M);
        for (int x = tid; x < RW; x += 256) {
            ad[x] = rint_i(M[0] * x * kAbScale);
            bd[x] = rint_i(M[3] * x * kAbScale);
        }
        float accF = 0.f;
        uint64_t accI = 0;
        int64_t sumI = 0, sumQ = 0;
        const int pdy = tid / 7, pdx = tid - pdy * 7;

        for (int t0 = 0; t0 < th; t0 += a.rc) {
            const int rc = min(a.rc, th - t0), nsrc = rc + 6;
            __syncthreads();
            if (tid < nsrc) {
                const int y = t0 + tid;
                x0r[tid] = rint_i((M[1] * y + M[2]) * kAbScale) + kRoundDelta;
                y0r[tid] = rint_i((M[4] * y + M[5]) * kAbScale) + kRoundDelta;
            }
            // template rows -> LDS (dword loads, bytes beyond tw zeroed)
            const int twd = L.TBp >> 2;
            for (int r = 0; r < rc; ++r) {
                const uint8_t* trow = a.tmpl + (size_t)(t0 + r) * a.tp;
                for (int c = tid; c < twd; c += 256) {
                    uint32_t wv = 0;
                    if (4 * c < tw) {
                        wv = *(const uint32_t*)(trow + 4 * c);
                        const int valid = tw - 4 * c;
                        if (valid < 4) wv &= (1u << (8 * valid)) - 1u;
                    }
                    *(uint32_t*)(TB + (size_t)r * L.TBp + 4 * c) = wv;
                }
            }
            __syncthreads();
            // sample the ROI rows (getRotatedROI -> warpAffine, border 0)
            for (int r = 0; r < nsrc; ++r) {
                uint8_t* sbr = SB + (size_t)r * L.SBp;
                const int X0 = x0r[r], Y0 = y0r[r];
                for (int c = tid; c < L.SBp; c += 256) {
                    int v = 0;
                    if (c < RW) {
                        const int X = (X0 + ad[c]) >> (kAbBits - kInterBits);
                        const int Y = (Y0 + bd[c]) >> (kAbBits - kInterBits);
                        v = warp_tap(lvl, a.W, a.H, a.P, X, Y, 0);
                    }
                    sbr[c] = (uint8_t)v;
                }
            }
            __syncthreads();
            // full-row sums of I and I^2 (one wave per row)
            for (int r = wave; r < nsrc; r += 4) {
                const uint8_t* sbr = SB + (size_t)r * L.SBp;
                int s1 = 0, s2 = 0;
                for (int c = lane; c < RW; c += 64) { const int v = sbr[c]; s1 += v; s2 += v * v; }
                for (int off = 32; off > 0; off >>= 1) { s1 += __shfl_xor(s1, off); s2 += __shfl_xor(s2, off); }
                if (lane == 0) { rall[r] = s1; rallq[r] = s2; }
            }
            // per-row dot products: thread = (template row tl, offset dy), 7 dx accumulators
            {
                const int tl = tid & 31, dy = tid >> 5;
                if (dy < 7 && tl < rc) {
                    const uint32_t* trw = (const uint32_t*)(TB + (size_t)tl * L.TBp);
                    const uint32_t* srw = (const uint32_t*)(SB + (size_t)(tl + dy) * L.SBp);
                    uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0, c5 = 0, c6 = 0;
                    uint32_t wa = srw[0], wb = srw[1];
#pragma unroll 4
                    for (int k = 0; k < L.ntw; ++k) {
                        const uint32_t wc = srw[k + 2], t = trw[k];
                        c0 = __builtin_amdgcn_udot4(t, wa, c0, false);
                        c1 = __builtin_amdgcn_udot4(t, __builtin_amdgcn_alignbyte(wb, wa, 1), c1, false);
                        c2 = __builtin_amdgcn_udot4(t, __builtin_amdgcn_alignbyte(wb, wa, 2), c2, false);
                        c3 = __builtin_amdgcn_udot4(t, __builtin_amdgcn_alignbyte(wb, wa, 3), c3, false);
                        c4 = __builtin_amdgcn_udot4(t, wb, c4, false);
                        c5 = __builtin_amdgcn_udot4(t, __builtin_amdgcn_alignbyte(wc, wb, 1), c5, false);
                        c6 = __builtin_amdgcn_udot4(t, __builtin_amdgcn_alignbyte(wc, wb, 2), c6, false);
                        wa = wb;
                        wb = wc;
                    }
                    uint32_t* o = rs + tl * 49 + dy * 7;
                    o[0] = c0; o[1] = c1; o[2] = c2; o[3] = c3; o[4] = c4; o[5] = c5; o[6] = c6;
                }
            }
            __syncthreads();
            // fold in template-row order + exact window sums
            if (tid < 49) {
                for (int tl = 0; tl < rc; ++tl) {
                    const uint32_t v = rs[tl * 49 + tid];
                    if (a.fold) accF = accF + (float)(int)v;
                    else accI += v;
                    const int r = tl + pdy;
                    const uint8_t* sbr = SB + (size_t)r * L.SBp;
                    int s1 = rall[r], s2 = rallq[r];
                    for (int c = 0; c < pdx; ++c) { const int q = sbr[c]; s1 -= q; s2 -= q * q; }
                    for (int c = pdx + tw; c < RW; ++c) { const int q = sbr[c]; s1 -= q; s2 -= q * q; }
                    sumI += s1;
                    sumQ += s2;
                }
            }
        }
        if (tid < 49) {
            const double num = a.fold ? (double)accF : (double)(float)(double)accI;
            sc[tid] = ccoeff(num, (double)sumI, (double)sumQ, a.mean, a.norm, a.inv_area);
        }
        __syncthreads();
        if (tid == 0) {
            float best = sc[0];
            int bi = 0;
            for (int k = 1; k < 49; ++k)
                if (sc[k] > best) { best = sc[k]; bi = k; }
            const int mx = bi % 7, my = bi / 7;
            out->score = best;
            out->mx = (int16_t)mx;
            out->my = (int16_t)my;
            const int border = (mx == 0 || my == 0 || mx == 6 || my == 6) ? 1 : 0;
            out->on_border = border;
            for (int x = -1; x <= 1; ++x)
                for (int y = -1; y <= 1; ++y)
                    out->vec[(x + 1) * 3 + (y + 1)] = border ? 0.f : sc[(my + y) * 7 + (mx + x)];
        }
        __syncthreads();
    }
}

void launch_roi_corr(const RoiArgs& a, int max_items, hipStream_t st) {
    if (max_items <= 0) return;
    const size_t lds = roi_lds_bytes(a.tw, a.th, a.rc);
    static size_t lds_attr = 0;
    if (lds > 65536 && lds > lds_attr) {
        (void)hipFuncSetAttribute((const void*)k_roi_corr, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        lds_attr = lds;
    }
    int grid = max_items < 4096 ? max_items : 4096;
    hipLaunchKernelGGL(k_roi_corr, dim3(grid), dim3(256), lds, st, a);
}

// ============================================================================================== step
__global__ __launch_bounds__(256) void k_cand_step(StepArgs a) {
    const int n = *a.live_in_count;
    for (int li = blockIdx.x * 256 + threadIdx.x; li < n; li += gridDim.x * 256) {
        const int id = a.live_in[li];
        CandState s = a.state[id];
        const RoiRecord* r = a.rec + (size_t)id * a.n3;
        int imax = 0;
        double big = -1;
        for (int j = 0; j < a.n3; ++j)
            if ((double)r[j].score > big) { imax = j; big = r[j].score; }
        if ((double)r[imax].score < a.thr) {   // :331-332
            s.alive = 0;
            a.state[id] = s;
            continue;
        }
        const int child = s.node * a.n3 + imax;
        const AngleNode nd = a.nodes[child];
        const F2 sc = f2((a.W - 1) / 2.0f, (a.H - 1) / 2.0f);
        // :350-353
        const F2 r0 = rotate_pt(f2(s.lt.x * 2, s.lt.y * 2), sc, nd.c, nd.s);
        const F2 pad = f2(r0.x - 3, r0.y - 3);
        F2 p = f2((float)((double)r[imax].mx + pad.x), (float)((double)r[imax].my + pad.y));
        p = rotate_pt(p, sc, nd.cn, nd.sn);
        s.lt = p;          // :366
        s.node = child;    // :363 (angle = node angle)
        s.reached0 = a.mark_reached0;
        a.state[id] = s;
        const int slot = atomicAdd(a.live_out_count, 1);
        a.live_out[slot] = id;
    }
}

void launch_cand_step(const StepArgs& a, int max_items, hipStream_t st) {
    if (max_items <= 0) return;
    int grid = (max_items + 255) / 256;
    if (grid > 1024) grid = 1024;
    hipLaunchKernelGGL(k_cand_step, dim3(grid), dim3(256), 0, st, a);
}

}  // namespace fpm
