// roi_microbench.hip — profiling harness (not part of the product): times k_roi_rows / k_roi_eval / k_pyr_down
// on a fixed Src7-sized problem (4024x3036 level, 762x521 template, 264 ROIs = 8 sources x 11 candidates x 3)
// with ablation modes, to attribute time to sampling / correlation / window sums.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/roi_microbench.hip -o build/roi_mb
#include "../fastest_image_pattern_matching_amd/csrc/fpm_kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace fpm;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

// ---- standalone ROI warp variants (materialise ROIs to HBM) ------------------------------------------------
template <int PX, bool U16>
__global__ __launch_bounds__(256) void k_warp_mat(RoiArgs a, uint8_t* out, int RWp) {
    const int RW = a.tw + 6, RH = a.th + 6;
    const int gpr = (RW + PX - 1) / PX;
    const long total = (long)(*a.live_count) * a.n3 * RH * gpr;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const int g = (int)(i % gpr);
        const long rr = i / gpr;
        const int y = (int)(rr % RH);
        const int ri = (int)(rr / RH);
        const int li = ri / a.n3, jj = ri - li * a.n3;
        const int id = a.live[li];
        const CandState st = a.state[id];
        const AngleNode nd = a.nodes[st.node * a.n3 + jj];
        const uint8_t* lvl = a.level + (size_t)(id / a.per_source) * a.level_stride;
        double M[6];
        roi_matrix(a.W, a.H, f2(st.lt.x * 2, st.lt.y * 2), nd.c, nd.s, M);
        const int X0 = rint_i((M[1] * y + M[2]) * kAbScale) + kRoundDelta;
        const int Y0 = rint_i((M[4] * y + M[5]) * kAbScale) + kRoundDelta;
        uint32_t packed = 0;
#pragma unroll
        for (int q = 0; q < PX; ++q) {
            const int x = g * PX + q;
            const int X = (X0 + rint_i(M[0] * x * kAbScale)) >> 5, Y = (Y0 + rint_i(M[3] * x * kAbScale)) >> 5;
            int v;
            if (U16) {
                const int sx = X >> 5, sy = Y >> 5, fx = X & 31, fy = Y & 31;
                if ((unsigned)sx < (unsigned)(a.W - 1) && (unsigned)sy < (unsigned)(a.H - 1)) {
                    const uint8_t* p = lvl + (size_t)sy * a.P + sx;
                    const uint32_t t0 = *(const uint16_t*)p, t1 = *(const uint16_t*)(p + a.P);
                    const int v0 = t0 & 255, v1 = t0 >> 8, v2 = t1 & 255, v3 = t1 >> 8;
                    const int h0 = 32 * v0 + fx * (v1 - v0), h1 = 32 * v2 + fx * (v3 - v2);
                    v = (32 * h0 + fy * (h1 - h0) + 512) >> 10;
                } else {
                    v = roi_tap(lvl, a.W, a.H, a.P, X, Y);
                }
            } else {
                v = roi_tap(lvl, a.W, a.H, a.P, X, Y);
            }
            packed |= (uint32_t)(v & 255) << (8 * q);
        }
        uint8_t* o = out + ((size_t)ri * RH + y) * RWp + g * PX;
        if (PX == 4) *(uint32_t*)o = packed; else *o = (uint8_t)packed;
    }
}

template <int PX, bool U16> float time_warp(const RoiArgs& a, uint8_t* out, int RWp, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int grid = 8192;
    hipLaunchKernelGGL((k_warp_mat<PX, U16>), dim3(grid), dim3(256), 0, 0, a, out, RWp);
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_warp_mat<PX, U16>), dim3(grid), dim3(256), 0, 0, a, out, RWp);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1000.f / reps;
}


// ---- split pipeline prototype: tables -> warp (materialise) -> correlation ---------------------------------
struct RoiTab { int RWp, RHp; };   // per ROI: int ad[RWp], bd[RWp], x0[RHp], y0[RHp]

__global__ __launch_bounds__(256) void k_mb_tables(RoiArgs a, int* tab, int RWp, int RHp) {
    const int ri = blockIdx.x;
    const int li = ri / a.n3, jj = ri - li * a.n3;
    const int id = a.live[li];
    const CandState st = a.state[id];
    const AngleNode nd = a.nodes[st.node * a.n3 + jj];
    double M[6];
    roi_matrix(a.W, a.H, f2(st.lt.x * 2, st.lt.y * 2), nd.c, nd.s, M);
    int* t = tab + (size_t)ri * 2 * (RWp + RHp);
    for (int x = threadIdx.x; x < RWp; x += 256) {
        t[x] = rint_i(M[0] * x * kAbScale);
        t[RWp + x] = rint_i(M[3] * x * kAbScale);
    }
    for (int y = threadIdx.x; y < RHp; y += 256) {
        t[2 * RWp + y] = rint_i((M[1] * y + M[2]) * kAbScale) + kRoundDelta;
        t[2 * RWp + RHp + y] = rint_i((M[4] * y + M[5]) * kAbScale) + kRoundDelta;
    }
}

template <int PX>
__global__ __launch_bounds__(256) void k_mb_warp(RoiArgs a, const int* tab, int RWp, int RHp, uint8_t* out, int OP) {
    const int RW = a.tw + 6, RH = a.th + 6;
    const int gpr = (RW + PX - 1) / PX;
    const int nroi = *a.live_count * a.n3;
    const long total = (long)nroi * RH * gpr;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const int g = (int)(i % gpr);
        const long rr = i / gpr;
        const int y = (int)(rr % RH);
        const int ri = (int)(rr / RH);
        const int id = a.live[ri / a.n3];
        const uint8_t* lvl = a.level + (size_t)(id / a.per_source) * a.level_stride;
        const int* t = tab + (size_t)ri * 2 * (RWp + RHp);
        const int X0 = t[2 * RWp + y], Y0 = t[2 * RWp + RHp + y];
        uint32_t pk[PX / 4];
#pragma unroll
        for (int q = 0; q < PX / 4; ++q) pk[q] = 0;
        int adv[PX], bdv[PX];
#pragma unroll
        for (int q = 0; q < PX; q += 4) {
            const int4 A = *(const int4*)(t + g * PX + q);
            const int4 B = *(const int4*)(t + RWp + g * PX + q);
            adv[q] = A.x; adv[q + 1] = A.y; adv[q + 2] = A.z; adv[q + 3] = A.w;
            bdv[q] = B.x; bdv[q + 1] = B.y; bdv[q + 2] = B.z; bdv[q + 3] = B.w;
        }
#pragma unroll
        for (int q = 0; q < PX; ++q) {
            const int X = (X0 + adv[q]) >> 5, Y = (Y0 + bdv[q]) >> 5;
            const int v = (g * PX + q < RW) ? roi_tap(lvl, a.W, a.H, a.P, X, Y) : 0;
            pk[q >> 2] |= (uint32_t)v << (8 * (q & 3));
        }
        uint8_t* o = out + ((size_t)ri * RH + y) * OP + g * PX;
        if (PX == 4) *(uint32_t*)o = pk[0];
        else if (PX == 8) *(uint2*)o = make_uint2(pk[0], pk[1]);
        else *(uint4*)o = make_uint4(pk[0], pk[1], pk[2], pk[3]);
    }
}


// 2D-blocked warp: one wave = 16 ROI rows x 16 ROI columns (lane = row*4 + colgroup, 4 px per lane)
__global__ __launch_bounds__(256) void k_mb_warp2d(RoiArgs a, const int* tab, int RWp, int RHp, uint8_t* out, int OP) {
    const int RW = a.tw + 6, RH = a.th + 6;
    const int bxn = (RW + 15) / 16, byn = (RH + 15) / 16;
    const int nroi = *a.live_count * a.n3;
    const long total = (long)nroi * byn * bxn;   // wave tasks
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int lr = lane >> 2, lg = lane & 3;
    for (long task = (long)blockIdx.x * 4 + wv; task < total; task += (long)gridDim.x * 4) {
        const int bx = (int)(task % bxn);
        const long rr = task / bxn;
        const int by = (int)(rr % byn);
        const int ri = (int)(rr / byn);
        const int id = a.live[ri / a.n3];
        const uint8_t* lvl = a.level + (size_t)(id / a.per_source) * a.level_stride;
        const int* t = tab + (size_t)ri * 2 * (RWp + RHp);
        const int y = by * 16 + lr, x0 = bx * 16 + lg * 4;
        if (y >= RH) continue;
        const int X0 = t[2 * RWp + y], Y0 = t[2 * RWp + RHp + y];
        const int4 A = *(const int4*)(t + x0);
        const int4 B = *(const int4*)(t + RWp + x0);
        const int adv[4] = {A.x, A.y, A.z, A.w}, bdv[4] = {B.x, B.y, B.z, B.w};
        uint32_t pk = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int X = (X0 + adv[q]) >> 5, Y = (Y0 + bdv[q]) >> 5;
            const int v = (x0 + q < RW) ? roi_tap(lvl, a.W, a.H, a.P, X, Y) : 0;
            pk |= (uint32_t)v << (8 * q);
        }
        *(uint32_t*)(out + ((size_t)ri * RH + y) * OP + x0) = pk;
    }
}

template <int RC>
__global__ __launch_bounds__(256) void k_mb_corr(RoiArgs a, const uint8_t* roi, int OP) {
    constexpr int NS = RC + 6;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tw = a.tw, th = a.th, RW = tw + 6, RH = th + 6;
    const int ntw = (tw + 3) / 4;
    int SBp = 4 * ntw + 12; if (SBp < RW) SBp = (RW + 3) & ~3; if (((SBp >> 2) & 1) == 0) SBp += 4;
    int TBp = 4 * ntw; if (((TBp >> 2) & 1) == 0) TBp += 4;
    uint8_t* SB = smem;
    uint8_t* TB = smem + ((NS * SBp + 15) & ~15);
    const int tid = threadIdx.x;
    const int nchunk = (th + RC - 1) / RC;
    const int items = *a.live_count * a.n3 * nchunk;
    for (int item = blockIdx.x; item < items; item += gridDim.x) {
        const int ri = item / nchunk, chunk = item - ri * nchunk;
        const int t0 = chunk * RC, rc = min(RC, th - t0), nsrc = rc + 6;
        __syncthreads();
        // ROI rows -> LDS with dword loads (OP is a multiple of 16)
        const int swd = SBp >> 2;
        for (int i = tid; i < nsrc * swd; i += 256) {
            const int r = i / swd, c = i - r * swd;
            uint32_t wv = 0;
            if (4 * c < RW) wv = *(const uint32_t*)(roi + ((size_t)ri * RH + t0 + r) * OP + 4 * c);
            *(uint32_t*)(SB + (size_t)r * SBp + 4 * c) = wv;
        }
        const int twd = TBp >> 2;
        for (int i = tid; i < rc * twd; i += 256) {
            const int r = i / twd, c = i - r * twd;
            uint32_t wv = 0;
            if (4 * c < tw) {
                wv = *(const uint32_t*)(a.tmpl + (size_t)(t0 + r) * a.tp + 4 * c);
                const int valid = tw - 4 * c;
                if (valid < 4) wv &= (1u << (8 * valid)) - 1u;
            }
            *(uint32_t*)(TB + (size_t)r * TBp + 4 * c) = wv;
        }
        __syncthreads();
        const int tl = tid % RC, dy = tid / RC;
        if (dy < 7 && tl < rc) {
            const uint32_t* trw = (const uint32_t*)(TB + (size_t)tl * TBp);
            const uint32_t* srw = (const uint32_t*)(SB + (size_t)(tl + dy) * SBp);
            uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0, c5 = 0, c6 = 0;
            uint32_t wa = srw[0], wb = srw[1];
#pragma unroll 4
            for (int k = 0; k < ntw; ++k) {
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
            uint32_t* o = a.rowsum + ((size_t)ri * th + t0 + tl) * 49 + dy * 7;
            o[0] = c0; o[1] = c1; o[2] = c2; o[3] = c3; o[4] = c4; o[5] = c5; o[6] = c6;
        }
    }
}

template <int RC> float time_corr(const RoiArgs& a, const uint8_t* roi, int OP, int reps) {
    const int tw = a.tw, ntw = (tw + 3) / 4, RW = tw + 6;
    int SBp = 4 * ntw + 12; if (SBp < RW) SBp = (RW + 3) & ~3; if (((SBp >> 2) & 1) == 0) SBp += 4;
    int TBp = 4 * ntw; if (((TBp >> 2) & 1) == 0) TBp += 4;
    const size_t lds = (((RC + 6) * SBp + 15) & ~15) + (size_t)RC * TBp;
    CK(hipFuncSetAttribute((const void*)k_mb_corr<RC>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const int items = a.slot_cap * ((a.th + RC - 1) / RC);
    const int grid = items < 8192 ? items : 8192;
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_mb_corr<RC>, dim3(grid), dim3(256), lds, 0, a, roi, OP);
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_mb_corr<RC>, dim3(grid), dim3(256), lds, 0, a, roi, OP);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("  (corr RC=%d lds %zu)\n", RC, lds);
    return ms * 1000.f / reps;
}


__global__ __launch_bounds__(256) void k_stream_read(const uint4* __restrict__ src, size_t n16, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const uint4 v = src[i];
        acc ^= v.x + v.y + v.z + v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}
__global__ __launch_bounds__(256) void k_stream_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) dst[i] = src[i];
}

int main(int argc, char** argv) {
    const int W = 4024, H = 3036, P = 4096, TW = 762, TH = 521, TP = 832;
    const int nsrc = 8, ncand = 11, n3 = 3;
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    std::vector<uint8_t> img((size_t)P * (H + 1) * nsrc), tm((size_t)TP * (TH + 1));
    srand(1);
    for (auto& v : img) v = rand() & 255;
    for (auto& v : tm) v = rand() & 255;
    uint8_t *d_img, *d_tm;
    CK(hipMalloc(&d_img, img.size())); CK(hipMalloc(&d_tm, tm.size()));
    CK(hipMemcpy(d_img, img.data(), img.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_tm, tm.data(), tm.size(), hipMemcpyHostToDevice));
    const int C = nsrc * ncand;
    std::vector<CandState> st(C);
    std::vector<int> live(C);
    std::vector<AngleNode> nodes(C * n3);
    for (int i = 0; i < C; ++i) {
        st[i].lt = f2(300.f + 137.f * (i % 11), 200.f + 91.f * (i % 7));
        st[i].lt.x /= 2; st[i].lt.y /= 2;
        st[i].node = i; st[i].alive = 1; st[i].reached0 = 1;
        live[i] = i;
        for (int j = 0; j < n3; ++j) {
            const double ang = -170.0 + 31.7 * i + 0.075 * (j - 1), r = ang * kD2R;
            nodes[i * n3 + j] = {ang, cos(r), sin(r), cos(-r), sin(-r)};
        }
    }
    CandState* d_st; int *d_live, *d_cnt; AngleNode* d_nodes;
    CK(hipMalloc(&d_st, sizeof(CandState) * C)); CK(hipMalloc(&d_live, 4 * C)); CK(hipMalloc(&d_cnt, 4));
    CK(hipMalloc(&d_nodes, sizeof(AngleNode) * C * n3));
    CK(hipMemcpy(d_st, st.data(), sizeof(CandState) * C, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_live, live.data(), 4 * C, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_cnt, &C, 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_nodes, nodes.data(), sizeof(AngleNode) * C * n3, hipMemcpyHostToDevice));
    RoiArgs a{};
    a.level = d_img; a.level_stride = (size_t)P * (H + 1); a.W = W; a.H = H; a.P = P;
    a.tmpl = d_tm; a.tw = TW; a.th = TH; a.tp = TP;
    a.n3 = n3; a.rc = argc > 2 ? atoi(argv[2]) : roi_pick_rc(TW, TH); a.nchunk = (TH + a.rc - 1) / a.rc;
    a.fold = 1; a.equal1 = 0; a.per_source = ncand; a.slot_base = 0; a.slot_cap = C * n3;
    a.mean = 100; a.norm = 5000; a.inv_area = 1.0 / (TW * TH);
    a.live = d_live; a.live_count = d_cnt; a.state = d_st; a.nodes = d_nodes;
    CK(hipMalloc(&a.rowsum, (size_t)C * n3 * TH * 49 * 4));
    CK(hipMalloc(&a.wsum, (size_t)C * n3 * a.nchunk * 49 * 4));
    CK(hipMalloc(&a.wsq, (size_t)C * n3 * a.nchunk * 49 * 8));
    CK(hipMalloc(&a.rec, sizeof(RoiRecord) * C * n3));
        printf("rois %d rc %d chunks %d corr lds %zu\n", C * n3, a.rc, a.nchunk, roi_corr_lds(roi_pitch_for(TW), TW, a.rc));
    // ---- product kernels (tables -> warp -> corr -> eval) --------------------------------------------------
    a.tabw = roi_pitch_for(TW); a.tabh = ((TH + 6) + 3) & ~3;
    a.roi_pitch = roi_pitch_for(TW); a.roi_stride = ((size_t)a.roi_pitch * (TH + 7) + 255) & ~(size_t)255;
    CK(hipMalloc(&a.tab, (size_t)C * n3 * 2 * (a.tabw + a.tabh) * 4));
    CK(hipMalloc(&a.roi, (size_t)C * n3 * a.roi_stride));
    auto timeit = [&](auto fn, const char* name) {
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        fn();
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) fn();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-20s %8.1f us\n", name, ms * 1000.f / reps);
    };
    timeit([&] { launch_roi_tables(a, 0); }, "prod tables");
    timeit([&] { launch_roi_warp(a, 0); }, "prod warp");
    timeit([&] { launch_roi_corr(a, 0); }, "prod corr");
    timeit([&] { launch_roi_eval(a, 0); }, "prod eval");
    {
        const int RWp = 784, RH = TH + 6;
        uint8_t* d_roi; CK(hipMalloc(&d_roi, (size_t)C * n3 * RH * RWp));
        printf("warp-mat 1px byte   %8.1f us\n", time_warp<1, false>(a, d_roi, RWp, reps));
        printf("warp-mat 4px byte   %8.1f us\n", time_warp<4, false>(a, d_roi, RWp, reps));
        printf("warp-mat 4px u16    %8.1f us\n", time_warp<4, true>(a, d_roi, RWp, reps));
        printf("warp-mat 1px u16    %8.1f us\n", time_warp<1, true>(a, d_roi, RWp, reps));
        // split pipeline
        const int TRW = 784, TRH = 544;
        int* d_tab; CK(hipMalloc(&d_tab, (size_t)C * n3 * 2 * (TRW + TRH) * 4));
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        float ms;
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_mb_tables, dim3(C * n3), dim3(256), 0, 0, a, d_tab, TRW, TRH);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
        printf("split tables        %8.1f us\n", ms * 1000.f / reps);
        const int OP = 784;
        uint8_t* d_roi2; CK(hipMalloc(&d_roi2, (size_t)C * n3 * RH * OP));
        auto tw8 = [&](auto kern, const char* name) {
            CK(hipEventRecord(e0));
            for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(8192), dim3(256), 0, 0, a, d_tab, TRW, TRH, d_roi2, OP);
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float m2; CK(hipEventElapsedTime(&m2, e0, e1));
            printf("%s %8.1f us\n", name, m2 * 1000.f / reps);
        };
        tw8(k_mb_warp<4>, "split warp 4px     ");
        tw8(k_mb_warp<8>, "split warp 8px     ");
        tw8(k_mb_warp<16>, "split warp 16px    ");
        tw8(k_mb_warp2d, "split warp 2d16x16 ");
        printf("split corr rc16     %8.1f us\n", time_corr<16>(a, d_roi2, OP, reps));
        printf("split corr rc32     %8.1f us\n", time_corr<32>(a, d_roi2, OP, reps));
    }
    {
        const size_t bytes = img.size(), n16 = bytes / 16;
        uint32_t* d_o; CK(hipMalloc(&d_o, 64));
        uint8_t* d_c; CK(hipMalloc(&d_c, bytes));
        for (int grid : {2048, 8192, 32768}) {
            timeit([&] { hipLaunchKernelGGL(k_stream_read, dim3(grid), dim3(256), 0, 0, (const uint4*)d_img, n16, d_o); },
                   grid == 2048 ? "stream read g2048" : grid == 8192 ? "stream read g8192" : "stream read g32768");
        }
        timeit([&] { hipLaunchKernelGGL(k_stream_copy, dim3(8192), dim3(256), 0, 0, (const uint4*)d_img, (uint4*)d_c, n16); },
               "stream copy g8192");
        printf("(%zu bytes per pass)\n", bytes);
    }
    {   // pyramid level 0 -> 1 for 8 sources
        const int dw = (W + 1) / 2, dh = (H + 1) / 2, dp = 2048;
        uint8_t* d_out; CK(hipMalloc(&d_out, (size_t)dp * (dh + 1) * nsrc));
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        launch_pyr_down(d_img, W, H, P, a.level_stride, d_out, dw, dh, dp, (size_t)dp * (dh + 1), nsrc, 0);
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r)
            launch_pyr_down(d_img, W, H, P, a.level_stride, d_out, dw, dh, dp, (size_t)dp * (dh + 1), nsrc, 0);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1000.0 / reps, bytes = (double)nsrc * ((double)W * H + (double)dw * dh);
        printf("pyr_down L0->L1 x8  %8.1f us  %.0f GB/s algorithmic\n", us, bytes / us / 1e3);
        dim3 grid((dw + 127) / 128, (dh + 31) / 32, nsrc);
        timeit([&] { hipLaunchKernelGGL(k_pyr_down<1>, grid, dim3(256), 0, 0, d_img, W, H, P, a.level_stride, d_out, dw, dh, dp, (size_t)dp * (dh + 1)); }, "pyr loads only");
        timeit([&] { hipLaunchKernelGGL(k_pyr_down<2>, grid, dim3(256), 0, 0, d_img, W, H, P, a.level_stride, d_out, dw, dh, dp, (size_t)dp * (dh + 1)); }, "pyr +lds tile");
        timeit([&] { hipLaunchKernelGGL(k_pyr_down<3>, grid, dim3(256), 0, 0, d_img, W, H, P, a.level_stride, d_out, dw, dh, dp, (size_t)dp * (dh + 1)); }, "pyr +horizontal");
        timeit([&] { hipLaunchKernelGGL(k_pyr_down<0>, grid, dim3(256), 0, 0, d_img, W, H, P, a.level_stride, d_out, dw, dh, dp, (size_t)dp * (dh + 1)); }, "pyr full");
    }
    return 0;
}
