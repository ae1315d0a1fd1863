// roi_microbench.hip — profiling harness (not part of the product): times the product refinement kernels
// (k_roi_tables / k_roi_warp / k_roi_corr / k_roi_eval) and k_pyr_down on a fixed Src7 layer-0-sized problem
// (4024x3036 level, 762x521 template, 264 ROIs = 8 sources x 11 candidates x 3), checks k_roi_corr's row dot
// products and window partials of a few ROIs against a host computation, and measures stream ceilings.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/roi_microbench.hip -o build/roi_mb
#include "../fastest_image_pattern_matching_amd/csrc/fpm_kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

using namespace fpm;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

// ---- standalone ROI warp variants (materialise ROIs to HBM) ------------------------------------------------
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

// ---- the round-3 k_roi_warp3 (per-row staging loop into VGPRs, 68-byte footprint pitch, shift + mad24 tap
// addressing), kept here as the A/B reference of the product kernel; reads the product's scaled tables
template <int FB, int WPE, int PF = 0, int TH0 = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_roi_warp3_r03(RoiArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t ft_all[4 * ROI_FT + 16];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t* FT = ft_all + wv * ROI_FT;
    const int RW = a.tw + 6, RH = a.th + 6, W = a.W, H = a.H;
    const int txn = (RW + ROI_T - 1) / ROI_T, tyn = (RH + ROI_T - 1) / ROI_T;
    const int per_roi = txn * tyn;
    const int tasks = roi_count(a) / 3 * per_roi;
    const int lr = lane >> 3, lg = lane & 7;
    const XcdSplit xs = xcd_split(tasks);
    const int tstride = xs.nk * 4;
    const uint32_t st_lane = 4u * lg + 32u * lr;
    constexpr int ftw = kFtPitch;
    // the next task's three tile descriptors are loaded (wave-uniform) while the current task runs
    int task = xs.lo + xs.k * 4 + wv;
    int4 nd[3];
    auto prefetch = [&](int t) {
        const int c_ = t / per_roi, r_ = t - c_ * per_roi;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int4 d = a.tdesc[(size_t)(3 * c_ + j) * a.tdesc_stride + r_];
            nd[j] = make_int4(__builtin_amdgcn_readfirstlane(d.x), __builtin_amdgcn_readfirstlane(d.y),
                              __builtin_amdgcn_readfirstlane(d.z), __builtin_amdgcn_readfirstlane(d.w));
        }
    };
    if (PF && task < xs.hi) prefetch(task);
    for (; task < xs.hi; task += tstride) {
        if (!PF) prefetch(task);
        const int cand = task / per_roi;
        const int rem = task - cand * per_roi;
        const int ty = rem / txn, tx = rem - ty * txn;
        const int cx0 = tx * ROI_T, cx1 = min(cx0 + ROI_T, RW) - 1;
        const int ry0 = ty * ROI_T, ry1 = min(ry0 + ROI_T, RH) - 1;
        const int c0 = cx0 + 4 * lg;
        int4 cd[3] = {nd[0], nd[1], nd[2]};
        if (PF && task + tstride < xs.hi) prefetch(task + tstride);
        int bx[3], by[3], wp[3], fh[3], fl[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int4 d = cd[j];
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
        const bool uni = any_lds && uwpr <= 16 && kFtPitch * ufth <= ROI_FT;
        // the lane's warp-table entries of one ROI (columns c0 .. c0 + 3, rows ry0 + lr + 8i); the first ROI's are
        // requested before the staging, whose round trip they then share
        const int cc = min(c0, cx1 & ~3);
        int4 tA, tB, tX, tY;
        auto load_tabs = [&](int slot_) {
            const int32_t* tb = a.tab + (size_t)slot_ * 2 * (a.tabw + a.tabh);
            tA = ld_at<int4>(tb, 4u * cc);
            tB = ld_at<int4>(tb, 4u * (a.tabw + cc));
            tX = ld_at<int4>(tb, 4u * (2 * a.tabw + ry0 + 4 * lr));
            tY = ld_at<int4>(tb, 4u * (2 * a.tabw + a.tabh + ry0 + 4 * lr));
        };
        if (TH0) load_tabs(3 * cand);
        if (uni) {
            wave_sync();   // previous task's gathers are done with FT
            stage_footprint32<FB, kFtPitch>(FT, uwpr, ufth, lvl + (size_t)uy0 * a.P + ux0, a.P, lane);
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
                if ((flags & kTileAny) && in_lds)
                    stage_footprint32<FB, kFtPitch>(FT, wp[j], fh[j], lvl + (size_t)by0 * a.P + bxa, a.P, lane);
                wave_sync();
            }
            if (!TH0 || j > 0) load_tabs(slot);
            const int adv[4] = {tA.x, tA.y, tA.z, tA.w}, bdv[4] = {tB.x, tB.y, tB.z, tB.w};
            const int X0r[4] = {tX.x, tX.y, tX.z, tX.w}, Y0r[4] = {tY.x, tY.y, tY.z, tY.w};
            uint8_t* tile = a.roi + (size_t)slot * a.roi_stride + ((size_t)rem << 10);
            if (c0 > cx1) continue;
            if ((flags & kTileInterior) && in_lds) {
                const int nvalid = RW - c0;
                const uint32_t colmask = nvalid >= 4 ? 0xffffffffu : (1u << (8 * nvalid)) - 1u;
                const int xo = ((int)lds_offset_of(FT) - bxa) << kTabFrac, yo = -(by0 << kTabFrac);
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
                    lds_taps16<kFtPitch>(off, v);
                    const uint32_t pk = bilerp_row4(v, fxv, fyv);
                    if (ry0 + lr + 8 * i <= ry1) st_at<uint32_t>(tile, st_lane + 256u * i, (pk & colmask) ^ kRoiFlip);
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
}


int main(int argc, char** argv) {
    // problem shape (defaults: Src7 layer 0); MB_W / MB_H / MB_P / MB_TW / MB_TH / MB_NSRC override (layer-1 shape:
    // MB_W=2012 MB_H=1518 MB_P=2048 MB_TW=381 MB_TH=261); MB_WARP_ONLY=1 stops after the warp section
    auto envi = [](const char* k, int d) { const char* v = getenv(k); return v ? atoi(v) : d; };
    const int W = envi("MB_W", 4024), H = envi("MB_H", 3036), P = envi("MB_P", 4096), TW = envi("MB_TW", 762),
              TH = envi("MB_TH", 521), TP = (TW + 70) / 64 * 64 + 64;
    const int nsrc = envi("MB_NSRC", 8), ncand = 11, n3 = 3;
    const float sc = W / 4024.f;
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    std::vector<uint8_t> img((size_t)P * (H + 1) * nsrc + 16 * (size_t)P + 256), tm((size_t)TP * (TH + 1));
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
        st[i].lt = f2(sc * (300.f + 137.f * (i % 11)), sc * (200.f + 91.f * (i % 7)));
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
    {   // MFMA operands: T ^ 0x80 with zero padding, per-row sums
        const int p8 = 64 * ((TW + 63) / 64), rows8 = (TH + kMmaRows - 1) / kMmaRows * kMmaRows;
        std::vector<int8_t> t8((size_t)p8 * rows8 + 512, 0);
        std::vector<int32_t> ts(rows8, 0);
        for (int y = 0; y < TH; ++y)
            for (int x = 0; x < TW; ++x) { t8[(size_t)y * p8 + x] = (int8_t)(tm[(size_t)y * TP + x] ^ 0x80); ts[y] += tm[(size_t)y * TP + x]; }
        int8_t* d8; int32_t* dts;
        CK(hipMalloc(&d8, t8.size())); CK(hipMalloc(&dts, ts.size() * 4));
        CK(hipMemcpy(d8, t8.data(), t8.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(dts, ts.data(), ts.size() * 4, hipMemcpyHostToDevice));
        a.tmpl8 = d8; a.tp8 = p8; a.nk = (TW + 63) / 64; a.tsum = dts;
    }
    a.n3 = n3; a.rc = argc > 2 ? atoi(argv[2]) : roi_pick_rc(TW, TH); a.nchunk = (TH + a.rc - 1) / a.rc;
    a.fold = 1; a.equal1 = 0; a.per_source = ncand; a.slot_base = 0; a.slot_cap = C * n3;
    a.mean = 100; a.norm = 5000; a.inv_area = 1.0 / (TW * TH);
    a.live = d_live; a.live_count = d_cnt; a.state = d_st; a.nodes = d_nodes;
    CK(hipMalloc(&a.rowsum, (size_t)C * n3 * ((TH * 49 + 3) & ~3) * 4));
    CK(hipMalloc(&a.wsum, (size_t)C * n3 * a.nchunk * 49 * 4));
    CK(hipMalloc(&a.wsq, (size_t)C * n3 * a.nchunk * 49 * 8));
    CK(hipMalloc(&a.rec, sizeof(RoiRecord) * C * n3));
        printf("rois %d rc %d chunks %d corr lds %zu / %zu\n", C * n3, a.rc, a.nchunk, roi_corr_lds(roi_pitch_for(TW), TW, a.rc, false), roi_corr_lds(roi_pitch_for(TW), TW, a.rc, true));
    // ---- product kernels (tables -> warp -> corr -> eval) --------------------------------------------------
    a.tabw = roi_pitch_for(TW); a.tabh = roi_tab_rows(TH);
    a.roi_pitch = roi_pitch_for(TW); a.roi_stride = roi_tiles_bytes(TW, TH);
    CK(hipMalloc(&a.tab, (size_t)C * n3 * 2 * (a.tabw + a.tabh) * 4));
    a.tdesc_stride = roi_tiles_for(TW, TH);
    CK(hipMalloc(&a.tdesc, (size_t)C * n3 * a.tdesc_stride * sizeof(int4)));
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
    {   // tile classes of this geometry: interior + in LDS (the fast path), in LDS with border taps, global taps
        std::vector<int4> td((size_t)C * n3 * a.tdesc_stride);
        CK(hipMemcpy(td.data(), a.tdesc, td.size() * sizeof(int4), hipMemcpyDeviceToHost));
        long fast = 0, lds_border = 0, glob = 0, empty = 0;
        for (const int4& d : td) {
            if (!(d.w & kTileAny)) ++empty;
            else if ((d.w & kTileLds) && (d.w & kTileInterior)) ++fast;
            else if (d.w & kTileLds) ++lds_border;
            else ++glob;
        }
        printf("tiles: %ld interior+LDS, %ld LDS border, %ld global taps, %ld empty\n", fast, lds_border, glob, empty);
    }
    timeit([&] { launch_roi_warp(a, 0); }, "prod warp");
    if (!envi("MB_CORR", 0) && !envi("MB_SMALL_ONLY", 0)) {
        const long tiles = (long)a.slot_cap * ((TH + 6 + 31) / 32) * ((TW + 6 + 31) / 32);
        const int grid = (int)std::min<long>((tiles + 3) / 4, 16384);
        timeit([&] { hipLaunchKernelGGL(k_roi_warp<0>, dim3(grid), dim3(256), 0, 0, a); }, "warp foot LDS-DMA");
        timeit([&] { hipLaunchKernelGGL(k_roi_warp<12>, dim3(grid), dim3(256), 0, 0, a); }, "warp b12 7 waves (first)");
        if (!getenv("MB_SHORT")) {
            timeit([&] { hipLaunchKernelGGL((k_roi_warp<12, 0, 8>), dim3(grid), dim3(256), 0, 0, a); }, "warp b12 8 waves");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp<12, 0, 7>), dim3(grid), dim3(256), 0, 0, a); }, "warp b12 7 waves");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp<8, 0, 8>), dim3(grid), dim3(256), 0, 0, a); }, "warp b8 8 waves");
        }
        {
            const int grid3 = (int)std::min<long>((tiles / 3 + 3) / 4, 16384);
            timeit([&] { hipLaunchKernelGGL((k_roi_warp3_r03<12, 7, 0, 1>), dim3(grid3), dim3(256), 0, 0, a); }, "warp3 r03 7w");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp3<8>), dim3(grid3), dim3(256), 0, 0, a); }, "warp3 8w");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp3<7>), dim3(grid3), dim3(256), 0, 0, a); }, "warp3 7w");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp3<6>), dim3(grid3), dim3(256), 0, 0, a); }, "warp3 6w");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp3<7, 68, 0>), dim3(grid3), dim3(256), 0, 0, a); }, "warp3 7w p68");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp3<7, 68, 1>), dim3(grid3), dim3(256), 0, 0, a); }, "warp3 7w p68 r03stg");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp3<8, 68, 0>), dim3(grid3), dim3(256), 0, 0, a); }, "warp3 8w p68");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp3<7, 68, 0, 1>), dim3(grid3), dim3(256), 0, 0, a); }, "warp3 abl no staging");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp3<7, 68, 0, 2>), dim3(grid3), dim3(256), 0, 0, a); }, "warp3 abl no lerp");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp3<7, 68, 0, 3>), dim3(grid3), dim3(256), 0, 0, a); }, "warp3 abl addr only");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp3<7, 68, 0, 4>), dim3(grid3), dim3(256), 0, 0, a); }, "warp3 abl no stores");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp3<7, 68, 0, 5>), dim3(grid3), dim3(256), 0, 0, a); }, "warp3 abl no interior");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp3<7, 68, 0, 0, false, true>), dim3(grid3), dim3(256), 0, 0, a); }, "warp3 7w sld");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp3<7, 68, 0, 0, true>), dim3(grid3), dim3(256), 0, 0, a); }, "warp3 7w pft");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp3<6, 68, 0, 0, true>), dim3(grid3), dim3(256), 0, 0, a); }, "warp3 6w pft");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp3<7, 68, 0, 6>), dim3(grid3), dim3(256), 0, 0, a); }, "warp3 abl -stage");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp3<7, 68, 0, 7>), dim3(grid3), dim3(256), 0, 0, a); }, "warp3 abl -tables");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp3<7, 68, 0, 8>), dim3(grid3), dim3(256), 0, 0, a); }, "warp3 abl -border");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp3<7, 64, 1>), dim3(grid3), dim3(256), 0, 0, a); }, "warp3 7w p64 r03stg");
            {   // every warp3 form writes the same ROI bytes as the round-3 form
                const size_t nb = (size_t)a.slot_cap * a.roi_stride;
                std::vector<uint8_t> ref(nb), got(nb);
                auto run_cmp = [&](auto launch, const char* name) {
                    CK(hipMemset(a.roi, 0x5a, nb));
                    launch();
                    CK(hipDeviceSynchronize());
                    CK(hipMemcpy(got.data(), a.roi, nb, hipMemcpyDeviceToHost));
                    size_t bad = 0;
                    for (size_t i = 0; i < nb; ++i) bad += got[i] != ref[i];
                    printf("warp check %-22s %s (%zu bytes differ)\n", name, bad ? "FAIL" : "OK", bad);
                };
                CK(hipMemset(a.roi, 0x5a, nb));
                hipLaunchKernelGGL((k_roi_warp3_r03<12, 7, 0, 1>), dim3(grid3), dim3(256), 0, 0, a);
                CK(hipDeviceSynchronize());
                CK(hipMemcpy(ref.data(), a.roi, nb, hipMemcpyDeviceToHost));
                run_cmp([&] { hipLaunchKernelGGL((k_roi_warp3<7>), dim3(grid3), dim3(256), 0, 0, a); }, "p64");
                run_cmp([&] { hipLaunchKernelGGL((k_roi_warp3<7, 68, 0>), dim3(grid3), dim3(256), 0, 0, a); }, "p68");
                run_cmp([&] { hipLaunchKernelGGL((k_roi_warp3<7, 68, 1>), dim3(grid3), dim3(256), 0, 0, a); }, "p68 r03stg");
                run_cmp([&] { hipLaunchKernelGGL((k_roi_warp3<7, 68, 0, 0, true>), dim3(grid3), dim3(256), 0, 0, a); }, "p68 pft");
                run_cmp([&] { hipLaunchKernelGGL((k_roi_warp3<7, 68, 0, 0, false, true>), dim3(grid3), dim3(256), 0, 0, a); }, "p68 sld");
                run_cmp([&] { launch_roi_warp(a, 0); }, "product");
            }

            timeit([&] { hipLaunchKernelGGL((k_roi_warp<12, 5, 8>), dim3(grid), dim3(256), 0, 0, a); }, "warp no stores");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp<12, 6, 8>), dim3(grid), dim3(256), 0, 0, a); }, "warp gathers only");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp<12, 7, 8>), dim3(grid), dim3(256), 0, 0, a); }, "warp gathers, no LDS");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp<12, 8, 8>), dim3(grid), dim3(256), 0, 0, a); }, "warp gathers, no math");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp<12, 9, 8>), dim3(grid), dim3(256), 0, 0, a); }, "warp gathers, 2 reads/px");
        }
        timeit([&] { hipLaunchKernelGGL((k_roi_warp<12, 1, 8>), dim3(grid), dim3(256), 0, 0, a); }, "warp no staging");
        timeit([&] { hipLaunchKernelGGL((k_roi_warp<12, 2, 8>), dim3(grid), dim3(256), 0, 0, a); }, "warp no gathers");
        timeit([&] { hipLaunchKernelGGL((k_roi_warp<12, 4, 8>), dim3(grid), dim3(256), 0, 0, a); }, "warp dot4 taps");
        timeit([&] { hipLaunchKernelGGL((k_roi_warp<12, 3, 8>), dim3(grid), dim3(256), 0, 0, a); }, "warp tables only");
        printf("tiles %ld\n", tiles);
    }
    if (envi("MB_WARP_ONLY", 0)) return 0;
    if (!envi("MB_SMALL_ONLY", 0)) {   // MB_SMALL_ONLY=1: the small-template section only
    launch_roi_warp(a, 0);   // the product's ROIs (the warp variants above may have left other bytes)
    timeit([&] { launch_roi_corr(a, 0); }, "prod corr");
    if (TW > 512 && TW <= 768) {   // register-A form (12 k-steps, the Src7 layer-0 product) and its phase ablations
        const size_t lds = roi_corr_lds(a.roi_pitch, a.tw, a.rc, true);
        const long items = (long)a.slot_cap * ((TH + 31) / 32);
        const int grid = (int)std::min<long>(items, 768);
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<0, true, 3, 12, false>), dim3(grid), dim3(256), lds, 0, a); }, "corrA full");
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<0, true, 3, 12, false, 0>), dim3(grid), dim3(256), lds, 0, a); }, "corrA RS0 full");
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<0, true, 3, 12, false, 1, true>), dim3(grid), dim3(256), lds, 0, a); }, "corrA SE full");
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<0, true, 3, 12, false, 1, true, true>), dim3(grid), dim3(256), lds, 0, a); }, "corrA SE DMA 3w");
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<0, true, 4, 12, false, 1, true, true>), dim3((int)std::min<long>(items, 1024)), dim3(256), lds, 0, a); }, "corrA SE DMA 4w");
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<0, true, 4, 12, false, 1, false, true>), dim3((int)std::min<long>(items, 1024)), dim3(256), lds, 0, a); }, "corrA DMA 4w");
        // round 5: the product form's phases (MODE ablations of k_roi_corr<., true, 4, 12, false, 1, true, true>)
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<2, true, 4, 12, false, 1, true, true>), dim3((int)std::min<long>(items, 1024)), dim3(256), lds, 0, a); }, "corrA SE DMA 4w no mfma+epi");
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<5, true, 4, 12, false, 1, true, true>), dim3((int)std::min<long>(items, 1024)), dim3(256), lds, 0, a); }, "corrA SE DMA 4w no stores");
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<6, true, 4, 12, false, 1, true, true>), dim3((int)std::min<long>(items, 1024)), dim3(256), lds, 0, a); }, "corrA SE DMA 4w no partials");
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<7, true, 4, 12, false, 1, true, true>), dim3((int)std::min<long>(items, 1024)), dim3(256), lds, 0, a); }, "corrA SE DMA 4w no rowsums");
        {
            const size_t lds_db = lds + 16 + (size_t)38 * a.roi_pitch;
            hipFuncSetAttribute((const void*)k_roi_corr<0, true, 2, 12, false, 1, true, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_db);
            hipFuncSetAttribute((const void*)k_roi_corr<0, true, 3, 12, false, 1, true, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_db);
            printf("corr DB lds %zu\n", lds_db);
            timeit([&] { hipLaunchKernelGGL((k_roi_corr<0, true, 2, 12, false, 1, true, true, true>), dim3((int)std::min<long>(items, 512)), dim3(256), lds_db, 0, a); }, "corrA SE DMA DB 2w");
            timeit([&] { hipLaunchKernelGGL((k_roi_corr<0, true, 3, 12, false, 1, true, true, true>), dim3((int)std::min<long>(items, 512)), dim3(256), lds_db, 0, a); }, "corrA SE DMA DB 3wr");
        }
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<2, true, 3, 12, false>), dim3(grid), dim3(256), lds, 0, a); }, "corrA no mfma+epi");
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<4, true, 3, 12, false>), dim3(grid), dim3(256), lds, 0, a); }, "corrA no edges");
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<5, true, 3, 12, false>), dim3(grid), dim3(256), lds, 0, a); }, "corrA no stores");
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<6, true, 3, 12, false>), dim3(grid), dim3(256), lds, 0, a); }, "corrA no partials");
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<7, true, 3, 12, false>), dim3(grid), dim3(256), lds, 0, a); }, "corrA no rowsums");
        if (envi("MB_CORR_ONLY", 0)) { launch_roi_corr(a, 0); }
    }
    if (TW > 256 && TW <= 512) {   // 8 k-steps (the Src7 layer-1 product): 3 vs 4 waves per SIMD
        const size_t lds = roi_corr_lds(a.roi_pitch, a.tw, a.rc, true);
        const long items = (long)a.slot_cap * ((TH + 31) / 32);
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<0, true, 3, 8, false>), dim3((int)std::min<long>(items, 768)), dim3(256), lds, 0, a); }, "corrA8 3 waves");
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<0, true, 3, 8, false, 1, true>), dim3((int)std::min<long>(items, 768)), dim3(256), lds, 0, a); }, "corrA8 SE 3 waves");
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<0, true, 4, 8, false, 1, true>), dim3((int)std::min<long>(items, 1024)), dim3(256), lds, 0, a); }, "corrA8 SE 4 waves");
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<0, true, 4, 8, false, 1, true, true>), dim3((int)std::min<long>(items, 1024)), dim3(256), lds, 0, a); }, "corrA8 SE DMA 4w");
        {
            const size_t lds_db = lds + 16 + (size_t)38 * a.roi_pitch;
            hipFuncSetAttribute((const void*)k_roi_corr<0, true, 4, 8, false, 1, true, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_db);
            printf("corr8 DB lds %zu\n", lds_db);
            timeit([&] { hipLaunchKernelGGL((k_roi_corr<0, true, 4, 8, false, 1, true, true, true>), dim3((int)std::min<long>(items, 1024)), dim3(256), lds_db, 0, a); }, "corrA8 SE DMA DB 4w");
        }
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<0, true, 3, 8, false, 0>), dim3((int)std::min<long>(items, 768)), dim3(256), lds, 0, a); }, "corrA8 RS0 3 waves");
    }
    timeit([&] { launch_roi_eval(a, 0); }, "prod eval");
    {
        const size_t lds0 = roi_corr_lds(a.roi_pitch, a.tw, a.rc, false), lds1 = roi_corr_lds(a.roi_pitch, a.tw, a.rc, true);
        const int grid = std::min(C * n3 * ((TH + 31) / 32), 16384);
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<0, false, 1>), dim3(grid), dim3(256), lds0, 0, a); }, "corr ldsA free");
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<0, false, 4>), dim3(grid), dim3(256), lds0, 0, a); }, "corr ldsA w4");
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<0, true, 1>), dim3(grid), dim3(256), lds1, 0, a); }, "corr globA free");
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<0, true, 3>), dim3(grid), dim3(256), lds1, 0, a); }, "corr globA w3");
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<0, true, 4>), dim3(grid), dim3(256), lds1, 0, a); }, "corr globA w4");
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<2, true, 4>), dim3(grid), dim3(256), lds1, 0, a); }, "corr globA w4 no mfma");
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<3, true, 4>), dim3(grid), dim3(256), lds1, 0, a); }, "corr globA w4 no stage");
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<3, true, 3>), dim3(grid), dim3(256), lds1, 0, a); }, "corr globA w3 no stage");
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<2, true, 3>), dim3(grid), dim3(256), lds1, 0, a); }, "corr globA w3 no mfma");
        launch_roi_corr(a, 0);
        if (envi("MB_DMA_CHECK", 0)) {   // the host check below then checks the LDS-DMA staged form
            hipMemset(a.rowsum, 0xff, (size_t)C * n3 * ((TH * 49 + 3) & ~3) * 4);
            const long items = (long)a.slot_cap * ((TH + 31) / 32);
            if (TW > 512 && TW <= 768)
                hipLaunchKernelGGL((k_roi_corr<0, true, 4, 12, false, 1, true, true>), dim3((int)std::min<long>(items, 1024)), dim3(256), lds1, 0, a);
            else if (TW > 256 && TW <= 512)
                hipLaunchKernelGGL((k_roi_corr<0, true, 4, 8, false, 1, true, true>), dim3((int)std::min<long>(items, 1024)), dim3(256), lds1, 0, a);
            printf("host check of the DMA form\n");
        }
        if (envi("MB_DB_CHECK", 0)) {   // the host check below then checks the double-buffered LDS-DMA form
            hipMemset(a.rowsum, 0xff, (size_t)C * n3 * ((TH * 49 + 3) & ~3) * 4);
            const long items = (long)a.slot_cap * ((TH + 31) / 32);
            const size_t lds_db = lds1 + 16 + (size_t)38 * a.roi_pitch;
            if (TW > 512 && TW <= 768)
                hipLaunchKernelGGL((k_roi_corr<0, true, 2, 12, false, 1, true, true, true>), dim3((int)std::min<long>(items, 512)), dim3(256), lds_db, 0, a);
            else if (TW > 256 && TW <= 512)
                hipLaunchKernelGGL((k_roi_corr<0, true, 4, 8, false, 1, true, true, true>), dim3((int)std::min<long>(items, 1024)), dim3(256), lds_db, 0, a);
            printf("host check of the DB form\n");
        }
        if (envi("MB_SE_CHECK", 0)) {   // the host check below then checks the LDS-staged epilogue form
            hipMemset(a.rowsum, 0xff, (size_t)C * n3 * ((TH * 49 + 3) & ~3) * 4);
            const long items = (long)a.slot_cap * ((TH + 31) / 32);
            if (TW > 512 && TW <= 768)
                hipLaunchKernelGGL((k_roi_corr<0, true, 3, 12, false, 1, true>), dim3((int)std::min<long>(items, 768)), dim3(256), lds1, 0, a);
            else if (TW > 256 && TW <= 512)
                hipLaunchKernelGGL((k_roi_corr<0, true, 4, 8, false, 1, true>), dim3((int)std::min<long>(items, 1024)), dim3(256), lds1, 0, a);
            printf("host check of the SE form\n");
        }
    }
    {   // host check of k_roi_corr on a few ROI slots
        const int RW = TW + 6;
        int bad = 0;
        for (int slot : {0, 1, 131, C * n3 - 1}) {
            std::vector<uint8_t> roi_t(a.roi_stride);
            const int txn = (TW + 6 + 31) / 32;
            auto roi_at = [&](int r, int c) { return (uint8_t)(roi_t[((size_t)((r >> 5) * txn + (c >> 5)) << 10) + (r & 31) * 32 + (c & 31)] ^ 0x80); };   // stored flipped
            std::vector<uint32_t> rs((size_t)TH * 49), ws((size_t)a.nchunk * 49);
            std::vector<uint64_t> wq((size_t)a.nchunk * 49);
            CK(hipMemcpy(roi_t.data(), a.roi + (size_t)slot * a.roi_stride, a.roi_stride, hipMemcpyDeviceToHost));
            CK(hipMemcpy(rs.data(), a.rowsum + (size_t)slot * ((TH * 49 + 3) & ~3), rs.size() * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(ws.data(), a.wsum + (size_t)slot * a.nchunk * 49, ws.size() * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(wq.data(), a.wsq + (size_t)slot * a.nchunk * 49, wq.size() * 8, hipMemcpyDeviceToHost));
            for (int t = 0; t < TH; ++t)
                for (int dy = 0; dy < 7; ++dy)
                    for (int dx = 0; dx < 7; ++dx) {
                        uint32_t ref = 0;
                        for (int c = 0; c < TW; ++c) ref += (uint32_t)tm[(size_t)t * TP + c] * roi_at(t + dy, c + dx);
                        if (ref != rs[(size_t)t * 49 + dy * 7 + dx]) ++bad;
                    }
            for (int ch = 0; ch < a.nchunk; ++ch)
                for (int k = 0; k < 49; ++k) {
                    const int dy = k / 7, dx = k % 7;
                    uint32_t s1 = 0; uint64_t s2 = 0;
                    for (int t = ch * a.rc; t < std::min(TH, (ch + 1) * a.rc); ++t)
                        for (int c = 0; c < TW; ++c) { const uint32_t v = roi_at(t + dy, c + dx); s1 += v; s2 += v * v; }
                    if (s1 != ws[(size_t)ch * 49 + k] || s2 != wq[(size_t)ch * 49 + k]) ++bad;
                }
            (void)RW;
        }
        printf("corr host check: %s (%d mismatches)\n", bad ? "FAIL" : "OK", bad);
    }
    }
    if (envi("MB_CORR", 0)) return 0;
    {   // small-template single-kernel refinement at Src7 layer-3 geometry: 96x66 template, 503x380 level,
        // 224 candidates x 3 angles (8 sources x 28), grid sized like the product (slot_cap WGs, most idle)
        const int TW3 = 96, TH3 = 66, W3 = 503, H3 = 380, nc3 = 28, C3 = nsrc * nc3;
        RoiArgs b = a;
        b.W = W3; b.H = H3; b.tw = TW3; b.th = TH3;
        const int p8 = 128, rows8 = 80;
        std::vector<int8_t> t8((size_t)p8 * rows8 + 512, 0);
        std::vector<int32_t> ts(rows8, 0);
        for (int y = 0; y < TH3; ++y)
            for (int x = 0; x < TW3; ++x) { t8[(size_t)y * p8 + x] = (int8_t)(tm[(size_t)y * TP + x] ^ 0x80); ts[y] += tm[(size_t)y * TP + x]; }
        int8_t* d8; int32_t* dts;
        CK(hipMalloc(&d8, t8.size())); CK(hipMalloc(&dts, ts.size() * 4));
        CK(hipMemcpy(d8, t8.data(), t8.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(dts, ts.data(), ts.size() * 4, hipMemcpyHostToDevice));
        b.tmpl8 = d8; b.tp8 = p8; b.nk = 2; b.tsum = dts;
        b.nchunk = (TH3 + 15) / 16; b.rc = 16; b.per_source = nc3;
        std::vector<CandState> st3(C3);
        std::vector<int> live3(C3);
        for (int i = 0; i < C3; ++i) {
            st3[i].lt = f2(40.f + 11.f * (i % 23), 30.f + 9.f * (i % 19));
            st3[i].node = i % C; st3[i].alive = 1; st3[i].reached0 = 0;
            live3[i] = i;
        }
        CandState* d_st3; int *d_live3, *d_cnt3;
        CK(hipMalloc(&d_st3, sizeof(CandState) * C3)); CK(hipMalloc(&d_live3, 4 * C3)); CK(hipMalloc(&d_cnt3, 4));
        CK(hipMemcpy(d_st3, st3.data(), sizeof(CandState) * C3, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_live3, live3.data(), 4 * C3, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_cnt3, &C3, 4, hipMemcpyHostToDevice));
        b.state = d_st3; b.live = d_live3; b.live_count = d_cnt3;
        // records of this section's C3 x n3 ROIs (k_roi_small writes rec[id * n3 + j]; the layer-0 section's buffer
        // holds C x n3 only -- sharing it overran that allocation, which faulted the GPU at MB_NSRC=43)
        RoiRecord* d_rec3;
        CK(hipMalloc(&d_rec3, sizeof(RoiRecord) * (size_t)C3 * n3));
        b.rec = d_rec3;
        b.slot_cap = std::max(7872, C3 * n3);   // the product's plan capacity for the 8-source batch (most WGs idle)
        const size_t lds = roi_small_lds(TW3, TH3);
        printf("small L3: rois %d lds %zu\n", C3 * n3, lds);
        timeit([&] { launch_roi_small(b, 0); }, "small prod");
        timeit([&] { hipLaunchKernelGGL(k_roi_small<1>, dim3(b.slot_cap), dim3(256), lds, 0, b); }, "small sample only");
        timeit([&] { hipLaunchKernelGGL(k_roi_small<2>, dim3(b.slot_cap), dim3(256), lds, 0, b); }, "small +sums");
        timeit([&] { hipLaunchKernelGGL(k_roi_small<3>, dim3(b.slot_cap), dim3(256), lds, 0, b); }, "small +bands nofold");
        timeit([&] { hipLaunchKernelGGL(k_roi_small<0>, dim3(C3 * n3), dim3(256), lds, 0, b); }, "small exact grid");
        timeit([&] { hipLaunchKernelGGL(k_roi_small<5>, dim3(C3 * n3), dim3(256), lds, 0, b); }, "small byte-gather taps");
        {   // per-phase s_memtime stamps of the first 64 workgroups
            uint64_t* d_stamps;
            CK(hipMalloc(&d_stamps, 64 * 16 * 8));
            CK(hipMemset(d_stamps, 0, 64 * 16 * 8));
            b.stamps = d_stamps;
            hipLaunchKernelGGL(k_roi_small<9>, dim3(C3 * n3), dim3(256), lds, 0, b);
            CK(hipDeviceSynchronize());
            std::vector<uint64_t> hs(64 * 16);
            CK(hipMemcpy(hs.data(), d_stamps, hs.size() * 8, hipMemcpyDeviceToHost));
            const char* names[7] = {"ids+tables", "sampling", "sums+tmpl", "edges", "totals", "bands+fold", "argmax+rec"};
            double acc[7] = {0};
            for (int w = 0; w < 64; ++w)
                for (int k = 0; k < 7; ++k) acc[k] += (double)(hs[w * 16 + k + 1] - hs[w * 16 + k]);
            printf("small L3 phases (cycles, mean of 64 WGs):");
            for (int k = 0; k < 7; ++k) printf(" %s %.0f", names[k], acc[k] / 64);
            printf("\n");
            double st = 0, ga = 0, tail = 0;
            int ng = 0;
            for (int w = 0; w < 64; ++w)
                if (hs[w * 16 + 8] && hs[w * 16 + 9]) {   // whole-footprint path: staging / gathers / barrier tail
                    st += (double)(hs[w * 16 + 8] - hs[w * 16 + 1]);
                    ga += (double)(hs[w * 16 + 9] - hs[w * 16 + 8]);
                    tail += (double)(hs[w * 16 + 2] - hs[w * 16 + 9]);
                    ++ng;
                }
            if (ng) printf("  sampling split over %d whole-footprint WGs: stage %.0f gathers %.0f barrier %.0f\n", ng,
                           st / ng, ga / ng, tail / ng);
            b.stamps = nullptr;
        }
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
        // levels 1 and 2: two one-level launches vs one k_pyr_down2 launch, and their bytes compared
        const int cw = (dw + 1) / 2, chh = (dh + 1) / 2, cp = 1024;
        const size_t b_img = (size_t)dp * (dh + 1), c_img = (size_t)cp * (chh + 1);
        uint8_t *d_c1, *d_b2, *d_c2;
        CK(hipMalloc(&d_c1, c_img * nsrc)); CK(hipMalloc(&d_b2, b_img * nsrc)); CK(hipMalloc(&d_c2, c_img * nsrc));
        CK(hipMemset(d_c1, 0, c_img * nsrc)); CK(hipMemset(d_b2, 0, b_img * nsrc)); CK(hipMemset(d_c2, 0, c_img * nsrc));
        CK(hipMemset(d_out, 0, b_img * nsrc));
        timeit([&] {
            launch_pyr_down(d_img, W, H, P, a.level_stride, d_out, dw, dh, dp, b_img, nsrc, 0);
            launch_pyr_down(d_out, dw, dh, dp, b_img, d_c1, cw, chh, cp, c_img, nsrc, 0);
        }, "pyr L0->L2 2 launches");
        timeit([&] { launch_pyr_down2(d_img, W, H, P, a.level_stride, d_b2, dw, dh, dp, b_img, d_c2, cw, chh, cp, c_img, nsrc, 0); },
               "pyr L0->L2 pyr_down2");
        {
            const long units2 = (long)((cw + 63) / 64) * ((dh + 31) / 32) * nsrc;
            for (int seg : {2, 3, 4, 6, 8, 12, 16}) {
                char name[64];
                snprintf(name, sizeof name, "pyr2 seg %d (%ld WGs)", seg, (units2 + seg - 1) / seg);
                timeit([&] { launch_pyr_down2(d_img, W, H, P, a.level_stride, d_b2, dw, dh, dp, b_img, d_c2, cw, chh, cp, c_img, nsrc, 0, seg); }, name);
            }
            // the pair starting at level 1 (input d_out) and level 2 (input d_c1), all sources
            {
                launch_pyr_down(d_out, dw, dh, dp, b_img, d_c1, cw, chh, cp, c_img, nsrc, 0);
                struct Lv { const uint8_t* p; int w, h, pitch; size_t img; };
                for (Lv in : {Lv{d_out, dw, dh, dp, b_img}, Lv{d_c1, cw, chh, cp, c_img}}) {
                    const int w1 = (in.w + 1) / 2, h1 = (in.h + 1) / 2, w2 = (w1 + 1) / 2, h2 = (h1 + 1) / 2;
                    const int p1 = (w1 + 4 + 63) & ~63, p2 = (w2 + 4 + 63) & ~63;
                    const size_t i1 = (size_t)p1 * (h1 + 1), i2 = (size_t)p2 * (h2 + 1);
                    uint8_t *o1, *o2;
                    CK(hipMalloc(&o1, i1 * nsrc)); CK(hipMalloc(&o2, i2 * nsrc));
                    char name[64];
                    snprintf(name, sizeof name, "pyr %dx%d 2 launches", in.w, in.h);
                    timeit([&] {
                        launch_pyr_down(in.p, in.w, in.h, in.pitch, in.img, o1, w1, h1, p1, i1, nsrc, 0);
                        launch_pyr_down(o1, w1, h1, p1, i1, o2, w2, h2, p2, i2, nsrc, 0);
                    }, name);
                    snprintf(name, sizeof name, "pyr %dx%d pyr_down2", in.w, in.h);
                    timeit([&] { launch_pyr_down2(in.p, in.w, in.h, in.pitch, in.img, o1, w1, h1, p1, i1, o2, w2, h2, p2, i2, nsrc, 0); }, name);
                    CK(hipDeviceSynchronize());
                    CK(hipFree(o1)); CK(hipFree(o2));
                }
            }
            timeit([&] {
                launch_pyr_down(d_img, W, H, P, a.level_stride, d_out, dw, dh, dp, b_img, 1, 0);
                launch_pyr_down(d_out, dw, dh, dp, b_img, d_c1, cw, chh, cp, c_img, 1, 0);
            }, "pyr 1 src 2 launches");
            timeit([&] { launch_pyr_down2(d_img, W, H, P, a.level_stride, d_b2, dw, dh, dp, b_img, d_c2, cw, chh, cp, c_img, 1, 0); },
                   "pyr 1 src pyr_down2");
        }
        CK(hipDeviceSynchronize());
        std::vector<uint8_t> x1(b_img * nsrc), x2(b_img * nsrc);
        size_t bad = 0;
        CK(hipMemcpy(x1.data(), d_out, b_img * nsrc, hipMemcpyDeviceToHost));
        CK(hipMemcpy(x2.data(), d_b2, b_img * nsrc, hipMemcpyDeviceToHost));
        for (int s = 0; s < nsrc; ++s)
            for (int y = 0; y < dh; ++y)
                for (int x = 0; x < dw; ++x) bad += x1[s * b_img + (size_t)y * dp + x] != x2[s * b_img + (size_t)y * dp + x];
        x1.resize(c_img * nsrc); x2.resize(c_img * nsrc);
        CK(hipMemcpy(x1.data(), d_c1, c_img * nsrc, hipMemcpyDeviceToHost));
        CK(hipMemcpy(x2.data(), d_c2, c_img * nsrc, hipMemcpyDeviceToHost));
        for (int s = 0; s < nsrc; ++s)
            for (int y = 0; y < chh; ++y)
                for (int x = 0; x < cw; ++x) bad += x1[s * c_img + (size_t)y * cp + x] != x2[s * c_img + (size_t)y * cp + x];
        printf("pyr_down2 check: %s (%zu bytes differ)\n", bad ? "FAIL" : "OK", bad);
    }
    return 0;
}
