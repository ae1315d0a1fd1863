// warp4_bench.hip — profiling harness (not part of the product): k_roi_warp4 (the sampler with its per-task round
// trips off the critical path) against the product k_roi_warp3 on the Src7 layer-0 problem of roi_microbench.hip
// (MB_NSRC sources x 11 candidates x 3 angles, default 43 sources), every ROI byte compared.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/warp4_bench.hip -o build/warp4_bench
#include "../fastest_image_pattern_matching_amd/csrc/fpm_kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

using namespace fpm;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

namespace fpm {
// ---- K6b, round 5: k_roi_warp3's product path with its per-task memory round trips taken off the critical path.  A
// task of k_roi_warp3 waits for up to four dependent round trips: its three tile descriptors, the staged footprint, and
// the tables of ROIs 1 and 2 (ROI 0's share the staging's).  Options (PF bits):
//  * 1: the tables of all three ROIs (4 x 128 B each: the tile's 32 columns of adelta / bdelta and 32 rows of X0 / Y0)
//    are copied into wave LDS by LDS-DMA (global_load_lds_dwordx4, no VGPRs), the next task's issued while this
//    task's last ROI is sampled, and each ROI reads its lane's 4 x 16 bytes from LDS;
//  * 2: the next task's three descriptors are scalar loads issued at the start of this task (SGPRs);
//  * 4 (needs 2): the next task's union footprint is loaded into VGPRs before this task's last ROI is sampled and
//    written to LDS at the next task's start, so no task waits for its own footprint (16 VGPRs across that ROI).
// Same pixels, same bytes as k_roi_warp3 (main() below compares every ROI byte).  Measured (round 5, 43 sources,
// profiles/r05a/warp4_r05a.txt): no option is faster -- PF 0/1/2/3 at 7 waves 379-407 us against 380 for k_roi_warp3,
// PF 7 at 6 / 5 waves 418-430 us: the per-task round trips are hidden by the other waves already; the sampler is
// bound by instruction issue (VALU and LDS), so the kernel stays in this measurement program only.
template <int WPE, int PF>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_roi_warp4(RoiArgs a) {
    constexpr int ftw = kFtPitch;
    constexpr int kTabLds = 12 * 128;
    constexpr int kWaveLds = ROI_FT + ((PF & 1) ? kTabLds : 0);
    __shared__ __attribute__((aligned(16))) uint8_t ft_all[4 * kWaveLds + 16];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t* FT = ft_all + wv * kWaveLds;
    uint8_t* TB = FT + ROI_FT;
    const uint32_t ft_lds = lds_offset_of(FT);
    const int RW = a.tw + 6, RH = a.th + 6, W = a.W, H = a.H, P = a.P;
    const int txn = (RW + ROI_T - 1) / ROI_T, tyn = (RH + ROI_T - 1) / ROI_T;
    const int per_roi = txn * tyn;
    const int tasks = roi_count(a) / 3 * per_roi;
    const int lr = lane >> 3, lg = lane & 7;
    const XcdSplit xs = xcd_split(tasks);
    const int tstride = xs.nk * 4;
    const uint32_t st_lane = 4u * lg + 32u * lr;
    const uint32_t stage_goff = (uint32_t)((lane >> 2) * P + 16 * (lane & 3));
    const uint32_t stage_lds = ft_lds + (uint32_t)((lane >> 2) * ftw + 16 * (lane & 3));
    const size_t tab_stride = (size_t)2 * (a.tabw + a.tabh);
    const uint32_t pitch_v = __builtin_amdgcn_readfirstlane(ftw);
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    typedef int sv4 __attribute__((ext_vector_type(4)));
    // a task's three tile descriptors, raw (wave-uniform)
    auto load_desc = [&](int t, sv4 q[3]) {
        const int cand = t / per_roi, rem = t - cand * per_roi;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            if (PF & 2) {
                q[j] = *(const __attribute__((address_space(4))) sv4*)(size_t)(a.tdesc + (size_t)(3 * cand + j) * a.tdesc_stride + rem);
            } else {
                const int4 v = a.tdesc[(size_t)(3 * cand + j) * a.tdesc_stride + rem];
                q[j] = sv4{__builtin_amdgcn_readfirstlane(v.x), __builtin_amdgcn_readfirstlane(v.y),
                           __builtin_amdgcn_readfirstlane(v.z), __builtin_amdgcn_readfirstlane(v.w)};
            }
        }
    };
    // union of the boxes that stage into LDS; true: it fits the wave's buffer
    auto union_box = [&](const sv4 q[3], int& ux0, int& uy0, int& ufth) {
        int x0 = INT_MAX, y0 = INT_MAX, x1 = INT_MIN, y1 = INT_MIN;
#pragma unroll
        for (int j = 0; j < 3; ++j)
            if ((q[j].w & kTileAny) && (q[j].w & kTileLds)) {
                x0 = min(x0, q[j].x); y0 = min(y0, q[j].y);
                x1 = max(x1, q[j].x + 4 * (q[j].z & 0xffff)); y1 = max(y1, q[j].y + (q[j].z >> 16));
            }
        ux0 = x0; uy0 = y0;
        ufth = y1 - y0;
        return x0 != INT_MAX && ((x1 - x0) >> 2) <= 16 && ftw * ufth <= ROI_FT;
    };
    // footprint pieces (<= 4 per lane): issue into `sv`, commit to LDS
    auto stage_issue = [&](u32x4 (&sv)[4], int fth, const uint8_t* gsrc) {
        const int n = (fth + 15) >> 4;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (k < n) sv[k] = ld_at<u32x4>(gsrc + (size_t)k * 16 * P, stage_goff);
    };
    auto stage_commit = [&](const u32x4 (&sv)[4], int fth) {
        const int n = (fth + 15) >> 4;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (k >= n) continue;
            if ((lane >> 2) + 16 * k < ROI_FT / ftw) {
                __attribute__((address_space(3))) uint32_t* d =
                    (__attribute__((address_space(3))) uint32_t*)(size_t)(stage_lds + 16 * ftw * k);
                d[0] = sv[k].x; d[1] = sv[k].y; d[2] = sv[k].z; d[3] = sv[k].w;
            }
        }
    };
    auto stage_now = [&](int fth, const uint8_t* gsrc) {   // (a fresh register set: nothing live across tasks)
        u32x4 v[4];
        stage_issue(v, fth, gsrc);
        stage_commit(v, fth);
    };
    u32x4 svn[4];   // (PF & 4) the next task's union footprint, in flight across this task's last ROI
    // the 12 table blocks of task t into TB (block 4 j + q: q = adelta, bdelta, X0, Y0 of ROI j): two DMA instructions
    auto tab_dma = [&](int t) {
        const int cand = t / per_roi, rem = t - cand * per_roi;
        const int ty = rem / txn, tx = rem - ty * txn;
        const int cx0 = tx * ROI_T, ry0 = ty * ROI_T;
#pragma unroll
        for (int ins = 0; ins < 2; ++ins) {
            if (ins == 1 && lane >= 32) continue;
            const int b = (lane >> 3) + 8 * ins, j = b >> 2, q = b & 3;
            const int off = q == 0 ? cx0 : q == 1 ? a.tabw + cx0 : q == 2 ? 2 * a.tabw + ry0 : 2 * a.tabw + a.tabh + ry0;
            const int32_t* src = a.tab + (size_t)(3 * cand + j) * tab_stride + off + 4 * (lane & 7);
            __builtin_amdgcn_global_load_lds((fpm_gbl_vp)src, (fpm_lds_vp)(TB + 1024 * ins), 16, 0, 0);
        }
    };
    int task = xs.lo + xs.k * 4 + wv;
    if (task >= xs.hi) return;
    sv4 qn[3];   // (PF & 2) the current task's descriptors, loaded during the previous task
    if (PF & 2) load_desc(task, qn);
    if (PF & 1) tab_dma(task);
    bool pre = false;   // (PF & 4) sv holds this task's union footprint
    if (PF & 4) {
        int x0, y0, f;
        if (union_box(qn, x0, y0, f)) {
            stage_issue(svn, f, a.level + (size_t)(qn[0].w >> kTileSrcShift) * a.level_stride + (size_t)y0 * P + x0);
            pre = true;
        }
    }
    for (; task < xs.hi; task += tstride) {
        const int ntask = task + tstride;
        const bool has_next = ntask < xs.hi;
        sv4 q[3];
        if (PF & 2) {
#pragma unroll
            for (int j = 0; j < 3; ++j) q[j] = qn[j];
            if (has_next) load_desc(ntask, qn);
        } else {
            load_desc(task, q);
        }
        const int cand = task / per_roi;
        const int rem = task - cand * per_roi;
        const int ty = rem / txn, tx = rem - ty * txn;
        const int cx0 = tx * ROI_T, cx1 = min(cx0 + ROI_T, RW) - 1;
        const int ry0 = ty * ROI_T, ry1 = min(ry0 + ROI_T, RH) - 1;
        const int c0 = cx0 + 4 * lg;
        const uint8_t* lvl = a.level + (size_t)(q[0].w >> kTileSrcShift) * a.level_stride;
        int ux0, uy0, ufth;
        const bool uni = union_box(q, ux0, uy0, ufth);
        const int cc = min(c0, cx1 & ~3);
        const uint32_t oA = 4u * cc, oB = 4u * (a.tabw + cc), oX = 4u * (2 * a.tabw + ry0 + 4 * lr),
                       oY = oX + 4u * a.tabh;
        const int nvalid = RW - c0;
        const uint32_t colmask = nvalid >= 4 ? 0xffffffffu : (1u << (8 * max(nvalid, 0))) - 1u;
        int4 tA, tB, tX, tY;
        auto load_tabs = [&](int j) {
            if (PF & 1) {
                tA = *(const int4*)(TB + 512 * j + 16 * lg);
                tB = *(const int4*)(TB + 512 * j + 128 + 16 * lg);
                tX = *(const int4*)(TB + 512 * j + 256 + 16 * lr);
                tY = *(const int4*)(TB + 512 * j + 384 + 16 * lr);
            } else {
                const int32_t* tb = a.tab + (size_t)(3 * cand + j) * tab_stride;
                tA = ld_at<int4>(tb, oA);
                tB = ld_at<int4>(tb, oB);
                tX = ld_at<int4>(tb, oX);
                tY = ld_at<int4>(tb, oY);
            }
        };
        if (!(PF & 1)) load_tabs(0);
        if (uni) {
            wave_sync();   // previous task's gathers are done with FT
            if (pre) stage_commit(svn, ufth);
            else stage_now(ufth, lvl + (size_t)uy0 * P + ux0);
            wave_sync();
        }
        pre = false;
        if (PF & 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this task's tables (DMA) have landed
#pragma unroll 1
        for (int j = 0; j < 3; ++j) {
            const int slot = 3 * cand + j;
            const sv4 qj = j == 0 ? q[0] : (j == 1 ? q[1] : q[2]);   // (uniform selects: no indexed private array)
            const int flags = qj.w;
            const bool in_lds = (flags & kTileLds) != 0;
            int bxa = qj.x, by0 = qj.y;
            if (uni) {
                bxa = ux0; by0 = uy0;
            } else {
                wave_sync();
                if ((flags & kTileAny) && in_lds) stage_now(qj.z >> 16, lvl + (size_t)by0 * P + bxa);
                wave_sync();
            }
            if (PF & 1) {
                load_tabs(j);
            } else if (j > 0 && (flags & kTileAny)) {
                load_tabs(j);
            }
            if (j == 2 && has_next) {
                if (PF & 1) {
                    // this task's table reads are complete before the next task's DMA overwrites TB
                    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
                    asm volatile("" ::: "memory");
                    tab_dma(ntask);
                }
                if (PF & 4) {
                    int x0, y0, f;
                    if (union_box(qn, x0, y0, f)) {
                        stage_issue(svn, f, a.level + (size_t)(qn[0].w >> kTileSrcShift) * a.level_stride +
                                       (size_t)y0 * P + x0);
                        pre = true;
                    }
                }
            }
            const uint32_t adv[4] = {(uint32_t)tA.x, (uint32_t)tA.y, (uint32_t)tA.z, (uint32_t)tA.w};
            const uint32_t bdv[4] = {(uint32_t)tB.x, (uint32_t)tB.y, (uint32_t)tB.z, (uint32_t)tB.w};
            const uint32_t X0r[4] = {(uint32_t)tX.x, (uint32_t)tX.y, (uint32_t)tX.z, (uint32_t)tX.w};
            const uint32_t Y0r[4] = {(uint32_t)tY.x, (uint32_t)tY.y, (uint32_t)tY.z, (uint32_t)tY.w};
            uint8_t* tile = a.roi + (size_t)slot * a.roi_stride + ((size_t)rem << 10);
            if (c0 > cx1) continue;
            if (!(flags & kTileAny)) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (ry0 + lr + 8 * i <= ry1) st_at<uint32_t>(tile, st_lane + 256u * i, kRoiFlip);
                continue;
            }
            if ((flags & kTileInterior) && in_lds) {
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
                    int v[4][4];
                    lds_taps16<ftw>(off, v);
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
                    const int X = (int)(X0r[i] + adv[u]) >> kTapShift;
                    const int Y = (int)(Y0r[i] + bdv[u]) >> kTapShift;
                    int v;
                    if (in_lds) {
                        v = ft_tap_general(FT, ftw, bxa, by0, W, H, X, Y);
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

}   // namespace fpm


int main(int argc, char** argv) {
    // problem shape (defaults: Src7 layer 0); MB_W / MB_H / MB_P / MB_TW / MB_TH / MB_NSRC override (layer-1 shape:
    // MB_W=2012 MB_H=1518 MB_P=2048 MB_TW=381 MB_TH=261); MB_WARP_ONLY=1 stops after the warp section
    auto envi = [](const char* k, int d) { const char* v = getenv(k); return v ? atoi(v) : d; };
    const int W = envi("MB_W", 4024), H = envi("MB_H", 3036), P = envi("MB_P", 4096), TW = envi("MB_TW", 762),
              TH = envi("MB_TH", 521), TP = (TW + 70) / 64 * 64 + 64;
    const int nsrc = envi("MB_NSRC", 43), ncand = 11, n3 = 3;
    const float sc = W / 4024.f;
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
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
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) fn();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-28s %8.1f us\n", name, ms * 1000.f / reps);
    };
    launch_roi_tables(a, 0);
    CK(hipDeviceSynchronize());
    const long tiles = (long)a.slot_cap * ((TH + 6 + 31) / 32) * ((TW + 6 + 31) / 32);
    const int grid3 = (int)std::min<long>((tiles / 3 + 3) / 4, 16384);
    const size_t nb = (size_t)a.slot_cap * a.roi_stride;
    std::vector<uint8_t> ref(nb), got(nb);
    CK(hipMemset(a.roi, 0x5a, nb));
    hipLaunchKernelGGL((k_roi_warp3<7, kFtPitch, 0>), dim3(grid3), dim3(256), 0, 0, a);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(ref.data(), a.roi, nb, hipMemcpyDeviceToHost));
    auto check = [&](auto launch, const char* name) {
        CK(hipMemset(a.roi, 0x5a, nb));
        launch();
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got.data(), a.roi, nb, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 0; i < nb; ++i) bad += got[i] != ref[i];
        printf("check %-22s %s (%zu bytes differ)\n", name, bad ? "FAIL" : "OK", bad);
    };
#define W4(WPE, PF) do { \
        auto l = [&] { hipLaunchKernelGGL((k_roi_warp4<WPE, PF>), dim3(grid3), dim3(256), 0, 0, a); }; \
        check(l, "warp4 w" #WPE " pf" #PF); timeit(l, "warp4 w" #WPE " pf" #PF); } while (0)
    for (int rep = 0; rep < 2; ++rep) {
        timeit([&] { hipLaunchKernelGGL((k_roi_warp3<7, kFtPitch, 0>), dim3(grid3), dim3(256), 0, 0, a); }, "warp3 product");
        W4(7, 0); W4(7, 1); W4(7, 2); W4(7, 3); W4(6, 3); W4(6, 7); W4(5, 7); W4(7, 7);
    }
    return 0;
}
