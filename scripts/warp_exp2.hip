// warp_exp2.hip — profiling harness (not part of the product): K6b ROI sampling with the NEXT tile's source
// footprint staged by LDS-DMA (global_load_lds_dword, no VGPRs) into the wave's second footprint buffer while the
// current tile gathers from the first, timed against the product k_roi_warp on the microbenchmark's Src7 problem
// (MB_* env overrides as in roi_microbench.hip), outputs compared byte for byte with the product's.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/warp_exp2.hip -o build/warp_exp2
#include "../fastest_image_pattern_matching_amd/csrc/fpm_kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace fpm;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

// per-wave footprint buffer: every interior 32x32 tile's box is <= 56 x 49 bytes (31*sqrt(2) + 5 columns rounded to
// an odd dword count, 31*sqrt(2) + 4 rows), so 3 KB + slack holds it at any angle
constexpr int kFtBuf = 3072;
constexpr int kFtStride = kFtBuf + 64;

// one LDS-DMA dword per lane: LDS[m0 + 4 * lane] = *gaddr (the compiler does not see it; callers order it with an
// explicit s_waitcnt vmcnt)
__device__ __forceinline__ void dma_dword(const uint8_t* gaddr, uint32_t lds_base) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gaddr), "s"(lds_base) : "memory");
}

// the tile's footprint (wpr dwords x fth rows, row-major, pitch wpr) by LDS-DMA: dword L of the image comes from
// lane L % 64 of instruction L / 64
__device__ __forceinline__ void issue_footprint_dma(uint8_t* FT, int wpr, int fth, const uint8_t* gsrc, size_t gpitch,
                                                    int lane) {
    const int total = wpr * fth;
    int r = lane / wpr, c = lane - r * wpr;
    const int dr = 64 / wpr, dc = 64 - dr * wpr;
    const uint32_t base = (uint32_t)__builtin_amdgcn_readfirstlane((int)lds_offset_of(FT));
    for (int i0 = 0; i0 < total; i0 += 64) {
        if (i0 + lane < total) dma_dword(gsrc + (size_t)r * gpitch + 4 * c, base + 4 * i0);
        r += dr;
        c += dc;
        if (c >= wpr) { c -= wpr; ++r; }
    }
}

template <int VAR>
__global__ __launch_bounds__(256) void k_warp_db(RoiArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t ft_all[4 * 2 * kFtStride];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint8_t* FTw = ft_all + wv * 2 * kFtStride;
    const int RW = a.tw + 6, RH = a.th + 6, W = a.W, H = a.H;
    const int txn = (RW + ROI_T - 1) / ROI_T, tyn = (RH + ROI_T - 1) / ROI_T;
    const int per_roi = txn * tyn;
    const int tasks = roi_count(a) * per_roi;
    const int lr = lane >> 3, lg = lane & 7;
    const XcdSplit xs = xcd_split(tasks);
    const int tstride = xs.nk * 4;
    auto staged = [](const WarpTask& w) {
        return (w.dsc.w & kTileAny) && (w.dsc.w & kTileLds) && (w.dsc.z & 0xffff) * (w.dsc.z >> 16) <= kFtBuf;
    };
    auto dma = [&](const WarpTask& w, uint8_t* FT) {
        const int ftw = w.dsc.z & 0xffff, fth = w.dsc.z >> 16;
        issue_footprint_dma(FT, ftw >> 2, fth, w.lvl + (size_t)w.dsc.y * a.P + w.dsc.x, a.P, lane);
    };
    int task = xs.lo + xs.k * 4 + wv;
    WarpTask cur;
    if (task < xs.hi) {
        warp_task_load(a, task, xs.hi, per_roi, txn, RW, RH, lr, lg, cur);
        if (staged(cur)) dma(cur, FTw);
    }
    for (int k = 0; task < xs.hi; task += tstride, ++k) {
        const int ntask = task + tstride;
        WarpTask nxt;
        if (ntask < xs.hi) warp_task_load(a, ntask, xs.hi, per_roi, txn, RW, RH, lr, lg, nxt);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this tile's footprint landed; next task's inputs loaded
        wave_sync();
        uint8_t* FT = FTw + (k & 1) * kFtStride;
        if (ntask < xs.hi && staged(nxt)) dma(nxt, FTw + ((k + 1) & 1) * kFtStride);
        const int slot = task / per_roi;
        const int rem = task - slot * per_roi;
        const int ty = rem / txn, tx = rem - ty * txn;
        const int cx0 = tx * ROI_T, cx1 = min(cx0 + ROI_T, RW) - 1;
        const int ry0 = ty * ROI_T, ry1 = min(ry0 + ROI_T, RH) - 1;
        const int c0 = cx0 + 4 * lg;
        const int4 dsc = cur.dsc, A = cur.A, B = cur.B;
        const uint8_t* lvl = cur.lvl;
        const int bxa = dsc.x, by0 = dsc.y, ftw = dsc.z & 0xffff, flags = dsc.w;
        const bool in_lds = staged(cur);
        if (c0 <= cx1) {
            uint8_t* dst = a.roi + (size_t)slot * a.roi_stride + ((size_t)(ty * txn + tx) << 10) + 4 * lg - (size_t)ry0 * ROI_T;
            const int adv[4] = {A.x, A.y, A.z, A.w}, bdv[4] = {B.x, B.y, B.z, B.w};
            if ((flags & kTileInterior) && in_lds) {
                const int nvalid = RW - c0;
                const uint32_t colmask = nvalid >= 4 ? 0xffffffffu : (1u << (8 * nvalid)) - 1u;
                const int xo = ((int)lds_offset_of(FT) - bxa) << kAbBits, yo = -(by0 << kAbBits);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int r = ry0 + lr + 8 * i;
                    const int x0r = cur.X0r[i] + xo, y0r = cur.Y0r[i] + yo;
                    uint32_t off[4];
                    int fxv[4], fyv[4], v[4][4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int sxv = x0r + adv[u], syv = y0r + bdv[u];
                        fxv[u] = __builtin_amdgcn_ubfe(sxv, kAbBits - kInterBits, kInterBits);
                        fyv[u] = __builtin_amdgcn_ubfe(syv, kAbBits - kInterBits, kInterBits);
                        off[u] = (uint32_t)mad24(syv >> kAbBits, ftw, sxv >> kAbBits);
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) lds_taps(off[u], ftw, v[u]);
                    uint32_t pk = 0;
#pragma unroll
                    for (int u = 0; u < 4; ++u) pk |= (uint32_t)bilerp24(v[u], fxv[u], fyv[u]) << (8 * u);
                    if (r <= ry1) *(uint32_t*)(dst + (size_t)r * ROI_T) = pk & colmask;
                }
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int r = ry0 + lr + 8 * i;
                    if (r > ry1) break;
                    uint32_t pk = 0;
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int X = (cur.X0r[i] + adv[u]) >> (kAbBits - kInterBits);
                        const int Y = (cur.Y0r[i] + bdv[u]) >> (kAbBits - kInterBits);
                        int v = in_lds ? ft_tap_general(FT, ftw, bxa, by0, W, H, X, Y) : roi_tap(lvl, W, H, a.P, X, Y);
                        if (c0 + u >= RW) v = 0;
                        pk |= (uint32_t)v << (8 * u);
                    }
                    *(uint32_t*)(dst + (size_t)r * ROI_T) = pk;
                }
            }
        }
        cur = nxt;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int main(int argc, char** argv) {
    auto envi = [](const char* k, int d) { const char* v = getenv(k); return v ? atoi(v) : d; };
    const int W = envi("MB_W", 4024), H = envi("MB_H", 3036), P = envi("MB_P", 4096), TW = envi("MB_TW", 762),
              TH = envi("MB_TH", 521);
    const int nsrc = envi("MB_NSRC", 8), ncand = 11, n3 = 3;
    const float sc = W / 4024.f;
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    std::vector<uint8_t> img((size_t)P * (H + 1) * nsrc);
    srand(1);
    for (auto& v : img) v = rand() & 255;
    uint8_t* d_img;
    CK(hipMalloc(&d_img, img.size()));
    CK(hipMemcpy(d_img, img.data(), img.size(), hipMemcpyHostToDevice));
    const int C = nsrc * ncand;
    std::vector<CandState> st(C);
    std::vector<int> live(C);
    std::vector<AngleNode> nodes(C * n3);
    for (int i = 0; i < C; ++i) {
        st[i].lt = f2(sc * (300.f + 137.f * (i % 11)) / 2, sc * (200.f + 91.f * (i % 7)) / 2);
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
    a.tw = TW; a.th = TH;
    a.n3 = n3; a.per_source = ncand; a.slot_base = 0; a.slot_cap = C * n3;
    a.live = d_live; a.live_count = d_cnt; a.state = d_st; a.nodes = d_nodes;
    a.tabw = roi_pitch_for(TW); a.tabh = roi_tab_rows(TH);
    a.roi_pitch = roi_pitch_for(TW); a.roi_stride = roi_tiles_bytes(TW, TH);
    CK(hipMalloc(&a.tab, (size_t)C * n3 * 2 * (a.tabw + a.tabh) * 4));
    a.tdesc_stride = roi_tiles_for(TW, TH);
    CK(hipMalloc(&a.tdesc, (size_t)C * n3 * a.tdesc_stride * sizeof(int4)));
    const size_t roi_bytes = (size_t)C * n3 * a.roi_stride;
    CK(hipMalloc(&a.roi, roi_bytes));
    auto timeit = [&](auto fn, const char* name) {
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        fn();
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) fn();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-28s %8.1f us\n", name, ms * 1000.f / reps);
    };
    launch_roi_tables(a, 0);
    CK(hipDeviceSynchronize());
    CK(hipMemset(a.roi, 0, roi_bytes));
    timeit([&] { launch_roi_warp(a, 0); }, "product warp");
    std::vector<uint8_t> h_ref(roi_bytes), h_got(roi_bytes);
    CK(hipMemcpy(h_ref.data(), a.roi, roi_bytes, hipMemcpyDeviceToHost));
    const long tiles = (long)a.slot_cap * ((TH + 6 + 31) / 32) * ((TW + 6 + 31) / 32);
    auto check = [&](const char* name) {
        CK(hipMemcpy(h_got.data(), a.roi, roi_bytes, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 0; i < roi_bytes; ++i) bad += h_got[i] != h_ref[i];
        printf("  %-26s %s (%zu bytes differ)\n", name, bad ? "MISMATCH" : "identical", bad);
        CK(hipMemset(a.roi, 0, roi_bytes));
    };
    CK(hipMemset(a.roi, 0, roi_bytes));
    for (int g : {1024, 2048, 4096, 8192, 16384}) {
        const int grid = (int)std::min<long>((tiles + 3) / 4, g);
        char nm[64];
        snprintf(nm, sizeof nm, "dma double-buffer g%d", grid);
        timeit([&] { hipLaunchKernelGGL((k_warp_db<0>), dim3(grid), dim3(256), 0, 0, a); }, nm);
        check(nm);
    }
    timeit([&] { launch_roi_warp(a, 0); }, "product warp (again)");
    printf("tiles %ld\n", tiles);
    return 0;
}
