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

int main(int argc, char** argv) {
    // problem shape (defaults: Src7 layer 0); MB_W / MB_H / MB_P / MB_TW / MB_TH / MB_NSRC override (layer-1 shape:
    // MB_W=2012 MB_H=1518 MB_P=2048 MB_TW=381 MB_TH=261); MB_WARP_ONLY=1 stops after the warp section
    auto envi = [](const char* k, int d) { const char* v = getenv(k); return v ? atoi(v) : d; };
    const int W = envi("MB_W", 4024), H = envi("MB_H", 3036), P = envi("MB_P", 4096), TW = envi("MB_TW", 762),
              TH = envi("MB_TH", 521), TP = (TW + 70) / 64 * 64 + 64;
    const int nsrc = envi("MB_NSRC", 8), ncand = 11, n3 = 3;
    const float sc = W / 4024.f;
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    std::vector<uint8_t> img((size_t)P * (H + 1) * nsrc + 4 * (size_t)P + 256), tm((size_t)TP * (TH + 1));
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
    timeit([&] { launch_roi_warp(a, 0); }, "prod warp");
    if (!envi("MB_CORR", 0)) {   // MB_CORR=1: the correlation section only (the ROIs from the product warp above)
        const long tiles = (long)a.slot_cap * ((TH + 6 + 31) / 32) * ((TW + 6 + 31) / 32);
        const int grid = (int)std::min<long>((tiles + 3) / 4, 16384);
        timeit([&] { hipLaunchKernelGGL(k_roi_warp<0>, dim3(grid), dim3(256), 0, 0, a); }, "warp foot LDS-DMA");
        timeit([&] { hipLaunchKernelGGL(k_roi_warp<12>, dim3(grid), dim3(256), 0, 0, a); }, "warp b12 7 waves (first)");
        if (!getenv("MB_SHORT")) {
            timeit([&] { hipLaunchKernelGGL((k_roi_warp<12, 0, 8>), dim3(grid), dim3(256), 0, 0, a); }, "warp b12 8 waves");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp<12, 0, 7>), dim3(grid), dim3(256), 0, 0, a); }, "warp b12 7 waves");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp<8, 0, 8>), dim3(grid), dim3(256), 0, 0, a); }, "warp b8 8 waves");
            const int grid3 = (int)std::min<long>((tiles / 3 + 3) / 4, 16384);
            timeit([&] { hipLaunchKernelGGL((k_roi_warp3<8>), dim3(grid3), dim3(256), 0, 0, a); }, "warp3 8w");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp3<7>), dim3(grid3), dim3(256), 0, 0, a); }, "warp3 7w");
            timeit([&] { hipLaunchKernelGGL((k_roi_warp3<6>), dim3(grid3), dim3(256), 0, 0, a); }, "warp3 6w");

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
    timeit([&] { launch_roi_corr(a, 0); }, "prod corr");
    if (TW > 512 && TW <= 768) {   // register-A form (12 k-steps, the Src7 layer-0 product) and its phase ablations
        const size_t lds = roi_corr_lds(a.roi_pitch, a.tw, a.rc, true);
        const long items = (long)a.slot_cap * ((TH + 31) / 32);
        const int grid = (int)std::min<long>(items, 768);
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<0, true, 3, 12, false>), dim3(grid), dim3(256), lds, 0, a); }, "corrA full");
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<0, true, 3, 12, false, 0>), dim3(grid), dim3(256), lds, 0, a); }, "corrA RS0 full");
        timeit([&] { hipLaunchKernelGGL((k_roi_corr<0, true, 3, 12, false, 1, true>), dim3(grid), dim3(256), lds, 0, a); }, "corrA SE full");
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
            auto roi_at = [&](int r, int c) { return roi_t[((size_t)((r >> 5) * txn + (c >> 5)) << 10) + (r & 31) * 32 + (c & 31)]; };
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
    }
    return 0;
}
