// corr16_bench.hip — profiling harness (not part of the product): k_roi_corr16 (16-row items, 2-wave workgroups)
// against the product k_roi_corr on the microbenchmark's Src7 problem
// (random 4024x3036 levels, 762x521 template, 11 candidates x 3 angles per source; MB_* env overrides as in
// roi_microbench.hip, e.g. the layer-1 shape MB_W=2012 MB_H=1518 MB_P=2048 MB_TW=381 MB_TH=261).  Checks that the
// row dot products and window-sum partials (k_roi_eval's inputs) and the records k_roi_eval makes of them are
// identical, then times both.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/corr16_bench.hip -o build/corr16_bench
#define FPM_EXPERIMENTAL   // k_roi_corr16 is compiled only into this harness
#include "../fastest_image_pattern_matching_amd/csrc/fpm_kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace fpm;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

int main(int argc, char** argv) {
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
    for (int i = 0; i < C; ++i) {   // positions spread over the level, some ROIs crossing its border
        st[i].lt = f2(sc * (300.f + 137.f * (i % 11)) / 2, sc * (200.f + 91.f * (i % 7)) / 2);
        if (i % 13 == 5) st[i].lt = f2(-sc * 200.f, sc * 1400.f);
        if (i % 17 == 3) st[i].lt = f2(sc * 3700.f / 2, sc * 2900.f / 2);
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
    a.n3 = n3; a.rc = roi_pick_rc(TW, TH); a.nchunk = (TH + a.rc - 1) / a.rc;
    a.fold = 1; a.equal1 = 0; a.per_source = ncand; a.slot_base = 0; a.slot_cap = C * n3;
    a.mean = 100; a.norm = 5000; a.inv_area = 1.0 / (TW * TH);
    a.live = d_live; a.live_count = d_cnt; a.state = d_st; a.nodes = d_nodes;
    const size_t rs_n = (size_t)C * n3 * ((TH * 49 + 3) & ~3), ws_n = (size_t)C * n3 * a.nchunk * 49;
    CK(hipMalloc(&a.rowsum, rs_n * 4));
    CK(hipMalloc(&a.wsum, ws_n * 4));
    CK(hipMalloc(&a.wsq, ws_n * 8));
    CK(hipMalloc(&a.rec, sizeof(RoiRecord) * C * n3));
    a.tabw = roi_pitch_for(TW); a.tabh = roi_tab_rows(TH);
    a.roi_pitch = roi_pitch_for(TW); a.roi_stride = roi_tiles_bytes(TW, TH);
    CK(hipMalloc(&a.tab, (size_t)C * n3 * 2 * (a.tabw + a.tabh) * 4));
    a.tdesc_stride = roi_tiles_for(TW, TH);
    CK(hipMalloc(&a.tdesc, (size_t)C * n3 * a.tdesc_stride * sizeof(int4)));
    CK(hipMalloc(&a.roi, (size_t)C * n3 * a.roi_stride));
    CK(hipMemset(a.roi, 0x5a, (size_t)C * n3 * a.roi_stride));   // stale scratch: bytes k_roi_warp never writes
    auto timeit = [&](auto fn, const char* name) {
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        fn();
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) fn();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-34s %8.1f us\n", name, ms * 1000.f / reps);
        return ms * 1000.f / reps;
    };
    printf("rois %d  template %dx%d  nk %d  corr16 lds %zu B\n", C * n3, TW, TH, a.nk, roi_corr16_lds(a.roi_pitch));
    // reference: the product chain
    std::vector<uint32_t> r_rs(rs_n), r_ws(ws_n), g_rs(rs_n), g_ws(ws_n);
    std::vector<uint64_t> r_wq(ws_n), g_wq(ws_n);
    std::vector<RoiRecord> r_rec(C * n3), g_rec(C * n3);
    auto clear = [&] {
        CK(hipMemset(a.rowsum, 0xcd, rs_n * 4)); CK(hipMemset(a.wsum, 0xcd, ws_n * 4));
        CK(hipMemset(a.wsq, 0xcd, ws_n * 8)); CK(hipMemset(a.rec, 0xcd, sizeof(RoiRecord) * C * n3));
    };
    clear();
    launch_roi_tables(a, 0); launch_roi_warp(a, 0); launch_roi_corr(a, 0); launch_roi_eval(a, 0);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(r_rs.data(), a.rowsum, rs_n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r_ws.data(), a.wsum, ws_n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r_wq.data(), a.wsq, ws_n * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r_rec.data(), a.rec, sizeof(RoiRecord) * C * n3, hipMemcpyDeviceToHost));
    clear();
    if (!launch_roi_corr16(a, 0)) { printf("corr16 does not fit this shape\n"); return 1; }
    launch_roi_eval(a, 0);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(g_rs.data(), a.rowsum, rs_n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(g_ws.data(), a.wsum, ws_n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(g_wq.data(), a.wsq, ws_n * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(g_rec.data(), a.rec, sizeof(RoiRecord) * C * n3, hipMemcpyDeviceToHost));
    size_t bad_rs = 0, bad_ws = 0, bad_wq = 0, bad_rec = 0, first = (size_t)-1;
    const size_t per = (TH * 49 + 3) & ~3;
    for (size_t i = 0; i < rs_n; ++i)
        if (i % per < (size_t)TH * 49 && r_rs[i] != g_rs[i]) { ++bad_rs; if (first == (size_t)-1) first = i; }
    for (size_t i = 0; i < ws_n; ++i) { bad_ws += r_ws[i] != g_ws[i]; bad_wq += r_wq[i] != g_wq[i]; }
    bad_rec = memcmp(r_rec.data(), g_rec.data(), sizeof(RoiRecord) * C * n3) != 0;
    printf("check: rowsum %zu / wsum %zu / wsq %zu differ, records %s\n", bad_rs, bad_ws, bad_wq, bad_rec ? "DIFFER" : "identical");
    if (first != (size_t)-1) {
        const size_t sl = first / per, e = first % per;
        printf("  first rowsum mismatch: slot %zu row %zu k %zu: ref %u got %u\n", sl, e / 49, e % 49, r_rs[first], g_rs[first]);
    }
    for (int rep = 0; rep < 3; ++rep) {
        timeit([&] { launch_roi_corr(a, 0); }, "product corr");
        timeit([&] { launch_roi_corr16(a, 0); }, "corr16");
    }
    timeit([&] { launch_roi_tables(a, 0); launch_roi_warp(a, 0); launch_roi_corr(a, 0); }, "product chain");
    timeit([&] { launch_roi_tables(a, 0); launch_roi_warp(a, 0); launch_roi_corr16(a, 0); }, "chain with corr16");
    return bad_rs || bad_ws || bad_wq || bad_rec ? 2 : 0;
}
