// s_BlockMax peak-loop probe: an 899x899 top-layer-sized map with 144 smooth peaks on a low background (the shape
// of the Src10 config's top layer), 14x14 blocks, TargetNum 100; times k_nms_blocks + k_nms_fast, reads the
// per-phase cycle totals of k_nms_fast (NmsArgs::stamps) and checks its peaks against the global-memory k_nms.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/nms_probe.hip -o build/nms_probe
#include "../fastest_image_pattern_matching_amd/csrc/fpm_kernels.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace fpm;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

int main() {
    const int mw = 899, mh = 899, tw = 14, th = 14, cap = 105;
    std::vector<float> map((size_t)mw * mh);
    unsigned rs = 12345u;
    auto rnd = [&]() { rs = rs * 1664525u + 1013904223u; return (rs >> 8) * (1.0f / 16777216.0f); };
    for (auto& v : map) v = 0.45f * rnd() - 0.2f;
    for (int gy = 0; gy < 12; ++gy)
        for (int gx = 0; gx < 12; ++gx) {
            const float cx = 37.f + gx * 75.f + 10.f * (rnd() - 0.5f), cy = 37.f + gy * 75.f + 10.f * (rnd() - 0.5f);
            const float pk = 0.75f + 0.23f * rnd();
            for (int y = (int)cy - 6; y <= (int)cy + 6; ++y)
                for (int x = (int)cx - 6; x <= (int)cx + 6; ++x) {
                    const float d2 = (x - cx) * (x - cx) + (y - cy) * (y - cy);
                    float& v = map[(size_t)y * mw + x];
                    v = std::max(v, pk * std::exp(-d2 / 6.f));
                }
        }
    BlockGeom g;
    g.ncol = mw / tw; g.nrow = mh / th; g.rw = mw - g.ncol * tw; g.rh = mh - g.nrow * th;
    g.nb = g.ncol * g.nrow + (g.rw > 0) + (g.rh > 0) + (g.rw > 0 && g.rh > 0);
    float *d_map, *d_bmax;
    int32_t *d_bloc, *d_cand, *d_ccnt, *d_cnt;
    Peak* d_pk;
    NmsJob* d_job;
    uint64_t* d_st;
    CK(hipMalloc(&d_map, map.size() * 4));
    CK(hipMalloc(&d_bmax, g.nb * 4)); CK(hipMalloc(&d_bloc, g.nb * 4));
    CK(hipMalloc(&d_cand, kNmsCandCap * 4)); CK(hipMalloc(&d_ccnt, 4)); CK(hipMalloc(&d_cnt, 4));
    CK(hipMalloc(&d_pk, cap * sizeof(Peak))); CK(hipMalloc(&d_job, sizeof(NmsJob))); CK(hipMalloc(&d_st, 128));
    NmsJob job{d_map, d_bmax, d_bloc, mw, mh};
    CK(hipMemcpy(d_job, &job, sizeof(job), hipMemcpyHostToDevice));
    NmsArgs a{};
    a.jobs = d_job; a.peaks = d_pk; a.counts = d_cnt; a.tw = tw; a.th = th; a.cap = cap; a.by_block = 1;
    a.thr = 0.7 * 0.81; a.overlap = 0.0; a.cand = d_cand; a.cand_cnt = d_ccnt; a.cand_cap = kNmsCandCap;
    auto run = [&](bool fast, bool stamps) {
        CK(hipMemcpy(d_map, map.data(), map.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemset(d_ccnt, 0, 4));
        NmsArgs b = a;
        b.stamps = stamps ? d_st : nullptr;
        if (!fast) { b.cand = nullptr; b.cand_cnt = nullptr; }
        hipEvent_t e0, e1;
        hipEventCreate(&e0); hipEventCreate(&e1);
        hipEventRecord(e0);
        if (fast) {
            launch_nms(b, 1, g.nb, 899, ((mw + tw - 1) / tw) * ((mh + th - 1) / th), 0);
        } else {
            hipLaunchKernelGGL(k_nms_blocks, dim3((g.nb + 3) / 4), dim3(256), 0, 0, b);
            b.lds_blocks = 0;
            hipLaunchKernelGGL(k_nms, dim3(1), dim3(256), 0, 0, b, CandInitArgs{}, 0, 0);
        }
        hipEventRecord(e1);
        CK(hipEventSynchronize(e1));
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        std::vector<Peak> pk(cap);
        int cnt = 0;
        CK(hipMemcpy(&cnt, d_cnt, 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(pk.data(), d_pk, cap * sizeof(Peak), hipMemcpyDeviceToHost));
        pk.resize(cnt);
        return std::make_pair(ms, pk);
    };
    run(true, false);
    auto f = run(true, false);
    auto s = run(false, false);
    bool same = f.second.size() == s.second.size();
    for (size_t k = 0; same && k < f.second.size(); ++k)
        same = f.second[k].x == s.second[k].x && f.second[k].y == s.second[k].y && f.second[k].score == s.second[k].score;
    int ccnt = 0;
    CK(hipMemcpy(&ccnt, d_ccnt, 4, hipMemcpyDeviceToHost));
    printf("nms fast %.1f us, global %.1f us, peaks %zu / %zu, candidates %d, identical %s\n", f.first * 1e3,
           s.first * 1e3, f.second.size(), s.second.size(), ccnt, same ? "yes" : "NO");
    run(true, true);
    uint64_t st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    CK(hipMemcpy(st, d_st, 8 * 8, hipMemcpyDeviceToHost));
    const double it = st[5] > 0 ? (double)st[5] : 1;
    printf("k_nms_fast phases (cycles): setup %llu | per iteration: enumeration %.0f re-scan %.0f groups %.0f final %.0f"
           " | iterations %llu sparse %llu blocks re-scanned %llu\n", (unsigned long long)st[0], st[1] / it, st[2] / it,
           st[3] / it, st[4] / it, (unsigned long long)st[5], (unsigned long long)st[6], (unsigned long long)st[7]);
    return same ? 0 : 1;
}
