// fpm_engine.hip — host orchestration of the MI355X template matcher and the C ABI (include/fpm.h).
//
// Mirrors TemplateMatcher::learnPattern / match (src/TemplateMatcher.cpp:45-437) with this split:
//   host, once per (template, params, source size):  angle list (:130-144), per-angle canvas size and
//       warp matrix (:163-173, :901-969), refinement angle tree with glibc cos/sin (:282-298), buffer layout;
//   device, per search (one stream, no host sync until the end):  pyramid (K1), top-layer rotation + NCC +
//       peak extraction for every (source, angle) (K2-K5), candidate init, and the layer loop
//       L-1 .. 0 (K6-K8 fused + best-of-3 step) over a device-compacted live-candidate list;
//   host, after ONE device->host copy:  reference-order candidate sort (:214), layer-0 decision / sub-pixel /
//       back-mapping (:331-358), filterWithScore, filterWithRotatedRect, final sort and s_SingleTargetMatch
//       conversion (:373-432).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/fpm.h"
#include "fpm_host.h"
#include "fpm_kernels.h"

using namespace fpm;

namespace {

inline int round_up(int v, int a) { return (v + a - 1) / a * a; }
inline size_t round_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

struct DevBuf {
    void* p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= n && p) return hipSuccess;
        if (p) { (void)hipFree(p); p = nullptr; n = 0; }
        if (bytes == 0) bytes = 256;
        hipError_t e = hipMalloc(&p, bytes);
        if (e == hipSuccess) n = bytes;
        return e;
    }
    void release() { if (p) (void)hipFree(p); p = nullptr; n = 0; }
    template <class T> T* as(size_t byte_off = 0) const { return (T*)((char*)p + byte_off); }
};

struct PinBuf {
    void* p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= n && p) return hipSuccess;
        if (p) { (void)hipHostFree(p); p = nullptr; n = 0; }
        if (bytes == 0) bytes = 256;
        hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocMapped);   // device-visible (k_pack writes it)
        if (e == hipSuccess) n = bytes;
        return e;
    }
    void release() { if (p) (void)hipHostFree(p); p = nullptr; n = 0; }
    template <class T> T* as(size_t byte_off = 0) const { return (T*)((char*)p + byte_off); }
};

struct TmplLevel {
    int w, h, pitch;
    size_t off;              // offset in the device template slab
    size_t off8;             // offset in the i8 template slab (T ^ 0x80, zero padded; MFMA A operand)
    int p8;                  // its row pitch: 64 * ceil(w / 64)
    size_t tsum_off;         // offset (elements) of the per-row sums in d_tsum
    double mean, norm, inv_area;
    bool equal1;
    std::vector<uint8_t> px; // host copy (dense)
};

struct SrcLevel {
    int w, h, pitch;
    size_t img_bytes;        // pitch * h (rounded), per source image
    size_t off;              // offset of source 0 in the device source slab
};

// Everything that depends only on (template, params, source size, batch size).
struct Plan {
    bool valid = false;
    int sw = 0, sh = 0, S = 0, L = 0;
    fpm_params prm{};
    int nang = 0, cap = 0, n3 = 1, C = 0;      // C = S * nang * cap candidate slots
    int a0 = 0, nang_all = 0;                  // this plan's angles = [a0, a0 + nang) of the full top-layer list
    int shard = 0, shards = 1;                 // angle shard the plan was built for (fpm_set_angle_shard)
    bool by_block = false;
    uint32_t step_layers = 0;                  // bit d: the last pass launched k_cand_step for layer depth d (profiling)
    bool top_lists = false;                    // the last pass took its top-layer peaks from k_top_mma's lists
    std::vector<double> angles, layer_score;
    std::vector<TopAngle> top;
    std::vector<AngleNode> top_nodes;
    std::vector<std::vector<AngleNode>> nodes;  // [d], d = 0 <-> layer L-1
    std::vector<size_t> node_off;                // device offsets (elements)
    F2 center;
    // top-layer layout (per source)
    std::vector<size_t> canvas_off, map_off, blk_off;
    std::vector<int> canvas_pitch, map_w, map_h, nblk;
    std::vector<int32_t> order;                // k_top_fused workgroup -> job (costliest angles first)
    size_t canvas_bytes = 0, map_floats = 0, blk_count = 0;
    int max_canvas = 0, max_map = 0, max_nblk = 0, max_cells = 0, max_nitems = 0;
    int off_skey = 0, nzero = 0;   // d_livecnt layout: strip keys' offset, words zeroed by k_warp
    // the matrix-core top layer (k_top_mma + k_nms_greedy on its candidate lists): layout and
    // constants of the launch (pointers set at plan time), the unit list and B fragments in d_tmu, the values of the
    // lists in d_tcandv (indices in d_ncand), their counts at d_livecnt + L + 2 (zeroed by the first pyramid launch)
    bool top_mma = false;
    TopMmaArgs tma{};
    int tcand_cap = 0;
    DevBuf d_tmu, d_tcandv;
    // device buffers owned by the plan
    DevBuf d_ncand;                            // s_BlockMax candidate lists (k_nms_blocks -> k_nms_fast)
    DevBuf d_canvas, d_map, d_bmax, d_bloc, d_jobs, d_nodes, d_top, d_topn, d_peaks, d_counts, d_state,
        d_live, d_livecnt, d_rec, d_rowsum, d_wsum, d_wsq, d_tab, d_roi, d_tdesc, d_state2, d_rec2;
    int tabw = 0, tabh = 0, roi_pitch = 0, tdesc_stride = 1;
    size_t roi_stride = 0;
    int slot_cap = 0;                          // ROIs per refinement round (bounded scratch)
    size_t off_warp = 0, off_ncc = 0, off_nms = 0, off_order = 0;
    PinBuf h_out;
    size_t h_counts = 0, h_peaks = 0, h_live = 0, h_live0 = 0, h_state = 0, h_rec = 0, h_total = 0;
    char* h_dev = nullptr;   // device-side address of h_out (k_pack writes it over PCIe)
    void release() {
        for (DevBuf* b : {&d_tmu, &d_tcandv, &d_ncand, &d_canvas, &d_map, &d_bmax, &d_bloc, &d_jobs, &d_nodes, &d_top, &d_topn, &d_peaks,
                          &d_counts, &d_state, &d_live, &d_livecnt, &d_rec, &d_rowsum, &d_wsum, &d_wsq, &d_tab, &d_roi, &d_tdesc, &d_state2, &d_rec2})
            b->release();
        h_out.release();
        valid = false;
    }
};

struct KProf {
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
    size_t used = 0;
    double ms = 0;
    int64_t launches = 0, bytes = 0;
};

}  // namespace

struct fpm_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    fpm_params prm{};
    std::string err;
    // template (s_TemplData)
    bool learned = false;
    int border = 0;
    std::vector<TmplLevel> tmpl;
    DevBuf d_tmpl, d_tmpl8, d_tsum;
    uint64_t tmpl_gen = 0;
    // staged sources
    int S = 0, sw = 0, sh = 0, src_L = -1;
    // angle shard (fpm_set_angle_shard): this context's slice of the top-layer angle list
    int shard = 0, shards = 1;
    std::vector<SrcLevel> src;
    DevBuf d_src;
    // plan
    Plan plan;
    uint64_t plan_gen = ~0ull;
    // op scratch
    DevBuf d_op_a, d_op_b, d_op_job;
    // filterWithRotatedRect on the device (overlap_filter_device): rectangles + counters; staging and mapped outputs
    DevBuf d_ov;
    PinBuf h_ov_in, h_ov_out;
    // last search stats
    std::vector<int64_t> stats;
    int64_t alg_bytes[3] = {0, 0, 0};   // SURVEY.md §8(d) algorithmic bytes of the last search: B_pyr, B_top, B_ref
    // profiling
    bool prof = false;
    KProf kp[FPM_K_COUNT];
    // the whole device-resident search captured once per (plan, source slab) and replayed as one hipGraph
    hipGraphExec_t graph = nullptr;
    uint64_t graph_plan = ~0ull;
    const void* graph_src = nullptr;
    uint64_t plan_builds = 0;
    // timing of the last search (fpm_profile_last)
    hipEvent_t t_ev[2] = {nullptr, nullptr};
    double last_device_ms = 0, last_host_ms = 0, last_call_ms = 0;
    std::chrono::steady_clock::time_point t_call0;
    bool pending = false;    // a staged search is in flight (fpm_match_staged_launch)
    bool staged = false;     // the source slab holds an fpm_stage_sources batch (fpm_match re-lays it out for one source)
    fpm_params run_prm{};    // parameters of the search in flight (snapshot at launch; the host tail reads these)
    // per-source candidate records of the last search (collect_candidates; fpm_match_*candidates)
    std::vector<std::vector<fpm_candidate>> cands;
    std::vector<std::vector<fpm_result>> results;   // of the last search, per source (fpm_last_results)
};

#define HIP_TRY(expr)                                                                   \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess) {                                                         \
            ctx->err = std::string(#expr) + ": " + hipGetErrorString(e_);               \
            return FPM_E_DEVICE;                                                        \
        }                                                                               \
    } while (0)

namespace {

// ---------------------------------------------------------------------------------------------------------
// profiling helpers
// ---------------------------------------------------------------------------------------------------------
struct ProfScope {
    fpm_ctx* ctx;
    int k;
    hipEvent_t b = nullptr, e = nullptr;
    ProfScope(fpm_ctx* c, int kk, int64_t bytes) : ctx(c), k(kk) {
        if (!ctx->prof) return;
        KProf& p = ctx->kp[k];
        if (p.used == p.ev.size()) {
            hipEvent_t x, y;
            if (hipEventCreate(&x) != hipSuccess || hipEventCreate(&y) != hipSuccess) return;
            p.ev.push_back({x, y});
        }
        b = p.ev[p.used].first;
        e = p.ev[p.used].second;
        p.used++;
        p.launches++;
        p.bytes += bytes;
        (void)hipEventRecord(b, ctx->stream);
    }
    ~ProfScope() {
        if (b) (void)hipEventRecord(e, ctx->stream);
    }
};

void prof_collect(fpm_ctx* ctx) {
    if (!ctx->prof) return;
    for (int k = 0; k < FPM_K_COUNT; ++k) {
        KProf& p = ctx->kp[k];
        for (size_t i = 0; i < p.used; ++i) {
            float ms = 0;
            if (hipEventElapsedTime(&ms, p.ev[i].first, p.ev[i].second) == hipSuccess) p.ms += ms;
        }
        p.used = 0;
    }
}

// ---------------------------------------------------------------------------------------------------------
// host restatements of reference helpers
// ---------------------------------------------------------------------------------------------------------
int top_layer(int w, int h, int min_len) {   // getTopLayer (TemplateMatcher.cpp:445-455)
    int L = 0, mra = min_len * min_len, area = w * h;
    while (area > mra) { area /= 4; ++L; }
    return L;
}

void mean_stddev(const std::vector<uint8_t>& px, double* mean, double* sdv) {  // cv::meanStdDev, 8UC1
    int64_t s = 0, q = 0;
    for (uint8_t v : px) { s += v; q += (int64_t)v * v; }
    const double scale = px.empty() ? 0. : 1. / (double)px.size();
    const double m = (double)s * scale;
    *mean = m;
    *sdv = std::sqrt(std::max((double)q * scale - m * m, 0.));
}

// getBestRotationSize (TemplateMatcher.cpp:901-969); ptRotatePt2f with glibc trig of angle*D2R
void best_rotation_size(int sw, int sh, int dw, int dh, double ang, int* ow, int* oh) {
    const double rad = ang * kD2R, c = std::cos(rad), s = std::sin(rad);
    const F2 ctr = f2((sw - 1) / 2.0f, (sh - 1) / 2.0f);
    const F2 lt = rotate_pt(f2(0.f, 0.f), ctr, c, s);
    const F2 lb = rotate_pt(f2(0.f, (float)(sh - 1)), ctr, c, s);
    const F2 rb = rotate_pt(f2((float)(sw - 1), (float)(sh - 1)), ctr, c, s);
    const F2 rt = rotate_pt(f2((float)(sw - 1), 0.f), ctr, c, s);
    const float top = std::max(std::max(lt.y, lb.y), std::max(rb.y, rt.y));
    const float bottom = std::min(std::min(lt.y, lb.y), std::min(rb.y, rt.y));
    const float right = std::max(std::max(lt.x, lb.x), std::max(rb.x, rt.x));
    const float left = std::min(std::min(lt.x, lb.x), std::min(rb.x, rt.x));
    if (ang > 360) ang -= 360;
    else if (ang < 0) ang += 360;
    if (std::fabs(std::fabs(ang) - 90) < kVisionTol || std::fabs(std::fabs(ang) - 270) < kVisionTol) {
        *ow = sh; *oh = sw;
        return;
    }
    if (std::fabs(ang) < kVisionTol || std::fabs(std::fabs(ang) - 180) < kVisionTol) {
        *ow = sw; *oh = sh;
        return;
    }
    double a = ang;
    if (a > 90 && a < 180) a -= 90;
    else if (a > 180 && a < 270) a -= 180;
    else if (a > 270 && a < 360) a -= 270;
    const float h1 = dw * std::sin(a * kD2R) * std::cos(a * kD2R);
    const float h2 = dh * std::sin(a * kD2R) * std::cos(a * kD2R);
    const int half_h = (int)std::ceil(top - ctr.y - h1);
    const int half_w = (int)std::ceil(right - ctr.x - h2);
    int rw = half_w * 2, rh = half_h * 2;
    const bool wrong = (dw < rw && dh > rh) || ((dw > rw && dh < rh) || (int64_t)dw * dh > (int64_t)rw * rh);
    if (wrong) { rw = int(right - left + 0.5); rh = int(top - bottom + 0.5); }
    *ow = rw;
    *oh = rh;
}

AngleNode make_node(double angle) {
    AngleNode n;
    n.angle = angle;
    const double r = angle * kD2R;
    n.c = std::cos(r); n.s = std::sin(r);
    n.cn = std::cos(-r); n.sn = std::sin(-r);
    return n;
}

// ---------------------------------------------------------------------------------------------------------
// plan
// ---------------------------------------------------------------------------------------------------------
bool same_search_params(const fpm_params& a, const fpm_params& b) {
    return a.max_pos == b.max_pos && a.min_reduce_area == b.min_reduce_area && a.max_overlap == b.max_overlap &&
           a.score == b.score && a.tolerance_angle == b.tolerance_angle && a.use_simd == b.use_simd &&
           a.tolerance_range == b.tolerance_range && a.semantics == b.semantics &&
           a.top_angle_step == b.top_angle_step && std::equal(a.tolerance, a.tolerance + 4, b.tolerance);
}

// Input guard of the angle list (TemplateMatcher.cpp:130-144 accumulates `a += step` until the tolerance): a non-finite
// tolerance or step, or a step so small that the list would exceed kMaxTopAngles, is refused up front (the oracle
// applies the same rule) instead of looping without end / growing the list until memory runs out.
constexpr double kMaxTopAngles = 100000;
static bool angle_list_ok(const fpm_params& prm, double step, bool mfc) {
    if (!std::isfinite(step) || step <= 0) return false;
    auto span = [&](double lo, double hi) { return (hi - lo) / step + 2; };
    double n;
    if (mfc && prm.tolerance_range) {
        for (double t : prm.tolerance)
            if (!std::isfinite(t)) return false;
        n = span(prm.tolerance[0], prm.tolerance[1]) + span(prm.tolerance[2], prm.tolerance[3]);
    } else {
        if (!std::isfinite(prm.tolerance_angle)) return false;
        n = prm.tolerance_angle < kVisionTol ? 1 : 2 * span(0, prm.tolerance_angle);
    }
    return n <= kMaxTopAngles;
}

// The matrix-core top layer's plan (k_top_mma): whether it applies, its strip width and row runs
// (work units), the B fragments of the top template level and the candidate-list buffers.  Applies where the template
// level fits the kernel's two MFMA layouts, the layer score is > 0.01 (the greedy peak forms need thr > 0, and the lists
// stay short), there is a pyramid launch to zero the list counters (L >= 1), the level is not flat (ResultEqual1) and
// the greedy form can hold the maps' coverage cells; FPM_TOP_MMA=0 keeps the split / fused kernels (read when the plan is
// built).
int plan_top_mma(fpm_ctx* ctx, Plan& P, const TmplLevel& tt) {
    P.top_mma = false;
    const char* env = getenv("FPM_TOP_MMA");
    if (env && atoi(env) == 0) return FPM_OK;
    const int L = P.L, S = ctx->S, J = S * P.nang;
    const double thr = P.layer_score[L];
    int max_mw = 0, max_mh = 0;
    for (int a = 0; a < P.nang; ++a) { max_mw = std::max(max_mw, P.map_w[a]); max_mh = std::max(max_mh, P.map_h[a]); }
    if (L < 1 || J <= 0 || !top_mma_fits(tt.w, tt.h) || tt.equal1 || !(thr > 0.01) || max_mw <= 0 ||
        std::max(max_mw, max_mh) >= 65536 || P.cap > 256 || P.max_cells > 12 * 1024)
        return FPM_OK;
    // strip width: one strip up to 192 output columns, else the fewest strips of at most 192, evened out
    const int nstrip = (max_mw + kTopMmaMaxSw - 1) / kTopMmaMaxSw;
    const int sw = (((max_mw + nstrip - 1) / nstrip) + 15) / 16 * 16;
    // row runs: the longest (fewer first-band re-samplings of th - 1 rows) that still give >= 2048 units
    std::vector<TopUnit> units;
    int seg = 64;
    for (int cand : {1 << 30, 256, 128, 64}) {
        long n = 0;
        for (int a = 0; a < P.nang; ++a)
            if (P.map_w[a] > 0 && P.map_h[a] > 0)
                n += (long)((P.map_w[a] + sw - 1) / sw) * ((P.map_h[a] + std::min(cand, P.map_h[a]) - 1) /
                                                           std::min(cand, P.map_h[a]));
        seg = cand;
        if (n * S >= 2048) break;
    }
    // plain-peak searches with few work units (< 128 workgroups: a lone Src7 search's 41 small maps make 82) and few
    // peaks per map (MaxPos <= 10, the reference's own s_BlockMax threshold) run faster on the split kernels, whose
    // grids cover the chip: device 0.233 vs 0.248 ms for the lone Src7 search.  Many peaks per map keep the lists, whose
    // greedy pass beats k_nms's painted-rectangle loop even on one map (Src3 / Dst3 at 0 deg, MaxPos 38, 3 units: 0.170
    // vs 0.229 ms), and so do s_BlockMax searches and many-unit sweeps (profiles/r06_lone/); FPM_TOP_MMA=1 keeps the form
    {
        long nunits = 0;
        for (int a = 0; a < P.nang; ++a)
            if (P.map_w[a] > 0 && P.map_h[a] > 0)
                nunits += (long)((P.map_w[a] + sw - 1) / sw) * ((P.map_h[a] + std::min(seg, P.map_h[a]) - 1) /
                                                               std::min(seg, P.map_h[a]));
        if (!(env && atoi(env) == 1) && !P.by_block && ctx->prm.max_pos <= 10 && nunits * S < 128 &&
            ncc_tile_fits(tt.w, tt.h))
            return FPM_OK;
    }
    int max_rows = 0;
    for (int s = 0; s < S; ++s)
        for (int a = 0; a < P.nang; ++a) {
            const int mw = P.map_w[a], mh = P.map_h[a];
            if (mw <= 0 || mh <= 0) continue;
            const int run = std::min(seg, mh);
            for (int x0 = 0; x0 < mw; x0 += sw)
                for (int y0 = 0; y0 < mh; y0 += run) {
                    TopUnit u;
                    u.job = s * P.nang + a; u.x0 = x0; u.y0 = y0; u.y1 = std::min(mh, y0 + run);
                    units.push_back(u);
                    max_rows = std::max(max_rows, u.y1 - u.y0);
                }
        }
    TopMmaArgs& A = P.tma;
    A = TopMmaArgs{};
    A.tw = tt.w; A.th = tt.h; A.area = tt.w * tt.h;
    top_mma_layout(A, sw, max_rows);
    if (top_mma_lds(A) > 160 * 1024 - 1024) return FPM_OK;
    uint32_t tsum = 0;
    for (uint8_t v : tt.px) tsum += v;
    A.tsum = tsum;
    // B fragments: slot q, lane (n = lane & 15, g = lane >> 4), byte i is k = 16 g + i -> template row r, column c - n
    std::vector<int8_t> bf((size_t)A.nq * 64 * 16, 0);
    for (int q = 0; q < A.nq; ++q)
        for (int lane = 0; lane < 64; ++lane)
            for (int i = 0; i < 16; ++i) {
                const int n = lane & 15, g = lane >> 4;
                const int r = A.R == 2 ? 2 * q + (g >> 1) : q;
                const int c = (A.R == 2 ? 16 * (g & 1) : 16 * g) + i - n;
                if (r < tt.h && c >= 0 && c < tt.w)
                    bf[((size_t)q * 64 + lane) * 16 + i] = (int8_t)((int)tt.px[(size_t)r * tt.w + c] - 128);
            }
    const size_t ubytes = ((units.size() * sizeof(TopUnit)) + 255) & ~(size_t)255;
    HIP_TRY(P.d_tmu.ensure(ubytes + bf.size()));
    HIP_TRY(hipMemcpyAsync(P.d_tmu.p, units.data(), units.size() * sizeof(TopUnit), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(P.d_tmu.as<char>(ubytes), bf.data(), bf.size(), hipMemcpyHostToDevice, ctx->stream));
    // candidate lists: s_BlockMax maps share d_ncand with k_nms_blocks' fallback lists (kNmsCandCap per map); plain
    // maps need no more than the greedy form takes
    P.tcand_cap = P.by_block ? kNmsCandCap : 512;
    // FPM_TOP_LIST_CAP=n (tests): lists of n entries, so every map with more candidates takes the fallback path
    if (const char* lc = getenv("FPM_TOP_LIST_CAP"))
        if (atoi(lc) > 0) P.tcand_cap = std::min(P.tcand_cap, atoi(lc));
    HIP_TRY(P.d_ncand.ensure(sizeof(int32_t) * (size_t)P.tcand_cap * J));
    HIP_TRY(P.d_tcandv.ensure(sizeof(float) * (size_t)P.tcand_cap * J));
    A.wjobs = P.d_jobs.as<WarpJob>(P.off_warp);
    A.njobs = P.d_jobs.as<NccJob>(P.off_ncc);
    A.units = P.d_tmu.as<TopUnit>();
    A.nunits = (int)units.size();
    A.bfrag = P.d_tmu.as<uint8_t>(ubytes);
    A.prefilter = A.area <= 258 ? 1 : 0;
    const double tm = thr * (1.0 - 1e-5);
    A.thrK = (float)(tm * tm * tt.norm * tt.norm * (double)A.area);
    A.E = 1024.f;
    A.thr = thr; A.mean = tt.mean; A.norm = tt.norm; A.inv_area = tt.inv_area;
    A.cand = P.d_ncand.as<int32_t>();
    A.cand_val = P.d_tcandv.as<float>();
    A.cand_cap = P.tcand_cap;
    if (!P.by_block) {   // plain maps: the list counters follow the live counts (s_BlockMax plans already zero them)
        P.nzero = L + 2 + J;
        HIP_TRY(P.d_livecnt.ensure(sizeof(int32_t) * (size_t)P.nzero));
    }
    A.cand_cnt = P.d_livecnt.as<int32_t>() + L + 2;
    P.top_mma = true;
    return FPM_OK;
}

int build_plan(fpm_ctx* ctx) {
    Plan& P = ctx->plan;
    const int L = ctx->src_L;
    if (P.valid && ctx->plan_gen == ctx->tmpl_gen && P.sw == ctx->sw && P.sh == ctx->sh && P.S == ctx->S &&
        P.L == L && same_search_params(P.prm, ctx->prm) && P.shard == ctx->shard && P.shards == ctx->shards)
        return FPM_OK;
    P.valid = false;
    P.sw = ctx->sw; P.sh = ctx->sh; P.S = ctx->S; P.L = L; P.prm = ctx->prm;
    P.shard = ctx->shard; P.shards = ctx->shards;
    const fpm_params& prm = ctx->prm;
    const TmplLevel& tt = ctx->tmpl[L];
    // angle list (TemplateMatcher.cpp:130-144); the step override is an extension (fpm_params.top_angle_step)
    const double step = prm.top_angle_step > 0 ? prm.top_angle_step : std::atan(2.0 / std::max(tt.w, tt.h)) * kR2D;
    const bool mfc = prm.semantics == FPM_SEMANTICS_MFC;
    P.angles.clear();
    if (!angle_list_ok(prm, step, mfc)) {   // the reference would loop without end or exhaust memory on these
        ctx->err = "angle list: non-finite tolerance or step, or more than 100000 top-layer angles";
        return FPM_E_INVALID_ARG;
    }
    if (mfc && prm.tolerance_range) {   // MFC angle ranges (MatchToolDlg.cpp:805-815)
        const double* t = prm.tolerance;
        if (t[0] >= t[1] || t[2] >= t[3]) { ctx->err = "angle ranges need tolerance[0] < [1] and [2] < [3]"; return FPM_E_INVALID_ARG; }
        for (double a = t[0]; a < t[1] + step; a += step) P.angles.push_back(a);
        for (double a = t[2]; a < t[3] + step; a += step) P.angles.push_back(a);
    } else if (prm.tolerance_angle < kVisionTol) {
        P.angles.push_back(0.0);
    } else {
        for (double a = 0; a < prm.tolerance_angle + step; a += step) P.angles.push_back(a);
        for (double a = -step; a > -prm.tolerance_angle - step; a -= step) P.angles.push_back(a);
    }
    // angle shard: a contiguous block [a0, a1) of the reference's list, so the concatenation of the shards' candidate
    // lists in shard order is the reference's push order (angle-major, TemplateMatcher.cpp:157-211)
    P.nang_all = (int)P.angles.size();
    P.a0 = (int)((int64_t)P.nang_all * P.shard / P.shards);
    const int a1 = (int)((int64_t)P.nang_all * (P.shard + 1) / P.shards);
    P.angles = std::vector<double>(P.angles.begin() + P.a0, P.angles.begin() + a1);
    P.nang = (int)P.angles.size();
    P.layer_score.assign(L + 1, prm.score);
    for (int l = 1; l <= L; ++l) P.layer_score[l] = P.layer_score[l - 1] * 0.9;
    const SrcLevel& top = ctx->src[L];
    P.center = f2((top.w - 1) / 2.0f, (top.h - 1) / 2.0f);
    P.by_block = ((top.w * top.h) / (tt.w * tt.h) > 500) && prm.max_pos > 10;
    P.cap = std::max(prm.max_pos + kMatchCandidateNum, 1);
    P.n3 = (prm.tolerance_range || prm.tolerance_angle >= kVisionTol) ? 3 : 1;
    P.C = ctx->S * P.nang * P.cap;
    // per-angle canvas geometry (TemplateMatcher.cpp:163-175)
    P.top.resize(P.nang);
    P.top_nodes.resize(P.nang);
    P.canvas_off.resize(P.nang); P.map_off.resize(P.nang); P.blk_off.resize(P.nang);
    P.canvas_pitch.resize(P.nang); P.map_w.resize(P.nang); P.map_h.resize(P.nang); P.nblk.resize(P.nang);
    std::vector<std::array<double, 6>> mats(P.nang);
    size_t co = 0, mo = 0, bo = 0;
    P.max_canvas = 0; P.max_map = 0; P.max_nblk = 0; P.max_cells = 0; P.max_nitems = 0;
    for (int a = 0; a < P.nang; ++a) {
        int bw, bh;
        best_rotation_size(top.w, top.h, tt.w, tt.h, P.angles[a], &bw, &bh);
        TopAngle& ta = P.top[a];
        ta.bw = bw; ta.bh = bh;
        ta.tx = (bw - 1) / 2.0f - P.center.x;
        ta.ty = (bh - 1) / 2.0f - P.center.y;
        const double r = P.angles[a] * kD2R;
        double m[6];
        rotation_matrix(P.center, std::cos(r), std::sin(r), m);
        m[2] += ta.tx;
        m[5] += ta.ty;
        invert_affine(m);
        std::copy(m, m + 6, mats[a].begin());
        P.top_nodes[a] = make_node(P.angles[a]);
        const bool ok = bw >= tt.w && bh >= tt.h && bw > 0 && bh > 0;
        P.canvas_pitch[a] = round_up(std::max(bw, 1), 64);
        P.canvas_off[a] = co;
        co += round_up((size_t)P.canvas_pitch[a] * std::max(bh, 1), (size_t)256);
        P.map_w[a] = ok ? bw - tt.w + 1 : 0;
        P.map_h[a] = ok ? bh - tt.h + 1 : 0;
        P.map_off[a] = mo;
        mo += round_up((size_t)P.map_w[a] * P.map_h[a], (size_t)64);
        int nb = 0;
        if (P.by_block && ok) {   // s_BlockMax blocks (BlockGeom in fpm_kernels.hip: Qt or MFC layout)
            const int bw = mfc ? 2 * tt.w : tt.w, bh = mfc ? 2 * tt.h : tt.h;
            const int ncol = P.map_w[a] / bw, nrow = P.map_h[a] / bh;
            const int rw = P.map_w[a] - ncol * bw, rh = P.map_h[a] - nrow * bh;
            if (!mfc) nb = ncol * nrow + (rw > 0) + (rh > 0) + (rw > 0 && rh > 0);
            else nb = (ncol == 0 || nrow == 0) ? 0 : ncol * nrow + ((rw > 0 && rh > 0) ? 2 : 1);
            P.max_nitems = std::max(P.max_nitems, nms_block_items(P.map_w[a], P.map_h[a], tt.w, tt.h, mfc ? 1 : 0));
        }
        if (ok)   // coverage cells of the greedy peak forms (k_nms_greedy), plain and s_BlockMax alike
            P.max_cells = std::max(P.max_cells, ((P.map_w[a] + tt.w - 1) / tt.w) * ((P.map_h[a] + tt.h - 1) / tt.h));
        P.nblk[a] = nb;
        P.max_nblk = std::max(P.max_nblk, nb);
        P.blk_off[a] = bo;
        bo += round_up((size_t)nb, (size_t)64);
        P.max_canvas = std::max(P.max_canvas, bw * bh);
        P.max_map = std::max(P.max_map, P.map_w[a] * P.map_h[a]);
    }
    P.canvas_bytes = co; P.map_floats = mo; P.blk_count = bo;
    // refinement angle tree: level d has nang * n3^(d+1) nodes (TemplateMatcher.cpp:282-298)
    P.nodes.assign(L, {});
    P.node_off.assign(L, 0);
    size_t noff = 0;
    for (int d = 0; d < L; ++d) {
        const int layer = L - 1 - d;
        const double astep = std::atan(2.0 / std::max(ctx->tmpl[layer].w, ctx->tmpl[layer].h)) * kR2D;
        const size_t parents = d == 0 ? (size_t)P.nang : P.nodes[d - 1].size();
        std::vector<AngleNode>& lv = P.nodes[d];
        lv.resize(parents * P.n3);
        for (size_t p = 0; p < parents; ++p) {
            const double matched = d == 0 ? P.angles[p] : P.nodes[d - 1][p].angle;
            for (int j = 0; j < P.n3; ++j) {
                double ang;
                if (P.n3 == 1) ang = 0.0;
                else ang = matched + astep * (j - 1);
                lv[p * P.n3 + j] = make_node(ang);
            }
        }
        P.node_off[d] = noff;
        noff += lv.size();
    }
    // device buffers
    const int S = ctx->S, J = S * P.nang;
    HIP_TRY(P.d_canvas.ensure(P.canvas_bytes * S));
    HIP_TRY(P.d_map.ensure(sizeof(float) * P.map_floats * S));
    HIP_TRY(P.d_bmax.ensure(sizeof(float) * std::max<size_t>(P.blk_count, 1) * S));
    HIP_TRY(P.d_bloc.ensure(sizeof(int32_t) * std::max<size_t>(P.blk_count, 1) * S));
    P.off_warp = 0;
    P.off_ncc = round_up(sizeof(WarpJob) * J, (size_t)256);
    P.off_nms = P.off_ncc + round_up(sizeof(NccJob) * J, (size_t)256);
    P.off_order = P.off_nms + round_up(sizeof(NmsJob) * J, (size_t)256);
    HIP_TRY(P.d_jobs.ensure(P.off_order + sizeof(int32_t) * J));
    HIP_TRY(P.d_nodes.ensure(sizeof(AngleNode) * std::max<size_t>(noff, 1)));
    HIP_TRY(P.d_top.ensure(sizeof(TopAngle) * P.nang));
    HIP_TRY(P.d_topn.ensure(sizeof(AngleNode) * P.nang));
    HIP_TRY(P.d_peaks.ensure(sizeof(Peak) * (size_t)P.C));
    HIP_TRY(P.d_counts.ensure(sizeof(int32_t) * J));
    if (P.by_block) HIP_TRY(P.d_ncand.ensure(sizeof(int32_t) * (size_t)kNmsCandCap * J));
    HIP_TRY(P.d_state.ensure(sizeof(CandState) * (size_t)P.C));
    HIP_TRY(P.d_live.ensure(sizeof(int32_t) * (size_t)P.C * 2));
    // live counts [L + 2], then (s_BlockMax) the per-map candidate counts [J]: zeroed together by k_warp
    // (s_BlockMax) then the strip-block keys [J][3] (u64, 8-aligned) and chunk counts [J][3] of k_nms_blocks
    P.off_skey = round_up(L + 2 + J, 2);
    P.nzero = L + 2 + (P.by_block ? P.off_skey - (L + 2) + 9 * J : 0);
    HIP_TRY(P.d_livecnt.ensure(sizeof(int32_t) * (size_t)P.nzero));
    HIP_TRY(P.d_rec.ensure(sizeof(RoiRecord) * (size_t)P.C * P.n3));
    // the prologue-stepped run of small layers (below) alternates state and records between two buffers each
    HIP_TRY(P.d_state2.ensure(sizeof(CandState) * (size_t)P.C));
    HIP_TRY(P.d_rec2.ensure(sizeof(RoiRecord) * (size_t)P.C * P.n3));
    {   // refinement scratch per ROI (tables, sampled ROI, row sums, window partials); bounded, rounds cover the rest
        size_t max_rows = 1, max_chunks = 1;
        int max_w = 1;
        P.tdesc_stride = 1;
        for (int l = 0; l < L; ++l) {
            P.tdesc_stride = std::max(P.tdesc_stride, roi_tiles_for(ctx->tmpl[l].w, ctx->tmpl[l].h));
            const int rc = roi_pick_rc(ctx->tmpl[l].w, ctx->tmpl[l].h);
            max_rows = std::max(max_rows, (size_t)ctx->tmpl[l].h);
            max_chunks = std::max(max_chunks, (size_t)(ctx->tmpl[l].h + rc - 1) / rc);
            max_w = std::max(max_w, ctx->tmpl[l].w);
        }
        P.roi_pitch = roi_pitch_for(max_w);
        P.tabw = P.roi_pitch;
        P.tabh = roi_tab_rows((int)max_rows);
        P.roi_stride = 0;
        for (int l = 0; l < L; ++l)
            P.roi_stride = std::max(P.roi_stride, roi_tiles_bytes(ctx->tmpl[l].w, ctx->tmpl[l].h));
        const size_t per_roi = sizeof(int32_t) * 2 * (P.tabw + P.tabh) + sizeof(int4) * P.tdesc_stride + P.roi_stride + max_rows * 49 * 4 +
                               max_chunks * 49 * 12;
        // slots are sized for the worst case (every top candidate alive at every layer) so the captured graph needs
        // no host round trip; up to a sixth of the free HBM (<= 48 GB of 288; FPM_SCRATCH_MB caps it) holds them,
        // rounds only beyond that.  A floor of min(4 GB, half the free HBM) keeps a batch in few rounds when another
        // allocator in the process holds most of the device; an allocation failure halves the slots (more rounds)
        // instead of failing the search.
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = (size_t)16 << 30;
        size_t budget = std::min((size_t)48 << 30, std::max(std::min((size_t)4 << 30, free_b / 2), free_b / 6));
        if (const char* e = getenv("FPM_SCRATCH_MB")) {
            const long mb = atol(e);
            if (mb > 0) budget = std::min(budget, (size_t)mb << 20);
        }
        const size_t want = (size_t)P.C * P.n3;
        // rounds hold whole candidates (k_roi_eval steps a candidate from its n3 records)
        P.slot_cap = (int)std::max<size_t>((size_t)P.n3, std::min(want, budget / per_roi) / P.n3 * P.n3);
        for (;;) {
            hipError_t e = P.d_tab.ensure((size_t)P.slot_cap * 2 * (P.tabw + P.tabh) * sizeof(int32_t));
            if (e == hipSuccess) e = P.d_tdesc.ensure((size_t)P.slot_cap * P.tdesc_stride * sizeof(int4));
            if (e == hipSuccess) e = P.d_roi.ensure((size_t)P.slot_cap * P.roi_stride);
            if (e == hipSuccess) e = P.d_rowsum.ensure((size_t)P.slot_cap * round_up(max_rows * 49, (size_t)4) * 4);
            if (e == hipSuccess) e = P.d_wsum.ensure((size_t)P.slot_cap * max_chunks * 49 * 4);
            if (e == hipSuccess) e = P.d_wsq.ensure((size_t)P.slot_cap * max_chunks * 49 * 8);
            if (e == hipSuccess) break;
            (void)hipGetLastError();   // clear the sticky allocation error
            if (e != hipErrorOutOfMemory || P.slot_cap <= P.n3) HIP_TRY(e);
            P.d_tab.release(); P.d_tdesc.release(); P.d_roi.release();
            P.d_rowsum.release(); P.d_wsum.release(); P.d_wsq.release();
            P.slot_cap = std::max(P.n3, P.slot_cap / 2 / P.n3 * P.n3);
        }
    }
    // job tables
    std::vector<WarpJob> wj(J);
    std::vector<NccJob> nj(J);
    std::vector<NmsJob> mj(J);
    const uint8_t* dsrc = ctx->d_src.as<uint8_t>();
    for (int s = 0; s < S; ++s)
        for (int a = 0; a < P.nang; ++a) {
            const int k = s * P.nang + a;
            uint8_t* canvas = P.d_canvas.as<uint8_t>() + P.canvas_bytes * s + P.canvas_off[a];
            float* map = P.d_map.as<float>() + P.map_floats * s + P.map_off[a];
            WarpJob& w = wj[k];
            w.src = dsrc + top.off + top.img_bytes * s;
            w.sw = top.w; w.sh = top.h; w.sp = top.pitch;
            w.dst = canvas;
            w.dw = P.top[a].bw; w.dh = P.top[a].bh; w.dp = P.canvas_pitch[a];
            w.border = ctx->border;
            w.pad = 0;
            std::copy(mats[a].begin(), mats[a].end(), w.M);
            NccJob& n = nj[k];
            n.img = canvas; n.iw = w.dw; n.ih = w.dh; n.ip = w.dp;
            n.tmpl = ctx->d_tmpl.as<uint8_t>() + tt.off; n.tw = tt.w; n.th = tt.h; n.tp = tt.pitch;
            n.out = map; n.ow = P.map_w[a]; n.oh = P.map_h[a];
            n.fold = 0;   // top layer: cv::matchTemplate(TM_CCORR) (:177 -> :514)
            n.equal1 = tt.equal1 ? 1 : 0;
            n.mean = tt.mean; n.norm = tt.norm; n.inv_area = tt.inv_area;
            NmsJob& m = mj[k];
            m.map = map; m.mw = P.map_w[a]; m.mh = P.map_h[a];
            m.bmax = P.d_bmax.as<float>() + P.blk_count * s + P.blk_off[a];
            m.bloc = P.d_bloc.as<int32_t>() + P.blk_count * s + P.blk_off[a];
        }
    HIP_TRY(hipMemcpyAsync(P.d_jobs.as<char>(P.off_warp), wj.data(), sizeof(WarpJob) * J, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(P.d_jobs.as<char>(P.off_ncc), nj.data(), sizeof(NccJob) * J, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(P.d_jobs.as<char>(P.off_nms), mj.data(), sizeof(NmsJob) * J, hipMemcpyHostToDevice, ctx->stream));
    {
        const int rc = plan_top_mma(ctx, P, tt);
        if (rc != FPM_OK) return rc;
    }
    {   // k_top_fused's workgroup -> job order: the angles with the largest map x template work first, every source's
        // job of an angle together (one launch covers S x nang jobs in ~1.4 rounds of resident workgroups at Src7: the
        // cheap jobs fill the last round); a scheduling choice only, every job writes its own outputs
        std::vector<int> ang(P.nang);
        for (int a = 0; a < P.nang; ++a) ang[a] = a;
        auto cost = [&](int a) {
            return (double)P.map_w[a] * P.map_h[a] * tt.w * tt.h + (double)P.top[a].bw * P.top[a].bh;
        };
        std::stable_sort(ang.begin(), ang.end(), [&](int x, int y) { return cost(x) > cost(y); });
        P.order.resize(J);
        for (int i = 0; i < P.nang; ++i)
            for (int s = 0; s < S; ++s) P.order[(size_t)i * S + s] = s * P.nang + ang[i];
        HIP_TRY(hipMemcpyAsync(P.d_jobs.as<char>(P.off_order), P.order.data(), sizeof(int32_t) * J,
                               hipMemcpyHostToDevice, ctx->stream));
    }
    for (int d = 0; d < L; ++d)
        HIP_TRY(hipMemcpyAsync(P.d_nodes.as<AngleNode>() + P.node_off[d], P.nodes[d].data(),
                               sizeof(AngleNode) * P.nodes[d].size(), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(P.d_top.p, P.top.data(), sizeof(TopAngle) * P.nang, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(P.d_topn.p, P.top_nodes.data(), sizeof(AngleNode) * P.nang, hipMemcpyHostToDevice, ctx->stream));
    // pinned host buffer written by k_pack: counts | peaks | live counts | layer-0 ids | states | records
    P.h_counts = 0;
    P.h_peaks = round_up(sizeof(int32_t) * J, (size_t)256);
    P.h_live = P.h_peaks + round_up(sizeof(Peak) * (size_t)P.C, (size_t)256);
    P.h_live0 = P.h_live + round_up(sizeof(int32_t) * (L + 2), (size_t)256);
    P.h_state = P.h_live0 + round_up(sizeof(int32_t) * (size_t)P.C, (size_t)256);
    P.h_rec = P.h_state + round_up(sizeof(CandState) * (size_t)P.C, (size_t)256);
    P.h_total = P.h_rec + sizeof(RoiRecord) * (size_t)P.C * P.n3;
    HIP_TRY(P.h_out.ensure(P.h_total));
    {
        void* dp = nullptr;
        HIP_TRY(hipHostGetDevicePointer(&dp, P.h_out.p, 0));
        P.h_dev = (char*)dp;
    }
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    P.valid = true;
    ctx->plan_gen = ctx->tmpl_gen;
    ctx->plan_builds++;
    return FPM_OK;
}

// ---------------------------------------------------------------------------------------------------------
// sources
// ---------------------------------------------------------------------------------------------------------
int layout_sources(fpm_ctx* ctx, int count, int w, int h) {
    const int L = top_layer(ctx->tmpl[0].w, ctx->tmpl[0].h, (int)std::sqrt((double)ctx->prm.min_reduce_area));
    if (L >= (int)ctx->tmpl.size()) {
        ctx->err = "MinReduceArea changed after learnPattern: template pyramid too shallow";
        return FPM_E_INVALID_ARG;
    }
    ctx->S = count; ctx->sw = w; ctx->sh = h; ctx->src_L = L;
    ctx->src.assign(L + 1, {});
    size_t off = 0;
    int lw = w, lh = h;
    for (int l = 0; l <= L; ++l) {
        SrcLevel& s = ctx->src[l];
        s.w = lw; s.h = lh;
        s.pitch = round_up(lw + 4, 64);          // +4: aligned dword over-reads stay in the row
        s.img_bytes = round_up((size_t)s.pitch * (lh + 1), (size_t)256);
        s.off = off;
        off += s.img_bytes * count;
        lw = (lw + 1) / 2;
        lh = (lh + 1) / 2;
    }
    // slack: the ROI sampler's footprint staging reads whole 16-row groups, up to 15 rows past a box (k_roi_warp3),
    // i.e. past the last image's spare row
    HIP_TRY(ctx->d_src.ensure(off + 16 * (size_t)ctx->src[0].pitch + 256));
    return FPM_OK;
}

int check_sizes(fpm_ctx* ctx, int w, int h) {   // TemplateMatcher.cpp:99-114
    if (!ctx->learned) { ctx->err = "template not learned"; return FPM_E_NOT_LEARNED; }
    const TmplLevel& t = ctx->tmpl[0];
    if ((t.w < w && t.h > h) || (t.w > w && t.h < h)) { ctx->err = "template/source orientation mismatch"; return FPM_E_SIZE; }
    if ((int64_t)t.w * t.h > (int64_t)w * h) { ctx->err = "template larger than source"; return FPM_E_SIZE; }
    return FPM_OK;
}

// ---------------------------------------------------------------------------------------------------------
// search
// ---------------------------------------------------------------------------------------------------------
constexpr int kPrologueMaxSources = 2;            // step prologue of the small layers up to this batch size
constexpr int64_t kPyr2MaxBytes = 16ll << 20;     // two-level pyramid launches up to this many input bytes

int enqueue_search(fpm_ctx* ctx) {
    Plan& P = ctx->plan;
    const int L = P.L, S = P.S, J = S * P.nang;
    hipStream_t st = ctx->stream;
    uint8_t* dsrc = ctx->d_src.as<uint8_t>();
    const SrcLevel& top = ctx->src[L];
    const TmplLevel& tt = ctx->tmpl[L];
    P.step_layers = 0;   // (set again by the launches recorded below)
    P.top_lists = false;
    // small canvases with the plain peak path: the whole top layer as one kernel (k_top_fused), canvas and map in
    // LDS, when there are enough (source, angle) jobs to fill the chip: one workgroup runs a job's warp, map and
    // peak loop serially (33 us for a single Src7 source's 41 jobs against 24 us for the three split kernels; 75.5
    // against 106.4 us at 1763 jobs, profiles/r02_z/lat_r02_z.txt).  FPM_TOP_FUSED=0 keeps the three-kernel form,
    // FPM_TOP_FUSED=1 forces the fused one whatever the job count (tests, profiling comparisons)
    size_t fused_lds = 0;
    const char* top_env = getenv("FPM_TOP_FUSED");   // read when the search is recorded (once per plan)
    const int top_mode = top_env ? atoi(top_env) : -1;
    if (!P.by_block && ncc_tile_fits(tt.w, tt.h) && J > 0 && (J >= kTopFusedMinJobs || top_mode == 1)) {
        for (int a = 0; a < P.nang; ++a)
            fused_lds = std::max(fused_lds, top_fused_lds(P.top[a].bw, P.top[a].bh, tt.w, tt.h));
        // the dynamic LDS plus the kernel's static arrays (peaks, reduction slots, as compiled) within the default 64 KB
        // launch limit (tests/test_gpu_parity.py::test_top_fused_lds_threshold runs canvases either side of it)
        if (top_mode == 0 || fused_lds > top_fused_lds_limit()) fused_lds = 0;
    }
    // the matrix-core top layer (k_top_mma + greedy peaks from its lists) where the plan admits it, except where the
    // fused small-canvas kernel applies; FPM_TOP_MMA=1 takes it there too (read when the search is recorded)
    const char* mma_env = getenv("FPM_TOP_MMA");
    const bool use_mma = P.top_mma && (fused_lds == 0 || (mma_env && atoi(mma_env) == 1));
    if (use_mma) fused_lds = 0;
    int32_t* live[2] = {P.d_live.as<int32_t>(), P.d_live.as<int32_t>() + P.C};
    int32_t* livecnt = P.d_livecnt.as<int32_t>();
    CandInitArgs ca;   // the top peaks -> candidate states and the first live list (k_cand_init, or fused in k_nms)
    ca.peaks = P.d_peaks.as<Peak>();
    ca.counts = P.d_counts.as<int32_t>();
    ca.angles = P.d_top.as<TopAngle>();
    ca.top_nodes = P.d_topn.as<AngleNode>();
    ca.state = P.d_state.as<CandState>();
    ca.live = live[0];
    ca.live_count = livecnt + 0;
    ca.nang = P.nang; ca.cap = P.cap; ca.total = P.C;
    ca.center = P.center;
    ca.refine = L > 0 ? (L == 1 ? 2 : 1) : 0;
    bool cand_fused = false;
    // the fused top layer also initialises the candidates (cand_init_job) when the peaks fit its LDS list; its
    // live-list atomics then need the counters zeroed by an earlier launch: the first pyramid level's
    const bool top_init = fused_lds > 0 && P.cap <= kNmsInitCap && (size_t)J * P.cap == (size_t)P.C;
    // L >= 1: the first pyrDown launch zeroes the counters before the top kernel's live-list atomics.  L == 0: no
    // pyramid launch precedes it, so its block 0 zeroes them -- safe only because the candidate init then runs in
    // mode 1 (refine == 0: states and live list written directly, no live-count atomics); launch_top_fused checks it
    const bool pyr_zero = (top_init && L >= 1) || use_mma;   // (use_mma implies L >= 1: plan_top_mma)
    // K1: source pyramid (all staged sources per launch).  Two levels per launch (k_pyr_down2) where the pair's input
    // is small (<= kPyr2MaxBytes over the batch: launch-bound levels, e.g. every pair of a single Src7 search: 14.8 ->
    // 11.3 us for levels 0-2), else one level per launch (k_pyr_down_s keeps more workgroups in flight: 43 Src7 levels
    // 0-2 in 197 us vs 217-258 us, profiles/r04/mb32_r04g.txt).  FPM_PYR2=0 / 1 forces one form.
    const char* pyr2_env = getenv("FPM_PYR2");
    const int pyr2_mode = pyr2_env ? atoi(pyr2_env) : -1;
    for (int l = 1; l <= L;) {
        const SrcLevel& a = ctx->src[l - 1];
        const SrcLevel& b = ctx->src[l];
        int32_t* zero = l == 1 && pyr_zero ? P.d_livecnt.as<int32_t>() : nullptr;
        const int nzero = l == 1 && pyr_zero ? P.nzero : 0;
        const int64_t in_bytes = (int64_t)S * a.w * a.h;
        const bool two = l + 1 <= L && (pyr2_mode >= 0 ? pyr2_mode != 0 : in_bytes <= kPyr2MaxBytes);
        const SrcLevel& c = ctx->src[two ? l + 1 : l];
        l += two ? 2 : 1;
        if (two) {
            ProfScope ps(ctx, FPM_K_PYR, (int64_t)S * ((int64_t)a.w * a.h + (int64_t)b.w * b.h + (int64_t)c.w * c.h));
            launch_pyr_down2(dsrc + a.off, a.w, a.h, a.pitch, a.img_bytes, dsrc + b.off, b.w, b.h, b.pitch, b.img_bytes,
                             dsrc + c.off, c.w, c.h, c.pitch, c.img_bytes, S, st, 0, zero, nzero);
        } else {
            ProfScope ps(ctx, FPM_K_PYR, (int64_t)S * ((int64_t)a.w * a.h + (int64_t)b.w * b.h));
            launch_pyr_down(dsrc + a.off, a.w, a.h, a.pitch, a.img_bytes, dsrc + b.off, b.w, b.h, b.pitch, b.img_bytes, S,
                            st, 0, zero, nzero);
        }
    }
    NmsArgs na{};
    na.jobs = P.d_jobs.as<NmsJob>(P.off_nms);
    na.peaks = P.d_peaks.as<Peak>();
    na.counts = P.d_counts.as<int32_t>();
    na.tw = tt.w; na.th = tt.h; na.cap = P.cap; na.by_block = P.by_block ? 1 : 0;
    na.mfc = ctx->prm.semantics == FPM_SEMANTICS_MFC ? 1 : 0;
    na.thr = P.layer_score[L]; na.overlap = ctx->prm.max_overlap;
    na.lds_blocks = 0;
    na.cand = nullptr; na.cand_cnt = nullptr; na.cand_cap = 0; na.cand_lds = 0; na.stamps = nullptr;
    na.skey = nullptr; na.sdone = nullptr;
    if (fused_lds > 0) {
        int64_t bytes = (int64_t)P.nang * top.w * top.h;
        for (int a = 0; a < P.nang; ++a) bytes += 4LL * P.map_w[a] * P.map_h[a];
        ProfScope ps(ctx, FPM_K_TOP_NCC, bytes * S);
        launch_top_fused(P.d_jobs.as<WarpJob>(P.off_warp), P.d_jobs.as<NccJob>(P.off_ncc), na, J, fused_lds,
                         pyr_zero ? nullptr : P.d_livecnt.as<int32_t>(), pyr_zero ? 0 : P.nzero, st,
                         top_init ? &ca : nullptr, P.d_jobs.as<int32_t>(P.off_order));
        cand_fused = top_init;
    }
    if (use_mma) {
        int mdim = 0;
        long mpx = 0;
        for (int a = 0; a < P.nang; ++a) {
            mdim = std::max(mdim, std::max(P.map_w[a], P.map_h[a]));
            mpx = std::max(mpx, (long)P.map_w[a] * P.map_h[a]);
        }
        TopMmaArgs ta = P.tma;
        {   // canvases, correlation, scores and the lists of outputs >= the layer score; profiling bytes: the top level
            // read per angle (its share of B_top; the map is never written)
            ProfScope ps(ctx, FPM_K_TOP_NCC, (int64_t)S * P.nang * top.w * top.h);
            ta.mode = 0;
            launch_top_mma(ta, st);
        }
        const bool ci_ok = !P.by_block && P.cap <= kNmsInitCap && (size_t)J * P.cap == (size_t)P.C;
        NmsArgs ga = na;
        ga.cand = P.d_ncand.as<int32_t>(); ga.cand_val = P.d_tcandv.as<float>();
        ga.cand_cnt = ta.cand_cnt; ga.cand_cap = P.tcand_cap;
        ga.reset_untaken = P.by_block ? 1 : 0;
        {   // (its bytes, the map term of B_top the lists stand in for, are added when the pass completes)
            ProfScope ps(ctx, FPM_K_TOP_NMS, 0);
            launch_top_greedy(ga, J, P.max_cells, st, ci_ok ? &ca : nullptr);
        }
        P.top_lists = true;
        {   // the maps the lists could not give (overflow, or a shape the greedy form does not take): full maps
            ProfScope ps(ctx, FPM_K_TOP_MAP, 0);
            ta.mode = 1;
            launch_top_mma(ta, st);
        }
        {   // ... and their peaks by the split kernels, which skip the maps the greedy form took (cand_cnt < 0)
            ProfScope ps(ctx, FPM_K_TOP_NMS, 0);
            NmsArgs fa = na;
            fa.cand = ga.cand; fa.cand_cnt = ga.cand_cnt; fa.cand_cap = P.tcand_cap;
            if (P.by_block) {
                fa.skey = (uint64_t*)(P.d_livecnt.as<int32_t>() + P.off_skey);
                fa.sdone = P.d_livecnt.as<int32_t>() + P.off_skey + 6 * J;
            }
            launch_nms(fa, J, P.max_nblk, mdim, P.max_cells, st, P.max_nitems, ci_ok ? &ca : nullptr, mpx);
        }
        cand_fused = ci_ok;
    }
    // profiling bytes: each kernel's share of §8(d)'s B_top = sum_angles (W_L H_L + 4 |R_a|): the rotation reads the
    // top level, the correlation writes the map (the rotated canvases are this design's scratch)
    if (fused_lds == 0 && !use_mma) {
        const int64_t bytes = (int64_t)P.nang * top.w * top.h;
        ProfScope ps(ctx, FPM_K_TOP_WARP, bytes * S);
        launch_warp(P.d_jobs.as<WarpJob>(P.off_warp), J, P.max_canvas, st, P.d_livecnt.as<int32_t>(), P.nzero);
    }
    if (fused_lds == 0 && !use_mma) {
        int64_t bytes = 0;
        for (int a = 0; a < P.nang; ++a) bytes += 4LL * P.map_w[a] * P.map_h[a];
        ProfScope ps(ctx, FPM_K_TOP_NCC, bytes * S);
        if (ncc_tile_fits(tt.w, tt.h)) {
            int mw = 0, mh = 0;
            for (int a = 0; a < P.nang; ++a) { mw = std::max(mw, P.map_w[a]); mh = std::max(mh, P.map_h[a]); }
            launch_ncc_tile(P.d_jobs.as<NccJob>(P.off_ncc), J, mw, mh, tt.w, tt.h, st);
        } else {
            launch_ncc_map(P.d_jobs.as<NccJob>(P.off_ncc), J, P.max_map, tt.w * tt.h, st);
        }
    }
    if (fused_lds == 0 && !use_mma) {
        ProfScope ps(ctx, FPM_K_TOP_NMS, 0);   // (reads the maps counted once in B_top)
        if (P.by_block) {   // (the counts and strip keys were zeroed by k_warp)
            na.cand = P.d_ncand.as<int32_t>(); na.cand_cnt = P.d_livecnt.as<int32_t>() + L + 2; na.cand_cap = kNmsCandCap;
            na.skey = (uint64_t*)(P.d_livecnt.as<int32_t>() + P.off_skey);
            na.sdone = P.d_livecnt.as<int32_t>() + P.off_skey + 6 * J;
        }
        int mdim = 0;
        long mpx = 0;
        for (int a = 0; a < P.nang; ++a) {
            mdim = std::max(mdim, std::max(P.map_w[a], P.map_h[a]));
            mpx = std::max(mpx, (long)P.map_w[a] * P.map_h[a]);
        }
        // plain path: k_nms also initialises the candidates (the live counter was zeroed by k_warp)
        cand_fused = !P.by_block && P.cap <= kNmsInitCap && (size_t)J * P.cap == (size_t)P.C;
        launch_nms(na, J, P.max_nblk, mdim, P.max_cells, st, P.max_nitems, cand_fused ? &ca : nullptr, mpx);
    }
    if (!cand_fused) {
        ProfScope ps(ctx, FPM_K_CAND_INIT, 0);
        launch_cand_init(ca, st);
    }
    // the prologue-stepped run: layers L-1 .. run_end, the leading small layers above layer 0 (none of them a
    // matResult = 1 layer).  From its second layer on, a layer's k_roi_small steps the previous layer's candidates in
    // its prologue over the unchanged live list (k_cand_step launches saved: run length - 1); one k_cand_step after
    // the run's last layer steps and compacts.  FPM_STEP_PROLOGUE=0 keeps one k_cand_step per layer (result-neutral).
    // Used for batches of at most kPrologueMaxSources sources, where the saved launches outweigh the prologue's
    // dependent loads on every workgroup's critical path (single Src7 search: 23 dispatches, 236.8 us of kernels vs
    // 25 and 244.6; a 43-source batch: k_roi_small 181 -> 218 us per pass, profiles/r04/gpu_r04g).
    // FPM_STEP_PROLOGUE=1 forces it, =0 disables it (read when the search is recorded, once per plan).
    const char* prol_env = getenv("FPM_STEP_PROLOGUE");
    const bool step_prologue = prol_env ? atoi(prol_env) != 0 : S <= kPrologueMaxSources;
    int run_end = L;
    if (step_prologue)
        for (int l = L - 1; l >= 1; --l) {
            if (!roi_small_fits(ctx->tmpl[l].w, ctx->tmpl[l].h) || ctx->tmpl[l].equal1) break;
            run_end = l;
        }
    if (L - run_end < 2) run_end = L;   // a run of one layer has no prologue to fuse
    CandState* const state_buf[2] = {P.d_state.as<CandState>(), P.d_state2.as<CandState>()};
    RoiRecord* const rec_buf[2] = {P.d_rec.as<RoiRecord>(), P.d_rec2.as<RoiRecord>()};
    int cur_list = 0;   // live[cur_list]: the list the layer's ROIs come from; its count is livecnt[list_cnt]
    int list_cnt = 0;
    int run_k = 0;      // layers of the run done
    // the next layer's warp tables written by the step of this layer (RoiArgs::nt_tab): where that layer takes tables
    // (not small, not equal1) and every layer runs as one round; FPM_STEP_TABLES=0 keeps the k_roi_tables launches
    // (result-neutral: the same pure functions of the stepped state)
    const char* stab_env = getenv("FPM_STEP_TABLES");
    const bool step_tables = (stab_env ? atoi(stab_env) != 0 : true) && (size_t)P.C * P.n3 <= (size_t)P.slot_cap;
    bool tables_done = false;   // this layer's tables were written by the previous layer's step
    for (int l = L - 1; l >= 0; --l) {
        const int d = L - 1 - l;
        const SrcLevel& lv = ctx->src[l];
        const TmplLevel& tl = ctx->tmpl[l];
        const bool in_run = l >= run_end;
        RoiArgs ra{};
        ra.level = dsrc + lv.off; ra.level_stride = lv.img_bytes;
        ra.W = lv.w; ra.H = lv.h; ra.P = lv.pitch;
        ra.tmpl = ctx->d_tmpl.as<uint8_t>() + tl.off; ra.tw = tl.w; ra.th = tl.h; ra.tp = tl.pitch;
        ra.tmpl8 = ctx->d_tmpl8.as<int8_t>() + tl.off8; ra.tp8 = tl.p8; ra.nk = (tl.w + 63) / 64;
        ra.tsum = ctx->d_tsum.as<int32_t>() + tl.tsum_off;
        ra.n3 = P.n3;
        ra.rc = roi_pick_rc(tl.w, tl.h);
        ra.nchunk = (tl.h + ra.rc - 1) / ra.rc;
        ra.fold = ctx->prm.use_simd ? 1 : 0;
        ra.equal1 = tl.equal1 ? 1 : 0;
        ra.per_source = P.nang * P.cap;
        ra.mean = tl.mean; ra.norm = tl.norm; ra.inv_area = tl.inv_area;
        ra.live = live[cur_list];
        ra.live_count = livecnt + list_cnt;
        ra.state = P.d_state.as<CandState>();
        ra.nodes = P.d_nodes.as<AngleNode>() + P.node_off[d];
        // per-level scratch geometry (the buffers are sized for the largest level)
        ra.tab = P.d_tab.as<int32_t>(); ra.tabw = roi_pitch_for(tl.w); ra.tabh = roi_tab_rows(tl.h);
        ra.tdesc = P.d_tdesc.as<int4>(); ra.tdesc_stride = P.tdesc_stride;
        ra.roi = P.d_roi.as<uint8_t>(); ra.roi_pitch = roi_pitch_for(tl.w); ra.roi_stride = P.roi_stride;
        ra.rowsum = P.d_rowsum.as<uint32_t>();
        ra.wsum = P.d_wsum.as<uint32_t>();
        ra.wsq = P.d_wsq.as<uint64_t>();
        ra.rec = P.d_rec.as<RoiRecord>();
        ra.step = l > 0 ? 1 : 0;   // candidate step fused into k_roi_eval (layer 0 is decided on the host)
        ra.mark_reached0 = l - 1 == 0 ? 1 : 0;
        ra.live_out = live[cur_list ^ 1];
        ra.live_out_count = livecnt + d + 1;
        ra.thr = P.layer_score[l];
        if (in_run) {
            // run layer k reads state_buf[(k + 1) & 1] (k = 0: the initial states, buffer 0) and records of layer k - 1
            // from rec_buf[(k + 1) & 1], writes state_buf[k & 1] and records to rec_buf[k & 1]
            ra.rec = rec_buf[run_k & 1];
            if (run_k > 0) {
                ra.state = state_buf[(run_k + 1) & 1];
                ra.state_out = state_buf[run_k & 1];
                ra.prev_rec = rec_buf[(run_k + 1) & 1];
                ra.prev_nodes = P.d_nodes.as<AngleNode>() + P.node_off[d - 1];
                ra.prev_thr = P.layer_score[l + 1];
                ra.prev_W = ctx->src[l + 1].w;
                ra.prev_H = ctx->src[l + 1].h;
                ra.live_out_count = livecnt + d;   // the survivors entering this layer (counted, not listed)
            }
        }
        if (step_tables && l >= 1 && ra.step && !roi_small_fits(ctx->tmpl[l - 1].w, ctx->tmpl[l - 1].h) &&
            !ctx->tmpl[l - 1].equal1) {
            const TmplLevel& nt = ctx->tmpl[l - 1];
            ra.nt_tab = P.d_tab.as<int32_t>();
            ra.nt_nodes = P.d_nodes.as<AngleNode>() + P.node_off[d + 1];
            ra.nt_tabw = roi_pitch_for(nt.w); ra.nt_tabh = roi_tab_rows(nt.h);
            ra.nt_tw = nt.w; ra.nt_th = nt.h;
            ra.nt_W = ctx->src[l - 1].w; ra.nt_H = ctx->src[l - 1].h;
        }
        const int total_rois = P.C * P.n3;
        const bool small = roi_small_fits(tl.w, tl.h);   // one-kernel refinement of the ROI in LDS
        for (int base = 0; base < total_rois; base += P.slot_cap) {
            ra.slot_base = base;
            ra.slot_cap = std::min(P.slot_cap, total_rois - base);
            if (small) {
                ProfScope ps(ctx, FPM_K_ROI_SMALL, 0);
                launch_roi_small(ra, st);
                continue;
            }
            if (!tables_done) {
                ProfScope ps(ctx, FPM_K_ROI_TABLES, 0);
                launch_roi_tables(ra, st);
            }
            {
                ProfScope ps(ctx, FPM_K_ROI_WARP, 0);
                launch_roi_warp(ra, st);
            }
            {
                ProfScope ps(ctx, FPM_K_ROI_CORR, 0);
                launch_roi_corr(ra, st);
            }
            {
                ProfScope ps(ctx, FPM_K_ROI_EVAL, 0);
                launch_roi_eval(ra, st);
            }
        }
        tables_done = ra.nt_tab != nullptr;
        if (in_run && l > run_end) {   // the step runs in the next layer's prologue
            tables_done = false;
            ++run_k;
            continue;
        }
        if (small && ra.step) {
            ProfScope ps(ctx, FPM_K_CAND_STEP, 0);
            if (in_run && run_k > 0) {   // the run's last layer: step from its buffers into the canonical state
                ra.state = state_buf[run_k & 1];
                ra.state_out = state_buf[0];
                ra.rec = rec_buf[run_k & 1];
                ra.live_out_count = livecnt + d + 1;
            }
            launch_cand_step(ra, P.C, st);
            P.step_layers |= 1u << d;
        }
        if (ra.step) {
            cur_list ^= 1;
            list_cnt = d + 1;
        }
    }
    HIP_TRY(hipGetLastError());
    // results into pinned host memory (one kernel; only the layer-0 candidates' states and records)
    {
        PackArgs pa;
        pa.counts = P.d_counts.as<int32_t>(); pa.J = J;
        pa.peaks = P.d_peaks.as<Peak>(); pa.C = P.C;
        pa.cap = P.cap;
        if ((size_t)J * P.cap != (size_t)P.C) { ctx->err = "plan layout: C != J * cap"; return FPM_E_INTERNAL; }
        pa.livecnt = livecnt; pa.nlive = L + 2;
        pa.live0 = L > 0 ? live[cur_list] : nullptr;   // the layer-0 list
        pa.live0_count = livecnt + (L > 0 ? L - 1 : 0);
        pa.state = P.d_state.as<CandState>();
        pa.rec = P.d_rec.as<RoiRecord>();
        pa.n3 = P.n3;
        pa.host = P.h_dev;
        pa.o_counts = P.h_counts; pa.o_peaks = P.h_peaks; pa.o_live = P.h_live;
        pa.o_live0 = P.h_live0; pa.o_state0 = P.h_state; pa.o_rec0 = P.h_rec;
        launch_pack(pa, st);
        HIP_TRY(hipGetLastError());
    }
    return FPM_OK;
}

// Host half of the search, split at the one point where a search can be sharded by angle:
//   collect_candidates: every top-layer candidate of source s in the reference's push order (angle-major, then
//     peak order, TemplateMatcher.cpp:157-211) with its own refinement outcome (:262-371) — each candidate's
//     descent is independent of every other candidate's, so a shard of the angle list yields exactly the
//     records of its angles;
//   merge_candidates: everything after that which couples candidates — the std::sort of the top list (:214),
//     vecAllResult in sorted order, filterWithScore, filterWithRotatedRect, the final sort and the
//     s_SingleTargetMatch conversion (:373-432).  It needs the complete push-order sequence, i.e. the shards'
//     records concatenated in shard order.
// pos[id] = index of candidate id in the layer-0 live list (k_pack's compact states / records), -1 if absent.
void collect_candidates(fpm_ctx* ctx, int s, const std::vector<int>& pos, std::vector<fpm_candidate>& out) {
    Plan& P = ctx->plan;
    const int L = P.L;
    out.clear();
    if (P.nang == 0) return;
    const char* h = P.h_out.as<char>();
    const int32_t* counts = (const int32_t*)(h + P.h_counts);
    const Peak* peaks = (const Peak*)(h + P.h_peaks);
    const CandState* state = (const CandState*)(h + P.h_state);
    const RoiRecord* rec = (const RoiRecord*)(h + P.h_rec);
    const TmplLevel& t0 = ctx->tmpl[0];
    const double astep = std::atan(2.0 / std::max(t0.w, t0.h)) * kR2D;   // layer 0's angle step (:283)
    const SrcLevel& lv = ctx->src[0];
    const F2 sc = f2((lv.w - 1) / 2.0f, (lv.h - 1) / 2.0f);
    // each angle's candidates go to their place in push order (angle-major): the angles run on the host pool when
    // there are many candidates
    std::vector<int> first(P.nang + 1, 0);
    for (int a = 0; a < P.nang; ++a) first[a + 1] = first[a] + counts[s * P.nang + a];
    out.resize(first[P.nang]);
    auto angle = [&](int a) {
        const int job = s * P.nang + a;
        HostMatch nm[3];   // one candidate's n3 (1 or 3) angle results
        int o = first[a];
        for (int r = 0; r < counts[job]; ++r) {
            const int id = job * P.cap + r;
            const Peak& pk = peaks[id];
            fpm_candidate c{};
            c.top_score = (double)pk.score;
            c.angle_index = P.a0 + a;
            c.peak_rank = r;
            c.source = s;
            if (L == 0) {   // iTopLayer <= iStopLayer (:272-276)
                const F2 pt = f2((float)pk.x - P.top[a].tx, (float)pk.y - P.top[a].ty);
                const double rad = -P.angles[a] * kD2R;
                const F2 lt = rotate_pt(f2(pt.x, pt.y), P.center, std::cos(rad), std::sin(rad));
                c.x = lt.x; c.y = lt.y; c.score = pk.score; c.angle = P.angles[a]; c.kept = 1;
                out[o++] = c;
                continue;
            }
            const int li = pos[id];
            if (li < 0) { out[o++] = c; continue; }   // broke out at a layer > 0 (:331-332)
            const CandState& cs = state[li];
            // layer 0 (:282-358) from the device's ROI records
            const int d = L - 1;
            int imax = 0;
            double big = -1;
            for (int j = 0; j < P.n3; ++j) {
                const RoiRecord& rr = rec[(size_t)li * P.n3 + j];
                HostMatch m{};
                m.ptx = rr.mx; m.pty = rr.my;
                m.score = rr.score;
                m.angle = P.nodes[d][(size_t)cs.node * P.n3 + j].angle;
                m.on_border = rr.on_border != 0;
                for (int x = 0; x < 3; ++x)
                    for (int y = 0; y < 3; ++y) m.vec[x][y] = rr.vec[x * 3 + y];
                nm[j] = m;
                if (nm[j].score > big) { imax = j; big = nm[j].score; }
            }
            if (nm[imax].score < P.layer_score[0]) { out[o++] = c; continue; }
            if (ctx->run_prm.subpixel && !nm[imax].on_border && imax != 0 && imax != 2) {
                double nx = 0, ny = 0, na = 0;
                subpix_estimation(nm, &nx, &ny, &na, astep, imax);
                nm[imax].ptx = nx; nm[imax].pty = ny;
                nm[imax].angle = na;
            }
            const double nang = nm[imax].angle;
            const double rad = nang * kD2R;
            const F2 r0 = rotate_pt(f2(cs.lt.x * 2, cs.lt.y * 2), sc, std::cos(rad), std::sin(rad));
            const F2 pad = f2(r0.x - 3, r0.y - 3);
            F2 p = f2((float)(nm[imax].ptx + pad.x), (float)(nm[imax].pty + pad.y));
            const double nrad = -nang * kD2R;
            p = rotate_pt(p, sc, std::cos(nrad), std::sin(nrad));
            c.x = p.x; c.y = p.y; c.score = nm[imax].score; c.angle = nang; c.kept = 1;
            out[o++] = c;
        }
    };
    if (first[P.nang] < 1024) {
        for (int a = 0; a < P.nang; ++a) angle(a);
    } else {
        host_parallel(P.nang, angle);
    }
}

// vecAllResult after filterWithScore (:214, :262-358, :373-378) when that needs no sort emulation: if the kept
// candidates scoring at least the threshold have pairwise distinct scores (and none is NaN), the sorted order after
// filterWithScore is the unique descending order, whatever the push order and the first std::sort did with equal
// top scores.  LSD radix sort on order-preserving 64-bit keys; false (nothing decided) on a tie or a NaN, and the
// caller replays both std::sorts.
static bool select_distinct_scores(const fpm_params& prm, const fpm_candidate* cand, int n, std::vector<int>& src) {
    struct SK { uint64_t k; int32_t i; };
    std::vector<SK> a, b;
    a.reserve(n);
    for (int i = 0; i < n; ++i) {
        const fpm_candidate& c = cand[i];
        if (!c.kept) continue;
        if (std::isnan(c.score)) return false;
        if (c.score < prm.score) continue;
        uint64_t u;
        std::memcpy(&u, &c.score, 8);
        u = (u >> 63) ? ~u : (u | (1ULL << 63));   // ascending key = ascending score
        a.push_back({~u, i});                        // ascending ~key = descending score
    }
    const size_t m = a.size();
    b.resize(m);
    uint64_t diff = 0;
    for (size_t t = 1; t < m; ++t) diff |= a[t].k ^ a[0].k;
    for (int sh = 0; sh < 64; sh += 8) {
        if (!((diff >> sh) & 0xFF)) continue;   // every key shares this byte
        size_t cnt[257] = {};
        for (const SK& e : a) cnt[((e.k >> sh) & 0xFF) + 1]++;
        for (int d = 0; d < 256; ++d) cnt[d + 1] += cnt[d];
        for (const SK& e : a) b[cnt[(e.k >> sh) & 0xFF]++] = e;
        a.swap(b);
    }
    for (size_t t = 1; t < m; ++t)
        if (cand[a[t].i].score == cand[a[t - 1].i].score) return false;   // equal scores (+0 == -0 included)
    src.resize(m);
    for (size_t t = 0; t < m; ++t) src[t] = a[t].i;
    return true;
}

// filterWithRotatedRect (:1133-1194) with its pair tests on the device: k_overlap_pairs decides every pair i < j
// whose boxes overlap (the exact test of fpm_rrect.h, bit-identical to the host's), and the host replays the
// reference's loop on those decisions -- for i in order, skipped once deleted, each listed j not yet deleted
// deletes the lower-scored of the two (j, as v is sorted by descending score) -- evaluating itself only the pairs
// whose point order needs acos.  The same deletions as filter_with_rotated_rect.  Returns false (nothing done, the
// caller runs the host filter) without a context, for short lists, or when a rectangle has more overlapping
// partners than the kernel keeps.
constexpr int kOverlapDeviceMin = 1024;   // FPM_OVERLAP_DEVICE_MIN overrides (tests force small lists through it)
struct OverlapStats {
    int host_pairs = 0, flags = 0, entries = 0;
};
static bool overlap_filter_device(fpm_ctx* ctx, std::vector<HostMatch>& v, double max_overlap, int min_n = 0,
                                  OverlapStats* st = nullptr) {
    const int n = (int)v.size();
    if (min_n <= 0) {
        min_n = kOverlapDeviceMin;
        if (const char* e = getenv("FPM_OVERLAP_DEVICE_MIN")) min_n = std::max(1, atoi(e));
    }
    if (!ctx || n < min_n) return false;
    const int cap = 48 * n;
    const size_t boff = (sizeof(OvRect) * (size_t)n + 15) / 16 * 16;
    const size_t rbytes = boff + sizeof(float4) * (size_t)n;   // rects, then boxes
    if (ctx->h_ov_in.ensure(rbytes) != hipSuccess || ctx->d_ov.ensure(rbytes + 64) != hipSuccess ||
        ctx->h_ov_out.ensure(sizeof(int32_t) * ((size_t)cap + 2 * (size_t)n + 16)) != hipSuccess)
        return false;
    OvRect* rin = ctx->h_ov_in.as<OvRect>();
    float4* bin = ctx->h_ov_in.as<float4>(boff);
    static const bool tail_times = [] { const char* e = getenv("FPM_TAIL_TIMES"); return e && *e == '1'; }();
    using clk = std::chrono::steady_clock;
    const clk::time_point q0 = clk::now();
    auto geom = [&](int i0, int i1) {   // corners and boxes exactly as filter_with_rotated_rect computes them
        for (int i = i0; i < i1; ++i) {
            OvRect& o = rin[i];
            rrect_corners(v[i].rect, o.c);
            float x0 = o.c[0].x, x1 = o.c[0].x, y0 = o.c[0].y, y1 = o.c[0].y;
            for (int k = 1; k < 4; ++k) {
                x0 = std::min(x0, o.c[k].x); x1 = std::max(x1, o.c[k].x);
                y0 = std::min(y0, o.c[k].y); y1 = std::max(y1, o.c[k].y);
            }
            o.w = v[i].rect.w; o.h = v[i].rect.h;
            bin[i] = make_float4(x0 - 1.f, y0 - 1.f, x1 + 1.f, y1 + 1.f);
        }
    };
    host_parallel((n + 511) / 512, [&](int t) { geom(t * 512, std::min(n, t * 512 + 512)); });
    const clk::time_point q1 = clk::now();
    int32_t* hout = ctx->h_ov_out.as<int32_t>();   // [meta 16][offcnt 2n][lists cap]
    int32_t* dout = nullptr;
    if (hipHostGetDevicePointer((void**)&dout, ctx->h_ov_out.p, 0) != hipSuccess) return false;
    OvRect* drects = ctx->d_ov.as<OvRect>();
    int32_t* dmeta = (int32_t*)((char*)ctx->d_ov.p + rbytes);
    if (hipMemcpyAsync(drects, rin, rbytes, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
        hipMemsetAsync(dmeta, 0, 2 * sizeof(int32_t), ctx->stream) != hipSuccess)
        return false;
    launch_overlap_pairs(drects, ctx->d_ov.as<float4>(boff), n, max_overlap, dout + 16 + 2 * n, cap, dout + 16, dmeta,
                         ctx->stream);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(hout, dmeta, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
        hipStreamSynchronize(ctx->stream) != hipSuccess)
        return false;
    const clk::time_point q2 = clk::now();
    if (st) { st->flags = hout[1]; st->entries = hout[0]; }
    if (hout[1] != 0) return false;   // a rectangle with too many partners, or the list overflowed
    // the outputs, written by the device into mapped host memory, read once into ordinary memory
    std::vector<int32_t> local((size_t)2 * n + hout[0]);
    std::memcpy(local.data(), hout + 16, sizeof(int32_t) * local.size());
    const clk::time_point q3 = clk::now();
    const int32_t* offcnt = local.data();
    const int32_t* lists = local.data() + 2 * n;
    std::vector<char> del(n, 0);
    int host_pairs = 0;
    // v is sorted by descending score, so "the lower-scored of the two" is j; a NaN score breaks that order, and then
    // the scores are compared as the reference does
    bool monotone = true;
    for (int i = 0; i + 1 < n && monotone; ++i) monotone = v[i].score >= v[i + 1].score;
    for (int i = 0; i < n; ++i) {
        if (del[i]) continue;
        const int32_t* L = lists + offcnt[2 * i];
        for (int k = 0; k < offcnt[2 * i + 1]; ++k) {
            const int32_t e = L[k];
            const int j = e >= 0 ? e : ~e;
            if (del[j]) continue;
            if (e < 0 && (++host_pairs, !rrect_pair_drops(v[i].rect, v[j].rect, max_overlap))) continue;
            if (monotone || v[i].score >= v[j].score) del[j] = 1;
            else del[i] = 1;
        }
    }
    size_t w = 0;
    for (int i = 0; i < n; ++i)
        if (!del[i]) v[w++] = v[i];
    v.resize(w);
    if (st) st->host_pairs = host_pairs;
    if (tail_times) {
        auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        fprintf(stderr, "overlap-dev n=%d geom %.3f device %.3f read %.3f replay %.3f ms, %d pair entries, %d decided on the host\n",
                n, ms(q0, q1), ms(q1, q2), ms(q2, q3), ms(q3, clk::now()), hout[0], host_pairs);
    }
    return true;
}

// Returns false when `cand` is not in push order (angle_index ascending, peak_rank 0, 1, ... within an angle).
bool merge_candidates(const fpm_params& prm, int t0w, int t0h, const fpm_candidate* cand, int n,
                      std::vector<fpm_result>& out, fpm_ctx* dev_ctx) {
    out.clear();
    for (int i = 0; i < n; ++i) {
        const bool first = i == 0 || cand[i].angle_index != cand[i - 1].angle_index;
        if (first ? (cand[i].peak_rank != 0 || (i > 0 && cand[i].angle_index < cand[i - 1].angle_index))
                  : cand[i].peak_rank != cand[i - 1].peak_rank + 1)
            return false;
    }
    // FPM_TAIL_TIMES=1: per-stage wall clocks of this tail on stderr (profiling aid)
    static const bool tail_times = [] { const char* e = getenv("FPM_TAIL_TIMES"); return e && *e == '1'; }();
    using clk = std::chrono::steady_clock;
    const clk::time_point t0 = clk::now();
    clk::time_point t1 = t0;
    std::vector<HostMatch> all;
    // vecAllResult entry from a candidate record, with its rotated rectangle (:380-390)
    auto fill = [&](HostMatch& m, const fpm_candidate& c) {
        m = HostMatch{};
        m.ptx = c.x; m.pty = c.y; m.score = c.score; m.angle = c.angle;
        const double rad = -m.angle * kD2R;
        const float cs = (float)std::cos(rad), sn = (float)std::sin(rad);
        const F2 lt = f2((float)m.ptx, (float)m.pty);
        const F2 rt = f2(lt.x + t0w * cs, lt.y - t0w * sn);
        const F2 rb = f2(rt.x + t0h * sn, rt.y + t0h * cs);
        m.rect = rrect_from3(lt, rt, rb);
        m.del = false;
    };
    std::vector<int> src;   // candidate index of each vecAllResult entry after filterWithScore
    if (select_distinct_scores(prm, cand, n, src)) {
        t1 = clk::now();
    } else {
        // std::sort(vecMatchParameter, compareScoreBig2Small) (:214) over the push-order sequence.  The permutation
        // std::sort produces depends only on the sequence of comparison results, so sorting light (score, index)
        // keys with the same comparator reproduces the reference's order of equal scores exactly.
        struct Key { double score; int i; };
        auto by_score = [](const Key& l, const Key& r) { return l.score > r.score; };
        std::vector<Key> order(n);
        for (int i = 0; i < n; ++i) order[i] = {cand[i].top_score, i};
        std::sort(order.begin(), order.end(), by_score);
        // vecAllResult in sorted-candidate order (:262-358) is the kept candidates' sequence; filterWithScore's
        // std::sort (:373-378) sees exactly their scores in that order, so it runs on (score, candidate) keys too
        std::vector<Key> ks;
        ks.reserve(n);
        for (const Key& k : order)
            if (cand[k.i].kept) ks.push_back({cand[k.i].score, k.i});
        t1 = clk::now();
        std::sort(ks.begin(), ks.end(), by_score);
        size_t m = 0;   // the sorted list ends at the first score below the threshold (filter_with_score)
        while (m < ks.size() && !(ks[m].score < prm.score)) ++m;
        src.resize(m);
        for (size_t t = 0; t < m; ++t) src[t] = ks[t].i;
    }
    const clk::time_point t2 = clk::now();
    const int na = (int)src.size();
    all.resize(na);
    if (na <= 512) {
        for (int i = 0; i < na; ++i) fill(all[i], cand[src[i]]);
    } else {
        host_parallel((na + 255) / 256, [&](int t) {
            for (int i = t * 256; i < std::min(na, t * 256 + 256); ++i) fill(all[i], cand[src[i]]);
        });
    }
    const clk::time_point t3 = clk::now();
    if (!overlap_filter_device(dev_ctx, all, prm.max_overlap)) filter_with_rotated_rect(all, prm.max_overlap);
    const clk::time_point t4 = clk::now();
    std::sort(all.begin(), all.end(), score_big2small);
    if (tail_times) {
        auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        fprintf(stderr, "tail n=%d sort1+collect %.3f score %.3f rects %.3f overlap %.3f final %.3f ms -> %zu\n", n,
                ms(t0, t1), ms(t1, t2), ms(t2, t3), ms(t3, t4), ms(t4, clk::now()), all.size());
    }
    if (prm.semantics == FPM_SEMANTICS_MFC) {   // MatchToolDlg.cpp:1080-1116
        for (const HostMatch& m : all) {
            const double rad = -m.angle * kD2R;
            fpm_result o;
            o.lt_x = m.ptx; o.lt_y = m.pty;   // f64 corners from the f64 point (the Qt class rounds to Point2f)
            o.rt_x = o.lt_x + t0w * std::cos(rad); o.rt_y = o.lt_y - t0w * std::sin(rad);
            o.lb_x = o.lt_x + t0h * std::sin(rad); o.lb_y = o.lt_y + t0h * std::cos(rad);
            o.rb_x = o.rt_x + t0h * std::sin(rad); o.rb_y = o.rt_y + t0h * std::cos(rad);
            o.cx = (o.lt_x + o.rt_x + o.rb_x + o.lb_x) / 4;
            o.cy = (o.lt_y + o.rt_y + o.rb_y + o.lb_y) / 4;
            o.angle = -m.angle;   // negated, wrapped to [-180, 180]
            if (o.angle < -180) o.angle += 360;
            if (o.angle > 180) o.angle -= 360;
            o.score = m.score;
            out.push_back(o);
            if ((int)out.size() == prm.max_pos) break;   // at most MaxPos rows (:1115-1116)
        }
        return true;
    }
    for (const HostMatch& m : all) {   // :406-432
        const double rad = -m.angle * kD2R;
        const float cs = (float)std::cos(rad), sn = (float)std::sin(rad);
        const F2 lt = f2((float)m.ptx, (float)m.pty);
        const F2 rt = f2(lt.x + t0w * cs, lt.y - t0w * sn);
        const F2 lb = f2(lt.x + t0h * sn, lt.y + t0h * cs);
        const F2 rb = f2(rt.x + t0h * sn, rt.y + t0h * cs);
        const F2 c = f2((lt.x + rt.x + lb.x + rb.x) / 4.0f, (lt.y + rt.y + lb.y + rb.y) / 4.0f);
        fpm_result o;
        o.lt_x = lt.x; o.lt_y = lt.y; o.rt_x = rt.x; o.rt_y = rt.y;
        o.rb_x = rb.x; o.rb_y = rb.y; o.lb_x = lb.x; o.lb_y = lb.y;
        o.cx = c.x; o.cy = c.y; o.angle = m.angle; o.score = m.score;
        out.push_back(o);
    }
    return true;
}

// Launch the search: replay the captured graph (every pointer and launch shape is fixed by the plan and the
// source slab; data-dependent work sizes live in device counters), or enqueue it eagerly when profiling.
int launch_search(fpm_ctx* ctx) {
    if (ctx->prof) return enqueue_search(ctx);   // per-launch HIP events need the eager path
    if (!ctx->graph || ctx->graph_plan != ctx->plan_builds || ctx->graph_src != ctx->d_src.p) {
        if (ctx->graph) { (void)hipGraphExecDestroy(ctx->graph); ctx->graph = nullptr; }
        hipGraph_t g = nullptr;
        HIP_TRY(hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
        const int rc = enqueue_search(ctx);
        const hipError_t e = hipStreamEndCapture(ctx->stream, &g);
        if (rc != FPM_OK) { if (g) (void)hipGraphDestroy(g); return rc; }
        HIP_TRY(e);
        const hipError_t ie = hipGraphInstantiate(&ctx->graph, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        HIP_TRY(ie);
        ctx->graph_plan = ctx->plan_builds;
        ctx->graph_src = ctx->d_src.p;
    }
    HIP_TRY(hipGraphLaunch(ctx->graph, ctx->stream));
    return FPM_OK;
}

// First half of a staged search: plan, then the whole device pass enqueued on the context's stream (no wait).
int start_staged(fpm_ctx* ctx) {
    ctx->t_call0 = std::chrono::steady_clock::now();
    ctx->cands.clear();
    ctx->stats.clear();
    int rc = build_plan(ctx);
    if (rc != FPM_OK) return rc;
    if (!ctx->t_ev[0]) {
        HIP_TRY(hipEventCreate(&ctx->t_ev[0]));
        HIP_TRY(hipEventCreate(&ctx->t_ev[1]));
    }
    HIP_TRY(hipEventRecord(ctx->t_ev[0], ctx->stream));
    if (ctx->plan.nang > 0) {   // an angle shard with no angles has no device work (and no candidates)
        rc = launch_search(ctx);
        if (rc != FPM_OK) return rc;
    }
    HIP_TRY(hipEventRecord(ctx->t_ev[1], ctx->stream));
    ctx->run_prm = ctx->prm;
    ctx->pending = true;
    return FPM_OK;
}

// Second half: wait for the device pass, then the host's reference-order post-processing per source.
int complete_staged(fpm_ctx* ctx, std::vector<std::vector<fpm_result>>& results, bool merge = true) {
    if (!ctx->pending) { ctx->err = "no search in flight"; return FPM_E_INVALID_ARG; }
    ctx->pending = false;
    const auto c0 = ctx->t_call0;
    {   // a large host tail follows (thousands of top-layer candidates per source): wake the host pool now, so its
        // workers are spinning, not asleep, when the tail's parallel regions start after the device wait
        const Plan& P = ctx->plan;
        if ((size_t)P.nang * P.cap >= 2048)
            host_pool_warm((int)std::min(10000.0, 1000.0 * std::max(1.0, (double)ctx->last_device_ms) + 1000.0));
    }
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    const auto c1 = std::chrono::steady_clock::now();
    {
        float ms = 0;
        if (hipEventElapsedTime(&ms, ctx->t_ev[0], ctx->t_ev[1]) == hipSuccess) ctx->last_device_ms = ms;
    }
    prof_collect(ctx);
    Plan& P = ctx->plan;
    results.assign(P.S, {});
    std::vector<int> pos;
    if (P.L > 0 && P.nang > 0) {
        const char* hb = P.h_out.as<char>();
        const int n0 = ((const int32_t*)(hb + P.h_live))[P.L - 1];
        const int32_t* ids = (const int32_t*)(hb + P.h_live0);
        pos.assign(P.C, -1);
        for (int li = 0; li < n0; ++li) pos[ids[li]] = li;
    }
    ctx->cands.assign(P.S, {});
    for (int s = 0; s < P.S; ++s) {
        collect_candidates(ctx, s, pos, ctx->cands[s]);
        if (merge)
            merge_candidates(ctx->run_prm, ctx->tmpl[0].w, ctx->tmpl[0].h, ctx->cands[s].data(), (int)ctx->cands[s].size(),
                             results[s], ctx);
    }
    // stats: [angles, top candidates, live entering layer L-1 .. 0] (totals over the batch)
    const char* h = P.h_out.as<char>();
    const int32_t* counts = (const int32_t*)(h + P.h_counts);
    int64_t topc = 0;
    for (int k = 0; k < P.S * P.nang; ++k) topc += counts[k];
    ctx->stats.assign({(int64_t)P.nang, topc});
    static const int32_t zeros[64] = {};
    const int32_t* lc = P.nang > 0 ? (const int32_t*)(h + P.h_live) : zeros;
    for (int d = 0; d < P.L; ++d) ctx->stats.push_back(lc[d]);
    // SURVEY.md §8(d) algorithmic bytes (compulsory input + output of each stage, u8 = 1 B, f32 = 4 B; scratch
    // between the stages of this design is not counted), summed over the batch:
    //   B_pyr = sum_{l<L} (W_l H_l + W_{l+1} H_{l+1});  B_top = sum_angles (W_L H_L + 4 |R_a|);
    //   B_ref = sum_{l<L} sum_{live ROIs at l} ((w_l + 6)(h_l + 6) + w_l h_l + 49 * 4)
    {
        int64_t bp = 0, bt = 0, br = 0;
        for (int l = 0; l < P.L; ++l)
            bp += (int64_t)ctx->src[l].w * ctx->src[l].h + (int64_t)ctx->src[l + 1].w * ctx->src[l + 1].h;
        for (int a = 0; a < P.nang; ++a)
            bt += (int64_t)ctx->src[P.L].w * ctx->src[P.L].h + 4LL * P.map_w[a] * P.map_h[a];
        for (int d = 0; d < P.L && P.nang > 0; ++d) {
            const TmplLevel& t = ctx->tmpl[P.L - 1 - d];
            br += (int64_t)lc[d] * P.n3 * ((int64_t)(t.w + 6) * (t.h + 6) + (int64_t)t.w * t.h + 49 * 4);
        }
        ctx->alg_bytes[0] = bp * P.S;
        ctx->alg_bytes[1] = bt * P.S;
        ctx->alg_bytes[2] = br;
    }
    if (ctx->prof && P.nang > 0) {   // per-kernel share of B_ref (the live counts are known only now)
        // the matrix-core top layer never writes its maps: the peak extraction over them (the greedy form on the
        // lists) is charged the map term of B_top, 4 |R_a| per source and angle
        if (P.top_lists)
            for (int a = 0; a < P.nang; ++a) ctx->kp[FPM_K_TOP_NMS].bytes += 4LL * P.map_w[a] * P.map_h[a] * P.S;
        for (int d = 0; d < P.L; ++d) {
            const int l = P.L - 1 - d;
            const TmplLevel& t = ctx->tmpl[l];
            const int64_t rois = (int64_t)lc[d] * P.n3;
            const int64_t foot = (int64_t)(t.w + 6) * (t.h + 6), tmpl = (int64_t)t.w * t.h;
            if (P.step_layers & (1u << d))   // the step: its candidates' records and state (design state, not §8(d))
                ctx->kp[FPM_K_CAND_STEP].bytes +=
                    (int64_t)lc[d] * (P.n3 * (int64_t)sizeof(RoiRecord) + 2 * (int64_t)sizeof(CandState) + 4);
            if (roi_small_fits(t.w, t.h)) {   // one kernel: footprint + template in, the 7x7 scores out
                ctx->kp[FPM_K_ROI_SMALL].bytes += rois * (foot + tmpl + 49 * 4);
                continue;
            }
            // the sampled ROI, row sums and window partials are this design's scratch, not §8(d) traffic: the
            // sampling kernel is charged the footprint read, the correlation the template, the evaluation the scores
            ctx->kp[FPM_K_ROI_WARP].bytes += rois * foot;
            ctx->kp[FPM_K_ROI_CORR].bytes += rois * tmpl;
            ctx->kp[FPM_K_ROI_EVAL].bytes += rois * 49 * 4;
        }
    }
    const auto c2 = std::chrono::steady_clock::now();
    ctx->last_host_ms = std::chrono::duration<double, std::milli>(c2 - c1).count();
    ctx->last_call_ms = std::chrono::duration<double, std::milli>(c2 - c0).count();
    return FPM_OK;
}

int run_staged(fpm_ctx* ctx, std::vector<std::vector<fpm_result>>& results) {
    const int rc = start_staged(ctx);
    if (rc != FPM_OK) return rc;
    return complete_staged(ctx, results);
}

int upload_sources(fpm_ctx* ctx, const uint8_t* const* grays, int count, int w, int h, size_t stride) {
    int rc = layout_sources(ctx, count, w, h);
    if (rc != FPM_OK) return rc;
    const SrcLevel& l0 = ctx->src[0];
    for (int s = 0; s < count; ++s)
        HIP_TRY(hipMemcpy2DAsync(ctx->d_src.as<uint8_t>() + l0.off + l0.img_bytes * s, l0.pitch, grays[s], stride, w, h,
                                 hipMemcpyHostToDevice, ctx->stream));
    return FPM_OK;
}

}  // namespace

// =========================================================================================================
// C ABI
// =========================================================================================================
extern "C" {

void fpm_params_default(fpm_params* p) {
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    p->max_pos = 70;            // TemplateMatcher.cpp:29
    p->max_overlap = 0.0;       // :30
    p->score = 0.7;             // :31
    p->tolerance_angle = 0.0;   // :32
    p->min_reduce_area = 256;   // :33
    p->use_simd = 1;            // :34
    p->subpixel = 0;            // :35
    p->tolerance_range = 0;     // :38
    p->semantics = FPM_SEMANTICS_QT;
    p->top_angle_step = 0.0;    // extension: the reference's derived step
}

int fpm_abi_version(void) { return FPM_ABI_VERSION; }

int fpm_create(int device, fpm_ctx** out) {
    if (!out) return FPM_E_INVALID_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || device < 0 || device >= n) return FPM_E_DEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return FPM_E_DEVICE;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return FPM_E_DEVICE;
    fpm_ctx* ctx = new (std::nothrow) fpm_ctx();
    if (!ctx) return FPM_E_INTERNAL;
    ctx->device = device;
    fpm_params_default(&ctx->prm);
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return FPM_E_DEVICE;
    }
    *out = ctx;
    return FPM_OK;
}

int fpm_destroy(fpm_ctx* ctx) {
    if (!ctx) return FPM_E_INVALID_ARG;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->graph) (void)hipGraphExecDestroy(ctx->graph);
    for (hipEvent_t e : ctx->t_ev)
        if (e) (void)hipEventDestroy(e);
    ctx->plan.release();
    ctx->d_tmpl.release(); ctx->d_tmpl8.release(); ctx->d_tsum.release(); ctx->d_src.release();
    ctx->d_op_a.release(); ctx->d_op_b.release(); ctx->d_op_job.release();
    ctx->d_ov.release(); ctx->h_ov_in.release(); ctx->h_ov_out.release();
    for (auto& k : ctx->kp)
        for (auto& e : k.ev) { (void)hipEventDestroy(e.first); (void)hipEventDestroy(e.second); }
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return FPM_OK;
}

const char* fpm_last_error(const fpm_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int fpm_set_params(fpm_ctx* ctx, const fpm_params* p) {
    if (!ctx || !p) return FPM_E_INVALID_ARG;
    if (ctx->pending) { ctx->err = "a search is in flight (fpm_match_staged_finish first)"; return FPM_E_INVALID_ARG; }
    ctx->prm = *p;
    return FPM_OK;
}

int fpm_get_params(const fpm_ctx* ctx, fpm_params* p) {
    if (!ctx || !p) return FPM_E_INVALID_ARG;
    *p = ctx->prm;
    return FPM_OK;
}

// TemplateMatcher::learnPattern (TemplateMatcher.cpp:45-95)
int fpm_learn(fpm_ctx* ctx, const uint8_t* gray, int32_t w, int32_t h, size_t stride) {
    if (!ctx) return FPM_E_INVALID_ARG;
    if (!gray || w <= 0 || h <= 0 || stride < (size_t)w) { ctx->err = "empty template"; return FPM_E_INVALID_ARG; }
    if (ctx->pending) { ctx->err = "a search is in flight (fpm_match_staged_finish first)"; return FPM_E_INVALID_ARG; }
    HIP_TRY(hipSetDevice(ctx->device));
    ctx->learned = false;
    ctx->staged = false;
    ctx->tmpl.clear();
    const int L = top_layer(w, h, (int)std::sqrt((double)ctx->prm.min_reduce_area));
    std::vector<TmplLevel> lv(L + 1);
    size_t off = 0;
    int lw = w, lh = h;
    for (int l = 0; l <= L; ++l) {
        lv[l].w = lw; lv[l].h = lh;
        lv[l].pitch = round_up(lw + 4, 64);
        lv[l].off = off;
        off += round_up((size_t)lv[l].pitch * (lh + 1), (size_t)256);
        lw = (lw + 1) / 2;
        lh = (lh + 1) / 2;
    }
    HIP_TRY(ctx->d_tmpl.ensure(off));
    uint8_t* base = ctx->d_tmpl.as<uint8_t>();
    HIP_TRY(hipMemsetAsync(base, 0, off, ctx->stream));
    HIP_TRY(hipMemcpy2DAsync(base + lv[0].off, lv[0].pitch, gray, stride, w, h, hipMemcpyHostToDevice, ctx->stream));
    for (int l = 1; l <= L; ++l)   // cv::buildPyramid (:55) on the device
        launch_pyr_down(base + lv[l - 1].off, lv[l - 1].w, lv[l - 1].h, lv[l - 1].pitch, 0, base + lv[l].off, lv[l].w,
                        lv[l].h, lv[l].pitch, 0, 1, ctx->stream);
    HIP_TRY(hipGetLastError());
    for (int l = 0; l <= L; ++l) {
        lv[l].px.resize((size_t)lv[l].w * lv[l].h);
        HIP_TRY(hipMemcpy2DAsync(lv[l].px.data(), lv[l].w, base + lv[l].off, lv[l].pitch, lv[l].w, lv[l].h,
                                 hipMemcpyDeviceToHost, ctx->stream));
    }
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    double m0, s0;
    mean_stddev(lv[0].px, &m0, &s0);
    ctx->border = m0 < 128 ? 255 : 0;   // :58-59
    for (int l = 0; l <= L; ++l) {      // :66-91
        const double inv_area = 1.0 / ((double)lv[l].h * lv[l].w);
        double mean, sdv;
        mean_stddev(lv[l].px, &mean, &sdv);
        double norm = sdv * sdv;
        lv[l].equal1 = norm < DBL_EPSILON;
        norm = std::sqrt(norm);
        norm /= std::sqrt(inv_area);
        lv[l].mean = mean; lv[l].norm = norm; lv[l].inv_area = inv_area;
    }
    {   // MFMA operand copies: T ^ 0x80 (= T - 128 as i8), zero beyond the template; per-row sums of T
        size_t o8 = 0, os = 0;
        for (int l = 0; l <= L; ++l) {
            lv[l].p8 = 64 * ((lv[l].w + 63) / 64);
            lv[l].off8 = o8;
            o8 += (size_t)lv[l].p8 * round_up(lv[l].h, kMmaRows);
            lv[l].tsum_off = os;
            os += round_up(lv[l].h, kMmaRows);
        }
        o8 += 256;   // slack: k_roi_corr prefetches up to 2 64-byte blocks past a row's last
        std::vector<int8_t> h8(o8, 0);
        std::vector<int32_t> hs(os, 0);
        for (int l = 0; l <= L; ++l)
            for (int y = 0; y < lv[l].h; ++y) {
                int32_t sum = 0;
                for (int x = 0; x < lv[l].w; ++x) {
                    const uint8_t v = lv[l].px[(size_t)y * lv[l].w + x];
                    h8[lv[l].off8 + (size_t)y * lv[l].p8 + x] = (int8_t)(v ^ 0x80);
                    sum += v;
                }
                hs[lv[l].tsum_off + y] = sum;
            }
        HIP_TRY(ctx->d_tmpl8.ensure(o8));
        HIP_TRY(ctx->d_tsum.ensure(os * sizeof(int32_t)));
        HIP_TRY(hipMemcpy(ctx->d_tmpl8.p, h8.data(), o8, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(ctx->d_tsum.p, hs.data(), os * sizeof(int32_t), hipMemcpyHostToDevice));
    }
    ctx->tmpl = std::move(lv);
    ctx->learned = true;
    ctx->tmpl_gen++;
    return FPM_OK;
}

int fpm_clear_pattern(fpm_ctx* ctx) {
    if (!ctx) return FPM_E_INVALID_ARG;
    if (ctx->pending) { ctx->err = "a search is in flight (fpm_match_staged_finish first)"; return FPM_E_INVALID_ARG; }
    ctx->learned = false;
    ctx->staged = false;
    ctx->tmpl.clear();
    ctx->tmpl_gen++;
    return FPM_OK;
}

int fpm_is_learned(const fpm_ctx* ctx) { return ctx && ctx->learned ? 1 : 0; }

int fpm_stage_sources(fpm_ctx* ctx, const uint8_t* const* grays, int32_t count, int32_t w, int32_t h, size_t stride) {
    if (!ctx) return FPM_E_INVALID_ARG;
    if (!grays || count <= 0 || w <= 0 || h <= 0 || stride < (size_t)w) { ctx->err = "bad sources"; return FPM_E_INVALID_ARG; }
    for (int i = 0; i < count; ++i)
        if (!grays[i]) { ctx->err = "null source"; return FPM_E_INVALID_ARG; }
    if (ctx->pending) { ctx->err = "a search is in flight (fpm_match_staged_finish first)"; return FPM_E_INVALID_ARG; }
    int rc = check_sizes(ctx, w, h);
    if (rc != FPM_OK) return rc;
    HIP_TRY(hipSetDevice(ctx->device));
    ctx->staged = false;
    rc = upload_sources(ctx, grays, count, w, h, stride);
    if (rc != FPM_OK) return rc;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    ctx->staged = true;
    return FPM_OK;
}

static int copy_results(const std::vector<std::vector<fpm_result>>& res, fpm_result* out, int32_t cap,
                        int32_t* n_results) {
    int status = FPM_OK;
    for (size_t s = 0; s < res.size(); ++s) {
        n_results[s] = (int32_t)res[s].size();
        for (int i = 0; i < (int)res[s].size(); ++i) {
            if (i < cap && out) out[s * (size_t)cap + i] = res[s][i];
            else status = FPM_E_CAPACITY;
        }
    }
    return status;
}

int fpm_match_staged_launch(fpm_ctx* ctx) {
    if (!ctx) return FPM_E_INVALID_ARG;
    if (!ctx->learned) { ctx->err = "template not learned"; return FPM_E_NOT_LEARNED; }
    if (ctx->S <= 0 || !ctx->staged) { ctx->err = "no staged sources (fpm_match replaces a staged batch)"; return FPM_E_INVALID_ARG; }
    if (ctx->pending) { ctx->err = "a search is already in flight"; return FPM_E_INVALID_ARG; }
    HIP_TRY(hipSetDevice(ctx->device));
    return start_staged(ctx);
}

int fpm_match_staged_finish(fpm_ctx* ctx, fpm_result* out, int32_t cap, int32_t* n_results) {
    if (!ctx || !n_results) return FPM_E_INVALID_ARG;
    HIP_TRY(hipSetDevice(ctx->device));
    ctx->results.clear();
    const int rc = complete_staged(ctx, ctx->results, out != nullptr);
    if (rc != FPM_OK) return rc;
    return copy_results(ctx->results, out, cap, n_results);
}

int fpm_match_staged(fpm_ctx* ctx, fpm_result* out, int32_t cap, int32_t* n_results) {
    if (!n_results) return FPM_E_INVALID_ARG;
    const int rc = fpm_match_staged_launch(ctx);
    if (rc != FPM_OK) return rc;
    return fpm_match_staged_finish(ctx, out, cap, n_results);
}

// TemplateMatcher::match (TemplateMatcher.cpp:97-437)
int fpm_match(fpm_ctx* ctx, const uint8_t* gray, int32_t w, int32_t h, size_t stride, fpm_result* out, int32_t cap,
              int32_t* n_results, double* seconds) {
    if (!ctx || !n_results) return FPM_E_INVALID_ARG;
    *n_results = 0;
    if (ctx->pending) { ctx->err = "a search is in flight (fpm_match_staged_finish first)"; return FPM_E_INVALID_ARG; }
    // a failed call leaves no stale candidate records behind (fpm_last_candidates of a sharded search)
    ctx->cands.clear();
    ctx->stats.clear();
    ctx->results.clear();
    if (!gray || w <= 0 || h <= 0 || stride < (size_t)w) { ctx->err = "empty source"; return FPM_E_INVALID_ARG; }
    int rc = check_sizes(ctx, w, h);
    if (rc != FPM_OK) return rc;
    HIP_TRY(hipSetDevice(ctx->device));
    ctx->staged = false;   // the slab is re-laid out for this one source
    // the reference deep-copies the source before its clock starts (TemplateMatcher.cpp:104 then :117): the upload
    // is that copy, so getLastExecutionTime() starts once it has landed
    rc = upload_sources(ctx, &gray, 1, w, h, stride);
    if (rc != FPM_OK) return rc;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    const auto t0 = std::chrono::high_resolution_clock::now();
    rc = run_staged(ctx, ctx->results);
    if (rc != FPM_OK) return rc;
    const auto t1 = std::chrono::high_resolution_clock::now();
    const std::vector<fpm_result>& r = ctx->results[0];
    *n_results = (int32_t)r.size();
    if (!r.empty() && seconds) *seconds = std::chrono::duration<double>(t1 - t0).count();
    for (int i = 0; i < (int)r.size() && i < cap && out; ++i) out[i] = r[i];
    return (int)r.size() > cap ? FPM_E_CAPACITY : FPM_OK;
}

int fpm_last_results(const fpm_ctx* ctx, fpm_result* out, int32_t cap, int32_t* n_results) {
    if (!ctx || !n_results) return FPM_E_INVALID_ARG;
    if (ctx->pending) return FPM_E_INVALID_ARG;
    return copy_results(ctx->results, out, cap, n_results);
}

// --- angle sharding of one search ---------------------------------------------------------
int fpm_set_angle_shard(fpm_ctx* ctx, int32_t shard, int32_t shards) {
    if (!ctx) return FPM_E_INVALID_ARG;
    if (shards < 1 || shard < 0 || shard >= shards) { ctx->err = "bad angle shard"; return FPM_E_INVALID_ARG; }
    if (ctx->pending) { ctx->err = "a search is in flight (fpm_match_staged_finish first)"; return FPM_E_INVALID_ARG; }
    ctx->shard = shard;
    ctx->shards = shards;
    return FPM_OK;
}

int fpm_get_angle_shard(const fpm_ctx* ctx, int32_t* shard, int32_t* shards) {
    if (!ctx || !shard || !shards) return FPM_E_INVALID_ARG;
    *shard = ctx->shard;
    *shards = ctx->shards;
    return FPM_OK;
}

int fpm_last_candidates(const fpm_ctx* ctx, int32_t source, fpm_candidate* out, int32_t cap, int32_t* n) {
    if (!ctx || !n) return FPM_E_INVALID_ARG;
    *n = 0;
    if (source < 0 || source >= (int)ctx->cands.size()) return FPM_E_INVALID_ARG;
    const std::vector<fpm_candidate>& c = ctx->cands[source];
    *n = (int32_t)c.size();
    for (int i = 0; i < (int)c.size() && i < cap && out; ++i) out[i] = c[i];
    return (int)c.size() > cap ? FPM_E_CAPACITY : FPM_OK;
}

int fpm_merge_candidates(const fpm_params* p, int32_t tmpl_w, int32_t tmpl_h, const fpm_candidate* cand, int32_t n,
                         fpm_result* out, int32_t cap, int32_t* n_results) {
    if (!p || !n_results || tmpl_w <= 0 || tmpl_h <= 0 || n < 0 || (n > 0 && !cand)) return FPM_E_INVALID_ARG;
    *n_results = 0;
    if (n >= 2048) host_pool_warm(2000);   // a large tail: the pool's workers awake for its parallel regions
    std::vector<fpm_result> res;
    if (!merge_candidates(*p, tmpl_w, tmpl_h, cand, n, res, nullptr)) return FPM_E_INVALID_ARG;
    *n_results = (int32_t)res.size();
    for (int i = 0; i < (int)res.size() && i < cap && out; ++i) out[i] = res[i];
    return (int)res.size() > cap ? FPM_E_CAPACITY : FPM_OK;
}

int fpm_search_bytes(const fpm_ctx* ctx, int64_t* b_pyr, int64_t* b_top, int64_t* b_ref) {
    if (!ctx || !b_pyr || !b_top || !b_ref) return FPM_E_INVALID_ARG;
    *b_pyr = ctx->alg_bytes[0];
    *b_top = ctx->alg_bytes[1];
    *b_ref = ctx->alg_bytes[2];
    return FPM_OK;
}

int fpm_search_stats(const fpm_ctx* ctx, int64_t* stats, int32_t cap) {
    if (!ctx || !stats) return FPM_E_INVALID_ARG;
    int n = 0;
    for (int64_t v : ctx->stats)
        if (n < cap) stats[n++] = v;
    return n;
}

int fpm_op_overlap_filter(fpm_ctx* ctx, const float* corners, const double* scores, int32_t n, double max_overlap,
                          int32_t mode, int32_t* keep, int32_t* n_keep, int32_t* stats) {
    if (!ctx || !n_keep || n < 0 || (n > 0 && (!corners || !scores || !keep)) || (mode != 0 && mode != 1))
        return FPM_E_INVALID_ARG;
    *n_keep = 0;
    if (stats) stats[0] = stats[1] = stats[2] = stats[3] = 0;
    HIP_TRY(hipSetDevice(ctx->device));
    std::vector<HostMatch> v((size_t)n);
    for (int i = 0; i < n; ++i) {
        HostMatch& m = v[(size_t)i];
        m = HostMatch{};
        const float* c = corners + 6 * (size_t)i;
        m.rect = rrect_from3(f2(c[0], c[1]), f2(c[2], c[3]), f2(c[4], c[5]));
        m.score = scores[i];
        m.id = i;
    }
    int path = 0;
    OverlapStats st;
    if (mode == 1 && n > 0) {
        path = overlap_filter_device(ctx, v, max_overlap, 1, &st) ? 1 : 2;
        if (path == 2) filter_with_rotated_rect(v, max_overlap);
    } else {
        filter_with_rotated_rect(v, max_overlap);
    }
    for (size_t i = 0; i < v.size(); ++i) keep[i] = v[i].id;
    *n_keep = (int32_t)v.size();
    if (stats) { stats[0] = path; stats[1] = st.host_pairs; stats[2] = st.flags; stats[3] = st.entries; }
    return FPM_OK;
}

int fpm_template_info(const fpm_ctx* ctx, int32_t* levels, int32_t* border_color) {
    if (!ctx || !levels || !border_color) return FPM_E_INVALID_ARG;
    if (!ctx->learned) return FPM_E_NOT_LEARNED;
    *levels = (int32_t)ctx->tmpl.size();
    *border_color = ctx->border;
    return FPM_OK;
}

int fpm_template_level(const fpm_ctx* ctx, int32_t level, int32_t* w, int32_t* h, double* mean, double* norm,
                       double* inv_area, int32_t* result_equal1, uint8_t* pixels, size_t stride) {
    if (!ctx || !w || !h || !mean || !norm || !inv_area || !result_equal1) return FPM_E_INVALID_ARG;
    if (!ctx->learned) return FPM_E_NOT_LEARNED;
    if (level < 0 || level >= (int)ctx->tmpl.size()) return FPM_E_INVALID_ARG;
    const TmplLevel& t = ctx->tmpl[level];
    *w = t.w; *h = t.h; *mean = t.mean; *norm = t.norm; *inv_area = t.inv_area; *result_equal1 = t.equal1 ? 1 : 0;
    if (pixels)
        for (int y = 0; y < t.h; ++y) std::memcpy(pixels + (size_t)y * stride, t.px.data() + (size_t)y * t.w, (size_t)t.w);
    return FPM_OK;
}

// ---- pixel operators ----------------------------------------------------------------------------------
int fpm_op_pyr_down(fpm_ctx* ctx, const uint8_t* src, int32_t w, int32_t h, size_t ss, uint8_t* dst, size_t ds) {
    if (!ctx) return FPM_E_INVALID_ARG;
    if (!src || !dst || w <= 0 || h <= 0 || ss < (size_t)w) { ctx->err = "bad image"; return FPM_E_INVALID_ARG; }
    const int dw = (w + 1) / 2, dh = (h + 1) / 2;
    if (ds < (size_t)dw) { ctx->err = "bad dst stride"; return FPM_E_INVALID_ARG; }
    HIP_TRY(hipSetDevice(ctx->device));
    const int sp = round_up(w + 4, 64), dp = round_up(dw + 4, 64);
    HIP_TRY(ctx->d_op_a.ensure((size_t)sp * (h + 1)));
    HIP_TRY(ctx->d_op_b.ensure((size_t)dp * (dh + 1)));
    HIP_TRY(hipMemcpy2DAsync(ctx->d_op_a.p, sp, src, ss, w, h, hipMemcpyHostToDevice, ctx->stream));
    // 3-chunk segments: every image taller than 64 output rows goes through the carried-window path
    launch_pyr_down(ctx->d_op_a.as<uint8_t>(), w, h, sp, 0, ctx->d_op_b.as<uint8_t>(), dw, dh, dp, 0, 1, ctx->stream, 3);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpy2DAsync(dst, ds, ctx->d_op_b.p, dp, dw, dh, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return FPM_OK;
}

int fpm_op_pyr_down2(fpm_ctx* ctx, const uint8_t* src, int32_t w, int32_t h, size_t ss, uint8_t* dst1, size_t ds1,
                     uint8_t* dst2, size_t ds2, int32_t seg_chunks, int32_t chunk_rows) {
    if (!ctx) return FPM_E_INVALID_ARG;
    if (!src || !dst1 || !dst2 || w <= 0 || h <= 0 || ss < (size_t)w || seg_chunks < 0 ||
        (chunk_rows != 0 && chunk_rows != 16 && chunk_rows != 32)) {
        ctx->err = "bad image";
        return FPM_E_INVALID_ARG;
    }
    const int bw = (w + 1) / 2, bh = (h + 1) / 2, cw = (bw + 1) / 2, ch = (bh + 1) / 2;
    if (ds1 < (size_t)bw || ds2 < (size_t)cw) { ctx->err = "bad dst stride"; return FPM_E_INVALID_ARG; }
    HIP_TRY(hipSetDevice(ctx->device));
    // the search's level layout: pitch round_up(w + 4, 64), one spare row
    const int sp = round_up(w + 4, 64), bp = round_up(bw + 4, 64), cp = round_up(cw + 4, 64);
    const size_t boff = round_up((size_t)bp * (bh + 1), (size_t)256);
    HIP_TRY(ctx->d_op_a.ensure((size_t)sp * (h + 1)));
    HIP_TRY(ctx->d_op_b.ensure(boff + (size_t)cp * (ch + 1)));
    HIP_TRY(hipMemcpy2DAsync(ctx->d_op_a.p, sp, src, ss, w, h, hipMemcpyHostToDevice, ctx->stream));
    uint8_t* b = ctx->d_op_b.as<uint8_t>();
    launch_pyr_down2(ctx->d_op_a.as<uint8_t>(), w, h, sp, 0, b, bw, bh, bp, 0, b + boff, cw, ch, cp, 0, 1, ctx->stream,
                     seg_chunks, nullptr, 0, chunk_rows);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpy2DAsync(dst1, ds1, b, bp, bw, bh, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipMemcpy2DAsync(dst2, ds2, b + boff, cp, cw, ch, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return FPM_OK;
}

int fpm_op_warp_affine(fpm_ctx* ctx, const uint8_t* src, int32_t w, int32_t h, size_t ss, const double m[6],
                       uint8_t* dst, int32_t dw, int32_t dh, size_t ds, int32_t border) {
    if (!ctx) return FPM_E_INVALID_ARG;
    if (!src || !dst || !m || w <= 0 || h <= 0 || dw <= 0 || dh <= 0 || ss < (size_t)w || ds < (size_t)dw) {
        ctx->err = "bad warp arguments";
        return FPM_E_INVALID_ARG;
    }
    HIP_TRY(hipSetDevice(ctx->device));
    const int sp = round_up(w + 4, 64), dp = round_up(dw + 4, 64);
    HIP_TRY(ctx->d_op_a.ensure((size_t)sp * (h + 1)));
    HIP_TRY(ctx->d_op_b.ensure((size_t)dp * (dh + 1)));
    HIP_TRY(ctx->d_op_job.ensure(sizeof(WarpJob)));
    WarpJob j{};
    j.src = ctx->d_op_a.as<uint8_t>(); j.sw = w; j.sh = h; j.sp = sp;
    j.dst = ctx->d_op_b.as<uint8_t>(); j.dw = dw; j.dh = dh; j.dp = dp;
    j.border = border;
    std::copy(m, m + 6, j.M);
    invert_affine(j.M);
    HIP_TRY(hipMemcpyAsync(ctx->d_op_job.p, &j, sizeof(j), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpy2DAsync(ctx->d_op_a.p, sp, src, ss, w, h, hipMemcpyHostToDevice, ctx->stream));
    launch_warp(ctx->d_op_job.as<WarpJob>(), 1, dw * dh, ctx->stream);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpy2DAsync(dst, ds, ctx->d_op_b.p, dp, dw, dh, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return FPM_OK;
}

int fpm_op_ncc_map(fpm_ctx* ctx, const uint8_t* src, int32_t w, int32_t h, size_t ss, int32_t layer, int32_t fold,
                   float* out) {
    if (!ctx) return FPM_E_INVALID_ARG;
    if (!ctx->learned) { ctx->err = "template not learned"; return FPM_E_NOT_LEARNED; }
    if (!src || !out || w <= 0 || h <= 0 || ss < (size_t)w || layer < 0 || layer >= (int)ctx->tmpl.size()) {
        ctx->err = "bad ncc arguments";
        return FPM_E_INVALID_ARG;
    }
    const TmplLevel& t = ctx->tmpl[layer];
    if (w < t.w || h < t.h) { ctx->err = "image smaller than template level"; return FPM_E_SIZE; }
    HIP_TRY(hipSetDevice(ctx->device));
    const int ow = w - t.w + 1, oh = h - t.h + 1;
    const int sp = round_up(w + 4, 64);
    HIP_TRY(ctx->d_op_a.ensure((size_t)sp * (h + 1)));
    HIP_TRY(ctx->d_op_b.ensure(sizeof(float) * (size_t)ow * oh));
    HIP_TRY(ctx->d_op_job.ensure(sizeof(NccJob)));
    NccJob j{};
    j.img = ctx->d_op_a.as<uint8_t>(); j.iw = w; j.ih = h; j.ip = sp;
    j.tmpl = ctx->d_tmpl.as<uint8_t>() + t.off; j.tw = t.w; j.th = t.h; j.tp = t.pitch;
    j.out = ctx->d_op_b.as<float>(); j.ow = ow; j.oh = oh;
    j.fold = fold ? 1 : 0;
    j.equal1 = t.equal1 ? 1 : 0;
    j.mean = t.mean; j.norm = t.norm; j.inv_area = t.inv_area;
    HIP_TRY(hipMemcpyAsync(ctx->d_op_job.p, &j, sizeof(j), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpy2DAsync(ctx->d_op_a.p, sp, src, ss, w, h, hipMemcpyHostToDevice, ctx->stream));
    if (ncc_tile_fits(t.w, t.h)) launch_ncc_tile(ctx->d_op_job.as<NccJob>(), 1, ow, oh, t.w, t.h, ctx->stream);
    else launch_ncc_map(ctx->d_op_job.as<NccJob>(), 1, ow * oh, t.w * t.h, ctx->stream);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(out, ctx->d_op_b.p, sizeof(float) * (size_t)ow * oh, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return FPM_OK;
}

// ---- profiling ----------------------------------------------------------------------------------------
int fpm_profile_enable(fpm_ctx* ctx, int32_t enable) {
    if (!ctx) return FPM_E_INVALID_ARG;
    ctx->prof = enable != 0;
    return FPM_OK;
}

int fpm_profile_reset(fpm_ctx* ctx) {
    if (!ctx) return FPM_E_INVALID_ARG;
    for (auto& k : ctx->kp) { k.ms = 0; k.launches = 0; k.bytes = 0; k.used = 0; }
    return FPM_OK;
}

int fpm_profile_last(const fpm_ctx* ctx, double* device_ms, double* host_ms, double* call_ms) {
    if (!ctx || !device_ms || !host_ms || !call_ms) return FPM_E_INVALID_ARG;
    *device_ms = ctx->last_device_ms;
    *host_ms = ctx->last_host_ms;
    *call_ms = ctx->last_call_ms;
    return FPM_OK;
}

int fpm_profile_get(const fpm_ctx* ctx, int32_t kernel, double* total_ms, int64_t* launches, int64_t* bytes) {
    if (!ctx || kernel < 0 || kernel >= FPM_K_COUNT || !total_ms || !launches || !bytes) return FPM_E_INVALID_ARG;
    *total_ms = ctx->kp[kernel].ms;
    *launches = ctx->kp[kernel].launches;
    *bytes = ctx->kp[kernel].bytes;
    return FPM_OK;
}

}  // extern "C"
