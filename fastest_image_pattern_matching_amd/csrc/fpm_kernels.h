// fpm_kernels.h — device job descriptors and kernel launchers (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fpm_geom.h"

namespace fpm {

// K2 / fpm_op_warp_affine: one inverse-mapped bilinear warp (cv::warpAffine INTER_LINEAR, BORDER_CONSTANT).
struct WarpJob {
    const uint8_t* src;
    uint8_t* dst;
    int32_t sw, sh, sp;      // source size, row pitch (bytes)
    int32_t dw, dh, dp;      // destination size, row pitch
    int32_t border;
    int32_t pad;
    double M[6];             // INVERTED matrix (dst -> src)
};

// K3+K4 / fpm_op_ncc_map: full NCC map of an image against one template level.
struct NccJob {
    const uint8_t* img;
    const uint8_t* tmpl;
    float* out;              // dense (ow x oh)
    int32_t iw, ih, ip;
    int32_t tw, th, tp;
    int32_t ow, oh;
    int32_t fold;            // 1: IM_Conv_SIMD per-row float fold; 0: TM_CCORR exact sum -> f32
    int32_t equal1;          // s_TemplData::vecResultEqual1 -> map of ones
    double mean, norm, inv_area;
};

// K5: peak extraction on one top-layer map (plain getNextMaxLoc or s_BlockMax).
struct NmsJob {
    float* map;
    float* bmax;             // s_BlockMax scratch (block mode), nb entries
    int32_t* bloc;
    int32_t mw, mh;
};

struct Peak {
    int32_t x, y;
    float score;
    int32_t pad;
};

struct NmsArgs {
    const NmsJob* jobs;
    Peak* peaks;             // [job][cap]
    int32_t* counts;         // [job]
    int32_t tw, th;          // top template size
    int32_t cap;             // max_pos + MATCH_CANDIDATE_NUM
    int32_t by_block;
    int32_t mfc;             // MFC s_BlockMax semantics (fpm_params.semantics, MatchToolDlg.h:93-210)
    int32_t lds_blocks;      // block-maxima capacity in LDS (set by launch_nms; 0 = global scratch)
    int32_t* cand;           // s_BlockMax mode: indices of the map pixels >= thr, [job][cand_cap] (k_nms_blocks)
    int32_t* cand_cnt;       // [job], zeroed before the launch
    int32_t cand_cap;        // kNmsCandCap
    int32_t cand_lds;        // candidate capacity in LDS (set by launch_nms)
    double thr;              // vecLayerScore[top]
    double overlap;
    uint64_t* stamps;        // profiling only (scripts/nms_probe.hip): k_nms_fast phase cycles of job 0, else null
    uint64_t* skey;          // s_BlockMax mode: [job][3] strip-block maxima keys, zeroed before the launch
    int32_t* sdone;          // [job][3] finished chunks of each strip block, zeroed before the launch
    const float* cand_val;   // k_nms_greedy: the candidates' values (k_top_mma's lists), nullptr = read the map
    int32_t reset_untaken;   // k_nms_greedy: a map it does not take gets cand_cnt = 0 (k_nms_blocks recounts it)
    int32_t greedy_cap;      // k_nms_greedy: sort capacity in LDS (power of 2; 0 = kGreedyMax)
};

// Angle-tree node: the reference's refinement angle for one path, with glibc trig of angle*D2R.
struct AngleNode {
    double angle;
    double c, s;             // cos, sin of (angle * D2R)
    double cn, sn;           // cos, sin of -(angle * D2R)
};

// Top-layer per-angle constants (host-computed, TemplateMatcher.cpp:163-173).
struct TopAngle {
    float tx, ty;            // fTranslationX/Y
    int32_t bw, bh;          // sizeBest
};

struct CandInitArgs {
    const Peak* peaks;
    const int32_t* counts;
    const TopAngle* angles;  // [nang]
    const AngleNode* top_nodes;  // [nang] angle, cos/sin of +-angle*D2R
    CandState* state;        // [cap_total]
    int32_t* live;           // output live list (layer top-1)
    int32_t* live_count;
    int32_t nang, cap;       // per source
    int32_t total;           // sources * nang * cap
    F2 center;               // top-layer ptCenter
    int32_t refine;          // top layer > 0
};

struct RoiArgs {
    const uint8_t* level;    // source pyramid level base (source 0); + src * level_stride
    size_t level_stride;
    int32_t W, H, P;         // level size and pitch
    const uint8_t* tmpl;     // template level
    int32_t tw, th, tp;
    const int8_t* tmpl8;     // template level as i8 (T ^ 0x80), zero beyond tw / th: [round_up(th,16)][tp8]
    int32_t tp8;             // its row pitch (multiple of 64)
    int32_t nk;              // ceil(tw / 64): MFMA k-steps per row
    const int32_t* tsum;     // per template row: sum of T (u8)
    int32_t n3;              // refinement angles per candidate (1 or 3)
    int32_t rc;              // template rows per correlation chunk
    int32_t nchunk;          // ceil(th / rc)
    int32_t fold;            // use_simd
    int32_t equal1;
    int32_t per_source;      // candidates per source (nang * cap)
    int32_t slot_base;       // this round covers live ROIs [slot_base, slot_base + slot_cap)
    int32_t slot_cap;
    double mean, norm, inv_area;
    const int32_t* live;
    const int32_t* live_count;
    CandState* state;        // read by the ROI kernels, stepped by k_roi_eval
    const AngleNode* nodes;  // level nodes; child = parent * n3 + j
    int32_t* tab;            // [slot] fixed-point warp tables: ad[tabw], bd[tabw], x0[tabh], y0[tabh]
    int32_t tabw, tabh;
    int4* tdesc;             // [slot][tdesc_stride] per 32x32 ROI tile: source footprint box + flags
    int32_t tdesc_stride;
    uint8_t* roi;            // [slot] sampled ROI, tile-major: 32 x 32 tiles of 1 KB, row of tiles by row
    int32_t roi_pitch;       // LDS row pitch of staged ROI rows (k_roi_corr)
    size_t roi_stride;
    int32_t nparts;          // k_roi_fused: runs of bands per ROI (work unit = (ROI, run of bands))
    uint32_t* rowsum;        // [slot][th][49] exact int32 per-row dot products
    uint32_t* wsum;          // [slot][nchunk][49] window-sum partials of I
    uint64_t* wsq;           // [slot][nchunk][49] window-sum partials of I^2
    RoiRecord* rec;          // [cand * n3 + j]
    // candidate step fused into k_roi_eval (TemplateMatcher.cpp:329-366) when step != 0
    int32_t step;            // 1: best of n3, early break, back-mapping, append to live_out
    int32_t mark_reached0;   // next layer is 0
    int32_t* live_out;
    int32_t* live_out_count;
    double thr;              // vecLayerScore[layer]
    // k_roi_small with prev_rec set (consecutive small layers above layer 0): the previous
    // layer's candidate step runs in each workgroup's prologue (every workgroup of a candidate computes the same
    // stepped state; jj 0 stores it to state_out and counts the survivor in *live_out_count), over the previous
    // layer's live list unchanged -- candidates that died stay in it as holes their workgroups skip.  k_cand_step
    // after the run's last layer compacts the list.  k_cand_step also writes state_out (nullptr = state).
    const RoiRecord* prev_rec;   // the previous layer's records [cand * n3 + j]
    const AngleNode* prev_nodes; // the previous layer's nodes
    double prev_thr;             // vecLayerScore of the previous layer
    int32_t prev_W, prev_H;      // the previous layer's level size
    CandState* state_out;
    // nt_tab != nullptr: the step (k_roi_eval, k_cand_step -> k_cand_step_tab) also writes the next layer's warp tables
    // and tile descriptors for each survivor at its next-list position, so that layer launches no k_roi_tables (the
    // next layer takes tables and runs as one round; tdesc / tdesc_stride / per_source are shared with it)
    int32_t* nt_tab;
    const AngleNode* nt_nodes;   // the next layer's nodes
    int32_t nt_tabw, nt_tabh, nt_tw, nt_th, nt_W, nt_H;
    uint64_t* stamps;        // profiling ablations only (scripts/roi_microbench.hip): per-phase s_memtime stamps
};


// Final pack of a search's results into pinned host memory (replaces several device -> host copies): top-peak
// counts and peaks, live counts, and for the candidates that reached layer 0 (the layer-0 live list) their ids,
// states and refinement records, compacted by live index.
struct PackArgs {
    const int32_t* counts; int32_t J;
    const Peak* peaks; int32_t C;
    int32_t cap;                   // peak slots per job (C == J * cap)
    const int32_t* livecnt; int32_t nlive;
    const int32_t* live0;          // layer-0 live list (nullptr when the top layer is layer 0)
    const int32_t* live0_count;
    const CandState* state;
    const RoiRecord* rec;
    int32_t n3;
    char* host;                    // pinned host buffer
    size_t o_counts, o_peaks, o_live, o_live0, o_state0, o_rec0;
};

// launchers (stream-ordered, no synchronisation)
// seg_chunks > 0 forces that many 32-row chunks per workgroup (the op entry point uses it so single images exercise
// the carried-window path); 0 = sized for the grid
// zero / nzero: as launch_warp (the search's first pyramid launch clears the counters when the top layer's kernel
// also writes the live list)
void launch_pyr_down(const uint8_t* src, int sw, int sh, int sp, size_t s_img, uint8_t* dst, int dw, int dh,
                     int dp, size_t d_img, int nimg, hipStream_t st, int seg_chunks = 0, int32_t* zero = nullptr,
                     int nzero = 0);
// two pyramid levels in one launch: src -> b (level l+1, written) -> c (level l+2); same arguments per level
void launch_pyr_down2(const uint8_t* src, int sw, int sh, int sp, size_t s_img, uint8_t* bdst, int bw, int bh, int bp,
                      size_t b_img, uint8_t* cdst, int cw, int ch, int cp, size_t c_img, int nimg, hipStream_t st,
                      int seg_chunks = 0, int32_t* zero = nullptr, int nzero = 0, int chunk_rows = 0);
// zero / nzero: counters the search zeroes before its later kernels use them (block (0, 0) clears them), so the
// graph carries no memset nodes
void launch_warp(const WarpJob* jobs, int njobs, int max_pixels, hipStream_t st, int32_t* zero = nullptr,
                 int nzero = 0);
void launch_ncc_map(const NccJob* jobs, int njobs, int max_out, int tmpl_bytes, hipStream_t st);
bool ncc_tile_fits(int tw, int th);   // LDS-tiled variant applies (templates up to 128 x 64)
void launch_ncc_tile(const NccJob* jobs, int njobs, int max_ow, int max_oh, int tw, int th, hipStream_t st);
constexpr int kNmsCandCap = 8192;   // s_BlockMax candidates (pixels >= the top-layer score) kept per map
// max_blocks: s_BlockMax blocks of the largest map (block mode); max_map_dim: largest map width or height
// max_cells: the largest ceil(mw / tw) * ceil(mh / th) over the maps (k_nms_greedy's coverage cells)
// max_items: the largest nms_block_items of the maps (k_nms_blocks' grid: strip blocks are scanned in chunks)
// ci (plain getNextMaxLoc path only, cap <= kNmsInitCap): k_nms also does k_cand_init's work for its job's
// candidate slots (one launch fewer); the live counter must have been zeroed by an earlier launch
constexpr int kNmsInitCap = 128;
// max_map_px: the largest map's pixel count (sizes k_nms's dynamic LDS; -1 = unknown)
void launch_nms(const NmsArgs& a, int njobs, int max_blocks, int max_map_dim, int max_cells, hipStream_t st,
                int max_items = 0, const CandInitArgs* ci = nullptr, long max_map_px = -1);
int nms_block_items(int mw, int mh, int tw, int th, int mfc);
void launch_cand_init(const CandInitArgs& a, hipStream_t st);
// K2-K5 fused for small canvases (plain peak path): LDS bytes of one (source, angle) job, and the launch (one
// workgroup per job; zero / nzero as launch_warp)
size_t top_fused_lds(int bw, int bh, int tw, int th);
size_t top_fused_lds_limit();   // 64 KB minus k_top_fused's static LDS (hipFuncGetAttributes, per device)
constexpr int kTopFusedMinJobs = 256;   // fewer jobs than CUs: the three split kernels finish sooner
// ci (cap <= kNmsInitCap): the candidate init fused as in k_nms; the live counter must be zero before the launch
// (zero / nzero are then 0: block 0's clearing would race with the other blocks' atomics)
// order (optional): the job each workgroup takes, costliest angles first (fewer workgroups than resident slots are
// left for the last round)
void launch_top_fused(const WarpJob* wjobs, const NccJob* njobs, const NmsArgs& a, int njobs_n, size_t lds,
                      int32_t* zero, int nzero, hipStream_t st, const CandInitArgs* ci = nullptr,
                      const int32_t* order = nullptr);
// ---- the top layer on the matrix cores (k_top_mma): warp + TM_CCORR + CCOEFF_Denominator for every (source, angle)
// job without materialising the rotated canvas or the map.  Work unit = (job, strip of output columns, run of output
// rows); the host builds the unit list (top_mma_plan).
struct TopUnit { int32_t job, x0, y0, y1; };
constexpr int kTopMmaMaxSw = 192;              // strip width cap (output columns)   // output columns [x0, x0 + sw) and rows [y0, y1) of map `job`
struct TopMmaArgs {
    const WarpJob* wjobs;    // per job: source level, canvas size (dw x dh), inverse matrix, border
    const NccJob* njobs;     // per job: map size (ow x oh) and, for mode 1, the map
    const TopUnit* units;
    int32_t nunits;
    const uint8_t* bfrag;    // [nq][64 lanes][16 B] the correlation's B fragments (T - 128 as i8, Toeplitz-banded)
    int32_t nq, R;           // MFMA slots per 16 x 16 output tile; template rows per slot (2: tw <= 17, 1: tw <= 49)
    int32_t tw, th, area;
    uint32_t tsum;           // sum of the template level's pixels
    int32_t sw;              // strip width (output columns, multiple of 16)
    int32_t cp;              // canvas ring row pitch (bytes; the kernel's compile-time TM_CP)
    int32_t rr;              // ring rows per plane (power of two >= 16 + th - 1; the kernel form's RR)
    int32_t ct, rt;          // column / row table capacity (entries)
    int32_t o_colt, o_rowt, o_bf, o_ft;   // dynamic LDS offsets (bytes)
    int32_t nqm;             // B slots staged in LDS (the kernel form's unrolled slot count; zero past nq)
    int32_t mode;            // 0: candidate lists, 1: full maps of the jobs with cand_cnt >= 0 (fallback)
    int32_t prefilter;       // 1: f32 bound before the exact f64 score (area <= 258, thr > 0)
    float thrK, E;           // prefilter: (thr (1 - 1e-5))^2 * norm^2 * area, absolute slack of the f32 terms
    double thr, mean, norm, inv_area;
    int32_t* cand;           // [job][cand_cap] map indices of the outputs with score >= thr
    float* cand_val;         // [job][cand_cap] their scores
    int32_t* cand_cnt;       // [job] (zeroed before mode 0; may exceed cand_cap)
    int32_t cand_cap;
};
size_t top_mma_lds(const TopMmaArgs& a);
// fills the layout fields of `a` (sw, cp, rr, hp, ct, rt, o_*) for a strip width and the largest unit height
void top_mma_layout(TopMmaArgs& a, int sw, int max_rows);
bool top_mma_fits(int tw, int th);   // template shapes the kernel takes (R = 2 up to 17 wide, R = 1 up to 49)
void launch_top_mma(const TopMmaArgs& a, hipStream_t st);
// k_nms_greedy over k_top_mma's lists (a.cand_val set): plain getNextMaxLoc key (by_block 0) or s_BlockMax key; with ci
// (plain, cap <= kNmsInitCap) the candidate init of the jobs it takes
void launch_top_greedy(const NmsArgs& a, int njobs, int max_cells, hipStream_t st, const CandInitArgs* ci);
void launch_roi_tables(const RoiArgs& a, hipStream_t st);
void launch_roi_warp(const RoiArgs& a, hipStream_t st);
void launch_roi_corr(const RoiArgs& a, hipStream_t st);
void launch_roi_eval(const RoiArgs& a, hipStream_t st);
#ifdef FPM_EXPERIMENTAL   // measurement-only fused K6+K7 (scripts/fused_bench.hip; never in libfpm_hip.so)
bool launch_roi_corr16(const RoiArgs& a, hipStream_t st);   // k_roi_corr16 (scripts/corr16_bench.hip)
bool roi_fused_fits(int tw);           // the fused sampling + correlation kernel applies (templates <= 1024 wide)
int roi_fused_parts(int th);           // runs of bands per ROI (work units per ROI) of k_roi_fused
void launch_roi_fused(const RoiArgs& a, hipStream_t st);
#endif
bool roi_small_fits(int tw, int th);   // the single-kernel small-template refinement applies
size_t roi_small_lds(int tw, int th);
void launch_roi_small(const RoiArgs& a, hipStream_t st);
void launch_cand_step(const RoiArgs& a, int max_items, hipStream_t st);
void launch_pack(const PackArgs& a, hipStream_t st);

// ---- filterWithRotatedRect's pair decisions on the device (TemplateMatcher.cpp:1133-1194) ----
// One result's rotated rectangle: its corners (rrect corners, host-computed from the cv::RotatedRect) and size; its
// corner box widened by 1 px (the host's prefilter: boxes farther apart cannot intersect) in a separate float4 array
// (x0, y0, x1, y1), which the all-pairs sweep reads.
struct OvRect { F2 c[4]; float w, h; };
constexpr int kOverlapMaxCand = 512;   // overlapping partners of one rectangle decided on the device
// For every pair i < j of the n rectangles (sorted as the filter sees them) whose boxes overlap, the exact
// rotatedRectangleIntersection + sortPtWithCenter + area test (fpm_rrect.h); the j of every pair whose overlap
// exceeds max_overlap are written, ascending, to lists[off[i] .. off[i] + cnt[i]) (offcnt[2i], offcnt[2i+1]), as ~j
// when the point order depends on acos (the host decides that pair).  meta[0] = entries written (atomic allocator,
// zeroed by the caller), meta[1] bit 0 = more than kOverlapMaxCand overlapping partners, bit 1 = list full.
// lists / offcnt may be mapped host memory (plain stores only); meta must be device memory.
void launch_overlap_pairs(const OvRect* r, const float4* box, int n, double max_overlap, int32_t* lists, int list_cap,
                          int32_t* offcnt, int32_t* meta, hipStream_t st);
int roi_pick_rc(int tw, int th);
int roi_pitch_for(int tw);
int roi_tab_rows(int th);   // rows of a ROI's X0 / Y0 tables: th + 6 rounded up to a 32-row tile
size_t roi_tiles_bytes(int tw, int th);
int roi_tiles_for(int tw, int th);   // 32x32 warp tiles of a (tw+6) x (th+6) ROI
size_t roi_corr_lds(int roi_pitch, int tw, int rc, bool global_a);
constexpr int kMmaRows = 16;   // template rows per MFMA correlation chunk (M of v_mfma_i32_16x16x64_i8)

}  // namespace fpm
