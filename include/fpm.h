/*
 * fpm.h — C ABI of the MI355X-native NCC template matcher (libfpm_hip.so).
 *
 * Drop-in boundary for the reference's `TemplateMatcher` (lrm2017/Fastest_Image_Pattern_Matching,
 * include/TemplateMatcher.h:9-90, src/TemplateMatcher.cpp:1-1239).  Every entry point below names the
 * reference interface it replaces.  Plain pointers and sizes only: no torch / OpenCV / Qt types.
 *
 * Conventions
 *   - Images are 8-bit single-channel (CV_8UC1) row-major with an explicit row stride in bytes, exactly
 *     what `cv::imread(..., IMREAD_GRAYSCALE)` yields (src/MatchToolDialog.cpp:314, 341).
 *   - Host image pointers are copied to device memory inside the call; the library never retains them.
 *   - Every function returns an `int` status: FPM_OK (0) or a negative FPM_E_* code.  "No match" is
 *     FPM_OK with *n_results == 0, mirroring the reference's empty vector (TemplateMatcher.cpp:99-114, 398).
 *   - One context per host thread; a context is bound to one HIP device and owns one HIP stream.
 *   - fpm_last_error() returns a human-readable message for the last failing call on a context.
 */
#ifndef FPM_H_
#define FPM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FPM_ABI_VERSION 9

/* status codes */
#define FPM_OK 0
#define FPM_E_INVALID_ARG (-1)   /* null pointer, non-positive size, bad stride            */
#define FPM_E_NOT_LEARNED (-2)   /* match() before learnPattern() (TemplateMatcher.cpp:99)   */
#define FPM_E_SIZE (-3)          /* source smaller than template (TemplateMatcher.cpp:107-114)*/
#define FPM_E_DEVICE (-4)        /* HIP runtime error / no gfx950 device                     */
#define FPM_E_CAPACITY (-5)      /* caller-provided result buffer too small                 */
#define FPM_E_INTERNAL (-6)

/* Result semantics (fpm_params.semantics).  The drop-in target is the Qt TemplateMatcher (src/TemplateMatcher.cpp);
 * the README's published numbers come from the MFC tool (MatchTool/MatchToolDlg.cpp), whose search differs in
 * a few places.  FPM_SEMANTICS_MFC reproduces those:
 *   - s_BlockMax blocks of 2x the template, right + bottom strips without a corner block, the last block on
 *     equal maxima, and a full-map minMaxLoc when the map holds no whole block (MatchToolDlg.h:108-210);
 *   - the angle list from the tolerance ranges when tolerance_range is set (MatchToolDlg.cpp:805-815);
 *   - corners and centre in f64, the reported angle negated and wrapped to [-180, 180], at most max_pos
 *     results (MatchToolDlg.cpp:1080-1116). */
#define FPM_SEMANTICS_QT 0
#define FPM_SEMANTICS_MFC 1

/* Search parameters: the 7 public setters of TemplateMatcher (TemplateMatcher.h:22-28) plus the hidden
 * fixed members m_bToleranceRange / m_dTolerance1..4 (TemplateMatcher.h:88-89, TemplateMatcher.cpp:38).
 * Defaults (fpm_params_default) equal the reference constructor (TemplateMatcher.cpp:28-39). */
typedef struct fpm_params {
    int32_t max_pos;          /* setMaxPositions      (default 70)   */
    int32_t min_reduce_area;  /* setMinReduceArea     (default 256)  */
    double max_overlap;       /* setMaxOverlap        (default 0.0)  */
    double score;             /* setScore             (default 0.7)  */
    double tolerance_angle;   /* setToleranceAngle    (default 0.0)  */
    int32_t use_simd;         /* setUseSIMD           (default 1): lower layers use the per-row int32 ->
                                 float fold of IM_Conv_SIMD (TemplateMatcher.cpp:487-512); 0 = TM_CCORR */
    int32_t subpixel;         /* setSubPixelEstimation(default 0)    */
    int32_t tolerance_range;  /* m_bToleranceRange    (fixed false in the Qt class; MFC toggles it,
                                 MatchToolDlg.cpp:2137): 3 refinement angles always; with FPM_SEMANTICS_MFC
                                 also the top-layer angle list from tolerance[0..3]                   */
    int32_t semantics;        /* FPM_SEMANTICS_QT (default) or FPM_SEMANTICS_MFC                       */
    double tolerance[4];      /* m_dTolerance1..4: the MFC ranges [t1, t2] and [t3, t4] (MatchToolDlg.cpp:812-815) */
    double top_angle_step;    /* extension, no reference knob: the top-layer angle step in degrees replacing the
                                 derived atan(2 / max(w, h)) of TemplateMatcher.cpp:130 when > 0 (BASELINE
                                 configs[3] "1 degree step"); 0 = the reference's step (default)     */
} fpm_params;

/* One result; POD-identical to s_SingleTargetMatch (DataStructures.h:97-115): five cv::Point2d then two
 * doubles, 12 f64 in total, same order. */
typedef struct fpm_result {
    double lt_x, lt_y;        /* ptLT     */
    double rt_x, rt_y;        /* ptRT     */
    double rb_x, rb_y;        /* ptRB     */
    double lb_x, lb_y;        /* ptLB     */
    double cx, cy;            /* ptCenter */
    double angle;             /* dMatchedAngle (Qt: +dMatchAngle, TemplateMatcher.cpp:428; MFC: negated and
                                 wrapped, MatchToolDlg.cpp:1093-1099) */
    double score;             /* dMatchScore */
} fpm_result;

typedef struct fpm_ctx fpm_ctx;

/* --- lifecycle -------------------------------------------------------------------------------------- */
void fpm_params_default(fpm_params* p);                 /* TemplateMatcher::TemplateMatcher (:28-39) */
int fpm_create(int device, fpm_ctx** out);               /* TemplateMatcher::TemplateMatcher          */
int fpm_destroy(fpm_ctx* ctx);                           /* TemplateMatcher::~TemplateMatcher (:41)   */
const char* fpm_last_error(const fpm_ctx* ctx);
int fpm_abi_version(void);

/* --- parameters ------------------------------------------------------------------------------------- */
int fpm_set_params(fpm_ctx* ctx, const fpm_params* p);   /* the 7 setters (TemplateMatcher.h:22-28)   */
int fpm_get_params(const fpm_ctx* ctx, fpm_params* p);   /* the 7 getters (TemplateMatcher.h:31-37)   */

/* --- template ----------------------------------------------------------------------------------------*/
/* TemplateMatcher::learnPattern (TemplateMatcher.cpp:45-95).  Returns FPM_E_INVALID_ARG on an empty image
 * (the reference returns false, :47-49). */
int fpm_learn(fpm_ctx* ctx, const uint8_t* gray, int32_t width, int32_t height, size_t stride);
int fpm_clear_pattern(fpm_ctx* ctx);                     /* clearPattern (:439-443)                   */
int fpm_is_learned(const fpm_ctx* ctx);                  /* isPatternLearned (TemplateMatcher.h:43)   */

/* --- search ------------------------------------------------------------------------------------------*/
/* TemplateMatcher::match (TemplateMatcher.cpp:97-437).  Writes at most `cap` results (sorted by
 * descending score, exactly the reference's vector order) and the count to *n_results.
 * *seconds receives getLastExecutionTime() semantics: the pyramid->filter wall time; left unchanged when
 * there is no result (the reference returns before updating it, :398-404).  seconds may be NULL. */
int fpm_match(fpm_ctx* ctx, const uint8_t* gray, int32_t width, int32_t height, size_t stride,
              fpm_result* out, int32_t cap, int32_t* n_results, double* seconds);

/* Batched / device-resident search (no reference equivalent: the UI calls match() once per image).
 * Sources are staged into context-owned HBM once (fpm_stage_sources), then fpm_match_staged runs the
 * whole search for all staged sources layer-synchronously with one device->host copy at the end.
 * out is [count][cap_per_source]; n_results is [count]. */
int fpm_stage_sources(fpm_ctx* ctx, const uint8_t* const* grays, int32_t count, int32_t width,
                      int32_t height, size_t stride);
int fpm_match_staged(fpm_ctx* ctx, fpm_result* out, int32_t cap_per_source, int32_t* n_results);
/* fpm_match_staged split in two: _launch enqueues the whole device pass on the context's stream and returns;
 * _finish waits for it and runs the host post-processing.  Several contexts (one stream each) on one device
 * can have searches in flight at once; the staged sources must not be re-staged in between. */
int fpm_match_staged_launch(fpm_ctx* ctx);
/* out == NULL skips the host tail (sort, filters, conversion; n_results[s] = 0): for an angle-sharded context whose
 * candidate records (fpm_last_candidates) are merged elsewhere. */
int fpm_match_staged_finish(fpm_ctx* ctx, fpm_result* out, int32_t cap_per_source, int32_t* n_results);
/* The results of the last fpm_match / fpm_match_staged(_finish) call once more, laid out as fpm_match_staged's
 * output ([sources][cap_per_source], counts in n_results[sources]; one source after fpm_match).  No reference
 * equivalent (match() returns a growing std::vector): after FPM_E_CAPACITY the caller grows its buffer and fetches
 * the results already computed instead of searching again. */
int fpm_last_results(const fpm_ctx* ctx, fpm_result* out, int32_t cap_per_source, int32_t* n_results);

/* --- angle sharding of one search (no reference equivalent: the reference loops over the
 * whole angle list on one thread, TemplateMatcher.cpp:157-211) ----------------------------------------------
 * A search splits at the reference's own seam: the top-layer sweep and every candidate's pyramid descent
 * (:157-371) are independent per angle, while the std::sort of the top candidates (:214) and the result
 * filters (:373-432) need all of them.  So: every rank runs the search restricted to its shard of the angle
 * list, exports its candidate records, the records are all-gathered in shard order (RCCL over xGMI on a node),
 * and fpm_merge_candidates runs the coupled tail.  The merged results equal the unsharded search's bit for bit.
 *
 * One top-layer candidate (an s_MatchParameter of vecMatchParameter, DataStructures.h:58-94) and the outcome of
 * its refinement. */
typedef struct fpm_candidate {
    double top_score;     /* dMatchScore at the top layer: the key of std::sort(compareScoreBig2Small) (:214) */
    double x, y;          /* refined ptLT at layer 0 (the vecAllResult entry's pt, :346-356), when kept     */
    double score;         /* refined dMatchScore (:312), when kept                                         */
    double angle;         /* refined dMatchAngle (sub-pixel estimate applied, :334-344), when kept          */
    int32_t angle_index;  /* index of the candidate's angle in the full top-layer angle list (:130-144)    */
    int32_t peak_rank;    /* push order of the peak within its angle (0 = the minMaxLoc / s_BlockMax max)  */
    int32_t source;       /* source index within a staged batch (0 for fpm_match)                           */
    int32_t kept;         /* 1: reaches vecAllResult; 0: left the descent at a layer score (:331-332)       */
} fpm_candidate;

/* Restrict this context's searches to shard `shard` of `shards`: the contiguous block
 * [n*shard/shards, n*(shard+1)/shards) of the n top-layer angles.  (0, 1) = the whole list (default).  fpm_match /
 * fpm_match_staged on a sharded context return the results of that block alone. */
int fpm_set_angle_shard(fpm_ctx* ctx, int32_t shard, int32_t shards);
int fpm_get_angle_shard(const fpm_ctx* ctx, int32_t* shard, int32_t* shards);
/* Candidate records of source `source` of the last fpm_match / fpm_match_staged* call, in push order
 * (angle_index ascending, then peak_rank), every top-layer candidate of the context's shard included. */
int fpm_last_candidates(const fpm_ctx* ctx, int32_t source, fpm_candidate* out, int32_t cap, int32_t* n);
/* The coupled tail of TemplateMatcher::match (:214, :262-432) over the candidate records of ONE source: `cand` is
 * the concatenation of every shard's records in shard order (push order; FPM_E_INVALID_ARG otherwise).  Host
 * only, no context or device needed; tmpl_w/tmpl_h = the learned template's level-0 size. */
int fpm_merge_candidates(const fpm_params* p, int32_t tmpl_w, int32_t tmpl_h, const fpm_candidate* cand, int32_t n,
                         fpm_result* out, int32_t cap, int32_t* n_results);

/* --- pixel operators (L1 kernels exposed for parity tests and standalone use) ----------------------- */
/* cv::pyrDown (8U, 5x5 Gaussian, reflect-101), as called by cv::buildPyramid (TemplateMatcher.cpp:55,124).
 * dst is ((w+1)/2) x ((h+1)/2) with row stride dst_stride. */
int fpm_op_pyr_down(fpm_ctx* ctx, const uint8_t* src, int32_t w, int32_t h, size_t src_stride,
                    uint8_t* dst, size_t dst_stride);
/* Two cv::pyrDown levels in one device launch (the search's pyramid kernel, k_pyr_down2): dst1 = pyrDown(src),
 * dst2 = pyrDown(dst1), each with cv::pyrDown's own reflect-101 border at its level (buildPyramid,
 * TemplateMatcher.cpp:124).  Level 1 is walked in chunks of 16 or 32 rows: chunk_rows 16 or 32 forces that
 * height, 0 lets the kernel choose as the search does (32, or 16 where 32-row chunks would leave CUs idle).
 * seg_chunks > 0 gives each workgroup that many chunks of level 1 (runs that start mid-image, as a multi-source
 * search has them); 0 sizes the grid as the search does. */
int fpm_op_pyr_down2(fpm_ctx* ctx, const uint8_t* src, int32_t w, int32_t h, size_t src_stride,
                     uint8_t* dst1, size_t dst1_stride, uint8_t* dst2, size_t dst2_stride, int32_t seg_chunks,
                     int32_t chunk_rows);
/* cv::warpAffine(INTER_LINEAR, BORDER_CONSTANT=border) with forward 2x3 matrix m (row-major), as called at
 * TemplateMatcher.cpp:175 (top layer) and :1089 (getRotatedROI, border 0). */
int fpm_op_warp_affine(fpm_ctx* ctx, const uint8_t* src, int32_t w, int32_t h, size_t src_stride,
                       const double m[6], uint8_t* dst, int32_t dw, int32_t dh, size_t dst_stride,
                       int32_t border);
/* TemplateMatcher::MatchTemplate + CCOEFF_Denominator (TemplateMatcher.cpp:485-598) of `src` against
 * pyramid level `layer` of the learned template.  fold=1 selects the IM_Conv_SIMD per-row float fold
 * (:496-510), fold=0 the TM_CCORR path (:514).  out is (w-tw+1) x (h-th+1) f32, dense. */
int fpm_op_ncc_map(fpm_ctx* ctx, const uint8_t* src, int32_t w, int32_t h, size_t src_stride,
                   int32_t layer, int32_t fold, float* out);
/* filterWithRotatedRect (TemplateMatcher.cpp:1133-1194, with sortPtWithCenter :1093-1131) on n rectangles given as
 * corners[6 i .. 6 i + 5] = ptLT, ptRT, ptRB (cv::RotatedRect(p1, p2, p3), as match() builds them, :380-390) with
 * scores[i], in the caller's order (the reference's: by descending score).  mode 0 runs the host filter, mode 1 the
 * device pair test (k_overlap_pairs, whatever n) with the host replaying its decisions and falling back to the host
 * filter where the device lists cannot hold the pairs -- the two paths of a search's tail.  keep receives the indices
 * of the surviving rectangles in order (*n_keep of them); stats (may be NULL) receives [0] the path taken (0 host,
 * 1 device, 2 device fell back to the host), [1] pairs whose point order the host decided with acos, [2] the device
 * fallback flags (1: a rectangle with more partners than the kernel keeps, 2: the pair list overflowed), [3] the
 * device pair-list entries. */
int fpm_op_overlap_filter(fpm_ctx* ctx, const float* corners, const double* scores, int32_t n, double max_overlap,
                          int32_t mode, int32_t* keep, int32_t* n_keep, int32_t* stats);
/* Learned-template introspection: number of pyramid levels, per-level size and statistics
 * (s_TemplData, DataStructures.h:16-55). */
int fpm_template_info(const fpm_ctx* ctx, int32_t* levels, int32_t* border_color);
int fpm_template_level(const fpm_ctx* ctx, int32_t level, int32_t* w, int32_t* h, double* mean,
                       double* norm, double* inv_area, int32_t* result_equal1, uint8_t* pixels,
                       size_t stride);

/* --- instrumentation -------------------------------------------------------------------------------- */
/* Per-search counters of the last fpm_match / fpm_match_staged call (source 0 for staged batches):
 *   [0] top-layer angles  [1] top-layer candidates  [2..2+L) live candidates entering layer L-1..0
 * Returns the number of entries written. */
int fpm_search_stats(const fpm_ctx* ctx, int64_t* stats, int32_t cap);
/* SURVEY.md §8(d) algorithmic bytes of the last search, summed over its sources: B_pyr (pyramid in + out), B_top
 * (top-layer level read per angle + the f32 maps), B_ref (per live refinement ROI: the source footprint, the template
 * level and the 7x7 f32 scores).  The roofline's achieved bandwidth is these bytes over the measured time. */
int fpm_search_bytes(const fpm_ctx* ctx, int64_t* b_pyr, int64_t* b_top, int64_t* b_ref);

/* Kernel timing: when enabled, HIP events bracket every launch of each kernel on the context's stream (the
 * search then runs eagerly instead of as a replayed graph); fpm_profile_get returns total milliseconds, launch
 * count and algorithmic bytes (compulsory inputs + outputs, u8 = 1 B, f32 = 4 B) accumulated since the last
 * reset (bytes: each kernel's share of SURVEY.md §8(d)'s per-stage figures, as fpm_search_bytes; intermediate
 * scratch of this design is not counted).  One index per kernel. */
#define FPM_K_PYR 0         /* k_pyr_down     K1 pyrDown                                          */
#define FPM_K_TOP_WARP 1    /* k_warp         K2 top-layer rotation                               */
#define FPM_K_TOP_NCC 2     /* k_top_mma / k_ncc_tile / k_ncc_map  K2-K4 top-layer CCORR + norm.  */
#define FPM_K_TOP_NMS 3     /* k_nms / k_nms_greedy  K5 peak extraction                           */
#define FPM_K_CAND_INIT 4   /* k_cand_init    candidates from the top-layer peaks                 */
#define FPM_K_ROI_TABLES 5  /* k_roi_tables   K6a refinement warp tables + tile descriptors       */
#define FPM_K_ROI_WARP 6    /* k_roi_warp     K6b refinement ROI sampling                         */
#define FPM_K_ROI_CORR 7    /* k_roi_corr     K7 refinement row correlation (i8 MFMA) + windows   */
#define FPM_K_ROI_EVAL 8    /* k_roi_eval     K8 row fold, CCOEFF, argmax, 3x3, candidate step    */
#define FPM_K_ROI_SMALL 9   /* k_roi_small    K6-K8 in one kernel for small templates             */
#define FPM_K_CAND_STEP 10  /* k_cand_step    candidate step after k_roi_small                    */
#define FPM_K_TOP_MAP 11    /* k_top_map: full maps of the jobs the list path left (fallback) */
#define FPM_K_COUNT 12
int fpm_profile_enable(fpm_ctx* ctx, int32_t enable);
int fpm_profile_reset(fpm_ctx* ctx);
int fpm_profile_get(const fpm_ctx* ctx, int32_t kernel, double* total_ms, int64_t* launches,
                    int64_t* bytes);
/* Timing of the last fpm_match / fpm_match_staged call (always collected): device_ms = GPU time of the search
 * (events around the whole device pass, results copy included), host_ms = host post-processing after the device
 * pass (reference-order sort, layer-0 decision, filters, conversion), call_ms = wall time of the call. */
int fpm_profile_last(const fpm_ctx* ctx, double* device_ms, double* host_ms, double* call_ms);

#ifdef __cplusplus
}
#endif

#endif /* FPM_H_ */
