// TemplateMatcher_fpm.cpp — the drop-in replacement for the reference's src/TemplateMatcher.cpp.
//
// It defines the reference's own `class TemplateMatcher` (declared, unchanged, in the reference's
// include/TemplateMatcher.h:9-90) on top of the MI355X matcher's C ABI (include/fpm.h, libfpm_hip.so).  A maintainer
// swaps one line of the reference build — src/TemplateMatcher.cpp -> this file in the SOURCES list
// (CMakeLists.txt:104-110) — and links libfpm_hip.so; TemplateMatcher.h, DataStructures.h, MatchToolDialog and the
// rest of the UI stay untouched: `m_matchResults = m_matcher.match(m_sourceImage)` (src/MatchToolDialog.cpp:286)
// still returns std::vector<s_SingleTargetMatch>, `m_matcher.setUserDefinedRect(cv::Rect())` (:1344, :1366) still
// takes a cv::Rect.  INTEGRATION.md shows the build change.
//
// The header declares no member for a device context, so each object's fpm_ctx lives in a side table keyed by the
// object's address (created in the constructor, destroyed in the destructor).  The reference class is copyable by
// its implicit copy constructor / assignment; a copy has no table entry (or a stale one) and gets its own context on
// first use, re-learning the template from m_TemplData.vecPyramid[0] — which, as in the reference, shares the
// learned image's pixels (cv::buildPyramid's level 0 is the input Mat, TemplateMatcher.cpp:55).
//
// Behaviour kept from the reference (file:line of src/TemplateMatcher.cpp):
//   constructor defaults (:28-39) — the setters are inline in the header and write the members read here;
//   learnPattern: false on an empty image (:47-49), m_TemplData.clear() first, so the user rectangle is reset too
//     (:51, DataStructures.h:27-35);
//   match: empty vector on an empty source / unlearned template / size mismatch (:99-114); results sorted by score,
//     s_SingleTargetMatch fields as :406-432; m_dLastExecutionTime updated only when there is a result (:398-404),
//     timed from after the source copy (:104, :117);
//   clearPattern (:439-443), set/get/hasUserDefinedRect (:1224-1238): stored only.
// Differences: images must be CV_8UC1 (what the UI loads, src/MatchToolDialog.cpp:314, 341; the reference does not
// check the type) — anything else is treated like an empty image; the device is FPM_DEVICE (default 0).
#include "TemplateMatcher.h"

#include <cstdlib>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "fpm.h"

namespace {

struct FpmSlot {
    fpm_ctx* ctx = nullptr;
    const unsigned char* learned = nullptr;   // pixels the context's template was learned from
    int learned_w = 0, learned_h = 0;
    std::vector<fpm_result> buf;
};

std::mutex g_mu;
std::unordered_map<const TemplateMatcher*, FpmSlot>& slots() {
    static std::unordered_map<const TemplateMatcher*, FpmSlot> m;
    return m;
}

int fpm_device() {
    const char* e = std::getenv("FPM_DEVICE");
    return e ? std::atoi(e) : 0;
}

// this object's slot, creating its context on first use (nullptr when no gfx950 device / HIP runtime)
FpmSlot* slot_of(const TemplateMatcher* self) {
    std::lock_guard<std::mutex> lock(g_mu);
    FpmSlot& s = slots()[self];
    if (!s.ctx && fpm_create(fpm_device(), &s.ctx) != FPM_OK) s.ctx = nullptr;
    return s.ctx ? &s : nullptr;
}

bool is_gray8(const cv::Mat& m) { return !m.empty() && m.type() == CV_8UC1; }

}  // namespace

TemplateMatcher::TemplateMatcher()
    : m_iMaxPos(70)
    , m_dMaxOverlap(0.0)
    , m_dScore(0.7)
    , m_dToleranceAngle(0.0)
    , m_iMinReduceArea(256)
    , m_bUseSIMD(true)
    , m_bSubPixelEstimation(false)
    , m_dLastExecutionTime(0.0)
{
    m_bToleranceRange = false;
    m_dTolerance1 = m_dTolerance2 = m_dTolerance3 = m_dTolerance4 = 0.0;
    (void)slot_of(this);
}

TemplateMatcher::~TemplateMatcher()
{
    std::lock_guard<std::mutex> lock(g_mu);
    auto it = slots().find(this);
    if (it == slots().end()) return;
    if (it->second.ctx) fpm_destroy(it->second.ctx);
    slots().erase(it);
}

static void fill_params(fpm_params* p, int max_pos, double overlap, double score, double tol, int mra, bool simd,
                        bool subpixel, bool range)
{
    fpm_params_default(p);
    p->max_pos = max_pos;
    p->max_overlap = overlap;
    p->score = score;
    p->tolerance_angle = tol;
    p->min_reduce_area = mra;
    p->use_simd = simd ? 1 : 0;
    p->subpixel = subpixel ? 1 : 0;
    p->tolerance_range = range ? 1 : 0;
}

bool TemplateMatcher::learnPattern(const cv::Mat& templateImage)
{
    if (templateImage.empty()) return false;
    m_TemplData.clear();
    m_TemplData.bIsPatternLearned = false;
    if (!is_gray8(templateImage)) return false;
    FpmSlot* s = slot_of(this);
    if (!s) return false;
    fpm_params p;
    fill_params(&p, m_iMaxPos, m_dMaxOverlap, m_dScore, m_dToleranceAngle, m_iMinReduceArea, m_bUseSIMD,
                m_bSubPixelEstimation, m_bToleranceRange);
    if (fpm_set_params(s->ctx, &p) != FPM_OK) return false;
    if (fpm_learn(s->ctx, templateImage.data, templateImage.cols, templateImage.rows, templateImage.step[0]) != FPM_OK)
        return false;
    s->learned = templateImage.data;
    s->learned_w = templateImage.cols;
    s->learned_h = templateImage.rows;
    m_TemplData.vecPyramid.assign(1, templateImage);   // level 0 shares the caller's pixels, as buildPyramid's does
    m_TemplData.bIsPatternLearned = true;
    return true;
}

std::vector<s_SingleTargetMatch> TemplateMatcher::match(const cv::Mat& sourceImage)
{
    std::vector<s_SingleTargetMatch> out;
    if (sourceImage.empty() || !m_TemplData.bIsPatternLearned || m_TemplData.vecPyramid.empty()) return out;
    if (!is_gray8(sourceImage)) return out;
    FpmSlot* s = slot_of(this);
    if (!s) return out;
    fpm_params p;
    fill_params(&p, m_iMaxPos, m_dMaxOverlap, m_dScore, m_dToleranceAngle, m_iMinReduceArea, m_bUseSIMD,
                m_bSubPixelEstimation, m_bToleranceRange);
    if (fpm_set_params(s->ctx, &p) != FPM_OK) return out;
    const cv::Mat& t0 = m_TemplData.vecPyramid[0];
    if (s->learned != t0.data || s->learned_w != t0.cols || s->learned_h != t0.rows) {   // a copied / assigned object
        if (fpm_learn(s->ctx, t0.data, t0.cols, t0.rows, t0.step[0]) != FPM_OK) return out;
        s->learned = t0.data;
        s->learned_w = t0.cols;
        s->learned_h = t0.rows;
    }
    if (s->buf.empty()) s->buf.resize(256);
    int32_t n = 0;
    double seconds = m_dLastExecutionTime;
    int rc = fpm_match(s->ctx, sourceImage.data, sourceImage.cols, sourceImage.rows, sourceImage.step[0], s->buf.data(),
                       (int32_t)s->buf.size(), &n, &seconds);
    if (rc == FPM_E_CAPACITY) {   // more results than the buffer: fetch the ones just computed, no second search
        s->buf.resize((size_t)n);
        rc = fpm_last_results(s->ctx, s->buf.data(), (int32_t)s->buf.size(), &n);
    }
    if (rc != FPM_OK) return out;
    m_dLastExecutionTime = seconds;   // unchanged by fpm_match when there is no result (:398-404)
    out.reserve((size_t)n);
    for (int i = 0; i < n; ++i) {
        const fpm_result& r = s->buf[(size_t)i];
        s_SingleTargetMatch m;
        m.ptLT = cv::Point2d(r.lt_x, r.lt_y);
        m.ptRT = cv::Point2d(r.rt_x, r.rt_y);
        m.ptRB = cv::Point2d(r.rb_x, r.rb_y);
        m.ptLB = cv::Point2d(r.lb_x, r.lb_y);
        m.ptCenter = cv::Point2d(r.cx, r.cy);
        m.dMatchedAngle = r.angle;
        m.dMatchScore = r.score;
        out.push_back(m);
    }
    return out;
}

void TemplateMatcher::clearPattern()
{
    m_TemplData.clear();
    m_TemplData.bIsPatternLearned = false;
    std::lock_guard<std::mutex> lock(g_mu);
    auto it = slots().find(this);
    if (it != slots().end() && it->second.ctx) {
        fpm_clear_pattern(it->second.ctx);
        it->second.learned = nullptr;
    }
}

void TemplateMatcher::setUserDefinedRect(const cv::Rect& rect)
{
    m_TemplData.userDefinedRect = rect;
    m_TemplData.hasUserRect = true;
}

cv::Rect TemplateMatcher::getUserDefinedRect() const { return m_TemplData.userDefinedRect; }

bool TemplateMatcher::hasUserDefinedRect() const { return m_TemplData.hasUserRect; }
