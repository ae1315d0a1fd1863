// fpm_template_matcher.hpp — header-only C++ mirror of the reference's TemplateMatcher over the fpm C ABI.
//
// Same method names, argument meaning and error behaviour as include/TemplateMatcher.h:9-51 of
// lrm2017/Fastest_Image_Pattern_Matching, so a caller (e.g. MatchToolDialog, src/MatchToolDialog.cpp:265-377)
// switches by changing the include and the type name.  Images are passed as (pointer, width, height, stride)
// of 8-bit gray pixels; when OpenCV is available, cv::Mat overloads identical to the reference's are compiled
// too.  Results use fpm::SingleTargetMatch, field-for-field s_SingleTargetMatch (DataStructures.h:97-115).
#ifndef FPM_TEMPLATE_MATCHER_HPP_
#define FPM_TEMPLATE_MATCHER_HPP_

#include <stdexcept>
#include <string>
#include <vector>

#include "fpm.h"

#if defined(__has_include)
#if __has_include(<opencv2/core.hpp>)
#include <opencv2/core.hpp>
#define FPM_HAVE_OPENCV 1
#endif
#endif

namespace fpm {

struct Point2d {
    double x = 0, y = 0;
};

// s_SingleTargetMatch (DataStructures.h:97-115)
struct SingleTargetMatch {
    Point2d ptLT, ptRT, ptRB, ptLB, ptCenter;
    double dMatchedAngle = 0;
    double dMatchScore = 0;
};

class TemplateMatcher {
public:
    // TemplateMatcher::TemplateMatcher (TemplateMatcher.cpp:28-39): defaults from fpm_params_default.
    explicit TemplateMatcher(int device = 0) {
        fpm_params_default(&p_);
        if (fpm_create(device, &ctx_) != FPM_OK)
            throw std::runtime_error("fpm_create failed: no gfx950 device or HIP runtime");
    }
    ~TemplateMatcher() { if (ctx_) fpm_destroy(ctx_); }
    TemplateMatcher(const TemplateMatcher&) = delete;
    TemplateMatcher& operator=(const TemplateMatcher&) = delete;

    // learnPattern (TemplateMatcher.cpp:45-95): false on an empty image.
    bool learnPattern(const uint8_t* gray, int width, int height, size_t stride) {
        if (!gray || width <= 0 || height <= 0) return false;
        if (fpm_set_params(ctx_, &p_) != FPM_OK) return false;
        return fpm_learn(ctx_, gray, width, height, stride) == FPM_OK;
    }
    // match (TemplateMatcher.cpp:97-437): empty vector when unlearned / empty / too small / nothing found.
    std::vector<SingleTargetMatch> match(const uint8_t* gray, int width, int height, size_t stride) {
        std::vector<SingleTargetMatch> out;
        if (!gray || width <= 0 || height <= 0 || !isPatternLearned()) return out;
        if (fpm_set_params(ctx_, &p_) != FPM_OK) return out;
        std::vector<fpm_result> buf((size_t)cap_);
        int32_t n = 0;
        double sec = last_time_;
        int rc = fpm_match(ctx_, gray, width, height, stride, buf.data(), cap_, &n, &sec);
        if (rc == FPM_E_CAPACITY) {
            cap_ = n;
            buf.resize((size_t)cap_);
            rc = fpm_match(ctx_, gray, width, height, stride, buf.data(), cap_, &n, &sec);
        }
        if (rc != FPM_OK) return out;
        last_time_ = sec;
        out.reserve((size_t)n);
        for (int i = 0; i < n; ++i) out.push_back(convert(buf[(size_t)i]));
        return out;
    }
#ifdef FPM_HAVE_OPENCV
    bool learnPattern(const cv::Mat& templateImage) {
        if (templateImage.empty() || templateImage.type() != CV_8UC1) return false;
        return learnPattern(templateImage.data, templateImage.cols, templateImage.rows, templateImage.step[0]);
    }
    std::vector<SingleTargetMatch> match(const cv::Mat& sourceImage) {
        if (sourceImage.empty() || sourceImage.type() != CV_8UC1) return {};
        return match(sourceImage.data, sourceImage.cols, sourceImage.rows, sourceImage.step[0]);
    }
#endif

    // setters / getters (TemplateMatcher.h:22-37)
    void setMaxPositions(int v) { p_.max_pos = v; }
    void setMaxOverlap(double v) { p_.max_overlap = v; }
    void setScore(double v) { p_.score = v; }
    void setToleranceAngle(double v) { p_.tolerance_angle = v; }
    void setMinReduceArea(int v) { p_.min_reduce_area = v; }
    void setUseSIMD(bool v) { p_.use_simd = v ? 1 : 0; }
    void setSubPixelEstimation(bool v) { p_.subpixel = v ? 1 : 0; }
    int getMaxPositions() const { return p_.max_pos; }
    double getMaxOverlap() const { return p_.max_overlap; }
    double getScore() const { return p_.score; }
    double getToleranceAngle() const { return p_.tolerance_angle; }
    int getMinReduceArea() const { return p_.min_reduce_area; }
    bool getUseSIMD() const { return p_.use_simd != 0; }
    bool getSubPixelEstimation() const { return p_.subpixel != 0; }
    double getLastExecutionTime() const { return last_time_; }   // seconds (:398-404)

    bool isPatternLearned() const { return fpm_is_learned(ctx_) == 1; }
    void clearPattern() { fpm_clear_pattern(ctx_); }
    // user-defined rect: stored only, unused by matching (TemplateMatcher.h:45-51)
    void setUserDefinedRect(int x, int y, int w, int h) { rect_[0] = x; rect_[1] = y; rect_[2] = w; rect_[3] = h; has_rect_ = true; }
    bool hasUserDefinedRect() const { return has_rect_; }
    const int* getUserDefinedRect() const { return rect_; }

    // angle sharding of one search across ranks (fpm.h): search this rank's block of the top-layer
    // angle list, export its candidate records, and merge every rank's records (rank order) on any host
    bool setAngleShard(int shard, int shards) { return fpm_set_angle_shard(ctx_, shard, shards) == FPM_OK; }
    std::vector<fpm_candidate> lastCandidates(int source = 0) const {
        int32_t n = 0;
        fpm_last_candidates(ctx_, source, nullptr, 0, &n);
        std::vector<fpm_candidate> out((size_t)n);
        if (n > 0 && fpm_last_candidates(ctx_, source, out.data(), n, &n) != FPM_OK) out.clear();
        return out;
    }
    std::vector<SingleTargetMatch> mergeCandidates(const std::vector<fpm_candidate>& all) const {
        std::vector<SingleTargetMatch> out;
        int32_t levels = 0, border = 0, tw = 0, th = 0, eq = 0;
        double mean = 0, norm = 0, inv = 0;
        if (fpm_template_info(ctx_, &levels, &border) != FPM_OK ||
            fpm_template_level(ctx_, 0, &tw, &th, &mean, &norm, &inv, &eq, nullptr, 0) != FPM_OK)
            return out;
        std::vector<fpm_result> buf(all.size() + 1);
        int32_t n = 0;
        if (fpm_merge_candidates(&p_, tw, th, all.data(), (int32_t)all.size(), buf.data(), (int32_t)buf.size(), &n) != FPM_OK)
            return out;
        for (int i = 0; i < n; ++i) out.push_back(convert(buf[(size_t)i]));
        return out;
    }

    std::string lastError() const { const char* s = fpm_last_error(ctx_); return s ? s : ""; }
    fpm_ctx* context() const { return ctx_; }

private:
    static SingleTargetMatch convert(const fpm_result& r) {
        SingleTargetMatch m;
        m.ptLT = {r.lt_x, r.lt_y}; m.ptRT = {r.rt_x, r.rt_y}; m.ptRB = {r.rb_x, r.rb_y}; m.ptLB = {r.lb_x, r.lb_y};
        m.ptCenter = {r.cx, r.cy};
        m.dMatchedAngle = r.angle;
        m.dMatchScore = r.score;
        return m;
    }
    fpm_ctx* ctx_ = nullptr;
    fpm_params p_{};
    int32_t cap_ = 1024;
    double last_time_ = 0;
    int rect_[4] = {0, 0, 0, 0};
    bool has_rect_ = false;
};

}  // namespace fpm

#endif  // FPM_TEMPLATE_MATCHER_HPP_
