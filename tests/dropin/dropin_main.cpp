// TEST DRIVER (tests/dropin): runs a search through the drop-in `TemplateMatcher` (TemplateMatcher_fpm.cpp, the
// replacement of the reference's src/TemplateMatcher.cpp) exactly as the UI calls it (src/MatchToolDialog.cpp:
// 265-286, 358, 1344) and prints every result field as a hex float, plus the class-behaviour checks, for
// tests/test_dropin.py to compare with the CPU oracle.
// usage: dropin_main tmpl.raw tw th src.raw sw sh max_pos max_overlap score tolerance mra use_simd subpixel
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "TemplateMatcher.h"

static cv::Mat read_raw(const char* path, int w, int h) {
    cv::Mat m(h, w, CV_8UC1);
    FILE* f = std::fopen(path, "rb");
    if (!f || std::fread(m.data, 1, (size_t)w * h, f) != (size_t)w * h) { std::fprintf(stderr, "read %s\n", path); std::exit(2); }
    std::fclose(f);
    return m;
}

static void print_results(const char* tag, const std::vector<s_SingleTargetMatch>& r) {
    for (const s_SingleTargetMatch& m : r)
        std::printf("%s %a %a %a %a %a %a %a %a %a %a %a %a\n", tag, m.ptLT.x, m.ptLT.y, m.ptRT.x, m.ptRT.y, m.ptRB.x,
                    m.ptRB.y, m.ptLB.x, m.ptLB.y, m.ptCenter.x, m.ptCenter.y, m.dMatchedAngle, m.dMatchScore);
}

static bool same(const std::vector<s_SingleTargetMatch>& a, const std::vector<s_SingleTargetMatch>& b) {
    if (a.size() != b.size()) return false;
    for (size_t i = 0; i < a.size(); ++i)
        if (std::memcmp(&a[i], &b[i], sizeof(s_SingleTargetMatch)) != 0) return false;
    return true;
}

int main(int argc, char** argv) {
    if (argc != 14) { std::fprintf(stderr, "usage: see header\n"); return 2; }
    cv::Mat tmpl = read_raw(argv[1], std::atoi(argv[2]), std::atoi(argv[3]));
    cv::Mat src = read_raw(argv[4], std::atoi(argv[5]), std::atoi(argv[6]));
    TemplateMatcher m;
    std::printf("CHECK learned_before %d\n", m.isPatternLearned() ? 1 : 0);
    std::printf("CHECK empty_learn %d\n", m.learnPattern(cv::Mat()) ? 1 : 0);
    m.setUserDefinedRect(cv::Rect(3, 4, 50, 60));
    std::printf("CHECK rect_set %d\n", (m.hasUserDefinedRect() && m.getUserDefinedRect() == cv::Rect(3, 4, 50, 60)) ? 1 : 0);
    // MatchToolDialog order: learn on template load (:358) with the object's MinReduceArea at that time (the
    // constructor's 256 before the first Execute), then on Execute the setters (:265-271, MinReduceArea included)
    // and match (:286) -- no re-learn: match() takes its top layer from the current MinReduceArea (TemplateMatcher.cpp:120)
    std::printf("CHECK learn %d\n", m.learnPattern(tmpl) ? 1 : 0);
    std::printf("CHECK rect_reset_by_learn %d\n", m.hasUserDefinedRect() ? 0 : 1);   // m_TemplData.clear() (:51)
    m.setMaxPositions(std::atoi(argv[7]));
    m.setMaxOverlap(std::atof(argv[8]));
    m.setScore(std::atof(argv[9]));
    m.setToleranceAngle(std::atof(argv[10]));
    m.setMinReduceArea(std::atoi(argv[11]));
    m.setUseSIMD(std::atoi(argv[12]) != 0);
    m.setSubPixelEstimation(std::atoi(argv[13]) != 0);
    std::vector<s_SingleTargetMatch> results = m.match(src);
    print_results("R", results);
    const double t1 = m.getLastExecutionTime();
    std::printf("CHECK time_positive %d\n", (results.empty() || t1 > 0) ? 1 : 0);
    // a copy of the object (implicit copy constructor) searches the same template on its own context
    {
        TemplateMatcher c = m;
        std::printf("CHECK copy_same %d\n", same(c.match(src), results) ? 1 : 0);
    }
    std::printf("CHECK again_same %d\n", same(m.match(src), results) ? 1 : 0);
    // nothing found keeps the previous execution time (:398-404)
    cv::Mat flat(src.rows, src.cols, CV_8UC1);
    const double t2 = m.getLastExecutionTime();
    std::printf("CHECK none_found %d\n", m.match(flat).empty() ? 1 : 0);
    std::printf("CHECK time_kept %d\n", m.getLastExecutionTime() == t2 ? 1 : 0);
    m.setUserDefinedRect(cv::Rect());   // MatchToolDialog.cpp:1344, 1366
    std::printf("CHECK rect_cleared %d\n", (m.hasUserDefinedRect() && m.getUserDefinedRect() == cv::Rect()) ? 1 : 0);
    m.clearPattern();
    std::printf("CHECK cleared %d\n", (!m.isPatternLearned() && m.match(src).empty()) ? 1 : 0);
    cv::Mat color(src.rows, src.cols, CV_8UC3);
    std::printf("CHECK color_refused %d\n", m.learnPattern(color) ? 0 : 1);
    return 0;
}
