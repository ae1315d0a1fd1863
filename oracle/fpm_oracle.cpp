// fpm_oracle.cpp — TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference's hot path.
//
// This file is the parity oracle for the MI355X matcher.  Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg may load it (as liboracle_fpm.so); the product library never links it.
//
// What it restates (reference = lrm2017/Fastest_Image_Pattern_Matching @ /root/reference):
//   * src/TemplateMatcher.cpp:45-598, 901-1221  (learnPattern, match, getTopLayer, IM_Conv_SIMD,
//     MatchTemplate, CCOEFF_Denominator, getBestRotationSize, ptRotatePt2f, filterWithScore,
//     subPixEstimation, getRotatedROI, sortPtWithCenter, filterWithRotatedRect, getNextMaxLoc x2)
//   * include/DataStructures.h:10-246          (s_TemplData, s_MatchParameter, s_BlockMax)
//   * the OpenCV primitives those call, per SURVEY.md Appendix A (OpenCV 4.5.x CPU, non-IPP):
//     buildPyramid/pyrDown, getRotationMatrix2D, warpAffine(INTER_LINEAR, BORDER_CONSTANT), integral,
//     meanStdDev, minMaxLoc, rectangle(FILLED), RotatedRect, rotatedRectangleIntersection, contourArea.
//
// Pinning.  The reference cannot be compiled here (OpenCV absent), so this restatement is
// pinned by constructed known-answer tests (tests/test_oracle_kat.py) and by the committed golden vectors
// it generated (tests/golden/).  Against real OpenCV the parity is UNPINNED; the one intentional deviation
// is TM_CCORR, restated as the exact integer sum rounded once to f32 (Appendix A.4).  A test-only second mode
// (orc_set_ccorr_mode(h, 1)) computes TM_CCORR as OpenCV's crossCorr does, in float32 DFTs, to measure how the
// reference's screenshots respond to that arithmetic (cross_corr_f32 below; tests/test_reference_pins.py).
//
// Build: oracle/Makefile (g++ -O3, -ffp-contract=off, no -ffast-math: the float/double operation order
// below IS the contract).
#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <emmintrin.h>
#include <vector>

#include "../include/fpm.h"

namespace orc {

static const double kPi = 3.1415926535897932384626433832795;  // CV_PI
static const double D2R = kPi / 180.0;                         // DataStructures.h:11
static const double R2D = 180.0 / kPi;                         // DataStructures.h:12
static const double VISION_TOLERANCE = 0.0000001;              // DataStructures.h:10
static const int MATCH_CANDIDATE_NUM = 5;                      // DataStructures.h:13

struct P2f { float x = 0, y = 0; P2f() {} P2f(float a, float b) : x(a), y(b) {} };
struct P2d { double x = 0, y = 0; P2d() {} P2d(double a, double b) : x(a), y(b) {} };
struct RectI { int x = 0, y = 0, w = 0, h = 0; RectI() {} RectI(int a, int b, int c, int d) : x(a), y(b), w(c), h(d) {} };

// cv::Rect::operator&  (intersection; empty -> all zero)
static RectI rect_and(const RectI& a, const RectI& b) {
    int x1 = std::max(a.x, b.x), y1 = std::max(a.y, b.y);
    int w = std::min(a.x + a.w, b.x + b.w) - x1;
    int h = std::min(a.y + a.h, b.y + b.h) - y1;
    if (w <= 0 || h <= 0) return RectI();
    return RectI(x1, y1, w, h);
}

struct Mat8 {
    int w = 0, h = 0;
    std::vector<uint8_t> px;
    Mat8() {}
    Mat8(int w_, int h_, uint8_t v = 0) : w(w_), h(h_), px((size_t)w_ * h_, v) {}
    uint8_t* row(int y) { return px.data() + (size_t)y * w; }
    const uint8_t* row(int y) const { return px.data() + (size_t)y * w; }
    bool empty() const { return w <= 0 || h <= 0; }
};

struct MatF {
    int w = 0, h = 0;
    std::vector<float> px;
    MatF() {}
    MatF(int w_, int h_, float v = 0.f) : w(w_), h(h_), px((size_t)w_ * h_, v) {}
    float& at(int y, int x) { return px[(size_t)y * w + x]; }
    float at(int y, int x) const { return px[(size_t)y * w + x]; }
};

// ---------------------------------------------------------------------------------------------------
// OpenCV primitives
// ---------------------------------------------------------------------------------------------------

// borderInterpolate(p, n, BORDER_REFLECT_101)
static inline int reflect101(int p, int n) {
    if (n == 1) return 0;
    while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
    return p;
}

// cv::pyrDown 8U (A.1): out = (sum_{i,j} k_i k_j src(r101(2x+i-2), r101(2y+j-2)) + 128) >> 8.
static Mat8 pyr_down(const Mat8& s) {
    static const int k[5] = {1, 4, 6, 4, 1};
    Mat8 d((s.w + 1) / 2, (s.h + 1) / 2);
    std::vector<int> xi((size_t)d.w * 5);
    for (int x = 0; x < d.w; ++x)
        for (int i = 0; i < 5; ++i) xi[(size_t)x * 5 + i] = reflect101(2 * x + i - 2, s.w);
    std::vector<int> rowsum((size_t)5 * d.w);
    for (int y = 0; y < d.h; ++y) {
        for (int j = 0; j < 5; ++j) {
            const uint8_t* r = s.row(reflect101(2 * y + j - 2, s.h));
            int* o = &rowsum[(size_t)j * d.w];
            for (int x = 0; x < d.w; ++x) {
                const int* c = &xi[(size_t)x * 5];
                o[x] = r[c[0]] + 4 * r[c[1]] + 6 * r[c[2]] + 4 * r[c[3]] + r[c[4]];
            }
        }
        uint8_t* out = d.row(y);
        for (int x = 0; x < d.w; ++x) {
            int v = 0;
            for (int j = 0; j < 5; ++j) v += k[j] * rowsum[(size_t)j * d.w + x];
            out[x] = (uint8_t)((v + 128) >> 8);
        }
    }
    return d;
}

// cv::buildPyramid(src, dst, maxlevel): dst[0] = src, dst[i] = pyrDown(dst[i-1])  (A.1)
static std::vector<Mat8> build_pyramid(const Mat8& src, int max_level) {
    std::vector<Mat8> v;
    v.push_back(src);
    for (int i = 1; i <= max_level; ++i) v.push_back(pyr_down(v.back()));
    return v;
}

// cv::getRotationMatrix2D(center, angle_deg, 1)  (A.2)
static void rotation_matrix(P2f c, double angle, double m[6]) {
    angle *= kPi / 180;
    double alpha = std::cos(angle) * 1.0;
    double beta = std::sin(angle) * 1.0;
    m[0] = alpha; m[1] = beta; m[2] = (1 - alpha) * c.x - beta * c.y;
    m[3] = -beta; m[4] = alpha; m[5] = beta * c.x + (1 - alpha) * c.y;
}

static inline int cv_round(double v) { return (int)std::lrint(v); }   // saturate_cast<int>(double)
static inline short sat_short(int v) { return (short)std::min(std::max(v, -32768), 32767); }

// cv::warpAffine(src, dst, M, dsize, INTER_LINEAR, BORDER_CONSTANT, border)  (A.3)
static Mat8 warp_affine(const Mat8& src, const double m_in[6], int dw, int dh, int border) {
    double M[6];
    std::memcpy(M, m_in, sizeof(M));
    {   // invert the forward map (warpAffine without WARP_INVERSE_MAP)
        double D = M[0] * M[4] - M[1] * M[3];
        D = D != 0 ? 1. / D : 0;
        double A11 = M[4] * D, A22 = M[0] * D;
        M[0] = A11; M[1] *= -D;
        M[3] *= -D; M[4] = A22;
        double b1 = -M[0] * M[2] - M[1] * M[5];
        double b2 = -M[3] * M[2] - M[4] * M[5];
        M[2] = b1; M[5] = b2;
    }
    const int AB_BITS = 10, AB_SCALE = 1 << AB_BITS, INTER_BITS = 5, INTER_TAB = 1 << INTER_BITS;
    const int round_delta = AB_SCALE / INTER_TAB / 2;
    std::vector<int> adelta(dw), bdelta(dw);
    for (int x = 0; x < dw; ++x) {
        adelta[x] = cv_round(M[0] * x * AB_SCALE);
        bdelta[x] = cv_round(M[3] * x * AB_SCALE);
    }
    Mat8 dst(dw, dh);
    const unsigned width1 = (unsigned)std::max(src.w - 1, 0), height1 = (unsigned)std::max(src.h - 1, 0);
    const uint8_t cval = (uint8_t)std::min(std::max(border, 0), 255);
    for (int y = 0; y < dh; ++y) {
        int X0 = cv_round((M[1] * y + M[2]) * AB_SCALE) + round_delta;
        int Y0 = cv_round((M[4] * y + M[5]) * AB_SCALE) + round_delta;
        uint8_t* D = dst.row(y);
        for (int x = 0; x < dw; ++x) {
            int X = (X0 + adelta[x]) >> (AB_BITS - INTER_BITS);
            int Y = (Y0 + bdelta[x]) >> (AB_BITS - INTER_BITS);
            int sx = sat_short(X >> INTER_BITS), sy = sat_short(Y >> INTER_BITS);
            int fx = X & (INTER_TAB - 1), fy = Y & (INTER_TAB - 1);
            // BilinearTab_i (initInterTab2D, INTER_LINEAR): exact products, sum 32768.  The (0,0) entry
            // saturates to {32767,0,0,1}; with fx=fy=0 either table gives v0 exactly, so we use the
            // exact form.
            int w0 = (INTER_TAB - fy) * (INTER_TAB - fx) * 32, w1 = (INTER_TAB - fy) * fx * 32;
            int w2 = fy * (INTER_TAB - fx) * 32, w3 = fy * fx * 32;
            int v0, v1, v2, v3;
            if ((unsigned)sx < width1 && (unsigned)sy < height1) {
                const uint8_t* S = src.row(sy) + sx;
                v0 = S[0]; v1 = S[1]; v2 = S[src.w]; v3 = S[src.w + 1];
            } else if (sx >= src.w || sx + 1 < 0 || sy >= src.h || sy + 1 < 0) {
                D[x] = cval;
                continue;
            } else {
                bool x0in = sx >= 0 && sx < src.w, x1in = sx + 1 >= 0 && sx + 1 < src.w;
                bool y0in = sy >= 0 && sy < src.h, y1in = sy + 1 >= 0 && sy + 1 < src.h;
                v0 = x0in && y0in ? src.row(sy)[sx] : cval;
                v1 = x1in && y0in ? src.row(sy)[sx + 1] : cval;
                v2 = x0in && y1in ? src.row(sy + 1)[sx] : cval;
                v3 = x1in && y1in ? src.row(sy + 1)[sx + 1] : cval;
            }
            int v = (v0 * w0 + v1 * w1 + v2 * w2 + v3 * w3 + (1 << 14)) >> 15;
            D[x] = (uint8_t)std::min(std::max(v, 0), 255);
        }
    }
    return dst;
}

// cv::meanStdDev on 8UC1 (A.6): exact S, SQ; scale = 1/N; mean = S*scale; sdv = sqrt(max(SQ*scale-m^2,0))
static void mean_stddev(const Mat8& m, double* mean, double* sdv) {
    int64_t s = 0, sq = 0;
    for (uint8_t v : m.px) { s += v; sq += (int64_t)v * v; }
    double scale = m.px.empty() ? 0. : 1. / (double)m.px.size();
    double ds = (double)s * scale;
    *mean = ds;
    *sdv = std::sqrt(std::max((double)sq * scale - ds * ds, 0.));
}

// cv::minMaxLoc maximum: first occurrence, row-major, strict '>'  (A.7).  An empty ROI (a zero-width s_BlockMax strip)
// gives 0 at (-1, -1): cv::minMaxIdx leaves its index at 0 for an empty array, which reads as value 0 and a location
// of -1 in every dimension
static void max_loc(const MatF& m, int x0, int y0, int w, int h, double* vmax, int* lx, int* ly) {
    if (w <= 0 || h <= 0) { *vmax = 0; *lx = -1; *ly = -1; return; }
    float best = m.at(y0, x0);
    int bx = 0, by = 0;
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            float v = m.at(y0 + y, x0 + x);
            if (v > best) { best = v; bx = x; by = y; }
        }
    *vmax = best; *lx = bx; *ly = by;
}

// cv::rectangle(img, Rect, Scalar(v), FILLED)  (A.8)
static void fill_rect(MatF& m, RectI r, float v) {
    if (r.w <= 0 || r.h <= 0) return;
    int x1 = std::max(r.x, 0), y1 = std::max(r.y, 0);
    int x2 = std::min(r.x + r.w - 1, m.w - 1), y2 = std::min(r.y + r.h - 1, m.h - 1);
    for (int y = y1; y <= y2; ++y)
        for (int x = x1; x <= x2; ++x) m.at(y, x) = v;
}

// ---- rotated rectangles (A.9) -----------------------------------------------------------------------
struct RotRect { P2f c; float w = 0, h = 0, angle = 0; };

static inline double norm2f(float x, float y) { return std::sqrt((double)x * x + (double)y * y); }

// cv::RotatedRect(p1, p2, p3)
static RotRect rotrect_from3(P2f p1, P2f p2, P2f p3) {
    RotRect r;
    r.c = P2f(0.5f * (p1.x + p3.x), 0.5f * (p1.y + p3.y));
    float v0x = p1.x - p2.x, v0y = p1.y - p2.y, v1x = p2.x - p3.x, v1y = p2.y - p3.y;
    // (the reference's perpendicularity CV_Assert is not restated: it can only abort)
    int wd = std::fabs(v1y) < std::fabs(v1x) ? 1 : 0;
    float wx = wd ? v1x : v0x, wy = wd ? v1y : v0y, hx = wd ? v0x : v1x, hy = wd ? v0y : v1y;
    r.angle = std::atan(wy / wx) * 180.0f / (float)kPi;
    r.w = (float)norm2f(wx, wy);
    r.h = (float)norm2f(hx, hy);
    return r;
}

// cv::RotatedRect::points
static void rotrect_points(const RotRect& r, P2f pt[4]) {
    double a_ = r.angle * kPi / 180.;
    float b = (float)std::cos(a_) * 0.5f;
    float a = (float)std::sin(a_) * 0.5f;
    pt[0].x = r.c.x - a * r.h - b * r.w;
    pt[0].y = r.c.y + b * r.h - a * r.w;
    pt[1].x = r.c.x + a * r.h - b * r.w;
    pt[1].y = r.c.y - b * r.h - a * r.w;
    pt[2].x = 2 * r.c.x - pt[0].x;
    pt[2].y = 2 * r.c.y - pt[0].y;
    pt[3].x = 2 * r.c.x - pt[1].x;
    pt[3].y = 2 * r.c.y - pt[1].y;
}

enum { INTERSECT_NONE = 0, INTERSECT_PARTIAL = 1, INTERSECT_FULL = 2 };

// cv::rotatedRectangleIntersection (OpenCV 4.5.x)
static int rotrect_intersection(const RotRect& r1, const RotRect& r2, std::vector<P2f>& out) {
    out.clear();
    float eps = 1e-6f * std::max(r1.w * r1.h, r2.w * r2.h);
    P2f p1[4], p2[4], v1[4], v2[4];
    rotrect_points(r1, p1);
    rotrect_points(r2, p2);
    bool same = true;
    for (int i = 0; i < 4; ++i)
        if (std::fabs(p1[i].x - p2[i].x) > eps || std::fabs(p1[i].y - p2[i].y) > eps) { same = false; break; }
    if (same) {
        for (int i = 0; i < 4; ++i) out.push_back(p1[i]);
        return INTERSECT_FULL;
    }
    for (int i = 0; i < 4; ++i) {
        v1[i] = P2f(p1[(i + 1) % 4].x - p1[i].x, p1[(i + 1) % 4].y - p1[i].y);
        v2[i] = P2f(p2[(i + 1) % 4].x - p2[i].x, p2[(i + 1) % 4].y - p2[i].y);
    }
    for (int i = 0; i < 4; ++i) {
        eps = std::min(eps, std::sqrt(v1[i].x * v1[i].x + v1[i].y * v1[i].y));
        eps = std::min(eps, std::sqrt(v2[i].x * v2[i].x + v2[i].y * v2[i].y));
    }
    eps = std::max(1e-16f, eps);
    int ret = INTERSECT_FULL;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            const float x21 = p2[j].x - p1[i].x, y21 = p2[j].y - p1[i].y;
            float vx1 = v1[i].x, vy1 = v1[i].y, vx2 = v2[j].x, vy2 = v2[j].y;
            float det = vx2 * vy1 - vx1 * vy2;
            if (std::fabs(det) < 1e-12) continue;
            float t1 = (vx2 * y21 - vy2 * x21) / det;
            float t2 = (vx1 * y21 - vy1 * x21) / det;
            if (std::isinf(t1) || std::isinf(t2) || std::isnan(t1) || std::isnan(t2)) continue;
            if (t1 >= 0.0f && t1 <= 1.0f && t2 >= 0.0f && t2 <= 1.0f)
                out.push_back(P2f(p1[i].x + v1[i].x * t1, p1[i].y + v1[i].y * t1));
        }
    if (!out.empty()) ret = INTERSECT_PARTIAL;
    for (int pass = 0; pass < 2; ++pass) {
        const P2f* pa = pass == 0 ? p1 : p2;
        const P2f* pb = pass == 0 ? p2 : p1;
        const P2f* vb = pass == 0 ? v2 : v1;
        for (int i = 0; i < 4; ++i) {
            float x = pa[i].x, y = pa[i].y;
            int pos = 0, neg = 0;
            for (int j = 0; j < 4; ++j) {
                float A = -vb[j].y, B = vb[j].x;
                float C = -(A * pb[j].x + B * pb[j].y);
                float s = A * x + B * y + C;
                if (s >= 0) ++pos; else ++neg;
            }
            if (pos == 4 || neg == 4) out.push_back(pa[i]);
        }
    }
    int N = (int)out.size();
    if (N == 0) return INTERSECT_NONE;
    const int Ns = N;
    std::vector<float> dist((size_t)N * N, 0.f);
    std::vector<int> remap(N);
    for (int i = 0; i < N; ++i) {
        const P2f q0 = out[i];
        remap[i] = i;
        for (int j = i + 1; j < N;) {
            const P2f q1 = out[j];
            float dx = q1.x - q0.x, dy = q1.y - q0.y;
            float d2 = dx * dx + dy * dy;
            if (d2 <= eps) {
                if (j < N - 1) out[j] = out[N - 1];
                N--;
                continue;
            }
            dist[(size_t)i * Ns + j] = d2;
            ++j;
        }
    }
    while (N > 8) {
        int mi = 0, mj = 1;
        float md = dist[1];
        for (int i = 0; i < N - 1; ++i) {
            const float* pd = dist.data() + (size_t)Ns * remap[i];
            for (int j = i + 1; j < N; ++j) {
                float d = pd[remap[j]];
                if (d < md) { md = d; mi = i; mj = j; }
            }
        }
        (void)mi;
        if (mj < N - 1) { out[mj] = out[N - 1]; remap[mj] = remap[N - 1]; }
        N--;
    }
    out.resize(N);
    return ret;
}

// cv::contourArea(points, oriented=false)
static double contour_area(const std::vector<P2f>& p) {
    int n = (int)p.size();
    if (n == 0) return 0.;
    double a = 0;
    P2f prev = p[n - 1];
    for (int i = 0; i < n; ++i) {
        a += (double)prev.x * p[i].y - (double)prev.y * p[i].x;
        prev = p[i];
    }
    return std::fabs(a * 0.5);
}

// ---------------------------------------------------------------------------------------------------
// TemplateMatcher restatement
// ---------------------------------------------------------------------------------------------------

// s_TemplData (DataStructures.h:16-55)
struct TemplData {
    std::vector<Mat8> pyr;
    std::vector<double> mean, norm, inv_area;
    std::vector<bool> equal1;
    bool learned = false;
    int border = 0;
};

// s_MatchParameter (DataStructures.h:58-94); vecResult zero-initialised (reference: uninitialised)
struct MatchParam {
    P2d pt;
    double score = 0, angle = 0;
    RotRect rectR;
    bool del = false;
    double vecResult[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    bool on_border = false;
    int origin = -1;   // not in the reference: push index into vecMatchParameter, to export candidate records
    MatchParam() {}
    MatchParam(P2f p, double s, double a) : pt(p.x, p.y), score(s), angle(a) {}
};

static bool score_big2small(const MatchParam& l, const MatchParam& r) { return l.score > r.score; }

// s_BlockMax: Qt semantics (DataStructures.h:118-246) or, with mfc, the MFC tool's (MatchTool/MatchToolDlg.h:93-210)
struct BlockMax {
    struct Block { RectI r; double vmax; int mx, my; };
    std::vector<Block> blocks;
    MatF* m = nullptr;
    bool mfc = false;
    void add(RectI r) {
        Block b; b.r = r;
        int lx, ly;
        max_loc(*m, r.x, r.y, r.w, r.h, &b.vmax, &lx, &ly);
        b.mx = r.x + lx; b.my = r.y + ly;
        blocks.push_back(b);
    }
    BlockMax(MatF& mat, int tw, int th, bool mfc_ = false) : m(&mat), mfc(mfc_) {
        if (!mfc) {   // blocks of the template size: grid, right strip, bottom strip, corner (DataStructures.h:150-213)
            const int bw = tw, bh = th;
            int ncol = mat.w / bw, nrow = mat.h / bh;
            for (int y = 0; y < nrow; ++y)
                for (int x = 0; x < ncol; ++x) add(RectI(x * bw, y * bh, bw, bh));
            if (ncol * bw < mat.w) add(RectI(ncol * bw, 0, mat.w - ncol * bw, mat.h));
            if (nrow * bh < mat.h) add(RectI(0, nrow * bh, ncol * bw, mat.h - nrow * bh));
            if (ncol * bw < mat.w && nrow * bh < mat.h)
                add(RectI(ncol * bw, nrow * bh, mat.w - ncol * bw, mat.h - nrow * bh));
            return;
        }
        // MFC (MatchToolDlg.h:108-175): blocks of twice the template size, none at all when the map holds no whole
        // block; then right + bottom strips, the right strip alone, or else the full-width bottom strip (empty when
        // there is no residue at all)
        const int bw = tw * 2, bh = th * 2;
        const int ncol = mat.w / bw, nrow = mat.h / bh;
        const bool hres = mat.w % bw != 0, vres = mat.h % bh != 0;
        if (ncol == 0 || nrow == 0) return;
        for (int y = 0; y < nrow; ++y)
            for (int x = 0; x < ncol; ++x) add(RectI(x * bw, y * bh, bw, bh));
        if (hres && vres) {
            add(RectI(ncol * bw, 0, mat.w - ncol * bw, mat.h));
            add(RectI(0, nrow * bh, ncol * bw, mat.h - nrow * bh));
        } else if (hres) {
            add(RectI(ncol * bw, 0, mat.w - ncol * bw, mat.h));
        } else {
            add(RectI(0, nrow * bh, mat.w, mat.h - nrow * bh));
        }
    }
    void update(RectI ignore) {
        for (auto& b : blocks) {
            RectI in = rect_and(b.r, ignore);
            if (in.w * in.h > 0) {
                int lx, ly;
                max_loc(*m, b.r.x, b.r.y, b.r.w, b.r.h, &b.vmax, &lx, &ly);
                b.mx = b.r.x + lx; b.my = b.r.y + ly;
            }
        }
    }
    void get_max(double* v, int* x, int* y) const {
        if (mfc) {   // GetMaxValueLoc (MatchToolDlg.h:194-210): the whole map without blocks, else the LAST maximum
            if (blocks.empty()) { max_loc(*m, 0, 0, m->w, m->h, v, x, y); return; }
            size_t k = 0;
            for (size_t i = 1; i < blocks.size(); ++i)
                if (blocks[i].vmax >= blocks[k].vmax) k = i;
            *v = blocks[k].vmax; *x = blocks[k].mx; *y = blocks[k].my;
            return;
        }
        if (blocks.empty()) { *v = -1; *x = -1; *y = -1; return; }
        auto it = std::max_element(blocks.begin(), blocks.end(),
                                   [](const Block& a, const Block& b) { return a.vmax < b.vmax; });
        *v = it->vmax; *x = it->mx; *y = it->my;
    }
};

struct SearchStats {
    int top_angles = 0, top_candidates = 0;
    std::vector<int> live_per_layer;  // entering layer L-1 .. 0
    std::vector<MatchParam> top_list; // vecMatchParameter before the sort (reference push order)
    std::vector<fpm_candidate> cands; // per push-order candidate: top score, angle index, peak rank, refined pose
    // per-layer refinement decisions (only when Matcher::trace is set; a diagnostic, no reference counterpart):
    // rows of kTraceCols doubles = origin, layer, n3, imax, then (angle, score, mx, my, runner-up score of the
    // map) for j = 0..2
    std::vector<double> trace;
};
static const int kTraceCols = 19;

// ---------------------------------------------------------------------------------------------------
// cv::matchTemplate(TM_CCORR) as OpenCV's CPU crossCorr computes it: float32 DFTs (SENSITIVITY MODE).
//
// Every TM_CCORR call of the reference goes through OpenCV's crossCorr (imgproc/src/templmatch.cpp, 4.5.x,
// non-IPP): for 8-bit inputs the working depth is CV_32F, the correlation map is tiled into blocks of
// max(round(4.5 * templ), 256 - templ + 1) (clipped to the map), each block's image window and the template are
// zero-padded to getOptimalDFTSize(block + templ - 1), and the block is Re(IDFT(DFT(img) * conj(DFT(templ))))
// scaled by 1 / (W * H), all in float32.  Callers: the top layer always (TemplateMatcher.cpp:177 -> :514,
// MatchToolDlg.cpp:858 -> :1304) and every refinement layer when SIMD is off (:489 / MatchToolDlg.cpp:1277, whose
// "SIMD" checkbox is unchecked by default: MatchTool.rc:118 has no BS_CHECKED state and nothing sets it).
//
// OpenCV's own DFT kernels (CCS-packed real transforms, its radix order) are not reproduced: this is a plain
// mixed-radix (2/3/5) complex DIT FFT in float32 with double-computed twiddles rounded to float, i.e. arithmetic of
// the same precision and block structure whose rounding noise has the same magnitude, not the same bits.  It is a
// test-only mode (orc_set_ccorr_mode) used to measure how the reference-held screenshots respond to float TM_CCORR
// (tests/test_reference_pins.py); the parity mode (0) stays the exact integer sum rounded once (Appendix A.4).
// ---------------------------------------------------------------------------------------------------
static int optimal_dft_size(int n) {   // cv::getOptimalDFTSize: the smallest 2^a 3^b 5^c >= n
    if (n <= 1) return 1;
    for (int m = n;; ++m) {
        int r = m;
        for (int p : {2, 3, 5})
            while (r % p == 0) r /= p;
        if (r == 1) return m;
    }
}

struct Cf { float re, im; };

class Fft32 {
public:
    explicit Fft32(int n) : n_(n), tw_(n) {
        for (int k = 0; k < n; ++k) {
            double a = -2.0 * kPi * k / n;
            tw_[k].re = (float)std::cos(a);
            tw_[k].im = (float)std::sin(a);
        }
    }
    // in-place 1-D transform of n elements spaced by `stride` (forward e^{-2 pi i jk/n}; inverse unscaled)
    void run(Cf* x, int stride, bool inverse) {
        buf_.resize(n_);
        out_.resize(n_);
        for (int i = 0; i < n_; ++i) buf_[i] = x[(size_t)i * stride];
        rec(buf_.data(), 1, out_.data(), n_, 1, inverse);
        for (int i = 0; i < n_; ++i) x[(size_t)i * stride] = out_[i];
    }

private:
    int n_;
    std::vector<Cf> tw_, buf_, out_;
    Cf w(int k, bool inverse) const {
        Cf t = tw_[k % n_];
        if (inverse) t.im = -t.im;
        return t;
    }
    void rec(const Cf* in, int stride, Cf* out, int n, int tstep, bool inverse) {
        if (n == 1) { out[0] = in[0]; return; }
        int p = n % 2 == 0 ? 2 : n % 3 == 0 ? 3 : 5;
        int m = n / p;
        for (int r = 0; r < p; ++r) rec(in + (size_t)r * stride, stride * p, out + (size_t)r * m, m, tstep * p, inverse);
        Cf xr[5], y[5];
        for (int k = 0; k < m; ++k) {
            for (int r = 0; r < p; ++r) {
                Cf a = out[r * m + k], t = w(r * k * tstep, inverse);
                xr[r].re = a.re * t.re - a.im * t.im;
                xr[r].im = a.re * t.im + a.im * t.re;
            }
            for (int q = 0; q < p; ++q) {
                Cf s = xr[0];
                for (int r = 1; r < p; ++r) {
                    Cf t = w(((r * q) % p) * (n_ / p), inverse);
                    s.re += xr[r].re * t.re - xr[r].im * t.im;
                    s.im += xr[r].re * t.im + xr[r].im * t.re;
                }
                y[q] = s;
            }
            for (int q = 0; q < p; ++q) out[k + q * m] = y[q];
        }
    }
};

// 2-D transform of a dh x dw complex array (rows, then columns)
static void fft2_f32(std::vector<Cf>& a, int dw, int dh, bool inverse) {
    Fft32 fr(dw), fc(dh);
    for (int y = 0; y < dh; ++y) fr.run(a.data() + (size_t)y * dw, 1, inverse);
    for (int x = 0; x < dw; ++x) fc.run(a.data() + x, dw, inverse);
}

// OpenCV crossCorr (templmatch.cpp, 4.5.x) for one 8-bit image and template, anchor (0, 0), delta 0
static void cross_corr_f32(const Mat8& img, const Mat8& t, MatF& corr) {
    corr = MatF(img.w - t.w + 1, img.h - t.h + 1, 0.f);
    const double blockScale = 4.5;
    const int minBlockSize = 256;
    int bw = (int)std::lrint(t.w * blockScale), bh = (int)std::lrint(t.h * blockScale);
    bw = std::min(std::max(bw, minBlockSize - t.w + 1), corr.w);
    bh = std::min(std::max(bh, minBlockSize - t.h + 1), corr.h);
    const int dw = std::max(optimal_dft_size(bw + t.w - 1), 2), dh = optimal_dft_size(bh + t.h - 1);
    bw = std::min(dw - t.w + 1, corr.w);
    bh = std::min(dh - t.h + 1, corr.h);
    std::vector<Cf> ft((size_t)dw * dh, Cf{0.f, 0.f}), fi((size_t)dw * dh);
    for (int y = 0; y < t.h; ++y)
        for (int x = 0; x < t.w; ++x) ft[(size_t)y * dw + x].re = (float)t.row(y)[x];
    fft2_f32(ft, dw, dh, false);
    const float scale = (float)(1.0 / ((double)dw * dh));
    for (int y0 = 0; y0 < corr.h; y0 += bh)
        for (int x0 = 0; x0 < corr.w; x0 += bw) {
            int bsw = std::min(bw, corr.w - x0), bsh = std::min(bh, corr.h - y0);
            int sw = bsw + t.w - 1, sh = bsh + t.h - 1;
            std::fill(fi.begin(), fi.end(), Cf{0.f, 0.f});
            for (int y = 0; y < sh; ++y)
                for (int x = 0; x < sw; ++x) fi[(size_t)y * dw + x].re = (float)img.row(y0 + y)[x0 + x];
            fft2_f32(fi, dw, dh, false);
            for (size_t i = 0; i < fi.size(); ++i) {   // mulSpectrums(img, templ, conjB = true)
                Cf a = fi[i], b = ft[i];
                fi[i].re = a.re * b.re + a.im * b.im;
                fi[i].im = a.im * b.re - a.re * b.im;
            }
            fft2_f32(fi, dw, dh, true);
            for (int y = 0; y < bsh; ++y)
                for (int x = 0; x < bsw; ++x) corr.at(y0 + y, x0 + x) = fi[(size_t)y * dw + x].re * scale;
        }
}

class Matcher {
public:
    fpm_params prm;
    TemplData T;
    double last_seconds = 0.0;
    SearchStats stats;
    bool trace = false;
    int ccorr_mode = 0;   // TM_CCORR arithmetic: 0 = exact integer sum rounded once (parity), 1 = f32 DFT (above)

    Matcher() { fpm_params_default(&prm); }

    // TemplateMatcher::getTopLayer (TemplateMatcher.cpp:445-455)
    static int top_layer(int w, int h, int min_len) {
        int L = 0, mra = min_len * min_len, area = w * h;
        while (area > mra) { area /= 4; ++L; }
        return L;
    }

    // TemplateMatcher::learnPattern (TemplateMatcher.cpp:45-95)
    bool learn(const Mat8& tmpl) {
        if (tmpl.empty()) return false;
        T = TemplData();
        int L = top_layer(tmpl.w, tmpl.h, (int)std::sqrt((double)prm.min_reduce_area));
        T.pyr = build_pyramid(tmpl, L);
        double m0, s0;
        mean_stddev(tmpl, &m0, &s0);   // cv::mean == meanStdDev's mean
        T.border = m0 < 128 ? 255 : 0;
        int n = (int)T.pyr.size();
        T.mean.assign(n, 0); T.norm.assign(n, 0); T.inv_area.assign(n, 1); T.equal1.assign(n, false);
        for (int i = 0; i < n; ++i) {
            double inv_area = 1.0 / ((double)T.pyr[i].h * T.pyr[i].w);
            double mean, sdv;
            mean_stddev(T.pyr[i], &mean, &sdv);
            double norm = sdv * sdv + 0.0 * 0.0 + 0.0 * 0.0 + 0.0 * 0.0;
            if (norm < DBL_EPSILON) T.equal1[i] = true;
            norm = std::sqrt(norm);
            norm /= std::sqrt(inv_area);
            T.inv_area[i] = inv_area; T.mean[i] = mean; T.norm[i] = norm;
        }
        T.learned = true;
        return true;
    }

    // IM_Conv_SIMD (TemplateMatcher.cpp:461-483): exact int32 dot product of one template row.
    static inline int row_dot(const uint8_t* k, const uint8_t* c, int n) {
        __m128i acc = _mm_setzero_si128();
        const __m128i z = _mm_setzero_si128();
        int i = 0;
        for (; i + 16 <= n; i += 16) {
            __m128i a = _mm_loadu_si128((const __m128i*)(k + i));
            __m128i b = _mm_loadu_si128((const __m128i*)(c + i));
            acc = _mm_add_epi32(acc, _mm_madd_epi16(_mm_unpacklo_epi8(a, z), _mm_unpacklo_epi8(b, z)));
            acc = _mm_add_epi32(acc, _mm_madd_epi16(_mm_unpackhi_epi8(a, z), _mm_unpackhi_epi8(b, z)));
        }
        int lanes[4];
        _mm_storeu_si128((__m128i*)lanes, acc);
        int s = lanes[0] + lanes[1] + lanes[2] + lanes[3];
        for (; i < n; ++i) s += k[i] * c[i];
        return s;
    }

    // TemplateMatcher::MatchTemplate (TemplateMatcher.cpp:485-525)
    void match_template(const Mat8& src, int layer, bool use_simd, MatF& res) const {
        const Mat8& t = T.pyr[layer];
        res = MatF(src.w - t.w + 1, src.h - t.h + 1, 0.f);
        if (prm.use_simd && use_simd) {
            for (int r = 0; r < res.h; ++r)
                for (int c = 0; c < res.w; ++c) {
                    float acc = 0.f;
                    for (int tr = 0; tr < t.h; ++tr)
                        acc = acc + (float)row_dot(t.row(tr), src.row(r + tr) + c, t.w);
                    res.at(r, c) = acc;
                }
        } else if (ccorr_mode == 1) {
            cross_corr_f32(src, t, res);   // test-only sensitivity mode (see cross_corr_f32)
        } else {
            // cv::matchTemplate(TM_CCORR): exact integer sum rounded once to f32 (Appendix A.4)
            for (int r = 0; r < res.h; ++r)
                for (int c = 0; c < res.w; ++c) {
                    int64_t s = 0;
                    for (int tr = 0; tr < t.h; ++tr) s += row_dot(t.row(tr), src.row(r + tr) + c, t.w);
                    res.at(r, c) = (float)s;
                }
        }
        ccoeff_denominator(src, layer, res);
    }

    // TemplateMatcher::CCOEFF_Denominator (TemplateMatcher.cpp:527-598)
    void ccoeff_denominator(const Mat8& src, int layer, MatF& res) const {
        if (T.equal1[layer]) {
            std::fill(res.px.begin(), res.px.end(), 1.f);
            return;
        }
        // cv::integral(src, sum, sqsum, CV_64F): (H+1)x(W+1), exact
        const int iw = src.w + 1;
        std::vector<double> sum((size_t)(src.h + 1) * iw, 0.0), sq((size_t)(src.h + 1) * iw, 0.0);
        for (int y = 0; y < src.h; ++y) {
            double rs = 0, rq = 0;
            for (int x = 0; x < src.w; ++x) {
                double v = src.row(y)[x];
                rs += v; rq += v * v;
                sum[(size_t)(y + 1) * iw + x + 1] = sum[(size_t)y * iw + x + 1] + rs;
                sq[(size_t)(y + 1) * iw + x + 1] = sq[(size_t)y * iw + x + 1] + rq;
            }
        }
        const int tw = T.pyr[layer].w, th = T.pyr[layer].h;
        const double mean0 = T.mean[layer], tnorm = T.norm[layer], inv_area = T.inv_area[layer];
        for (int i = 0; i < res.h; ++i)
            for (int j = 0; j < res.w; ++j) {
                size_t i0 = (size_t)i * iw + j, i2 = (size_t)(i + th) * iw + j;
                double num = res.at(i, j), t;
                double wndMean2 = 0, wndSum2 = 0;
                t = sum[i0] - sum[i0 + tw] - sum[i2] + sum[i2 + tw];
                wndMean2 += t * t;
                num -= t * mean0;
                wndMean2 *= inv_area;
                t = sq[i0] - sq[i0 + tw] - sq[i2] + sq[i2 + tw];
                wndSum2 += t;
                double diff2 = std::max(wndSum2 - wndMean2, 0.0);
                if (diff2 <= std::min(0.5, 10 * FLT_EPSILON * wndSum2))
                    t = 0;
                else
                    t = std::sqrt(diff2) * tnorm;
                if (std::fabs(num) < t)
                    num /= t;
                else if (std::fabs(num) < t * 1.125)
                    num = num > 0 ? 1 : -1;
                else
                    num = 0;
                res.at(i, j) = (float)num;
            }
    }

    // TemplateMatcher::ptRotatePt2f (TemplateMatcher.cpp:971-982)
    static P2f rotate_pt(P2f in, P2f org, double a) {
        double w = org.x * 2;
        double h = org.y * 2;
        double y1 = h - in.y, y2 = h - org.y;
        double x = (in.x - org.x) * std::cos(a) - (y1 - org.y) * std::sin(a) + org.x;
        double y = (in.x - org.x) * std::sin(a) + (y1 - org.y) * std::cos(a) + y2;
        (void)w;
        y = -y + h;
        return P2f((float)x, (float)y);
    }

    // TemplateMatcher::getBestRotationSize (TemplateMatcher.cpp:901-969)
    static void best_rotation_size(int sw, int sh, int dw_, int dh_, double ang, int* ow, int* oh) {
        double rad = ang * D2R;
        P2f c((sw - 1) / 2.0f, (sh - 1) / 2.0f);
        P2f lt = rotate_pt(P2f(0.f, 0.f), c, rad);
        P2f lb = rotate_pt(P2f(0.f, (float)(sh - 1)), c, rad);
        P2f rb = rotate_pt(P2f((float)(sw - 1), (float)(sh - 1)), c, rad);
        P2f rt = rotate_pt(P2f((float)(sw - 1), 0.f), c, rad);
        float top = std::max(std::max(lt.y, lb.y), std::max(rb.y, rt.y));
        float bottom = std::min(std::min(lt.y, lb.y), std::min(rb.y, rt.y));
        float right = std::max(std::max(lt.x, lb.x), std::max(rb.x, rt.x));
        float left = std::min(std::min(lt.x, lb.x), std::min(rb.x, rt.x));
        if (ang > 360) ang -= 360;
        else if (ang < 0) ang += 360;
        if (std::fabs(std::fabs(ang) - 90) < VISION_TOLERANCE || std::fabs(std::fabs(ang) - 270) < VISION_TOLERANCE) {
            *ow = sh; *oh = sw; return;
        } else if (std::fabs(ang) < VISION_TOLERANCE || std::fabs(std::fabs(ang) - 180) < VISION_TOLERANCE) {
            *ow = sw; *oh = sh; return;
        }
        double a = ang;
        if (a > 0 && a < 90) {
        } else if (a > 90 && a < 180) a -= 90;
        else if (a > 180 && a < 270) a -= 180;
        else if (a > 270 && a < 360) a -= 270;
        float h1 = dw_ * std::sin(a * D2R) * std::cos(a * D2R);
        float h2 = dh_ * std::sin(a * D2R) * std::cos(a * D2R);
        int half_h = (int)std::ceil(top - c.y - h1);
        int half_w = (int)std::ceil(right - c.x - h2);
        int rw = half_w * 2, rh = half_h * 2;
        bool wrong = (dw_ < rw && dh_ > rh) || (dw_ > rw && dh_ < rh || (int64_t)dw_ * dh_ > (int64_t)rw * rh);
        if (wrong) { rw = int(right - left + 0.5); rh = int(top - bottom + 0.5); }
        *ow = rw; *oh = rh;
    }

    // TemplateMatcher::getRotatedROI (TemplateMatcher.cpp:1074-1090)
    static Mat8 rotated_roi(const Mat8& src, int tw, int th, P2f lt, double ang) {
        double rad = ang * D2R;
        P2f c((src.w - 1) / 2.0f, (src.h - 1) / 2.0f);
        P2f ltr = rotate_pt(lt, c, rad);
        double m[6];
        rotation_matrix(c, ang, m);
        m[2] -= ltr.x - 3;
        m[5] -= ltr.y - 3;
        return warp_affine(src, m, tw + 6, th + 6, 0);
    }

    // TemplateMatcher::getNextMaxLoc, plain (TemplateMatcher.cpp:1196-1206)
    static void next_max_loc(MatF& r, int& px, int& py, int tw, int th, double& v, double ov) {
        int sx = px - tw * (1 - ov);
        int sy = py - th * (1 - ov);
        fill_rect(r, RectI(sx, sy, 2 * tw * (1 - ov), 2 * th * (1 - ov)), -1.f);
        max_loc(r, 0, 0, r.w, r.h, &v, &px, &py);
    }

    // TemplateMatcher::getNextMaxLoc, s_BlockMax (TemplateMatcher.cpp:1208-1221)
    static void next_max_loc_block(MatF& r, int& px, int& py, int tw, int th, double& v, double ov, BlockMax& bm) {
        int sx = int(px - tw * (1 - ov));
        int sy = int(py - th * (1 - ov));
        RectI ig(sx, sy, int(2 * tw * (1 - ov)), int(2 * th * (1 - ov)));
        fill_rect(r, ig, -1.f);
        bm.update(ig);
        bm.get_max(&v, &px, &py);
    }

    // TemplateMatcher::sortPtWithCenter (TemplateMatcher.cpp:1093-1131)
    static void sort_pt_with_center(std::vector<P2f>& v) {
        int n = (int)v.size();
        P2f c;
        for (int i = 0; i < n; ++i) { c.x += v[i].x; c.y += v[i].y; }
        c.x = c.x / n; c.y = c.y / n;
        std::vector<std::pair<P2f, double>> pa(n);
        for (int i = 0; i < n; ++i) {
            pa[i].first = v[i];
            P2f d(v[i].x - c.x, v[i].y - c.y);
            float nrm = d.x * d.x + d.y * d.y;
            float dot = d.x;
            if (d.y < 0) pa[i].second = std::acos(dot / nrm) * R2D;
            else if (d.y > 0) pa[i].second = 360 - std::acos(dot / nrm) * R2D;
            else pa[i].second = (d.x - c.x > 0) ? 0 : 180;
        }
        std::sort(pa.begin(), pa.end(),
                  [](const std::pair<P2f, double> l, const std::pair<P2f, double> r) { return l.second < r.second; });
        for (int i = 0; i < n; ++i) v[i] = pa[i].first;
    }

    // TemplateMatcher::filterWithScore (TemplateMatcher.cpp:984-1000)
    static void filter_with_score(std::vector<MatchParam>& v, double s) {
        std::sort(v.begin(), v.end(), score_big2small);
        int n = (int)v.size(), del = n + 1;
        for (int i = 0; i < n; ++i)
            if (v[i].score < s) { del = i; break; }
        if (del == n + 1) return;
        v.erase(v.begin() + del, v.end());
    }

    // TemplateMatcher::filterWithRotatedRect (TemplateMatcher.cpp:1133-1194), iMethod = TM_CCOEFF_NORMED
    static void filter_with_rotated_rect(std::vector<MatchParam>& v, double max_ov) {
        if (v.empty()) return;
        int n = (int)v.size();
        std::vector<P2f> inter;
        for (int i = 0; i < n - 1; ++i) {
            if (v[i].del) continue;
            for (int j = i + 1; j < n; ++j) {
                if (v[j].del) continue;
                const RotRect& r1 = v[i].rectR;
                const RotRect& r2 = v[j].rectR;
                int type = rotrect_intersection(r1, r2, inter);
                if (type == INTERSECT_NONE) continue;
                if (type == INTERSECT_FULL) {
                    int d = (v[i].score >= v[j].score) ? j : i;
                    v[d].del = true;
                } else {
                    if (inter.size() < 3) continue;
                    sort_pt_with_center(inter);
                    double area = contour_area(inter);
                    double ratio = area / (r1.w * r1.h);
                    if (ratio > max_ov) {
                        int d = (v[i].score >= v[j].score) ? j : i;
                        v[d].del = true;
                    }
                }
            }
        }
        v.erase(std::remove_if(v.begin(), v.end(), [](const MatchParam& p) { return p.del; }), v.end());
    }

    // 10x10 LU inverse with partial pivoting (cv::invert DECOMP_LU -> hal::LU64f)
    static bool lu_inverse(double* A, int n, double* B) {
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) B[i * n + j] = i == j ? 1.0 : 0.0;
        const double eps = DBL_EPSILON * 100;
        for (int i = 0; i < n; ++i) {
            int k = i;
            for (int j = i + 1; j < n; ++j)
                if (std::fabs(A[j * n + i]) > std::fabs(A[k * n + i])) k = j;
            if (std::fabs(A[k * n + i]) < eps) return false;
            if (k != i) {
                for (int j = i; j < n; ++j) std::swap(A[i * n + j], A[k * n + j]);
                for (int j = 0; j < n; ++j) std::swap(B[i * n + j], B[k * n + j]);
            }
            double d = -1 / A[i * n + i];
            for (int j = i + 1; j < n; ++j) {
                double alpha = A[j * n + i] * d;
                for (int c = i + 1; c < n; ++c) A[j * n + c] += alpha * A[i * n + c];
                for (int c = 0; c < n; ++c) B[j * n + c] += alpha * B[i * n + c];
            }
        }
        for (int i = n - 1; i >= 0; --i)
            for (int j = 0; j < n; ++j) {
                double s = B[i * n + j];
                for (int c = i + 1; c < n; ++c) s -= A[i * n + c] * B[c * n + j];
                B[i * n + j] = s / A[i * n + i];
            }
        return true;
    }

    // TemplateMatcher::subPixEstimation (TemplateMatcher.cpp:1002-1072)
    static void subpix(const std::vector<MatchParam>& v, double* dx, double* dy, double* dang, double step, int im) {
        double A[27][10], S[27];
        double x0 = v[im].pt.x, y0 = v[im].pt.y, t0 = v[im].angle;
        int row = 0;
        for (int th = 0; th <= 2; ++th)
            for (int y = -1; y <= 1; ++y)
                for (int x = -1; x <= 1; ++x) {
                    double X = x0 + x, Y = y0 + y, Tt = (t0 + (th - 1) * step) * D2R;
                    double* a = A[row];
                    a[0] = X * X; a[1] = Y * Y; a[2] = Tt * Tt; a[3] = X * Y; a[4] = X * Tt; a[5] = Y * Tt;
                    a[6] = X; a[7] = Y; a[8] = Tt; a[9] = 1.0;
                    S[row] = v[im + (th - 1)].vecResult[x + 1][y + 1];
                    ++row;
                }
        double AtA[100], inv[100], AtS[10], Z[10];
        for (int i = 0; i < 10; ++i) {
            for (int j = 0; j < 10; ++j) {
                double s = 0;
                for (int r = 0; r < 27; ++r) s += A[r][i] * A[r][j];
                AtA[i * 10 + j] = s;
            }
        }
        if (!lu_inverse(AtA, 10, inv)) std::fill(inv, inv + 100, 0.0);
        // Z = (inv * A^T) * S, evaluated left to right as in the reference expression
        std::vector<double> invAt(10 * 27);
        for (int i = 0; i < 10; ++i)
            for (int r = 0; r < 27; ++r) {
                double s = 0;
                for (int k = 0; k < 10; ++k) s += inv[i * 10 + k] * A[r][k];
                invAt[i * 27 + r] = s;
            }
        for (int i = 0; i < 10; ++i) {
            double s = 0;
            for (int r = 0; r < 27; ++r) s += invAt[i * 27 + r] * S[r];
            Z[i] = s;
        }
        (void)AtS;
        double K1[9] = {2 * Z[0], Z[3], Z[4], Z[3], 2 * Z[1], Z[5], Z[4], Z[5], 2 * Z[2]};
        double K2[3] = {-Z[6], -Z[7], -Z[8]};
        // 3x3 inverse, closed form (cv::invert DECOMP_LU, n == 3)
        auto M = [&](int r, int c) { return K1[r * 3 + c]; };
        double d = M(0, 0) * (M(1, 1) * M(2, 2) - M(1, 2) * M(2, 1)) - M(0, 1) * (M(1, 0) * M(2, 2) - M(1, 2) * M(2, 0)) +
                   M(0, 2) * (M(1, 0) * M(2, 1) - M(1, 1) * M(2, 0));
        double t[9] = {0};
        if (d != 0.) {
            d = 1. / d;
            t[0] = (M(1, 1) * M(2, 2) - M(1, 2) * M(2, 1)) * d;
            t[1] = (M(0, 2) * M(2, 1) - M(0, 1) * M(2, 2)) * d;
            t[2] = (M(0, 1) * M(1, 2) - M(0, 2) * M(1, 1)) * d;
            t[3] = (M(1, 2) * M(2, 0) - M(1, 0) * M(2, 2)) * d;
            t[4] = (M(0, 0) * M(2, 2) - M(0, 2) * M(2, 0)) * d;
            t[5] = (M(0, 2) * M(1, 0) - M(0, 0) * M(1, 2)) * d;
            t[6] = (M(1, 0) * M(2, 1) - M(1, 1) * M(2, 0)) * d;
            t[7] = (M(0, 1) * M(2, 0) - M(0, 0) * M(2, 1)) * d;
            t[8] = (M(0, 0) * M(1, 1) - M(0, 1) * M(1, 0)) * d;
        }
        *dx = t[0] * K2[0] + t[1] * K2[1] + t[2] * K2[2];
        *dy = t[3] * K2[0] + t[4] * K2[1] + t[5] * K2[2];
        *dang = (t[6] * K2[0] + t[7] * K2[1] + t[8] * K2[2]) * R2D;
    }

    // TemplateMatcher::match (TemplateMatcher.cpp:97-437)
    // candidate-record export (test infrastructure for the angle-sharded merge; no reference counterpart)
    void note_candidate(MatchParam& m, int angle_index, int peak_rank) {
        m.origin = (int)stats.cands.size();
        fpm_candidate c;
        std::memset(&c, 0, sizeof(c));
        c.top_score = m.score;
        c.angle_index = angle_index;
        c.peak_rank = peak_rank;
        stats.cands.push_back(c);
    }
    void note_kept(int origin, const MatchParam& m) {
        fpm_candidate& c = stats.cands[origin];
        c.x = m.pt.x; c.y = m.pt.y; c.score = m.score; c.angle = m.angle; c.kept = 1;
    }

    int match(const Mat8& src, std::vector<fpm_result>& out) {
        out.clear();
        stats = SearchStats();
        if (src.empty() || !T.learned) return src.empty() ? FPM_E_INVALID_ARG : FPM_E_NOT_LEARNED;
        const Mat8& t0 = T.pyr[0];
        if ((t0.w < src.w && t0.h > src.h) || (t0.w > src.w && t0.h < src.h)) return FPM_E_SIZE;
        if ((int64_t)t0.w * t0.h > (int64_t)src.w * src.h) return FPM_E_SIZE;
        auto t_start = std::chrono::high_resolution_clock::now();

        int L = top_layer(t0.w, t0.h, (int)std::sqrt((double)prm.min_reduce_area));
        if (L >= (int)T.pyr.size()) return FPM_E_INVALID_ARG;  // MinReduceArea changed after learn (UB in the reference)
        std::vector<Mat8> spyr = build_pyramid(src, L);

        double step = std::atan(2.0 / std::max(T.pyr[L].w, T.pyr[L].h)) * R2D;
        if (prm.top_angle_step > 0) step = prm.top_angle_step;   // extension (fpm.h): the top-layer step override
        const bool mfc = prm.semantics == FPM_SEMANTICS_MFC;
        {   // input guard (no reference counterpart: it would loop without end or exhaust memory), as the engine's
            auto span = [&](double lo, double hi) { return (hi - lo) / step + 2; };
            bool ok = std::isfinite(step) && step > 0;
            double n = 0;
            if (ok && mfc && prm.tolerance_range) {
                for (double t : prm.tolerance) ok = ok && std::isfinite(t);
                n = span(prm.tolerance[0], prm.tolerance[1]) + span(prm.tolerance[2], prm.tolerance[3]);
            } else if (ok) {
                ok = std::isfinite(prm.tolerance_angle);
                n = prm.tolerance_angle < VISION_TOLERANCE ? 1 : 2 * span(0, prm.tolerance_angle);
            }
            if (!ok || !(n <= 100000)) return FPM_E_INVALID_ARG;
        }
        std::vector<double> angles;
        if (mfc && prm.tolerance_range) {   // MatchToolDlg.cpp:805-815
            const double* t = prm.tolerance;
            if (t[0] >= t[1] || t[2] >= t[3]) return FPM_E_INVALID_ARG;   // the tool refuses the ranges (:807-811)
            for (double a = t[0]; a < t[1] + step; a += step) angles.push_back(a);
            for (double a = t[2]; a < t[3] + step; a += step) angles.push_back(a);
        } else if (prm.tolerance_angle < VISION_TOLERANCE) {
            angles.push_back(0.0);
        } else {
            for (double a = 0; a < prm.tolerance_angle + step; a += step) angles.push_back(a);
            for (double a = -step; a > -prm.tolerance_angle - step; a -= step) angles.push_back(a);
        }
        int topW = spyr[L].w, topH = spyr[L].h;
        P2f center((topW - 1) / 2.0f, (topH - 1) / 2.0f);
        int nang = (int)angles.size();
        std::vector<MatchParam> cand;
        std::vector<double> layer_score(L + 1, prm.score);
        for (int l = 1; l <= L; ++l) layer_score[l] = layer_score[l - 1] * 0.9;
        const int tw = T.pyr[L].w, th = T.pyr[L].h;
        bool by_block = ((topW * topH) / (tw * th) > 500) && prm.max_pos > 10;

        for (int i = 0; i < nang; ++i) {
            double m[6];
            rotation_matrix(center, angles[i], m);
            int bw, bh;
            best_rotation_size(topW, topH, tw, th, angles[i], &bw, &bh);
            float tx = (bw - 1) / 2.0f - center.x;
            float ty = (bh - 1) / 2.0f - center.y;
            m[2] += tx;
            m[5] += ty;
            if (bw < tw || bh < th) continue;  // cv::matchTemplate would throw (reference: uncaught)
            Mat8 rot = warp_affine(spyr[L], m, bw, bh, T.border);
            MatF res;
            match_template(rot, L, false, res);
            int px, py;
            double v, vmax;
            if (by_block) {
                BlockMax bm(res, tw, th, mfc);
                bm.get_max(&vmax, &px, &py);
                if (vmax < layer_score[L]) continue;
                cand.push_back(MatchParam(P2f(px - tx, py - ty), vmax, angles[i]));
                note_candidate(cand.back(), i, 0);
                for (int j = 0; j < prm.max_pos + MATCH_CANDIDATE_NUM - 1; ++j) {
                    next_max_loc_block(res, px, py, tw, th, v, prm.max_overlap, bm);
                    if (v < layer_score[L]) break;
                    cand.push_back(MatchParam(P2f(px - tx, py - ty), v, angles[i]));
                    note_candidate(cand.back(), i, j + 1);
                }
            } else {
                max_loc(res, 0, 0, res.w, res.h, &vmax, &px, &py);
                if (vmax < layer_score[L]) continue;
                cand.push_back(MatchParam(P2f(px - tx, py - ty), vmax, angles[i]));
                note_candidate(cand.back(), i, 0);
                for (int j = 0; j < prm.max_pos + MATCH_CANDIDATE_NUM - 1; ++j) {
                    next_max_loc(res, px, py, tw, th, v, prm.max_overlap);
                    if (v < layer_score[L]) break;
                    cand.push_back(MatchParam(P2f(px - tx, py - ty), v, angles[i]));
                    note_candidate(cand.back(), i, j + 1);
                }
            }
        }
        stats.top_angles = nang;
        stats.top_candidates = (int)cand.size();
        stats.top_list = cand;
        stats.live_per_layer.assign(L, 0);

        std::sort(cand.begin(), cand.end(), score_big2small);
        int dstW = T.pyr[L].w, dstH = T.pyr[L].h;
        const bool subpixel = prm.subpixel != 0;
        const int stop = 0;
        std::vector<MatchParam> all;
        for (int i = 0; i < (int)cand.size(); ++i) {
            double rad = -cand[i].angle * D2R;
            P2f lt = rotate_pt(P2f((float)cand[i].pt.x, (float)cand[i].pt.y), center, rad);
            double astep = std::atan(2.0 / std::max(dstW, dstH)) * R2D;
            if (L <= stop) {
                P2f p(lt.x * ((L == 0) ? 1 : 2), lt.y * ((L == 0) ? 1 : 2));
                cand[i].pt = P2d(p.x, p.y);
                all.push_back(cand[i]);
                note_kept(cand[i].origin, all.back());
                continue;
            }
            for (int l = L - 1; l >= stop; --l) {
                stats.live_per_layer[L - 1 - l]++;
                astep = std::atan(2.0 / std::max(T.pyr[l].w, T.pyr[l].h)) * R2D;
                std::vector<double> a3;
                double matched = cand[i].angle;
                if (prm.tolerance_range) {
                    for (int k = -1; k <= 1; ++k) a3.push_back(matched + astep * k);
                } else {
                    if (prm.tolerance_angle < VISION_TOLERANCE)
                        a3.push_back(0.0);
                    else
                        for (int k = -1; k <= 1; ++k) a3.push_back(matched + astep * k);
                }
                P2f sc((spyr[l].w - 1) / 2.0f, (spyr[l].h - 1) / 2.0f);
                int n3 = (int)a3.size();
                std::vector<MatchParam> nm(n3);
                double second[3] = {0, 0, 0};
                int imax = 0;
                double big = -1;
                for (int j = 0; j < n3; ++j) {
                    P2f lt2(lt.x * 2, lt.y * 2);
                    Mat8 roi = rotated_roi(spyr[l], T.pyr[l].w, T.pyr[l].h, lt2, a3[j]);
                    MatF res;
                    match_template(roi, l, true, res);
                    double vmax;
                    int mx, my;
                    max_loc(res, 0, 0, res.w, res.h, &vmax, &mx, &my);
                    if (trace) {
                        second[j] = -2;
                        for (int k = 0; k < (int)res.px.size(); ++k)
                            if (k != my * res.w + mx) second[j] = std::max(second[j], (double)res.px[k]);
                    }
                    nm[j] = MatchParam(P2f((float)mx, (float)my), vmax, a3[j]);
                    if (nm[j].score > big) { imax = j; big = nm[j].score; }
                    if (mx == 0 || my == 0 || mx == res.w - 1 || my == res.h - 1) nm[j].on_border = true;
                    if (!nm[j].on_border)
                        for (int y = -1; y <= 1; ++y)
                            for (int x = -1; x <= 1; ++x) nm[j].vecResult[x + 1][y + 1] = res.at(my + y, mx + x);
                }
                if (trace) {
                    double row[kTraceCols] = {(double)cand[i].origin, (double)l, (double)n3, (double)imax};
                    for (int j = 0; j < n3; ++j) {
                        row[4 + 5 * j] = nm[j].angle; row[5 + 5 * j] = nm[j].score;
                        row[6 + 5 * j] = nm[j].pt.x; row[7 + 5 * j] = nm[j].pt.y; row[8 + 5 * j] = second[j];
                    }
                    stats.trace.insert(stats.trace.end(), row, row + kTraceCols);
                }
                if (nm[imax].score < layer_score[l]) break;
                if (subpixel && l == 0 && !nm[imax].on_border && imax != 0 && imax != 2) {
                    double nx = 0, ny = 0, na = 0;
                    subpix(nm, &nx, &ny, &na, astep, imax);
                    nm[imax].pt = P2d(nx, ny);
                    nm[imax].angle = na;
                }
                double nang2 = nm[imax].angle;
                P2f r0 = rotate_pt(P2f(lt.x * 2, lt.y * 2), sc, nang2 * D2R);
                P2f pad(r0.x - 3, r0.y - 3);
                P2f p((float)(nm[imax].pt.x + pad.x), (float)(nm[imax].pt.y + pad.y));
                p = rotate_pt(p, sc, -nang2 * D2R);
                if (l == stop) {
                    int f = stop == 0 ? 1 : 2;
                    P2f pf(p.x * f, p.y * f);
                    nm[imax].pt = P2d(pf.x, pf.y);
                    all.push_back(nm[imax]);
                    note_kept(cand[i].origin, all.back());
                } else {
                    cand[i].angle = nang2;
                    lt = p;
                }
            }
        }
        filter_with_score(all, prm.score);
        dstW = T.pyr[stop].w * (stop == 0 ? 1 : 2);
        dstH = T.pyr[stop].h * (stop == 0 ? 1 : 2);
        for (auto& r : all) {
            double rad = -r.angle * D2R;
            P2f lt((float)r.pt.x, (float)r.pt.y);
            P2f rt(lt.x + dstW * (float)std::cos(rad), lt.y - dstW * (float)std::sin(rad));
            P2f lb(lt.x + dstH * (float)std::sin(rad), lt.y + dstH * (float)std::cos(rad));
            P2f rb(rt.x + dstH * (float)std::sin(rad), rt.y + dstH * (float)std::cos(rad));
            (void)lb;
            r.rectR = rotrect_from3(lt, rt, rb);
        }
        filter_with_rotated_rect(all, prm.max_overlap);
        std::sort(all.begin(), all.end(), score_big2small);
        if (all.empty()) return FPM_OK;
        const int iW = T.pyr[0].w, iH = T.pyr[0].h;
        auto t_end = std::chrono::high_resolution_clock::now();
        last_seconds = std::chrono::duration<double>(t_end - t_start).count();
        for (const auto& r : all) {
            double rad = -r.angle * D2R;
            if (mfc) {   // MatchToolDlg.cpp:1080-1116: f64 corners, negated + wrapped angle, at most MaxPos results
                fpm_result o;
                o.lt_x = r.pt.x; o.lt_y = r.pt.y;
                o.rt_x = o.lt_x + iW * std::cos(rad); o.rt_y = o.lt_y - iW * std::sin(rad);
                o.lb_x = o.lt_x + iH * std::sin(rad); o.lb_y = o.lt_y + iH * std::cos(rad);
                o.rb_x = o.rt_x + iH * std::sin(rad); o.rb_y = o.rt_y + iH * std::cos(rad);
                o.cx = (o.lt_x + o.rt_x + o.rb_x + o.lb_x) / 4; o.cy = (o.lt_y + o.rt_y + o.rb_y + o.lb_y) / 4;
                o.angle = -r.angle;
                o.score = r.score;
                if (o.angle < -180) o.angle += 360;
                if (o.angle > 180) o.angle -= 360;
                out.push_back(o);
                if ((int)out.size() == prm.max_pos) break;
                continue;
            }
            P2f lt((float)r.pt.x, (float)r.pt.y);
            P2f rt(lt.x + iW * (float)std::cos(rad), lt.y - iW * (float)std::sin(rad));
            P2f lb(lt.x + iH * (float)std::sin(rad), lt.y + iH * (float)std::cos(rad));
            P2f rb(rt.x + iH * (float)std::sin(rad), rt.y + iH * (float)std::cos(rad));
            P2f c((lt.x + rt.x + lb.x + rb.x) / 4.0f, (lt.y + rt.y + lb.y + rb.y) / 4.0f);
            fpm_result o;
            o.lt_x = lt.x; o.lt_y = lt.y; o.rt_x = rt.x; o.rt_y = rt.y;
            o.rb_x = rb.x; o.rb_y = rb.y; o.lb_x = lb.x; o.lb_y = lb.y;
            o.cx = c.x; o.cy = c.y; o.angle = r.angle; o.score = r.score;
            out.push_back(o);
        }
        return FPM_OK;
    }
};

static Mat8 from_strided(const uint8_t* p, int w, int h, size_t stride) {
    Mat8 m(w, h);
    for (int y = 0; y < h; ++y) std::memcpy(m.row(y), p + (size_t)y * stride, (size_t)w);
    return m;
}

}  // namespace orc

// -------------------------------------------------------------------------------------------------------
// C entry points (loaded by tests via ctypes)
// -------------------------------------------------------------------------------------------------------
extern "C" {

// the oracle carries its own copy of the reference defaults (TemplateMatcher.cpp:28-39)
void fpm_params_default(fpm_params* p) {
    std::memset(p, 0, sizeof(*p));
    p->max_pos = 70; p->min_reduce_area = 256; p->max_overlap = 0.0; p->score = 0.7;
    p->tolerance_angle = 0.0; p->use_simd = 1; p->subpixel = 0; p->tolerance_range = 0;
    p->semantics = FPM_SEMANTICS_QT; p->top_angle_step = 0.0;
}

void* orc_create(void) { return new orc::Matcher(); }
void orc_destroy(void* h) { delete (orc::Matcher*)h; }
void orc_set_params(void* h, const fpm_params* p) { ((orc::Matcher*)h)->prm = *p; }
void orc_get_params(void* h, fpm_params* p) { *p = ((orc::Matcher*)h)->prm; }

int orc_learn(void* h, const uint8_t* g, int w, int hh, size_t stride) {
    if (!g || w <= 0 || hh <= 0) return FPM_E_INVALID_ARG;
    return ((orc::Matcher*)h)->learn(orc::from_strided(g, w, hh, stride)) ? FPM_OK : FPM_E_INVALID_ARG;
}

int orc_match(void* h, const uint8_t* g, int w, int hh, size_t stride, fpm_result* out, int cap, int* n,
              double* seconds) {
    auto* m = (orc::Matcher*)h;
    *n = 0;
    if (!g || w <= 0 || hh <= 0) return FPM_E_INVALID_ARG;
    std::vector<fpm_result> res;
    int rc = m->match(orc::from_strided(g, w, hh, stride), res);
    if (rc != FPM_OK) return rc;
    *n = (int)res.size();
    for (int i = 0; i < (int)res.size() && i < cap; ++i) out[i] = res[i];
    if (seconds) *seconds = m->last_seconds;
    return (int)res.size() > cap ? FPM_E_CAPACITY : FPM_OK;
}

// counters of the last match: [angles, top candidates, live entering layer L-1 .. 0]
int orc_search_stats(void* h, int64_t* s, int cap) {
    auto* m = (orc::Matcher*)h;
    int n = 0;
    if (n < cap) s[n++] = m->stats.top_angles;
    if (n < cap) s[n++] = m->stats.top_candidates;
    for (int v : m->stats.live_per_layer)
        if (n < cap) s[n++] = v;
    return n;
}

// candidate records of the last match in push order (fpm_candidate, include/fpm.h); returns the count
int orc_candidates(void* h, fpm_candidate* out, int cap) {
    auto* m = (orc::Matcher*)h;
    int n = (int)m->stats.cands.size();
    for (int i = 0; i < n && i < cap; ++i) out[i] = m->stats.cands[i];
    return n;
}

// TM_CCORR arithmetic of the next matches: 0 = exact (the parity contract), 1 = OpenCV crossCorr in float32 DFTs
// (sensitivity mode for the reference-held screenshots; see orc::cross_corr_f32)
int orc_set_ccorr_mode(void* h, int mode) {
    if (mode != 0 && mode != 1) return FPM_E_INVALID_ARG;
    ((orc::Matcher*)h)->ccorr_mode = mode;
    return FPM_OK;
}

// the f32-DFT TM_CCORR map of one image and template (both u8, contiguous rows given by stride), for the KAT
// that checks it against numpy's float32 FFT and the exact sum
int orc_cross_corr_f32(const uint8_t* img, int w, int h, size_t is, const uint8_t* t, int tw, int th, size_t ts,
                       float* out) {
    if (tw > w || th > h || tw <= 0 || th <= 0) return FPM_E_INVALID_ARG;
    orc::MatF r;
    orc::cross_corr_f32(orc::from_strided(img, w, h, is), orc::from_strided(t, tw, th, ts), r);
    std::memcpy(out, r.px.data(), r.px.size() * sizeof(float));
    return FPM_OK;
}

// refinement decision trace of the next matches (diagnostic): rows of 19 doubles, see SearchStats::trace
void orc_set_trace(void* h, int on) { ((orc::Matcher*)h)->trace = on != 0; }
int orc_trace(void* h, double* out, int cap_rows) {
    auto* m = (orc::Matcher*)h;
    int n = (int)(m->stats.trace.size() / orc::kTraceCols);
    for (int i = 0; i < n && i < cap_rows; ++i)
        std::memcpy(out + (size_t)i * orc::kTraceCols, &m->stats.trace[(size_t)i * orc::kTraceCols],
                    sizeof(double) * orc::kTraceCols);
    return n;
}

// The top layer's peak sequence on a given f32 map (TemplateMatcher.cpp:179-210; MFC MatchToolDlg.cpp:860-888):
// s_BlockMax + getNextMaxLoc when by_block, else minMaxLoc + the painting getNextMaxLoc; at most 1 + iters peaks,
// stopping below thr.  out: (value, x, y) per peak; returns the count.  The map is copied (it gets painted).
int orc_peak_sequence(const float* map, int w, int h, int tw, int th, int by_block, int mfc, double overlap, int iters,
                      double thr, double* out) {
    orc::MatF m(w, h, 0.f);
    std::memcpy(m.px.data(), map, sizeof(float) * (size_t)w * h);
    int n = 0, px, py;
    double v;
    auto push = [&](double val, int x, int y) { out[3 * n] = val; out[3 * n + 1] = x; out[3 * n + 2] = y; ++n; };
    if (by_block) {
        orc::BlockMax bm(m, tw, th, mfc != 0);
        bm.get_max(&v, &px, &py);
        if (v < thr) return 0;
        push(v, px, py);
        for (int j = 0; j < iters; ++j) {
            orc::Matcher::next_max_loc_block(m, px, py, tw, th, v, overlap, bm);
            if (v < thr) break;
            push(v, px, py);
        }
    } else {
        orc::max_loc(m, 0, 0, w, h, &v, &px, &py);
        if (v < thr) return 0;
        push(v, px, py);
        for (int j = 0; j < iters; ++j) {
            orc::Matcher::next_max_loc(m, px, py, tw, th, v, overlap);
            if (v < thr) break;
            push(v, px, py);
        }
    }
    return n;
}

// top-layer candidates in reference push order: (x, y, score, angle) per entry
int orc_top_candidates(void* h, double* out, int cap) {
    auto* m = (orc::Matcher*)h;
    int n = (int)m->stats.top_list.size();
    for (int i = 0; i < n && i < cap; ++i) {
        out[4 * i + 0] = m->stats.top_list[i].pt.x;
        out[4 * i + 1] = m->stats.top_list[i].pt.y;
        out[4 * i + 2] = m->stats.top_list[i].score;
        out[4 * i + 3] = m->stats.top_list[i].angle;
    }
    return n;
}

int orc_template_info(void* h, int* levels, int* border) {
    auto* m = (orc::Matcher*)h;
    *levels = (int)m->T.pyr.size();
    *border = m->T.border;
    return m->T.learned ? FPM_OK : FPM_E_NOT_LEARNED;
}

int orc_template_level(void* h, int lv, int* w, int* hh, double* mean, double* norm, double* inv_area, int* eq1,
                       uint8_t* px, size_t stride) {
    auto* m = (orc::Matcher*)h;
    if (lv < 0 || lv >= (int)m->T.pyr.size()) return FPM_E_INVALID_ARG;
    const orc::Mat8& t = m->T.pyr[lv];
    *w = t.w; *hh = t.h; *mean = m->T.mean[lv]; *norm = m->T.norm[lv]; *inv_area = m->T.inv_area[lv];
    *eq1 = m->T.equal1[lv] ? 1 : 0;
    if (px)
        for (int y = 0; y < t.h; ++y) std::memcpy(px + (size_t)y * stride, t.row(y), (size_t)t.w);
    return FPM_OK;
}

void orc_pyr_down(const uint8_t* src, int w, int h, size_t ss, uint8_t* dst, size_t ds) {
    orc::Mat8 d = orc::pyr_down(orc::from_strided(src, w, h, ss));
    for (int y = 0; y < d.h; ++y) std::memcpy(dst + (size_t)y * ds, d.row(y), (size_t)d.w);
}

void orc_warp_affine(const uint8_t* src, int w, int h, size_t ss, const double m[6], uint8_t* dst, int dw, int dh,
                     size_t ds, int border) {
    orc::Mat8 d = orc::warp_affine(orc::from_strided(src, w, h, ss), m, dw, dh, border);
    for (int y = 0; y < d.h; ++y) std::memcpy(dst + (size_t)y * ds, d.row(y), (size_t)d.w);
}

void orc_rotation_matrix(float cx, float cy, double angle, double m[6]) {
    orc::rotation_matrix(orc::P2f(cx, cy), angle, m);
}

int orc_ncc_map(void* h, const uint8_t* src, int w, int hh, size_t ss, int layer, int fold, float* out) {
    auto* m = (orc::Matcher*)h;
    if (!m->T.learned) return FPM_E_NOT_LEARNED;
    if (layer < 0 || layer >= (int)m->T.pyr.size()) return FPM_E_INVALID_ARG;
    orc::MatF res;
    int saved = m->prm.use_simd;
    m->prm.use_simd = 1;
    m->match_template(orc::from_strided(src, w, hh, ss), layer, fold != 0, res);
    m->prm.use_simd = saved;
    std::memcpy(out, res.px.data(), res.px.size() * sizeof(float));
    return FPM_OK;
}

// filterWithRotatedRect (TemplateMatcher.cpp:1133-1194) on n rectangles (corners[6i..6i+5] = ptLT, ptRT, ptRB) with
// scores, in the given order: the surviving indices in order; returns their count
int orc_filter_rotated_rect(const float* corners, const double* scores, int n, double max_overlap, int32_t* keep) {
    std::vector<orc::MatchParam> v((size_t)n);
    for (int i = 0; i < n; ++i) {
        const float* c = corners + 6 * (size_t)i;
        v[i].rectR = orc::rotrect_from3(orc::P2f(c[0], c[1]), orc::P2f(c[2], c[3]), orc::P2f(c[4], c[5]));
        v[i].score = scores[i];
        v[i].origin = i;
        v[i].del = false;
    }
    orc::Matcher::filter_with_rotated_rect(v, max_overlap);
    for (size_t i = 0; i < v.size(); ++i) keep[i] = v[i].origin;
    return (int)v.size();
}

// rotated-rectangle overlap primitive (filterWithRotatedRect's building block) for KATs:
// rects given as (ptLT, ptRT, ptRB); returns the intersection type, *area = contourArea after sortPtWithCenter
int orc_rotrect_overlap(const float a[6], const float b[6], double* area, int* npts) {
    orc::RotRect r1 = orc::rotrect_from3(orc::P2f(a[0], a[1]), orc::P2f(a[2], a[3]), orc::P2f(a[4], a[5]));
    orc::RotRect r2 = orc::rotrect_from3(orc::P2f(b[0], b[1]), orc::P2f(b[2], b[3]), orc::P2f(b[4], b[5]));
    std::vector<orc::P2f> pts;
    int t = orc::rotrect_intersection(r1, r2, pts);
    *npts = (int)pts.size();
    if (pts.size() >= 3) {
        orc::Matcher::sort_pt_with_center(pts);
        *area = orc::contour_area(pts);
    } else {
        *area = 0;
    }
    return t;
}

}  // extern "C"
