// fpm_geom.h — search geometry shared by host and device code.
//
// Every function here is compiled twice (x86 host and gfx950 device) with -ffp-contract=off and must give
// bit-identical results on both: plain IEEE float/double +,-,*,/ in the reference's operation order, no
// transcendental calls.  cos/sin values are passed in (computed once on the host with glibc and shipped to
// HBM as the angle table), which is what makes device-side geometry equal to the reference's by
// construction.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define FPM_HD __host__ __device__ __forceinline__

namespace fpm {

constexpr double kPi = 3.1415926535897932384626433832795;  // CV_PI
constexpr double kD2R = kPi / 180.0;                         // D2R, DataStructures.h:11
constexpr double kR2D = 180.0 / kPi;                         // R2D, DataStructures.h:12
constexpr double kVisionTol = 0.0000001;                     // VISION_TOLERANCE, DataStructures.h:10
constexpr int kMatchCandidateNum = 5;                        // MATCH_CANDIDATE_NUM, DataStructures.h:13

struct F2 { float x, y; };

FPM_HD F2 f2(float x, float y) { F2 r; r.x = x; r.y = y; return r; }

// ptRotatePt2f (TemplateMatcher.cpp:971-982) with c = cos(angle), s = sin(angle) supplied.
FPM_HD F2 rotate_pt(F2 in, F2 org, double c, double s) {
    double h = org.y * 2;
    double y1 = h - in.y, y2 = h - org.y;
    double x = (in.x - org.x) * c - (y1 - org.y) * s + org.x;
    double y = (in.x - org.x) * s + (y1 - org.y) * c + y2;
    y = -y + h;
    return f2((float)x, (float)y);
}

// cv::getRotationMatrix2D(center, angle, 1) with c = cos(angle*CV_PI/180), s = sin(...) supplied.
FPM_HD void rotation_matrix(F2 ctr, double c, double s, double m[6]) {
    double alpha = c * 1.0, beta = s * 1.0;
    m[0] = alpha; m[1] = beta; m[2] = (1 - alpha) * ctr.x - beta * ctr.y;
    m[3] = -beta; m[4] = alpha; m[5] = beta * ctr.x + (1 - alpha) * ctr.y;
}

// cv::warpAffine's inversion of the forward matrix (no WARP_INVERSE_MAP), in place.
FPM_HD void invert_affine(double M[6]) {
    double D = M[0] * M[4] - M[1] * M[3];
    D = D != 0 ? 1. / D : 0;
    double A11 = M[4] * D, A22 = M[0] * D;
    M[0] = A11; M[1] *= -D;
    M[3] *= -D; M[4] = A22;
    double b1 = -M[0] * M[2] - M[1] * M[5];
    double b2 = -M[3] * M[2] - M[4] * M[5];
    M[2] = b1; M[5] = b2;
}

// getRotatedROI (TemplateMatcher.cpp:1074-1090): forward matrix of the (w+6)x(h+6) ROI around lt rotated
// by the angle whose cos/sin (of angle*D2R) are given; returns the INVERTED matrix ready for sampling.
FPM_HD void roi_matrix(int src_w, int src_h, F2 lt, double c, double s, double M[6]) {
    F2 ctr = f2((src_w - 1) / 2.0f, (src_h - 1) / 2.0f);
    F2 ltr = rotate_pt(lt, ctr, c, s);
    rotation_matrix(ctr, c, s, M);
    M[2] -= ltr.x - 3;
    M[5] -= ltr.y - 3;
    invert_affine(M);
}

// Fixed-point sampling constants of cv::warpAffine INTER_LINEAR.
constexpr int kAbBits = 10, kAbScale = 1 << kAbBits, kInterBits = 5, kInterTab = 1 << kInterBits;
constexpr int kRoundDelta = kAbScale / kInterTab / 2;

// One score/position record of a refinement ROI (7x7 NCC map reduced), written by the device.
struct RoiRecord {
    float score;        // minMaxLoc max
    int16_t mx, my;     // its location in the 7x7 map
    int32_t on_border;  // bPosOnBorder (TemplateMatcher.cpp:321-322)
    float vec[9];       // vecResult[x+1][y+1] stored at [(x+1)*3 + (y+1)] (TemplateMatcher.cpp:323-328)
};

// Per-candidate refinement state in HBM.
struct CandState {
    F2 lt;              // ptLT at the current layer's resolution
    int32_t node;       // angle-tree node index at the current level (-1 at the top)
    int32_t alive;      // 1 while the candidate descends
    int32_t reached0;   // 1 if it entered layer 0 (host finishes it)
    int32_t pad;
};

}  // namespace fpm
