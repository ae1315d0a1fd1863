// fpm_rrect.h — the exact rotated-rectangle pair test of filterWithRotatedRect (TemplateMatcher.cpp:1133-1194),
// shared by the host tail and the device pair kernel (k_overlap_pairs).  Compiled for x86 and gfx950 with
// -ffp-contract=off: plain IEEE float/double +,-,*,/ and correctly rounded sqrt (HIP's default on the device), so both
// give the same bits.  The one transcendental of the test -- acos in the reference's point sort key
// (sortPtWithCenter) -- is never evaluated here: sort_pts_fast orders the points without it whenever the order does
// not depend on acos's last bits and reports the other cases, which the host then finishes with its own acos.
#pragma once
#include "fpm_geom.h"

namespace fpm {

FPM_HD float fmax_std(float a, float b) { return (a < b) ? b : a; }   // std::max
FPM_HD float fmin_std(float a, float b) { return (b < a) ? b : a; }   // std::min

// cv::rotatedRectangleIntersection (OpenCV 4.5.x) on the two rectangles' corners A, B (rrect corners, in order) and
// their sizes: 0 = INTERSECT_NONE, 1 = INTERSECT_PARTIAL, 2 = INTERSECT_FULL; the intersection points go to pts
// (room for 24: at most 16 edge crossings + 8 corners before the near-duplicate pass, at most 8 after it).
// FULL = false (the device kernel): where more than 8 points survive the near-duplicate pass (rare) it returns -1 instead
// of running the reference's closest-pair reduction, whose 24 x 24 distance table would otherwise sit in every lane's
// scratch (2.7 KB per lane: few waves in flight); the caller hands such a pair to the host.
template <bool FULL = true>
FPM_HD int rrect_isect_pts(float wa, float ha, float wb, float hb, const F2* A, const F2* B, F2* pts, int* np) {
    int n = 0;
    F2 eA[4], eB[4];
    float eps = 1e-6f * fmax_std(wa * ha, wb * hb);
    bool coincident = true;
    for (int i = 0; i < 4 && coincident; ++i)
        coincident = !(fabsf(A[i].x - B[i].x) > eps || fabsf(A[i].y - B[i].y) > eps);
    if (coincident) {
        for (int i = 0; i < 4; ++i) pts[i] = A[i];
        *np = 4;
        return 2;
    }
    for (int i = 0; i < 4; ++i) {
        const int k = (i + 1) & 3;
        eA[i] = f2(A[k].x - A[i].x, A[k].y - A[i].y);
        eB[i] = f2(B[k].x - B[i].x, B[k].y - B[i].y);
    }
    for (int i = 0; i < 4; ++i) {
        eps = fmin_std(eps, sqrtf(eA[i].x * eA[i].x + eA[i].y * eA[i].y));
        eps = fmin_std(eps, sqrtf(eB[i].x * eB[i].x + eB[i].y * eB[i].y));
    }
    eps = fmax_std(1e-16f, eps);
    int kind = 2;
    // edge-edge crossings
    for (int i = 0; i < 4; ++i) {
        for (int j = 0; j < 4; ++j) {
            const float dx = B[j].x - A[i].x, dy = B[j].y - A[i].y;
            const float det = eB[j].x * eA[i].y - eA[i].x * eB[j].y;
            if (fabs((double)det) < 1e-12) continue;
            const float ta = (eB[j].x * dy - eB[j].y * dx) / det;
            const float tb = (eA[i].x * dy - eA[i].y * dx) / det;
            if (!__builtin_isfinite(ta) || !__builtin_isfinite(tb)) continue;
            if (ta >= 0.0f && ta <= 1.0f && tb >= 0.0f && tb <= 1.0f)
                pts[n++] = f2(A[i].x + eA[i].x * ta, A[i].y + eA[i].y * ta);
        }
    }
    if (n > 0) kind = 1;
    // corners of one rectangle inside the other (sign test against the 4 edge lines)
    auto inside = [](const F2& p, const F2* Q, const F2* eQ) {
        int pos = 0, neg = 0;
        for (int j = 0; j < 4; ++j) {
            const float a = -eQ[j].y, b = eQ[j].x;
            const float c = -(a * Q[j].x + b * Q[j].y);
            const float s = a * p.x + b * p.y + c;
            if (s >= 0) ++pos; else ++neg;
        }
        return pos == 4 || neg == 4;
    };
    for (int i = 0; i < 4; ++i)
        if (inside(A[i], B, eB)) pts[n++] = A[i];
    for (int i = 0; i < 4; ++i)
        if (inside(B[i], A, eA)) pts[n++] = B[i];
    if (n == 0) { *np = 0; return 0; }
    // drop near-duplicates (swap-with-last).  The pairwise distances are only read when more than 8 points remain,
    // which is rare: a first pass without them, and only then the pass that records them, from the same points.
    {
        F2 q[24];
        int m = n;
        for (int i = 0; i < n; ++i) q[i] = pts[i];
        for (int i = 0; i < m; ++i) {
            const F2 p = q[i];
            int j = i + 1;
            while (j < m) {
                const float ddx = q[j].x - p.x, ddy = q[j].y - p.y;
                if (ddx * ddx + ddy * ddy <= eps) {
                    if (j < m - 1) q[j] = q[m - 1];
                    --m;
                    continue;
                }
                ++j;
            }
        }
        if (m <= 8) {
            for (int i = 0; i < m; ++i) pts[i] = q[i];
            *np = m;
            return kind;
        }
    }
    if constexpr (!FULL) {
        *np = n;
        return -1;
    }
    const int stride = n;
    float dist[24 * 24];
    int slot[24];
    for (int i = 0; i < n * n; ++i) dist[i] = 0.f;
    for (int i = 0; i < n; ++i) {
        slot[i] = i;
        const F2 p = pts[i];
        int j = i + 1;
        while (j < n) {
            const float ddx = pts[j].x - p.x, ddy = pts[j].y - p.y;
            const float d2 = ddx * ddx + ddy * ddy;
            if (d2 <= eps) {
                if (j < n - 1) pts[j] = pts[n - 1];
                --n;
                continue;
            }
            dist[(size_t)i * stride + j] = d2;
            ++j;
        }
    }
    while (n > 8) {
        int bj = 1;
        float bd = dist[1];
        for (int i = 0; i < n - 1; ++i) {
            const float* row = dist + (size_t)stride * slot[i];
            for (int j = i + 1; j < n; ++j)
                if (row[slot[j]] < bd) { bd = row[slot[j]]; bj = j; }
        }
        if (bj < n - 1) { pts[bj] = pts[n - 1]; slot[bj] = slot[n - 1]; }
        --n;
    }
    *np = n;
    return kind;
}

// cv::contourArea of the points in their given order: |shoelace| / 2 in double
FPM_HD double contour_area_pts(const F2* pts, int n) {
    if (n == 0) return 0.;
    double acc = 0;
    F2 prev = pts[n - 1];
    for (int i = 0; i < n; ++i) {
        acc += (double)prev.x * pts[i].y - (double)prev.y * pts[i].x;
        prev = pts[i];
    }
    return fabs(acc * 0.5);
}

// sortPtWithCenter's permutation (TemplateMatcher.cpp:1093-1131) where it is decided without evaluating acos: the
// host's sort_pts_center (fpm_host.cpp) with its acos-free fast path only (two equal arguments have equal acos values,
// so that comparison needs no acos either).  Returns false -- pts then partly reordered and to be redone by the host --
// for more than 16 points, an off-row |x| > 1/2, or a comparison of two different keys closer than 2^-16 (the cases
// in which the host evaluates acos and its last bits could matter).
FPM_HD bool sort_pts_fast(F2* pts, int n) {
    if (n > 16) return false;
    F2 ctr = f2(0.f, 0.f);
    for (int i = 0; i < n; ++i) { ctr.x += pts[i].x; ctr.y += pts[i].y; }
    ctr.x = ctr.x / n;
    ctr.y = ctr.y / n;
    F2 p[16];
    float xs[16];
    int band[16];
    for (int i = 0; i < n; ++i) {
        const F2 d = f2(pts[i].x - ctr.x, pts[i].y - ctr.y);
        p[i] = pts[i];
        xs[i] = 0.f;
        if (d.y < 0 || d.y > 0) {
            const float nn = d.x * d.x + d.y * d.y;
            const float x = d.x / nn;
            if (!(fabsf(x) <= 0.5f)) return false;
            xs[i] = x;
            band[i] = d.y < 0 ? 1 : 3;
        } else {
            band[i] = (d.x - ctr.x > 0) ? 0 : 2;
        }
    }
    bool ok = true;
    auto less = [&](int ba, float xa, int bb, float xb) {
        if (ba != bb) return ba < bb;
        if (ba == 0 || ba == 2) return false;
        if (fabsf(xa - xb) >= 0x1p-16f) return ba == 1 ? xa > xb : xa < xb;
        if (xa == xb) return false;   // equal arguments: equal acos values, so neither key is less
        ok = false;
        return false;
    };
    for (int i = 1; i < n; ++i) {   // libstdc++ __insertion_sort
        const F2 vp = p[i];
        const float vx = xs[i];
        const int vb = band[i];
        int j = i;
        while (j > 0 && less(vb, vx, band[j - 1], xs[j - 1])) {
            p[j] = p[j - 1]; xs[j] = xs[j - 1]; band[j] = band[j - 1];
            --j;
        }
        if (!ok) return false;
        p[j] = vp; xs[j] = vx; band[j] = vb;
    }
    for (int i = 0; i < n; ++i) pts[i] = p[i];
    return true;
}

}  // namespace fpm
