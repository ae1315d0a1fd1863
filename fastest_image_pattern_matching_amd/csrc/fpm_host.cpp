// fpm_host.cpp — host stages of the search: final score filter, rotated-rectangle overlap suppression and the
// optional sub-pixel quadric fit.  These are O(n^2)/O(1) control code over a few hundred results, run once
// per search after the single device->host copy; they follow the reference line by line so that the surviving
// set and order are identical (TemplateMatcher.cpp:373-395, 984-1194) and the OpenCV geometry primitives
// they call (OpenCV 4.5.x semantics).  Compile with -ffp-contract=off.
#include "fpm_host.h"
#include "fpm_rrect.h"

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cmath>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>

namespace fpm {
#ifdef FPM_HOST_STATS
long g_stats[40];
#endif

bool score_big2small(const HostMatch& a, const HostMatch& b) { return a.score > b.score; }

// worker threads for the overlap filter's independent components: FPM_HOST_THREADS if set (>= 1), else the
// hardware concurrency capped at 8
int host_thread_count() {
    static const int n = [] {
        if (const char* e = std::getenv("FPM_HOST_THREADS")) {
            const int v = std::atoi(e);
            if (v >= 1) return std::min(v, 64);
        }
        const int hw = (int)std::thread::hardware_concurrency();
        return std::max(1, std::min(hw, 8));
    }();
    return n;
}

// Persistent worker pool for the host tail's independent pieces (per-candidate geometry, per-cluster overlap
// tests).  Thread creation per search cost more than the work it spread; the workers spin for a short while after
// a region (the tail runs a few regions back to back) and then sleep on a condition variable.  One region at a time:
// a caller that finds the pool busy (another context finishing on another host thread) runs its tasks inline.
// Results never depend on which thread runs a task.
namespace {
// spin-wait hint: the x86 pause instruction where there is one, a scheduler yield elsewhere
inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#else
    std::this_thread::yield();
#endif
}

struct Pool {
    std::mutex m, region;
    std::condition_variable cv;
    std::atomic<uint64_t> gen{0};
    const std::function<void(int)>* fn = nullptr;   // guarded by m; null between regions
    int ntasks = 0;
    std::atomic<int> next{0}, done{0}, active{0};
    std::atomic<int64_t> spin_until{0};   // steady_clock ns: idle workers spin instead of sleeping until then

    static int64_t now_ns() {
        return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
            .count();
    }
    void worker() {
        uint64_t seen = 0;
        for (;;) {
            auto t0 = std::chrono::steady_clock::now();
            while (gen.load(std::memory_order_acquire) == seen) {
                if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(300) &&
                    now_ns() >= spin_until.load(std::memory_order_relaxed)) {
                    std::unique_lock<std::mutex> lk(m);
                    cv.wait(lk, [&] {
                        return gen.load(std::memory_order_acquire) != seen ||
                               now_ns() < spin_until.load(std::memory_order_relaxed);
                    });
                    t0 = std::chrono::steady_clock::now();
                } else {
                    cpu_relax();
                }
            }
            const std::function<void(int)>* f;
            int nt;
            {
                std::lock_guard<std::mutex> lk(m);
                seen = gen.load(std::memory_order_acquire);
                f = fn;
                nt = ntasks;
                if (f) active.fetch_add(1, std::memory_order_acq_rel);
            }
            if (!f) continue;
            for (int t = next.fetch_add(1); t < nt; t = next.fetch_add(1)) {
                (*f)(t);
                done.fetch_add(1, std::memory_order_acq_rel);
            }
            active.fetch_sub(1, std::memory_order_acq_rel);
        }
    }
};

// Leaked on purpose: the detached workers block forever, nothing is torn down at exit -- so libfpm_hip.so must not be
// dlclose'd while the process lives (ctypes never unloads it; the drop-in links it)
Pool* pool_instance(int workers) {
    static Pool* p = [&] {
        Pool* q = new Pool;
        for (int i = 0; i < workers; ++i) std::thread([q] { q->worker(); }).detach();
        return q;
    }();
    return p;
}
}  // namespace

// FPM_HOST_WARM: 0 turns the warm-up off (processes sharing the host with other work), a positive value caps the
// spin in microseconds (default 10000); the warm-up only moves when the tail's workers start, never its results
static int host_warm_cap_us() {
    static const int cap = [] {
        const char* e = std::getenv("FPM_HOST_WARM");
        return e ? std::max(0, atoi(e)) : 10000;
    }();
    return cap;
}

void host_pool_warm(int us) {
    const int nthreads = host_thread_count();
    us = std::min(us, host_warm_cap_us());
    if (nthreads <= 1 || us <= 0) return;
    Pool* p = pool_instance(nthreads - 1);
    p->spin_until.store(Pool::now_ns() + (int64_t)us * 1000, std::memory_order_relaxed);
    std::lock_guard<std::mutex> lk(p->m);
    p->cv.notify_all();
}

void host_parallel(int ntasks, const std::function<void(int)>& fn) {
    const int nthreads = host_thread_count();
    if (ntasks <= 1 || nthreads <= 1) {
        for (int t = 0; t < ntasks; ++t) fn(t);
        return;
    }
    Pool* p = pool_instance(nthreads - 1);
    std::unique_lock<std::mutex> reg(p->region, std::try_to_lock);
    if (!reg.owns_lock()) {
        for (int t = 0; t < ntasks; ++t) fn(t);
        return;
    }
    {
        std::lock_guard<std::mutex> lk(p->m);
        p->fn = &fn;
        p->ntasks = ntasks;
        p->next.store(0);
        p->done.store(0);
        p->gen.fetch_add(1, std::memory_order_acq_rel);
    }
    p->cv.notify_all();
    static const bool trace = [] { const char* e = std::getenv("FPM_POOL_TRACE"); return e && *e == '1'; }();
    const auto r0 = std::chrono::steady_clock::now();
    int mine = 0;
    for (int t = p->next.fetch_add(1); t < ntasks; t = p->next.fetch_add(1)) {
        fn(t);
        ++mine;
        p->done.fetch_add(1, std::memory_order_acq_rel);
    }
    while (p->done.load(std::memory_order_acquire) < ntasks) cpu_relax();
    {
        std::lock_guard<std::mutex> lk(p->m);
        p->fn = nullptr;   // workers that wake from here on skip this region
    }
    while (p->active.load(std::memory_order_acquire) > 0) cpu_relax();
    if (trace)
        fprintf(stderr, "pool region: %d tasks, %d by the caller, %.1f us\n", ntasks, mine,
                std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - r0).count());
}

static inline double len2(float x, float y) { return std::sqrt((double)x * x + (double)y * y); }

RRect rrect_from3(F2 p1, F2 p2, F2 p3) {
    RRect r;
    r.c = f2(0.5f * (p1.x + p3.x), 0.5f * (p1.y + p3.y));
    const F2 e0 = f2(p1.x - p2.x, p1.y - p2.y);
    const F2 e1 = f2(p2.x - p3.x, p2.y - p3.y);
    // width = the edge whose slope lies in [-1, 1]; preference to e1 as in OpenCV
    const bool w_is_e1 = std::fabs(e1.y) < std::fabs(e1.x);
    const F2 we = w_is_e1 ? e1 : e0, he = w_is_e1 ? e0 : e1;
    r.angle = std::atan(we.y / we.x) * 180.0f / (float)kPi;
    r.w = (float)len2(we.x, we.y);
    r.h = (float)len2(he.x, he.y);
    return r;
}

void rrect_corners(const RRect& r, F2 pt[4]) {
    const double rad = r.angle * kPi / 180.;
    const float b = (float)std::cos(rad) * 0.5f;
    const float a = (float)std::sin(rad) * 0.5f;
    pt[0] = f2(r.c.x - a * r.h - b * r.w, r.c.y + b * r.h - a * r.w);
    pt[1] = f2(r.c.x + a * r.h - b * r.w, r.c.y - b * r.h - a * r.w);
    pt[2] = f2(2 * r.c.x - pt[0].x, 2 * r.c.y - pt[0].y);
    pt[3] = f2(2 * r.c.x - pt[1].x, 2 * r.c.y - pt[1].y);
}

// cv::rotatedRectangleIntersection on precomputed corners (fpm_rrect.h, shared with the device pair kernel)
static int rrect_isect(const RRect& ra, const RRect& rb, const F2* A, const F2* B, F2* pts, int* np) {
    return rrect_isect_pts(ra.w, ra.h, rb.w, rb.h, A, B, pts, np);
}

int rrect_intersection(const RRect& ra, const RRect& rb, std::vector<F2>& pts) {
    F2 A[4], B[4], p[24];
    rrect_corners(ra, A);
    rrect_corners(rb, B);
    int n = 0;
    const int kind = rrect_isect(ra, rb, A, B, p, &n);
    pts.assign(p, p + n);
    return kind;
}

// sortPtWithCenter (TemplateMatcher.cpp:1093-1131) with its own keys: acos(x) * R2D above the centre, 360 - that
// below, x = dot / |v|^2 (the squared norm is the reference's), 0 / 180 on the centre's row; std::sort by key.
static void sort_pts_keyed(F2* pts, int n) {
    F2 ctr = f2(0.f, 0.f);
    for (int i = 0; i < n; ++i) { ctr.x += pts[i].x; ctr.y += pts[i].y; }
    ctr.x = ctr.x / n;
    ctr.y = ctr.y / n;
    std::pair<F2, double> keyed[24];   // n <= 24 (rrect_isect)
    for (int i = 0; i < n; ++i) {
        const F2 d = f2(pts[i].x - ctr.x, pts[i].y - ctr.y);
        const float nn = d.x * d.x + d.y * d.y;
        double key;
        if (d.y < 0) key = std::acos(d.x / nn) * kR2D;
        else if (d.y > 0) key = 360 - std::acos(d.x / nn) * kR2D;
        else key = (d.x - ctr.x > 0) ? 0 : 180;
        keyed[i] = std::make_pair(pts[i], key);
    }
    std::sort(keyed, keyed + n,
              [](const std::pair<F2, double> l, const std::pair<F2, double> r) { return l.second < r.second; });
    for (int i = 0; i < n; ++i) pts[i] = keyed[i].first;
}

// The same permutation without a transcendental per point.  For n <= 16 libstdc++'s std::sort is one insertion
// sort (introsort stops at 16 elements), so the result depends only on the outcomes of `key_a < key_b`.  With every
// off-row |x| <= 1/2 the keys fall in disjoint bands -- row-left 0 < above (60..120) < row-right 180 < below
// (240..300) -- and within a band acos is strictly monotone with slope >= 1 in magnitude, so two x at least 2^-16
// apart have keys ordered as their x (acosf's error is a few ulp of at most 2^-22); only closer pairs, which may
// round to equal keys, compare acosf results exactly as the key does (both keys are monotone in the float acosf).
// Anything outside that envelope takes the keyed path.
static void sort_pts_center(F2* pts, int n) {
    if (n > 16) { sort_pts_keyed(pts, n); return; }
    F2 ctr = f2(0.f, 0.f);
    for (int i = 0; i < n; ++i) { ctr.x += pts[i].x; ctr.y += pts[i].y; }
    ctr.x = ctr.x / n;
    ctr.y = ctr.y / n;
    struct E { F2 p; float x; int band; };
    E e[16];
    for (int i = 0; i < n; ++i) {
        const F2 d = f2(pts[i].x - ctr.x, pts[i].y - ctr.y);
        e[i].p = pts[i];
        e[i].x = 0.f;
        if (d.y < 0 || d.y > 0) {
            const float nn = d.x * d.x + d.y * d.y;
            const float x = d.x / nn;
            if (!(std::fabs(x) <= 0.5f)) { sort_pts_keyed(pts, n); return; }
            e[i].x = x;
            e[i].band = d.y < 0 ? 1 : 3;
        } else {
            e[i].band = (d.x - ctr.x > 0) ? 0 : 2;
        }
    }
    auto less = [](const E& a, const E& b) {
        if (a.band != b.band) return a.band < b.band;
        if (a.band == 0 || a.band == 2) return false;
        if (std::fabs(a.x - b.x) >= 0x1p-16f) return a.band == 1 ? a.x > b.x : a.x < b.x;
        const float fa = std::acos(a.x), fb = std::acos(b.x);
        return a.band == 1 ? fa < fb : fa > fb;
    };
    for (int i = 1; i < n; ++i) {   // libstdc++ __insertion_sort
        const E v = e[i];
        int j = i;
        while (j > 0 && less(v, e[j - 1])) { e[j] = e[j - 1]; --j; }
        e[j] = v;
    }
    for (int i = 0; i < n; ++i) pts[i] = e[i].p;
}

void sort_pt_with_center(std::vector<F2>& pts) {
    if (!pts.empty()) sort_pts_center(pts.data(), (int)pts.size());
}

void sort_pt_with_center_keyed(std::vector<F2>& pts) {
    if (!pts.empty()) sort_pts_keyed(pts.data(), (int)pts.size());
}

static double contour_area_a(const F2* pts, int n) { return contour_area_pts(pts, n); }

double contour_area(const std::vector<F2>& pts) { return contour_area_a(pts.data(), (int)pts.size()); }

// filterWithRotatedRect's decision for one pair (pair_del below, without the score rule): does a's overlap with b
// exceed max_overlap (ratio to a's area)
bool rrect_pair_drops(const RRect& ra, const RRect& rb, double max_overlap) {
    F2 A[4], B[4], p[24];
    rrect_corners(ra, A);
    rrect_corners(rb, B);
    int np = 0;
    const int kind = rrect_isect(ra, rb, A, B, p, &np);
    if (kind == 0) return false;
    if (kind == 2) return true;
    if (np < 3) return false;
    sort_pts_center(p, np);
    return contour_area_a(p, np) / (ra.w * ra.h) > max_overlap;
}


void filter_with_score(std::vector<HostMatch>& v, double score) {
    // std::sort's permutation depends only on the comparison results, so sorting light (score, index) keys with
    // the same comparator reproduces the reference's order of equal scores; the heavy records move once
    struct K { double score; int i; };
    std::vector<K> k(v.size());
    for (size_t i = 0; i < v.size(); ++i) k[i] = {v[i].score, (int)i};
    std::sort(k.begin(), k.end(), [](const K& a, const K& b) { return a.score > b.score; });
    size_t n = 0;
    while (n < k.size() && !(k[n].score < score)) ++n;
    std::vector<HostMatch> out;
    out.reserve(n);
    for (size_t i = 0; i < n; ++i) out.push_back(v[k[i].i]);
    v.swap(out);
}

void filter_with_rotated_rect(std::vector<HostMatch>& v, double max_overlap) {
    if (v.empty()) return;
    const int n = (int)v.size();
    // FPM_TAIL_TIMES=1: phase clocks on stderr (profiling aid)
    static const bool tail_times = [] { const char* e = std::getenv("FPM_TAIL_TIMES"); return e && *e == '1'; }();
    using clk = std::chrono::steady_clock;
    const clk::time_point q0 = clk::now();
    clk::time_point q1 = q0, q2 = q0, q3 = q0;
    // corner bounding boxes: pairs whose boxes are > 1 px apart cannot have an edge crossing or a contained corner,
    // so rrect_intersection would return INTERSECT_NONE; skipping them keeps the reference's O(n^2) loop order
    // and deletions exactly while avoiding the exact test for far-apart detections
    std::vector<float> box((size_t)4 * n);
    std::vector<F2> corners((size_t)4 * n);
    auto geom = [&](int i0, int i1) {
        for (int i = i0; i < i1; ++i) {
            F2* c = &corners[(size_t)4 * i];
            rrect_corners(v[i].rect, c);
            float x0 = c[0].x, x1 = c[0].x, y0 = c[0].y, y1 = c[0].y;
            for (int k = 1; k < 4; ++k) {
                x0 = std::min(x0, c[k].x); x1 = std::max(x1, c[k].x);
                y0 = std::min(y0, c[k].y); y1 = std::max(y1, c[k].y);
            }
            box[4 * i] = x0 - 1.f; box[4 * i + 1] = y0 - 1.f; box[4 * i + 2] = x1 + 1.f; box[4 * i + 3] = y1 + 1.f;
        }
    };
    if (n <= 512) geom(0, n);
    else host_parallel((n + 511) / 512, [&](int t) { geom(t * 512, std::min(n, t * 512 + 512)); });
    q1 = clk::now();
    // the reference's inner-loop body for (i, j), boxes overlapping: the index it deletes, or -1
    auto pair_del = [&](int i, int j) {
        F2 pts[24];
        int np = 0;
        const int kind = rrect_isect(v[i].rect, v[j].rect, &corners[(size_t)4 * i], &corners[(size_t)4 * j], pts, &np);
#ifdef FPM_HOST_STATS
        g_stats[kind]++; g_stats[3 + np]++;
#endif
        if (kind == 0) return -1;
        bool drop = kind == 2;
        if (kind == 1) {
            if (np < 3) return -1;
            sort_pts_center(pts, np);
            const double ratio = contour_area_a(pts, np) / (v[i].rect.w * v[i].rect.h);
            drop = ratio > max_overlap;
        }
        return drop ? ((v[i].score >= v[j].score) ? j : i) : -1;
    };
    auto pair = [&](int i, int j) {
        const int d = pair_del(i, j);
        if (d >= 0) v[d].del = true;
    };
    auto overlap = [&](int i, int j) {
        const float* bi = &box[4 * i];
        const float* bj = &box[4 * j];
        return !(bj[0] > bi[2] || bj[2] < bi[0] || bj[1] > bi[3] || bj[3] < bi[1]);
    };
    if (n <= 64) {
        for (int i = 0; i + 1 < n; ++i) {
            if (v[i].del) continue;
            for (int j = i + 1; j < n; ++j)
                if (!v[j].del && overlap(i, j)) pair(i, j);
        }
    } else {
        // uniform grid over the boxes (cell = the largest box extent): for each i only the j > i whose boxes
        // overlap its box, in ascending order -- the same (i, j) sequence as the full loop minus no-op pairs
        float gx0 = box[0], gy0 = box[1], gx1 = box[2], gy1 = box[3], cs = 1.f;
        for (int i = 0; i < n; ++i) {
            gx0 = std::min(gx0, box[4 * i]); gy0 = std::min(gy0, box[4 * i + 1]);
            gx1 = std::max(gx1, box[4 * i + 2]); gy1 = std::max(gy1, box[4 * i + 3]);
            cs = std::max(cs, std::max(box[4 * i + 2] - box[4 * i], box[4 * i + 3] - box[4 * i + 1]));
        }
        const int gnx = std::min(1024, (int)((gx1 - gx0) / cs) + 1), gny = std::min(1024, (int)((gy1 - gy0) / cs) + 1);
        const float sx = gnx / std::max(gx1 - gx0, 1e-3f), sy = gny / std::max(gy1 - gy0, 1e-3f);
        auto cell = [&](float x, float s_, float o, int nmax) { return std::min(nmax - 1, std::max(0, (int)((x - o) * s_))); };
        // cell -> ascending box indices, as CSR (count, prefix sum, fill)
        const size_t ncell = (size_t)gnx * gny;
        std::vector<int> cell_off(ncell + 1, 0), cell_box;
        std::vector<int4> span(n);   // cx0, cy0, cx1, cy1 per box
        for (int i = 0; i < n; ++i) {
            span[i] = make_int4(cell(box[4 * i], sx, gx0, gnx), cell(box[4 * i + 1], sy, gy0, gny),
                                cell(box[4 * i + 2], sx, gx0, gnx), cell(box[4 * i + 3], sy, gy0, gny));
            for (int cy = span[i].y; cy <= span[i].w; ++cy)
                for (int cx = span[i].x; cx <= span[i].z; ++cx) cell_off[(size_t)cy * gnx + cx + 1]++;
        }
        for (size_t c = 0; c < ncell; ++c) cell_off[c + 1] += cell_off[c];
        cell_box.resize(cell_off[ncell]);
        {
            std::vector<int> fill(cell_off.begin(), cell_off.end() - 1);
            for (int i = 0; i < n; ++i)
                for (int cy = span[i].y; cy <= span[i].w; ++cy)
                    for (int cx = span[i].x; cx <= span[i].z; ++cx) cell_box[fill[(size_t)cy * gnx + cx]++] = i;
        }
        // v is sorted by descending score, so pair(i, j) with i < j only ever deletes j: i is decided by the pairs
        // (i', i), i' < i, with overlapping boxes.  Overlapping boxes share a grid cell, so the sets of boxes
        // connected through shared cells are closed under the overlap relation and independent of each other; they
        // are processed in parallel, each in the reference's ascending (i, j) order -- the same deletions exactly.
        std::vector<int> root(n);
        for (int i = 0; i < n; ++i) root[i] = i;
        auto find = [&](int x) { while (root[x] != x) { root[x] = root[root[x]]; x = root[x]; } return x; };
        for (size_t c = 0; c < ncell; ++c)
            for (int k = cell_off[c] + 1; k < cell_off[c + 1]; ++k) {
                const int a = find(cell_box[cell_off[c]]), b = find(cell_box[k]);
                if (a != b) root[std::max(a, b)] = std::min(a, b);
            }
        std::vector<int> comp_of(n, -1), comp_off, members, comp_size;
        int ncomp = 0;
        for (int i = 0; i < n; ++i) {
            const int r = find(i);
            if (comp_of[r] < 0) { comp_of[r] = ncomp++; comp_size.push_back(0); }
            comp_of[i] = comp_of[r];
            comp_size[comp_of[i]]++;
        }
        comp_off.assign(ncomp + 1, 0);
        for (int c = 0; c < ncomp; ++c) comp_off[c + 1] = comp_off[c] + comp_size[c];
        members.resize(n);
        {
            std::vector<int> fill(comp_off.begin(), comp_off.end() - 1);
            for (int i = 0; i < n; ++i) members[fill[comp_of[i]]++] = i;   // ascending within a component
        }
        // a box's position inside its component (members ascending): the components keep their deletion flags in
        // private arrays while they run and write them back at the end, so workers never share a written cache line
        std::vector<int> local(n);
        for (int c = 0; c < ncomp; ++c)
            for (int k = comp_off[c]; k < comp_off[c + 1]; ++k) local[members[k]] = k - comp_off[c];
        q2 = clk::now();
        auto run_comp = [&](int c, std::vector<int>& nb, std::vector<char>& del) {
            const int m0 = comp_off[c], m1 = comp_off[c + 1];
            del.assign(m1 - m0, 0);
            for (int k = m0; k < m1; ++k) {
                const int i = members[k];
                if (del[k - m0]) continue;
                nb.clear();
                for (int cy = span[i].y; cy <= span[i].w; ++cy)
                    for (int cx = span[i].x; cx <= span[i].z; ++cx) {
                        const size_t c = (size_t)cy * gnx + cx;
                        for (int k = cell_off[c]; k < cell_off[c + 1]; ++k)
                            if (cell_box[k] > i) nb.push_back(cell_box[k]);
                    }
                std::sort(nb.begin(), nb.end());
                nb.erase(std::unique(nb.begin(), nb.end()), nb.end());
                for (int j : nb)
                    if (!del[local[j]] && overlap(i, j)) {
                        const int d = pair_del(i, j);
                        if (d >= 0) del[local[d]] = 1;
                    }
            }
            for (int k = m0; k < m1; ++k)
                if (del[k - m0]) v[members[k]].del = true;
        };
        // workers only where there is exact-test work to spread (clusters of duplicate detections)
        if (ncomp < 8 || n - ncomp < 64) {
            std::vector<int> nb;
            std::vector<char> del;
            for (int c = 0; c < ncomp; ++c) run_comp(c, nb, del);
        } else {
            host_parallel(ncomp, [&](int c) {
                thread_local std::vector<int> nb;
                thread_local std::vector<char> del;
                run_comp(c, nb, del);
            });
        }
        q3 = clk::now();
        if (tail_times)
            fprintf(stderr, "overlap n=%d comps=%d geom %.3f grid+comps %.3f tests %.3f ms\n", n, ncomp,
                    std::chrono::duration<double, std::milli>(q1 - q0).count(),
                    std::chrono::duration<double, std::milli>(q2 - q1).count(),
                    std::chrono::duration<double, std::milli>(q3 - q2).count());
    }
    v.erase(std::remove_if(v.begin(), v.end(), [](const HostMatch& m) { return m.del; }), v.end());
}

// (A^T A)^-1 by LU with partial pivoting (cv::invert, DECOMP_LU -> hal::LU64f), n x n, row-major.
static bool invert_lu(std::vector<double> a, int n, std::vector<double>& inv) {
    inv.assign((size_t)n * n, 0.0);
    for (int i = 0; i < n; ++i) inv[(size_t)i * n + i] = 1.0;
    for (int i = 0; i < n; ++i) {
        int piv = i;
        for (int r = i + 1; r < n; ++r)
            if (std::fabs(a[(size_t)r * n + i]) > std::fabs(a[(size_t)piv * n + i])) piv = r;
        if (std::fabs(a[(size_t)piv * n + i]) < DBL_EPSILON * 100) return false;
        if (piv != i) {
            for (int c = i; c < n; ++c) std::swap(a[(size_t)i * n + c], a[(size_t)piv * n + c]);
            for (int c = 0; c < n; ++c) std::swap(inv[(size_t)i * n + c], inv[(size_t)piv * n + c]);
        }
        const double d = -1 / a[(size_t)i * n + i];
        for (int r = i + 1; r < n; ++r) {
            const double alpha = a[(size_t)r * n + i] * d;
            for (int c = i + 1; c < n; ++c) a[(size_t)r * n + c] += alpha * a[(size_t)i * n + c];
            for (int c = 0; c < n; ++c) inv[(size_t)r * n + c] += alpha * inv[(size_t)i * n + c];
        }
    }
    for (int i = n - 1; i >= 0; --i)
        for (int c = 0; c < n; ++c) {
            double s = inv[(size_t)i * n + c];
            for (int k = i + 1; k < n; ++k) s -= a[(size_t)i * n + k] * inv[(size_t)k * n + c];
            inv[(size_t)i * n + c] = s / a[(size_t)i * n + i];
        }
    return true;
}

void subpix_estimation(const HostMatch* v, double* dx, double* dy, double* dangle, double angle_step,
                       int imax) {
    double A[27][10], S[27];
    const double x0 = v[imax].ptx, y0 = v[imax].pty, t0 = v[imax].angle;
    int row = 0;
    for (int th = 0; th <= 2; ++th)
        for (int y = -1; y <= 1; ++y)
            for (int x = -1; x <= 1; ++x, ++row) {
                const double X = x0 + x, Y = y0 + y, T = (t0 + (th - 1) * angle_step) * kD2R;
                const double r[10] = {X * X, Y * Y, T * T, X * Y, X * T, Y * T, X, Y, T, 1.0};
                for (int k = 0; k < 10; ++k) A[row][k] = r[k];
                S[row] = v[imax + (th - 1)].vec[x + 1][y + 1];
            }
    std::vector<double> ata(100), inv;
    for (int i = 0; i < 10; ++i)
        for (int j = 0; j < 10; ++j) {
            double s = 0;
            for (int r = 0; r < 27; ++r) s += A[r][i] * A[r][j];
            ata[(size_t)i * 10 + j] = s;
        }
    if (!invert_lu(ata, 10, inv)) inv.assign(100, 0.0);
    double Z[10];
    std::vector<double> ia(10 * 27);
    for (int i = 0; i < 10; ++i)
        for (int r = 0; r < 27; ++r) {
            double s = 0;
            for (int k = 0; k < 10; ++k) s += inv[(size_t)i * 10 + k] * A[r][k];
            ia[(size_t)i * 27 + r] = s;
        }
    for (int i = 0; i < 10; ++i) {
        double s = 0;
        for (int r = 0; r < 27; ++r) s += ia[(size_t)i * 27 + r] * S[r];
        Z[i] = s;
    }
    const double K[3][3] = {{2 * Z[0], Z[3], Z[4]}, {Z[3], 2 * Z[1], Z[5]}, {Z[4], Z[5], 2 * Z[2]}};
    const double rhs[3] = {-Z[6], -Z[7], -Z[8]};
    // closed-form 3x3 inverse (cv::invert for n == 3)
    double det = K[0][0] * (K[1][1] * K[2][2] - K[1][2] * K[2][1]) - K[0][1] * (K[1][0] * K[2][2] - K[1][2] * K[2][0]) +
                 K[0][2] * (K[1][0] * K[2][1] - K[1][1] * K[2][0]);
    double t[9] = {0};
    if (det != 0.) {
        det = 1. / det;
        t[0] = (K[1][1] * K[2][2] - K[1][2] * K[2][1]) * det;
        t[1] = (K[0][2] * K[2][1] - K[0][1] * K[2][2]) * det;
        t[2] = (K[0][1] * K[1][2] - K[0][2] * K[1][1]) * det;
        t[3] = (K[1][2] * K[2][0] - K[1][0] * K[2][2]) * det;
        t[4] = (K[0][0] * K[2][2] - K[0][2] * K[2][0]) * det;
        t[5] = (K[0][2] * K[1][0] - K[0][0] * K[1][2]) * det;
        t[6] = (K[1][0] * K[2][1] - K[1][1] * K[2][0]) * det;
        t[7] = (K[0][1] * K[2][0] - K[0][0] * K[2][1]) * det;
        t[8] = (K[0][0] * K[1][1] - K[0][1] * K[1][0]) * det;
    }
    *dx = t[0] * rhs[0] + t[1] * rhs[1] + t[2] * rhs[2];
    *dy = t[3] * rhs[0] + t[4] * rhs[1] + t[5] * rhs[2];
    *dangle = (t[6] * rhs[0] + t[7] * rhs[1] + t[8] * rhs[2]) * kR2D;
}

}  // namespace fpm
