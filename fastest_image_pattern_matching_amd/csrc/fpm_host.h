// fpm_host.h — host-side stages of the search that are not data-parallel.
#pragma once
#include <functional>
#include <vector>

#include "fpm_geom.h"

namespace fpm {

// cv::RotatedRect (center, size, angle in degrees)
struct RRect {
    F2 c;
    float w, h, angle;
};

// s_MatchParameter subset carried through the host stages (DataStructures.h:58-94)
struct HostMatch {
    double ptx, pty;
    double score, angle;
    RRect rect;
    bool del;
    bool on_border;
    double vec[3][3];
    int32_t id;   // caller's index (fpm_op_overlap_filter)
};

RRect rrect_from3(F2 p1, F2 p2, F2 p3);                              // cv::RotatedRect(p1, p2, p3)
void rrect_corners(const RRect& r, F2 pt[4]);                        // cv::RotatedRect::points
bool rrect_pair_drops(const RRect& a, const RRect& b, double max_overlap);   // one pair of filterWithRotatedRect
int rrect_intersection(const RRect& a, const RRect& b, std::vector<F2>& pts);  // rotatedRectangleIntersection
void sort_pt_with_center(std::vector<F2>& pts);                      // TemplateMatcher.cpp:1093-1131
void sort_pt_with_center_keyed(std::vector<F2>& pts);                // the same with explicit acos keys (checks)
double contour_area(const std::vector<F2>& pts);                     // cv::contourArea
void filter_with_score(std::vector<HostMatch>& v, double score);     // TemplateMatcher.cpp:984-1000
void filter_with_rotated_rect(std::vector<HostMatch>& v, double max_overlap);  // :1133-1194
void subpix_estimation(const HostMatch* v, double* dx, double* dy, double* dangle,
                       double angle_step, int imax);                 // :1002-1072
bool score_big2small(const HostMatch& a, const HostMatch& b);        // compareScoreBig2Small (:14-17)
// runs fn(0 .. ntasks-1) on the host worker pool (FPM_HOST_THREADS, default min(hardware threads, 8)), caller included
void host_parallel(int ntasks, const std::function<void(int)>& fn);
int host_thread_count();   // threads host_parallel uses: FPM_HOST_THREADS, else the hardware concurrency capped at 8
// wake the pool's workers now and keep them spinning for `us` microseconds, so that a host tail expected after a device
// wait starts without the wake-up latency of sleeping threads
void host_pool_warm(int us);

}  // namespace fpm
