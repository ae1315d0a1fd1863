// Host pool scaling on this machine: a compute-bound region (sum of sqrt over n elements, ~0.2 ms on one thread) run
// through host_parallel in 64 tasks, after the pool was warmed; wall time per region at the thread count given by
// FPM_HOST_THREADS.  Profiling aid.  build: hipcc -O3 -x hip --offload-arch=gfx950 scripts/pool_probe.cpp
//   fastest_image_pattern_matching_amd/csrc/fpm_host.cpp -o build/pool_probe -pthread
#include <chrono>
#include <cmath>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <sched.h>
#include <cstdlib>
#include <hip/hip_runtime.h>
#include "../fastest_image_pattern_matching_amd/csrc/fpm_host.h"
using namespace fpm;
static double now() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
static int cpus() { cpu_set_t m; CPU_ZERO(&m); sched_getaffinity(0, sizeof(m), &m); return CPU_COUNT(&m); }
int main() {
    std::printf("affinity before HIP: %d CPUs\n", cpus());
    if (std::getenv("POOL_PROBE_HIP")) {   // initialise the GPU runtime first, as a search process does
        (void)hipSetDevice(0);
        void* d = nullptr;
        (void)hipMalloc(&d, 1 << 20);
        (void)hipDeviceSynchronize();
        std::printf("affinity after HIP init: %d CPUs\n", cpus());
    }
    const int n = 1 << 16;
    std::vector<double> out(64);
    std::vector<double> ts;
    host_pool_warm(1000000);
    for (int it = 0; it < 200; ++it) {
        const double t0 = now();
        host_parallel(64, [&](int t) {
            double s = 0;
            for (int i = t * (n / 64); i < (t + 1) * (n / 64); ++i) s += std::sqrt((double)i * 1.000001 + s * 1e-9);
            out[t] = s;
        });
        ts.push_back(now() - t0);
    }
    double seq0 = now(), s = 0;
    for (int i = 0; i < n; ++i) s += std::sqrt((double)i * 1.000001 + s * 1e-9);
    const double seq = now() - seq0;
    std::sort(ts.begin(), ts.end());
    std::printf("threads %d: region median %.3f ms min %.3f ms; sequential %.3f ms (%g)\n", host_thread_count(), ts[ts.size() / 2], ts[0], seq, s + out[0]);
}
