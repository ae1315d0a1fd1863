// Single-search latency through the C ABI (what the drop-in does per match() call): host array -> results, with the
// library's own split (fpm_profile_last: device pass, host tail, launch-to-finish).  Profiling aid, not a test.
// build: g++ -O2 -std=c++17 scripts/latency_probe.cpp -Iinclude -Lfastest_image_pattern_matching_amd/lib -lfpm_hip
//        -Wl,-rpath,$PWD/fastest_image_pattern_matching_amd/lib -o build/latency_probe
// usage: latency_probe tmpl.raw tw th src.raw sw sh [reps]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "fpm.h"

static std::vector<uint8_t> rd(const char* p, size_t n) {
    std::vector<uint8_t> v(n);
    FILE* f = std::fopen(p, "rb");
    if (!f || std::fread(v.data(), 1, n, f) != n) { std::fprintf(stderr, "read %s\n", p); std::exit(2); }
    std::fclose(f);
    return v;
}

int main(int argc, char** argv) {
    if (argc < 7) return 2;
    const int tw = std::atoi(argv[2]), th = std::atoi(argv[3]), sw = std::atoi(argv[5]), sh = std::atoi(argv[6]);
    const int reps = argc > 7 ? std::atoi(argv[7]) : 50;
    auto t = rd(argv[1], (size_t)tw * th);
    auto s = rd(argv[4], (size_t)sw * sh);
    fpm_ctx* c = nullptr;
    if (fpm_create(0, &c) != FPM_OK) { std::puts("no device"); return 1; }
    fpm_params p;
    fpm_params_default(&p);
    p.max_pos = 3; p.tolerance_angle = 180; p.score = 0.7;
    fpm_set_params(c, &p);
    fpm_learn(c, t.data(), tw, th, tw);
    std::vector<fpm_result> out(64);
    int32_t n = 0;
    double sec = 0;
    std::vector<double> tot, dev, host, call;
    for (int i = 0; i < reps + 5; ++i) {
        const auto a = std::chrono::steady_clock::now();
        fpm_match(c, s.data(), sw, sh, sw, out.data(), 64, &n, &sec);
        const auto b = std::chrono::steady_clock::now();
        double d, h, cl;
        fpm_profile_last(c, &d, &h, &cl);
        if (i >= 5) {
            tot.push_back(std::chrono::duration<double, std::milli>(b - a).count());
            dev.push_back(d); host.push_back(h); call.push_back(cl);
        }
    }
    auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    std::printf("{\"single_search_ms\": %.4f, \"device_ms\": %.4f, \"host_tail_ms\": %.4f, \"launch_to_finish_ms\": %.4f, "
                "\"upload_and_rest_ms\": %.4f, \"results\": %d, \"getLastExecutionTime_ms\": %.4f}\n",
                med(tot), med(dev), med(host), med(call), med(tot) - med(call), n, sec * 1e3);
    fpm_destroy(c);
    return 0;
}
