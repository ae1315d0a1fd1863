"""Timing of the BASELINE configs other than the headline one (bench.py measures configs[1], Src7, batched):
per config the device-resident ms per search on one GPU (sources staged in HBM, median over repeated passes of
the staged batch; latency view: one context, pass after pass), the pipelined ms per search (two contexts as a
stream of passes, host tail overlapped: throughput view) next to one oracle search on the host (the CPU
restatement, one thread), plus the result count of each.  Writes one JSON line per config.

The reference's own shipped inputs with a published time (README.md:65, 68-70; --ref-only runs just these): Test6
(Src6/Dst6), Test4 (Src3/Dst3), Test5 (Src4/Dst4) and Test1 (Src9/Dst9) with the parameters of the screenshot pins
(tests/golden/reference_pins.json: the published ones where README states them, Test1 also at its published Score
0.8), MFC semantics (the README times are the MFC tool's), next to the README figure; for these the single-search
end-to-end time of TemplateMatcher.match on the host array (upload included: the drop-in's use) is reported too,
and the result count is asserted equal to the pin's.
usage: python scripts/bench_configs.py [reps] [--no-cpu] [--only=K ...] [--with-64] [--ref-only]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fastest_image_pattern_matching_amd import TemplateMatcher, synth  # noqa: E402
from tests import oracle  # noqa: E402  (timed CPU baseline only)

REPS = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 10
CPU = "--no-cpu" not in sys.argv
ONLY = [int(a.split("=")[1]) for a in sys.argv if a.startswith("--only=")]   # config positions to run
ALL64 = "--with-64" in sys.argv
PIPE = "--no-pipe" not in sys.argv   # --no-pipe: latency view only (one context: clean kernel traces)   # also the whole 64-source configs[3] at 1 deg on one GPU (~1 GB of sources)


REF_ONLY = "--ref-only" in sys.argv
# README.md:65, 68-70 (i7-10700): (test, pin name, README ms with SIMD where stated, README ms without)
README_TESTS = [("Test6", "test6_src6", 657.0, 1157.0), ("Test4", "test4_src3", 21.0, None),
                ("Test5", "test5_src4", 27.0, None), ("Test1", "test1_src9", 80.0, 164.0)]


def reference_inputs():
    from fastest_image_pattern_matching_amd.images import imread_gray

    golden = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")
    pins = {p["name"]: p for p in json.load(open(os.path.join(golden, "reference_pins.json")))}

    def img(name):
        path = os.path.join(golden, "ref", name)
        return imread_gray(path if os.path.exists(path) else os.path.join(golden, name))

    for test, name, simd_ms, plain_ms in README_TESTS:
        pin = pins[name]
        s, t = img(pin["source"]), img(pin["template"])
        runs = [("pin", pin["params"], pin["count"])]
        if pin.get("count_at_published") is not None:
            runs.append(("published", pin["published"], pin["count_at_published"]))
        for tag, prm, count in runs:
            label = (f"README {test}: {pin['source']} {s.shape[1]}x{s.shape[0]} / {pin['template']} "
                     f"{t.shape[1]}x{t.shape[0]}, {tag} parameters {prm}")
            yield (label, [s], t, dict(prm, semantics=1),
                   {"readme_ms_simd": simd_ms, "readme_ms_no_simd": plain_ms, "expect_matches": count,
                    "fitted": pin["fitted"] if tag == "pin" else []})


def configs():
    if REF_ONLY:
        return
    T = synth.load_templates()
    s10, t10 = synth.src10_scene(T["Dst10"])
    yield ("configs[2] Src10 3648x3648 / Dst10 54x54, Tol 0, TargetNum 100 (s_BlockMax)", [s10], t10,
           dict(max_pos=100, score=0.7, tolerance_angle=0.0))
    yield ("configs[2] stress: Src10 3648x3648, +-180 deg, TargetNum 100", [s10], t10,
           dict(max_pos=100, score=0.7, tolerance_angle=180.0))
    srcs, t = synth.batch_sources(8)
    yield ("configs[3] 8 x 4096x4096 / 512x512 crop, +-180 deg (reference step), TargetNum 1", srcs, t,
           dict(max_pos=1, tolerance_angle=180.0))
    # BASELINE configs[3] as stated: +-180 at a 1 deg top-layer step (fpm_params.top_angle_step, a flagged extension;
    # the reference derives 7.125 deg, TemplateMatcher.cpp:130): 8 sources = one GPU's share of the 64-source,
    # 8-GPU config; then all 64 on one GPU
    yield ("configs[3] 8 x 4096x4096 / 512x512 crop, +-180 deg at 1 deg top step (361 angles), TargetNum 1", srcs, t,
           dict(max_pos=1, tolerance_angle=180.0, top_angle_step=1.0))
    if ALL64:
        srcs64, t = synth.batch_sources(64)
        yield ("configs[3] 64 x 4096x4096 / 512x512 crop, +-180 deg at 1 deg top step, TargetNum 1, one GPU", srcs64,
               t, dict(max_pos=1, tolerance_angle=180.0, top_angle_step=1.0))
        del srcs64
    srcs5, t5 = synth.src5_set(T["Dst5"])
    yield ("configs[4] Src5 rotation set 8 x 640x480 / Dst5 160x159, +-180 deg, sub-pixel", srcs5, t5,
           dict(max_pos=1, tolerance_angle=180.0, subpixel=1))
    s7, t7 = synth.src7_scene(T["Dst7"])
    yield ("configs[1] single Src7 source (latency view of the headline config)", [s7], t7,
           dict(max_pos=3, tolerance_angle=180.0, score=0.7, min_reduce_area=256, max_overlap=0.0, use_simd=1))


def pipelined(m, srcs, t, prm):
    """Throughput view: a second context (HIP stream) holding the same batch; the two run as a stream of passes
    (bench.py's scheme), so one context's host tail overlaps the other's device work."""
    m2 = TemplateMatcher(0)
    for k, v in prm.items():
        setattr(m2._params, k, v)
    assert m2.learnPattern(t)
    m2.stage(srcs)
    m2.match_staged_array()
    ctxs = [m, m2]
    for c in ctxs:
        c.match_staged_launch()
    t0 = time.perf_counter()
    for k in range(REPS):
        for c in ctxs:
            c.match_staged_finish_array()
            if k + 1 < REPS:
                c.match_staged_launch()
    pipe_ms = (time.perf_counter() - t0) * 1e3 / (REPS * len(ctxs))
    return {"pipelined_ms_per_search": round(pipe_ms / len(srcs), 3),
            "pipelined_searches_per_s": round(1e3 * len(srcs) / pipe_ms, 1)}


def end_to_end_ms(m, src):
    """TemplateMatcher.match on the host array (upload + device pass + host tail): median of REPS calls."""
    m.match(src)
    ts = []
    for _ in range(REPS):
        t0 = time.perf_counter()
        m.match(src)
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e3


def main():
    items = [(n, s_, t_, p_, None) for n, s_, t_, p_ in configs()] + list(reference_inputs())
    for pos, (name, srcs, t, prm, ref) in enumerate(items):
        if ONLY and pos not in ONLY:
            continue
        m = TemplateMatcher(0)
        for k, v in prm.items():
            setattr(m._params, k, v)
        assert m.learnPattern(t)
        m.stage(srcs)
        cnt, _ = m.match_staged_array()          # warm: plan + graph
        cnt = cnt.copy()
        ts = []
        for _ in range(REPS):
            t0 = time.perf_counter()
            m.match_staged_array()
            ts.append(time.perf_counter() - t0)
        ms = float(np.median(ts)) * 1e3
        dev_ms, host_ms, _ = m.profile_last()   # the last pass: device span and host post-processing
        out = {"config": name, "sources": len(srcs), "gpu_ms_per_pass": round(ms, 3),
               "last_pass_device_ms": round(dev_ms, 3), "last_pass_host_ms": round(host_ms, 3),
               "gpu_ms_per_search": round(ms / len(srcs), 3), "gpu_searches_per_s": round(1e3 * len(srcs) / ms, 1),
               "matches": [int(x) for x in cnt]}
        if ref is not None:
            out.update(ref)
            assert out["matches"] == [ref["expect_matches"]], (name, out["matches"])
            out["readme_over_gpu_latency"] = round(ref["readme_ms_simd"] / out["gpu_ms_per_search"], 1)
        if PIPE:
            out.update(pipelined(m, srcs, t, prm))
        if ref is not None:   # after the staged passes: match() on a host array replaces the staged batch
            out["gpu_ms_end_to_end"] = round(end_to_end_ms(m, srcs[0]), 3)
        if CPU:
            o = oracle.OracleMatcher().set(**prm)
            o.learnPattern(t)
            t0 = time.perf_counter()
            r = o.match(srcs[0])
            cpu = time.perf_counter() - t0
            out.update({"cpu_oracle_ms_per_search": round(cpu * 1e3, 1), "cpu_matches_src0": len(r),
                        "gpu_vs_cpu": round(cpu * 1e3 / (ms / len(srcs)), 1)})
            assert len(r) == int(cnt[0]), (name, len(r), int(cnt[0]))
        print(json.dumps(out), flush=True)
        del m


if __name__ == "__main__":
    main()
