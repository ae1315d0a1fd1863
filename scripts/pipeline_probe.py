"""Host-side pipeline probe: time fpm_match_staged_launch (graph launch) and fpm_match_staged_finish (wait +
post-processing) separately while sweeping contexts x batch, to see whether the pipelined bench is device- or
host-bound.  usage: python scripts/pipeline_probe.py [steps]"""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
from fastest_image_pattern_matching_amd import TemplateMatcher, synth  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
templ = synth.load_templates()["Dst7"]
src_all = bench.make_sources(templ, 32, 7)


def mk(srcs):
    c = TemplateMatcher(0)
    for k, v in bench.PARAMS.items():
        setattr(c._params, k, v)
    assert c.learnPattern(templ)
    c.stage(srcs)
    c.match_staged_array()
    return c


for batch in (8, 16, 32):
    for G in (1, 2, 3, 4):
        if G > batch:
            continue
        chunks = [src_all[i * batch // G:(i + 1) * batch // G] for i in range(G)]
        ctxs = [mk(ch) for ch in chunks]
        tl, tf = [], []

        def run(k):
            for c in ctxs:
                c.match_staged_launch()
            for i in range(k):
                for c in ctxs:
                    t0 = time.perf_counter()
                    c.match_staged_finish_array()
                    t1 = time.perf_counter()
                    tf.append(t1 - t0)
                    if i + 1 < k:
                        c.match_staged_launch()
                        tl.append(time.perf_counter() - t1)

        run(10)
        tl.clear(), tf.clear()
        t0 = time.perf_counter()
        run(steps)
        el = time.perf_counter() - t0
        dev = [c.profile_last() for c in ctxs]
        print(f"batch {batch:2d} ctx {G}: {batch * steps / el:9.1f} searches/s  step {el / steps * 1e3:.3f} ms  "
              f"launch {np.median(tl) * 1e6:6.1f} us  finish(wait+post) {np.median(tf) * 1e6:6.1f} us  "
              f"last dev/host/call ms {[tuple(round(x, 3) for x in d) for d in dev]}", flush=True)
        del ctxs
