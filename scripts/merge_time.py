#!/usr/bin/env python3
"""Wall time of the coupled host tail (fpm_merge_candidates: both std::sort replays, filterWithScore, rotated
rectangles, filterWithRotatedRect, final sort, conversion) over the Src10 +-180 records (tests/golden/
merge_src10_180.npz, 4935 candidates -> 144 results), checked against the fixture's results.  The C ABI is called
directly with preallocated buffers; each timed call follows an untimed one (warm host pool, as in a search, where
the pool is woken when the device pass is launched and the tail starts after the device wait).
usage: FPM_HOST_THREADS=n python3 scripts/merge_time.py [iterations]"""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from fastest_image_pattern_matching_amd.matcher import CANDIDATE_DTYPE, SingleTargetMatch  # noqa: E402
from fastest_image_pattern_matching_amd import _lib as L  # noqa: E402

z = np.load(os.path.join(ROOT, "tests", "golden", "merge_src10_180.npz"))
lib = L.load()
p = L.Params()
lib.fpm_params_default(p)
p.max_pos, p.score, p.tolerance_angle, p.max_overlap = int(z["params"][0]), *map(float, z["params"][1:])
rec = np.ascontiguousarray(z["records"].view(CANDIDATE_DTYPE))
tw, th = int(z["tmpl_wh"][0]), int(z["tmpl_wh"][1])
cap = len(rec)
out = (L.Result * cap)()
n = C.c_int32()
args = (C.byref(p), tw, th, rec.ctypes.data_as(C.POINTER(L.Candidate)), len(rec), out, cap, C.byref(n))
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 200
ts = []
for _ in range(iters):
    assert lib.fpm_merge_candidates(*args) == L.FPM_OK
    t0 = time.perf_counter()
    rc = lib.fpm_merge_candidates(*args)
    ts.append((time.perf_counter() - t0) * 1e3)
    assert rc == L.FPM_OK
res = np.array([SingleTargetMatch.from_c(out[i]).as_tuple() for i in range(n.value)])
assert res.shape == z["results"].shape and np.array_equal(res, z["results"]), "results differ from the fixture"
ts.sort()
print(f"threads {os.environ.get('FPM_HOST_THREADS', 'default')}: merge median {ts[len(ts) // 2]:.3f} ms, "
      f"min {ts[0]:.3f} ms over {iters} calls ({len(rec)} candidates -> {len(res)} results, equal to the fixture)")
