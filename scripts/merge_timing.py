"""Host-tail timing (profiling aid, not a test): the C ABI's fpm_merge_candidates over the Src10 +-180 records
(tests/golden/merge_src10_180.npz, 4935 top-layer candidates -> 144 matches), median of repeated calls.

    FPM_HOST_THREADS=8 python scripts/merge_timing.py [reps]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fastest_image_pattern_matching_amd import _lib as L  # noqa: E402
from fastest_image_pattern_matching_amd.matcher import CANDIDATE_DTYPE, merge_candidates  # noqa: E402

z = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "merge_src10_180.npz"))
p = L.Params()
L.load().fpm_params_default(p)
p.max_pos, p.score, p.tolerance_angle, p.max_overlap = int(z["params"][0]), *map(float, z["params"][1:])
rec = z["records"].view(CANDIDATE_DTYPE)
tw, th = int(z["tmpl_wh"][0]), int(z["tmpl_wh"][1])
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
import ctypes as C  # noqa: E402

lib = L.load()
c = np.ascontiguousarray(rec, CANDIDATE_DTYPE)
buf = (L.Result * len(c))()
cnt = C.c_int32()
cp = c.ctypes.data_as(C.POINTER(L.Candidate))
ts = []
for _ in range(reps):   # the C call alone (the Python wrapper's result conversion excluded)
    t0 = time.perf_counter()
    lib.fpm_merge_candidates(C.byref(p), tw, th, cp, len(c), buf, len(c), C.byref(cnt))
    ts.append(time.perf_counter() - t0)
out = merge_candidates(p, tw, th, rec)
res = np.array([r.as_tuple() for r in out])
same = res.shape == z["results"].shape and np.array_equal(res, z["results"])
ts = np.array(ts[reps // 10:]) * 1e3
print(f"n={len(rec)} -> {len(out)} matches, identical={same}, merge ms: median {np.median(ts):.3f} "
      f"p10 {np.percentile(ts, 10):.3f} p90 {np.percentile(ts, 90):.3f} (threads={os.environ.get('FPM_HOST_THREADS', 'default')})")
