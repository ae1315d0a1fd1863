"""Candidate records of one tests/test_gpu_fuzz.py case on the GPU (current env forms) vs the oracle (debug helper).
usage: python scripts/debug_fuzz_case.py SEED"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from fastest_image_pattern_matching_amd import TemplateMatcher  # noqa: E402
from fastest_image_pattern_matching_amd import _lib as L  # noqa: E402
from tests import oracle  # noqa: E402
from tests.test_gpu_fuzz import _case  # noqa: E402

seed = int(sys.argv[1])
s, t, prm = _case(seed)
print("src", s.shape, "tmpl", t.shape, prm)
o = oracle.OracleMatcher().set(**prm)
o.learnPattern(t)
orc = o.match(s)
oc = o.candidates()
m = TemplateMatcher(0)
for k, v in prm.items():
    setattr(m._params, k, v)
m.learnPattern(t)
m.profile(True)
m.profile_reset()
g = m.match(s)
gc = m.last_candidates(0)
print("launches", {n: m.profile_get(k)[1] for k, n in enumerate(L.KERNEL_NAMES) if m.profile_get(k)[1]})
print("stats gpu", m.search_stats(), "orc", o.stats())
for i in range(max(len(gc), len(oc))):
    a = gc[i].tolist() if i < len(gc) else None
    b = oc[i].tolist() if i < len(oc) else None
    print("same" if a == b else "DIFF", a, b)
print("results equal", [r.as_tuple() for r in g] == orc)
