"""Print GPU vs oracle results/stats for one golden case (debug helper)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from tests.test_oracle_golden import apply_params, golden
from tests import oracle
from fastest_image_pattern_matching_amd import TemplateMatcher
name = sys.argv[1]
z = golden()
m = TemplateMatcher(0)
apply_params(m._params, z[f"{name}__params"])
m.learnPattern(z[f"{name}__tmpl"])
g = [r.as_tuple() for r in m.match(z[f"{name}__src"])]
print("gpu stats", m.search_stats()); print("orc stats", z[f"{name}__stats"].tolist())
for r in g: print("gpu", [round(v, 4) for v in r[8:]])
for r in z[f"{name}__results"]: print("orc", [round(v, 4) for v in r[8:]])
