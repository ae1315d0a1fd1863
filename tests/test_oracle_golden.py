"""The oracle still reproduces its committed golden vectors (tests/golden/golden.npz, make_golden.py)."""
import os

import numpy as np
import pytest

from tests import oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "golden.npz")
PARAM_KEYS = ("max_pos", "min_reduce_area", "max_overlap", "score", "tolerance_angle", "use_simd", "subpixel",
              "tolerance_range")


def golden():
    return np.load(GOLDEN)


def case_names():
    with np.load(GOLDEN) as z:
        return [str(c) for c in z["cases"]]


def apply_params(obj, vec):
    for k, v in zip(PARAM_KEYS, vec):
        cur = getattr(obj, k)
        setattr(obj, k, type(cur)(v) if not isinstance(cur, float) else float(v))


@pytest.mark.parametrize("name", case_names())
def test_oracle_golden_search(name):
    z = golden()
    o = oracle.OracleMatcher()
    apply_params(o.params, z[f"{name}__params"])
    assert o.learnPattern(z[f"{name}__tmpl"])
    res = np.array(o.match(z[f"{name}__src"]), np.float64).reshape(-1, 12)
    assert np.array_equal(res, z[f"{name}__results"])
    assert o.stats() == z[f"{name}__stats"].tolist()
    assert np.array_equal(o.top_candidates(), z[f"{name}__top"])


def test_oracle_golden_primitives():
    z = golden()
    assert np.array_equal(oracle.pyr_down(z["p_pyr__in"]), z["p_pyr__out"])
    assert np.array_equal(oracle.warp_affine(z["p_warp__in"], z["p_warp__m"], (41, 35), 77), z["p_warp__out"])
    o = oracle.OracleMatcher().set(min_reduce_area=4096)
    o.learnPattern(z["p_ncc__tmpl"])
    assert np.array_equal(o.ncc_map(z["p_ncc__in"], 0, True), z["p_ncc__fold"])
    assert np.array_equal(o.ncc_map(z["p_ncc__in"], 0, False), z["p_ncc__ccorr"])
