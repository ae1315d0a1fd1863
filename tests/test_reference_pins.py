"""The reference's own published results as pins (tests/golden/reference_pins.json, made by
tests/golden/make_reference_pins.py from README.md:62-71 and "Result Images/"): the shipped source/template pairs,
decoded with IMREAD_GRAYSCALE semantics by images.py, searched with the published parameters.

Each pin asserts the number of detections the screenshot labels and that every centre cross read from the screenshot
has a searched centre under it: a per-axis scale + offset is fitted between the crosses and their nearest centres
(the screenshots are scaled, Result3 also slightly cropped; scale within 3 % of nominal, offset within 8 display px)
and the largest residual must stay below 1.5 display px (the tool draws its crosses at integer display positions,
then JPEG).  The oracle is checked on CPU; the HIP path on the GPU, bit-identical to the oracle.

Semantics: the screenshots come from the MFC tool (README.md:45), so the pins run with FPM_SEMANTICS_MFC; the Qt
class finds the same detection set (also asserted).  Unpinned by these: scores and angles (not legible), the label
order (the screenshots predate the score-sorted listing: Result4's labels run by x).
"""
import json
import os

import numpy as np
import pytest

from fastest_image_pattern_matching_amd.images import imread_gray
from tests import oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
with open(os.path.join(GOLDEN, "reference_pins.json")) as _fh:
    PINS = {p["name"]: p for p in json.load(_fh)}


def _image(name):
    path = os.path.join(GOLDEN, "ref", name)
    if not os.path.exists(path):
        path = os.path.join(GOLDEN, name)
    return imread_gray(path)


def _load(pin):
    return _image(pin["source"]), _image(pin["template"])


def cross_residual(pin, shape, results):
    """Largest residual (display px) of the fitted scale + offset between the screenshot's crosses and the nearest
    result centres; the centres' nominal display positions choose the nearest one."""
    h, w = shape
    dw, dh = pin["display"]
    sx, sy = dw / w, dh / h
    cen = np.array([[r[8], r[9]] for r in results], np.float64)
    crs = np.array(pin["crosses"], np.float64)
    near = [int(np.argmin(((cen[:, 0] * sx - c[0]) ** 2 + (cen[:, 1] * sy - c[1]) ** 2))) for c in crs]
    assert len(set(near)) == len(near), "two crosses on one detection"
    worst = 0.0
    for ax, nominal in ((0, sx), (1, sy)):
        a, b = np.polyfit(cen[near, ax], crs[:, ax], 1)
        # the view's scale within 3 % of width / display width, its crop offset within 8 display px
        assert abs(a / nominal - 1) < 0.03 and abs(b) < 8, (ax, a / nominal, b)
        worst = max(worst, float(np.max(np.abs(a * cen[near, ax] + b - crs[:, ax]))))
    return worst


def _search(s, t, **prm):
    o = oracle.OracleMatcher().set(**prm)
    assert o.learnPattern(t)
    return o.match(s)


@pytest.mark.parametrize("name", sorted(PINS))
def test_oracle_reproduces_reference_screenshot(name):
    pin = PINS[name]
    s, t = _load(pin)
    res = _search(s, t, semantics=1, **pin["params"])
    assert len(res) == pin["count"]
    assert cross_residual(pin, s.shape, res) < 1.5
    qt = _search(s, t, **pin["params"])
    # the same detections (centres: f32 in the Qt class, f64 in the MFC tool)
    key = lambda r: (round(r[8], 2), round(r[9], 2))  # noqa: E731
    assert sorted(map(key, qt[:pin["count"]])) == sorted(map(key, res))


@pytest.mark.gpu
@pytest.mark.parametrize("semantics", [0, 1])
@pytest.mark.parametrize("name", sorted(PINS))
def test_gpu_reproduces_reference_screenshot(gpu_matcher_factory, name, semantics):
    pin = PINS[name]
    s, t = _load(pin)
    m = gpu_matcher_factory(semantics=semantics, **pin["params"])
    assert m.learnPattern(t)
    got = [r.as_tuple() for r in m.match(s)]
    exp = _search(s, t, semantics=semantics, **pin["params"])
    assert got == exp
    if semantics == 1:
        assert len(got) == pin["count"]
        assert cross_residual(pin, s.shape, got) < 1.5
