"""The reference's own published results as pins (tests/golden/reference_pins.json, made by
tests/golden/make_reference_pins.py from README.md:62-71 and "Result Images/"): the shipped source/template pairs,
decoded with IMREAD_GRAYSCALE semantics by images.py, searched with the published parameters.

Each pin asserts
* the number of detections the screenshot labels, and that every centre cross read from the screenshot has a
  searched centre under it: a per-axis scale + offset is fitted between the crosses and their nearest centres (the
  screenshots are scaled, Result3 also slightly cropped; scale within 3 % of nominal, offset within 8 display px) and
  the largest residual must stay below 1.5 display px;
* the index labels the tool drew (hand-transcribed into the JSON): for the score-sorted screenshots (Result6,
  Result8; MatchToolDlg.cpp:1071, 378-379) the oracle's result index of every box equals its label, i.e. the
  reference's score ranking; for the two screenshots of an older build that sorted by centre x (Result3, Result4;
  the call left commented out at MatchToolDlg.cpp:1118) the oracle's centre x is non-decreasing in label order.

Where the oracle departs from a screenshot the departure is pinned exactly (``EXPECTED_MISMATCH``) and explained:
* Result6, labels 8 <-> 9 (column 3, rows 2 and 3; oracle scores 0.92458 / 0.92487).  The order is decided at the
  top layer: box B's (label 9's) winning refinement path starts from a peak whose top-layer NCC is 8.4e-5 above the
  next peak at the same angle (the neighbouring box, one template height lower); getNextMaxLoc paints a 2w x 2h
  rectangle around the first peak (TemplateMatcher.cpp:1196-1206), so whichever of the two comes first suppresses
  the other's best pixel.  With the exact decode here B's peak comes first and its path ends at 0.92487; with the
  other order B starts one pixel off and ends at 0.92374, below box A's 0.92458 -- the screenshot's order.  +-1 LSB
  on 1 % of the decoded source pixels, the level at which JPEG decoders differ, gives the screenshot's full order in
  most perturbations (scripts/result6_sensitivity.py), and one such perturbation is pinned
  below.  The exact-decode full order is therefore an expected failure whose cause lies in the unpinned decoder
  (OpenCV's bundled libjpeg, MatchToolDlg.cpp:62), not in the oracle's semantics.
* Result3 (older build): 34 of the 35 adjacent label pairs are x-ordered; two are not, by one source pixel
  (labels 21/22 and 30/31).  Src3/Dst3 are lossless 8-bit BMPs, but the search is not integer end to end in the
  reference: its TM_CCORR is OpenCV's float32 DFT crossCorr at the top layer always (MatchToolDlg.cpp:858 -> :1304)
  and at every refinement layer when the tool's SIMD box is unchecked (:1277; unchecked by default, MatchTool.rc:118).
  The oracle's sensitivity mode restates that arithmetic (orc_set_ccorr_mode 1, oracle/fpm_oracle.cpp
  cross_corr_f32); ``test_ccorr_sensitivity`` runs all four pins in {exact, f32 DFT} x {SIMD on, off}: every mode
  gives the same detections and the same mismatch set, so float TM_CCORR explains neither Result3's two pairs nor
  Result6's 8/9 swap.  Result3's pairs stay unexplained by anything in the shipped code (recorded as a difference
  of that older build, which also drew different labels and sorted differently).

Result7 (Src8/Dst8, round 5) is the one screenshot whose detections depend on filterWithRotatedRect keeping an
overlapping pair (TemplateMatcher.cpp:1133-1194, MatchToolDlg.cpp:1071): its two right-hand boxes overlap, all three
labels are reproduced in score order, and ``test_result7_overlap_decides`` pins that the pair survives only when
MaxOverlap exceeds its overlap ratio (between 0.3 and 0.4 of the box area; label 2 is the one deleted below that).

Parameters: pins run ``params``; ``fitted`` names the ones chosen by running the oracle (not published).  README
Test1's published Score 0.8 gives one detection (``count_at_published``), the screenshot shows four: their oracle
scores are 0.999 / 0.764 / 0.764 / 0.703, so the screenshot cannot have been taken at 0.8 -- the pin runs 0.7.
The oracle is checked on CPU; the HIP path on the GPU, bit-identical to the oracle.
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

# labels the oracle does not reproduce (score order: labels whose box gets another index; x order: label k with
# x(k) > x(k+1)), each explained in the module docstring
EXPECTED_MISMATCH = {"test6_src6": [8, 9], "test4_src3": [21, 30], "test1_src9": [], "test5_src4": [],
                     "result7_src8": []}
# the pinned decoder-level perturbation of Src6 (scripts/result6_sensitivity.py): FITTED -- salt 2 at 1 % of the
# pixels is one of the 10 of 32 salts that give the screenshot's full order at that level (6/32 at 0.3 %, 20/32 at
# 3 %); the JSON records it as fitted together with those rates
_PERT = PINS["test6_src6"]["perturbation"]
RESULT6_SALT, RESULT6_FRAC = _PERT["salt"], _PERT["frac"]
# TM_CCORR sensitivity (scripts/ccorr_sensitivity.py): labels not reproduced per (ccorr mode, use_simd); float32
# DFT TM_CCORR changes none of them
CCORR_MODES = [(0, 1), (0, 0), (1, 1), (1, 0)]


def _image(name):
    path = os.path.join(GOLDEN, "ref", name)
    if not os.path.exists(path):
        path = os.path.join(GOLDEN, name)
    return imread_gray(path)


def _load(pin):
    return _image(pin["source"]), _image(pin["template"])


def perturb_lsb(img: np.ndarray, salt: int, frac: float) -> np.ndarray:
    """+-1 LSB on ~frac of the pixels, chosen (and signed) by a splitmix64-style hash of (pixel index + salt)."""
    idx = np.arange(img.size, dtype=np.uint64) + np.uint64(salt)
    h = idx * np.uint64(0x9E3779B97F4A7C15)
    h ^= h >> np.uint64(29)
    h *= np.uint64(0xBF58476D1CE4E5B9)
    h ^= h >> np.uint64(32)
    hit = (h & np.uint64(0xFFFFFFFF)) < np.uint64(int(frac * 2 ** 32))
    sign = np.where((h >> np.uint64(40)) & np.uint64(1), 1, -1)
    return np.clip(img.astype(np.int16).ravel() + hit * sign, 0, 255).astype(np.uint8).reshape(img.shape)


def _nearest(pin, shape, results):
    """label -> index of the result whose centre is nearest the label's box (nominal display scale)."""
    h, w = shape
    dw, dh = pin["display"]
    cen = np.array([[r[8] * dw / w, r[9] * dh / h] for r in results], np.float64)
    near = {lab: int(np.argmin(np.hypot(cen[:, 0] - x, cen[:, 1] - y))) for lab, x, y in pin["labels"]}
    assert len(set(near.values())) == len(near), "two labels on one detection"
    return near


def label_mismatches(pin, shape, results):
    near = _nearest(pin, shape, results)
    if pin["order"] == "score":
        return sorted(lab for lab, i in near.items() if i != lab)
    xs = [results[near[k]][8] for k in range(len(near))]
    return [k for k in range(len(xs) - 1) if xs[k] > xs[k + 1]]


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


def test_pin_parameters_are_labelled():
    for p in PINS.values():
        assert sorted(lab for lab, _, _ in p["labels"]) == list(range(p["count"]))
        if p["published"] is None:
            assert sorted(p["fitted"]) == sorted(p["params"])
        else:
            assert sorted(k for k in p["params"] if p["params"][k] != p["published"].get(k)) == sorted(p["fitted"])


@pytest.mark.parametrize("name", sorted(PINS))
def test_oracle_reproduces_reference_screenshot(name):
    pin = PINS[name]
    s, t = _load(pin)
    res = _search(s, t, semantics=1, **pin["params"])
    assert len(res) == pin["count"]
    assert cross_residual(pin, s.shape, res) < 1.5
    assert label_mismatches(pin, s.shape, res) == EXPECTED_MISMATCH[name]
    qt = _search(s, t, **pin["params"])
    # the same detections (centres: f32 in the Qt class, f64 in the MFC tool)
    key = lambda r: (round(r[8], 2), round(r[9], 2))  # noqa: E731
    assert sorted(map(key, qt[:pin["count"]])) == sorted(map(key, res))


def test_result7_overlap_decides():
    """Result7's overlapping pair (labels 1 and 2) is kept by filterWithRotatedRect at the pin's MaxOverlap and at
    0.4, and at 0.3 the lower-scored box (label 2) is deleted -- in both semantics; the rest of the list is unchanged."""
    pin = PINS["result7_src8"]
    s, t = _load(pin)
    for semantics in (0, 1):
        full = _search(s, t, semantics=semantics, **pin["params"])
        for ov, n in pin["overlap_count"].items():
            res = _search(s, t, semantics=semantics, **dict(pin["params"], max_overlap=float(ov)))
            assert len(res) == n
            if n == 2:
                near = _nearest(pin, s.shape, full)
                assert res == [full[near[0]], full[near[1]]]


def test_result6_perturbation_is_labelled_fitted():
    assert _PERT["fitted"] is True and _PERT["full_order_rate"]["0.01"] == "10/32"


@pytest.mark.parametrize("ccorr,simd", CCORR_MODES)
@pytest.mark.parametrize("name", sorted(PINS))
def test_ccorr_sensitivity(name, ccorr, simd, request):
    """The reference's float TM_CCORR (OpenCV crossCorr in float32 DFTs) as the cause of the residual mismatches:
    under every (TM_CCORR arithmetic, SIMD) combination the pins give the same count, residual bound and mismatch
    set as the exact parity mode -- the float path explains none of them -- and the same poses
    with scores within 1e-5 of it."""
    if (name, ccorr, simd) == ("test6_src6", 1, 0) and request.config.getoption("-m") == "not gpu and not slow":
        pytest.skip("34 s on one core: runs in the full CPU suite")
    pin = PINS[name]
    s, t = _load(pin)
    o = oracle.OracleMatcher().set(semantics=1, **dict(pin["params"], use_simd=simd)).set_ccorr_mode(ccorr)
    assert o.learnPattern(t)
    res = o.match(s)
    assert len(res) == pin["count"]
    assert cross_residual(pin, s.shape, res) < 1.5
    assert label_mismatches(pin, s.shape, res) == EXPECTED_MISMATCH[name]
    # against the parity mode: the same poses (centres, angles) and scores within north_star's 1e-5
    base = _search(s, t, semantics=1, **pin["params"])
    for r in res:
        b = min(base, key=lambda q: (q[8] - r[8]) ** 2 + (q[9] - r[9]) ** 2)
        assert (b[8], b[9], b[10]) == (r[8], r[9], r[10]) and abs(b[11] - r[11]) < 1e-5


def test_test1_at_published_score():
    """README Test1 (README.md:65) at its published Score 0.8: one detection, not the screenshot's four."""
    pin = PINS["test1_src9"]
    s, t = _load(pin)
    res = _search(s, t, semantics=1, **pin["published"])
    assert len(res) == pin["count_at_published"] == 1
    fitted = _search(s, t, semantics=1, **pin["params"])
    assert [round(r[11], 3) for r in fitted] == [0.999, 0.764, 0.764, 0.703]


@pytest.mark.xfail(strict=True, reason="Result6 labels 8/9: decided by an 8.4e-5 top-layer tie that the unpinned "
                                       "JPEG decode settles (see module docstring, test_result6_swap_cause)")
def test_result6_full_order_exact_decode():
    pin = PINS["test6_src6"]
    s, t = _load(pin)
    assert label_mismatches(pin, s.shape, _search(s, t, semantics=1, **pin["params"])) == []


def test_result6_swap_cause():
    pin = PINS["test6_src6"]
    s, t = _load(pin)
    o = oracle.OracleMatcher().set(semantics=1, **pin["params"])
    assert o.learnPattern(t)
    res = o.match(s)
    # box of label 9 (column 3, row 3) is result 8 here; its record is the kept candidate with that pose
    near = _nearest(pin, s.shape, res)
    assert (near[8], near[9]) == (9, 8)
    cand = o.candidates()
    rb = res[near[9]]
    (k,) = [i for i, c in enumerate(cand) if c["kept"] and c["score"] == rb[11]]
    same = [c for c in cand if c["angle_index"] == cand[k]["angle_index"]]
    nxt = [c for c in same if c["peak_rank"] == cand[k]["peak_rank"] + 1][0]
    gap = cand[k]["top_score"] - nxt["top_score"]
    assert 0 < gap < 1e-4                      # the top-layer tie (8.4e-5)
    assert res[near[8]][11] - rb[11] < 0 and rb[11] - res[near[8]][11] < 3e-4
    # decoder-level perturbation: the screenshot's full order
    sp = perturb_lsb(s, RESULT6_SALT, RESULT6_FRAC)
    assert np.count_nonzero(sp != s) / s.size < 0.011
    rp = o.match(sp)
    assert len(rp) == pin["count"] and label_mismatches(pin, s.shape, rp) == []


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
        assert label_mismatches(pin, s.shape, got) == EXPECTED_MISMATCH[name]


@pytest.mark.gpu
def test_gpu_result6_perturbed_order(gpu_matcher_factory):
    """The HIP path on the pinned decoder-level perturbation of Src6: bit-identical to the oracle and all 15 labels
    of the screenshot in order."""
    pin = PINS["test6_src6"]
    s, t = _load(pin)
    sp = perturb_lsb(s, RESULT6_SALT, RESULT6_FRAC)
    m = gpu_matcher_factory(semantics=1, **pin["params"])
    assert m.learnPattern(t)
    got = [r.as_tuple() for r in m.match(sp)]
    assert got == _search(sp, t, semantics=1, **pin["params"])
    assert label_mismatches(pin, s.shape, got) == []
