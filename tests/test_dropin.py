"""The C++ drop-in for src/TemplateMatcher.cpp (fastest_image_pattern_matching_amd/dropin/TemplateMatcher_fpm.cpp).

CPU: every public member function the reference header declares (include/TemplateMatcher.h:9-51, read from
/root/reference when present) is declared by the test fixture header and defined by the drop-in, and the test driver
builds against libfpm_hip.so.  GPU: full searches through the C++ class, as MatchToolDialog calls it
(src/MatchToolDialog.cpp:265-286, 358, 1344), bit-identical to the oracle, plus the class behaviour checks the
driver prints (copies, user rectangle, clearPattern, getLastExecutionTime).
"""
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

from fastest_image_pattern_matching_amd import synth
from tests import oracle
from tests.cases import CASES

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(REPO, "build", "dropin_main")
DROPIN = os.path.join(REPO, "fastest_image_pattern_matching_amd", "dropin", "TemplateMatcher_fpm.cpp")
FIXTURE_H = os.path.join(REPO, "tests", "dropin", "TemplateMatcher.h")
REF_H = "/root/reference/include/TemplateMatcher.h"


def _public_decls(text):
    body = text[text.index("public:"):text.index("private:")]
    names = []
    for m in re.finditer(r"([\w:<>]+[\s&*]+)(~?\w+)\s*\(([^)]*)\)\s*(const)?", body):
        names.append((m.group(2), re.sub(r"\s+", "", m.group(3)), bool(m.group(4))))
    return names


def test_dropin_declares_reference_interface():
    if not os.path.exists(REF_H):
        pytest.skip("reference header not present (GPU box)")
    with open(REF_H, encoding="utf-8", errors="replace") as f:
        ref = _public_decls(f.read())
    with open(FIXTURE_H) as f:
        ours = _public_decls(f.read())
    assert len(ref) >= 20
    for d in ref:
        assert d in ours, f"reference public member {d} missing from the fixture header"
    with open(DROPIN) as f:
        src = f.read()
    inline = {"setMaxPositions", "setMaxOverlap", "setScore", "setToleranceAngle", "setMinReduceArea", "setUseSIMD",
              "setSubPixelEstimation", "getMaxPositions", "getMaxOverlap", "getScore", "getToleranceAngle",
              "getMinReduceArea", "getUseSIMD", "getSubPixelEstimation", "getLastExecutionTime", "isPatternLearned"}
    for name, _, _ in ref:
        if name in inline:
            continue
        assert re.search(r"TemplateMatcher::" + re.escape(name) + r"\s*\(", src), f"{name} not defined by the drop-in"


def test_dropin_driver_builds():
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "tests", "dropin")])
    assert os.access(DRIVER, os.X_OK)


def _run_driver(t, s, max_pos, overlap, score, tol, mra=256, simd=1, subpixel=0):
    with tempfile.TemporaryDirectory() as d:
        tp, sp = os.path.join(d, "t.raw"), os.path.join(d, "s.raw")
        np.ascontiguousarray(t).tofile(tp)
        np.ascontiguousarray(s).tofile(sp)
        args = [DRIVER, tp, str(t.shape[1]), str(t.shape[0]), sp, str(s.shape[1]), str(s.shape[0]), str(max_pos),
                repr(float(overlap)), repr(float(score)), repr(float(tol)), str(mra), str(simd), str(subpixel)]
        out = subprocess.run(args, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    res, checks = [], {}
    for line in out.stdout.splitlines():
        f = line.split()
        if f[0] == "R":
            res.append(tuple(float.fromhex(x) for x in f[1:]))
        elif f[0] == "CHECK":
            checks[f[1]] = int(f[2])
    return res, checks


EXPECTED_CHECKS = {"learned_before": 0, "empty_learn": 0, "rect_set": 1, "learn": 1, "rect_reset_by_learn": 1,
                   "time_positive": 1, "copy_same": 1, "again_same": 1, "none_found": 1, "time_kept": 1,
                   "rect_cleared": 1, "cleared": 1, "color_refused": 1}

def _oracle_ui_sequence(t, s, p):
    """The oracle driven as MatchToolDialog drives the class: learnPattern at template load with the constructor's
    parameters (MinReduceArea 256, src/MatchToolDialog.cpp:358), then the setters and match on Execute (:265-286)."""
    o = oracle.OracleMatcher()
    assert o.learnPattern(t)
    o.set(**p)
    return o.match(s)


DROPIN_CASES = {
    "dst10_multi": CASES["dst10_multi"],
    "dst5_subpixel": CASES["dst5_subpixel"],
    "dst4_overlap": CASES["dst4_overlap"],
    "top_is_layer0": CASES["top_is_layer0"],
}


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(DROPIN_CASES))
def test_dropin_search_parity(templates, case):
    make, prm = DROPIN_CASES[case]
    s, t = make(templates)
    p = dict(max_pos=70, max_overlap=0.0, score=0.7, tolerance_angle=0.0, min_reduce_area=256, use_simd=1, subpixel=0)
    p.update(prm)
    got, checks = _run_driver(t, s, p["max_pos"], p["max_overlap"], p["score"], p["tolerance_angle"],
                              p["min_reduce_area"], p["use_simd"], p["subpixel"])
    exp = _oracle_ui_sequence(t, s, p)
    assert got == exp, (case, got, exp)
    assert len(got) >= 1
    assert checks == EXPECTED_CHECKS, checks


@pytest.mark.gpu
@pytest.mark.parametrize("mra", [256, 1024])
def test_dropin_src7_full_size(templates, mra):
    """BASELINE configs[1] through the C++ class: 4024x3036 Src7 surrogate, Dst7, +-180, TargetNum 3; also the
    UI's learn at MinReduceArea 256 followed by an Execute at 1024 (one pyramid level fewer at match time)."""
    s, t = synth.src7_scene(templates["Dst7"])
    got, checks = _run_driver(t, s, 3, 0.0, 0.7, 180.0, mra)
    exp = _oracle_ui_sequence(t, s, dict(max_pos=3, tolerance_angle=180.0, score=0.7, min_reduce_area=mra))
    assert got == exp and len(got) == 3
    assert checks == EXPECTED_CHECKS, checks


@pytest.mark.gpu
def test_dropin_more_results_than_buffer(templates):
    """437 detections (the Qt class does not cap at MaxPos): more than the drop-in's first 256-entry buffer, so the
    rest is fetched with fpm_last_results (no second search) and still equals the oracle."""
    from tests.cases import _grid_scene

    s, t = _grid_scene(templates["Dst4"], 900, 600, 30, 11)
    got, checks = _run_driver(t, s, 500, 0.0, 0.7, 0.0)
    exp = _oracle_ui_sequence(t, s, dict(max_pos=500, score=0.7))
    assert len(exp) > 256 and got == exp
    assert checks == EXPECTED_CHECKS, checks
