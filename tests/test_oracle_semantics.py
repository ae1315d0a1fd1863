"""CPU checks of the oracle's search variants (no GPU): the top-layer step override and the MFC tool's result
semantics (MatchTool/MatchToolDlg.cpp:805-815, 1080-1116, MatchToolDlg.h:93-210), each
against the Qt-semantics search of the same scene, whose own parity is pinned by tests/test_oracle_*.py."""
import math

import pytest

from fastest_image_pattern_matching_amd import synth
from tests import oracle
from tests.cases import CASES

MFC = 1


def _search(s, t, **prm):
    o = oracle.OracleMatcher().set(**prm)
    assert o.learnPattern(t)
    return o.match(s), o.stats()


@pytest.fixture(scope="module")
def templates():
    return synth.load_templates()


def test_top_angle_step_counts(templates):
    s, t = CASES["dst10_multi"][0](templates)
    for step, n in ((1.0, 361), (10.0, 37), (45.0, 9)):
        _, st = _search(s, t, max_pos=5, tolerance_angle=180.0, top_angle_step=step)
        # 0, step, ... while < 180 + step, then -step, ... while > -180 - step (TemplateMatcher.cpp:134-143)
        assert st[0] == n
    res, _ = _search(s, t, max_pos=5, tolerance_angle=180.0, top_angle_step=1.0)
    assert len(res) == 3


@pytest.mark.parametrize("case", ["dst10_multi", "dst1_rot30", "score_low_many", "dst5_subpixel"])
def test_mfc_conversion_vs_qt(templates, case):
    """Same detections (no s_BlockMax in these cases): the MFC rows carry the negated, wrapped angle and f64
    corners computed from the same f64 point, within f32 rounding of the Qt rows."""
    make, prm = CASES[case]
    s, t = make(templates)
    qt, qst = _search(s, t, **prm)
    mfc, mst = _search(s, t, semantics=MFC, **prm)
    assert qst == mst and len(qt) == len(mfc) >= 1
    for a, b in zip(qt, mfc):
        assert a[11] == b[11]                                   # score
        assert b[10] == -a[10] and -180 <= b[10] <= 180         # angle
        assert a[0] == b[0] and a[1] == b[1]                    # ptLT: f32 in both
        for k in range(2, 10):
            assert abs(a[k] - b[k]) < 1e-3                      # f32 vs f64 corner arithmetic


def test_mfc_caps_results_at_maxpos(templates):
    make, prm = CASES["dst4_block"]
    s, t = make(templates)
    qt, _ = _search(s, t, **prm)
    mfc, _ = _search(s, t, semantics=MFC, **prm)
    assert len(qt) > prm["max_pos"] and len(mfc) == prm["max_pos"]


def test_mfc_blocks_differ_from_qt(templates):
    """Equal scores at many sites: Qt takes the first block, MFC (2x blocks) the last."""
    import numpy as np

    t = templates["Dst10"]
    s = np.full((1824, 1824), 90, np.uint8)
    for gy in range(9):
        for gx in range(9):
            synth.paste(s, t, 96 + 192 * gx, 96 + 192 * gy)
    qt, _ = _search(s, t, max_pos=50, score=0.7)
    mfc, _ = _search(s, t, max_pos=50, score=0.7, semantics=MFC)
    assert len(mfc) == 50 and [r[8:10] for r in qt[:50]] != [r[8:10] for r in mfc]


def test_mfc_tolerance_ranges(templates):
    t = templates["Dst10"]
    s = synth.noise(560, 400, 128, 10, 31)
    for cx, cy, a in [(120, 110, 40.0), (330, 250, -75.0), (440, 120, 150.0)]:
        synth.paste_rotated(s, t, cx, cy, a)
    o = oracle.OracleMatcher().set(max_pos=5, semantics=MFC, tolerance_range=1)
    for k, v in enumerate((-90.0, -30.0, 20.0, 60.0)):
        o.params.tolerance[k] = v
    assert o.learnPattern(t)
    res = o.match(s)
    got = sorted(round(r[10]) for r in res)
    # the tool reports -dMatchAngle: the +40 / -75 deg copies appear as -40 / +76 (Dst10's near-4-fold symmetry also
    # puts the 150 deg copy at 60.65 deg, inside [20, 60] + one step)
    assert {-40, 76} <= set(got) and all(-92 <= -a <= -29 or 19 <= -a <= 62 for a in got)
    assert all(math.isfinite(r[11]) for r in res)
    o.params.tolerance[1] = -95.0                          # t1 >= t2: refused (MatchToolDlg.cpp:807-811)
    assert o.match(s) == []
