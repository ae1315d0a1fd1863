"""HIP path vs the CPU oracle for the search variants beyond the Qt defaults, through the C ABI (gfx950 required):

* BASELINE configs[3] as stated — "+-180 deg at 1 deg step" — via the top-layer step override
  (fpm_params.top_angle_step, an extension: the reference derives the step, TemplateMatcher.cpp:130);
* the MFC tool's result semantics (fpm_params.semantics = FPM_SEMANTICS_MFC): 2x-template
  s_BlockMax blocks with last-block ties (MatchTool/MatchToolDlg.h:93-210), tolerance-range angle lists
  (MatchToolDlg.cpp:805-815), f64 corners, negated/wrapped angles and the MaxPos cap (:1080-1116);
* cv::minMaxLoc on an empty s_BlockMax strip (0 at (-1, -1)), reachable with a map narrower than the template.

Bar as in test_gpu_parity: every field of every result bit-identical, per-layer live counts equal.
"""
import numpy as np
import pytest

from fastest_image_pattern_matching_amd import synth
from tests import oracle
from tests.cases import CASES, _run_both
from tests.test_gpu_parity import assert_same_results

pytestmark = pytest.mark.gpu

MFC = 1


@pytest.fixture(scope="module")
def hip(gpu_matcher_factory):
    return gpu_matcher_factory()


def test_config3_one_degree_step(hip):
    """configs[3] at its stated 1-degree top-layer step (361 angles) on two 4096x4096 sources with the 512x512
    template, searched as one device batch."""
    srcs, t = synth.batch_sources(2)
    o = oracle.OracleMatcher().set(max_pos=1, tolerance_angle=180.0, top_angle_step=1.0)
    o.learnPattern(t)
    hip.resetParams()
    hip.setMaxPositions(1)
    hip.setToleranceAngle(180.0)
    hip._params.top_angle_step = 1.0
    assert hip.learnPattern(t)
    batch = hip.match_batch(srcs)
    for k, s in enumerate(srcs):
        orc = o.match(s)
        assert_same_results(batch[k], orc, f"batch4096_1deg_{k}")
        assert len(orc) >= 1
    assert hip.search_stats()[0] == 361
    # one source alone: identical per-layer live counts
    gpu = hip.match(srcs[1])
    assert_same_results(gpu, o.match(srcs[1]), "single_1deg")
    assert hip.search_stats() == o.stats()
    hip._params.top_angle_step = 0.0


@pytest.mark.parametrize("step", [0.5, 3.0, 10.0])
def test_top_angle_step_override(hip, templates, step):
    make, prm = CASES["dst10_multi"]
    s, t = make(templates)
    gpu, orc, ostats, gstats = _run_both(hip, s, t, top_angle_step=step, **prm)
    assert gstats == ostats
    assert_same_results(gpu, orc, f"step{step}")


@pytest.mark.parametrize("case", sorted(c for c in CASES if c != "dst3_range"))   # (ranges: test_mfc_tolerance_ranges)
def test_mfc_semantics_cases(hip, templates, case):
    make, prm = CASES[case]
    s, t = make(templates)
    gpu, orc, ostats, gstats = _run_both(hip, s, t, semantics=MFC, **prm)
    assert gstats == ostats, (gstats, ostats)
    assert_same_results(gpu, orc, f"mfc_{case}")
    assert len(gpu) <= max(prm.get("max_pos", 70), 1)
    for r in gpu:
        assert -180.0 <= r.dMatchedAngle <= 180.0


def test_mfc_src10_blockmax(hip, templates):
    """configs[2] (TargetNum 100, s_BlockMax) with MFC blocks: 2x template, last-block ties."""
    s, t = synth.src10_scene(templates["Dst10"])
    gpu, orc, ostats, gstats = _run_both(hip, s, t, max_pos=100, score=0.7, tolerance_angle=0.0, semantics=MFC)
    assert gstats == ostats
    assert_same_results(gpu, orc, "mfc_src10")
    assert len(gpu) == 100   # capped at MaxPos


def test_mfc_blockmax_ties(hip, templates):
    """Exactly equal scores in different MFC blocks: the LAST block wins (MatchToolDlg.h:206 '>=')."""
    t = templates["Dst10"]
    s = np.full((1824, 1824), 90, np.uint8)
    for gy in range(9):
        for gx in range(9):
            synth.paste(s, t, 96 + 192 * gx, 96 + 192 * gy)
    gpu, orc, ostats, gstats = _run_both(hip, s, t, max_pos=50, score=0.7, tolerance_angle=0.0, semantics=MFC)
    assert gstats == ostats
    assert_same_results(gpu, orc, "mfc_ties")
    q, qo = _run_both(hip, s, t, max_pos=50, score=0.7, tolerance_angle=0.0)[:2]
    assert [r.ptCenter for r in gpu] != [r.ptCenter for r in q[:50]]   # the tie rule shows


@pytest.mark.parametrize("prm", [dict(max_overlap=0.4, max_pos=60, score=0.5), dict(max_overlap=1.0),
                                 dict(score=0.05), dict(tolerance_angle=180.0, max_pos=40)],
                         ids=["overlap", "empty_rect", "many_candidates", "rotation"])
def test_mfc_blockmax_paths(hip, templates, prm):
    s, t = synth.src10_scene(templates["Dst10"])
    crop = np.ascontiguousarray(s[:1824, :1830])
    base = dict(max_pos=30, score=0.7, tolerance_angle=0.0, semantics=MFC)
    base.update(prm)
    gpu, orc, ostats, gstats = _run_both(hip, crop, t, **base)
    assert gstats == ostats
    assert_same_results(gpu, orc, f"mfc_blockmax_{prm}")


def test_mfc_tolerance_ranges(hip, templates):
    """MFC angle ranges [t1, t2] + [t3, t4] (MatchToolDlg.cpp:805-815); inverted ranges are refused (:807-811)."""
    t = templates["Dst10"]
    s = synth.noise(560, 400, 128, 10, 31)
    for cx, cy, a in [(120, 110, 40.0), (330, 250, -75.0), (440, 120, 150.0)]:
        synth.paste_rotated(s, t, cx, cy, a)
    rng = dict(max_pos=5, semantics=MFC, tolerance_range=1, tolerance_angle=0.0)
    hip.resetParams()
    o = oracle.OracleMatcher()
    for k, v in rng.items():
        setattr(hip._params, k, v)
        setattr(o.params, k, v)
    for k, v in enumerate((-90.0, -30.0, 20.0, 60.0)):
        hip._params.tolerance[k] = v
        o.params.tolerance[k] = v
    assert hip.learnPattern(t) and o.learnPattern(t)
    gpu, orc = hip.match(s), o.match(s)
    assert hip.search_stats() == o.stats()
    assert_same_results(gpu, orc, "mfc_ranges")
    assert len(gpu) >= 2
    hip._params.tolerance[1] = -95.0
    assert hip.match(s) == []


@pytest.mark.parametrize("semantics", [0, MFC])
def test_empty_strip_minmaxloc(hip, semantics):
    """A top-layer map narrower than the template: the Qt bottom strip has zero width (and MFC keeps the full-map
    scan), with score 0 so the strip's cv::minMaxLoc answer (0 at (-1, -1)) is a peak the reference accepts."""
    t = synth.box_blur(synth.noise(20, 20, 128, 40, 41), 3)
    s = synth.box_blur(synth.noise(30, 12000, 128, 40, 42), 3)
    synth.paste(s, t, 4, 6000)
    gpu, orc, ostats, gstats = _run_both(hip, s, t, max_pos=12, score=0.0, tolerance_angle=0.0, semantics=semantics)
    assert gstats == ostats
    assert_same_results(gpu, orc, f"empty_strip_{semantics}")
