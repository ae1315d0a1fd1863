"""The matrix-core top layer (k_top_mma -> k_nms_greedy on its candidate lists, with the full-map fallback) against the
oracle, on the BASELINE configs whose top layer it serves and on template shapes at the edges of its two MFMA layouts
(gfx950 required).

Forms, chosen per fresh context (the switches are read when its plan is built / its search recorded):
  default               k_top_mma wherever the plan admits it (except where the fused small-canvas kernel applies, and
                        plain-peak searches with MaxPos <= 10 and fewer than 128 work units: the split kernels)
  FPM_TOP_MMA=0         the split k_warp -> k_ncc_tile -> k_nms chain (or k_top_fused)
  FPM_TOP_MMA=1         k_top_mma also where k_top_fused would apply
  FPM_TOP_LIST_CAP=1    (with FPM_TOP_MMA=1) lists of one entry: every map with two or more outputs >= the layer score overflows and takes
                        the fallback (k_top_mma mode 1 writes its full map, the split peak kernels take it)
Every result field and every per-layer live count equals the oracle's (bit-identical).
"""
import numpy as np
import pytest

from fastest_image_pattern_matching_amd import _lib as L
from fastest_image_pattern_matching_amd import synth
from tests import oracle
from tests.test_gpu_parity import assert_same_results

pytestmark = pytest.mark.gpu

FORMS = {"default": {}, "split": {"FPM_TOP_MMA": "0"}, "forced": {"FPM_TOP_MMA": "1"},
         "fallback": {"FPM_TOP_MMA": "1", "FPM_TOP_LIST_CAP": "1"}}


def _set(monkeypatch, form):
    for k in ("FPM_TOP_MMA", "FPM_TOP_LIST_CAP"):
        monkeypatch.delenv(k, raising=False)
    for k, v in FORMS[form].items():
        monkeypatch.setenv(k, v)


def _search(gpu_matcher_factory, srcs, t, prm, profile=False):
    m = gpu_matcher_factory(**prm)
    assert m.learnPattern(t)
    if profile:
        m.profile(True)
        m.profile_reset()
    if len(srcs) == 1:
        got = [[r.as_tuple() for r in m.match(srcs[0])]]
    else:
        m.stage(srcs)
        got = [[r.as_tuple() for r in rr] for rr in m.match_staged()]
    stats = m.search_stats()
    launches = {k: m.profile_get(L.KERNEL_NAMES.index(k))[1] for k in ("top_ncc", "top_warp", "top_map")} if profile \
        else None
    return got, stats, launches


def _oracle(srcs, t, prm):
    o = oracle.OracleMatcher().set(**prm)
    assert o.learnPattern(t)
    out = [o.match(s) for s in srcs]
    return out, o.stats()


@pytest.mark.parametrize("form", ["default", "split", "fallback"])
def test_config3_one_degree_forms(gpu_matcher_factory, monkeypatch, form):
    """configs[3] at 1 deg (361 top angles of ~150 x 150 maps, a 16 x 16 top template: the two-row MFMA layout) on two
    4096 x 4096 sources as one batch, and one alone (per-layer live counts)."""
    _set(monkeypatch, form)
    srcs, t = synth.batch_sources(2)
    prm = dict(max_pos=1, tolerance_angle=180.0, top_angle_step=1.0)
    exp, _ = _oracle(srcs, t, prm)
    got, _, launches = _search(gpu_matcher_factory, srcs, t, prm, profile=True)
    assert got == exp and all(len(r) >= 1 for r in exp)
    if form == "split":
        assert launches["top_warp"] >= 1 and launches["top_map"] == 0
    else:
        assert launches["top_warp"] == 0 and launches["top_map"] >= 1
    got1, stats1, _ = _search(gpu_matcher_factory, srcs[1:], t, prm)
    exp1, ostats1 = _oracle(srcs[1:], t, prm)
    assert got1 == exp1 and stats1 == ostats1


@pytest.mark.parametrize("form", ["default", "split", "fallback"])
def test_src10_rotation_sweep_forms(gpu_matcher_factory, templates, monkeypatch, form):
    """configs[2] stress on its 1824 x 1824 quarter (+-180 deg, TargetNum 100: s_BlockMax peaks from the lists; a
    14 x 14 top template; wide maps cut into several strips and row runs)."""
    _set(monkeypatch, form)
    s, t = synth.src10_scene(templates["Dst10"])
    crop = np.ascontiguousarray(s[:1824, :1824])
    prm = dict(max_pos=100, score=0.7, tolerance_angle=180.0)
    exp, ostats = _oracle([crop], t, prm)
    got, stats, _ = _search(gpu_matcher_factory, [crop], t, prm)
    assert stats == ostats
    assert_same_results([_R(r) for r in got[0]], exp[0], f"src10_180 {form}")
    assert len(exp[0]) >= 30


class _R:
    def __init__(self, t):
        self.t = t

    def as_tuple(self):
        return self.t


@pytest.mark.parametrize("form", ["forced", "fallback"])
def test_src7_batch_forced(gpu_matcher_factory, templates, monkeypatch, form):
    """Src7's 12 x 9 top template (odd height: the last two-row slot has a zero row) on tiny maps, where the fused
    small-canvas kernel would otherwise run: a batch of two and one source alone."""
    _set(monkeypatch, "forced")
    if form == "fallback":
        monkeypatch.setenv("FPM_TOP_LIST_CAP", "1")
    t = templates["Dst7"]
    srcs = [synth.src7_scene(t, seed=31 + i)[0] for i in range(2)]
    prm = dict(max_pos=3, tolerance_angle=180.0, score=0.7)
    exp, _ = _oracle(srcs, t, prm)
    got, _, _ = _search(gpu_matcher_factory, srcs, t, prm)
    assert got == exp
    got1, stats1, _ = _search(gpu_matcher_factory, srcs[:1], t, prm)
    exp1, ostats1 = _oracle(srcs[:1], t, prm)
    assert got1 == exp1 and stats1 == ostats1


def _wide_scene(tw, th, seed, angles):
    t = synth.box_blur(synth.noise(tw, th, 128, 60, seed), 3)
    s = synth.box_blur(synth.noise(900, 700, 128, 60, seed + 1), 3)
    for k, a in enumerate(angles):
        synth.paste_rotated(s, t, 250.0 + 400.0 * (k % 2), 220.0 + 280.0 * (k // 2), a)
    return s, t


@pytest.mark.parametrize("form", ["forced", "fallback"])
@pytest.mark.parametrize("shape", [(80, 14, 256), (40, 28, 512), (34, 60, 1024), (6, 60, 256)])
def test_template_shapes(gpu_matcher_factory, monkeypatch, form, shape):
    """Top templates at the edges of the kernel's layouts: 20 x 4 (one-row slots of 64 columns, two pyramid levels),
    20 x 14 (one-row slots; area 280 > 258: no f32 prefilter, every output's exact score), 17 x 30 (the widest two-row
    layout, 15 slots, no prefilter), 3 x 30 (a narrow two-row layout); MaxPos 3 at +-180 with three pasted copies."""
    _set(monkeypatch, form)
    tw, th, mra = shape
    s, t = _wide_scene(tw, th, 90 + tw, [23.0, -61.0, 148.0])
    prm = dict(max_pos=3, tolerance_angle=180.0, score=0.6, min_reduce_area=mra)
    exp, ostats = _oracle([s], t, prm)
    got, stats, launches = _search(gpu_matcher_factory, [s], t, prm, profile=True)
    assert got == exp and stats == ostats
    assert len(exp[0]) >= 1


def test_plain_peaks_overlapping_rectangles(gpu_matcher_factory, templates, monkeypatch):
    """Plain getNextMaxLoc from the lists with MaxOverlap 0.6 (painted rectangles smaller than the template, so
    peaks sit close) and TargetNum 8 on a dense grid of copies: the greedy key is the row-major position."""
    _set(monkeypatch, "forced")
    t = templates["Dst10"]
    s = synth.noise(700, 520, 128, 8, 5)
    k = 0
    for y in range(60, 480, 70):
        for x in range(60, 660, 75):
            synth.paste_rotated(s, t, x, y, (k * 37) % 360 - 180.0)
            k += 1
    prm = dict(max_pos=8, tolerance_angle=180.0, score=0.6, max_overlap=0.6)
    exp, ostats = _oracle([s], t, prm)
    got, stats, _ = _search(gpu_matcher_factory, [s], t, prm)
    assert got == exp and stats == ostats


@pytest.mark.parametrize("form", ["forced", "forced_fallback", "split"])
def test_rect_missing_its_peak(gpu_matcher_factory, monkeypatch, form):
    """MaxOverlap 0.8 on a 107 x 35 template (top level 14 x 5): getNextMaxLoc paints int(2 * 5 * 0.2) = 1 row starting
    a row above the peak, so the peak survives and the reference takes it again with every remaining call (14 equal
    records per angle).  The greedy form reproduces the repeats (forced: a lone plain search this small takes the
    split kernels by default); records, stats and results equal the oracle's."""
    from tests.test_gpu_fuzz import _case

    _set(monkeypatch, "split" if form == "split" else "forced")
    if form == "forced_fallback":
        monkeypatch.setenv("FPM_TOP_LIST_CAP", "1")
    s, t, prm = _case(24)
    o = oracle.OracleMatcher().set(**prm)
    assert o.learnPattern(t)
    exp = o.match(s)
    m = gpu_matcher_factory(**prm)
    assert m.learnPattern(t)
    got = [r.as_tuple() for r in m.match(s)]
    assert m.last_candidates(0).tobytes() == o.candidates().tobytes()
    assert got == exp and m.search_stats() == o.stats()
