"""The device overlap filter (k_overlap_pairs + the host replay, fpm_engine.hip overlap_filter_device) and its
fallbacks against the oracle's sequential filterWithRotatedRect (TemplateMatcher.cpp:1133-1194), through the C-ABI
operator fpm_op_overlap_filter on crafted rectangle sets (gfx950 required).

Every case asserts the surviving indices equal the oracle's and that the path under test ran (stats: path 1 = device
decisions replayed, 2 = device fell back to the host filter; host-decided pairs; fallback flags):
* realistic sets at several MaxOverlap values (device path, no fallback);
* a rectangle with more than kOverlapMaxCand (512) overlapping partners (flag 1, host fallback);
* a pair list over its 48 n entries (flag 2, host fallback);
* pairs whose point order needs the host's acos: intersections of tiny rectangles, whose points lie within 2 px of
  their centre, so the reference's key argument d.x / |d|^2 leaves [-1/2, 1/2] (sort_pts_fast gives up);
* adversarial geometry: coincident and contained rectangles, near-equal angles, overlap ratios straddling MaxOverlap,
  a NaN score (the reference's delete rule compares the scores again).
"""
import math

import numpy as np
import pytest

from tests import oracle

pytestmark = pytest.mark.gpu


def rects(cx, cy, w, h, ang_deg):
    """(ptLT, ptRT, ptRB) rows of template-sized rectangles as match() builds them (TemplateMatcher.cpp:380-390):
    lt from the centre, then rt = lt + w (cos, -sin), rb = rt + h (sin, cos), all in f32."""
    cx, cy, a = (np.asarray(v, np.float64) for v in (cx, cy, ang_deg))
    rad = -a * math.pi / 180.0
    cs, sn = np.cos(rad).astype(np.float32), np.sin(rad).astype(np.float32)
    ltx = (cx - 0.5 * (w * cs + h * sn)).astype(np.float32)
    lty = (cy - 0.5 * (-w * sn + h * cs)).astype(np.float32)
    rtx = ltx + np.float32(w) * cs
    rty = lty - np.float32(w) * sn
    rbx = rtx + np.float32(h) * sn
    rby = rty + np.float32(h) * cs
    return np.stack([ltx, lty, rtx, rty, rbx, rby], 1).astype(np.float32)


def check(m, corners, scores, max_overlap):
    exp = oracle.filter_rotated_rect(corners, scores, max_overlap)
    host, hst = m.overlap_filter(corners, scores, max_overlap, device=False)
    dev, dst = m.overlap_filter(corners, scores, max_overlap, device=True)
    assert host == exp and hst[0] == 0
    assert dev == exp, (len(dev), len(exp))
    return dst


@pytest.fixture(scope="module")
def m(gpu_matcher_factory):
    return gpu_matcher_factory()


@pytest.mark.parametrize("max_overlap", [0.0, 0.2, 0.5, 0.8])
@pytest.mark.parametrize("seed", [0, 1])
def test_overlap_realistic(m, seed, max_overlap):
    rng = np.random.default_rng(seed)
    n = 400
    c = rects(rng.uniform(0, 500, n), rng.uniform(0, 400, n), 62.0, 41.0, rng.uniform(-180, 180, n))
    s = np.sort(rng.uniform(0.5, 1.0, n))[::-1]
    st = check(m, c, s, max_overlap)
    assert st[0] == 1 and st[2] == 0


def test_overlap_too_many_partners(m):
    """600 rectangles within a few pixels: every one overlaps 599 > 512 others -> flag 1, host filter."""
    rng = np.random.default_rng(5)
    n = 600
    c = rects(200 + rng.uniform(-3, 3, n), 150 + rng.uniform(-3, 3, n), 50.0, 30.0, rng.uniform(-20, 20, n))
    s = np.sort(rng.uniform(0.5, 1.0, n))[::-1]
    st = check(m, c, s, 0.5)
    assert st[0] == 2 and st[2] & 1


def test_overlap_list_overflow(m):
    """150 mutually overlapping rectangles at MaxOverlap 0 (every overlapping pair deletes one of the two, so every
    pair is listed): 11175 entries > 48 n = 7200 -> flag 2, host filter."""
    rng = np.random.default_rng(6)
    n = 150
    c = rects(300 + rng.uniform(-4, 4, n), 300 + rng.uniform(-4, 4, n), 80.0, 60.0, rng.uniform(-10, 10, n))
    s = np.sort(rng.uniform(0.5, 1.0, n))[::-1]
    st = check(m, c, s, 0.0)
    assert st[0] == 2 and st[2] == 2


@pytest.mark.parametrize("seed", [7, 8, 9])
def test_overlap_host_acos_pairs(m, seed):
    """Tiny rectangles (3 x 2 px) packed at random sub-pixel positions and angles: their intersection points lie
    within 2 px of the polygon centre, so the reference's acos argument leaves [-1/2, 1/2] and the device hands the
    pair's point order to the host."""
    rng = np.random.default_rng(seed)
    n = 500
    c = rects(rng.uniform(0, 40, n), rng.uniform(0, 40, n), 3.0, 2.0, rng.uniform(-180, 180, n))
    s = np.sort(rng.uniform(0.5, 1.0, n))[::-1]
    st = check(m, c, s, 0.1)
    assert st[0] == 1 and st[1] > 0


def test_overlap_adversarial(m):
    rng = np.random.default_rng(11)
    base = rects([100.0], [100.0], 60.0, 40.0, [30.0])
    parts = [base, base.copy(),                                      # coincident (INTERSECT_FULL)
             rects([100.0], [100.0], 60.0, 40.0, [30.0 + 1e-5]),       # near-equal angle
             rects([100.3], [100.2], 60.0, 40.0, [30.0]),              # shifted by a fraction of a pixel
             rects([400.0], [100.0], 60.0, 40.0, [0.0]),
             rects([400.0], [100.0], 60.0, 40.0, [90.0])]             # a cross (8 intersection points)
    # overlap ratios straddling MaxOverlap 0.5: axis-aligned copies shifted so the overlap is 0.5 -+ a few ulps of
    # the 60-px width
    for dx in (30.0 - 1e-4, 30.0, 30.0 + 1e-4):
        parts.append(rects([700.0, 700.0 + dx], [100.0, 100.0], 60.0, 40.0, [0.0, 0.0]))
    # a random cluster around a corner-touching pair
    parts.append(rects(900 + rng.uniform(-40, 40, 60), 300 + rng.uniform(-40, 40, 60), 60.0, 40.0,
                       rng.uniform(-180, 180, 60)))
    c = np.concatenate(parts)
    n = len(c)
    s = np.sort(rng.uniform(0.6, 1.0, n))[::-1].copy()
    s[5] = s[6]                                                      # a tie
    for mo in (0.0, 0.5, 0.9):
        st = check(m, c, s, mo)
        assert st[0] == 1
    s_nan = s.copy()
    s_nan[3] = np.nan                                                # non-monotone scores: the rule compares again
    st = check(m, c, s_nan, 0.5)
    assert st[0] == 1


def test_device_filter_twice_in_one_context(gpu_matcher_factory):
    """k_overlap_pairs writes its pair lists to mapped pinned host memory with plain stores and no fence (the host
    reads them after hipStreamSynchronize, the rule k_pack follows too): two device filters on different rectangle
    sets back to back in ONE context, then the first set again -- a stale list from the previous call would change
    the survivors.  Every call equals the oracle's sequential filter."""
    mm = gpu_matcher_factory()
    sets = []
    for seed, (n, w, h) in enumerate([(420, 62.0, 41.0), (380, 40.0, 70.0)]):
        rng = np.random.default_rng(700 + seed)
        c = rects(rng.uniform(0, 450, n), rng.uniform(0, 380, n), w, h, rng.uniform(-180, 180, n))
        sets.append((c, np.sort(rng.uniform(0.5, 1.0, n))[::-1].copy()))
    for c, s in sets + sets[:1]:
        exp = oracle.filter_rotated_rect(c, s, 0.3)
        dev, dst = mm.overlap_filter(c, s, 0.3, device=True)
        assert dst[0] == 1 and dev == exp
