"""Known-answer tests that pin the CPU oracle (SURVEY.md §4 "constructed KATs") — no GPU needed.

The reference ships no tests and cannot be built here (OpenCV absent), so the oracle is pinned by:
  * properties that hold for OpenCV's primitives independent of implementation details (constant images,
    exact 90-degree warps, integer translations, verbatim-pasted templates scoring 1, the ResultEqual1 branch);
  * independent numpy restatements of the integer pyrDown and the f64 normalisation;
  * the README's own Src7 answers (README.md:45-49) on a synthetic Src7 and the plumbing case of §8(d).
"""
import numpy as np
import pytest

from tests import oracle


def np_pyr_down(img):
    """Independent restatement of cv::pyrDown in numpy."""
    h, w = img.shape
    k = np.array([1, 4, 6, 4, 1], np.int64)

    def r101(p, n):
        p = np.abs(p)
        p = np.where(p >= n, 2 * n - 2 - p, p)
        return p

    dw, dh = (w + 1) // 2, (h + 1) // 2
    xs = r101(2 * np.arange(dw)[:, None] + np.arange(5)[None, :] - 2, w)
    ys = r101(2 * np.arange(dh)[:, None] + np.arange(5)[None, :] - 2, h)
    a = img.astype(np.int64)
    hor = (a[:, xs] * k[None, None, :]).sum(-1)            # h x dw
    ver = (hor[ys, :] * k[None, :, None]).sum(1)           # dh x dw
    return ((ver + 128) >> 8).astype(np.uint8)


@pytest.mark.parametrize("shape", [(1, 1), (2, 3), (5, 7), (17, 30), (64, 64), (101, 77), (300, 513)])
def test_pyr_down_matches_numpy(shape):
    rng = np.random.default_rng(shape[0] * 1000 + shape[1])
    img = rng.integers(0, 256, shape, dtype=np.uint8)
    if min(shape) >= 2:
        assert np.array_equal(oracle.pyr_down(img), np_pyr_down(img))


@pytest.mark.parametrize("v", [0, 1, 127, 255])
def test_pyr_down_constant(v):
    img = np.full((45, 62), v, np.uint8)
    assert np.all(oracle.pyr_down(img) == v)


@pytest.mark.parametrize("k", [1, 2, 3])
def test_warp_exact_quarter_turns(k):
    # rotation about the centre of a square image with an integer-valued matrix is a pixel permutation
    rng = np.random.default_rng(k)
    img = rng.integers(0, 256, (31, 31), dtype=np.uint8)
    m = oracle.rotation_matrix(15.0, 15.0, 90.0 * k)
    m = np.round(m)  # cos/sin of multiples of 90 degrees are exact up to 1e-16: the warp uses lrint anyway
    out = oracle.warp_affine(img, m, (31, 31), 0)
    assert np.array_equal(out, np.rot90(img, k))


def test_warp_identity_and_translation():
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (20, 33), dtype=np.uint8)
    out = oracle.warp_affine(img, [[1, 0, 0], [0, 1, 0]], (33, 20), 7)
    assert np.array_equal(out, img)
    out = oracle.warp_affine(img, [[1, 0, 5], [0, 1, -3]], (40, 25), 200)
    exp = np.full((25, 40), 200, np.uint8)
    exp[0:17, 5:38] = img[3:20, 0:33]
    assert np.array_equal(out, exp)


def test_warp_half_pixel_bilinear():
    # a 0.5 px shift averages neighbours with weights 16*32*32 = 16384 each: (a*16384 + b*16384 + 16384) >> 15
    img = np.array([[10, 20, 40, 80]], np.uint8).repeat(3, 0)
    out = oracle.warp_affine(img, [[1, 0, -0.5], [0, 1, 0]], (3, 3), 0)
    exp = ((img[:, :3].astype(int) + img[:, 1:].astype(int)) * 16384 + 16384) >> 15
    assert np.array_equal(out, exp.astype(np.uint8))


def np_ncc(img, t):
    """Independent f64 CCOEFF_NORMED with the reference's clamp branches (TemplateMatcher.cpp:527-598)."""
    img = img.astype(np.float64)
    t = t.astype(np.float64)
    th, tw = t.shape
    n = t.size
    tm = t.mean()
    tn = np.sqrt(((t - tm) ** 2).mean()) * np.sqrt(n)
    oh, ow = img.shape[0] - th + 1, img.shape[1] - tw + 1
    out = np.zeros((oh, ow))
    for y in range(oh):
        for x in range(ow):
            win = img[y:y + th, x:x + tw]
            num = (win * t).sum() - win.sum() * tm
            den = np.sqrt(max((win ** 2).sum() - win.sum() ** 2 / n, 0)) * tn
            out[y, x] = num / den if abs(num) < den else (np.sign(num) if den > 0 and abs(num) < den * 1.125 else 0)
    return out


def test_ncc_map_against_numpy(templates):
    rng = np.random.default_rng(11)
    t = rng.integers(0, 256, (9, 12), dtype=np.uint8)
    img = rng.integers(0, 256, (30, 41), dtype=np.uint8)
    m = oracle.OracleMatcher().set(min_reduce_area=4096)
    assert m.learnPattern(t)
    for fold in (False, True):
        got = m.ncc_map(img, 0, fold)
        assert np.allclose(got, np_ncc(img, t), atol=2e-6)


def test_pasted_template_scores_one(templates):
    t = templates["Dst10"]
    img = np.random.default_rng(4).integers(0, 256, (90, 120), dtype=np.uint8)
    img[20:74, 33:87] = t
    m = oracle.OracleMatcher().set(min_reduce_area=1 << 20)
    m.learnPattern(t)
    got = m.ncc_map(img, 0, True)
    y, x = np.unravel_index(np.argmax(got), got.shape)
    assert (y, x) == (20, 33) and got[y, x] >= 0.99999


def test_constant_template_result_equal1():
    t = np.full((10, 10), 77, np.uint8)
    img = np.random.default_rng(5).integers(0, 256, (40, 40), dtype=np.uint8)
    m = oracle.OracleMatcher().set(min_reduce_area=1024)
    m.learnPattern(t)
    levels, _ = m.template_levels()
    assert levels[0][4] is True
    assert np.all(m.ncc_map(img, 0, True) == 1.0)


def test_learn_statistics(templates):
    t = templates["Dst1"]
    m = oracle.OracleMatcher()
    m.learnPattern(t)
    levels, border = m.template_levels()
    assert len(levels) == 5                       # 466x135 -> top 30x9 at MinReduceArea 256
    assert levels[-1][0].shape == (9, 30)
    assert border == 255                          # mean 88.5 < 128 (TemplateMatcher.cpp:58-59)
    for px, mean, norm, inv, _ in levels:
        assert mean == pytest.approx(px.mean(), rel=1e-12)
        assert norm == pytest.approx(px.std() * np.sqrt(px.size), rel=1e-9)
        assert inv == 1.0 / px.size


def test_plumbing_kat(templates):
    """Dst1 pasted at (400, 300): one result, score ~1, centre (633, 367.5)."""
    from fastest_image_pattern_matching_amd import synth

    s, t = synth.plumbing_scene(templates["Dst1"])
    m = oracle.OracleMatcher().set(max_pos=1, tolerance_angle=0.0)
    m.learnPattern(t)
    r = m.match(s)
    assert len(r) == 1
    assert r[0][8:10] == (633.0, 367.5) and r[0][11] >= 0.999


@pytest.mark.slow
def test_src7_readme_poses(templates):
    """README.md:45-49 on the synthetic Src7: 3 targets at the published centres (±1 px) and angles (±0.3°,
    Qt sign)."""
    from fastest_image_pattern_matching_amd import synth

    s, t = synth.src7_scene(templates["Dst7"])
    m = oracle.OracleMatcher().set(max_pos=3, tolerance_angle=180.0, score=0.7)
    m.learnPattern(t)
    r = m.match(s)
    assert len(r) == 3
    for _, ang, cx, cy in synth.SRC7_POSES:
        best = min(r, key=lambda q: (q[8] - cx) ** 2 + (q[9] - cy) ** 2)
        assert abs(best[8] - cx) < 1.0 and abs(best[9] - cy) < 1.0
        assert abs(best[10] - (-ang)) < 0.3
        assert best[11] > 0.99


def test_rotrect_overlap_cases():
    sq = [(0, 0), (10, 0), (10, 10)]
    t, area, n = oracle.rotrect_overlap(sq, sq)
    assert t == 2                                           # coincident -> INTERSECT_FULL
    t, area, n = oracle.rotrect_overlap(sq, [(20, 0), (30, 0), (30, 10)])
    assert t == 0                                           # disjoint -> INTERSECT_NONE
    t, area, n = oracle.rotrect_overlap(sq, [(5, 0), (15, 0), (15, 10)])
    assert t == 1 and n == 4 and area == pytest.approx(50.0)


@pytest.mark.parametrize("shape,tshape", [((70, 90), (17, 24)), ((300, 280), (40, 31)), ((12, 9), (12, 9))])
def test_cross_corr_f32_sensitivity_mode(shape, tshape):
    """The oracle's float32-DFT TM_CCORR (sensitivity mode, OpenCV crossCorr's block structure; the 300x280 case
    spans several DFT blocks) against the exact integer sum: its error is of float32 DFT size -- the same order as
    numpy's float32 FFT of the same product."""
    rng = np.random.default_rng(sum(shape) + sum(tshape))
    img = rng.integers(0, 256, shape, dtype=np.uint8)
    t = rng.integers(0, 256, tshape, dtype=np.uint8)
    got = oracle.cross_corr_f32(img, t).astype(np.float64)
    (h, w), (th, tw) = shape, tshape
    ex = np.zeros((h - th + 1, w - tw + 1), np.float64)
    for y in range(th):
        for x in range(tw):
            ex += float(t[y, x]) * img[y:y + h - th + 1, x:x + w - tw + 1]
    H, W = h + th, w + tw
    A = np.fft.fft2(img.astype(np.float32), s=(H, W))
    B = np.fft.fft2(t.astype(np.float32), s=(H, W))
    npf = np.fft.ifft2(A * np.conj(B)).real[:h - th + 1, :w - tw + 1]
    err, np_err = np.abs(got - ex).max(), np.abs(npf - ex).max()
    assert err <= 8 * max(np_err, 1.0) and err / ex.max() < 1e-5
