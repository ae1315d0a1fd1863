"""The oracle's top-layer peak extraction against an independent line-by-line restatement of the reference's code
(ADVICE round 2): the Qt s_BlockMax (include/DataStructures.h:150-246) with getNextMaxLoc (src/TemplateMatcher.cpp:
179-194, 1208-1221), the MFC tool's s_BlockMax (MatchTool/MatchToolDlg.h:108-210) with its getNextMaxLoc
(MatchToolDlg.cpp:860-874, 1583-1596), and the plain minMaxLoc + painting loop (TemplateMatcher.cpp:195-210,
1196-1206), all written here in pure Python from the reference text -- not from the oracle -- on tiny hand-made
maps: every residue layout of the block grid (right + bottom strips, either alone, none -- the MFC "else" branch then
scans an EMPTY bottom strip, which cv::minMaxLoc reports as 0 at (-1, -1)), maps holding no whole block, exact ties
inside a block and across blocks (Qt keeps the first block, MFC the last), painted rectangles clipped at the borders,
and MaxOverlap > 0.

OpenCV semantics used: minMaxLoc = first maximum in row-major order with strict '>',
an empty array gives value 0 and location (-1, -1); Rect & Rect = the intersection or Rect() when empty;
rectangle(FILLED) fills the rect clipped to the image, nothing when w <= 0 or h <= 0.
"""
import ctypes as C
import itertools

import numpy as np
import pytest

from tests import oracle


def min_max_loc(m, x, y, w, h):
    if w <= 0 or h <= 0:
        return 0.0, (-1, -1)
    sub = m[y:y + h, x:x + w]
    best, bx, by = sub[0, 0], 0, 0
    for yy in range(h):
        for xx in range(w):
            if sub[yy, xx] > best:
                best, bx, by = sub[yy, xx], xx, yy
    return float(best), (bx, by)


def rect_and(a, b):
    x1, y1 = max(a[0], b[0]), max(a[1], b[1])
    x2, y2 = min(a[0] + a[2], b[0] + b[2]), min(a[1] + a[3], b[1] + b[3])
    if x2 - x1 <= 0 or y2 - y1 <= 0:
        return (0, 0, 0, 0)
    return (x1, y1, x2 - x1, y2 - y1)


def fill(m, r, v):
    x, y, w, h = r
    if w <= 0 or h <= 0:
        return
    x1, y1 = max(x, 0), max(y, 0)
    x2, y2 = min(x + w - 1, m.shape[1] - 1), min(y + h - 1, m.shape[0] - 1)
    if x2 >= x1 and y2 >= y1:
        m[y1:y2 + 1, x1:x2 + 1] = v


class QtBlockMax:
    """include/DataStructures.h:150-246"""

    def __init__(self, m, tw, th):
        self.m = m
        self.blocks = []
        bw, bh = tw, th
        ncol, nrow = m.shape[1] // bw, m.shape[0] // bh
        for y in range(nrow):
            for x in range(ncol):
                self._add((x * bw, y * bh, bw, bh))
        if ncol * bw < m.shape[1]:
            self._add((ncol * bw, 0, m.shape[1] - ncol * bw, m.shape[0]))
        if nrow * bh < m.shape[0]:
            self._add((0, nrow * bh, ncol * bw, m.shape[0] - nrow * bh))
        if ncol * bw < m.shape[1] and nrow * bh < m.shape[0]:
            self._add((ncol * bw, nrow * bh, m.shape[1] - ncol * bw, m.shape[0] - nrow * bh))

    def _add(self, r):
        v, (lx, ly) = min_max_loc(self.m, *r)
        self.blocks.append([r, v, (r[0] + lx, r[1] + ly)])

    def update(self, ign):
        for b in self.blocks:
            i = rect_and(b[0], ign)
            if i[2] * i[3] > 0:
                v, (lx, ly) = min_max_loc(self.m, *b[0])
                b[1], b[2] = v, (b[0][0] + lx, b[0][1] + ly)

    def get(self):
        if not self.blocks:
            return -1.0, (-1, -1)
        k = 0
        for i in range(1, len(self.blocks)):   # std::max_element with a.dMax < b.dMax: the first maximum
            if self.blocks[k][1] < self.blocks[i][1]:
                k = i
        return self.blocks[k][1], self.blocks[k][2]


class MfcBlockMax:
    """MatchTool/MatchToolDlg.h:108-210"""

    def __init__(self, m, tw, th):
        self.m = m
        self.blocks = []
        bw, bh = tw * 2, th * 2
        ncol, hres = m.shape[1] // bw, m.shape[1] % bw != 0
        nrow, vres = m.shape[0] // bh, m.shape[0] % bh != 0
        if ncol == 0 or nrow == 0:
            return
        for y in range(nrow):
            for x in range(ncol):
                self._add((x * bw, y * bh, bw, bh))
        if hres and vres:
            self._add((ncol * bw, 0, m.shape[1] - ncol * bw, m.shape[0]))
            self._add((0, nrow * bh, ncol * bw, m.shape[0] - nrow * bh))
        elif hres:
            self._add((ncol * bw, 0, m.shape[1] - ncol * bw, m.shape[0]))
        else:
            self._add((0, nrow * bh, m.shape[1], m.shape[0] - nrow * bh))

    def _add(self, r):
        v, (lx, ly) = min_max_loc(self.m, *r)
        self.blocks.append([r, v, (r[0] + lx, r[1] + ly)])

    def update(self, ign):
        for b in self.blocks:
            i = rect_and(ign, b[0])
            if i[2] == 0 and i[3] == 0:
                continue
            v, (lx, ly) = min_max_loc(self.m, *b[0])
            b[1], b[2] = v, (b[0][0] + lx, b[0][1] + ly)

    def get(self):
        if not self.blocks:
            return min_max_loc(self.m, 0, 0, self.m.shape[1], self.m.shape[0])
        k, dmax = 0, self.blocks[0][1]
        for i in range(1, len(self.blocks)):
            if self.blocks[i][1] >= dmax:
                k, dmax = i, self.blocks[i][1]
        return dmax, self.blocks[k][2]


def reference_sequence(m, tw, th, by_block, mfc, overlap, iters, thr):
    m = m.copy()
    out = []
    if by_block:
        bm = (MfcBlockMax if mfc else QtBlockMax)(m, tw, th)
        v, p = bm.get()
        if v < thr:
            return out
        out.append((v, p[0], p[1]))
        for _ in range(iters):
            ign = (int(p[0] - tw * (1 - overlap)), int(p[1] - th * (1 - overlap)), int(2 * tw * (1 - overlap)),
                   int(2 * th * (1 - overlap)))
            fill(m, ign, -1.0)
            bm.update(ign)
            v, p = bm.get()
            if v < thr:
                break
            out.append((v, p[0], p[1]))
    else:
        v, p = min_max_loc(m, 0, 0, m.shape[1], m.shape[0])
        if v < thr:
            return out
        out.append((v, p[0], p[1]))
        for _ in range(iters):
            ign = (int(p[0] - tw * (1 - overlap)), int(p[1] - th * (1 - overlap)), int(2 * tw * (1 - overlap)),
                   int(2 * th * (1 - overlap)))
            fill(m, ign, -1.0)
            v, p = min_max_loc(m, 0, 0, m.shape[1], m.shape[0])
            if v < thr:
                break
            out.append((v, p[0], p[1]))
    return out


def oracle_sequence(m, tw, th, by_block, mfc, overlap, iters, thr):
    lib = oracle.load()
    lib.orc_peak_sequence.argtypes = [C.POINTER(C.c_float), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                      C.c_double, C.c_int, C.c_double, C.POINTER(C.c_double)]
    m = np.ascontiguousarray(m, np.float32)
    out = np.zeros((iters + 1) * 3, np.float64)
    n = lib.orc_peak_sequence(m.ctypes.data_as(C.POINTER(C.c_float)), m.shape[1], m.shape[0], tw, th, int(by_block),
                              int(mfc), overlap, iters, thr, out.ctypes.data_as(C.POINTER(C.c_double)))
    return [(float(out[3 * i]), int(out[3 * i + 1]), int(out[3 * i + 2])) for i in range(n)]


def _map(w, h, seed, levels):
    """values on a coarse grid of `levels` steps in [-0.2, 1): frequent exact ties"""
    rng = np.random.default_rng(seed)
    return (rng.integers(0, levels, size=(h, w)) / levels * 1.2 - 0.2).astype(np.float32)


# (w, h, tw, th): map sizes against template sizes covering every residue layout of both block grids
SHAPES = [(24, 18, 3, 3), (24, 18, 4, 3), (25, 18, 4, 3), (24, 19, 4, 3), (25, 19, 4, 3), (23, 17, 5, 4),
          (12, 8, 3, 2), (7, 5, 4, 3), (5, 9, 3, 5), (16, 12, 4, 3), (17, 12, 4, 3), (16, 13, 4, 3)]


@pytest.mark.parametrize("w,h,tw,th", SHAPES)
@pytest.mark.parametrize("mfc,by_block", [(0, 1), (1, 1), (0, 0)])
def test_peak_sequence_matches_reference_restatement(w, h, tw, th, mfc, by_block):
    for seed, levels, overlap, thr in itertools.product(range(3), (7, 1000), (0.0, 0.3), (-2.0, 0.25)):
        m = _map(w, h, seed * 31 + w * 7 + h, levels)
        exp = reference_sequence(m, tw, th, by_block, mfc, overlap, 12, thr)
        got = oracle_sequence(m, tw, th, by_block, mfc, overlap, 12, thr)
        assert got == exp, (w, h, tw, th, mfc, by_block, seed, levels, overlap, thr)


def test_mfc_empty_bottom_strip_is_reported_as_reference():
    """No residue at all (24 x 12 map, 2 x (3 x 3) blocks): the MFC 'else' branch adds a zero-height bottom strip whose
    minMaxLoc is 0 at (-1, -1), shifted by the strip's origin to (-1, 11); with every real block painted below 0 the
    last-maximum rule then returns that strip's (0, (-1, 11)) -- kept as the reference would."""
    m = np.full((12, 24), -0.5, np.float32)
    m[3, 4] = 0.9
    exp = reference_sequence(m, 3, 3, 1, 1, 0.0, 3, -2.0)
    assert exp[0] == (pytest.approx(0.9, abs=1e-6), 4, 3)
    assert (exp[1][0], exp[1][1], exp[1][2]) == (0.0, -1, 11)
    assert oracle_sequence(m, 3, 3, 1, 1, 0.0, 3, -2.0) == exp
