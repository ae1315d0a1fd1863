"""Generates tests/golden/reference_pins.json and copies the reference's test images into tests/golden/ref/.

The pins are the reference's own published results (README.md:62-71 "Performance Tests", screenshots under
"Result Images/"): for each test the source/template pair shipped in "Test Images/", the parameters, the number of
detections the screenshot labels, the centre crosses (green '+', display coordinates) found in the screenshot by
a strict 11x11 cross detector (crosses hidden under label text are simply not listed), and the index label the
tool drew on every box, transcribed by hand from the screenshot (``labels``: [index, x, y] with x, y the display
position of that box's centre cross, read off the image; ``inferred`` lists labels clipped by the view's top edge
whose value follows from the other labels of their column).  The screenshot is a scaled (and for Result3 slightly
cropped) view, so the tests fit a per-axis scale + offset between the crosses and the searched centres.

What the labels mean.  The MFC tool numbers its results in list order and draws the number at the midpoint of the
box's top edge (MatchTool/MatchToolDlg.cpp:378-379).  Two tool versions made these screenshots:
  * ``order: "score"`` -- the shipped code: results sorted by score, best first (MatchToolDlg.cpp:1071);
    Result6 and Result8.  The labels are then the score ranking of the detections.
  * ``order: "pos_x"`` -- an older build that re-sorted the list by centre x (the call left commented out at
    MatchToolDlg.cpp:1118, compareMatchResultByPosX :44); Result3 and Result4, whose labels run by column / around
    the ring by x.  The labels then say: centre x is non-decreasing in label order.

Parameters.  ``published`` holds what README.md states for the test (null where it states nothing), ``params``
what the pin runs, and ``fitted`` names every parameter of ``params`` that is NOT published and was chosen by
running the oracle on the pair -- such a pin's count is fitted, not an independent check:
  Result3.jpg = Src3/Dst3, README Test4 parameters (TargetNum 38, Score 0.8, Tol 0, MRA 256): 36 detections;
  Result8.jpg = Src9/Dst9 (the README pairs Test1 with Result8; Src8.bmp is a different scene): README Test1 says
      TargetNum 5, Overlap 0.8, Score 0.8, Tol 180, but the screenshot's four detections score 0.999 / 0.764 /
      0.764 / 0.703 in the oracle, so at Score 0.8 it returns one (``count_at_published``); the pin runs Score 0.7
      (fitted);
  Result4.jpg = Src4/Dst4 (Test5, parameters not published): Tol 180, TargetNum 30, Score 0.7 (all fitted): 24;
  Result6.jpg = Src6/Dst6, README Test6 parameters: 15 detections;
  Result7.jpg = Src8/Dst8 (not in the README table; the view shows the Src8 scene: the gear top left, two
      overlapping E-clips top right, one clip bottom left; the template is the 200x200 clip Dst8): 3 detections,
      score order.  Its parameters are unpublished (all fitted); the values chosen are README Test1's (TargetNum 5,
      Overlap 0.8, Score 0.8, Tol 180), which reproduce the count.  It is the one shipped output whose result depends
      on filterWithRotatedRect KEEPING an overlapping pair (TemplateMatcher.cpp:1133-1194; MatchToolDlg.cpp:1071):
      the two right-hand boxes overlap by between 0.3 and 0.4 of the box area, so MaxOverlap <= 0.3 deletes label 2
      (``overlap_count``).  Its third cross is drawn with the vertical bar one column left of the box's middle
      column, so this pin reads crosses by their strongest row / column (``cross_bars``).
Result1/2/9 have no source image in the reference (Src1/2/10 are missing large blobs; Result9's scene is absent).

Run from the repo root with the reference at /root/reference (this container only); the outputs are committed.
"""
import json
import os
import shutil

import numpy as np
from PIL import Image
from scipy import ndimage

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _grid(xs, ys, cols):
    """labels of a grid given column by column (top to bottom) -> [[label, x, y], ...]"""
    return [[lab, x, y] for x, col in zip(xs, cols) for y, lab in zip(ys, col)]


PINS = [
    dict(name="test4_src3", screenshot="Result3.jpg", source="Src3.bmp", template="Dst3.bmp", count=36,
         params=dict(max_pos=38, score=0.8, tolerance_angle=0.0, min_reduce_area=256),
         published=dict(max_pos=38, score=0.8, tolerance_angle=0.0, min_reduce_area=256), fitted=[],
         order="pos_x",
         labels=_grid([182, 371, 556, 746], [37, 104, 171, 238, 305, 372, 439, 506, 573],
                      [[5, 2, 1, 0, 3, 7, 4, 8, 6], [9, 11, 13, 10, 14, 12, 16, 15, 17],
                       [20, 18, 19, 22, 21, 24, 23, 26, 25], [28, 31, 27, 30, 29, 33, 32, 34, 35]]),
         inferred=[5, 9, 20, 28]),
    dict(name="test1_src9", screenshot="Result8.jpg", source="Src9.bmp", template="Dst9.bmp", count=4,
         params=dict(max_pos=5, max_overlap=0.8, score=0.7, tolerance_angle=180.0),
         published=dict(max_pos=5, max_overlap=0.8, score=0.8, tolerance_angle=180.0), fitted=["score"],
         count_at_published=1, order="score",
         labels=[[0, 176, 145], [1, 267, 399], [2, 291, 490], [3, 598, 243]], inferred=[]),
    dict(name="test5_src4", screenshot="Result4.jpg", source="Src4.bmp", template="Dst4.bmp", count=24,
         params=dict(max_pos=30, score=0.7, tolerance_angle=180.0), published=None,
         fitted=["max_pos", "score", "tolerance_angle"], order="pos_x",
         labels=[[0, 65, 314], [1, 70, 383], [2, 75, 248], [3, 92, 445], [4, 104, 187], [5, 128, 500],
                 [6, 150, 136], [7, 180, 544], [8, 205, 98], [9, 241, 574], [10, 268, 76], [11, 307, 585],
                 [12, 336, 72], [13, 373, 581], [14, 401, 84], [15, 437, 561], [16, 463, 113], [17, 491, 521],
                 [18, 515, 157], [19, 538, 471], [20, 552, 213], [21, 566, 411], [22, 574, 280], [23, 579, 346]],
         inferred=[]),
    dict(name="test6_src6", screenshot="Result6.jpg", source="Src6.jpg", template="Dst6.bmp", count=15,
         params=dict(max_pos=15, score=0.8, tolerance_angle=180.0, min_reduce_area=256),
         published=dict(max_pos=15, score=0.8, tolerance_angle=180.0, min_reduce_area=256), fitted=[],
         order="score",
         labels=_grid([167, 326, 476], [107, 183, 258, 333, 408],
                      [[2, 0, 1, 3, 7], [13, 12, 11, 6, 4], [5, 8, 9, 10, 14]]),
         inferred=[],
         # the decoder-level perturbation tests/test_reference_pins.py pins (+-1 LSB on `frac` of the pixels, chosen
         # by a hash of index + salt): FITTED -- salt 2 is one of the salts that reproduce the screenshot's full
         # order; the rate over salts 0..31 (scripts/result6_sensitivity.py, profiles/r03/result6_sensitivity.txt)
         # is what it shows, not the salt itself
         perturbation=dict(salt=2, frac=0.01, fitted=True,
                           full_order_rate={"0.003": "6/32", "0.01": "10/32", "0.03": "20/32"})),
    dict(name="result7_src8", screenshot="Result7.jpg", source="Src8.bmp", template="Dst8.bmp", count=3,
         params=dict(max_pos=5, max_overlap=0.8, score=0.8, tolerance_angle=180.0), published=None,
         fitted=["max_overlap", "max_pos", "score", "tolerance_angle"], order="score",
         labels=[[0, 222, 459], [1, 470, 226], [2, 614, 263]], inferred=[], cross_bars=True,
         # detections at MaxOverlap 0.3 / 0.4 (the oracle; everything else as ``params``): the overlapping pair
         # is kept only above its overlap ratio
         overlap_count={"0.3": 2, "0.4": 3}),
]


def crosses(path, bars=False):
    """centre crosses of a screenshot; ``bars``: test the strongest row / column instead of the middle ones"""
    im = np.asarray(Image.open(path).convert("RGB")).astype(int)
    r, g, b = im[..., 0], im[..., 1], im[..., 2]
    lab, _ = ndimage.label((g > 150) & (r < 120) & (b < 120))
    out = []
    for i, sl in enumerate(ndimage.find_objects(lab)):
        h, w = sl[0].stop - sl[0].start, sl[1].stop - sl[1].start
        m = lab[sl] == i + 1
        row, col = (m.sum(axis=1).max(), m.sum(axis=0).max()) if bars else (m[h // 2, :].sum(), m[:, w // 2].sum())
        if 10 <= h <= 13 and 10 <= w <= 13 and row >= w - 2 and col >= h - 2 and m.sum() <= 3 * (w + h):
            ys, xs = np.nonzero(m)
            out.append([round(float(sl[1].start + xs.mean()), 2), round(float(sl[0].start + ys.mean()), 2)])
    return [im.shape[1], im.shape[0]], sorted(out)


def main():
    os.makedirs(os.path.join(OUT, "ref"), exist_ok=True)
    for p in PINS:
        assert sorted(lab for lab, _, _ in p["labels"]) == list(range(p["count"])), p["name"]
        for f in (p["source"], p["template"]):
            dst = os.path.join(OUT, "ref", f)
            if f == "Src6.jpg":
                continue   # already committed as tests/golden/Src6.jpg
            shutil.copyfile(os.path.join(REF, "Test Images", f), dst)
        p["display"], p["crosses"] = crosses(os.path.join(REF, "Result Images", p["screenshot"]),
                                             p.get("cross_bars", False))
    with open(os.path.join(OUT, "reference_pins.json"), "w") as fh:
        json.dump(PINS, fh, indent=1)


if __name__ == "__main__":
    main()
