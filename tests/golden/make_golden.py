"""Generate tests/golden/golden.npz: small seeded inputs and the oracle's expected outputs.

Run from the repo root after `make -C oracle`:  python tests/golden/make_golden.py
The inputs are stored (not regenerated from seeds) so the fixtures are self-contained; every case is small
enough for the oracle to finish in well under a second.  The same fixtures pin the oracle against regressions
(tests/test_oracle_golden.py, CPU) and the HIP path against the oracle (tests/test_gpu_golden.py, GPU).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from fastest_image_pattern_matching_amd import synth  # noqa: E402
from tests import oracle  # noqa: E402

PARAM_KEYS = ("max_pos", "min_reduce_area", "max_overlap", "score", "tolerance_angle", "use_simd", "subpixel",
              "tolerance_range")


def scene(tm, name, poses, size, seed, bg=(128, 10)):
    t = tm[name]
    s = synth.noise(size[0], size[1], bg[0], bg[1], seed)
    for cx, cy, ang in poses:
        synth.paste_rotated(s, t, cx, cy, ang)
    return s, t


def cases(tm):
    yield "g_dst10_rot", *scene(tm, "Dst10", [(80, 70, 25.0), (200, 150, -140.0)], (300, 240), 31), \
        dict(max_pos=3, tolerance_angle=180.0)
    yield "g_dst4_tol0", *scene(tm, "Dst4", [(40, 30, 0.0), (120, 90, 0.0), (200, 40, 0.0)], (260, 140), 32), \
        dict(max_pos=5, tolerance_angle=0.0)
    yield "g_dst3_sub", *scene(tm, "Dst3", [(120, 110, 61.0)], (260, 230), 33), \
        dict(max_pos=1, tolerance_angle=90.0, subpixel=1)
    yield "g_dst9_nosimd", *scene(tm, "Dst9", [(150, 140, -15.0)], (320, 300), 34), \
        dict(max_pos=2, tolerance_angle=30.0, use_simd=0)
    # s_BlockMax path: (top source area / top template area) = (450*350)/(17*9) > 500 and MaxPos > 10
    yy, xx = np.mgrid[0:700, 0:900]
    s = (((xx // 3 + yy // 5) % 64) + 96).astype(np.uint8)
    for y in range(8, 680, 31):
        for x in range(8, 860, 47):
            synth.paste(s, tm["Dst4"], x, y)
    yield "g_dst4_block", s, tm["Dst4"], dict(max_pos=60, tolerance_angle=0.0)


def main():
    tm = synth.load_templates()
    out = {}
    names = []
    for name, s, t, prm in cases(tm):
        o = oracle.OracleMatcher()
        for k, v in prm.items():
            setattr(o.params, k, v)
        o.learnPattern(t)
        res = o.match(s)
        out[f"{name}__src"] = s
        out[f"{name}__tmpl"] = t
        out[f"{name}__params"] = np.array([float(getattr(o.params, k)) for k in PARAM_KEYS])
        out[f"{name}__results"] = np.array(res, np.float64).reshape(-1, 12)
        out[f"{name}__stats"] = np.array(o.stats(), np.int64)
        out[f"{name}__top"] = o.top_candidates()
        names.append(name)
        print(name, s.shape, t.shape, len(res), o.stats())
    # primitive vectors
    rng = np.random.default_rng(2025)
    img = rng.integers(0, 256, (29, 37), dtype=np.uint8)
    out["p_pyr__in"] = img
    out["p_pyr__out"] = oracle.pyr_down(img)
    m = oracle.rotation_matrix(17.3, 11.9, 33.7)
    m[:, 2] += (2.25, -1.5)
    out["p_warp__in"] = img
    out["p_warp__m"] = m
    out["p_warp__out"] = oracle.warp_affine(img, m, (41, 35), 77)
    t = tm["Dst10"]
    o = oracle.OracleMatcher().set(min_reduce_area=4096)
    o.learnPattern(t)
    src = synth.noise(70, 66, 128, 30, 36)
    src[6:60, 9:63] = t
    out["p_ncc__in"] = src
    out["p_ncc__tmpl"] = t
    out["p_ncc__fold"] = o.ncc_map(src, 0, True)
    out["p_ncc__ccorr"] = o.ncc_map(src, 0, False)
    out["cases"] = np.array(names)
    np.savez_compressed(os.path.join(HERE, "golden.npz"), **out)
    print("wrote", os.path.join(HERE, "golden.npz"))


if __name__ == "__main__":
    main()
