"""Seeded synthetic scenes for the BASELINE.json configs.

The reference's large sources (Src1/Src7/Src10/Src5-*) are missing from its repository, so every config is
re-created from the templates it does ship (tests/golden/templates.npz, decoded with IMREAD_GRAYSCALE
semantics by tests/golden/make_templates.py) pasted into seeded backgrounds.  Rotated copies use bilinear
sampling in float64; the matcher under test never sees how a scene was made.
"""
from __future__ import annotations

import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TEMPLATES = os.path.join(REPO, "tests", "golden", "templates.npz")

# README.md:45-49 known answers for Src7 (MFC build): score, angle (MFC sign), centre x, centre y
SRC7_POSES = [(1.0, 0.046, 1725.857, 1045.433), (0.998, -119.979, 2662.869, 1537.446),
              (0.991, 120.150, 1768.936, 2098.494)]


def load_templates() -> dict:
    with np.load(TEMPLATES) as z:
        return {k: z[k] for k in z.files}


def noise(w: int, h: int, mean: float, sigma: float, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    return np.clip(np.rint(mean + rng.normal(0.0, sigma, (h, w))), 0, 255).astype(np.uint8)


def box_blur(img: np.ndarray, k: int) -> np.ndarray:
    a = img.astype(np.float64)
    pad = k // 2
    p = np.pad(a, pad, mode="reflect")
    c = p.cumsum(0).cumsum(1)
    c = np.pad(c, ((1, 0), (1, 0)))
    s = c[k:, k:] - c[:-k, k:] - c[k:, :-k] + c[:-k, :-k]
    return np.clip(np.rint(s / (k * k)), 0, 255).astype(np.uint8)


def paste(dst: np.ndarray, tmpl: np.ndarray, x: int, y: int) -> None:
    h, w = tmpl.shape
    dst[y:y + h, x:x + w] = tmpl


def paste_rotated(dst: np.ndarray, tmpl: np.ndarray, cx: float, cy: float, angle: float) -> None:
    """Paste ``tmpl`` centred at (cx, cy), turned so that the matcher reports dMatchedAngle ~= ``angle``
    (Qt sign convention, TemplateMatcher.cpp:428: the template appears rotated clockwise on screen)."""
    h, w = tmpl.shape
    t = np.deg2rad(angle)
    c, s = np.cos(t), np.sin(t)
    r = 0.5 * np.hypot(w, h) + 2
    x0, x1 = int(max(np.floor(cx - r), 0)), int(min(np.ceil(cx + r), dst.shape[1] - 1))
    y0, y1 = int(max(np.floor(cy - r), 0)), int(min(np.ceil(cy + r), dst.shape[0] - 1))
    ys, xs = np.mgrid[y0:y1 + 1, x0:x1 + 1].astype(np.float64)
    dx, dy = xs - cx, ys - cy
    # inverse of a clockwise-on-screen rotation (y down): u = R(-t) d
    u = c * dx + s * dy + (w - 1) / 2.0
    v = -s * dx + c * dy + (h - 1) / 2.0
    inside = (u >= 0) & (u <= w - 1) & (v >= 0) & (v <= h - 1)
    u0 = np.clip(np.floor(u).astype(np.int64), 0, w - 1)
    v0 = np.clip(np.floor(v).astype(np.int64), 0, h - 1)
    u1 = np.clip(u0 + 1, 0, w - 1)
    v1 = np.clip(v0 + 1, 0, h - 1)
    fu, fv = u - u0, v - v0
    T = tmpl.astype(np.float64)
    val = (T[v0, u0] * (1 - fu) * (1 - fv) + T[v0, u1] * fu * (1 - fv) + T[v1, u0] * (1 - fu) * fv +
           T[v1, u1] * fu * fv)
    region = dst[y0:y1 + 1, x0:x1 + 1]
    region[inside] = np.clip(np.rint(val[inside]), 0, 255).astype(np.uint8)


# ---- BASELINE.json configs ------------------------------------------------------------------------------
def plumbing_scene(t=None):
    """configs[0] surrogate: Dst1 at (400, 300) in 1280x1024, background 128 + N(0, 3), seed 1."""
    t = load_templates()["Dst1"] if t is None else t
    s = noise(1280, 1024, 128, 3, 1)
    paste(s, t, 400, 300)
    return s, t


def src7_scene(t=None, w: int = 4024, h: int = 3036, seed: int = 7):
    """configs[1] surrogate: 4024x3036, background 235 + N(0, 2), three Dst7 copies at the README poses
    (angles sign-flipped to the Qt convention)."""
    t = load_templates()["Dst7"] if t is None else t
    s = noise(w, h, 235, 2, seed)
    for _, ang, cx, cy in SRC7_POSES:
        paste_rotated(s, t, cx * w / 4024.0, cy * h / 3036.0, -ang)
    return s, t


def src10_scene(t=None, seed: int = 10):
    """configs[2] surrogate: 3648x3648 box-blurred N(128, 20), Dst10 at 144 jittered grid sites."""
    t = load_templates()["Dst10"] if t is None else t
    s = box_blur(noise(3648, 3648, 128, 20, seed), 3)
    rng = np.random.default_rng(seed + 1)
    for gy in range(12):
        for gx in range(12):
            x = 150 + gx * 300 + int(rng.integers(-20, 21))
            y = 150 + gy * 300 + int(rng.integers(-20, 21))
            paste(s, t, x, y)
    return s, t


def batch_sources(n: int, size: int = 4096, tsize: int = 512, seed0: int = 1000, first: int = 0):
    """configs[3]: n box-blurred uniform sources; the template is the tsize crop of source 0 at the centre,
    re-pasted into every source at a seeded angle and position.  ``first``: the sources first .. first + n - 1 of
    the same sequence (one rank's shard: every source depends only on its index)."""
    base = box_blur(np.random.default_rng(seed0).integers(0, 256, (size, size), dtype=np.uint8), 5)
    c0 = (size - tsize) // 2
    t = base[c0:c0 + tsize, c0:c0 + tsize].copy()
    out = []
    for i in range(first, first + n):
        s = base.copy() if i == 0 else box_blur(
            np.random.default_rng(seed0 + i).integers(0, 256, (size, size), dtype=np.uint8), 5)
        rng = np.random.default_rng(seed0 + 10_000 + i)
        ang = float(rng.uniform(-180, 180))
        cx = float(rng.uniform(tsize, size - tsize))
        cy = float(rng.uniform(tsize, size - tsize))
        paste_rotated(s, t, cx, cy, ang)
        out.append(s)
    return out, t


def src5_set(t=None, seed: int = 5):
    """configs[4] surrogate: Dst5 at the centre of a 640x480 N(60, 10) base, rotated by 0, 45, ..., 315."""
    t = load_templates()["Dst5"] if t is None else t
    base = noise(640, 480, 60, 10, seed)
    out = []
    for k in range(8):
        s = base.copy()
        paste_rotated(s, t, 319.5, 239.5, -45.0 * k)
        out.append(s)
    return out, t
