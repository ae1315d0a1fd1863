"""Seeded randomized parity sweep: random template crops (odd/even/skinny sizes), random sources with rotated and
partially off-image copies, random search parameters (angle tolerance, MaxPos, overlap, score, SIMD fold,
sub-pixel, MinReduceArea) — every result field bit-identical to the oracle restatement and identical per-layer
live-candidate counts.  Sizes are small so the CPU oracle stays in milliseconds per case."""
import numpy as np
import pytest

from fastest_image_pattern_matching_amd import synth
from tests import oracle
from tests.test_gpu_parity import assert_same_results

pytestmark = pytest.mark.gpu

N_CASES = 150


def _case(seed):
    rng = np.random.default_rng(1000 + seed)
    T = synth.load_templates()
    name = sorted(T)[int(rng.integers(0, len(T)))]
    full = T[name]
    # a random crop of a reference template: odd, even, skinny and square shapes
    big = seed % 5 == 0     # every fifth case: larger template and source (more pyramid layers)
    th = int(rng.integers(9, min(full.shape[0], 200 if big else 90) + 1))
    tw = int(rng.integers(9, min(full.shape[1], 260 if big else 120) + 1))
    y0 = int(rng.integers(0, full.shape[0] - th + 1))
    x0 = int(rng.integers(0, full.shape[1] - tw + 1))
    t = np.ascontiguousarray(full[y0:y0 + th, x0:x0 + tw])
    W = int(rng.integers(max(tw, th) + 20, 900 if big else 420))
    H = int(rng.integers(max(tw, th) + 20, 700 if big else 360))
    s = synth.box_blur(synth.noise(W, H, float(rng.integers(40, 200)), float(rng.integers(3, 30)), seed), 3)
    for _ in range(int(rng.integers(1, 4))):
        cx = float(rng.uniform(-0.2 * tw, W + 0.2 * tw))     # may hang over the border
        cy = float(rng.uniform(-0.2 * th, H + 0.2 * th))
        synth.paste_rotated(s, t, cx, cy, float(rng.uniform(-180, 180)))
    prm = dict(
        max_pos=int(rng.integers(1, 12)),
        tolerance_angle=float(rng.choice([0.0, 15.0, 90.0, 180.0])),
        score=float(rng.choice([0.5, 0.6, 0.7, 0.8])),
        max_overlap=float(rng.choice([0.0, 0.0, 0.3, 0.8])),
        use_simd=int(rng.integers(0, 2)),
        subpixel=int(rng.integers(0, 2)),
        min_reduce_area=int(rng.choice([64, 256, 256, 1024])),
        tolerance_range=int(rng.random() < 0.1),
    )
    return s, t, prm


@pytest.mark.parametrize("seed", range(N_CASES))
def test_fuzz_parity(gpu_matcher_factory, seed):
    s, t, prm = _case(seed)
    o = oracle.OracleMatcher().set(**prm)
    assert o.learnPattern(t)
    m = gpu_matcher_factory(**prm)
    assert m.learnPattern(t)
    orc = o.match(s)
    gpu = m.match(s)
    assert m.search_stats() == o.stats(), (seed, prm)
    assert_same_results(gpu, orc, f"fuzz{seed} {prm} t={t.shape} s={s.shape}")
