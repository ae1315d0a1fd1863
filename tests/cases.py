"""Search cases shared by the GPU parity tests and the CPU merge / sharding tests (seeded synthetic scenes)."""
from fastest_image_pattern_matching_amd import synth
from tests import oracle


def _scene_rotated(templates, name, poses, size, seed, bg=(128, 10)):
    t = templates[name]
    s = synth.noise(size[0], size[1], bg[0], bg[1], seed)
    for cx, cy, ang in poses:
        synth.paste_rotated(s, t, cx, cy, ang)
    return s, t


def _run_both(hip, s, t, **prm):
    o = oracle.OracleMatcher()
    hip.resetParams()
    for k, v in prm.items():
        setattr(o.params, k, v)
        setattr(hip._params, k, v)
    assert o.learnPattern(t) and hip.learnPattern(t)
    orc = o.match(s)
    gpu = hip.match(s)
    return gpu, orc, o.stats(), hip.search_stats()


CASES = {
    "plumbing_tol0": (lambda T: synth.plumbing_scene(T["Dst1"]), dict(max_pos=1)),
    "dst1_rot30": (lambda T: _scene_rotated(T, "Dst1", [(640, 512, 30.0)], (1280, 1024), 1),
                   dict(max_pos=1, tolerance_angle=180.0)),
    "dst10_multi": (lambda T: _scene_rotated(T, "Dst10", [(100, 90, 37.0), (300, 250, -100.0), (420, 120, 170.0)],
                                             (560, 400), 2), dict(max_pos=5, tolerance_angle=180.0)),
    "dst10_nosimd": (lambda T: _scene_rotated(T, "Dst10", [(100, 90, 37.0), (300, 250, -100.0)], (560, 400), 3),
                     dict(max_pos=5, tolerance_angle=180.0, use_simd=0)),
    "dst5_subpixel": (lambda T: _scene_rotated(T, "Dst5", [(200, 180, 44.3)], (420, 380), 4, (60, 10)),
                      dict(max_pos=1, tolerance_angle=180.0, subpixel=1)),
    "dst4_block": (lambda T: _grid_scene(T["Dst4"], 900, 900, 60, 5), dict(max_pos=40, tolerance_angle=0.0)),
    "dst4_overlap": (lambda T: _grid_scene(T["Dst4"], 400, 300, 20, 6),
                     dict(max_pos=30, tolerance_angle=10.0, max_overlap=0.5, score=0.6)),
    "dst3_range": (lambda T: _scene_rotated(T, "Dst3", [(150, 150, 12.0), (400, 260, -33.0)], (560, 420), 7),
                   dict(max_pos=4, tolerance_angle=40.0, tolerance_range=1)),
    "top_is_layer0": (lambda T: _scene_rotated(T, "Dst4", [(60, 50, 0.0), (150, 80, 0.0)], (220, 160), 8),
                      dict(max_pos=3, min_reduce_area=1024)),
    "score_low_many": (lambda T: _scene_rotated(T, "Dst9", [(200, 200, 5.0), (500, 300, 95.0)], (700, 520), 9),
                       dict(max_pos=10, tolerance_angle=180.0, score=0.5)),
}


def _grid_scene(t, w, h, pitch, seed):
    s = synth.box_blur(synth.noise(w, h, 128, 25, seed), 3)
    th, tw = t.shape
    for y in range(10, h - th - 10, pitch):
        for x in range(10, w - tw - 10, pitch + 7):
            synth.paste(s, t, x, y)
    return s, t
