"""HIP path vs the CPU oracle on the same seeded inputs, through the C ABI (gfx950 required).

Bar: bit-exact pixels / maps / positions / angles; scores within 1e-5 (BASELINE.json north_star) — the design
makes them bit-identical, and the tests assert the exact equality they claim.
"""
import numpy as np
import pytest

from fastest_image_pattern_matching_amd import synth
from fastest_image_pattern_matching_amd.matcher import SingleTargetMatch
from tests import oracle
from tests.cases import CASES, _grid_scene, _run_both, _scene_rotated  # noqa: F401

pytestmark = pytest.mark.gpu

FIELDS = ("lt_x", "lt_y", "rt_x", "rt_y", "rb_x", "rb_y", "lb_x", "lb_y", "cx", "cy", "angle", "score")


@pytest.fixture(scope="module")
def hip(gpu_matcher_factory):
    return gpu_matcher_factory()


def assert_same_results(gpu, orc, label=""):
    g = [r.as_tuple() for r in gpu]
    assert len(g) == len(orc), f"{label}: {len(g)} GPU results vs {len(orc)} oracle results\n{g}\n{orc}"
    for i, (a, b) in enumerate(zip(g, orc)):
        for f, x, y in zip(FIELDS, a, b):
            if f == "score":
                assert abs(x - y) <= 1e-5, (label, i, f, x, y)
            assert x == y, f"{label}: result {i} field {f}: gpu {x!r} oracle {y!r}"


# ---------------------------------------------------------------------------------------------------- K1
@pytest.mark.parametrize("shape", [(2, 2), (3, 5), (7, 130), (68, 136), (69, 137), (100, 333), (521, 762),
                                   (1518, 2012), (3036, 4024)])
def test_pyr_down(hip, shape):
    rng = np.random.default_rng(shape[0] * 7 + shape[1])
    img = rng.integers(0, 256, shape, dtype=np.uint8)
    assert np.array_equal(hip.pyr_down(img), oracle.pyr_down(img))


@pytest.mark.parametrize("shape", [(1, 1), (2, 2), (3, 5), (5, 3), (7, 130), (9, 257), (68, 136), (69, 137),
                                   (127, 255), (128, 256), (129, 258), (130, 514), (100, 333), (521, 762),
                                   (1518, 2012), (3036, 4024)])
@pytest.mark.parametrize("seg", [0, 1, 2, 3])
@pytest.mark.parametrize("rows", [0, 16, 32])
def test_pyr_down2(hip, shape, seg, rows):
    """Two levels in one launch (k_pyr_down2) = two oracle pyrDowns: strip edges at both levels (widths around the
    64-column level-2 strip), odd and tiny sizes, runs starting mid-image (seg 1-3 chunks per workgroup), with the
    level-1 chunk height the search would choose (rows 0: 16 for most single images) and each height forced, so the
    ring carry at a run start is pinned for both 16- and 32-row chunks on every shape."""
    rng = np.random.default_rng(shape[0] * 11 + shape[1] + seg)
    img = rng.integers(0, 256, shape, dtype=np.uint8)
    b, c = hip.pyr_down2(img, seg, rows)
    ob = oracle.pyr_down(img)
    assert np.array_equal(b, ob)
    assert np.array_equal(c, oracle.pyr_down(ob))


def test_pyr_down_strided_input(hip):
    img = np.random.default_rng(9).integers(0, 256, (300, 500), dtype=np.uint8)[10:250, 3:411]
    assert np.array_equal(hip.pyr_down(img), oracle.pyr_down(np.ascontiguousarray(img)))


# ---------------------------------------------------------------------------------------------------- K2
@pytest.mark.parametrize("seed", range(8))
def test_warp_affine(hip, seed):
    rng = np.random.default_rng(100 + seed)
    h, w = int(rng.integers(5, 200)), int(rng.integers(5, 200))
    img = rng.integers(0, 256, (h, w), dtype=np.uint8)
    ang = float(rng.uniform(-200, 200))
    m = oracle.rotation_matrix(float(rng.uniform(0, w)), float(rng.uniform(0, h)), ang)
    m[:, 2] += rng.uniform(-20, 20, 2)
    dw, dh = int(rng.integers(1, 260)), int(rng.integers(1, 260))
    border = int(rng.integers(0, 256))
    assert np.array_equal(hip.warp_affine(img, m, (dw, dh), border), oracle.warp_affine(img, m, (dw, dh), border))


# ---------------------------------------------------------------------------------------------------- learn
@pytest.mark.parametrize("name,mra", [("Dst1", 256), ("Dst7", 256), ("Dst10", 256), ("Dst4", 64), ("Dst6", 1024)])
def test_learn_pattern(hip, templates, name, mra):
    t = templates[name]
    hip.setMinReduceArea(mra)
    assert hip.learnPattern(t)
    o = oracle.OracleMatcher().set(min_reduce_area=mra)
    o.learnPattern(t)
    levels, border = o.template_levels()
    assert hip.template_info() == (len(levels), border)
    for i, (px, mean, norm, inv, eq) in enumerate(levels):
        gp, gm, gn, gi, ge = hip.template_level(i)
        assert np.array_equal(gp, px) and (gm, gn, gi, ge) == (mean, norm, inv, eq)
    hip.setMinReduceArea(256)


# ---------------------------------------------------------------------------------------------------- K3+K4
@pytest.mark.parametrize("fold", [False, True])
def test_ncc_map_all_layers(hip, templates, fold):
    t = templates["Dst1"]
    hip.setMinReduceArea(256)
    hip.learnPattern(t)
    o = oracle.OracleMatcher()
    o.learnPattern(t)
    rng = np.random.default_rng(42)
    levels, _ = o.template_levels()
    for layer, (px, *_rest) in enumerate(levels):
        th, tw = px.shape
        img = rng.integers(0, 256, (th + 13, tw + 9), dtype=np.uint8)
        img[5:5 + th, 3:3 + tw] = px
        assert np.array_equal(hip.ncc_map(img, layer, fold), o.ncc_map(img, layer, fold)), layer


@pytest.mark.parametrize("shape", [(48, 63), (150, 200), (77, 131)])
def test_ncc_map_tiled_multi_tile(hip, templates, shape):
    """The LDS-tiled top-layer NCC over maps spanning several (and partial) 64 x 16 tiles, TM_CCORR and fold."""
    t = templates["Dst7"]
    hip.setMinReduceArea(256)
    hip.learnPattern(t)
    o = oracle.OracleMatcher()
    o.learnPattern(t)
    levels, _ = o.template_levels()
    top = len(levels) - 1
    rng = np.random.default_rng(shape[0] * 7 + shape[1])
    img = rng.integers(0, 256, shape, dtype=np.uint8)
    img[10:10 + levels[top][0].shape[0], 20:20 + levels[top][0].shape[1]] = levels[top][0]
    for fold in (False, True):
        assert np.array_equal(hip.ncc_map(img, top, fold), o.ncc_map(img, top, fold)), (shape, fold)


# ---------------------------------------------------------------------------------------------------- search
@pytest.mark.parametrize("case", sorted(CASES))
def test_match_parity(hip, templates, case):
    make, prm = CASES[case]
    s, t = make(templates)
    gpu, orc, ostats, gstats = _run_both(hip, s, t, **prm)
    assert gstats == ostats, (gstats, ostats)
    assert_same_results(gpu, orc, case)
    assert len(orc) >= 1


def test_src7_full_search(hip, templates):
    """BASELINE configs[1] at full size: 4024x3036 / 762x521, +-180 deg, TargetNum 3."""
    s, t = synth.src7_scene(templates["Dst7"])
    gpu, orc, ostats, gstats = _run_both(hip, s, t, max_pos=3, tolerance_angle=180.0, score=0.7)
    assert gstats == ostats
    assert_same_results(gpu, orc, "src7")
    assert len(gpu) == 3


def test_wide_template_slot_major_correlation(gpu_matcher_factory):
    """A template wider than 1024 px (18 k-steps of 64 bytes): layer 0's correlation runs the slot-major
    k_roi_corr form (the register-A form holds at most 16 k-steps) -- every result field and live count equal the
    oracle's."""
    t = synth.box_blur(synth.noise(1100, 300, 128, 50, 61), 3)
    s = synth.box_blur(synth.noise(2600, 1400, 128, 50, 62), 3)
    synth.paste_rotated(s, t, 1300.0, 420.0, 4.0)
    synth.paste_rotated(s, t, 1290.0, 1000.0, -7.0)
    m = gpu_matcher_factory()
    gpu, orc, ostats, gstats = _run_both(m, s, t, max_pos=2, tolerance_angle=10.0, score=0.6)
    assert gstats == ostats
    assert_same_results(gpu, orc, "wide template")
    assert len(gpu) == 2


@pytest.mark.parametrize("top_fused", ["0", "1"])
def test_src7_top_layer_forms(gpu_matcher_factory, templates, monkeypatch, top_fused):
    """The top layer as one kernel (k_top_fused, FPM_TOP_FUSED=1 forces it below its job-count threshold) and as
    the split k_warp -> k_ncc_tile -> k_nms chain (FPM_TOP_FUSED=0; read when a fresh context records its search) on
    a batch of two Src7 sources and on one alone: both equal the oracle, result fields and per-layer live counts."""
    monkeypatch.setenv("FPM_TOP_FUSED", top_fused)
    t = templates["Dst7"]
    srcs = [synth.src7_scene(t, seed=11 + i)[0] for i in range(2)]
    m = gpu_matcher_factory(max_pos=3, tolerance_angle=180.0, score=0.7)
    assert m.learnPattern(t)
    m.stage(srcs)
    got = [[r.as_tuple() for r in rr] for rr in m.match_staged()]
    o = oracle.OracleMatcher().set(max_pos=3, tolerance_angle=180.0, score=0.7)
    o.learnPattern(t)
    assert got == [o.match(s) for s in srcs]
    gpu, orc, ostats, gstats = _run_both(m, srcs[0], t, max_pos=3, tolerance_angle=180.0, score=0.7)
    assert gstats == ostats
    assert_same_results(gpu, orc, f"src7 top_fused={top_fused}")


@pytest.mark.parametrize("caps", [{}, {"FPM_GRID_TOP": "7", "FPM_GRID_SMALL": "5", "FPM_GRID_WARP": "37",
                                      "FPM_GRID_CORR": "11"},
                                  {"FPM_GRID_TOP": "1000", "FPM_GRID_SMALL": "768", "FPM_GRID_WARP": "1536"},
                                  {"FPM_GRID_SMALL": "0", "FPM_GRID_WARP": "0"},
                                  {"FPM_GRID_CORR": "13"},
                                  {"FPM_SMALL_NT": "256"}, {"FPM_SMALL_NT": "128"}, {"FPM_SMALL_NT": "512"},
                                  {"FPM_SMALL_NT": "128", "FPM_GRID_SMALL": "5"}])
def test_src7_grid_caps(gpu_matcher_factory, templates, monkeypatch, caps):
    """The workgroup caps of the persistent forms (FPM_GRID_TOP / _SMALL / _WARP / _CORR; read when a fresh context
    records its search; {} = the defaults, "0" = uncapped grids; FPM_SMALL_NT=256 / 128 / 512 = four- / two- / eight-wave workgroups for every small-template layer where they
    apply; by default eight-wave ones for batches of at most two sources, two-wave ones for layers with more ROIs than
    the four-wave form holds at once): with tiny
    caps every workgroup of the fused top layer, the small-template refinement, the
    sampler and the correlation loops over many jobs; a batch of seven Src7 sources (fused top layer: >= 256 jobs)
    equals the oracle."""
    for k, v in caps.items():
        monkeypatch.setenv(k, v)
    t = templates["Dst7"]
    srcs = [synth.src7_scene(t, seed=21 + i)[0] for i in range(7)]
    m = gpu_matcher_factory(max_pos=3, tolerance_angle=180.0, score=0.7)
    assert m.learnPattern(t)
    m.stage(srcs)
    got = [[r.as_tuple() for r in rr] for rr in m.match_staged()]
    o = oracle.OracleMatcher().set(max_pos=3, tolerance_angle=180.0, score=0.7)
    o.learnPattern(t)
    assert got == [o.match(s) for s in srcs]


@pytest.mark.parametrize("nt", ["128", "256", "512"])
@pytest.mark.parametrize("shape", ["wide", "tall"])
def test_small_forms_wide_tall_templates(gpu_matcher_factory, templates, monkeypatch, nt, shape):
    """The two- / four- / eight-wave small-template workgroups (FPM_SMALL_NT, forced wherever they apply) and a tight
    correlation grid cap on a wide template (Dst6, 848 x 446) and a tall one (its transpose): every layer's footprint
    region, table and band layout of k_roi_small on shapes other than Src7's; two sources at +-180 equal the oracle."""
    monkeypatch.setenv("FPM_SMALL_NT", nt)
    monkeypatch.setenv("FPM_GRID_CORR", "13")
    t = np.ascontiguousarray(templates["Dst6"] if shape == "wide" else templates["Dst6"].T)
    h, w = (1300, 1700) if shape == "wide" else (1700, 1300)
    srcs = []
    for i in range(2):
        s = synth.noise(w, h, 128, 12, 77 + i)
        synth.paste_rotated(s, t, w * 0.45, h * 0.5, 35.0 - 70.0 * i)
        srcs.append(s)
    kw = dict(max_pos=2, tolerance_angle=180.0, score=0.7)
    m = gpu_matcher_factory(**kw)
    assert m.learnPattern(t)
    m.stage(srcs)
    got = [[r.as_tuple() for r in rr] for rr in m.match_staged()]
    o = oracle.OracleMatcher().set(**kw)
    o.learnPattern(t)
    exp = [o.match(s) for s in srcs]
    assert got == exp
    assert all(len(r) >= 1 for r in exp)


def test_top_fused_lds_threshold(gpu_matcher_factory, templates, monkeypatch):
    """k_top_fused forced (FPM_TOP_FUSED=1) on top canvases either side of its LDS limit (64 KB minus the kernel's
    static LDS, read with hipFuncGetAttributes): Dst10 at +-180 over square sources whose largest rotated top canvas
    needs 56.5 KB (364 px) up to ~67 KB (396 px) of dynamic LDS.  Below the limit the fused kernel runs, above it the
    engine falls back to another top-layer form (the matrix-core or the split one: no fused launch beyond the limit);
    every search equals the oracle."""
    from fastest_image_pattern_matching_amd import _lib as L

    monkeypatch.setenv("FPM_TOP_FUSED", "1")
    t = templates["Dst10"]
    fused = {}
    for size in (364, 372, 376, 380, 388, 396):
        s = synth.noise(size, size, 128, 10, size)
        synth.paste_rotated(s, t, size // 2, size // 2, 30.0)
        m = gpu_matcher_factory(max_pos=3, tolerance_angle=180.0)
        assert m.learnPattern(t)
        m.profile(True)
        m.profile_reset()
        got = [r.as_tuple() for r in m.match(s)]
        # the split form launches k_warp, the matrix-core form its map fallback (top_map)
        fused[size] = all(m.profile_get(L.KERNEL_NAMES.index(k))[1] == 0 for k in ("top_warp", "top_map"))
        m.profile(False)
        o = oracle.OracleMatcher().set(max_pos=3, tolerance_angle=180.0)
        assert o.learnPattern(t)
        assert got == o.match(s), size
    forms = [fused[k] for k in sorted(fused)]
    assert forms[0] and not forms[-1], fused
    assert forms == sorted(forms, reverse=True), fused   # one threshold


@pytest.mark.parametrize("size", [(500, 400), (1000, 900)])
def test_plain_peak_loop_map_sizes(hip, size):
    """The plain getNextMaxLoc loop (MaxPos 10: no s_BlockMax) on one large top map: a 20x20 template is searched at
    level 0 (MinReduceArea 1024: no pyramid), so the maps are 481 x 381 (183 K pixels: the 64-pixel block maxima in LDS, a partial last block) and
    981 x 881 (864 K pixels > 4096 blocks: the full-map scan form); both equal the oracle."""
    w, h = size
    t = synth.box_blur(synth.noise(20, 20, 128, 60, 5), 3)
    s = synth.box_blur(synth.noise(w, h, 128, 40, w), 3)
    for k in range(6):
        synth.paste_rotated(s, t, 40 + (w - 80) * k / 5, 40 + (h - 80) * k / 5, 0.0)
    gpu, orc, ostats, gstats = _run_both(hip, s, t, max_pos=10, tolerance_angle=0.0, score=0.3, min_reduce_area=1024)
    assert gstats == ostats, (gstats, ostats)
    assert_same_results(gpu, orc, f"plain_map_{w}x{h}")
    assert len(orc) == 15


@pytest.mark.parametrize("max_pos", [100, 150])
def test_plain_peaks_many(hip, templates, max_pos):
    """Plain getNextMaxLoc path (top map / template area <= 500) with ~80 peaks per map: MaxPos 100 (cap 105) runs the
    candidate init inside k_nms from its LDS peak list, MaxPos 150 (cap 155 > kNmsInitCap) the separate
    k_cand_init; both equal the oracle."""
    s, t = _grid_scene(templates["Dst4"], 400, 300, 20, 6)
    gpu, orc, ostats, gstats = _run_both(hip, s, t, max_pos=max_pos, tolerance_angle=10.0, max_overlap=0.5, score=0.6)
    assert gstats == ostats, (gstats, ostats)
    assert_same_results(gpu, orc, f"plain_many_{max_pos}")
    assert ostats[1] > 400


@pytest.mark.parametrize("scratch_mb", [8, 64])
def test_refinement_rounds(gpu_matcher_factory, templates, monkeypatch, scratch_mb):
    """A capped refinement scratch (FPM_SCRATCH_MB, read when a fresh context plans its search) splits every layer's
    ROIs into rounds of whole candidates (about 5 candidates per round at 8 MB); the batched Src7 search is
    unchanged (scratch bounded by the free HBM, more rounds instead of a failed allocation)."""
    monkeypatch.setenv("FPM_SCRATCH_MB", str(scratch_mb))
    t = templates["Dst7"]
    srcs = [synth.src7_scene(t, seed=7 + i)[0] for i in range(2)]
    m = gpu_matcher_factory(max_pos=3, tolerance_angle=180.0, score=0.7)
    assert m.learnPattern(t)
    m.stage(srcs)
    got = [[r.as_tuple() for r in rr] for rr in m.match_staged()]
    o = oracle.OracleMatcher().set(max_pos=3, tolerance_angle=180.0, score=0.7)
    o.learnPattern(t)
    assert got == [o.match(s) for s in srcs]


@pytest.mark.parametrize("prologue", ["0", "1"])
def test_step_prologue_forms(gpu_matcher_factory, templates, monkeypatch, prologue):
    """The candidate step of consecutive small layers in the next k_roi_small's prologue (FPM_STEP_PROLOGUE=1; by
    default for batches of <= 2 sources; Src7 layers 5-3, dead candidates kept as holes of the live list until
    k_cand_step compacts it after layer 3) and one k_cand_step launch per layer (FPM_STEP_PROLOGUE=0): a batch of three Src7 sources and one alone equal the oracle, result
    fields and the per-layer live counts (the prologue counts the survivors entering each layer)."""
    monkeypatch.setenv("FPM_STEP_PROLOGUE", prologue)
    t = templates["Dst7"]
    srcs = [synth.src7_scene(t, seed=31 + i)[0] for i in range(3)]
    m = gpu_matcher_factory(max_pos=3, tolerance_angle=180.0, score=0.7)
    assert m.learnPattern(t)
    m.stage(srcs)
    got = [[r.as_tuple() for r in rr] for rr in m.match_staged()]
    o = oracle.OracleMatcher().set(max_pos=3, tolerance_angle=180.0, score=0.7)
    o.learnPattern(t)
    assert got == [o.match(s) for s in srcs]
    gpu, orc, ostats, gstats = _run_both(m, srcs[0], t, max_pos=3, tolerance_angle=180.0, score=0.7)
    assert gstats == ostats
    assert_same_results(gpu, orc, f"src7 prologue={prologue}")
    # a low score threshold keeps more candidates alive through the small layers (more holes, more survivors)
    gpu, orc, ostats, gstats = _run_both(m, srcs[1], t, max_pos=8, tolerance_angle=180.0, score=0.3)
    assert gstats == ostats
    assert_same_results(gpu, orc, f"src7 prologue={prologue} score 0.3")


@pytest.mark.parametrize("warp3", ["0", "1"])
def test_src7_sampler_forms(gpu_matcher_factory, templates, monkeypatch, warp3):
    """The ROI sampler as one task per tile position of a candidate's three angle ROIs (k_roi_warp3, default) and as one
    task per ROI tile (k_roi_warp, FPM_WARP3=0), both with the empty-footprint tile path (a source whose candidates'
    ROIs reach past the image): a batch of two Src7 sources equals the oracle."""
    monkeypatch.setenv("FPM_WARP3", warp3)
    t = templates["Dst7"]
    srcs = [synth.src7_scene(t, seed=51 + i)[0] for i in range(2)]
    m = gpu_matcher_factory(max_pos=6, tolerance_angle=180.0, score=0.5)
    assert m.learnPattern(t)
    m.stage(srcs)
    got = [[r.as_tuple() for r in rr] for rr in m.match_staged()]
    o = oracle.OracleMatcher().set(max_pos=6, tolerance_angle=180.0, score=0.5)
    o.learnPattern(t)
    assert got == [o.match(s) for s in srcs]


@pytest.mark.parametrize("step_tables", ["0", "1"])
@pytest.mark.parametrize("nsrc", [1, 3])
def test_step_tables_forms(gpu_matcher_factory, templates, monkeypatch, step_tables, nsrc):
    """The next layer's warp tables written by the step (k_roi_eval / k_cand_step_tab, FPM_STEP_TABLES=1, the
    default) or by a k_roi_tables launch per layer (=0): the Src7 searches equal the oracle's either way."""
    monkeypatch.setenv("FPM_STEP_TABLES", step_tables)
    t = templates["Dst7"]
    srcs = [synth.src7_scene(t, seed=71 + i)[0] for i in range(nsrc)]
    m = gpu_matcher_factory(max_pos=3, tolerance_angle=180.0, score=0.7)
    assert m.learnPattern(t)
    m.stage(srcs)
    got = [[r.as_tuple() for r in rr] for rr in m.match_staged()]
    o = oracle.OracleMatcher().set(max_pos=3, tolerance_angle=180.0, score=0.7)
    o.learnPattern(t)
    assert got == [o.match(s) for s in srcs]


@pytest.mark.parametrize("pyr2", ["0", "1"])
def test_src7_batch_pyramid_forms(gpu_matcher_factory, templates, monkeypatch, pyr2):
    """The search pyramid as one launch per level (FPM_PYR2=0) and as two levels per launch at every pair
    (FPM_PYR2=1; by default only pairs whose input is small use it) on a batch of three Src7 sources: every search
    equals the oracle."""
    monkeypatch.setenv("FPM_PYR2", pyr2)
    t = templates["Dst7"]
    srcs = [synth.src7_scene(t, seed=41 + i)[0] for i in range(3)]
    m = gpu_matcher_factory(max_pos=3, tolerance_angle=180.0, score=0.7)
    assert m.learnPattern(t)
    m.stage(srcs)
    got = [[r.as_tuple() for r in rr] for rr in m.match_staged()]
    o = oracle.OracleMatcher().set(max_pos=3, tolerance_angle=180.0, score=0.7)
    o.learnPattern(t)
    assert got == [o.match(s) for s in srcs]


def test_constant_template(hip):
    t = np.full((40, 40), 90, np.uint8)
    s = synth.noise(200, 150, 90, 20, 12)
    gpu, orc, ostats, gstats = _run_both(hip, s, t, max_pos=2)
    assert gstats == ostats
    assert_same_results(gpu, orc, "equal1")


# ---------------------------------------------------------------------------------------- BASELINE configs
def test_config2_src10_blockmax(hip, templates):
    """configs[2] at full size: 3648x3648 Src10 surrogate, Dst10 x 144, TargetNum 100 -> s_BlockMax peaks."""
    s, t = synth.src10_scene(templates["Dst10"])
    gpu, orc, ostats, gstats = _run_both(hip, s, t, max_pos=100, score=0.7, tolerance_angle=0.0)
    assert gstats == ostats
    assert_same_results(gpu, orc, "src10")
    assert len(orc) >= 100


def test_blockmax_overlap(hip, templates):
    """s_BlockMax mode (map / template area > 500, MaxPos > 10) with MaxOverlap 0.4: painted rectangles smaller
    than two template sizes, so peaks sit close together and rectangles straddle block borders and strips."""
    s, t = synth.src10_scene(templates["Dst10"])
    crop = np.ascontiguousarray(s[:1824, :1830])
    for ov, n in ((0.4, 60), (0.8, 40)):
        gpu, orc, ostats, gstats = _run_both(hip, crop, t, max_pos=n, score=0.5, tolerance_angle=0.0, max_overlap=ov)
        assert gstats == ostats
        assert_same_results(gpu, orc, f"blockmax_ov{ov}")


def test_blockmax_ties_across_blocks(hip, templates):
    """Identical windows at many sites (the template pasted at 4-aligned positions of a flat background, so the
    top-layer windows are equal) give exactly equal scores in different s_BlockMax blocks: the peak order must
    follow the block order (max_element's first block), then the row-major position inside the block."""
    t = templates["Dst10"]
    s = np.full((1824, 1824), 90, np.uint8)
    for gy in range(9):
        for gx in range(9):
            synth.paste(s, t, 96 + 192 * gx, 96 + 192 * gy)
    gpu, orc, ostats, gstats = _run_both(hip, s, t, max_pos=50, score=0.7, tolerance_angle=0.0)
    assert gstats == ostats
    assert_same_results(gpu, orc, "blockmax_ties")


@pytest.mark.parametrize("prm", [dict(max_overlap=1.0), dict(score=0.05), dict(score=-0.5)],
                         ids=["empty_rect", "many_candidates", "negative_score"])
def test_blockmax_fallback_paths(hip, templates, prm):
    """s_BlockMax peak extraction off the greedy form's path: an empty painted rectangle (MaxOverlap 1: the same
    peak again, as the reference finds it), candidate lists too long for the sorted form, a threshold below the
    painted value's reach."""
    s, t = synth.src10_scene(templates["Dst10"])
    crop = np.ascontiguousarray(s[:1824, :1824])
    base = dict(max_pos=30, score=0.7, tolerance_angle=0.0)
    base.update(prm)
    gpu, orc, ostats, gstats = _run_both(hip, crop, t, **base)
    assert gstats == ostats
    assert_same_results(gpu, orc, f"blockmax_{prm}")


@pytest.mark.parametrize("overlap_on_device", [False, True])
def test_config2_src10_rotation_sweep(hip, templates, monkeypatch, overlap_on_device):
    """configs[2] stress (+-180 deg, 47 top angles, TargetNum 100) on the 1824x1824 top-left quarter; with the
    overlap filter's pair tests forced onto the device (FPM_OVERLAP_DEVICE_MIN=1) and on the host."""
    monkeypatch.setenv("FPM_OVERLAP_DEVICE_MIN", "1" if overlap_on_device else "1000000000")
    s, t = synth.src10_scene(templates["Dst10"])
    crop = np.ascontiguousarray(s[:1824, :1824])
    gpu, orc, ostats, gstats = _run_both(hip, crop, t, max_pos=100, score=0.7, tolerance_angle=180.0)
    assert gstats == ostats
    assert_same_results(gpu, orc, "src10_180")
    assert len(orc) >= 30


def test_config2_src10_full_rotation_sweep(hip, templates):
    """configs[2] stress at full size (3648x3648, +-180 deg, TargetNum 100: ~4900 top candidates, whose overlap
    filter runs its pair tests on the device by default) equal to the oracle."""
    s, t = synth.src10_scene(templates["Dst10"])
    gpu, orc, ostats, gstats = _run_both(hip, np.ascontiguousarray(s), t, max_pos=100, score=0.7,
                                         tolerance_angle=180.0)
    assert gstats == ostats
    assert gstats[1] >= 1024
    assert_same_results(gpu, orc, "src10_180_full")
    assert len(orc) >= 100


def test_config3_batch_4096(hip):
    """configs[3]: 4096x4096 sources searched as one device batch, 512x512 template, +-180 deg (reference step)."""
    srcs, t = synth.batch_sources(2)
    o = oracle.OracleMatcher().set(max_pos=1, tolerance_angle=180.0)
    o.learnPattern(t)
    hip.resetParams()
    hip.setMaxPositions(1)
    hip.setToleranceAngle(180.0)
    assert hip.learnPattern(t)
    batch = hip.match_batch(srcs)
    for k, s in enumerate(srcs):
        orc = o.match(s)
        assert_same_results(batch[k], orc, f"batch4096_{k}")
        assert len(orc) >= 1


def test_config4_src5_rotation_set(hip, templates):
    """configs[4]: the Src5 rotation set (0, 45, ..., 315 deg) with sub-pixel estimation, as one device batch."""
    srcs, t = synth.src5_set(templates["Dst5"])
    o = oracle.OracleMatcher().set(max_pos=1, tolerance_angle=180.0, subpixel=1)
    o.learnPattern(t)
    hip.resetParams()
    hip.setMaxPositions(1)
    hip.setToleranceAngle(180.0)
    hip.setSubPixelEstimation(True)
    assert hip.learnPattern(t)
    batch = hip.match_batch(srcs)
    for k, s in enumerate(srcs):
        orc = o.match(s)
        assert_same_results(batch[k], orc, f"src5_{45 * k}")
        assert len(orc) == 1


def test_batch_equals_single(hip, templates):
    t = templates["Dst10"]
    srcs = []
    for k in range(5):
        s = synth.noise(360, 300, 128, 10, 50 + k)
        synth.paste_rotated(s, t, 100 + 30 * k, 120 + 10 * k, 20.0 * k - 50)
        srcs.append(s)
    o = oracle.OracleMatcher().set(max_pos=2, tolerance_angle=180.0)
    o.learnPattern(t)
    hip.resetParams()
    hip.setMaxPositions(2)
    hip.setToleranceAngle(180.0)
    hip.learnPattern(t)
    batch = hip.match_batch(srcs)
    for k, s in enumerate(srcs):
        assert_same_results(batch[k], o.match(s), f"batch{k}")


def test_src7_batch_multichunk_pyramid(hip, templates):
    """configs[1] as a batch of 6 full-size sources: the batched pyrDown launch walks several 32-row chunks per
    workgroup (k_pyr_down_s's carried window at the sizes the bench runs), and every source's search equals the
    oracle's."""
    t = templates["Dst7"]
    srcs = [synth.src7_scene(t, seed=7 + 13 * k)[0] for k in range(6)]
    o = oracle.OracleMatcher().set(max_pos=3, tolerance_angle=180.0, score=0.7)
    o.learnPattern(t)
    hip.resetParams()
    hip.setMaxPositions(3)
    hip.setToleranceAngle(180.0)
    hip.setScore(0.7)
    assert hip.learnPattern(t)
    batch = hip.match_batch(srcs)
    for k, s in enumerate(srcs):
        orc = o.match(s)
        assert_same_results(batch[k], orc, f"src7_batch{k}")
        assert len(orc) == 3


def test_concurrent_contexts(hip, templates, gpu_matcher_factory):
    """Two contexts (two HIP streams) with searches in flight at once (fpm_match_staged_launch / _finish) give
    the oracle's results; staging or a second launch while a search is in flight is refused."""
    t = templates["Dst10"]
    srcs = []
    for k in range(6):
        s = synth.noise(360, 300, 128, 10, 70 + k)
        synth.paste_rotated(s, t, 110 + 25 * k, 130 + 8 * k, 35.0 * k - 80)
        srcs.append(s)
    o = oracle.OracleMatcher().set(max_pos=3, tolerance_angle=180.0)
    o.learnPattern(t)
    ms = [gpu_matcher_factory(max_pos=3, tolerance_angle=180.0) for _ in range(2)]
    for m, part in zip(ms, (srcs[:3], srcs[3:])):
        assert m.learnPattern(t)
        m.stage(part)
    for rep in range(2):
        for m in ms:
            m.match_staged_launch()
        with pytest.raises(ValueError):
            ms[0].stage(srcs[:3])
        with pytest.raises(RuntimeError):
            ms[1].match_staged_launch()
        outs = [m.match_staged_finish_array() for m in ms]
        got = [[SingleTargetMatch.from_row(res[s_, i]) for i in range(cnt[s_])] for cnt, res in outs
               for s_ in range(len(cnt))]
        for k, s in enumerate(srcs):
            assert_same_results(got[k], o.match(s), f"ctx{k // 3} src{k} rep{rep}")


def test_error_behaviour(hip, templates):
    hip.clearPattern()
    assert hip.match(np.zeros((50, 50), np.uint8)) == []        # not learned (TemplateMatcher.cpp:99)
    assert hip.learnPattern(np.zeros((0, 0), np.uint8)) is False
    hip.learnPattern(templates["Dst10"])
    assert hip.match(np.zeros((20, 200), np.uint8)) == []       # orientation mismatch (:107-110)
    assert hip.match(np.zeros((0, 0), np.uint8)) == []
    prev = hip.getLastExecutionTime()
    assert hip.match(np.full((80, 80), 7, np.uint8)) == []       # nothing found: time unchanged (:398-404)
    assert hip.getLastExecutionTime() == prev


def test_src6_real_image(hip, templates):
    """README Test6 (README.md:70; Result Images/Result6.jpg): Src6/Dst6, TargetNum 15, Score 0.8, Tol 180,
    MRA 256 -> 15 pocket detections, identical to the oracle."""
    import os

    from fastest_image_pattern_matching_amd.images import imread_gray

    src = imread_gray(os.path.join(os.path.dirname(__file__), "golden", "Src6.jpg"))
    gpu, orc, ostats, gstats = _run_both(hip, src, templates["Dst6"], max_pos=15, score=0.8, tolerance_angle=180.0)
    assert gstats == ostats
    assert_same_results(gpu, orc, "src6")
    assert len(gpu) == 15
