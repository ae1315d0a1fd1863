"""Context state rules of the C ABI on the GPU: a plain match() replaces a staged batch, the
parameters / template cannot change under a search in flight, and the angle-sharded wrapper leaves the matcher
searching the whole angle list and never merges a previous search's candidate records."""
import os

import numpy as np
import pytest

from fastest_image_pattern_matching_amd import synth
from fastest_image_pattern_matching_amd.sharding import match_angle_sharded
from tests import oracle
from tests.test_gpu_parity import assert_same_results

pytestmark = pytest.mark.gpu


def _scenes(t, n, seed):
    out = []
    for k in range(n):
        s = synth.noise(360, 300, 128, 10, seed + k)
        synth.paste_rotated(s, t, 110 + 25 * k, 130 + 8 * k, 35.0 * k - 80)
        out.append(s)
    return out


def test_match_replaces_staged_batch(gpu_matcher_factory, templates):
    t = templates["Dst10"]
    srcs = _scenes(t, 3, 90)
    m = gpu_matcher_factory(max_pos=3, tolerance_angle=180.0)
    o = oracle.OracleMatcher().set(max_pos=3, tolerance_angle=180.0)
    assert m.learnPattern(t) and o.learnPattern(t)
    m.stage(srcs)
    batch = m.match_staged()
    one = m.match(srcs[1])                       # re-lays the context out for one source
    assert_same_results(one, o.match(srcs[1]), "single after staged")
    with pytest.raises(RuntimeError):
        m.match_staged_launch()                  # the staged batch is gone: refused, not a 1-source replay
    m.stage(srcs)
    again = m.match_staged()
    for k in range(3):
        assert [r.as_tuple() for r in again[k]] == [r.as_tuple() for r in batch[k]]


def test_no_changes_while_in_flight(gpu_matcher_factory, templates):
    t = templates["Dst10"]
    srcs = _scenes(t, 2, 95)
    m = gpu_matcher_factory(max_pos=3, tolerance_angle=180.0)
    o = oracle.OracleMatcher().set(max_pos=3, tolerance_angle=180.0)
    assert m.learnPattern(t) and o.learnPattern(t)
    m.stage(srcs)
    m.match_staged_launch()
    assert m.learnPattern(templates["Dst4"]) is False            # fpm_learn refused while pending
    m.setScore(0.99)
    assert m._lib.fpm_set_params(m._ctx, m._params) != 0        # fpm_set_params refused while pending
    assert m._lib.fpm_clear_pattern(m._ctx) != 0
    counts, res = m.match_staged_finish_array()
    m.setScore(0.7)
    from fastest_image_pattern_matching_amd.matcher import SingleTargetMatch
    for k, s in enumerate(srcs):
        got = [SingleTargetMatch.from_row(res[k, i]) for i in range(counts[k])]
        assert_same_results(got, o.match(s), f"in-flight {k}")


def test_angle_sharded_wrapper_restores_shard(gpu_matcher_factory, templates, tmp_path):
    import torch.distributed as dist

    t = templates["Dst10"]
    s = _scenes(t, 1, 99)[0]
    o = oracle.OracleMatcher().set(max_pos=3, tolerance_angle=180.0)
    assert o.learnPattern(t)
    m = gpu_matcher_factory(max_pos=3, tolerance_angle=180.0)
    assert m.learnPattern(t)
    store = dist.FileStore(os.path.join(str(tmp_path), "store"), 1)
    dist.init_process_group("gloo", store=store, rank=0, world_size=1)
    try:
        sharded = match_angle_sharded(m, s)
        assert_same_results(sharded, o.match(s), "sharded world 1")
        assert m.getAngleShard() == (0, 1)
        assert_same_results(m.match(s), o.match(s), "plain after sharded")
        # a source failing the reference size checks: [] on every rank, never the previous search's records
        assert match_angle_sharded(m, np.zeros((20, 400), np.uint8)) == []
        assert m.getAngleShard() == (0, 1)
    finally:
        dist.destroy_process_group()
