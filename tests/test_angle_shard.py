"""Angle sharding of one search, host side: the coupled tail fpm_merge_candidates (libfpm_hip.so,
host code, no device) over candidate records, and the gloo all_gather of records between ranks.

The records come from the CPU oracle (tests/oracle.py: the restatement exports, for every top-layer candidate in
the reference's push order, its top score, angle index, peak rank and refined pose).  fpm_merge_candidates over
the full list must reproduce the oracle's own match() bit for bit, and so must the rank-order concatenation of
per-rank angle blocks after an all_gather.  The GPU side (records produced by the HIP path per shard) is
tests/test_gpu_angle_shard.py.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from fastest_image_pattern_matching_amd import sharding, synth
from fastest_image_pattern_matching_amd.matcher import CANDIDATE_DTYPE, merge_candidates
from tests import oracle
from tests.cases import CASES

FAST_CASES = ["plumbing_tol0", "dst10_multi", "dst10_nosimd", "dst5_subpixel", "dst4_overlap", "dst3_range",
              "top_is_layer0", "score_low_many"]


def _oracle_run(case, templates):
    make, prm = CASES[case]
    s, t = make(templates)
    o = oracle.OracleMatcher().set(**prm)
    assert o.learnPattern(t)
    res = o.match(s)
    return o, t, res, o.candidates()


def _tuples(results):
    return [r.as_tuple() for r in results]


@pytest.mark.parametrize("case", FAST_CASES)
def test_merge_reproduces_oracle(templates, case):
    o, t, res, cands = _oracle_run(case, templates)
    assert len(cands) == o.stats()[1]                 # one record per top-layer candidate
    assert np.all(np.diff(cands["angle_index"]) >= 0)
    merged = merge_candidates(o.params, t.shape[1], t.shape[0], cands)
    assert _tuples(merged) == res, case


@pytest.mark.parametrize("case", ["dst10_multi", "dst4_overlap", "score_low_many"])
@pytest.mark.parametrize("shards", [2, 3, 8, 50])
def test_block_concatenation_is_push_order(templates, case, shards):
    """Per-shard angle blocks (sharding.angle_block) concatenated in shard order = the full list, and merge it."""
    o, t, res, cands = _oracle_run(case, templates)
    nang = o.stats()[0]
    parts = []
    for k in range(shards):
        a0, a1 = sharding.angle_block(nang, k, shards)
        parts.append(cands[(cands["angle_index"] >= a0) & (cands["angle_index"] < a1)])
    cat = np.concatenate(parts)
    assert cat.tobytes() == cands.tobytes()
    assert _tuples(merge_candidates(o.params, t.shape[1], t.shape[0], cat)) == res


def test_merge_rejects_out_of_order(templates):
    o, t, res, cands = _oracle_run("dst10_multi", templates)
    assert len(np.unique(cands["angle_index"])) >= 2
    swapped = np.concatenate([cands[cands["angle_index"] > cands["angle_index"][0]],
                              cands[cands["angle_index"] == cands["angle_index"][0]]])
    with pytest.raises(ValueError):
        merge_candidates(o.params, t.shape[1], t.shape[0], swapped)
    bad = cands.copy()
    bad["peak_rank"][0] = 1
    with pytest.raises(ValueError):
        merge_candidates(o.params, t.shape[1], t.shape[0], bad)
    assert merge_candidates(o.params, t.shape[1], t.shape[0], cands[:0]) == []


def test_merge_equal_scores_keep_reference_order():
    """Equal top scores across angles: the tail's std::sort must see the push order (it is unstable), so the
    first-pushed of two equal, overlapping candidates survives the rotated-rect filter."""
    p = oracle.OracleMatcher().params
    p.max_overlap = 0.0
    rec = np.zeros(40, CANDIDATE_DTYPE)
    rec["top_score"] = 0.9
    rec["angle_index"] = np.arange(40)
    rec["kept"] = 1
    rec["x"], rec["y"] = 100.0, 100.0
    rec["score"] = 0.95
    rec["angle"] = np.arange(40) * 0.25
    out = merge_candidates(p, 30, 20, rec)
    assert len(out) == 1
    # std::sort (introsort, > 16 elements) of 40 equal keys: the survivor is whatever libstdc++ puts first, the
    # same element for any sharding of the same sequence
    again = merge_candidates(p, 30, 20, np.concatenate([rec[:13], rec[13:]]))
    assert _tuples(out) == _tuples(again)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, cases, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        templates = synth.load_templates()
        for case in cases:
            o, t, res, cands = _oracle_run(case, templates)
            a0, a1 = sharding.angle_block(o.stats()[0], rank, world)
            mine = cands[(cands["angle_index"] >= a0) & (cands["angle_index"] < a1)]
            full = sharding.gather_candidates(mine)
            merged = sharding.merge_gathered(o.params, t.shape[1], t.shape[0], full)
            q.put((rank, case, full.tobytes() == cands.tobytes(), _tuples(merged) == res, len(res)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_angle_sharded_gloo(world):
    cases = ["plumbing_tol0", "dst10_multi", "dst5_subpixel", "dst4_overlap"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cases, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=180) for _ in range(world * len(cases))]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(got) == world * len(cases)
    for rank, case, same_records, same_results, n in got:
        assert same_records, (rank, case)
        assert same_results, (rank, case)
        assert n >= 1, (rank, case)


_MERGE_CHILD = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from fastest_image_pattern_matching_amd.matcher import CANDIDATE_DTYPE, merge_candidates
from fastest_image_pattern_matching_amd import _lib as L
z = np.load(sys.argv[2])
p = L.Params(); L.load().fpm_params_default(p)
p.max_pos, p.score, p.tolerance_angle, p.max_overlap = int(z["params"][0]), *map(float, z["params"][1:])
rec = z["records"].view(CANDIDATE_DTYPE)
out = np.array([r.as_tuple() for r in merge_candidates(p, int(z["tmpl_wh"][0]), int(z["tmpl_wh"][1]), rec)])
print("SAME" if out.shape == z["results"].shape and np.array_equal(out, z["results"]) else "DIFF")
"""


@pytest.mark.parametrize("threads", ["1", "8"])
def test_merge_large_fixture_threads(threads):
    """Src10 +-180 records (4935 candidates, 144 duplicate clusters; tests/golden/make_merge_fixture.py): the merge's
    component-parallel rotated-rect filter gives the oracle's sequential result at 1 and 8 host threads."""
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, FPM_HOST_THREADS=threads)
    out = subprocess.run([sys.executable, "-c", _MERGE_CHILD, repo,
                          os.path.join(repo, "tests", "golden", "merge_src10_180.npz")],
                         env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip().endswith("SAME"), out.stdout + out.stderr


def _batch_worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        srcs, t = synth.src5_set()
        prm = dict(max_pos=1, tolerance_angle=180.0, subpixel=1)
        local, full_res = [], []
        for s in srcs:
            o = oracle.OracleMatcher().set(**prm)
            assert o.learnPattern(t)
            full_res.append(o.match(s))
            c = o.candidates()
            a0, a1 = sharding.angle_block(o.stats()[0], rank, world)
            local.append(c[(c["angle_index"] >= a0) & (c["angle_index"] < a1)])
        full = sharding.gather_candidates_batch(local)
        merged = [_tuples(merge_candidates(o.params, t.shape[1], t.shape[0], c)) for c in full]
        q.put((rank, merged == full_res, [len(c) for c in full], [len(c) for c in local]))
    finally:
        dist.destroy_process_group()


def test_gather_candidates_batch_config4_gloo():
    """bench.py --workload config4's per-step exchange (world 2, gloo): every rank holds its angle block's candidate
    records of each of the 8 Src5 images (oracle records); one batched all_gather (counts, then all records) gives
    every image's rank-order concatenation, whose merge equals the oracle's unsharded search of that image."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    procs = [ctx.Process(target=_batch_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, n_full, n_local in got:
        assert ok, rank
        assert len(n_full) == 8 and all(n > 0 for n in n_full)
    # the ranks' blocks partition each image's records
    by_rank = {r: nl for r, _, _, nl in got}
    assert [a + b for a, b in zip(by_rank[0], by_rank[1])] == got[0][2]
