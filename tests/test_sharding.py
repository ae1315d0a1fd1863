"""Multi-rank host logic: source sharding and the result all_gather, world_size 2 on gloo.

The pixel path needs a GPU, so the ranks here use a deterministic stand-in matcher, or the CPU restatement searching
real scenes (test_match_sharded_gloo_real_searches); the collective, packing, padding and source-order reassembly are
the code the MI355X run uses (over RCCL instead of gloo).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from fastest_image_pattern_matching_amd import sharding


class _Res:
    def __init__(self, t):
        self.t = t

    def as_tuple(self):
        return self.t


class FakeMatcher:
    """Result count and values derived from each source's pixels, so a misrouted source is detected."""

    def match_batch(self, sources):
        out = []
        for s in sources:
            k = int(s[0, 0]) % 4
            out.append([_Res(tuple(float(s[0, 0]) * 100 + j * 12 + f for f in range(12))) for j in range(k)])
        return out


def _expected(sources):
    return [[r.as_tuple() for r in res] for res in FakeMatcher().match_batch(sources)]


def _sources(n):
    return [np.full((4, 5), (7 * i + 3) % 251, dtype=np.uint8) for i in range(n)]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_list, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        for n in n_list:
            full = sharding.match_sharded(FakeMatcher(), _sources(n), cap=8)
            q.put((rank, n, full))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_match_sharded_gloo(world):
    n_list = [0, 1, 2, 5, 9]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_list, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world * len(n_list)):
        rank, n, full = q.get(timeout=120)
        got[(rank, n)] = full
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for n in n_list:
        exp = _expected(_sources(n))
        for r in range(world):
            assert got[(r, n)] == exp, (r, n)


def test_shard_range_partition():
    for n in range(0, 40):
        for world in range(1, 9):
            spans = [sharding.shard_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a0, b0), (a1, b1) in zip(spans, spans[1:]):
                assert b0 == a1
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        sharding.shard_range(4, 2, 2)


def test_pack_roundtrip_and_capacity():
    res = [[tuple(range(12))], [], [tuple(float(i) / 3 for i in range(12))] * 3]
    block = sharding.pack_results(res, 4, 3)
    assert block.shape == (4, 1 + 3 * 12)
    assert sharding.unpack_results(block, 3) == [[tuple(float(v) for v in r) for r in s] for s in res]
    with pytest.raises(ValueError):
        sharding.pack_results(res, 4, 2)
    with pytest.raises(ValueError):
        sharding.pack_results([[(1.0,) * 11]], 1, 1)


class OracleBatch:
    """The CPU restatement as the rank's matcher (test infrastructure: real result payloads -- 12 doubles per result,
    per-source counts from actual searches -- through the same sharding code the GPU ranks run)."""

    def __init__(self, templ, **prm):
        from tests import oracle

        self.o = oracle.OracleMatcher().set(**prm)
        assert self.o.learnPattern(templ)

    def match_batch(self, sources):
        return [[_Res(t) for t in self.o.match(s)] for s in sources]


def _real_scenes(n):
    from fastest_image_pattern_matching_amd import synth

    t = synth.load_templates()["Dst10"]
    srcs = []
    for k in range(n):
        s = synth.noise(240, 200, 128, 10, 70 + k)
        for c in range(k % 3 + 1):   # 1-3 copies: uneven result counts per source
            synth.paste_rotated(s, t, 50 + 60 * c, 60 + 40 * c, 25.0 * k - 40 * c)
        srcs.append(s)
    return t, srcs


def _oracle_worker(rank, world, port, n, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t, srcs = _real_scenes(n)
        full = sharding.match_sharded(OracleBatch(t, max_pos=4, tolerance_angle=180.0), srcs, cap=8)
        q.put((rank, full))
    finally:
        dist.destroy_process_group()


def test_match_sharded_gloo_real_searches():
    """world 2 over gloo with real searches on each rank (the oracle as the rank's matcher, 5 sources split 3 / 2):
    every rank ends with every source's results, in source order, equal to one process searching them all."""
    from tests import oracle

    n, world = 5, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_oracle_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        rank, full = q.get(timeout=300)
        got[rank] = full
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    t, srcs = _real_scenes(n)
    o = oracle.OracleMatcher().set(max_pos=4, tolerance_angle=180.0)
    assert o.learnPattern(t)
    exp = [[tuple(float(v) for v in r) for r in o.match(s)] for s in srcs]
    assert sum(len(e) for e in exp) >= n   # real detections in every source
    for r in range(world):
        assert got[r] == exp, r


def _views_of(per_source, cap_buf, runs):
    """per-source result tuples -> match_staged_array-style (counts, results) views, split into `runs` (one per
    context); the buffer beyond each count holds garbage, as a reused result buffer does."""
    out, pos = [], 0
    for n in runs:
        part = per_source[pos:pos + n]
        cnt = np.array([len(r) for r in part], np.int32)
        arr = np.full((n, cap_buf, 12), 777.0)
        for i, res in enumerate(part):
            for j, r in enumerate(res):
                arr[i, j] = r
        out.append((cnt, arr))
        pos += n
    return out


def _array_worker(rank, world, port, n, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a, b = sharding.shard_range(n, world, rank)
        mine = _expected(_sources(n))[a:b]
        k = b - a
        views = _views_of(mine, 6, [k // 2, k - k // 2])      # two contexts per rank
        cnt, arr = sharding.gather_result_arrays(views, n, cap=4)
        q.put((rank, cnt.tolist(), arr.tolist()))
    finally:
        dist.destroy_process_group()


def test_gather_result_arrays_gloo():
    """bench.py --workload config3's per-step exchange (world 2, gloo): each rank's context views all-gathered into
    the whole job's (counts, results) in source order, equal to the object path (gather_results)."""
    n, world = 9, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_array_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        rank, cnt, arr = q.get(timeout=120)
        got[rank] = (cnt, arr)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp = _expected(_sources(n))
    for r in range(world):
        cnt, arr = got[r]
        assert cnt == [len(e) for e in exp]
        assert [[tuple(arr[i][j]) for j in range(cnt[i])] for i in range(n)] == exp
        # padding is zeroed, not the stale buffer contents
        assert all(v == 0.0 for i in range(n) for j in range(cnt[i], 4) for v in arr[i][j])


def test_pack_result_arrays_matches_pack_results():
    per = _expected(_sources(7))
    views = _views_of(per, 5, [3, 0, 4])
    assert np.array_equal(sharding.pack_result_arrays(views, 8, 4), sharding.pack_results(per, 8, 4))
    with pytest.raises(ValueError):
        sharding.pack_result_arrays(views, 8, 2)      # a source with 3 results over capacity 2
    with pytest.raises(ValueError):
        sharding.pack_result_arrays(views, 6, 4)      # 7 sources, 6 slots


def test_config3_sources_shard_by_index():
    """configs[3]'s sources depend only on their index: a rank's block equals the same slice of the whole batch."""
    from fastest_image_pattern_matching_amd import synth

    full, t = synth.batch_sources(5, size=96, tsize=16)
    for a, b in [(0, 2), (2, 5), (4, 5)]:
        part, t2 = synth.batch_sources(b - a, size=96, tsize=16, first=a)
        assert np.array_equal(t, t2) and all(np.array_equal(x, y) for x, y in zip(part, full[a:b]))
