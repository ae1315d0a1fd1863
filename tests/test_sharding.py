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
