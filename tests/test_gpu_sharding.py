"""Source sharding with the GPU matcher on every rank (gfx950 required): two rank processes on the box's one GPU, each
with its own TemplateMatcher (its own HIP stream and plan), the results all-gathered over gloo by the same
sharding.match_sharded the N-GPU bench uses over RCCL.  Every rank must end with every source's results, in source
order, equal to the oracle's."""
import os
import socket

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _scenes(n):
    from fastest_image_pattern_matching_amd import synth

    t = synth.load_templates()["Dst10"]
    srcs = []
    for k in range(n):
        s = synth.noise(300, 260, 128, 10, 90 + k)
        for c in range(k % 3 + 1):
            synth.paste_rotated(s, t, 60 + 70 * c, 70 + 50 * c, 30.0 * k - 45 * c)
        srcs.append(s)
    return t, srcs


def _worker(rank, world, port, n, q):
    import torch.distributed as dist

    from fastest_image_pattern_matching_amd import TemplateMatcher, sharding

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t, srcs = _scenes(n)
        m = TemplateMatcher(0)
        m.setMaxPositions(4)
        m.setToleranceAngle(180.0)
        assert m.learnPattern(t)
        q.put((rank, sharding.match_sharded(m, srcs, cap=8)))
    finally:
        dist.destroy_process_group()


def test_match_sharded_gpu_ranks():
    from tests import oracle

    n, world = 7, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(world):
            rank, full = q.get(timeout=100)
            got[rank] = full
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    t, srcs = _scenes(n)
    o = oracle.OracleMatcher().set(max_pos=4, tolerance_angle=180.0)
    assert o.learnPattern(t)
    exp = [[tuple(float(v) for v in r) for r in o.match(s)] for s in srcs]
    assert sum(len(e) for e in exp) >= n
    for r in range(world):
        assert got[r] == exp, r
