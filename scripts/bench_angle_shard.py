#!/usr/bin/env python3
"""Strong scaling of ONE search split by angle (sharding.match_angle_sharded).

Workload (default): BASELINE configs[2] stress — Src10 surrogate 3648x3648, Dst10 54x54, ToleranceAngle 180,
TargetNum 100, Score 0.7 (47 top-layer angles, s_BlockMax peaks).  ``--config src7``: configs[1].

Two modes:
  * multi-rank (torchrun, one process per GPU, RCCL): every rank holds the same source resident in HBM, searches its
    angle block (fpm_set_angle_shard), the candidate records are all-gathered (two RCCL all_gathers) and every rank
    merges them (fpm_merge_candidates).  A step = one complete search; barrier + synchronize bracket K steps, max
    over ranks.  The merged results are checked against the unsharded search once before timing.
  * ``--simulate W1,W2,...`` (one GPU): each shard of each W timed alone on the one device, plus the host merge of
    the full record list; projected per-search time = max over shards + merge (the all_gather's xGMI latency is not
    in the projection — it is measured only in the multi-rank mode).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def workload(name):
    from fastest_image_pattern_matching_amd import synth

    T = synth.load_templates()
    if name == "src10":
        s, t = synth.src10_scene(T["Dst10"])
        return s, t, dict(max_pos=100, score=0.7, tolerance_angle=180.0), "Src10 3648x3648 / Dst10 54x54, +-180, TargetNum 100"
    s, t = synth.src7_scene(T["Dst7"])
    return s, t, dict(max_pos=3, score=0.7, tolerance_angle=180.0), "Src7 4024x3036 / Dst7 762x521, +-180, TargetNum 3"


def make_matcher(dev, t, prm):
    from fastest_image_pattern_matching_amd import TemplateMatcher

    m = TemplateMatcher(dev)
    for k, v in prm.items():
        setattr(m._params, k, v)
    assert m.learnPattern(t)
    return m


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    return (time.perf_counter() - t0) / steps * 1e3


def simulate(args):
    from fastest_image_pattern_matching_amd.matcher import merge_candidates

    s, t, prm, desc = workload(args.config)
    m = make_matcher(0, t, prm)
    m.stage([s])
    full_res = m.match_staged()[0]
    full_ms = timed(lambda: m.match_staged_array(), args.steps, args.warmup)
    rec = m.last_candidates(0)
    nang = m.search_stats()[0]
    merge_ms = timed(lambda: merge_candidates(m._params, t.shape[1], t.shape[0], rec), args.steps, 2)
    out = {"workload": desc, "top_angles": nang, "candidates": int(len(rec)), "results": len(full_res),
           "unsharded_ms_per_search": round(full_ms, 4), "merge_ms": round(merge_ms, 4), "shards": []}
    for W in args.simulate:
        per = []
        parts = []
        for k in range(W):
            m.setAngleShard(k, W)
            per.append(timed(lambda: m.match_staged_candidates(), args.steps, args.warmup))
            parts.append(m.last_candidates(0))
        m.setAngleShard(0, 1)
        merged = merge_candidates(m._params, t.shape[1], t.shape[0], np.concatenate(parts))
        assert [r.as_tuple() for r in merged] == [r.as_tuple() for r in full_res], f"W={W}: merged results differ"
        proj = max(per) + merge_ms
        out["shards"].append({"W": W, "shard_ms": [round(x, 4) for x in per], "max_shard_ms": round(max(per), 4),
                              "projected_ms_per_search": round(proj, 4),
                              "projected_speedup": round(full_ms / proj, 3)})
    print(json.dumps(out), flush=True)


def multirank(args):
    import torch
    import torch.distributed as dist

    from fastest_image_pattern_matching_amd import sharding

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    s, t, prm, desc = workload(args.config)
    m = make_matcher(local, t, prm)
    ref = [r.as_tuple() for r in m.match(s)]          # unsharded, for the check
    m.setAngleShard(rank, world)
    m.stage([s])

    def step():
        rec = m.match_staged_candidates()[0]
        full = sharding.gather_candidates(rec, device=dev)
        return sharding.merge_gathered(m._params, t.shape[1], t.shape[0], full)

    got = [r.as_tuple() for r in step()]
    assert got == ref, "angle-sharded results differ from the unsharded search"
    for _ in range(args.warmup):
        step()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    dist.barrier()
    torch.cuda.synchronize()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    el = float(el.item())
    if rank == 0:
        print(json.dumps({"metric": "searches/s (one search split by angle)", "value": round(args.steps / el, 3),
                          "unit": "searches/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_search": round(el / args.steps * 1e3, 4), "scaling": "strong",
                          "workload": desc, "results": len(ref)}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=["src10", "src7"], default="src10")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--simulate", type=lambda v: [int(x) for x in v.split(",")], default=None,
                    help="one GPU: comma-separated shard counts to time shard by shard")
    args = ap.parse_args()
    if args.simulate:
        simulate(args)
    else:
        multirank(args)


if __name__ == "__main__":
    main()
