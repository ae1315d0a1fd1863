"""Multi-GPU layer: one process per GPU; sources sharded across ranks (batch config), or the
angles of one search sharded across ranks with an all_gather of candidate records (single-image configs).

Every source image is an independent ``TemplateMatcher::match`` call (TemplateMatcher.cpp:97-437), so the path
partitions by source with no data-path collective: rank r searches the contiguous slice
``shard_range(n, world, r)`` of the batch on its own GPU.  The only exchange is the final report — one
``all_gather`` of fixed-capacity result blocks (12 f64 per s_SingleTargetMatch, DataStructures.h:97-115) so
every rank (or just rank 0) can assemble the per-source result lists in the original source order.

The exchange works with any torch.distributed backend: ``nccl`` (RCCL over xGMI, tensors on the rank's GPU)
on the MI355X node and ``gloo`` (CPU tensors) in the CPU tests.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np

FIELDS = 12   # lt, rt, rb, lb, center (x, y each), angle, score


def shard_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous block split of n sources over `world` ranks; the first n % world ranks get one extra."""
    if world <= 0 or not (0 <= rank < world) or n < 0:
        raise ValueError(f"bad shard request n={n} world={world} rank={rank}")
    q, r = divmod(n, world)
    start = rank * q + min(rank, r)
    return start, start + q + (1 if rank < r else 0)


def shard_sizes(n: int, world: int) -> List[int]:
    return [b - a for a, b in (shard_range(n, world, k) for k in range(world))]


def pack_results(per_source: Sequence[Sequence[Sequence[float]]], slots: int, cap: int) -> np.ndarray:
    """Pack up to `slots` per-source result lists (each result a 12-tuple) into a [slots, 1 + cap*12] f64
    block: column 0 = result count, then `cap` zero-padded results.  Raises if a source has > cap results."""
    block = np.zeros((slots, 1 + cap * FIELDS), dtype=np.float64)
    if len(per_source) > slots:
        raise ValueError(f"{len(per_source)} sources do not fit {slots} slots")
    for i, res in enumerate(per_source):
        if len(res) > cap:
            raise ValueError(f"source {i}: {len(res)} results exceed capacity {cap}")
        block[i, 0] = len(res)
        for j, r in enumerate(res):
            if len(r) != FIELDS:
                raise ValueError(f"result must have {FIELDS} fields, got {len(r)}")
            block[i, 1 + j * FIELDS:1 + (j + 1) * FIELDS] = r
    return block


def unpack_results(block: np.ndarray, count: int) -> List[List[Tuple[float, ...]]]:
    out = []
    cap = (block.shape[1] - 1) // FIELDS
    for i in range(count):
        k = int(block[i, 0])
        if not 0 <= k <= cap:
            raise ValueError(f"corrupt result block: count {k} > cap {cap}")
        out.append([tuple(float(v) for v in block[i, 1 + j * FIELDS:1 + (j + 1) * FIELDS]) for j in range(k)])
    return out


def gather_results(local: Sequence[Sequence[Sequence[float]]], n_total: int, cap: int, group=None,
                   device=None) -> List[List[Tuple[float, ...]]]:
    """all_gather every rank's shard of results; returns the full per-source list (source order) on every rank.

    `local` holds the results of this rank's shard_range(n_total, world, rank) sources, in order.  Blocks are
    padded to the largest shard so one fixed-size collective suffices (KB-scale: latency-bound over xGMI)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    sizes = shard_sizes(n_total, world)
    if len(local) != sizes[rank]:
        raise ValueError(f"rank {rank} holds {len(local)} results, its shard has {sizes[rank]} sources")
    slots = max(max(sizes), 1)
    mine = torch.from_numpy(pack_results(local, slots, cap))
    if device is not None:
        mine = mine.to(device)
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine, group=group)
    full: List[List[Tuple[float, ...]]] = []
    for k in range(world):
        full.extend(unpack_results(parts[k].cpu().numpy(), sizes[k]))
    return full


def pack_result_arrays(views: Sequence[Tuple[np.ndarray, np.ndarray]], slots: int, cap: int) -> np.ndarray:
    """pack_results from ``match_staged_array`` views -- (counts [n], results [n, buffer cap, 12]) of consecutive
    source runs, e.g. one per context -- without building Python objects (the per-step exchange of bench.py)."""
    block = np.zeros((slots, 1 + cap * FIELDS), dtype=np.float64)
    row = 0
    for cnt, res in views:
        n = len(cnt)
        if row + n > slots:
            raise ValueError(f"{row + n} sources do not fit {slots} slots")
        if n and int(cnt.max()) > cap:
            raise ValueError(f"{int(cnt.max())} results exceed capacity {cap}")
        k = min(cap, res.shape[1])
        block[row:row + n, 0] = cnt
        # rows past a source's count are zeroed so the block does not depend on stale buffer contents
        keep = np.arange(k)[None, :] < cnt[:, None]
        block[row:row + n, 1:1 + k * FIELDS] = np.where(keep[..., None], res[:, :k], 0.0).reshape(n, k * FIELDS)
        row += n
    return block


def gather_result_arrays(views: Sequence[Tuple[np.ndarray, np.ndarray]], n_total: int, cap: int, group=None,
                         device=None) -> Tuple[np.ndarray, np.ndarray]:
    """gather_results over array views: this rank's shard_range(n_total, world, rank) sources as (counts, results)
    runs; returns (counts [n_total], results [n_total, cap, 12]) in source order on every rank (one all_gather)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    sizes = shard_sizes(n_total, world)
    if sum(len(c) for c, _ in views) != sizes[rank]:
        raise ValueError(f"rank {rank}: views hold {sum(len(c) for c, _ in views)} sources, shard has {sizes[rank]}")
    slots = max(max(sizes), 1)
    mine = torch.from_numpy(pack_result_arrays(views, slots, cap))
    if device is not None:
        mine = mine.to(device)
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine, group=group)
    full = np.concatenate([parts[k].cpu().numpy()[:sizes[k]] for k in range(world)])
    counts = full[:, 0].astype(np.int64)
    if counts.size and (counts.min() < 0 or counts.max() > cap):
        raise ValueError("corrupt result block")
    return counts, full[:, 1:].reshape(len(full), cap, FIELDS)


def match_sharded(matcher, sources: Sequence[np.ndarray], cap: int = 256, group=None, device=None):
    """Search this rank's slice of `sources` with `matcher` (a TemplateMatcher bound to this rank's GPU) and
    return every source's results, in source order, on every rank."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    a, b = shard_range(len(sources), world, rank)
    mine = matcher.match_batch(list(sources[a:b])) if b > a else []
    local = [[r.as_tuple() for r in res] for res in mine]
    return gather_results(local, len(sources), cap, group=group, device=device)


# ---------------------------------------------------------------------------------------------------------------
# Angle sharding of ONE search (SURVEY.md §8(e), configs 2-±180 / 3-±180 / 5): every rank runs the top-layer sweep
# and the pyramid descent for a contiguous block of the angle list (fpm_set_angle_shard), the candidate records
# (fpm_candidate: top score, angle index, peak rank, refined pose) are all-gathered in rank order — which is the
# reference's push order of vecMatchParameter (TemplateMatcher.cpp:157-211) — and every rank runs the coupled
# tail (sort :214, filters and conversion :373-432) on the full list with fpm_merge_candidates.
# ---------------------------------------------------------------------------------------------------------------
def angle_block(n_angles: int, shard: int, shards: int) -> Tuple[int, int]:
    """The block [a0, a1) of the top-layer angle list that fpm_set_angle_shard(shard, shards) searches (the same
    integer formula as the engine's build_plan)."""
    if shards < 1 or not 0 <= shard < shards or n_angles < 0:
        raise ValueError(f"bad angle shard {shard}/{shards} of {n_angles}")
    return n_angles * shard // shards, n_angles * (shard + 1) // shards


def gather_candidates(local: np.ndarray, group=None, device=None) -> np.ndarray:
    """all_gather variable-length candidate record arrays (CANDIDATE_DTYPE); returns the rank-order concatenation
    on every rank.  Two collectives: the counts, then the records as bytes padded to the largest count."""
    import torch
    import torch.distributed as dist

    from .matcher import CANDIDATE_DTYPE

    local = np.ascontiguousarray(local, CANDIDATE_DTYPE)
    world = dist.get_world_size(group)
    cnt = torch.tensor([len(local)], dtype=torch.int64)
    if device is not None:
        cnt = cnt.to(device)
    counts = [torch.empty_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    counts = [int(c.item()) for c in counts]
    width = max(max(counts), 1) * CANDIDATE_DTYPE.itemsize
    buf = np.zeros(width, np.uint8)
    raw = local.view(np.uint8)
    buf[:raw.size] = raw
    mine = torch.from_numpy(buf)
    if device is not None:
        mine = mine.to(device)
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine, group=group)
    out = [parts[k].cpu().numpy()[:counts[k] * CANDIDATE_DTYPE.itemsize].view(CANDIDATE_DTYPE) for k in range(world)]
    return np.concatenate(out) if out else np.zeros(0, CANDIDATE_DTYPE)


def gather_candidates_batch(local: Sequence[np.ndarray], group=None, device=None) -> List[np.ndarray]:
    """gather_candidates for a batch of sources searched by angle shard on every rank (the same sources on every
    rank, each rank its angle block): per source, the rank-order concatenation of every rank's records -- that
    source's push order (TemplateMatcher.cpp:157-211).  Two collectives for the whole batch: the [sources] record
    counts, then every source's records back to back as bytes, padded to the largest total."""
    import torch
    import torch.distributed as dist

    from .matcher import CANDIDATE_DTYPE

    recs = [np.ascontiguousarray(x, CANDIDATE_DTYPE) for x in local]
    world = dist.get_world_size(group)
    n_src = len(recs)
    cnt = torch.tensor([len(x) for x in recs], dtype=torch.int64)
    if device is not None:
        cnt = cnt.to(device)
    counts = [torch.empty_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    counts = np.stack([c.cpu().numpy() for c in counts])            # [world, sources]
    item = CANDIDATE_DTYPE.itemsize
    width = max(int(counts.sum(1).max()), 1) * item
    buf = np.zeros(width, np.uint8)
    raw = np.concatenate([x.view(np.uint8) for x in recs]) if n_src else np.zeros(0, np.uint8)
    buf[:raw.size] = raw
    mine = torch.from_numpy(buf)
    if device is not None:
        mine = mine.to(device)
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine, group=group)
    per_rank = []
    for k in range(world):
        blob = parts[k].cpu().numpy()[:int(counts[k].sum()) * item].view(CANDIDATE_DTYPE)
        per_rank.append(np.split(blob, np.cumsum(counts[k])[:-1]) if n_src else [])
    return [np.concatenate([per_rank[k][s] for k in range(world)]) for s in range(n_src)]


def merge_gathered(params, tmpl_w: int, tmpl_h: int, cands: np.ndarray):
    """fpm_merge_candidates over gathered records (host only): the search's final s_SingleTargetMatch list."""
    from .matcher import merge_candidates

    return merge_candidates(params, tmpl_w, tmpl_h, cands)


def match_angle_sharded(matcher, source: np.ndarray, group=None, device=None):
    """One search of `source` split by angle over the ranks of `group`: this rank's matcher (bound to its GPU)
    searches its angle block, the candidate records are all-gathered, and every rank returns the full result
    list — identical to matcher.match(source) on one GPU."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    prev = matcher.getAngleShard()
    matcher.setAngleShard(rank, world)
    try:
        matcher.match(source)
        # None when the search did not run (empty source, unlearned template, size mismatch: TemplateMatcher.cpp:99-114);
        # those checks depend only on the source and the template, so every rank takes the same branch
        local = matcher.last_candidates_if_searched(0)
    finally:
        matcher.setAngleShard(*prev)   # later plain match() calls search the whole angle list again
    if local is None:
        return []
    full = gather_candidates(local, group=group, device=device)
    tw, th = matcher.template_level(0)[0].shape[::-1]
    return merge_gathered(matcher._params, tw, th, full)
