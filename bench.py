#!/usr/bin/env python3
"""bench.py — BASELINE.json configs[1]: Src7 4024x3036 / Dst7 762x521, ToleranceAngle 180, TargetNum 3.

A step is one full TemplateMatcher::match pass (pyramid -> top-layer rotation sweep -> NCC -> peaks -> pyramid
refinement -> host filters) over a batch of ``--batch`` synthetic Src7 sources per GPU that are already
resident in HBM (staged before timing; the PCIe upload is not in ``value``), split over ``--contexts`` contexts
(one HIP stream each) that run as a stream of passes: a context relaunches as soon as its previous pass is
finished, so host post-processing overlaps device work.  Defaults: 192 sources over 3 contexts (round 5, one box,
alternated: 34.17k / 34.23k searches/s at 128, 34.38k / 34.43k at 160, 34.51k / 34.52k at 192, 33.67k at 240;
3 contexts beat 2 and 4 at every batch, profiles/r05f, r05g).  ``value`` = searches/s over all
ranks.  Multi-GPU: one process per GPU (torchrun), every rank searches its own sources (weak scaling, no
data-path collective); barrier + synchronize bracket the K timed steps and the max time over ranks is used.

Also reported: the dominant kernel's roofline (HIP events around every launch on the library's stream, in a
second pass of K steps over one context's share of the sources, so the timed pass carries no event overhead) and the
CPU baseline (the oracle restatement, single thread, on a bounded sample of the same workload, rank 0 at N=1 only).
``roofline_issue`` puts the same kernel's instruction counters (committed SQ passes of the workload's kernel pass,
scripts/pmc_bench.sh) against the chip's VALU issue, LDS-array and matrix-pipe cycles in its measured launch time.

Roofline bytes are SURVEY.md §8(d)'s algorithmic bytes, reported by the library per search (fpm_search_bytes) and per
kernel (fpm_profile_get): B_pyr + B_top + B_ref, where a refinement ROI costs its source footprint, the template
level and the 7x7 f32 scores; scratch this design writes between its kernels (sampled ROIs, row sums) is not
algorithmic and shows up only in `traffic` (PMC HBM bytes), so traffic / algorithmic bytes measures that overhead.
``roofline`` is the dominant kernel's (its §8(d) share per launch / its average launch time); ``roofline_search``
is the whole search's (bytes of all searches of the timed region / its wall time).  §8(d) also asks for the MAC
view: ``roofline_mac`` = the §8(d) MACs of every search of the timed region (top-layer maps x top template +
49 w_l h_l per live refinement ROI) / the wall time against the i8 MFMA dense peak, and ``roofline_corr`` = the
refinement correlation kernel's useful MACs per launch / its average launch time on the same peak.

``--workload config3`` measures BASELINE.json configs[3] instead: 64 synthetic 4096x4096 sources, one 512x512
template, +-180 deg at a 1 deg top-layer step (fpm_params.top_angle_step; the reference derives 7.125 deg,
TemplateMatcher.cpp:130), the 64 sources sharded over the --gpus N ranks (strong scaling: the job is fixed) and
every step's results all-gathered over RCCL inside the timed region (the report exchange of SURVEY.md §8(e)).

``python bench.py --gpus N`` with no torchrun environment starts N ranks itself (torch.distributed.run, one process
per GPU) before anything touches a GPU; under torchrun, --gpus must equal WORLD_SIZE.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "template matches/sec + ms/search, 4024×3036 src ±180°; HBM GB/s vs roofline"
README_MS_PER_SEARCH = 76.0          # README.md:45-48 (MFC build), BASELINE.md row 1
HBM_PEAK_GBS = 8000.0                # MI355X_MICROARCH.md chip table (spec)
PARAMS = dict(max_pos=3, tolerance_angle=180.0, score=0.7, min_reduce_area=256, max_overlap=0.0, use_simd=1)
# BASELINE.json configs[3]: TargetNum 1 per source (one pasted copy), +-180 at the stated 1 deg top step
C3_PARAMS = dict(max_pos=1, tolerance_angle=180.0, top_angle_step=1.0)
C3_SOURCES = 64
# BASELINE.json configs[4]: the Src5 rotation set (8 images), TargetNum 1, +-180, sub-pixel estimation
C4_PARAMS = dict(max_pos=1, tolerance_angle=180.0, subpixel=1)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# committed rocprofv3 --pmc snapshots of each workload's kernel pass (scripts/pmc_bench.sh TAG WORKLOAD)
TRAFFIC_CSV = {"src7": os.path.join(REPO, "profiles", "latest", "pmc_traffic.csv"),
               "config3": os.path.join(REPO, "profiles", "latest", "pmc_traffic_config3.csv")}
TRAFFIC_SOURCE = ("committed rocprofv3 --pmc snapshot {} (scripts/pmc_bench.sh: separate FETCH_SIZE / WRITE_SIZE "
                  "passes of bench.py --workload {} --kernel-pass-only, FETCH_SIZE doubled for gfx950, mean per "
                  "dispatch); not measured in this run")
ISSUE_SOURCE = ("committed rocprofv3 --pmc snapshot {} (scripts/pmc_bench.sh: two SQ passes of bench.py --workload {} "
                "--kernel-pass-only, mean per dispatch); counters not measured in this run, launch time measured live")
SIMDS, CUS, CLOCK_GHZ = 1024, 256, 2.4   # MI355X_MICROARCH.md: 256 CUs x 4 SIMDs, 2.4 GHz peak engine clock
VALU_ISSUE_CYCLES = 2                    # a wave64 VALU instruction issues over 2 cycles (32 lanes per cycle)


def pmc_counters(kernel, workload):
    """Per-launch means of every counter of `kernel` (a profiling index name, _lib.KERNEL_NAMES) in the committed PMC
    snapshot of `workload`: every instantiation of the kernel's first matching symbol, weighted by its dispatches (the
    same launches the kernel pass averages over).  {} if not collected."""
    import csv

    from fastest_image_pattern_matching_amd import _lib as L

    path = TRAFFIC_CSV.get(workload)
    if not path or not os.path.exists(path):
        return {}
    rows = {}   # kernel name -> counter -> (mean per dispatch, dispatches)
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if " @grid=" in row["kernel"]:
                continue   # per-grid split entries (the aggregate row holds every dispatch)
            rows.setdefault(row["kernel"], {})[row["counter"]] = (float(row["mean_per_dispatch"]),
                                                                  int(row["dispatches"]))
    for sym in L.KERNEL_SYMBOLS.get(kernel, []):
        names = [n for n in rows if n.startswith(f"fpm::{sym}(") or n.startswith(f"void fpm::{sym}<")]
        if not names:
            continue
        out = {}
        for c in {c for n in names for c in rows[n]}:
            tot = sum(rows[n][c][0] * rows[n][c][1] for n in names if c in rows[n])
            cnt = sum(rows[n][c][1] for n in names if c in rows[n])
            out[c] = tot / cnt
        return out
    return {}


def pmc_traffic(kernel, workload="src7"):
    """HBM bytes per launch of `kernel` from the committed PMC snapshot of `workload` (FETCH_SIZE x2 for gfx950 +
    WRITE_SIZE, per-dispatch means); None if not collected for this kernel."""
    c = pmc_counters(kernel, workload)
    f, w = c.get("FETCH_BYTES(x2 corrected, B)"), c.get("WRITE_BYTES(B)")
    return int(f + w) if f is not None and w is not None else None


def roofline_issue(kernel, workload, avg_s):
    """The dominant kernel against the chip's issue and pipe capacities over its measured launch time: VALU issue
    (SQ_INSTS_VALU x 2 cycles per wave64 instruction over 1024 SIMDs), the LDS array (SQ_LDS_IDX_ACTIVE over 256 CUs)
    and the matrix pipe (SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs), from the committed SQ passes of the same kernel
    pass (scripts/pmc_bench.sh); the largest fraction is the bound.  None if not collected."""
    c = pmc_counters(kernel, workload)
    if "SQ_INSTS_VALU" not in c or avg_s <= 0:
        return None
    cyc = CLOCK_GHZ * 1e9 * avg_s
    fr = {"valu_issue": c["SQ_INSTS_VALU"] * VALU_ISSUE_CYCLES / (SIMDS * cyc)}
    if "SQ_LDS_IDX_ACTIVE" in c:
        fr["lds"] = c["SQ_LDS_IDX_ACTIVE"] / (CUS * cyc)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
        fr["mfma_pipe"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * cyc)
    bound = max(fr, key=fr.get)
    per_wave = {k: round(c[k] / c["SQ_WAVES"], 1) for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
                                                            "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU", "SQ_INSTS_MFMA")
                if k in c and c.get("SQ_WAVES")}
    return {"bound": bound, "frac": round(fr[bound], 4), "fracs": {k: round(v, 4) for k, v in fr.items()},
            "kernel": kernel, "avg_launch_us": round(avg_s * 1e6, 3), "waves_per_launch": int(c.get("SQ_WAVES", 0)),
            "per_wave": per_wave,
            "definition": "issue / pipe cycles the kernel's counters need per launch / the cycles the chip has in its "
                          "measured launch time (2.4 GHz): VALU 2 cycles per wave64 instruction per SIMD, LDS array "
                          "cycles per CU, matrix-pipe busy cycles per SIMD",
            "source": ISSUE_SOURCE.format(os.path.relpath(TRAFFIC_CSV[workload], REPO), workload)}


def make_sources(templ, n, seed0):
    from fastest_image_pattern_matching_amd import synth

    return [synth.src7_scene(templ, seed=seed0 + i)[0] for i in range(n)]


def _time_oracle(templ, src, budget_s, params, lib_path=None, threads=1):
    """Searches/s of the oracle on repeated searches of one source: `threads` OracleMatcher objects searching
    concurrently (ctypes releases the GIL around each C call), each until the budget is spent."""
    import threading

    from tests import oracle

    path = lib_path or oracle.ORACLE_LIB
    ms = [oracle.OracleMatcher(path).set(**params) for _ in range(threads)]
    counts = [0] * threads
    start = threading.Barrier(threads + 1)

    def work(i):
        ms[i].learnPattern(templ)
        ms[i].match(src)               # warm, outside the timed region
        start.wait()
        t0 = time.perf_counter()
        while True:
            ms[i].match(src)
            counts[i] += 1
            if time.perf_counter() - t0 >= budget_s or counts[i] >= 200:
                break

    th = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
    for t in th:
        t.start()
    start.wait()
    t0 = time.perf_counter()
    for t in th:
        t.join()
    el = time.perf_counter() - t0
    return sum(counts), el


def host_cores():
    """Threads this process may use, capped at the GPU box's 16-core share."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    return max(1, min(16, n))


def cpu_baseline(templ, src, budget_s, params, what):
    """Oracle (CPU port of the reference, SSE2 IM_Conv) on repeated searches of one source: the headline is
    one thread with the parity build's flags (the reference is single-threaded: its OpenMP code is dead); the
    variants are the reference's release flags (-ffast-math, CMakeLists.txt:67) on one thread and the parity
    build on every core this process may use (independent searches in parallel, capped at the GPU box's
    16-core share)."""
    from tests import oracle

    n, el = _time_oracle(templ, src, 0.5 * budget_s, params)
    base = {"value": n / el, "unit": "searches/s", "cores": 1, "kind": "port",
            "sample": f"{n} sequential searches of one {what} source ({el:.1f} s), oracle/fpm_oracle.cpp "
                      f"-O3 SSE2, single thread (the reference's OpenMP code is dead)"}
    variants = []
    if os.path.exists(oracle.ORACLE_LIB_FAST):
        n, el = _time_oracle(templ, src, 0.25 * budget_s, params, oracle.ORACLE_LIB_FAST)
        variants.append({"value": n / el, "unit": "searches/s", "cores": 1, "flags": "-O3 -ffast-math -msse2",
                         "sample": f"{n} sequential searches ({el:.1f} s)"})
    ncores = host_cores()
    n, el = _time_oracle(templ, src, 0.25 * budget_s, params, threads=ncores)
    variants.append({"value": n / el, "unit": "searches/s", "cores": ncores, "flags": "-O3 -msse2 (parity build)",
                     "sample": f"{n} searches on {ncores} threads, one oracle object each ({el:.1f} s)"})
    return base, variants


def oracle_verify(templ, sources, refs, params):
    """The timed work against the parity oracle: the oracle's search of every given source equals the GPU results of
    that source field for field (the GPU results are the reference pass's, which the timed pass reproduces exactly,
    `verify`).  Searches run on the host's cores (one oracle object per thread; ctypes releases the GIL).  Test
    infrastructure as the checker only; returns the number of sources checked, exits 4 on a mismatch."""
    import threading

    from tests import oracle

    nth = min(host_cores(), len(sources))
    bad = []
    nxt = iter(range(len(sources)))
    lock = threading.Lock()

    def work():
        o = oracle.OracleMatcher().set(**params)
        assert o.learnPattern(templ)
        while True:
            with lock:
                i = next(nxt, None)
            if i is None:
                return
            exp = o.match(sources[i])
            got = [x.as_tuple() for x in refs[i]]
            if got != exp:
                with lock:
                    bad.append((i, got, exp))

    th = [threading.Thread(target=work) for _ in range(nth)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if bad:
        i, got, exp = min(bad, key=lambda b: b[0])
        log(f"[bench] GPU results differ from the oracle on {len(bad)} timed source(s); first, source {i}:\n"
            f"GPU    {got}\noracle {exp}")
        sys.exit(4)
    return len(sources)


def kernel_pass(m, sources, steps, L, workload="src7"):
    """Kernel-level pass: one context over its share of the step's sources (the same launches as one context's pass
    in the timed run), eager launches with HIP events around each kernel on the library's stream (the kernels' own
    durations, not time shared with another context's stream).  Returns the per-kernel table and the roofline
    object of the dominant kernel."""
    m.stage(sources)
    m.match_staged_array()
    m.profile(True)
    m.profile_reset()
    for _ in range(steps):
        m.match_staged_array()
    m.profile(False)
    kern = {}
    for k, name in enumerate(L.KERNEL_NAMES):
        ms, launches, b = m.profile_get(k)
        if launches:
            kern[name] = {"ms_total": ms, "launches": launches, "bytes": b}
    dom = max(kern, key=lambda k: kern[k]["ms_total"])
    d = kern[dom]
    avg_s = d["ms_total"] / d["launches"] * 1e-3
    bytes_per_launch = d["bytes"] / d["launches"]
    achieved = bytes_per_launch / avg_s / 1e9 if avg_s > 0 else 0.0
    traffic = pmc_traffic(dom, workload)
    roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic, "kernel": dom,
                "avg_launch_us": round(avg_s * 1e6, 3), "algorithmic_bytes_per_launch": int(bytes_per_launch),
                "bytes_definition": "SURVEY.md §8(d) share of this kernel per launch (fpm_profile_get)",
                "traffic_source": (TRAFFIC_SOURCE.format(os.path.relpath(TRAFFIC_CSV[workload], REPO), workload)
                                   if traffic is not None else None)}
    return kern, roofline, roofline_issue(dom, workload, avg_s)


I8_MFMA_PEAK_TOPS = 5000.0           # MI355X_MICROARCH.md matrix-core table: I8 at 2x the BF16 rate (~2.5 PF dense)


def level_sizes(w, h, n):
    """(w_l, h_l) of pyramid levels 0..n (cv::pyrDown: ((w + 1) / 2, (h + 1) / 2))."""
    out = [(w, h)]
    for _ in range(n):
        w, h = (w + 1) // 2, (h + 1) // 2
        out.append((w, h))
    return out


def search_macs(ctx, src_wh, tmpl_wh, n_sources):
    """SURVEY.md §8(d) MACs of the context's last search pass (all its sources), from its live counts:
    MAC = sum_angles |R_a| w_L h_L + sum_l sum_live n_ang_l 49 w_l h_l.  |R_a| (top-layer map sizes) and n_ang_l come
    back out of the same pass's B_top and B_ref (fpm_search_bytes), so nothing is re-derived from the plan.
    Returns (mac_top, [mac_ref per refinement layer, top-most first])."""
    st = ctx.search_stats()
    nang, L = st[0], len(st) - 2
    live = st[2:2 + L]
    src = level_sizes(*src_wh, L)
    tm = level_sizes(*tmpl_wh, L)
    _, b_top, b_ref = ctx.search_bytes()
    sum_r = (b_top - n_sources * nang * src[L][0] * src[L][1]) // 4
    mac_top = sum_r * tm[L][0] * tm[L][1]
    layers = [tm[L - 1 - d] for d in range(L)]
    denom = sum(n * ((w + 6) * (h + 6) + w * h + 49 * 4) for n, (w, h) in zip(live, layers))
    n3 = round(b_ref / denom) if denom else 0
    return mac_top, [n * n3 * 49 * w * h for n, (w, h) in zip(live, layers)]


def cpu_identity():
    """CPU model (/proc/cpuinfo, as lscpu reports it) and the host's online CPU count."""
    model = None
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cpu_model": model, "nproc": os.cpu_count()}


def spawn_ranks(args):
    """`--gpus N` outside torchrun: run this script under torch.distributed.run with N processes (one per GPU) and
    return its exit status.  Nothing here touches a GPU; the ranks start fresh."""
    import socket
    import subprocess

    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    log(f"[bench] starting {args.gpus} ranks: {' '.join(cmd)}")
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", choices=("src7", "config3", "config4"), default="src7",
                    help="src7: BASELINE.json configs[1], the headline (default); config3: configs[3], 64 x 4096^2 "
                         "sources at a 1 deg top step sharded over the ranks; config4: configs[4], the 8-image Src5 "
                         "rotation set with every search's top-layer angles sharded over the ranks")
    ap.add_argument("--batch", type=int, default=192, help="src7: sources searched per GPU per step")
    ap.add_argument("--sources", type=int, default=C3_SOURCES,
                    help="config3: sources of the whole job per step, sharded over the ranks")
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU-baseline work (0 = skip)")
    ap.add_argument("--contexts", type=int, default=3, help="concurrent contexts (HIP streams) per GPU")
    ap.add_argument("--skip-latency", action="store_true",
                    help="skip the single-search latency probe (PMC runs: only batch dispatches)")
    ap.add_argument("--dry-run", action="store_true",
                    help="print each rank's (rank, world) and exit before any GPU work (launcher test)")
    ap.add_argument("--kernel-pass-only", action="store_true",
                    help="run only the per-kernel pass (one context, the whole batch, K eager steps) and print its "
                         "kernel table + roofline: the command whose rocprofv3 --kernel-trace --stats averages are "
                         "directly comparable to roofline.avg_launch_us")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a wrong n_gpus")
        sys.exit(2)
    if args.dry_run:
        # one write of the whole line (< PIPE_BUF): the ranks share the launcher's stdout and must not interleave
        line = {"rank": rank, "world": world, "local_rank": local, "workload": args.workload}
        if args.workload == "config3":
            from fastest_image_pattern_matching_amd.sharding import shard_range

            line["sources"] = list(shard_range(args.sources, world, rank))
        if args.workload == "config4":
            line["angle_shard"] = [rank, world]
        sys.stdout.write(json.dumps(line) + "\n")
        sys.stdout.flush()
        return
    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    def barrier_sync():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    from fastest_image_pattern_matching_amd import TemplateMatcher, sharding, synth
    from fastest_image_pattern_matching_amd import _lib as L

    if args.workload == "config4":
        return run_config4(args, world, rank, local, dist, barrier_sync)

    if args.workload == "src7":
        params, scaling, what = PARAMS, "weak", "Src7 surrogate"
        templ = synth.load_templates()["Dst7"]
        log(f"[rank {rank}] generating {args.batch} Src7 surrogate sources")
        sources = make_sources(templ, args.batch, 7 + 1000 * rank)
        per_rank, total = args.batch, args.batch * world
    else:
        params, scaling, what = C3_PARAMS, "strong", "configs[3] 4096x4096"
        lo, hi = sharding.shard_range(args.sources, world, rank)
        if hi - lo < 1:
            log(f"[bench] {args.sources} sources leave rank {rank} of {world} without a source")
            sys.exit(2)
        log(f"[rank {rank}] generating configs[3] sources {lo}..{hi - 1} of {args.sources}")
        sources, templ = synth.batch_sources(hi - lo, first=lo)
        per_rank, total = hi - lo, args.sources
        args.batch = per_rank

    m = TemplateMatcher(local)
    for k, v in params.items():
        setattr(m._params, k, v)
    assert m.learnPattern(templ)
    # G contexts (one HIP stream each) on this GPU, each holding batch / G of the sources (see run() below)
    G = max(1, min(args.contexts, args.batch))
    chunks = [sources[i * args.batch // G:(i + 1) * args.batch // G] for i in range(G)]
    # the kernel pass is one context's share of the step (chunks[0]), eager: the launches of the timed run's passes
    if args.kernel_pass_only:
        kern, roofline, issue = kernel_pass(m, chunks[0], args.steps, L, args.workload)
        print(json.dumps({"kernel_pass_only": True, "steps": args.steps, "sources_per_step": len(chunks[0]),
                          "kernels": kern, "roofline": roofline, "roofline_issue": issue}), flush=True)
        return
    # single-search latency (host upload included) for the record, after one warm call builds the plan
    lat_e2e = lat_split = None
    if not args.skip_latency:
        m.match(sources[0])
        lat, splits = [], []
        for _ in range(9):
            t0 = time.perf_counter()
            m.match(sources[0])
            lat.append(time.perf_counter() - t0)
            splits.append(m.profile_last())
        i = int(np.argsort(lat)[len(lat) // 2])
        lat_e2e = lat[i]
        dev, host, call = splits[i]
        # fpm_profile_last: device = events around the device pass, host = the reference-order tail, call = launch to
        # finish; the rest of the end-to-end time is the 12.2 MB host->HBM upload and the call overhead
        lat_split = {"device": round(dev, 4), "host_tail": round(host, 4),
                     "upload_and_call": round(lat_e2e * 1e3 - call, 4)}
    # a step launches every context's device pass, then finishes them in order, so host post-processing and the upper
    # pyramid layers' latency-bound kernels of one context overlap device work of the others
    ctxs = [m] + [TemplateMatcher(local) for _ in range(G - 1)]
    for c, ch in zip(ctxs, chunks):
        for k, v in params.items():
            setattr(c._params, k, v)
        if c is not m:
            assert c.learnPattern(templ)
        c.stage(ch)
    ref = [r for c in ctxs for r in c.match_staged()]   # object results once, for the report and checks
    views = [c.match_staged_array() for c in ctxs]
    assert [len(r) for r in ref] == [int(x) for cnt, _ in views for x in cnt]

    # config3 on several ranks: every step's results are all-gathered (RCCL) into the whole job's report inside the
    # timed region -- the report exchange SURVEY.md §8(e) names for the sharded batch
    exchange = dist is not None and args.workload == "config3"
    cap = max(16, params["max_pos"] + 5)
    gathered = []

    def run(k_steps):
        # K passes per context as a stream: each context relaunches its next pass as soon as it has finished (host
        # post-processing) the previous one, so the device never waits for the host between steps.  Returns every
        # context's last (counts, results) views (valid until that context's next pass).
        last = [None] * len(ctxs)
        for c in ctxs:
            c.match_staged_launch()
        for k in range(k_steps):
            for i, c in enumerate(ctxs):
                last[i] = c.match_staged_finish_array()
                if k + 1 < k_steps:
                    c.match_staged_launch()
            if exchange:
                gathered[:] = [sharding.gather_result_arrays(last, total, cap, device=torch.device("cuda", local))]
        return last

    def verify(last):
        """Every source's results of the last timed pass equal the reference pass's, field for field."""
        got = []
        for cnt, arr in last:
            got += [[tuple(float(v) for v in arr[s_, i]) for i in range(int(cnt[s_]))] for s_ in range(len(cnt))]
        return got == [[r.as_tuple() for r in rr] for rr in ref]

    run(args.warmup)
    log(f"[rank {rank}] warm; timing {args.steps} steps x {args.batch} {what} sources over {G} context(s)")

    barrier_sync()
    t0 = time.perf_counter()
    last = run(args.steps)   # K complete device passes + host finishes (C++) per context
    barrier_sync()
    elapsed = time.perf_counter() - t0
    # the work just timed must be the work reported: its last pass per context equals the reference pass
    if not verify(last):
        log(f"[rank {rank}] timed pass results differ from the reference pass")
        sys.exit(3)
    res = ref
    dev_ms, host_ms, call_ms = m.profile_last()
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # the report exchange of the sharded path (sharding.gather_results of the reference pass, outside the timed
    # region); config3's timed exchange of the last step must equal it
    if dist is not None:
        full = sharding.gather_results([[r.as_tuple() for r in rr] for rr in res], total, cap=64,
                                       device=torch.device("cuda", local))
        n_matches = [len(r) for r in full]
        if exchange:
            cnt, arr = gathered[0]
            if [[tuple(float(v) for v in arr[i, j]) for j in range(int(cnt[i]))] for i in range(total)] != full:
                log(f"[rank {rank}] the timed all-gather differs from the reference pass's report")
                sys.exit(3)
    else:
        n_matches = [len(r) for r in res]

    # §8(d) algorithmic bytes of one step on this rank (each context's last pass covers its share of the batch)
    b_pyr = b_top = b_ref = 0
    for c in ctxs:
        bp, bt, br = c.search_bytes()
        b_pyr, b_top, b_ref = b_pyr + bp, b_top + bt, b_ref + br
    step_bytes = b_pyr + b_top + b_ref
    if dist is not None:
        t = torch.tensor([step_bytes], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t)
        step_bytes = float(t.item())
    search_gbs = step_bytes * args.steps / elapsed / 1e9
    roofline_search = {"bound": "hbm", "achieved": round(search_gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": round(search_gbs / HBM_PEAK_GBS, 5),
                       "bytes_per_search": {"B_pyr": b_pyr // args.batch, "B_top": b_top // args.batch,
                                            "B_ref": b_ref // args.batch},
                       "definition": "SURVEY.md §8(d) B_pyr + B_top + B_ref of every search in the timed region "
                                     "(fpm_search_bytes, live counts of this workload) / the timed wall time"}

    # the same search on the §8(d) MAC count, against the i8 MFMA peak (the top-layer NCC runs on v_dot4, the
    # refinement correlation on the matrix cores)
    src_wh = (sources[0].shape[1], sources[0].shape[0])
    tmpl_wh = (templ.shape[1], templ.shape[0])
    step_macs = 0
    for c, ch in zip(ctxs, chunks):
        mt, mr = search_macs(c, src_wh, tmpl_wh, len(ch))
        step_macs += mt + sum(mr)
    if dist is not None:
        t = torch.tensor([float(step_macs)], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t)
        step_macs = float(t.item())
    search_tops = 2.0 * step_macs * args.steps / elapsed / 1e12
    roofline_mac = {"bound": "mfma", "achieved": round(search_tops, 3), "peak": I8_MFMA_PEAK_TOPS, "unit": "TOPS",
                    "frac": round(search_tops / I8_MFMA_PEAK_TOPS, 5),
                    "mac_per_search": int(step_macs // total),
                    "definition": "SURVEY.md §8(d) MAC of every search in the timed region (top-layer |R_a| w_L h_L + "
                                  "49 w_l h_l per live refinement ROI; 2 ops per MAC) / the timed wall time, vs the "
                                  "i8 MFMA dense peak"}

    kern, roofline, issue = kernel_pass(m, chunks[0], args.steps, L, args.workload)
    # the refinement correlation kernel (k_roi_corr: the layers whose template is too large for k_roi_small, the
    # lowest ones) on its useful MACs per launch -- the banded GEMM also computes the (t, s) pairs outside the band
    roofline_corr = None
    if "roi_corr" in kern:
        n_corr = kern["roi_corr"]["launches"] // args.steps
        _, mr = search_macs(m, src_wh, tmpl_wh, len(chunks[0]))
        if n_corr > 0:
            corr_macs = sum(mr[len(mr) - n_corr:]) / n_corr
            avg_s = kern["roi_corr"]["ms_total"] / kern["roi_corr"]["launches"] * 1e-3
            tops = 2.0 * corr_macs / avg_s / 1e12
            roofline_corr = {"bound": "mfma", "achieved": round(tops, 3), "peak": I8_MFMA_PEAK_TOPS, "unit": "TOPS",
                             "frac": round(tops / I8_MFMA_PEAK_TOPS, 5), "kernel": "roi_corr",
                             "avg_launch_us": round(avg_s * 1e6, 3), "useful_mac_per_launch": int(corr_macs)}

    searches = total * args.steps
    value = searches / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    if args.workload == "src7":
        config = {
            "workload": "Src7 surrogate (4024x3036, 235+N(0,2) background, 3 rotated Dst7 762x521 copies at the "
                        "README poses), ToleranceAngle 180, TargetNum 3, Score 0.7, MinReduceArea 256, Overlap 0, "
                        "SIMD fold on",
            "sources_per_gpu_per_step": args.batch,
            "global_batch": total,
            "parallelism": f"sources sharded over {world} GPU(s), one process per GPU; {G} concurrent contexts "
                           f"(HIP streams) per GPU",
            "contexts_per_gpu": G,
        }
    else:
        config = {
            "workload": "BASELINE.json configs[3]: synthetic 4096x4096 sources (box-blurred uniform noise), one "
                        "512x512 template (the centre crop of source 0, re-pasted into every source at a seeded "
                        "angle and centre), ToleranceAngle 180 at a 1 deg top-layer step (fpm_params."
                        "top_angle_step, 361 angles; the reference derives 7.125 deg), TargetNum 1, Score 0.7, "
                        "MinReduceArea 256",
            "sources_per_step": total,
            "sources_this_gpu": per_rank,
            "global_batch": total,
            "parallelism": f"{total} sources sharded over {world} GPU(s) (contiguous blocks), one process per GPU; "
                           f"{G} concurrent contexts (HIP streams) per GPU; "
                           + ("every step's results all-gathered over RCCL inside the timed region" if exchange
                              else "one rank: no exchange"),
            "contexts_per_gpu": G,
        }
    # the README's 76 ms is one Src7 search's latency on a CPU: vs_baseline_latency (one search, host array in,
    # results out) is the like-for-like ratio; vs_baseline divides batch throughput by that single-search time
    readme_ms = README_MS_PER_SEARCH if args.workload == "src7" else None
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "searches/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": round(value / (1000.0 / readme_ms), 3) if readme_ms else None,
        "dtype": "u8",
        "data": "synthetic",
        "config": config,
        "ms_per_search": round(elapsed * 1e3 / (args.batch * args.steps), 4),
        "last_step_split_ms_ctx0": {"device": round(dev_ms, 4), "host_finish": round(host_ms, 4),
                                    "launch_to_finish": round(call_ms, 4)},
        "single_search_ms_end_to_end": round(lat_e2e * 1e3, 3) if lat_e2e is not None else None,
        "single_search_split_ms": lat_split,
        "vs_baseline_latency": (round(readme_ms / (lat_e2e * 1e3), 2) if readme_ms and lat_e2e is not None
                                else None),
        "vs_baseline_note": ("vs_baseline_latency = README Src7 76 ms / this single search end to end (like for "
                             "like); vs_baseline = batch throughput / (1 / 76 ms), not like for like" if readme_ms
                             else "no published number for this config"),
        "timed_results_verified": True,
        "matches_per_search": n_matches,
        "kernels": kern,
        "roofline": roofline,
        "roofline_issue": issue,
        "roofline_search": roofline_search,
        "roofline_mac": roofline_mac,
        "roofline_corr": roofline_corr,
    }
    if world == 1 and rank == 0 and args.cpu_budget > 0:
        # the CPU leg first checks the timed work against the oracle: the reference pass (== the timed pass, verify)
        # equals the oracle on every timed source, field for field; exit 4 on any difference
        nver = oracle_verify(templ, sources, ref, params)   # exits 4 on a mismatch
        out["oracle_verified"] = nver == len(sources)
        out["oracle_verified_sources"] = f"{nver}/{len(sources)}"
        out["oracle_verified_detail"] = (
            "every timed source: GPU results == oracle/fpm_oracle.cpp, every s_SingleTargetMatch field bit-identical "
            "(else exit 4)")
        log("[rank 0] CPU baseline (oracle restatement: 1 thread, fast-math 1 thread, all cores)")
        out["cpu_baseline"], out["cpu_baseline_variants"] = cpu_baseline(templ, sources[0], args.cpu_budget, params,
                                                                         what)
        out["cpu_baseline"].update(cpu_identity())
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def run_config4(args, world, rank, local, dist, barrier_sync):
    """BASELINE.json configs[4]: the 8-image Src5 rotation set, sub-pixel estimation, every image's search split by
    top-layer angle over the ranks (sharding.match_angle_sharded's protocol for the whole set at
    once).  One step = the 8 searches: every rank runs the device pass over the 8 staged images for its angle block
    (fpm_set_angle_shard; one context), the candidate records of all 8 are all-gathered over RCCL (two collectives:
    counts, records), and every rank merges each image's records in rank order on the host (fpm_merge_candidates:
    the reference's sort, filters and sub-pixel fit) -- all inside the timed region.  `value` = 8 searches per step /
    the max step time over ranks (strong scaling: the job is fixed as N grows)."""
    import torch

    from fastest_image_pattern_matching_amd import TemplateMatcher, sharding, synth
    from fastest_image_pattern_matching_amd.matcher import merge_candidates

    params = C4_PARAMS
    sources, templ = synth.src5_set()
    # two contexts (HIP streams), each with the whole set staged, run the steps as a stream: while one context's
    # device pass runs, the other's records are exchanged and merged on the host (the step is otherwise host-bound:
    # 0.15 ms of device pass + ~0.1 ms of exchange and merge, profiles/r06_end3)
    G = 2
    ctxs = [TemplateMatcher(local) for _ in range(G)]
    for m in ctxs:
        for k, v in params.items():
            setattr(m._params, k, v)
        assert m.learnPattern(templ)
        m.stage(sources)
    m = ctxs[0]
    ref = [[r.as_tuple() for r in rr] for rr in m.match_staged()]   # the unsharded search of the set, for the checks
    for c in ctxs:
        c.setAngleShard(rank, world)
    tw, th = templ.shape[1], templ.shape[0]
    device = torch.device("cuda", local) if dist is not None else None

    def finish(c):
        local_c = c.match_staged_candidates_finish()
        full = sharding.gather_candidates_batch(local_c, device=device) if dist is not None else local_c
        return [[r.as_tuple() for r in merge_candidates(c._params, tw, th, x)] for x in full]

    def run(n_steps):
        # n_steps passes of the set, context i taking passes i, i + G, ...; every rank runs the same sequence, so the
        # collectives pair up
        res = None
        for i in range(min(G, n_steps)):
            ctxs[i].match_staged_launch()
        for k in range(n_steps):
            c = ctxs[k % G]
            res = finish(c)
            if k + G < n_steps:
                c.match_staged_launch()
        return res

    run(args.warmup)
    log(f"[rank {rank}] warm; timing {args.steps} steps of the 8-image Src5 set over {G} contexts, angle shard "
        f"{rank}/{world}")
    barrier_sync()
    t0 = time.perf_counter()
    res = run(args.steps)
    barrier_sync()
    elapsed = time.perf_counter() - t0
    if res != ref:
        log(f"[rank {rank}] the angle-sharded step's results differ from the unsharded search of the set")
        sys.exit(3)
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    value = len(sources) * args.steps / elapsed
    out = {
        "metric": METRIC, "value": round(value, 3), "unit": "searches/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": "BASELINE.json configs[4]: Src5 rotation set surrogate (Dst5 160x159 pasted at 0, 45, "
                               "..., 315 deg into one 640x480 N(60, 10) background), TargetNum 1, ToleranceAngle 180, "
                               "sub-pixel estimation",
                   "sources_per_step": len(sources), "global_batch": len(sources),
                   "parallelism": f"every search's top-layer angle list split into {world} contiguous blocks, one per "
                                  f"GPU (one process per GPU); candidate records all-gathered "
                                  + ("over RCCL" if dist is not None else "(one rank: none)")
                                  + f" and merged on every rank's host inside the timed region; the steps as a stream "
                                    f"over {G} contexts (one's device pass overlaps the other's exchange and merge)",
                   "contexts_per_gpu": G},
        "ms_per_search": round(elapsed * 1e3 / (len(sources) * args.steps), 4),
        "timed_results_verified": True,
        "matches_per_search": [len(r) for r in res],
        "vs_baseline_note": "no published number for this config",
    }
    if world == 1 and rank == 0 and args.cpu_budget > 0:
        from fastest_image_pattern_matching_amd.matcher import SingleTargetMatch

        refs = [[SingleTargetMatch.from_row(np.array(r)) for r in rr] for rr in res]
        nver = oracle_verify(templ, sources, refs, params)   # exits 4 on a mismatch
        out["oracle_verified"] = nver == len(sources)
        out["oracle_verified_sources"] = f"{nver}/{len(sources)}"
        out["cpu_baseline"], out["cpu_baseline_variants"] = cpu_baseline(templ, sources[0], args.cpu_budget, params,
                                                                         "Src5 set")
        out["cpu_baseline"].update(cpu_identity())
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
