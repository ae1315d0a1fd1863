"""bench.py's multi-GPU launch contract on CPU (no GPU work: --dry-run exits before touching a device): `--gpus N`
outside torchrun starts N ranks itself, and a WORLD_SIZE that disagrees with --gpus is refused instead of reporting
a wrong n_gpus."""
import json
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(kw)
    return env


def test_gpus_2_spawns_two_ranks():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], capture_output=True, text=True,
                         timeout=240, env=_env())
    assert out.returncode == 0, out.stderr
    ranks = [json.loads(m) for m in re.findall(r"\{[^{}]*\}", out.stdout)]
    assert sorted((r["rank"], r["world"]) for r in ranks) == [(0, 2), (1, 2)]


def test_gpus_mismatch_is_refused():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--dry-run"], capture_output=True, text=True,
                         timeout=60, env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert out.returncode == 2 and "WORLD_SIZE" in out.stderr


def test_default_is_one_rank():
    out = subprocess.run([sys.executable, BENCH, "--dry-run"], capture_output=True, text=True, timeout=60, env=_env())
    assert out.returncode == 0 and json.loads(out.stdout) == {"rank": 0, "world": 1, "local_rank": 0,
                                                              "workload": "src7"}


def test_config3_shards_sources_over_ranks():
    """--workload config3 (BASELINE.json configs[3]): the 64 sources of the job split into contiguous blocks, one per
    rank the launcher starts (strong scaling over --gpus N)."""
    out = subprocess.run([sys.executable, BENCH, "--workload", "config3", "--gpus", "2", "--dry-run"],
                         capture_output=True, text=True, timeout=240, env=_env())
    assert out.returncode == 0, out.stderr
    ranks = sorted((r["rank"], r["world"], r["workload"], tuple(r["sources"]))
                   for r in (json.loads(m) for m in re.findall(r"\{[^{}]*\}", out.stdout)))
    assert ranks == [(0, 2, "config3", (0, 32)), (1, 2, "config3", (32, 64))]


def _bench_module():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_search_macs_follow_survey_formula():
    """roofline_mac's MAC count: |R_a| and n_ang come back out of B_top / B_ref exactly (a fake context whose
    stats and bytes are built from known map sizes and live counts)."""
    b = _bench_module()
    assert b.level_sizes(762, 521, 2) == [(762, 521), (381, 261), (191, 131)]
    src_wh, tmpl_wh, S, L, n3 = (4024, 3036), (762, 521), 2, 6, 3
    src, tm = b.level_sizes(*src_wh, L), b.level_sizes(*tmpl_wh, L)
    maps = [(70, 66), (71, 64), (69, 69)]                  # per angle, per source
    live = [60, 56, 48, 22, 22, 22]                         # batch totals entering layers L-1 .. 0
    b_top = S * sum(src[L][0] * src[L][1] + 4 * w * h for w, h in maps)
    layers = [tm[L - 1 - d] for d in range(L)]
    b_ref = sum(n * n3 * ((w + 6) * (h + 6) + w * h + 49 * 4) for n, (w, h) in zip(live, layers))

    class Ctx:
        def search_stats(self):
            return [len(maps), 99] + live

        def search_bytes(self):
            return 0, b_top, b_ref

    mt, mr = b.search_macs(Ctx(), src_wh, tmpl_wh, S)
    assert mt == S * sum(w * h for w, h in maps) * tm[L][0] * tm[L][1]
    assert mr == [n * n3 * 49 * w * h for n, (w, h) in zip(live, layers)]


def test_config4_shards_angles_over_ranks():
    """--workload config4 (BASELINE.json configs[4]): the 8-image Src5 set searched on every rank, each rank its block
    of the top-layer angle list (angle shard rank / world)."""
    out = subprocess.run([sys.executable, BENCH, "--workload", "config4", "--gpus", "2", "--dry-run"],
                         capture_output=True, text=True, timeout=240, env=_env())
    assert out.returncode == 0, out.stderr
    ranks = sorted((r["rank"], r["world"], r["workload"], tuple(r["angle_shard"]))
                   for r in (json.loads(m) for m in re.findall(r"\{[^{}]*\}", out.stdout)))
    assert ranks == [(0, 2, "config4", (0, 2)), (1, 2, "config4", (1, 2))]
