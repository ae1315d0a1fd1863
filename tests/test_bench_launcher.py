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
    assert out.returncode == 0 and json.loads(out.stdout) == {"rank": 0, "world": 1, "local_rank": 0}
