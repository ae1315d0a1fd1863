"""bench.py's reading of the committed PMC snapshots (CPU only): the per-workload traffic the `roofline.traffic` field
takes, the instruction-issue fractions of `roofline_issue`, and scripts/pmc_summary.py's per-grid split of a kernel
dispatched with several grid sizes."""
import csv
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


@pytest.mark.parametrize("workload,kernel", [("src7", "roi_warp"), ("config3", "top_ncc")])
def test_committed_snapshot_traffic(workload, kernel):
    """Each workload's dominant kernel has FETCH + WRITE bytes in its committed snapshot (the config3 one is
    k_top_mma's list launch only: its map-fallback launch is the separate k_top_map symbol)."""
    t = bench.pmc_traffic(kernel, workload)
    assert t is not None and t > 0
    c = bench.pmc_counters(kernel, workload)
    assert t == int(c["FETCH_BYTES(x2 corrected, B)"] + c["WRITE_BYTES(B)"])
    assert bench.pmc_traffic("top_map", "config3") is not None   # k_top_map has its own rows


def test_roofline_issue_fractions():
    """roofline_issue: VALU instructions x 2 cycles over 1024 SIMDs, LDS-array cycles over 256 CUs, matrix-pipe cycles
    over 1024 SIMDs, each against the launch time at 2.4 GHz; the largest is the bound."""
    c = bench.pmc_counters("top_ncc", "config3")
    avg_s = 700e-6
    r = bench.roofline_issue("top_ncc", "config3", avg_s)
    cyc = 2.4e9 * avg_s
    assert r["fracs"]["valu_issue"] == pytest.approx(c["SQ_INSTS_VALU"] * 2 / (1024 * cyc), abs=1e-4)
    assert r["fracs"]["lds"] == pytest.approx(c["SQ_LDS_IDX_ACTIVE"] / (256 * cyc), abs=1e-4)
    assert r["fracs"]["mfma_pipe"] == pytest.approx(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc), abs=1e-4)
    assert r["bound"] == max(r["fracs"], key=r["fracs"].get) and r["frac"] == r["fracs"][r["bound"]]
    assert r["per_wave"]["SQ_INSTS_MFMA"] > 0 and r["waves_per_launch"] == int(c["SQ_WAVES"])
    assert bench.roofline_issue("no_such_kernel", "config3", avg_s) is None
    assert bench.roofline_issue("top_ncc", "config3", 0.0) is None


def test_pmc_summary_grid_split(tmp_path):
    """A kernel with two grid sizes gets its aggregate row plus one row per grid; bench reads the aggregate."""
    d = tmp_path / "pass" / "x"
    d.mkdir(parents=True)
    rows = [("1", "k", "4096", "SQ_WAVES", "10"), ("2", "k", "4096", "SQ_WAVES", "30"),
            ("3", "k", "256", "SQ_WAVES", "2"), ("4", "j", "64", "SQ_WAVES", "5")]
    with open(d / "run_counter_collection.csv", "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Grid_Size", "Counter_Name", "Counter_Value"])
        w.writerows(rows)
    out = tmp_path / "summary.csv"
    subprocess.run([sys.executable, os.path.join(REPO, "scripts", "pmc_summary.py"), str(out), str(tmp_path / "pass")],
                   check=True)
    got = {(r["kernel"], r["counter"]): (int(r["dispatches"]), float(r["mean_per_dispatch"]))
           for r in csv.DictReader(open(out))}
    assert got[("k", "SQ_WAVES")] == (3, 14.0)
    assert got[("k @grid=4096", "SQ_WAVES")] == (2, 20.0)
    assert got[("k @grid=256", "SQ_WAVES")] == (1, 2.0)
    assert got[("j", "SQ_WAVES")] == (1, 5.0) and ("j @grid=64", "SQ_WAVES") not in got
