#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection CSVs: per kernel name, mean of each counter per dispatch.

usage: pmc_summary.py OUT.csv PASS_DIR [PASS_DIR ...]
Applies the gfx950 FETCH_SIZE correction (x2, MI355X_MICROARCH.md "HBM") in an extra FETCH_BYTES column;
FETCH_SIZE / WRITE_SIZE are reported by rocprofv3 in KiB.  A kernel dispatched with several grid sizes also gets one
entry per grid size ("<name> @grid=<threads>").
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    out = sys.argv[1]
    acc = defaultdict(lambda: defaultdict(float))     # kernel -> counter -> sum over dispatches
    disp = defaultdict(lambda: defaultdict(set))      # kernel -> counter -> dispatch ids
    grids = defaultdict(set)
    rows = []
    for d in sys.argv[2:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    rows.append((f, row))
                    grids[row["Kernel_Name"]].add(row["Grid_Size"])
    # a kernel launched with several grid sizes (e.g. k_top_mma: the list launch, one workgroup per unit, and the
    # map fallback's persistent grid) also gets one entry per grid: "<name> @grid=<threads>"
    for f, row in rows:
        k, c = row["Kernel_Name"], row["Counter_Name"]
        keys = [k] + ([f"{k} @grid={row['Grid_Size']}"] if len(grids[k]) > 1 else [])
        for kk in keys:
            acc[kk][c] += float(row["Counter_Value"])
            disp[kk][c].add((f, row["Dispatch_Id"]))
    counters = sorted({c for k in acc for c in acc[k]})
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel", "counter", "dispatches", "mean_per_dispatch"])
        for k in sorted(acc):
            for c in counters:
                if c in acc[k]:
                    n = len(disp[k][c])
                    w.writerow([k, c, n, f"{acc[k][c] / n:.6g}"])
            if "FETCH_SIZE" in acc[k]:
                n = len(disp[k]["FETCH_SIZE"])
                w.writerow([k, "FETCH_BYTES(x2 corrected, B)", n, f"{acc[k]['FETCH_SIZE'] / n * 1024 * 2:.6g}"])
            if "WRITE_SIZE" in acc[k]:
                n = len(disp[k]["WRITE_SIZE"])
                w.writerow([k, "WRITE_BYTES(B)", n, f"{acc[k]['WRITE_SIZE'] / n * 1024:.6g}"])


if __name__ == "__main__":
    main()
