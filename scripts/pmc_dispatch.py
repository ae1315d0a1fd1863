#!/usr/bin/env python3
"""Per-dispatch counter values of one kernel from rocprofv3 --pmc counter_collection CSVs, in dispatch order.

usage: pmc_dispatch.py KERNEL_SUBSTRING PASS_DIR [PASS_DIR ...]
One line per dispatch (pass directory, dispatch id, counters).  The refinement kernels run once per pyramid layer
per search pass (layers L-1 .. 0 in order), so consecutive lines of one pass are consecutive layers.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    pat = sys.argv[1]
    vals = defaultdict(dict)   # (pass dir, dispatch id) -> counter -> value (summed over dimensions)
    for d in sys.argv[2:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if pat not in row["Kernel_Name"]:
                        continue
                    key = (d, int(row["Dispatch_Id"]))
                    c = row["Counter_Name"]
                    vals[key][c] = vals[key].get(c, 0.0) + float(row["Counter_Value"])
    counters = sorted({c for v in vals.values() for c in v})
    print("pass dispatch " + " ".join(counters))
    for key in sorted(vals):
        print(os.path.basename(key[0].rstrip("/")), key[1],
              " ".join(f"{vals[key].get(c, float('nan')):.4g}" for c in counters))


if __name__ == "__main__":
    main()
