#!/usr/bin/env python3
"""Per-dispatch timeline of the last complete search pass in a rocprofv3 kernel trace (run_kernel_trace.csv):
kernel, start offset, duration and gap to the previous dispatch, delimited by k_pack (one per pass)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_pack" in r["Kernel_Name"]]
a, b = idx[-2] + 1, idx[-1] + 1
prev_end = int(rows[a - 1]["End_Timestamp"])
t0 = int(rows[a]["Start_Timestamp"])
busy = 0.0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fpm::", "")
    print(f"{name:28s} start {(s - t0) / 1000:8.1f} dur {(e - s) / 1000:8.1f} gap {(s - prev_end) / 1000:6.1f}")
    busy += (e - s) / 1000
    prev_end = e
print(f"pass {(prev_end - t0) / 1000:.1f} us, kernels {busy:.1f} us")
