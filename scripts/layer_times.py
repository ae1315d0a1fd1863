"""Per-launch-position kernel durations from a rocprofv3 kernel trace of bench.py --kernel-pass-only: for every kernel,
the mean duration of its k-th launch within a pass (e.g. k_roi_warp's layer 2 / 1 / 0 launches).  Profiling aid.

    python scripts/layer_times.py gpurun_out/prof_TAG/run_kernel_trace.csv
"""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
short = lambda n: re.sub(r"\(.*", "", n).replace("void ", "").replace("fpm::", "")  # noqa: E731
# a pass starts at the first pyramid launch after a k_pack (or at the start)
passes, cur = [], []
for r in rows:
    n = short(r["Kernel_Name"])
    if n.startswith("__amd"):
        continue
    if n.startswith("k_pyr_down") and cur and short(cur[-1]["Kernel_Name"]).startswith("k_pack"):
        passes.append(cur)
        cur = []
    cur.append(r)
if cur:
    passes.append(cur)
acc = defaultdict(list)
for p in passes[1:]:
    seen = defaultdict(int)
    for r in p:
        n = short(r["Kernel_Name"])
        acc[(n, seen[n])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
        seen[n] += 1
for (n, k), v in sorted(acc.items(), key=lambda kv: -sum(kv[1]) / len(kv[1])):
    print(f"{n:38s} #{k}  {sum(v) / len(v):8.1f} us  ({len(v)} passes)")
