#!/usr/bin/env python3
"""Concurrency of the bench's timed region in a rocprofv3 kernel trace (profiling aid): the dispatches between the
first and the last k_pack of the timed passes (before the eager kernel pass, whose launches are serial), their
union busy time, the time-weighted number of kernels in flight, and per kernel the share of its time it ran
alone.  usage: overlap_trace.py run_kernel_trace.csv [n_timed_packs]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")
       .replace("fpm::", "").split("<")[0]) for r in rows]
packs = [k for k, x in enumerate(iv) if x[2] == "k_pack"]
n = int(sys.argv[2]) if len(sys.argv) > 2 else len(packs) // 2
# window: from the end of the n-th pack before the last timed one back over n packs
a = packs[len(packs) // 4]
b = packs[len(packs) // 4 + n]
win = iv[a + 1:b + 1]
t0, t1 = win[0][0], max(e for _, e, _ in win)
ev = sorted([(s, 1) for s, _, _ in win] + [(e, -1) for _, e, _ in win])
busy = 0
weighted = 0
cur = 0
last = t0
for t, d in ev:
    if cur > 0:
        busy += t - last
        weighted += cur * (t - last)
    cur += d
    last = t
alone = defaultdict(int)
tot = defaultdict(int)
for k, (s, e, nm) in enumerate(win):
    tot[nm] += e - s
    # time of [s, e) covered by no other dispatch
    others = [(s2, e2) for j, (s2, e2, _) in enumerate(win) if j != k and s2 < e and e2 > s]
    pts = sorted(set([s, e] + [max(s, x) for x, _ in others] + [min(e, y) for _, y in others]))
    for p, q in zip(pts, pts[1:]):
        if not any(x <= p and y >= q for x, y in others):
            alone[nm] += q - p
span = t1 - t0
print(f"window {span / 1e3:.1f} us, {len(win)} dispatches, busy {busy / span:.3f}, mean in flight {weighted / max(busy, 1):.2f}")
for nm in sorted(tot, key=lambda x: -tot[x]):
    print(f"{nm:18s} total {tot[nm] / 1e3:9.1f} us  alone {alone[nm] / max(tot[nm], 1):.2f}")
