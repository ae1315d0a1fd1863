#!/bin/bash
# k_roi_warp per-layer medians (kernel trace of the bench kernel pass) + the microbenchmark's layer-0 launch.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/wl -o run --output-format csv -- python3 $ROOT/bench.py --kernel-pass-only --steps 30 > $OUT/wl.json 2> $OUT/wl.log || exit $?
python3 - $OUT/wl <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0]
for key in ('k_roi_warp', 'k_roi_corr', 'k_roi_small'):
    seq = [r for r in csv.DictReader(open(f)) if key in r['Kernel_Name']]
    g = collections.defaultdict(list)
    for i, r in enumerate(seq):
        g[i % 3].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000)
    print(key, 'per-layer medians (us):', [round(sorted(v)[len(v) // 2], 1) for k, v in sorted(g.items())])
PY
cd $ROOT && [ -x build/warp_exp2 ] && timeout -k 10 100 ./build/warp_exp2 20 | head -1
exit 0
