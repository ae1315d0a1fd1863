#!/bin/bash
# After a kernel change: GPU parity tests, the bench's per-kernel pass under rocprofv3 --kernel-trace --stats, and
# the default bench.  usage: scripts/gpu_kpass.sh tag [skip_tests]
TAG=${1:-k}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT && export TMPDIR=/tmp
if [ -z "$2" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1; rc=$?
  tail -3 $OUT/pytest_gpu_$TAG.log
  [ $rc -ne 0 ] && exit $rc
fi
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv -- python3 $ROOT/bench.py --kernel-pass-only --steps 50 > $OUT/kpass_$TAG.json 2> $OUT/kpass_$TAG.log || exit $?
cd $ROOT
python3 - $OUT/kpass_$TAG.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); st = d["steps"]
for k, v in sorted(d["kernels"].items(), key=lambda x: -x[1]["ms_total"]):
    print(f"{k:12s} {v['ms_total'] / st * 1000:8.1f} us/pass {v['launches'] // st} launches")
print("total us/pass", round(sum(v["ms_total"] for v in d["kernels"].values()) / st * 1000, 1), "roofline", d["roofline"]["frac"], d["roofline"]["avg_launch_us"])
PY
S=$(find $OUT/prof_$TAG -name '*kernel_stats.csv' | head -1); [ -n "$S" ] && cp $S $OUT/kernel_stats_$TAG.csv && cut -d, -f1-4 $S | head -16
timeout -k 10 400 python -u bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.log || exit $?
python3 -c "import json,sys; d=json.load(open('$OUT/bench_$TAG.json')); print('bench', d['value'], d['ms_per_step'], d['single_search_ms_end_to_end'], d['single_search_split_ms'], d['roofline']['frac'])"
