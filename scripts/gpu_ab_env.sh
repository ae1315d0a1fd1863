#!/bin/bash
# A/B of an environment switch of the library: GPU tests with it on, then the bench's kernel pass under rocprofv3
# --kernel-trace --stats with it off and on (per-launch-position times: scripts/layer_times.py), then the default bench
# with it off and on.  usage: scripts/gpu_ab_env.sh VAR tag [tests]
VAR=$1; TAG=${2:-ab}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/ab_$TAG
mkdir -p $OUT && cd $ROOT && export TMPDIR=/tmp
if [ -n "$3" ]; then
  env $VAR=1 timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest_on.log 2>&1 || { tail -15 $OUT/pytest_on.log; exit 1; }
  tail -1 $OUT/pytest_on.log
fi
for v in 0 1; do
  cd /tmp && env $VAR=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/p$v -o run --output-format csv -- python3 $ROOT/bench.py --kernel-pass-only --steps 30 > $OUT/kpass$v.json 2> $OUT/kpass$v.log || exit 1
  cd $ROOT && echo "== $VAR=$v" && python3 scripts/layer_times.py $OUT/p$v/run_kernel_trace.csv | head -8
done
for v in 0 1; do
  env $VAR=$v timeout -k 10 300 python -u bench.py --cpu-budget 0 --skip-latency > $OUT/bench$v.json 2> $OUT/bench$v.log || exit 1
  python3 -c "import json; d=json.load(open('$OUT/bench$v.json')); print('$VAR=$v bench', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['timed_results_verified'])"
done
