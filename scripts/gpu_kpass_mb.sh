#!/bin/bash
# Kernel pass (+ rocprofv3 stats) and the ROI microbenchmark's warp section; usage: scripts/gpu_kpass_mb.sh tag [tests]
TAG=${1:-k}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT && export TMPDIR=/tmp
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1; rc=$?
  tail -2 $OUT/pytest_gpu_$TAG.log
  [ $rc -ne 0 ] && exit $rc
fi
MB_NSRC=${MB_NSRC:-43} MB_WARP_ONLY=1 timeout -k 10 120 ./build/roi_mb 20 > $OUT/mb_$TAG.txt 2>&1 || exit $?
cat $OUT/mb_$TAG.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv -- python3 $ROOT/bench.py --kernel-pass-only --steps 50 > $OUT/kpass_$TAG.json 2> $OUT/kpass_$TAG.log || exit $?
cd $ROOT
S=$(find $OUT/prof_$TAG -name '*kernel_stats.csv' | head -1); [ -n "$S" ] && cp $S $OUT/kernel_stats_$TAG.csv && cut -d, -f1-4 $S | head -8
