#!/bin/bash
# Kernel-pass layer times under rocprofv3 for several values of one environment override of the library.
# usage: scripts/gpu_env_sweep.sh VAR tag value [value ...]   (output: gpurun_out/sweep_<tag>/)
VAR=$1; TAG=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/sweep_$TAG
mkdir -p $OUT && export TMPDIR=/tmp
for v in "$@"; do
  cd /tmp && env $VAR=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/p$v -o run --output-format csv -- python3 $ROOT/bench.py --kernel-pass-only --steps 20 > $OUT/kpass$v.json 2> $OUT/kpass$v.log || exit 1
  cd $ROOT && echo "== $VAR=$v" && python3 scripts/layer_times.py $OUT/p$v/run_kernel_trace.csv | grep "${GREP:-.}"
done
