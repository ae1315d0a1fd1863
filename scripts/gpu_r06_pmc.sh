#!/bin/bash
# Round 6: top-layer parity, then the PMC snapshots (traffic + SQ issue) of the default and configs[3] kernel passes
# and the rocprofv3 kernel-trace stats of both.  usage: scripts/gpu_r06_pmc.sh tag
TAG=${1:-r06_pmc}
ROOT=$GRAFT_REPO_ROOT
cd $ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_top_mma.py > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
bash scripts/pmc_bench.sh ${TAG}_src7 src7 || exit $?
bash scripts/pmc_bench.sh ${TAG}_config3 config3 || exit $?
for W in src7 config3; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof_${TAG}_$W -o run --output-format csv -- python3 $ROOT/bench.py --workload $W --kernel-pass-only --steps 20 > $ROOT/gpurun_out/kpass_${TAG}_$W.json 2> $ROOT/gpurun_out/kpass_${TAG}_$W.log || exit $?
  cd $ROOT
  S=$(find gpurun_out/prof_${TAG}_$W -name '*kernel_stats.csv' | head -1); cp $S gpurun_out/kernel_stats_${TAG}_$W.csv && cut -d, -f1-4 $S | head -6 | cut -c1-150
done
