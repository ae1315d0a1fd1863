#!/bin/bash
# Throughput sweep of bench.py over sources per step and concurrent contexts (one GPU); one JSON line per run.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
# BATCHES / CONTEXTS override the grids (space-separated lists)
for b in ${BATCHES:-8 16 32 64}; do
  for c in ${CONTEXTS:-1 2 3 4}; do
    timeout -k 10 240 python -u bench.py --steps 100 --warmup 5 --batch $b --contexts $c --cpu-budget 0 --skip-latency \
      > $OUT/sweep_b${b}_c${c}.json 2> $OUT/sweep_b${b}_c${c}.log; rc=$?
    if [ $rc -ne 0 ]; then echo "b=$b c=$c rc=$rc: stopping"; exit $rc; fi
    python -c "import json,sys; d=json.load(open('$OUT/sweep_b${b}_c${c}.json')); print($b, $c, d['value'], d['ms_per_step'])"
  done
done
