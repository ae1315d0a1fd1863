#!/bin/bash
# Src10 +-180 host tail, round-3 build (build/r03_tree: git worktree of e5fb17b, its own libfpm_hip.so) against this
# tree's build on ONE box, alternated twice: configs[2] stress latency with the tail's stage clocks (FPM_TAIL_TIMES)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2 3; do
  for t in r03 cur; do
    d=$GRAFT_REPO_ROOT; [ $t = r03 ] && d=$GRAFT_REPO_ROOT/build/r03_tree
    (cd $d && FPM_TAIL_TIMES=1 timeout -k 10 240 python3 scripts/bench_configs.py 30 --no-cpu --only=1 --no-pipe) \
      > gpurun_out/tailab_${t}_$rep.jsonl 2> gpurun_out/tailab_${t}_$rep.err || { tail -5 gpurun_out/tailab_${t}_$rep.err; exit 1; }
    python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/tailab_${t}_$rep.jsonl')][-1]; print('$t', $rep, {k: d[k] for k in d if 'ms' in k})"
  done
done
