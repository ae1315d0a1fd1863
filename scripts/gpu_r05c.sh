#!/bin/bash
# Round 5: overlap filter without the per-workgroup system fence (tests + Src10 +-180 tail), then a grid-cap sweep of
# the bench (concurrent contexts: do smaller grids of the big kernels let the other contexts' kernels co-run?)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_overlap.py tests/test_gpu_parity.py -q -x -k "overlap or src10" --timeout 300 --timeout-method thread > gpurun_out/pytest_r05c.log 2>&1; rc=$?
tail -1 gpurun_out/pytest_r05c.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  FPM_TAIL_TIMES=1 timeout -k 10 240 python3 scripts/bench_configs.py 30 --no-cpu --only=1 --no-pipe > gpurun_out/tail_r05c_$rep.jsonl 2> gpurun_out/tail_r05c_$rep.err || exit 1
  grep "^tail" gpurun_out/tail_r05c_$rep.err | tail -2
  python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/tail_r05c_$rep.jsonl')][-1]; print({k: d[k] for k in d if 'ms' in k})"
done
run() {   # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 100 --cpu-budget 0 --skip-latency > gpurun_out/sw_$n.json 2> gpurun_out/sw_$n.log || { tail -3 gpurun_out/sw_$n.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/sw_$n.json')); print('$n', d['value'], d['ms_per_step'])"
}
run base FPM_NONE=1
run w1280 FPM_GRID_WARP=1280
run w1536 FPM_GRID_WARP=1536
run c768 FPM_GRID_CORR=768
run c512 FPM_GRID_CORR=512
run s768 FPM_GRID_SMALL=768
run s512 FPM_GRID_SMALL=512
run w1536c768 FPM_GRID_WARP=1536 FPM_GRID_CORR=768
run base2 FPM_NONE=1
# the round-2 fused sampler + correlation (k_roi_fused, FPM_EXPERIMENTAL) against today's split chain, 43 sources
MB_NSRC=43 timeout -k 10 300 ./build/fused_bench 10 > gpurun_out/fused_r05c.txt 2>&1 || { tail -5 gpurun_out/fused_r05c.txt; exit 1; }
tail -12 gpurun_out/fused_r05c.txt
