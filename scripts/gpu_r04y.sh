#!/bin/bash
# Round-4: next-layer tables written by the step (FPM_STEP_TABLES) -- GPU suite, bench 0 / 1, single-search trace
TAG=${1:-r04y}
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -1 gpurun_out/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/pytest_gpu_$TAG.log | head -20; exit $rc; }
for stb in 0 1; do
  FPM_STEP_TABLES=$stb timeout -k 10 300 python bench.py --steps 100 --warmup 5 --cpu-budget 0 --skip-latency > gpurun_out/bench_stb${stb}_$TAG.json 2> gpurun_out/bench_stb${stb}_$TAG.err || exit $?
  echo "stb $stb: $(python3 -c "import json; d=json.loads(open('gpurun_out/bench_stb${stb}_$TAG.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], {k: round(v['ms_total'],2) for k,v in d['kernels'].items() if k in ('roi_tables','roi_eval','cand_step')})")"
done
bash scripts/latency_trace.sh > gpurun_out/lat_$TAG.txt 2>&1 || exit $?
head -24 gpurun_out/lat_$TAG.txt
FPM_STEP_TABLES=0 bash scripts/latency_trace.sh > gpurun_out/lat0_$TAG.txt 2>&1 || exit $?
grep pass gpurun_out/lat0_$TAG.txt | head -1
