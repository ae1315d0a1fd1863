#!/bin/bash
# Round-4: two-level pyramid chunk height by unit count -- GPU suite, bench, single-search trace (and with FPM_PYR2_OH=32)
TAG=${1:-r04v2}
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -1 gpurun_out/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/pytest_gpu_$TAG.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --steps 100 --warmup 5 --cpu-budget 0 --skip-latency > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
echo "bench: $(python3 -c "import json; d=json.loads(open('gpurun_out/bench_$TAG.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], {k: round(v['ms_total'],2) for k,v in d['kernels'].items() if k in ('pyr_down',)})")"
bash scripts/latency_trace.sh > gpurun_out/lat_$TAG.txt 2>&1 || exit $?
grep -E "k_pyr|pass" gpurun_out/lat_$TAG.txt | head -4
FPM_PYR2_OH=32 bash scripts/latency_trace.sh > gpurun_out/lat32_$TAG.txt 2>&1 || exit $?
grep -E "k_pyr|pass" gpurun_out/lat32_$TAG.txt | head -4
