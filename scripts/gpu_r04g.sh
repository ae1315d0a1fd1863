#!/bin/bash
# Round-4: two-level pyramid (both chunk heights), prologue-stepped small layers (and the per-layer fallback), GPU
# suite, pyramid / correlation microbenchmarks, single-search dispatch timeline
TAG=${1:-r04g}
ROOT=$GRAFT_REPO_ROOT
cd $ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
for oh in 16 32; do
  FPM_PYR2_OH=$oh timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "pyr_down2" --timeout 120 --timeout-method thread > gpurun_out/pytest_pyr${oh}_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_pyr${oh}_$TAG.log; exit 1; }
  tail -1 gpurun_out/pytest_pyr${oh}_$TAG.log
done
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/pytest_gpu_$TAG.log | head -20; exit $rc; }
FPM_STEP_PROLOGUE=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_noprol_$TAG.log 2>&1; rc=$?
tail -1 gpurun_out/pytest_noprol_$TAG.log
[ $rc -ne 0 ] && exit $rc
for oh in 16 32; do
  FPM_PYR2_OH=$oh MB_NSRC=43 MB_SHORT=1 timeout -k 10 240 ./build/roi_mb 10 > gpurun_out/mb${oh}_$TAG.txt 2>&1 || exit $?
  echo "== OH $oh"; grep -E "pyr|prod" gpurun_out/mb${oh}_$TAG.txt
done
MB_NSRC=43 MB_CORR=1 MB_W=2012 MB_H=1518 MB_P=2048 MB_TW=381 MB_TH=261 timeout -k 10 180 ./build/roi_mb 10 > gpurun_out/mbl1_$TAG.txt 2>&1 || exit $?
grep -E "prod|corrA8|check" gpurun_out/mbl1_$TAG.txt
bash scripts/latency_trace.sh > gpurun_out/lat_$TAG.txt 2>&1 || exit $?
head -40 gpurun_out/lat_$TAG.txt
for rr in 1 2 4; do
  FPM_REF_ROUNDS=$rr timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_rr${rr}_$TAG.json 2> gpurun_out/bench_rr${rr}_$TAG.err || exit $?
  echo "rr $rr: $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_rr${rr}_$TAG.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'))")"
done
