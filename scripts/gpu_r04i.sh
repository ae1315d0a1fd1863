#!/bin/bash
# Round-4 check: GPU suite, bench, single-search dispatch timeline, DMA correlation host check at layer-1 geometry
TAG=${1:-r04i}
ROOT=$GRAFT_REPO_ROOT
cd $ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/pytest_gpu_$TAG.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/bench_$TAG.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d.get('single_search_split_ms'), {k: round(v['ms_total']*1000/v['launches'],1) for k,v in d['kernels'].items()})"
MB_NSRC=43 MB_CORR=1 MB_DMA_CHECK=1 MB_W=2012 MB_H=1518 MB_P=2048 MB_TW=381 MB_TH=261 timeout -k 10 180 ./build/roi_mb 1 > gpurun_out/mbl1dma_$TAG.txt 2>&1 || exit $?
grep -E "check" gpurun_out/mbl1dma_$TAG.txt
bash scripts/latency_trace.sh > gpurun_out/lat_$TAG.txt 2>&1 || exit $?
head -28 gpurun_out/lat_$TAG.txt
MB_NSRC=43 MB_WARP_ONLY=1 MB_SHORT=1 timeout -k 10 180 ./build/roi_mb 10 > gpurun_out/mbw_$TAG.txt 2>&1 || exit $?
cat gpurun_out/mbw_$TAG.txt
for oh in 16 32; do
  FPM_PYR2_OH=$oh timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "pyr_down2" --timeout 120 --timeout-method thread > gpurun_out/pytest_pyr${oh}_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_pyr${oh}_$TAG.log; exit 1; }
  tail -1 gpurun_out/pytest_pyr${oh}_$TAG.log
  FPM_PYR2_OH=$oh MB_NSRC=43 MB_SHORT=1 timeout -k 10 240 ./build/roi_mb 10 > gpurun_out/mb${oh}_$TAG.txt 2>&1 || exit $?
  echo "== OH $oh"; grep -E "pyr" gpurun_out/mb${oh}_$TAG.txt
done
FPM_TOP_FUSED=1 bash scripts/latency_trace.sh > gpurun_out/lat_topfused_$TAG.txt 2>&1 || exit $?
head -24 gpurun_out/lat_topfused_$TAG.txt
