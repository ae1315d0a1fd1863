#!/bin/bash
# Round 5: GPU suite with the persistent grids, then bench A/B (defaults vs the round-4 uncapped grids) and the top-layer
# / pyramid grid knobs
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
# k_roi_corr16 against the product correlation, Src7 layers 0 / 1 / 2 at 43 sources (every row result, partial and
# record compared; exit 2 on a difference)
MB_NSRC=43 timeout -k 10 200 ./build/corr16_bench 10 > gpurun_out/c16_l0.txt 2>&1 || { cat gpurun_out/c16_l0.txt | tail -5; exit 1; }
grep -E "check|corr|chain" gpurun_out/c16_l0.txt
MB_NSRC=43 MB_W=2012 MB_H=1518 MB_P=2048 MB_TW=381 MB_TH=261 timeout -k 10 200 ./build/corr16_bench 10 > gpurun_out/c16_l1.txt 2>&1 || { tail -5 gpurun_out/c16_l1.txt; exit 1; }
grep -E "check|corr|chain" gpurun_out/c16_l1.txt
MB_NSRC=43 MB_W=1006 MB_H=759 MB_P=1024 MB_TW=191 MB_TH=131 timeout -k 10 200 ./build/corr16_bench 10 > gpurun_out/c16_l2.txt 2>&1 || { tail -5 gpurun_out/c16_l2.txt; exit 1; }
grep -E "check|corr|chain" gpurun_out/c16_l2.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r05e.log 2>&1; rc=$?
tail -1 gpurun_out/pytest_gpu_r05e.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/pytest_gpu_r05e.log | head -20; exit $rc; }
run() {   # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 100 --cpu-budget 0 --skip-latency > gpurun_out/sw_$n.json 2> gpurun_out/sw_$n.log || { tail -3 gpurun_out/sw_$n.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/sw_$n.json')); print('$n', d['value'], d['ms_per_step'])"
}
run dflt FPM_NONE=1
run old FPM_GRID_SMALL=0 FPM_GRID_WARP=0
run t1280 FPM_GRID_TOP=1280
run t1024 FPM_GRID_TOP=1024
run t768 FPM_GRID_TOP=768
run p2048 FPM_PYR_WGS=2048
run p2048t1280 FPM_PYR_WGS=2048 FPM_GRID_TOP=1280
run c768 FPM_GRID_CORR=768
run corr16 FPM_CORR16=1
run dflt2 FPM_NONE=1
run old2 FPM_GRID_SMALL=0 FPM_GRID_WARP=0
# k_roi_corr layer-0 phases of the product form at 43 sources (roi_microbench's corr section)
MB_NSRC=43 MB_CORR=1 timeout -k 10 300 ./build/roi_mb 10 > gpurun_out/mb_corr_r05e.txt 2>&1 || { tail -5 gpurun_out/mb_corr_r05e.txt; exit 1; }
grep -E "corr" gpurun_out/mb_corr_r05e.txt | head -40
