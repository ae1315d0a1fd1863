#!/bin/bash
# Round 5: GPU suite with the persistent grids, then bench A/B (defaults vs the round-4 uncapped grids) and the top-layer
# / pyramid grid knobs
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
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
run dflt2 FPM_NONE=1
run old2 FPM_GRID_SMALL=0 FPM_GRID_WARP=0
# k_roi_corr layer-0 phases of the product form at 43 sources (roi_microbench's corr section)
MB_NSRC=43 MB_CORR=1 timeout -k 10 300 ./build/roi_mb 10 > gpurun_out/mb_corr_r05e.txt 2>&1 || { tail -5 gpurun_out/mb_corr_r05e.txt; exit 1; }
grep -E "corr" gpurun_out/mb_corr_r05e.txt | head -40
