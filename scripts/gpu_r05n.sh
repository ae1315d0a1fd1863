#!/bin/bash
# Round 5: two-wave k_roi_small at 5 waves per SIMD (10 per CU: Src7 layers 4-5 in one round at 64 sources per pass)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
FPM_SMALL_WPE=5 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x -k "grid_caps or src7" --timeout 200 --timeout-method thread > gpurun_out/pytest_r05n.log 2>&1; rc=$?
tail -1 gpurun_out/pytest_r05n.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/pytest_r05n.log | head -20; exit $rc; }
run() {   # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 100 --cpu-budget 0 --skip-latency > gpurun_out/so_$n.json 2> gpurun_out/so_$n.log || { tail -3 gpurun_out/so_$n.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/so_$n.json')); k=d['kernels']; print('$n', d['value'], d['ms_per_step'], d['roofline']['frac'], 'roi_small', round(k['roi_small']['ms_total'], 2))"
}
run w4 FPM_NONE=1
run w5 FPM_SMALL_WPE=5
run w4b FPM_NONE=1
run w5b FPM_SMALL_WPE=5
