#!/bin/bash
# Round 5: k_roi_warp3 with the workgroup's waves sharing its tasks (LDS counter) -- microbenchmark (byte check),
# the Src7 parity tests incl. the grid caps, then bench A/B (LQ on / off, alternated)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
MB_NSRC=43 MB_LQ=1 timeout -k 10 200 ./build/roi_mb 10 > gpurun_out/mb_lq_r05i.txt 2>&1 || { tail -5 gpurun_out/mb_lq_r05i.txt; exit 1; }
grep -E "warp3|prod" gpurun_out/mb_lq_r05i.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x -k "grid_caps or src7" --timeout 200 --timeout-method thread > gpurun_out/pytest_lq_r05i.log 2>&1; rc=$?
tail -1 gpurun_out/pytest_lq_r05i.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/pytest_lq_r05i.log | head -20; exit $rc; }
run() {   # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 100 --cpu-budget 0 --skip-latency > gpurun_out/sl_$n.json 2> gpurun_out/sl_$n.log || { tail -3 gpurun_out/sl_$n.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/sl_$n.json')); print('$n', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['roofline_search']['frac'])"
}
run lq1 FPM_NONE=1
run lq0 FPM_WARP_LQ=0
run lq1b FPM_NONE=1
run lq0b FPM_WARP_LQ=0
run lq1u FPM_GRID_WARP=0
