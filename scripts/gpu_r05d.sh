#!/bin/bash
# Round 5: second grid-cap sweep of the bench (k_roi_small / k_roi_warp3 / k_roi_corr / pyramid workgroup counts)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
run() {   # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 100 --cpu-budget 0 --skip-latency > gpurun_out/sw_$n.json 2> gpurun_out/sw_$n.log || { tail -3 gpurun_out/sw_$n.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/sw_$n.json')); print('$n', d['value'], d['ms_per_step'])"
}
run base FPM_NONE=1
run s768w1536 FPM_GRID_SMALL=768 FPM_GRID_WARP=1536
run s768w1792 FPM_GRID_SMALL=768 FPM_GRID_WARP=1792
run s1024 FPM_GRID_SMALL=1024
run s640 FPM_GRID_SMALL=640
run s768w1536c896 FPM_GRID_SMALL=768 FPM_GRID_WARP=1536 FPM_GRID_CORR=896
run s768w1536p2048 FPM_GRID_SMALL=768 FPM_GRID_WARP=1536 FPM_PYR_WGS=2048
run s768w1536p3072 FPM_GRID_SMALL=768 FPM_GRID_WARP=1536 FPM_PYR_WGS=3072
run s768w1280 FPM_GRID_SMALL=768 FPM_GRID_WARP=1280
run s768 FPM_GRID_SMALL=768
run base2 FPM_NONE=1
