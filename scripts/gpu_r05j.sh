#!/bin/bash
# Round 5: sampler grid cap between its residency and the full grid (bench, alternated)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
run() {   # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 100 --cpu-budget 0 --skip-latency > gpurun_out/sj_$n.json 2> gpurun_out/sj_$n.log || { tail -3 gpurun_out/sj_$n.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/sj_$n.json')); print('$n', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['roofline_search']['frac'])"
}
run w1792 FPM_NONE=1
run w3584 FPM_GRID_WARP=3584
run w2688 FPM_GRID_WARP=2688
run w0 FPM_GRID_WARP=0
run w1792b FPM_NONE=1
run w3584b FPM_GRID_WARP=3584
run w2688b FPM_GRID_WARP=2688
run w0b FPM_GRID_WARP=0
