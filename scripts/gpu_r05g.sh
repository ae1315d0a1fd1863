#!/bin/bash
# Round 5: batch A/B with the default grids (sampler capped), alternated on one box
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
run() {   # name, bench args...
  local n=$1; shift
  env FPM_NONE=1 timeout -k 10 300 python -u bench.py --steps 100 --cpu-budget 0 --skip-latency "$@" > gpurun_out/sg_$n.json 2> gpurun_out/sg_$n.log || { tail -3 gpurun_out/sg_$n.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/sg_$n.json')); print('$n', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_search']['frac'])"
}
run b128 --batch 128
run b192 --batch 192
run b160 --batch 160
run b128b --batch 128
run b192b --batch 192
run b240 --batch 240
run b160b --batch 160
