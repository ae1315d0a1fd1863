#!/bin/bash
# Round 5: batch x contexts sweep with the persistent grids, and the pyramid grid at its residency
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
run() {   # name, bench args..., then env after --
  local n=$1; shift
  local args=()
  while [ $# -gt 0 ] && [ "$1" != "--" ]; do args+=("$1"); shift; done
  [ "$1" = "--" ] && shift
  env FPM_NONE=1 "$@" timeout -k 10 300 python -u bench.py --steps 100 --cpu-budget 0 --skip-latency "${args[@]}" > gpurun_out/sb_$n.json 2> gpurun_out/sb_$n.log || { tail -3 gpurun_out/sb_$n.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/sb_$n.json')); print('$n', d['value'], d['ms_per_step'])"
}
run b128c3
run b128c4 --contexts 4
run b128c2 --contexts 2
run b192c3 --batch 192
run b192c4 --batch 192 --contexts 4
run b256c4 --batch 256 --contexts 4
run b96c3 --batch 96
run b128c3p1024 -- FPM_PYR_WGS=1024
run b128c3p2048 -- FPM_PYR_WGS=2048
run b128c3w -- FPM_GRID_WARP=1792
run b128c3b
run b128c3wb -- FPM_GRID_WARP=1792
