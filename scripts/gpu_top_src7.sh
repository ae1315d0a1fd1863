#!/bin/bash
# Src7 kernel pass: the default top layer (k_top_fused at >= 256 jobs) against the matrix-core form forced (FPM_TOP_MMA=1)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
for v in 0 1; do
  if [ $v = 1 ]; then export FPM_TOP_MMA=1; fi
  timeout -k 10 200 python -u bench.py --kernel-pass-only --steps 10 --warmup 2 --cpu-budget 0 > gpurun_out/kp_src7_mma$v.json 2> gpurun_out/kp_src7_mma$v.log || exit $?
  python3 -c "
import json
d=json.load(open('gpurun_out/kp_src7_mma$v.json'))
print('FPM_TOP_MMA=$v', {n: (v['launches'], round(v['ms_total']/max(v['launches'],1)*1000,1)) for n,v in d['kernels'].items() if v['launches']})"
done
