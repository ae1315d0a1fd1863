#!/bin/bash
# Kernel-pass timing of library variants built in build/abl/*.so (measurement builds, e.g. -DTOPMMA_ABL=n ablations):
# each is copied over the product library of this scratch copy in turn.  usage: gpu_abl.sh tag workload v1 v2 ...
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
T=$1; W=$2; shift 2
LIB=fastest_image_pattern_matching_amd/lib/libfpm_hip.so
cp $LIB build/abl/base.so
for v in base "$@"; do
  cp build/abl/$v.so $LIB
  timeout -k 10 200 python -u bench.py --workload $W --kernel-pass-only --steps 5 --warmup 1 --cpu-budget 0 > gpurun_out/abl_${T}_$v.json 2> gpurun_out/abl_${T}_$v.log || { echo "variant $v failed"; tail -5 gpurun_out/abl_${T}_$v.log; }
  python3 -c "
import json,sys
d=json.load(open('gpurun_out/abl_${T}_$v.json'))
k=d.get('kernels', {})
print('$v', {n: round(v['ms_total']/max(v['launches'],1)*1000,1) for n,v in k.items() if v['launches']})" || true
done
cp build/abl/base.so $LIB
