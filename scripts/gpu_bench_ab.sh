#!/bin/bash
# Whole-bench A/B of the in-tree library against build/abl/old.so, alternated (new, old, new, old), default and
# configs[3] workloads, no CPU leg; the in-tree library is restored at the end.  usage: scripts/gpu_bench_ab.sh tag
TAG=${1:-ab}
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
LIB=fastest_image_pattern_matching_amd/lib/libfpm_hip.so
cp $LIB build/abl/new.so
for v in new old new old; do
  cp build/abl/$v.so $LIB
  timeout -k 10 300 python -u bench.py --cpu-budget 0 --skip-latency > gpurun_out/ab_${TAG}_src7_$v.json 2> gpurun_out/ab_${TAG}_src7_$v.log || { cp build/abl/new.so $LIB; exit 1; }
  timeout -k 10 300 python -u bench.py --workload config3 --steps 60 --cpu-budget 0 --skip-latency > gpurun_out/ab_${TAG}_c3_$v.json 2> gpurun_out/ab_${TAG}_c3_$v.log || { cp build/abl/new.so $LIB; exit 1; }
  python3 -c "
import json
a=json.load(open('gpurun_out/ab_${TAG}_src7_$v.json')); b=json.load(open('gpurun_out/ab_${TAG}_c3_$v.json'))
print('$v', 'src7', a['value'], 'config3', b['value'])"
done
cp build/abl/new.so $LIB
