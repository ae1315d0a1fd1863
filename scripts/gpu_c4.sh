#!/bin/bash
# configs[4] bench line (one GPU, oracle-verified) and two repeats without the CPU leg.  usage: scripts/gpu_c4.sh tag
TAG=${1:-c4}
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --workload config4 > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.log || { tail -20 gpurun_out/bench_c4_$TAG.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_c4_$TAG.json')); print('config4', d['value'], d['ms_per_step'], d.get('oracle_verified_sources'), d['config']['contexts_per_gpu'])"
for i in 1 2; do
timeout -k 10 300 python -u bench.py --workload config4 --cpu-budget 0 > gpurun_out/c4r_$i.json 2> gpurun_out/c4r_$i.log || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/c4r_$i.json')); print('config4', d['value'], d['ms_per_step'])"
done
