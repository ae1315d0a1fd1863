#!/bin/bash
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
for i in 1 2 3; do
timeout -k 10 300 python -u bench.py --workload config4 --cpu-budget 0 > gpurun_out/c4_$i.json 2> gpurun_out/c4_$i.log || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/c4_$i.json')); print('config4', d['value'], d['ms_per_step'])"
done
