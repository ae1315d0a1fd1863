#!/bin/bash
# Round 5: batch sizes around the small-template / eval residency boundaries (62 sources per context = 2046 ROIs per
# layer <= 2048 two-wave slots), alternated
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
run() {   # name, batch
  timeout -k 10 300 python -u bench.py --steps 100 --cpu-budget 0 --skip-latency --batch $2 > gpurun_out/su_$1.json 2> gpurun_out/su_$1.log || { tail -3 gpurun_out/su_$1.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/su_$1.json')); k=d['kernels']; print('$1', d['value'], d['ms_per_step'], d['roofline']['frac'], {n: round(v['ms_total'], 2) for n, v in k.items()})"
}
run b192 192
run b186 186
run b180 180
run b192b 192
run b186b 186
run b180b 180
