#!/bin/bash
# configs[3] bench at 2 / 3 / 4 / 6 contexts per GPU (no CPU leg), alternated twice
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
for r in 1 2; do for g in 2 3 4 6; do
  timeout -k 10 300 python -u bench.py --workload config3 --steps 60 --contexts $g --cpu-budget 0 --skip-latency > gpurun_out/c3ctx_${g}_$r.json 2> gpurun_out/c3ctx_${g}_$r.log || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/c3ctx_${g}_$r.json')); print('contexts', $g, d['value'], d['ms_per_step'])"
done; done
