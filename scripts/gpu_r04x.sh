#!/bin/bash
# Round-4: layer-0 device-sized parts with per-part sampler grids -- parity, then the bench at 1 / 2 / 3 / 4 parts
TAG=${1:-r04x}
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "layer0_parts or src7" --timeout 200 --timeout-method thread > gpurun_out/pytest_parts_$TAG.log 2>&1; rc=$?
tail -1 gpurun_out/pytest_parts_$TAG.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/pytest_parts_$TAG.log | head; exit $rc; }
for rr in 1 2 3 4; do
  FPM_REF_ROUNDS=$rr timeout -k 10 300 python bench.py --steps 100 --warmup 5 --cpu-budget 0 --skip-latency > gpurun_out/bench_rr${rr}_$TAG.json 2> gpurun_out/bench_rr${rr}_$TAG.err || exit $?
  echo "rr $rr: $(python3 -c "import json; d=json.loads(open('gpurun_out/bench_rr${rr}_$TAG.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], {k: round(v['ms_total']*1000/v['launches']*v['launches']/ (100 if False else 1),1) for k,v in d['kernels'].items() if k in ('roi_warp','roi_corr')})")"
done
