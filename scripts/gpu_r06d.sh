#!/bin/bash
# Round 6: top-layer parity tests, the configs[3] kernel pass (per-kernel times), k_top_mma's SQ counters
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
T=${1:-r06d}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_top_mma.py \
  tests/test_gpu_semantics.py::test_config3_one_degree_step > gpurun_out/pytest_$T.log 2>&1 || { tail -40 gpurun_out/pytest_$T.log; exit 1; }
tail -2 gpurun_out/pytest_$T.log
timeout -k 10 200 python -u bench.py --workload config3 --kernel-pass-only --steps 5 --warmup 1 --cpu-budget 0 > gpurun_out/kp_$T.json 2> gpurun_out/kp_$T.log || exit 1
python3 -c "
import json
d=json.load(open('gpurun_out/kp_$T.json'))
print({n: round(v['ms_total']/max(v['launches'],1)*1000,1) for n,v in d['kernels'].items() if v['launches']})"
bash scripts/top_pmc.sh $T | cut -c1-400
