#!/bin/bash
# Round 6: configs[4] bench on one GPU (oracle-verified), the BASELINE configs / README inputs (bench_configs.py) and the
# configs[3] kernel pass with the per-kernel bytes.  usage: scripts/gpu_r06_cfg.sh tag
TAG=${1:-r06_cfg}
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --workload config4 > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.log || { tail -20 gpurun_out/bench_c4_$TAG.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_c4_$TAG.json')); print('config4', d['value'], d['unit'], d['ms_per_step'], d.get('oracle_verified_sources'), (d.get('cpu_baseline') or {}).get('value'))"
timeout -k 10 200 python -u bench.py --workload config3 --kernel-pass-only --steps 5 --warmup 1 > gpurun_out/kp_c3_$TAG.json 2> gpurun_out/kp_c3_$TAG.log || exit $?
python3 -c "
import json
d=json.load(open('gpurun_out/kp_c3_$TAG.json'))
print({n: (round(v['ms_total']/max(v['launches'],1)*1000,1), v['bytes']//max(v['launches'],1)) for n,v in d['kernels'].items() if v['launches']})
print(d['roofline']); print(d['roofline_issue'])"
timeout -k 10 900 python -u scripts/bench_configs.py 10 > gpurun_out/configs_$TAG.jsonl 2> gpurun_out/configs_$TAG.log || { tail -20 gpurun_out/configs_$TAG.log; exit 1; }
cut -c1-300 gpurun_out/configs_$TAG.jsonl
