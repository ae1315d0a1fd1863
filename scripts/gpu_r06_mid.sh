#!/bin/bash
# Round 6 mid-round check: the whole GPU suite, smoke, the default bench line and the configs[3] bench line.
# usage: scripts/gpu_r06_mid.sh tag
TAG=${1:-r06_mid}
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print('bench', d['value'], d['ms_per_step'], d['single_search_ms_end_to_end'], d['single_search_split_ms'], d['roofline']['kernel'], d['roofline']['frac'], d.get('oracle_verified_sources'))"
timeout -k 10 400 python -u bench.py --workload config3 --steps 100 > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.log || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_c3_$TAG.json')); print('config3', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d.get('oracle_verified_sources'))"
