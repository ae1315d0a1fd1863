#!/bin/bash
# Round-5 check: GPU suite, smoke, default bench, configs[3] bench (one GPU)
TAG=${1:-r05}
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -1 gpurun_out/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/pytest_gpu_$TAG.log | head -20; exit $rc; }
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['roofline_search']['frac'], d['oracle_verified_sources'], d['timed_results_verified'])"
timeout -k 10 400 python -u bench.py --workload config3 > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.log || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_c3_$TAG.json')); print('config3', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['oracle_verified_sources'], d['cpu_baseline']['value'])"
