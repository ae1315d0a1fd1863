#!/bin/bash
# Round 6: the whole GPU suite, then the lone-search probe and the configs table with the plain-peak small-search rule
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r06_lone.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r06_lone.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r06_lone.log
python3 scripts/make_src7_raw.py > /dev/null && timeout -k 10 120 ./build/latency_probe gpurun_out/dst7.raw 762 521 gpurun_out/src7.raw 4024 3036 100 > gpurun_out/latency_r06_lone.json || exit $?
cat gpurun_out/latency_r06_lone.json
timeout -k 10 500 python -u scripts/bench_configs.py 10 --no-cpu > gpurun_out/configs_r06_lone.jsonl 2> gpurun_out/configs_r06_lone.log || exit 1
python3 -c "
import json
for l in open('gpurun_out/configs_r06_lone.jsonl'):
    d=json.loads(l); print(d['config'][:70], d['gpu_ms_per_pass'], d['last_pass_device_ms'])"
