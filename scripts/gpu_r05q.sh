#!/bin/bash
# Round 5: eight-wave k_roi_small workgroups for lone searches -- the GPU suite, latency probe + timeline, bench
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_r05q.log 2>&1; rc=$?
tail -1 gpurun_out/pytest_r05q.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/pytest_r05q.log | head -20; exit $rc; }
python3 scripts/make_src7_raw.py > /dev/null && timeout -k 10 120 ./build/latency_probe gpurun_out/dst7.raw 762 521 gpurun_out/src7.raw 4024 3036 50 > gpurun_out/latency_r05q.json || exit $?
cat gpurun_out/latency_r05q.json
FPM_SMALL_NT=0 timeout -k 10 120 ./build/latency_probe gpurun_out/dst7.raw 762 521 gpurun_out/src7.raw 4024 3036 50 > gpurun_out/latency_r05q_nt0.json || exit $?
cat gpurun_out/latency_r05q_nt0.json
timeout -k 10 120 ./build/latency_probe gpurun_out/dst7.raw 762 521 gpurun_out/src7.raw 4024 3036 50 > gpurun_out/latency_r05q_b.json || exit $?
cat gpurun_out/latency_r05q_b.json
bash scripts/latency_trace.sh > gpurun_out/lat_r05q.txt 2>&1 || exit $?
head -24 gpurun_out/lat_r05q.txt
timeout -k 10 300 python -u bench.py --steps 100 --cpu-budget 0 > gpurun_out/bench_r05q.json 2> gpurun_out/bench_r05q.log || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_r05q.json')); print('bench', d['value'], d['ms_per_step'], d['single_search_ms_end_to_end'], d['single_search_split_ms'], d['roofline']['frac'])"
