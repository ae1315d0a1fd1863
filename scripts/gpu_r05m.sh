#!/bin/bash
# Round 5: lone-search latency after the small-launch rules (persistent sampler grid and four-wave small-template
# workgroups for small layers) -- parity tests of the grid / NT switches, latency probe, dispatch timeline, bench
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x -k "grid_caps or src7 or single" --timeout 200 --timeout-method thread > gpurun_out/pytest_r05m.log 2>&1; rc=$?
tail -1 gpurun_out/pytest_r05m.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/pytest_r05m.log | head -20; exit $rc; }
python3 scripts/make_src7_raw.py > /dev/null && timeout -k 10 120 ./build/latency_probe gpurun_out/dst7.raw 762 521 gpurun_out/src7.raw 4024 3036 50 > gpurun_out/latency_r05m.json || exit $?
cat gpurun_out/latency_r05m.json
bash scripts/latency_trace.sh > gpurun_out/lat_r05m.txt 2>&1 || exit $?
head -24 gpurun_out/lat_r05m.txt
timeout -k 10 300 python -u bench.py --steps 100 --cpu-budget 0 > gpurun_out/bench_r05m.json 2> gpurun_out/bench_r05m.log || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_r05m.json')); print('bench', d['value'], d['ms_per_step'], d['single_search_ms_end_to_end'], d['single_search_split_ms'], d['roofline']['frac'])"
