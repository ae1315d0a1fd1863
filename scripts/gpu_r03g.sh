#!/bin/bash
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
bash scripts/gpu_kpass_mb.sh r03g tests || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r03g.json 2> gpurun_out/bench_r03g.log || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_r03g.json')); print('bench', d['value'], d['ms_per_step'], d['single_search_ms_end_to_end'], d['single_search_split_ms'], d['roofline']['frac'], d['roofline']['avg_launch_us'])"
python3 scripts/make_src7_raw.py > /dev/null && timeout -k 10 120 ./build/latency_probe gpurun_out/dst7.raw 762 521 gpurun_out/src7.raw 4024 3036 50 | tee gpurun_out/latency_r03g.json
