#!/bin/bash
# Round-3 GPU pass: GPU tests, warp microbenchmark, rocprof kernel pass, default bench, C-ABI latency probe; usage: scripts/gpu_r03.sh tag
TAG=${1:-r03}
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
bash scripts/gpu_kpass_mb.sh $TAG tests || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print('bench', d['value'], d['ms_per_step'], d['single_search_ms_end_to_end'], d['single_search_split_ms'], d['roofline']['frac'], d['roofline']['avg_launch_us'])"
python3 scripts/make_src7_raw.py > /dev/null && timeout -k 10 120 ./build/latency_probe gpurun_out/dst7.raw 762 521 gpurun_out/src7.raw 4024 3036 50 | tee gpurun_out/latency_$TAG.json
