#!/bin/bash
# Round-4 closing GPU pass, part 1: GPU tests, smoke, bench (default and without the host pool warm-up), the kernel
# pass under rocprofv3 --kernel-trace --stats with the warp microbenchmark, C-ABI latency probe, dispatch timeline
# usage: scripts/gpu_r04_end.sh tag
TAG=${1:-r04_end}
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
bash scripts/gpu_kpass_mb.sh $TAG tests || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print('bench', d['value'], d['ms_per_step'], d['single_search_ms_end_to_end'], d['single_search_split_ms'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['roofline_search']['frac'], d.get('oracle_verified'))"
FPM_HOST_WARM=0 timeout -k 10 400 python -u bench.py > gpurun_out/bench_nowarm_$TAG.json 2> gpurun_out/bench_nowarm_$TAG.log || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_nowarm_$TAG.json')); print('bench FPM_HOST_WARM=0', d['value'], d['ms_per_step'])"
python3 scripts/make_src7_raw.py > /dev/null && timeout -k 10 120 ./build/latency_probe gpurun_out/dst7.raw 762 521 gpurun_out/src7.raw 4024 3036 50 > gpurun_out/latency_$TAG.json || exit $?
cat gpurun_out/latency_$TAG.json
bash scripts/latency_trace.sh > gpurun_out/lat_$TAG.txt 2>&1 || exit $?
head -26 gpurun_out/lat_$TAG.txt
