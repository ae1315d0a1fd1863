#!/bin/bash
# Round-5 closing pass, part 1: GPU suite + kernel pass under rocprofv3 (gpu_kpass_mb.sh), smoke, default bench,
# configs[3] bench, C-ABI latency probe and the single-search dispatch timeline.  usage: scripts/gpu_r05_end.sh tag
TAG=${1:-r05_end}
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
bash scripts/gpu_kpass_mb.sh $TAG tests || exit $?
cd $GRAFT_REPO_ROOT
# the PMC traffic of this build's kernel pass, installed where the bench reads it (the committed copy is updated from
# gpurun_out/pmc_bench_$TAG/summary.csv afterwards)
bash scripts/pmc_bench.sh $TAG || exit $?
cd $GRAFT_REPO_ROOT && cp gpurun_out/pmc_bench_$TAG/summary.csv profiles/latest/pmc_traffic.csv
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print('bench', d['value'], d['ms_per_step'], d['single_search_ms_end_to_end'], d['single_search_split_ms'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['roofline_search']['frac'], d.get('oracle_verified_sources'))"
timeout -k 10 400 python -u bench.py --workload config3 --steps 100 > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.log || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_c3_$TAG.json')); print('config3', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d.get('oracle_verified_sources'))"
python3 scripts/make_src7_raw.py > /dev/null && timeout -k 10 120 ./build/latency_probe gpurun_out/dst7.raw 762 521 gpurun_out/src7.raw 4024 3036 50 > gpurun_out/latency_$TAG.json || exit $?
cat gpurun_out/latency_$TAG.json
bash scripts/latency_trace.sh > gpurun_out/lat_$TAG.txt 2>&1 || exit $?
head -24 gpurun_out/lat_$TAG.txt
