#!/bin/bash
# Round-6 closing pass on the committed tree: the whole GPU suite, smoke, the default bench line, the configs[3] and
# configs[4] bench lines, the C-ABI lone-search latency probe, and the default kernel pass under rocprofv3 stats.
# usage: scripts/gpu_r06_end.sh tag
TAG=${1:-r06_end}
ROOT=$GRAFT_REPO_ROOT
cd $ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print('bench', d['value'], d['ms_per_step'], d['single_search_ms_end_to_end'], d['single_search_split_ms'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['traffic'], d['roofline_issue']['bound'], d['roofline_issue']['frac'], d['roofline_search']['frac'], d.get('oracle_verified_sources'))"
timeout -k 10 400 python -u bench.py --workload config3 --steps 100 > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.log || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_c3_$TAG.json')); print('config3', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_us'], d['roofline']['traffic'], d['roofline_issue']['fracs'], d.get('oracle_verified_sources'))"
timeout -k 10 400 python -u bench.py --workload config4 > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.log || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_c4_$TAG.json')); print('config4', d['value'], d['ms_per_step'], d.get('oracle_verified_sources'))"
python3 scripts/make_src7_raw.py > /dev/null && timeout -k 10 120 ./build/latency_probe gpurun_out/dst7.raw 762 521 gpurun_out/src7.raw 4024 3036 50 > gpurun_out/latency_$TAG.json || exit $?
cat gpurun_out/latency_$TAG.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $ROOT/bench.py --kernel-pass-only --steps 50 > $ROOT/gpurun_out/kpass_$TAG.json 2> $ROOT/gpurun_out/kpass_$TAG.log || exit $?
cd $ROOT && S=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1) && cp $S gpurun_out/kernel_stats_$TAG.csv && cut -d, -f1-4 $S | head -4 | cut -c1-150
