#!/bin/bash
# Round 5 final check of the committed tree: smoke, the default bench line
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r05_final.log 2>&1 || exit $?
tail -1 gpurun_out/smoke_r05_final.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r05_final.json 2> gpurun_out/bench_r05_final.log || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_r05_final.json')); print('bench', d['value'], d['ms_per_step'], d['single_search_ms_end_to_end'], d['single_search_split_ms'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['roofline_search']['frac'], d.get('oracle_verified_sources'), d['vs_baseline_latency'])"
