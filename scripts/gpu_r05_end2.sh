#!/bin/bash
# Round-5 closing pass, part 2: PMC traffic of the kernel pass (separate FETCH_SIZE / WRITE_SIZE passes), the BASELINE
# configs and the README reference inputs (scripts/bench_configs.py).  usage: scripts/gpu_r05_end2.sh tag
TAG=${1:-r05_end}
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
bash scripts/pmc_bench.sh $TAG || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u scripts/bench_configs.py 10 > gpurun_out/configs_$TAG.jsonl 2> gpurun_out/configs_$TAG.log || exit $?
cut -c1-300 gpurun_out/configs_$TAG.jsonl
