#!/bin/bash
# BASELINE configs and the README reference inputs (scripts/bench_configs.py).  usage: scripts/gpu_configs.sh tag
TAG=${1:-r05}
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/bench_configs.py 10 > gpurun_out/configs_$TAG.jsonl 2> gpurun_out/configs_$TAG.log || exit $?
cut -c1-200 gpurun_out/configs_$TAG.jsonl
