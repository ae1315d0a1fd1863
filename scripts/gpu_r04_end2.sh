#!/bin/bash
# Round-4 closing GPU pass, part 2: PMC traffic of the kernel pass (separate FETCH_SIZE / WRITE_SIZE passes), the
# BASELINE configs and the README reference inputs (scripts/bench_configs.py)
TAG=${1:-r04_end}
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
bash scripts/pmc_bench.sh $TAG || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u scripts/bench_configs.py 10 > gpurun_out/configs_$TAG.jsonl 2> gpurun_out/configs_$TAG.log || exit $?
cut -c1-400 gpurun_out/configs_$TAG.jsonl
MB_NSRC=43 MB_WARP_ONLY=1 MB_SHORT=1 timeout -k 10 180 ./build/roi_mb 10 > gpurun_out/mbw_$TAG.txt 2>&1 || exit $?
grep warp3 gpurun_out/mbw_$TAG.txt
