#!/bin/bash
# Round-4: the README reference inputs (scripts/bench_configs.py --ref-only) and the sampler ablations
TAG=${1:-r04k}
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/bench_configs.py 10 --ref-only > gpurun_out/configs_ref_$TAG.jsonl 2> gpurun_out/configs_ref_$TAG.log || { tail -5 gpurun_out/configs_ref_$TAG.log; exit 1; }
cut -c1-600 gpurun_out/configs_ref_$TAG.jsonl
MB_NSRC=43 MB_WARP_ONLY=1 MB_SHORT=1 timeout -k 10 180 ./build/roi_mb 10 > gpurun_out/mbw_$TAG.txt 2>&1 || exit $?
grep warp3 gpurun_out/mbw_$TAG.txt
