#!/bin/bash
# Round-4: README reference inputs, sampler ablations, double-buffered LDS-DMA correlation (timing + host checks)
TAG=${1:-r04l}
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
MB_NSRC=43 MB_CORR=1 timeout -k 10 180 ./build/roi_mb 10 > gpurun_out/mbc_$TAG.txt 2>&1 || exit $?
grep -E "prod corr|corrA|corr DB|check" gpurun_out/mbc_$TAG.txt
MB_NSRC=43 MB_CORR=1 MB_DB_CHECK=1 timeout -k 10 180 ./build/roi_mb 1 > gpurun_out/mbcdb_$TAG.txt 2>&1 || exit $?
grep -E "check" gpurun_out/mbcdb_$TAG.txt
MB_NSRC=43 MB_CORR=1 MB_W=2012 MB_H=1518 MB_P=2048 MB_TW=381 MB_TH=261 timeout -k 10 180 ./build/roi_mb 10 > gpurun_out/mbl1_$TAG.txt 2>&1 || exit $?
grep -E "prod corr|corrA8|DB|check" gpurun_out/mbl1_$TAG.txt
MB_NSRC=43 MB_CORR=1 MB_DB_CHECK=1 MB_W=2012 MB_H=1518 MB_P=2048 MB_TW=381 MB_TH=261 timeout -k 10 180 ./build/roi_mb 1 > gpurun_out/mbl1db_$TAG.txt 2>&1 || exit $?
grep -E "check" gpurun_out/mbl1db_$TAG.txt
MB_NSRC=43 MB_WARP_ONLY=1 MB_SHORT=1 timeout -k 10 180 ./build/roi_mb 10 > gpurun_out/mbw_$TAG.txt 2>&1 || exit $?
grep warp3 gpurun_out/mbw_$TAG.txt
timeout -k 10 600 python -u scripts/bench_configs.py 10 --ref-only > gpurun_out/configs_ref_$TAG.jsonl 2> gpurun_out/configs_ref_$TAG.log || { tail -5 gpurun_out/configs_ref_$TAG.log; exit 1; }
cut -c1-700 gpurun_out/configs_ref_$TAG.jsonl
