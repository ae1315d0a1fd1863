#!/bin/bash
# Round-4 sampler + correlation iteration: GPU tests, then the full ROI microbenchmark (warp, correlation, host check)
# usage: scripts/gpu_r04e.sh tag
TAG=${1:-r04e}
ROOT=$GRAFT_REPO_ROOT
cd $ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && exit $rc
MB_NSRC=43 MB_CORR=1 timeout -k 10 180 ./build/roi_mb 10 > gpurun_out/mb_$TAG.txt 2>&1 || exit $?
cat gpurun_out/mb_$TAG.txt
MB_NSRC=43 MB_CORR=1 MB_DMA_CHECK=1 timeout -k 10 180 ./build/roi_mb 1 > gpurun_out/mbdma_$TAG.txt 2>&1 || exit $?
grep -E "host check" gpurun_out/mbdma_$TAG.txt
