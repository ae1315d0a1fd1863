#!/bin/bash
# Round-4: two-level pyramid kernel parity + full GPU suite, warp forms A/B, full microbenchmark (pyramid section)
# usage: scripts/gpu_r04f.sh tag
TAG=${1:-r04f}
ROOT=$GRAFT_REPO_ROOT
cd $ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "pyr_down" --timeout 120 --timeout-method thread > gpurun_out/pytest_pyr_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_pyr_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && exit $rc
MB_NSRC=43 MB_WARP_ONLY=1 timeout -k 10 180 ./build/roi_mb 10 > gpurun_out/mbw_$TAG.txt 2>&1 || exit $?
cat gpurun_out/mbw_$TAG.txt
MB_NSRC=8 MB_SHORT=1 timeout -k 10 180 ./build/roi_mb 10 > gpurun_out/mb_$TAG.txt 2>&1 || exit $?
grep -E "pyr|check" gpurun_out/mb_$TAG.txt
