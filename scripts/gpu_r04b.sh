#!/bin/bash
# Round-4 sampler iteration: GPU tests (parity of the new k_roi_warp3), the warp microbenchmark and its SQ
# instruction counts; usage: scripts/gpu_r04b.sh tag [skip-tests]
TAG=${1:-r04b}
ROOT=$GRAFT_REPO_ROOT
cd $ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
if [ -z "$2" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
  tail -3 gpurun_out/pytest_gpu_$TAG.log
  [ $rc -ne 0 ] && exit $rc
fi
MB_NSRC=43 MB_WARP_ONLY=1 timeout -k 10 120 ./build/roi_mb 20 > gpurun_out/mb_$TAG.txt 2>&1 || exit $?
cat gpurun_out/mb_$TAG.txt
cd /tmp
MB_NSRC=43 MB_WARP_ONLY=1 MB_SHORT=1 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $ROOT/gpurun_out/sq_$TAG -o run --output-format csv -- $ROOT/build/roi_mb 1 > $ROOT/gpurun_out/sq_$TAG.log 2>&1 || exit $?
