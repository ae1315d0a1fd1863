#!/bin/bash
# Round-4 closing pass, part 2 on the final build: GPU suite, single-search timeline, PMC traffic of the kernel pass,
# the BASELINE configs and the README inputs
TAG=${1:-r04_end}
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu2_$TAG.log 2>&1; rc=$?
tail -1 gpurun_out/pytest_gpu2_$TAG.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/pytest_gpu2_$TAG.log | head -20; exit $rc; }
bash scripts/latency_trace.sh > gpurun_out/lat2_$TAG.txt 2>&1 || exit $?
head -25 gpurun_out/lat2_$TAG.txt
cd $GRAFT_REPO_ROOT && bash scripts/gpu_r04_end2.sh $TAG
