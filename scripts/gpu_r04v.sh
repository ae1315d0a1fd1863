#!/bin/bash
# Round-4: overlap-pair sweep with four chunks in flight -- GPU suite, single-search and Src10 +-180 timelines
TAG=${1:-r04v}
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -1 gpurun_out/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/pytest_gpu_$TAG.log | head -20; exit $rc; }
bash scripts/latency_trace.sh > gpurun_out/lat_$TAG.txt 2>&1 || exit $?
grep -E "overlap|pass|config" gpurun_out/lat_$TAG.txt | cut -c1-300
