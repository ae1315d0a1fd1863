#!/bin/bash
# Round-4: incremental plain-path peak loop -- GPU suite, README Test4 timeline, README inputs
TAG=${1:-r04p}
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/pytest_gpu_$TAG.log | head -20; exit $rc; }
bash scripts/gpu_r04o.sh || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u scripts/bench_configs.py 10 --ref-only > gpurun_out/configs_ref_$TAG.jsonl 2> gpurun_out/configs_ref_$TAG.log || { tail -5 gpurun_out/configs_ref_$TAG.log; exit 1; }
cut -c1-420 gpurun_out/configs_ref_$TAG.jsonl
