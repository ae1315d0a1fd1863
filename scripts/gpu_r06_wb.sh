#!/bin/bash
# Round 6: the whole GPU suite on the in-tree library, then its default-workload kernel pass against build/abl
# variants, twice (alternated).  usage: scripts/gpu_r06_wb.sh tag variant...
TAG=${1:-r06wb}; shift
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
bash scripts/gpu_abl.sh ${TAG}a src7 "$@" && bash scripts/gpu_abl.sh ${TAG}b src7 "$@"
