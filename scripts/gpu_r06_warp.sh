#!/bin/bash
# Round 6: k_roi_warp3 interior layout -- parity (parity / fuzz / semantics suites), then the default workload's
# kernel pass for the product build and the measurement variants in build/abl.  usage: scripts/gpu_r06_warp.sh tag v...
TAG=${1:-r06w}; shift
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_semantics.py > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
bash scripts/gpu_abl.sh $TAG src7 "$@"
