#!/bin/bash
# Round 6: the top-layer parity tests, then the kernel-pass ablations of k_top_mma (build/abl/*.so)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
T=${1:-r06c}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_top_mma.py \
  tests/test_gpu_semantics.py::test_config3_one_degree_step > gpurun_out/pytest_$T.log 2>&1 || { tail -40 gpurun_out/pytest_$T.log; exit 1; }
tail -2 gpurun_out/pytest_$T.log
shift
bash scripts/gpu_abl.sh $T config3 "$@"
