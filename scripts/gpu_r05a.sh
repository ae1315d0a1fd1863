#!/bin/bash
# pyramid walker + sampler microbenchmarks, then the round-5 check (scripts/gpu_r05.sh)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 120 ./build/pyr_walk 43 > gpurun_out/pyr_walk_r05a.txt 2>&1 || exit $?
grep -E "copy4 U4 g8192|read4|product|MISMATCH|FAIL" gpurun_out/pyr_walk_r05a.txt | head
timeout -k 10 180 ./build/warp4_bench > gpurun_out/warp4_r05a.txt 2>&1 || exit $?
grep -E "warp|FAIL" gpurun_out/warp4_r05a.txt | head -40
bash scripts/gpu_r05.sh r05a
