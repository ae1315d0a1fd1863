#!/bin/bash
# Host-tail timing on the GPU box's CPU (no GPU use): the library's fpm_merge_candidates over the Src10 +-180 records
# (tests/golden/merge_src10_180.npz) at 1 / 8 / 16 host threads, with the per-stage clocks of its last calls.
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
for t in 1 8 16; do
  echo "== FPM_HOST_THREADS=$t"
  FPM_TAIL_TIMES=1 FPM_HOST_THREADS=$t timeout -k 5 120 python3 scripts/merge_time.py 300 > /tmp/mt.txt 2>&1 || { cat /tmp/mt.txt; exit 1; }
  grep "^tail" /tmp/mt.txt | tail -3
  grep "^threads" /tmp/mt.txt
  FPM_HOST_THREADS=$t timeout -k 5 60 ./build/pool_probe
done
