#!/bin/bash
# debug_fuzz_case.py for the given seeds, default forms and FPM_TOP_MMA=0.  usage: scripts/gpu_dbg.sh seed...
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
for s in "$@"; do
  echo "== seed $s default"; timeout -k 10 120 python -u scripts/debug_fuzz_case.py $s || exit $?
  echo "== seed $s FPM_TOP_MMA=0"; FPM_TOP_MMA=0 timeout -k 10 120 python -u scripts/debug_fuzz_case.py $s || exit $?
done
