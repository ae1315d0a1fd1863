#!/bin/bash
# The whole GPU suite with the matrix-core top layer forced wherever its layouts fit (FPM_TOP_MMA=1), then with it off
# (FPM_TOP_MMA=0): every search of the suite through each top-layer form.  (Tests that set the switch themselves keep
# their own setting.)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
for v in 1 0; do
  FPM_TOP_MMA=$v timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_forms_$v.log 2>&1; rc=$?
  echo "FPM_TOP_MMA=$v: $(tail -1 gpurun_out/pytest_forms_$v.log)"
  grep "^FAILED" gpurun_out/pytest_forms_$v.log | head -20
  [ $rc -gt 1 ] && exit $rc
done
exit 0
