#!/bin/bash
# Round 5: k_roi_small in two-wave workgroups (FPM_SMALL_NT=128) -- the whole GPU suite with it forced, then bench A/B
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
FPM_SMALL_NT=128 timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_r05l.log 2>&1; rc=$?
tail -1 gpurun_out/pytest_r05l.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/pytest_r05l.log | head -20; exit $rc; }
run() {   # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 100 --cpu-budget 0 --skip-latency > gpurun_out/sn_$n.json 2> gpurun_out/sn_$n.log || { tail -3 gpurun_out/sn_$n.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/sn_$n.json')); k=d['kernels']; print('$n', d['value'], d['ms_per_step'], d['roofline']['frac'], 'roi_small', round(k['roi_small']['ms_total'], 2))"
}
run d FPM_NONE=1
run n4 FPM_SMALL_NT=128
run n3 FPM_SMALL_NT=128 FPM_SMALL_WPE=3
run db FPM_NONE=1
run n4b FPM_SMALL_NT=128
run n3b FPM_SMALL_NT=128 FPM_SMALL_WPE=3
