#!/bin/bash
# Round 5: k_roi_eval in 40-row blocks (three workgroups per CU) -- the GPU suite, then bench A/B against
# build/libfpm_hip_old.so (48-row blocks), alternated
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_r05o.log 2>&1; rc=$?
tail -1 gpurun_out/pytest_r05o.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/pytest_r05o.log | head -20; exit $rc; }
LIB=fastest_image_pattern_matching_amd/lib/libfpm_hip.so
cp $LIB build/libfpm_hip_cur.so
run() {   # name
  local n=$1
  timeout -k 10 300 python -u bench.py --steps 100 --cpu-budget 0 --skip-latency > gpurun_out/sp_$n.json 2> gpurun_out/sp_$n.log || { tail -3 gpurun_out/sp_$n.log; cp build/libfpm_hip_cur.so $LIB; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/sp_$n.json')); k=d['kernels']; print('$n', d['value'], d['ms_per_step'], d['roofline']['frac'], 'roi_eval', round(k['roi_eval']['ms_total'], 2))"
}
for v in old new old2 new2; do
  case $v in old*) cp build/libfpm_hip_old.so $LIB;; *) cp build/libfpm_hip_cur.so $LIB;; esac
  run $v
done
cp build/libfpm_hip_cur.so $LIB
