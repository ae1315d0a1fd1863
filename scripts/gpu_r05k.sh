#!/bin/bash
# Round 5: k_roi_small with the band row sums over the dead footprint / table region (Src7 layer 3: 4 workgroups per
# CU instead of 3) -- microbenchmark, parity tests, then bench A/B against build/libfpm_hip_old.so (alternated)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
MB_NSRC=43 MB_SMALL_ONLY=1 timeout -k 10 200 ./build/roi_mb 10 > gpurun_out/mb_small_r05k.txt 2>&1 || { tail -5 gpurun_out/mb_small_r05k.txt; exit 1; }
grep -E "small" gpurun_out/mb_small_r05k.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_r05k.log 2>&1; rc=$?
tail -1 gpurun_out/pytest_r05k.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/pytest_r05k.log | head -20; exit $rc; }
LIB=fastest_image_pattern_matching_amd/lib/libfpm_hip.so
cp $LIB build/libfpm_hip_cur.so
run() {   # name
  local n=$1
  timeout -k 10 300 python -u bench.py --steps 100 --cpu-budget 0 --skip-latency > gpurun_out/sk_$n.json 2> gpurun_out/sk_$n.log || { tail -3 gpurun_out/sk_$n.log; cp build/libfpm_hip_cur.so $LIB; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/sk_$n.json')); k=d['kernels']; print('$n', d['value'], d['ms_per_step'], d['roofline']['frac'], {n: round(v['ms_total'], 2) for n, v in k.items() if 'small' in n})"
}
for v in old new old2 new2; do
  case $v in old*) cp build/libfpm_hip_old.so $LIB;; *) cp build/libfpm_hip_cur.so $LIB;; esac
  run $v
done
cp build/libfpm_hip_cur.so $LIB
