#!/bin/bash
# Round 5: k_overlap_pairs without the reference's rare closest-pair reduction on the device (those pairs go to the
# host): scratch 2688 -> 576 bytes per lane -- overlap / Src10 parity tests, then the Src10 +-180 tail against
# build/libfpm_hip_old.so, alternated
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_overlap.py tests/test_gpu_parity.py -q -x -k "overlap or src10 or config2" --timeout 200 --timeout-method thread > gpurun_out/pytest_r05s.log 2>&1; rc=$?
tail -1 gpurun_out/pytest_r05s.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/pytest_r05s.log | head -20; exit $rc; }
LIB=fastest_image_pattern_matching_amd/lib/libfpm_hip.so
cp $LIB build/libfpm_hip_cur.so
for v in old new old2 new2; do
  case $v in old*) cp build/libfpm_hip_old.so $LIB;; *) cp build/libfpm_hip_cur.so $LIB;; esac
  FPM_TAIL_TIMES=1 timeout -k 10 200 python -u scripts/bench_configs.py 20 --no-cpu --only=1 --no-pipe > gpurun_out/tail_r05s_$v.jsonl 2> gpurun_out/tail_r05s_$v.err || { tail -3 gpurun_out/tail_r05s_$v.err; cp build/libfpm_hip_cur.so $LIB; exit 1; }
  echo "== $v"; grep overlap-dev gpurun_out/tail_r05s_$v.err | tail -2; grep "^tail" gpurun_out/tail_r05s_$v.err | tail -2
  python3 -c "import json; d=json.loads(open('gpurun_out/tail_r05s_$v.jsonl').readline()); print(d['gpu_ms_per_search'], d['last_pass_device_ms'], d['last_pass_host_ms'])"
done
cp build/libfpm_hip_cur.so $LIB
