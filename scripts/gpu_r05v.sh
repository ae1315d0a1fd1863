#!/bin/bash
# Round 5: k_overlap_pairs at 4 waves per SIMD (FPM_OV_WPE=4) vs 3 -- overlap tests with it, Src10 +-180 tail A/B
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
FPM_OV_WPE=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_overlap.py -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_r05v.log 2>&1; rc=$?
tail -1 gpurun_out/pytest_r05v.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/pytest_r05v.log | head -20; exit $rc; }
for v in w3 w4 w3b w4b; do
  case $v in w4*) E="FPM_OV_WPE=4";; *) E="FPM_NONE=1";; esac
  env $E FPM_TAIL_TIMES=1 timeout -k 10 200 python -u scripts/bench_configs.py 20 --no-cpu --only=1 --no-pipe > gpurun_out/tail_r05v_$v.jsonl 2> gpurun_out/tail_r05v_$v.err || { tail -3 gpurun_out/tail_r05v_$v.err; exit 1; }
  echo "== $v"; grep overlap-dev gpurun_out/tail_r05v_$v.err | tail -2
  python3 -c "import json; d=json.loads(open('gpurun_out/tail_r05v_$v.jsonl').readline()); print(d['gpu_ms_per_search'], d['last_pass_device_ms'], d['last_pass_host_ms'])"
done
