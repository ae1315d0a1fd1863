#!/bin/bash
# Round 5: the overlap filter's pair list in regions with their own counters -- overlap and Src10 parity tests, then
# the Src10 +-180 tail stage times with one counter vs the default, alternated
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_overlap.py tests/test_gpu_parity.py -q -x -k "overlap or src10 or config2" --timeout 200 --timeout-method thread > gpurun_out/pytest_r05p.log 2>&1; rc=$?
tail -1 gpurun_out/pytest_r05p.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/pytest_r05p.log | head -20; exit $rc; }
for v in c1 cd c1b cdb; do
  case $v in c1*) E="FPM_OV_CTRS=1";; *) E="FPM_NONE=1";; esac
  env $E FPM_TAIL_TIMES=1 timeout -k 10 200 python -u scripts/bench_configs.py 20 --no-cpu --only=1 --no-pipe > gpurun_out/tail_r05p_$v.jsonl 2> gpurun_out/tail_r05p_$v.err || { tail -3 gpurun_out/tail_r05p_$v.err; exit 1; }
  echo "== $v"; grep overlap-dev gpurun_out/tail_r05p_$v.err | tail -3; grep "^tail" gpurun_out/tail_r05p_$v.err | tail -2
  python3 -c "import json; d=json.loads(open('gpurun_out/tail_r05p_$v.jsonl').readline()); print(d['gpu_ms_per_search'], d['last_pass_device_ms'], d['last_pass_host_ms'])"
done
