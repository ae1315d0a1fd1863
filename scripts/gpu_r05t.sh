#!/bin/bash
# Round 5: lone-search small-template / eval forms -- the GPU suite, then every config's latency with the eight-wave
# small-template form off (FPM_SMALL_NT=0) vs the default, alternated on one box, and the Src7 latency probe
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_r05t.log 2>&1; rc=$?
tail -1 gpurun_out/pytest_r05t.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/pytest_r05t.log | head -20; exit $rc; }
for v in n0 d n0b db; do
  case $v in n0*) E="FPM_SMALL_NT=0";; *) E="FPM_NONE=1";; esac
  env $E timeout -k 10 300 python -u scripts/bench_configs.py 20 --no-cpu --no-pipe > gpurun_out/cfg_r05t_$v.jsonl 2> gpurun_out/cfg_r05t_$v.err || { tail -3 gpurun_out/cfg_r05t_$v.err; exit 1; }
  echo "== $v"; python3 -c "
import json
for l in open('gpurun_out/cfg_r05t_$v.jsonl'):
    d = json.loads(l); print(d['config'][:40], d['gpu_ms_per_search'], d['last_pass_device_ms'], d['last_pass_host_ms'])"
done
python3 scripts/make_src7_raw.py > /dev/null && timeout -k 10 120 ./build/latency_probe gpurun_out/dst7.raw 762 521 gpurun_out/src7.raw 4024 3036 100 > gpurun_out/latency_r05t.json && cat gpurun_out/latency_r05t.json
