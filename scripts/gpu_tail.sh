#!/bin/bash
# Src10 +-180 host tail on the GPU box: the device-overlap GPU tests, then configs[2] stress latency (device + host
# split) with the tail's stage clocks (FPM_TAIL_TIMES) and the fixture merge timing; usage: scripts/gpu_tail.sh tag
TAG=${1:-tail}
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 300 --timeout-method thread -k "src10" > gpurun_out/pytest_tail_$TAG.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_tail_$TAG.log; [ $rc -ne 0 ] && exit $rc
FPM_POOL_TRACE=1 FPM_TAIL_TIMES=1 timeout -k 10 300 python3 scripts/bench_configs.py 20 --no-cpu --only=1 --no-pipe > gpurun_out/cfg_tail_$TAG.jsonl 2> gpurun_out/cfg_tail_$TAG.err || { tail -5 gpurun_out/cfg_tail_$TAG.err; exit 1; }
cat gpurun_out/cfg_tail_$TAG.jsonl; grep -c "^tail" gpurun_out/cfg_tail_$TAG.err; grep "^tail\\|^pool\\|^overlap" gpurun_out/cfg_tail_$TAG.err | head -40
if [ -n "$PROF" ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_tail_$TAG -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_configs.py 5 --no-cpu --only=1 --no-pipe > /dev/null 2>&1 || exit 1
  cd $GRAFT_REPO_ROOT && S=$(find gpurun_out/prof_tail_$TAG -name '*kernel_stats.csv' | head -1) && cut -d, -f1-4 $S | grep -i "overlap\|Name"
fi
