#!/bin/bash
# Angle-shard probe on one GPU: the shard parity tests, then bench_angle_shard.py --simulate for Src10 +-180 and Src7.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-shard}
mkdir -p $OUT
cd $ROOT && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_angle_shard.py -q -x --timeout 120 > $OUT/pytest_shard_$TAG.log 2>&1 && \
timeout -k 10 300 python -u scripts/bench_angle_shard.py --simulate 1,2,4,8 --steps 10 > $OUT/shard_src10_$TAG.json 2> $OUT/shard_src10_$TAG.log && \
timeout -k 10 300 python -u scripts/bench_angle_shard.py --config src7 --simulate 1,2,4,8 --steps 20 > $OUT/shard_src7_$TAG.json 2> $OUT/shard_src7_$TAG.log
rc=$?; tail -3 $OUT/pytest_shard_$TAG.log; cat $OUT/shard_src10_$TAG.json $OUT/shard_src7_$TAG.json; exit $rc
