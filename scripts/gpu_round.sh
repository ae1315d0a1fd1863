#!/bin/bash
# One GPU-box pass: GPU parity tests, smoke, bench, rocprofv3 kernel trace.  Every GPU step has its own time
# limit; a fault / abort / timeout (anything but exit 0 or a plain test failure 1) ends the script there.
# usage: scripts/gpu_round.sh [tag] [pytest-args...]
TAG=${1:-r01}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $ROOT
stop_if_fault() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "FAULT/TIMEOUT rc=$1 in $2: stopping"; exit "$1"; fi; }

make -C fastest_image_pattern_matching_amd/csrc -j16 > $OUT/build.log 2>&1 && make -C oracle >> $OUT/build.log 2>&1 || { echo build failed; exit 3; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf "$@" > $OUT/pytest_gpu_$TAG.log 2>&1; rc=$?
echo "pytest gpu rc=$rc"; tail -5 $OUT/pytest_gpu_$TAG.log; stop_if_fault $rc pytest
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 $OUT/smoke_$TAG.log; stop_if_fault $rc smoke
timeout -k 10 420 python -u bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.log; rc=$?
echo "bench rc=$rc"; cat $OUT/bench_$TAG.json | head -c 3000; echo; stop_if_fault $rc bench
cd /tmp && timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv -- python3 $ROOT/bench.py --kernel-pass-only --steps 50 > $OUT/prof_bench_$TAG.json 2> $OUT/prof_$TAG.log; rc=$?
echo "rocprof rc=$rc"; stop_if_fault $rc rocprof
find $OUT/prof_$TAG -name '*stats*' | head
exit 0
