#!/bin/bash
# HBM traffic of the bench workload (its per-kernel pass, bench.py --kernel-pass-only): FETCH_SIZE and WRITE_SIZE in separate --pmc passes (no kernel/sys trace),
# as MI355X_MICROARCH.md's HBM section prescribes; summarised per kernel (FETCH_SIZE x2 gfx950 correction) by
# scripts/pmc_summary.py into gpurun_out/pmc_bench_<tag>/summary.csv.
# usage: scripts/pmc_bench.sh [tag]
TAG=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_bench_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $ROOT/bench.py --kernel-pass-only --steps 3 > $OUT/fetch.json 2> $OUT/fetch.log || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $ROOT/bench.py --kernel-pass-only --steps 3 > $OUT/write.json 2> $OUT/write.log || exit $?
python3 $ROOT/scripts/pmc_summary.py $OUT/summary.csv $OUT/fetch $OUT/write || exit $?
grep -E "FETCH_BYTES|WRITE_BYTES" $OUT/summary.csv
