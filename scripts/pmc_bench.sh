#!/bin/bash
# HBM traffic and instruction issue of a bench workload's per-kernel pass (bench.py --kernel-pass-only): FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes (no kernel/sys trace), as MI355X_MICROARCH.md's HBM section prescribes, plus two
# SQ passes (instruction counts, LDS / matrix-pipe cycles); summarised per kernel (FETCH_SIZE x2 gfx950 correction) by
# scripts/pmc_summary.py into gpurun_out/pmc_bench_<tag>/summary.csv.
# usage: scripts/pmc_bench.sh [tag] [workload: src7 (default) | config3]
TAG=${1:-r01}
W=${2:-src7}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_bench_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $ROOT/bench.py --workload $W --kernel-pass-only --steps 3"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B > $OUT/fetch.json 2> $OUT/fetch.log || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B > $OUT/write.json 2> $OUT/write.log || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT -d $OUT/sq1 -o run --output-format csv -- $B > $OUT/sq1.json 2> $OUT/sq1.log || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d $OUT/sq2 -o run --output-format csv -- $B > $OUT/sq2.json 2> $OUT/sq2.log || exit $?
python3 $ROOT/scripts/pmc_summary.py $OUT/summary.csv $OUT/fetch $OUT/write $OUT/sq1 $OUT/sq2 || exit $?
grep -E "FETCH_BYTES|WRITE_BYTES" $OUT/summary.csv | grep -v rocclr | cut -c1-160
