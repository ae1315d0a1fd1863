#!/bin/bash
# SQ counters of the bench workload (batch dispatches only), two --pmc passes, no kernel/sys trace;
# per-kernel means into gpurun_out/pmc_sq_<tag>/summary.csv.
TAG=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_sq_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $ROOT/bench.py --steps 3 --warmup 1 --cpu-budget 0 --skip-latency --contexts 1"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA -d $OUT/p1 -o run --output-format csv -- $B > $OUT/p1.json 2> $OUT/p1.log || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL -d $OUT/p2 -o run --output-format csv -- $B > $OUT/p2.json 2> $OUT/p2.log || exit $?
python3 $ROOT/scripts/pmc_summary.py $OUT/summary.csv $OUT/p1 $OUT/p2 || exit $?
echo ok
