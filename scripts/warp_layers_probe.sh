#!/bin/bash
# Why layer 0 of k_roi_warp runs at half the per-tile rate of layers 1-2: the warp microbenchmark on layer-0 and
# layer-1 shapes (and the two crossed), then per-dispatch SQ and TCP counters of the bench's kernel pass (8 sources;
# one dispatch per layer per pass, scripts/pmc_dispatch.py).  Each step has its own time limit; any failure ends it.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/warp_layers
mkdir -p $OUT
export TMPDIR=/tmp
cd $ROOT
MB=$ROOT/build/roi_mb
run_mb() { echo "== $1"; env $2 MB_WARP_ONLY=1 timeout -k 10 120 $MB 10 || exit $?; }
{
run_mb "L0 shape" ""
run_mb "L1 shape" "MB_W=2012 MB_H=1518 MB_P=2048 MB_TW=381 MB_TH=261"
run_mb "L0 template, L1-sized source" "MB_W=2012 MB_H=1518 MB_P=2048"
run_mb "L1 template, L0-sized source" "MB_TW=381 MB_TH=261"
} > $OUT/mb.txt 2>&1 || { cat $OUT/mb.txt; exit 1; }
cat $OUT/mb.txt
cd /tmp
B="python3 $ROOT/bench.py --kernel-pass-only --steps 2 --batch 8"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT -d $OUT/sq -o run --output-format csv -- $B > /dev/null 2> $OUT/sq.log || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum -d $OUT/tcp -o run --output-format csv -- $B > /dev/null 2> $OUT/tcp.log || exit $?
cd $ROOT
python3 scripts/pmc_dispatch.py k_roi_warp $OUT/sq $OUT/tcp
