#!/bin/bash
# k_top_mma's SQ counters in the configs[3] kernel pass (one pass: the list launch and the fallback launch); two
# separate --pmc passes (<= 8 SQ counters each).  usage: scripts/top_pmc.sh tag
TAG=${1:-t}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/top_pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $ROOT/bench.py --workload config3 --kernel-pass-only --steps 1 --warmup 0"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $OUT/sq1 -o run --output-format csv -- $B > /dev/null 2> $OUT/sq1.log || exit $?
timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d $OUT/sq2 -o run --output-format csv -- $B > /dev/null 2> $OUT/sq2.log || exit $?
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_ACTIVE_INST_MISC -d $OUT/sq3 -o run --output-format csv -- $B > /dev/null 2> $OUT/sq3.log || echo "sq3 failed (counter names)"
cd $ROOT
python3 scripts/pmc_dispatch.py k_top_mma $OUT/sq1 $OUT/sq2 $OUT/sq3 > $OUT/summary.txt
cat $OUT/summary.txt
