#!/bin/bash
# k_roi_warp's SQ counters in the bench's kernel pass (43 sources per pass, Src7 layers 2, 1, 0 per pass): issue
# counts, LDS array cycles and bank-conflict cycles, wave cycles.  Two separate --pmc passes (<= 8 SQ counters each);
# usage: scripts/warp_pmc.sh tag
TAG=${1:-w}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/warp_pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $ROOT/bench.py --kernel-pass-only --steps 2"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $OUT/sq1 -o run --output-format csv -- $B > /dev/null 2> $OUT/sq1.log || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d $OUT/sq2 -o run --output-format csv -- $B > /dev/null 2> $OUT/sq2.log || exit $?
cd $ROOT
python3 scripts/pmc_dispatch.py k_roi_warp $OUT/sq1 $OUT/sq2 > $OUT/summary.txt
cat $OUT/summary.txt
