#!/bin/bash
# PMC passes over the ROI microbenchmark (each counter group in its own run; no kernel/sys trace)
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-roi}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS -d $OUT/p1 -o run --output-format csv -- $ROOT/build/roi_mb 2 > $OUT/p1.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS_LOAD -d $OUT/p2 -o run --output-format csv -- $ROOT/build/roi_mb 2 > $OUT/p2.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_UNALIGNED_STALL SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC -d $OUT/p3 -o run --output-format csv -- $ROOT/build/roi_mb 2 > $OUT/p3.log 2>&1 || echo "p3 counters unavailable (see p3.log)"
python3 $ROOT/scripts/pmc_summary.py $OUT/summary.csv $OUT/p1 $OUT/p2 $OUT/p3
echo ok
