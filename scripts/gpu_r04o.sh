#!/bin/bash
# Round-4: kernel timeline of the README Test4 search (Src3/Dst3, Tol 0, TargetNum 38)
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/tr_test4 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_configs.py 10 --no-cpu --ref-only --only=1 --no-pipe > $OUT/tr_test4.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
python3 scripts/step_timeline.py $(find $OUT/tr_test4 -name '*kernel_trace.csv' | head -1) > $OUT/tl_test4.txt
cat $OUT/tl_test4.txt
