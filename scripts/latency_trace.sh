set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/tr_single -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_configs.py 30 --no-cpu --only=5 --no-pipe > $OUT/tr_single.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/tr_src10 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_configs.py 30 --no-cpu --only=1 --no-pipe > $OUT/tr_src10.log 2>&1
cd $GRAFT_REPO_ROOT
python3 scripts/step_timeline.py $(find $OUT/tr_single -name '*kernel_trace.csv' | head -1) > $OUT/tl_single.txt
python3 scripts/step_timeline.py $(find $OUT/tr_src10 -name '*kernel_trace.csv' | head -1) > $OUT/tl_src10.txt
cat $OUT/tl_single.txt $OUT/tl_src10.txt $OUT/tr_single.log $OUT/tr_src10.log | grep -v "^\[" | cut -c1-200
