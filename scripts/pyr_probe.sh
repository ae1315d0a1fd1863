#!/bin/bash
# pyrDown probe: GPU pyramid parity tests, then the kernel pass under rocprofv3 --stats for each workgroup count in
# WGS (FPM_PYR_WGS); prints the pyrDown rows.  SKIP_TESTS=1 skips the tests.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $ROOT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "${TESTS:-pyr or multichunk or learn}" --timeout 120 --timeout-method thread > $OUT/pyr_tests.log 2>&1; rc=$?
  tail -3 $OUT/pyr_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
for g in ${WGS:-2048 4096}; do
  export FPM_PYR_WGS=$g
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/pyr_g$g -o run --output-format csv -- python3 $ROOT/bench.py --kernel-pass-only --steps 30 > $OUT/pyr_g$g.json 2> $OUT/pyr_g$g.log; rc=$?
  [ $rc -eq 0 ] || { echo "g=$g rc=$rc"; exit $rc; }
  echo "WGS=$g"; find $OUT/pyr_g$g -name '*kernel_stats.csv' -exec grep -h pyr_down {} \; | cut -c1-30,100-200
done
exit 0
