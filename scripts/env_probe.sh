#!/bin/bash
# A/B probe of an environment switch: the kernel pass under rocprofv3 --stats with and without ENVVAR=1 (or each
# value in VALS); prints the rows of the kernels matching PAT.  usage: ENVVAR=FPM_X VALS="0 1" PAT=roi_corr bash scripts/env_probe.sh
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for v in ${VALS:-0 1}; do
  export $ENVVAR=$v
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ep_$v -o run --output-format csv -- python3 $ROOT/bench.py --kernel-pass-only --steps 30 > $OUT/ep_$v.json 2> $OUT/ep_$v.log; rc=$?
  [ $rc -eq 0 ] || { echo "$v rc=$rc"; exit $rc; }
  echo "$ENVVAR=$v"
  python3 - $OUT/ep_$v "$PAT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
tot = 0.0
for r in csv.DictReader(open(f)):
    tot += float(r['TotalDurationNs'])
    if sys.argv[2] in r['Name']:
        print(f"  {r['Name'][:70]:70s} calls {r['Calls']:>4} avg {float(r['AverageNs'])/1000:8.1f} us")
print(f"  all kernels total {tot/1e6:.2f} ms")
PY
done
