#!/bin/bash
# Round 5: lone-search latency with the 16-row-item correlation (FPM_CORR16=1) vs the default, alternated
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
python3 scripts/make_src7_raw.py > /dev/null || exit 1
for v in d c16 d2 c162; do
  case $v in c16*) E="FPM_CORR16=1";; *) E="FPM_NONE=1";; esac
  env $E timeout -k 10 120 ./build/latency_probe gpurun_out/dst7.raw 762 521 gpurun_out/src7.raw 4024 3036 100 > gpurun_out/latency_r05r_$v.json || exit $?
  echo "$v $(cat gpurun_out/latency_r05r_$v.json)"
done
