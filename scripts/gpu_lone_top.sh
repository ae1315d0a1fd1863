#!/bin/bash
# Lone Src7 search through the C ABI (latency probe): the default top-layer choice against FPM_TOP_MMA=0, alternated.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
python3 scripts/make_src7_raw.py > /dev/null || exit 1
for v in d 0 d 0; do
  if [ $v = 0 ]; then export FPM_TOP_MMA=0; else unset FPM_TOP_MMA; fi
  timeout -k 10 120 ./build/latency_probe gpurun_out/dst7.raw 762 521 gpurun_out/src7.raw 4024 3036 100 > gpurun_out/lone_$v.json || exit $?
  echo "FPM_TOP_MMA=$v $(cat gpurun_out/lone_$v.json)"
done
