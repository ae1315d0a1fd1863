#!/bin/bash
# k_pyr_down_s chunk height A/B (FPM_PYR_OH 32 vs 16): pyramid parity tests at 16, then the bench's kernel pass under
# rocprofv3 --kernel-trace --stats at each height; per-launch-position times by scripts/layer_times.py
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pyr_ab
mkdir -p $OUT && cd $ROOT && export TMPDIR=/tmp
FPM_PYR_OH=16 timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -k "pyr or src7 or config1" > $OUT/pytest16.log 2>&1 || { tail -5 $OUT/pytest16.log; exit 1; }
tail -1 $OUT/pytest16.log
for oh in 32 16; do
  cd /tmp && FPM_PYR_OH=$oh timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/p$oh -o run --output-format csv -- python3 $ROOT/bench.py --kernel-pass-only --steps 30 > $OUT/kpass$oh.json 2> $OUT/kpass$oh.log || exit 1
  cd $ROOT && echo "== OH $oh" && python3 scripts/layer_times.py $OUT/p$oh/run_kernel_trace.csv | grep pyr
done
