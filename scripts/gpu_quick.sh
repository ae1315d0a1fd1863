#!/bin/bash
# Quick GPU check after a kernel change: GPU parity tests, then the bench's per-kernel pass (batch 32) and the
# Src10 +-180 merge stage timer.  usage: scripts/gpu_quick.sh tag
TAG=${1:-q}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 > $OUT/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu_$TAG.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u bench.py --kernel-pass-only --steps 50 > $OUT/kpass_$TAG.json 2> $OUT/kpass_$TAG.log || exit $?
python3 - $OUT/kpass_$TAG.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); st = d["steps"]
for k, v in sorted(d["kernels"].items(), key=lambda x: -x[1]["ms_total"]):
    print(f"{k:12s} {v['ms_total'] / st * 1000:8.1f} us/step {v['launches'] // st} launches {v['bytes'] / v['ms_total'] / 1e6:8.1f} GB/s")
print("total us/step", sum(v["ms_total"] for v in d["kernels"].values()) / st * 1000)
PY
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace_$TAG -o run --output-format csv -- python3 $ROOT/bench.py --kernel-pass-only --steps 5 > /dev/null 2> $OUT/trace_$TAG.log || exit $?
cd $ROOT && python3 scripts/step_timeline.py $(find $OUT/trace_$TAG -name '*kernel_trace.csv' | head -1)
for t in 1 8; do FPM_HOST_THREADS=$t python3 scripts/merge_timing.py 300; done
lscpu | grep -i "model name"
timeout -k 10 300 python -u scripts/bench_configs.py 20 --no-cpu > $OUT/configs_$TAG.jsonl 2> $OUT/configs_$TAG.log || exit $?
cut -c1-330 $OUT/configs_$TAG.jsonl
exit 0
