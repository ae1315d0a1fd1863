#!/bin/bash
# BASELINE configs / README inputs (latency view, one context) with the default top-layer choice and with
# FPM_TOP_MMA=0 (the split / fused forms), to place k_top_mma's applicability threshold.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
for v in d 0; do
  if [ $v = 0 ]; then export FPM_TOP_MMA=0; else unset FPM_TOP_MMA; fi
  timeout -k 10 500 python -u scripts/bench_configs.py 10 --no-cpu --no-pipe > gpurun_out/cfgab_$v.jsonl 2> gpurun_out/cfgab_$v.log || { tail -5 gpurun_out/cfgab_$v.log; exit 1; }
done
python3 - <<'PY'
import json
def load(f):
    return {json.loads(l)['config'][:70]: json.loads(l) for l in open(f)}
a=load('gpurun_out/cfgab_d.jsonl'); b=load('gpurun_out/cfgab_0.jsonl')
for k in a: print(f"{k:72s} default {a[k]['gpu_ms_per_pass']:.3f} ({a[k]['last_pass_device_ms']:.3f})  mma0 {b[k]['gpu_ms_per_pass']:.3f} ({b[k]['last_pass_device_ms']:.3f})")
PY
