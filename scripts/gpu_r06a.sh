#!/bin/bash
# Round 6, first check of the matrix-core top layer (k_top_mma): its parity tests and the top-layer parity tests of the
# existing suite, then the configs[3] bench (A/B against the split top layer) and a rocprofv3 kernel summary.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
T=${1:-r06a}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_top_mma.py \
  tests/test_gpu_semantics.py::test_config3_one_degree_step \
  "tests/test_gpu_parity.py::test_config2_src10_rotation_sweep" "tests/test_gpu_parity.py::test_config2_src10_blockmax" \
  "tests/test_gpu_parity.py::test_src7_top_layer_forms" > gpurun_out/pytest_$T.log 2>&1 || { tail -40 gpurun_out/pytest_$T.log; exit 1; }
tail -3 gpurun_out/pytest_$T.log
timeout -k 10 300 python -u bench.py --workload config3 --steps 20 --warmup 3 --cpu-budget 0 --skip-latency > gpurun_out/bench_c3_$T.json 2> gpurun_out/bench_c3_$T.log || { tail -20 gpurun_out/bench_c3_$T.log; exit 1; }
FPM_TOP_MMA=0 timeout -k 10 300 python -u bench.py --workload config3 --steps 20 --warmup 3 --cpu-budget 0 --skip-latency > gpurun_out/bench_c3_split_$T.json 2> gpurun_out/bench_c3_split_$T.log || { tail -20 gpurun_out/bench_c3_split_$T.log; exit 1; }
python3 - <<PY
import json
for f in ("bench_c3_$T.json", "bench_c3_split_$T.json"):
    d = json.load(open("gpurun_out/" + f))
    k = d["kernels"]
    print(f, d["value"], d["ms_per_step"], {n: (round(v["ms_total"] / max(v["launches"], 1) * 1000, 1), v["launches"]) for n, v in k.items()})
PY
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$T -o kp --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload config3 --kernel-pass-only --steps 2 --warmup 1 --cpu-budget 0 > $GRAFT_REPO_ROOT/gpurun_out/kp_$T.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/kp_$T.log; exit 1; }
cd $GRAFT_REPO_ROOT && find gpurun_out/prof_$T -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/kernel_stats_$T.csv
head -20 gpurun_out/kernel_stats_$T.csv | cut -c1-160
