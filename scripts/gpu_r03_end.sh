#!/bin/bash
# Round-3 closing GPU pass: GPU tests, warp microbenchmark, rocprof kernel pass, default bench, C-ABI latency probe
# (scripts/gpu_r03.sh), then smoke and the PMC traffic of the kernel pass (scripts/pmc_bench.sh); usage: scripts/gpu_r03_end.sh tag
TAG=${1:-r03_end}
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
bash scripts/gpu_r03.sh $TAG || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/smoke_$TAG.log
bash scripts/pmc_bench.sh $TAG
