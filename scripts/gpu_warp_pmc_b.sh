#!/bin/bash
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT && MB_NSRC=43 MB_WARP_ONLY=1 timeout -k 10 120 ./build/roi_mb 20 > gpurun_out/mbB.txt 2>&1 || exit 1
grep -i "warp3" gpurun_out/mbB.txt | head -12
bash scripts/gpu_warp_pmc.sh | grep "^<7, 68, 0, 0, false, false>\|^<7, 68, 0, 3\|^<7, 68, 0, 2"
