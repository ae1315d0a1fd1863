cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for n in 43 8; do echo "== MB_NSRC=$n"; MB_NSRC=$n MB_WARP_ONLY=1 timeout -k 10 120 ./build/roi_mb 20 || exit $?; done > gpurun_out/mb_sweep.txt 2>&1
cat gpurun_out/mb_sweep.txt
