#!/bin/bash
# LDS bank conflicts of the ROI gathers vs the footprint pitch: the warp microbenchmark built with
# -DFPM_FT_PITCH_FORCE=p (footprint rows padded to p dwords where they fit; 0 = the product's odd-pitch rule),
# layer-0 and layer-1 shapes.  Each run has its own time limit; a failure ends the script.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
for p in 0 12 13 14 15 16; do
  for shape in "" "MB_W=2012 MB_H=1518 MB_P=2048 MB_TW=381 MB_TH=261"; do
    out=$(env $shape MB_WARP_ONLY=1 timeout -k 10 120 ./build/roi_mb_p$p 10) || { echo "p=$p failed"; exit 1; }
    echo "p=$p ${shape:-L0} $(echo "$out" | grep -E 'prod warp|warp no staging')" | tr '\n' ' '
    echo
  done
done
