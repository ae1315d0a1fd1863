#!/bin/bash
# A/B of two builds of libfpm_hip.so on one box: build/libfpm_hip_old.so vs the in-tree library, alternated
# (old, new, old, new), each through scripts/warp_layers.sh.  The in-tree library is restored at the end.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
LIB=fastest_image_pattern_matching_amd/lib/libfpm_hip.so
cp $LIB build/libfpm_hip_cur.so
for v in old new old new; do
  if [ $v = old ]; then cp build/libfpm_hip_old.so $LIB; else cp build/libfpm_hip_cur.so $LIB; fi
  echo "== $v"; bash scripts/warp_layers.sh | grep -v "^product" || { cp build/libfpm_hip_cur.so $LIB; exit 1; }
done
cp build/libfpm_hip_cur.so $LIB
