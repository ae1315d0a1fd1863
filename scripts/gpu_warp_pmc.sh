#!/bin/bash
# k_roi_warp3's LDS cycles by ablation: the ROI microbenchmark's warp section (layer 0, 43 Src7 sources) under one SQ
# --pmc pass (LDS array cycles, bank-conflict cycles, LDS / VALU instructions, waves) per kernel instantiation: the
# product form and its ablations (no staging, no interpolation, addressing only, no stores, no interior rows).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/warp_pmc
mkdir -p $OUT && export TMPDIR=/tmp && cd /tmp
MB_NSRC=43 MB_WARP_ONLY=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU -d $OUT/sq -o run --output-format csv -- $ROOT/build/roi_mb 3 > $OUT/mb.txt 2> $OUT/mb.log || exit $?
cd $ROOT && python3 scripts/pmc_summary.py $OUT/summary.csv $OUT/sq > /dev/null && python3 - <<'PY'
import csv, collections
d = collections.defaultdict(dict)
for r in csv.DictReader(open('gpurun_out/warp_pmc/summary.csv')):
    if 'k_roi_warp3' in r['kernel'] and '@grid' not in r['kernel']:
        d[r['kernel']][r['counter']] = float(r['mean_per_dispatch'])
for k, c in d.items():
    print(k[k.index('<'):k.index('>') + 1], {n: f"{v:.3g}" for n, v in c.items()})
PY
