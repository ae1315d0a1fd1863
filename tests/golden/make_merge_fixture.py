"""Generate tests/golden/merge_src10_180.npz: the oracle's candidate records and results of one large search.

BASELINE configs[2] stress — Src10 surrogate 3648x3648, Dst10 54x54, ToleranceAngle 180, TargetNum 100, Score 0.7:
4935 top-layer candidates (47 angles) refined to 144 results through clusters of ~34 duplicate detections, i.e. the
case where the host tail's rotated-rectangle filter runs its component-parallel path.  The records (fpm_candidate,
push order) and the results (s_SingleTargetMatch rows) both come from the oracle's sequential restatement
(oracle/fpm_oracle.cpp); tests/test_angle_shard.py merges the records with libfpm_hip.so's fpm_merge_candidates
at 1 and 8 host threads and expects the oracle's results bit for bit.

Run from the repo root after `make -C oracle` (about 10 s of oracle time):  python tests/golden/make_merge_fixture.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from fastest_image_pattern_matching_amd import synth  # noqa: E402
from tests import oracle  # noqa: E402

PARAMS = dict(max_pos=100, score=0.7, tolerance_angle=180.0, max_overlap=0.0)


def main():
    T = synth.load_templates()
    s, t = synth.src10_scene(T["Dst10"])
    o = oracle.OracleMatcher().set(**PARAMS)
    assert o.learnPattern(t)
    res = np.array(o.match(s), np.float64)
    rec = o.candidates()
    np.savez_compressed(os.path.join(HERE, "merge_src10_180.npz"), records=rec.view(np.uint8), results=res,
                        tmpl_wh=np.array([t.shape[1], t.shape[0]]),
                        params=np.array([PARAMS["max_pos"], PARAMS["score"], PARAMS["tolerance_angle"],
                                         PARAMS["max_overlap"]]))
    print(f"{len(rec)} records, {len(res)} results")


if __name__ == "__main__":
    main()
