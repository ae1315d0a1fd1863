"""Which reference screenshot labels does each TM_CCORR arithmetic reproduce?  (CPU, oracle only.)

The reference computes TM_CCORR with OpenCV's float32 DFT crossCorr at the top layer always
(TemplateMatcher.cpp:177 -> :514; MatchToolDlg.cpp:858 -> :1304) and at every refinement layer when its SIMD switch
is off (MatchToolDlg.cpp:1277; the MFC tool's "SIMD" checkbox starts unchecked, MatchTool.rc:118).  The parity
oracle restates TM_CCORR as the exact integer sum rounded once.  This script runs the four screenshot pins
(tests/golden/reference_pins.json) in MFC semantics under

    ccorr  exact | f32dft     (oracle orc_set_ccorr_mode 0 | 1)
    simd   on    | off        (fpm_params.use_simd)

and prints, per pin and mode, the detection count, the largest cross residual and the labels not reproduced.

    python scripts/ccorr_sensitivity.py [--json out.json]

Test infrastructure only (imports the oracle); tests/test_reference_pins.py asserts the table it prints.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import oracle  # noqa: E402
from tests.test_reference_pins import PINS, _load, cross_residual, label_mismatches  # noqa: E402

MODES = [("exact", 0, 1), ("exact", 0, 0), ("f32dft", 1, 1), ("f32dft", 1, 0)]


def run(name, ccorr, simd):
    pin = PINS[name]
    s, t = _load(pin)
    o = oracle.OracleMatcher().set(semantics=1, **dict(pin["params"], use_simd=simd)).set_ccorr_mode(ccorr)
    assert o.learnPattern(t)
    res = o.match(s)
    out = {"count": len(res)}
    if len(res) == pin["count"]:
        out["residual"] = round(cross_residual(pin, s.shape, res), 3)
        out["mismatch"] = label_mismatches(pin, s.shape, res)
    return out


def main():
    table = {}
    for name in sorted(PINS):
        for tag, ccorr, simd in MODES:
            t0 = time.time()
            r = run(name, ccorr, simd)
            key = f"{tag}/simd{'on' if simd else 'off'}"
            table.setdefault(name, {})[key] = r
            print(f"{name:12s} {key:14s} count {r['count']:3d} (pin {PINS[name]['count']:3d}) "
                  f"residual {r.get('residual')} mismatched {r.get('mismatch')}  [{time.time() - t0:.1f} s]",
                  flush=True)
    if len(sys.argv) > 2 and sys.argv[1] == "--json":
        with open(sys.argv[2], "w") as fh:
            json.dump(table, fh, indent=1)


if __name__ == "__main__":
    main()
