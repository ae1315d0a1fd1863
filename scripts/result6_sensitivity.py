"""Sensitivity of the Result6.jpg label order to decoder-level changes of the source pixels (CPU, oracle only).

The oracle (tests/oracle.py) searches Src6.jpg / Dst6.bmp with the README Test6 parameters in MFC semantics and
reproduces 13 of the 15 score-order labels of the reference's screenshot; labels 8 and 9 (column 3) come out
swapped.  The JPEG decoder that produced the reference tool's pixels (OpenCV's bundled libjpeg behind
imdecode(IMREAD_GRAYSCALE), MatchToolDlg.cpp:62) is unpinned, so this script asks how the order behaves when the
decoded source changes at that level: +-1 LSB on a fraction of the pixels, chosen by a fixed integer hash of the
pixel index and a salt (reproducible, no RNG state).  For every salt it reports how many of the 15 labels the
oracle reproduces.

    python scripts/result6_sensitivity.py [n_salts] [fractions...]

Test infrastructure only (imports the oracle); tests/test_reference_pins.py pins one salt of it.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import oracle  # noqa: E402
from tests.test_reference_pins import PINS, _load, label_mismatches, perturb_lsb  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    fracs = [float(f) for f in sys.argv[2:]] or [0.003, 0.01, 0.03]
    pin = PINS["test6_src6"]
    s, t = _load(pin)
    o = oracle.OracleMatcher().set(semantics=1, **pin["params"])
    assert o.learnPattern(t)
    base = label_mismatches(pin, s.shape, o.match(s))
    print(f"exact decode: mismatched labels {base}")
    for frac in fracs:
        hist = {}
        for salt in range(n):
            bad = tuple(label_mismatches(pin, s.shape, o.match(perturb_lsb(s, salt, frac))))
            hist[bad] = hist.get(bad, 0) + 1
        print(f"+-1 LSB on {frac:.1%} of the pixels, {n} salts:",
              "; ".join(f"{cnt} x mismatched {list(k)}" for k, cnt in sorted(hist.items(), key=lambda kv: -kv[1])))


if __name__ == "__main__":
    main()
