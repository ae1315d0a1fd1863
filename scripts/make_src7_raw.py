"""Writes gpurun_out/src7.raw (4024x3036 Src7 surrogate, seed 7) and gpurun_out/dst7.raw for scripts/latency_probe."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fastest_image_pattern_matching_amd import synth  # noqa: E402

t = synth.load_templates()["Dst7"]
s, _ = synth.src7_scene(t, seed=7)
os.makedirs("gpurun_out", exist_ok=True)
np.ascontiguousarray(s).tofile("gpurun_out/src7.raw")
np.ascontiguousarray(t).tofile("gpurun_out/dst7.raw")
print(t.shape, s.shape)
