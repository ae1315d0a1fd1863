"""Decode the reference's own template images into tests/golden/templates.npz (run in the build container only;
/root/reference does not exist on the GPU box).  Decoding follows cv::imread(IMREAD_GRAYSCALE) semantics via
fastest_image_pattern_matching_amd.images.imread_gray.  Src6.jpg (the README Test6 source, README.md:70) is
copied verbatim as a data file for the real-image known-answer test."""
import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from fastest_image_pattern_matching_amd.images import imread_gray  # noqa: E402

REF = "/root/reference/Test Images"
NAMES = ["Dst1.bmp", "Dst3.bmp", "Dst4.bmp", "Dst5.bmp", "Dst6.bmp", "Dst7.bmp", "Dst8.bmp", "Dst9.bmp", "Dst10.jpg"]

if __name__ == "__main__":
    arrs = {os.path.splitext(n)[0]: imread_gray(os.path.join(REF, n)) for n in NAMES}
    np.savez_compressed(os.path.join(HERE, "templates.npz"), **arrs)
    shutil.copyfile(os.path.join(REF, "Src6.jpg"), os.path.join(HERE, "Src6.jpg"))
    for k, v in arrs.items():
        print(k, v.shape, v.dtype, int(v.min()), int(v.max()), float(v.mean()))
