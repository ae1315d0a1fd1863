"""Gray image loading with ``cv::imread(path, IMREAD_GRAYSCALE)`` semantics (src/MatchToolDialog.cpp:314, 341).

* BMP 24/32-bit and palettised: OpenCV's fixed-point BGR->gray, ``(1868*B + 9617*G + 4899*R + 8192) >> 14``
  (applied to the palette for 8-bit images), SURVEY.md Appendix A.12.
* JPEG: the decoder's luminance (libjpeg ``JCS_GRAYSCALE`` output), obtained with PIL ``draft('L')``.
  Parity with OpenCV's bundled libjpeg(-turbo) IDCT is unpinned.
"""
from __future__ import annotations

import numpy as np

CB, CG, CR = 1868, 9617, 4899


def bgr_to_gray(rgb: np.ndarray) -> np.ndarray:
    """OpenCV icvCvt_BGR2Gray_8u_C3C1R on an RGB-ordered array."""
    r = rgb[..., 0].astype(np.int32)
    g = rgb[..., 1].astype(np.int32)
    b = rgb[..., 2].astype(np.int32)
    return ((b * CB + g * CG + r * CR + (1 << 13)) >> 14).astype(np.uint8)


def imread_gray(path: str) -> np.ndarray:
    from PIL import Image  # PIL is only needed to decode files, never on the matching path

    im = Image.open(path)
    fmt = (im.format or "").upper()
    if fmt == "JPEG":
        im.draft("L", im.size)
        if im.mode != "L":
            im = im.convert("L")
        return np.ascontiguousarray(np.asarray(im, dtype=np.uint8))
    if im.mode == "L":
        return np.ascontiguousarray(np.asarray(im, dtype=np.uint8))
    if im.mode == "P":
        pal = np.asarray(im.getpalette()[: 256 * 3], dtype=np.uint8).reshape(-1, 3)
        lut = bgr_to_gray(pal[None, :, :])[0]
        idx = np.asarray(im, dtype=np.uint8)
        return np.ascontiguousarray(lut[idx])
    if im.mode in ("RGB", "RGBA"):
        return bgr_to_gray(np.asarray(im.convert("RGB"), dtype=np.uint8))
    return np.ascontiguousarray(np.asarray(im.convert("L"), dtype=np.uint8))
