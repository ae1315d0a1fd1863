"""IMREAD_GRAYSCALE decode pins (the UI's loader src/MatchToolDialog.cpp:314, 341 and
the MFC tool's imdecode(IMREAD_GRAYSCALE), MatchTool/MatchToolDlg.cpp:62).

* 24-bit BMP: OpenCV's fixed-point BGR->gray ``(1868 B + 9617 G + 4899 R + 8192) >> 14``; the expected values below
  are computed by hand from that formula, and the files are written byte by byte here (no encoder involved).
* 8-bit palettised BMP: the palette goes through the same formula (OpenCV CvtPaletteToGray), then indexes; every
  8-bit BMP the reference ships has the identity gray palette, so its gray image is the index plane itself.
* JPEG: the decoder's luminance plane.  Src6.jpg (the only JPEG source the reference ships, one component) decodes
  here with Pillow's libjpeg-turbo (ISLOW IDCT); its hash is pinned together with that decoder identity, so a
  fixture decoded by anything else fails loudly.  Whether OpenCV's bundled libjpeg gives the same plane is
  unpinned (see tests/test_reference_pins.py for what that leaves open on Result6).
"""
import hashlib
import os
import struct

import numpy as np
import pytest

from fastest_image_pattern_matching_amd.images import imread_gray

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SRC6_SHA256 = "550995510c57455c7abc7af56b66ad1b64859aa8f4d12994dfbf8345178a144b"


def _bmp(path, w, h, bpp, rows, palette=None):
    """Bottom-up BITMAPINFOHEADER BMP; rows = list of h rows of raw pixel bytes (top row first)."""
    stride = (w * bpp // 8 + 3) // 4 * 4
    pal = b"" if palette is None else b"".join(bytes((b, g, r, 0)) for (b, g, r) in palette)
    off = 14 + 40 + len(pal)
    data = b"".join(bytes(r).ljust(stride, b"\0") for r in reversed(rows))
    hdr = b"BM" + struct.pack("<IHHI", off + len(data), 0, 0, off)
    info = struct.pack("<IiiHHIIiiII", 40, w, h, 1, bpp, 0, len(data), 2835, 2835,
                       0 if palette is None else len(palette), 0)
    with open(path, "wb") as fh:
        fh.write(hdr + info + pal + data)


# (B, G, R) -> hand-computed (1868 B + 9617 G + 4899 R + 8192) >> 14
KAT = [((255, 0, 0), 29), ((0, 255, 0), 150), ((0, 0, 255), 76), ((10, 20, 30), 22), ((200, 100, 50), 96),
       ((255, 255, 255), 255), ((1, 2, 3), 2), ((0, 0, 0), 0)]


def test_bmp24_fixed_point_gray(tmp_path):
    px = [bgr for bgr, _ in KAT]
    w = len(px)
    rows = [sum((list(p) for p in px), []), sum((list(p) for p in reversed(px)), [])]
    path = str(tmp_path / "k24.bmp")
    _bmp(path, w, 2, 24, rows)
    g = imread_gray(path)
    exp = [v for _, v in KAT]
    assert g.dtype == np.uint8 and g.shape == (2, w)
    assert g[0].tolist() == exp and g[1].tolist() == exp[::-1]


def test_bmp8_palette_through_formula(tmp_path):
    palette = [bgr for bgr, _ in KAT] + [(i, i, i) for i in range(8, 256)]
    idx = [[0, 1, 2, 3, 4, 5, 6, 7, 8, 200, 255]]
    path = str(tmp_path / "k8.bmp")
    _bmp(path, len(idx[0]), 1, 8, idx, palette)
    g = imread_gray(path)
    assert g[0].tolist() == [v for _, v in KAT] + [8, 200, 255]


@pytest.mark.parametrize("name", ["Src3.bmp", "Dst3.bmp", "Src4.bmp", "Dst4.bmp", "Src9.bmp", "Dst9.bmp",
                                  "Dst6.bmp"])
def test_reference_bmps_are_identity_gray(name):
    """The shipped 8-bit BMPs carry the identity gray palette: their gray image is the raw index plane."""
    with open(os.path.join(GOLDEN, "ref", name), "rb") as fh:
        b = fh.read()
    off = struct.unpack("<I", b[10:14])[0]
    w, h = struct.unpack("<ii", b[18:26])
    assert struct.unpack("<H", b[28:30])[0] == 8
    pal = np.frombuffer(b[54:54 + 1024], np.uint8).reshape(256, 4)[:, :3]
    assert (pal == np.arange(256)[:, None]).all()
    stride = (w + 3) // 4 * 4
    raw = np.frombuffer(b[off:off + stride * abs(h)], np.uint8).reshape(abs(h), stride)[:, :w]
    raw = raw[::-1] if h > 0 else raw
    assert np.array_equal(imread_gray(os.path.join(GOLDEN, "ref", name)), raw)


def test_src6_jpeg_decode_pinned():
    import PIL.features

    assert PIL.features.check_feature("libjpeg_turbo")
    g = imread_gray(os.path.join(GOLDEN, "Src6.jpg"))
    assert g.shape == (3000, 4096) and g.dtype == np.uint8
    assert hashlib.sha256(g.tobytes()).hexdigest() == SRC6_SHA256
