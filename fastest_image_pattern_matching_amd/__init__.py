"""MI355X-native NCC template matcher: a drop-in for lrm2017/Fastest_Image_Pattern_Matching's TemplateMatcher.

The pixel path (pyramid, rotation, NCC correlation + normalisation, peak extraction, pyramid refinement) runs
in hand-written gfx950 HIP kernels inside ``lib/libfpm_hip.so``; this package is the Python mirror of the
reference's C++ ``TemplateMatcher`` API over that library's C ABI (include/fpm.h).
"""
from ._lib import LIB_PATH, build_library, load  # noqa: F401
from .matcher import SingleTargetMatch, TemplateMatcher  # noqa: F401

__all__ = ["TemplateMatcher", "SingleTargetMatch", "load", "build_library", "LIB_PATH"]
