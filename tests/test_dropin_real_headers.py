"""The drop-in (fastest_image_pattern_matching_amd/dropin/TemplateMatcher_fpm.cpp) compiled and linked against the
reference's UNMODIFIED headers (include/TemplateMatcher.h, DataStructures.h, SIMDOptimization.h) -- CPU only.

The reference headers need OpenCV and Qt: Qt's headers are in this container (/opt/conda/include/qt; DataStructures.h
includes QString / QPointF / QRectF, DataStructures.h:5-7), OpenCV is not, so tests/dropin/opencv2/opencv.hpp stands
in for it with OpenCV 4.x's data layouts.  The test links a driver against libfpm_hip.so (no GPU call is made) and
checks that the class the drop-in defines has the reference build's layout: sizeof(TemplateMatcher) as OpenCV 4.x on
x86-64 gives it (include/TemplateMatcher.h:53-77: s_TemplData, cv::Mat m_sourceImage, the parameters).  Skipped
where the reference or Qt is absent (the GPU box keeps the header-excerpt build of tests/dropin/Makefile).
"""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_INC = "/root/reference/include"
QT = "/opt/conda/include/qt"

# OpenCV 4.x, x86-64: sizeof(cv::Mat) 96, cv::Rect 16, cv::Scalar 32, cv::RotatedRect 20, cv::Point2d 16
# s_TemplData: 5 vectors (4 x 24 + vector<bool> 40) + bool/int 8 + Rect 16 + bool (padded to 8) = 168
# TemplateMatcher: s_TemplData 168 + Mat 96 + int (8) + 3 double 24 + int/bool/bool (8) + double 8 + bool (8)
#                  + 4 double 32 = 352
EXPECTED = {"cv::Mat": 96, "cv::Rect": 16, "cv::Scalar": 32, "cv::RotatedRect": 20, "cv::Point2d": 16,
            "s_TemplData": 168, "s_SingleTargetMatch": 96, "TemplateMatcher": 352}

DRIVER = r"""
#include "TemplateMatcher.h"
#include <cstdio>
int main() {
    // the class as the reference header declares it, defined by the drop-in; nothing is constructed (no GPU here)
    bool (TemplateMatcher::*learn)(const cv::Mat&) = &TemplateMatcher::learnPattern;
    std::vector<s_SingleTargetMatch> (TemplateMatcher::*match)(const cv::Mat&) = &TemplateMatcher::match;
    void (TemplateMatcher::*rect)(const cv::Rect&) = &TemplateMatcher::setUserDefinedRect;
    (void)learn; (void)match; (void)rect;
    std::printf("cv::Mat %zu\ncv::Rect %zu\ncv::Scalar %zu\ncv::RotatedRect %zu\ncv::Point2d %zu\n", sizeof(cv::Mat),
                sizeof(cv::Rect), sizeof(cv::Scalar), sizeof(cv::RotatedRect), sizeof(cv::Point2d));
    std::printf("s_TemplData %zu\ns_SingleTargetMatch %zu\nTemplateMatcher %zu\n", sizeof(s_TemplData),
                sizeof(s_SingleTargetMatch), sizeof(TemplateMatcher));
    return 0;
}
"""


@pytest.mark.skipif(not (os.path.isdir(REF_INC) and os.path.isdir(QT) and shutil.which("g++")),
                    reason="reference headers or Qt headers absent (GPU box)")
def test_dropin_compiles_against_reference_headers(tmp_path):
    lib = os.path.join(REPO, "fastest_image_pattern_matching_amd", "lib")
    if not os.path.exists(os.path.join(lib, "libfpm_hip.so")):
        pytest.skip("libfpm_hip.so not built")
    drv = tmp_path / "driver.cpp"
    drv.write_text(DRIVER)
    exe = tmp_path / "driver"
    # the reference include directory first: TemplateMatcher.h / DataStructures.h / SIMDOptimization.h come from the
    # reference, only <opencv2/opencv.hpp> from the stand-in directory
    # QT_NO_VERSION_TAGGING: the Qt headers would otherwise reference libQt5Core's qt_version_tag; nothing of Qt is
    # called (the UI links Qt itself), and this container's Qt libraries need conda's older libstdc++
    cmd = ["g++", "-std=c++17", "-O1", "-Wall", "-fPIC", "-DQT_NO_VERSION_TAGGING", "-I" + REF_INC, "-I" + os.path.join(REPO, "tests", "dropin"),
           "-I" + os.path.join(REPO, "include"), "-I" + QT, "-I" + os.path.join(QT, "QtCore"),
           os.path.join(REPO, "fastest_image_pattern_matching_amd", "dropin", "TemplateMatcher_fpm.cpp"), str(drv),
           "-L" + lib, "-lfpm_hip", "-Wl,-rpath," + lib, "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    # the headers really were the reference's: the translation unit's dependency list names them
    dep = subprocess.run(cmd[:11] + ["-M", os.path.join(REPO, "fastest_image_pattern_matching_amd", "dropin",
                                                         "TemplateMatcher_fpm.cpp")],
                         capture_output=True, text=True, check=True).stdout
    for h in ("TemplateMatcher.h", "DataStructures.h", "SIMDOptimization.h"):
        assert os.path.join(REF_INC, h) in dep, h
    assert os.path.join(REPO, "tests", "dropin", "TemplateMatcher.h") not in dep
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout
    sizes = {k: int(v) for k, v in (line.rsplit(" ", 1) for line in out.strip().splitlines())}
    assert sizes == EXPECTED
