// TEST FIXTURE (tests/dropin): the parts of the reference's public data types (include/DataStructures.h:16-115)
// that the drop-in TemplateMatcher_fpm.cpp and its test driver use, same names and field order.  On the UI host the
// reference's own header is used instead.
#pragma once
#include <vector>

#include "opencv2/opencv.hpp"

struct s_TemplData {
    std::vector<cv::Mat> vecPyramid;
    bool bIsPatternLearned = false;
    cv::Rect userDefinedRect;
    bool hasUserRect = false;
    void clear() {
        std::vector<cv::Mat>().swap(vecPyramid);
        hasUserRect = false;
        userDefinedRect = cv::Rect();
    }
};

struct s_SingleTargetMatch {
    cv::Point2d ptLT, ptRT, ptRB, ptLB, ptCenter;
    double dMatchedAngle = 0;
    double dMatchScore = 0;
};
