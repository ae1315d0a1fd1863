// TEST FIXTURE (tests/dropin): the reference's TemplateMatcher interface (include/TemplateMatcher.h:9-90) as the
// drop-in translation unit sees it — every public member function with the reference's signature, and the data
// members the inline setters/getters use.  tests/test_dropin.py checks on CPU that every public declaration of the
// reference header is here and defined by the drop-in.  On the UI host the reference's own header is used.
#pragma once
#include <vector>

#include "DataStructures.h"

class TemplateMatcher {
public:
    TemplateMatcher();
    ~TemplateMatcher();

    bool learnPattern(const cv::Mat& templateImage);
    std::vector<s_SingleTargetMatch> match(const cv::Mat& sourceImage);

    void setMaxPositions(int maxPos) { m_iMaxPos = maxPos; }
    void setMaxOverlap(double maxOverlap) { m_dMaxOverlap = maxOverlap; }
    void setScore(double score) { m_dScore = score; }
    void setToleranceAngle(double angle) { m_dToleranceAngle = angle; }
    void setMinReduceArea(int area) { m_iMinReduceArea = area; }
    void setUseSIMD(bool useSIMD) { m_bUseSIMD = useSIMD; }
    void setSubPixelEstimation(bool enable) { m_bSubPixelEstimation = enable; }

    int getMaxPositions() const { return m_iMaxPos; }
    double getMaxOverlap() const { return m_dMaxOverlap; }
    double getScore() const { return m_dScore; }
    double getToleranceAngle() const { return m_dToleranceAngle; }
    int getMinReduceArea() const { return m_iMinReduceArea; }
    bool getUseSIMD() const { return m_bUseSIMD; }
    bool getSubPixelEstimation() const { return m_bSubPixelEstimation; }

    double getLastExecutionTime() const { return m_dLastExecutionTime; }
    bool isPatternLearned() const { return m_TemplData.bIsPatternLearned; }
    void clearPattern();

    void setUserDefinedRect(const cv::Rect& rect);
    cv::Rect getUserDefinedRect() const;
    bool hasUserDefinedRect() const;

private:
    s_TemplData m_TemplData;
    int m_iMaxPos;
    double m_dMaxOverlap;
    double m_dScore;
    double m_dToleranceAngle;
    int m_iMinReduceArea;
    bool m_bUseSIMD;
    bool m_bSubPixelEstimation;
    double m_dLastExecutionTime;
    bool m_bToleranceRange;
    double m_dTolerance1, m_dTolerance2, m_dTolerance3, m_dTolerance4;
};
