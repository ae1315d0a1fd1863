// TEST FIXTURE (tests/dropin): the handful of OpenCV core types the drop-in TemplateMatcher_fpm.cpp touches —
// cv::Mat (8-bit, refcounted pixels), cv::Point2d, cv::Rect — so the drop-in translation unit compiles and runs on
// the GPU box, which has no OpenCV.  Not OpenCV: only the members the drop-in uses, with OpenCV's meaning.
#pragma once
#include <cstddef>
#include <cstdint>
#include <memory>
#include <vector>

#define CV_8UC1 0
#define CV_8UC3 16

namespace cv {

struct Point2d {
    double x = 0, y = 0;
    Point2d() {}
    Point2d(double a, double b) : x(a), y(b) {}
};

struct Rect {
    int x = 0, y = 0, width = 0, height = 0;
    Rect() {}
    Rect(int a, int b, int c, int d) : x(a), y(b), width(c), height(d) {}
    bool operator==(const Rect& o) const { return x == o.x && y == o.y && width == o.width && height == o.height; }
};

class Mat {
public:
    int rows = 0, cols = 0;
    unsigned char* data = nullptr;
    size_t step[2] = {0, 1};
    Mat() {}
    // rows x cols 8-bit image (channels 1 or 3) owning zeroed pixels
    Mat(int r, int c, int type_) : rows(r), cols(c), type_(type_) {
        const int ch = type_ == CV_8UC3 ? 3 : 1;
        step[0] = (size_t)c * ch;
        step[1] = (size_t)ch;
        buf_ = std::make_shared<std::vector<unsigned char>>((size_t)r * step[0]);
        data = buf_->data();
    }
    bool empty() const { return data == nullptr || rows <= 0 || cols <= 0; }
    int type() const { return type_; }

private:
    int type_ = CV_8UC1;
    std::shared_ptr<std::vector<unsigned char>> buf_;
};

}  // namespace cv
