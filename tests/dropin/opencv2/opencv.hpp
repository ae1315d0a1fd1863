// TEST FIXTURE (tests/dropin): the OpenCV core types the drop-in TemplateMatcher_fpm.cpp and the reference's own
// headers (include/DataStructures.h, TemplateMatcher.h, SIMDOptimization.h) name, so the drop-in translation unit
// compiles -- against this directory's header excerpts on the GPU box, and against the unmodified reference headers
// in tests/test_dropin_real_headers.py -- where no OpenCV exists.  Not OpenCV: the member functions are the ones
// those files use, with OpenCV's meaning; the DATA LAYOUT of every type a reference struct holds by value is OpenCV
// 4.x's on x86-64 (cv::Mat's 12 members, 96 bytes; Rect_ / Point_ / Size_ / Scalar_ / RotatedRect as in
// core/types.hpp), so sizeof(TemplateMatcher) compiled here equals the reference build's.
#pragma once
#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <memory>
#include <vector>

#define CV_8U 0
#define CV_8UC1 0
#define CV_8UC3 16
#define CV_32FC1 5
#define CV_PI 3.1415926535897932384626433832795
#define CV_MAT_TYPE_MASK 0xFFF

namespace cv {

typedef unsigned char uchar;

template <typename T>
struct Point_ {
    T x = 0, y = 0;
    Point_() {}
    Point_(T a, T b) : x(a), y(b) {}
    template <typename U>
    Point_(const Point_<U>& o) : x((T)o.x), y((T)o.y) {}
};
typedef Point_<int> Point;
typedef Point_<float> Point2f;
typedef Point_<double> Point2d;

template <typename T>
struct Size_ {
    T width = 0, height = 0;
    Size_() {}
    Size_(T w, T h) : width(w), height(h) {}
};
typedef Size_<int> Size;
typedef Size_<float> Size2f;

template <typename T>
struct Rect_ {
    T x = 0, y = 0, width = 0, height = 0;
    Rect_() {}
    Rect_(T a, T b, T c, T d) : x(a), y(b), width(c), height(d) {}
    T area() const { return width * height; }
    bool operator==(const Rect_& o) const { return x == o.x && y == o.y && width == o.width && height == o.height; }
};
typedef Rect_<int> Rect;
// cv::Rect::operator& (intersection; empty -> all zero)
inline Rect operator&(const Rect& a, const Rect& b) {
    const int x1 = std::max(a.x, b.x), y1 = std::max(a.y, b.y);
    const int w = std::min(a.x + a.width, b.x + b.width) - x1, h = std::min(a.y + a.height, b.y + b.height) - y1;
    return (w <= 0 || h <= 0) ? Rect() : Rect(x1, y1, w, h);
}

template <typename T>
struct Scalar_ {
    T val[4] = {0, 0, 0, 0};
};
typedef Scalar_<double> Scalar;

struct RotatedRect {
    Point2f center;
    Size2f size;
    float angle = 0;
};

enum TemplateMatchModes { TM_SQDIFF = 0, TM_SQDIFF_NORMED = 1, TM_CCORR = 2, TM_CCORR_NORMED = 3, TM_CCOEFF = 4,
                          TM_CCOEFF_NORMED = 5 };

struct MatAllocator;
struct UMatData;
struct MatSize {
    int* p = nullptr;
};
struct MatStep {
    size_t* p = buf;
    size_t buf[2] = {0, 1};
    MatStep() {}
    MatStep(const MatStep& o) : p(buf) { buf[0] = o.buf[0]; buf[1] = o.buf[1]; }
    MatStep& operator=(const MatStep& o) { buf[0] = o.buf[0]; buf[1] = o.buf[1]; p = buf; return *this; }
    size_t operator[](int i) const { return buf[i]; }
    size_t& operator[](int i) { return buf[i]; }
};

// cv::Mat with OpenCV 4.x's members (flags, dims, rows, cols, data, datastart, dataend, datalimit, allocator, u,
// size, step: 96 bytes); the pixels of an owning Mat live in a shared buffer kept by a small side object.
class Mat {
public:
    int flags = 0x42FF0000;   // MAGIC_VAL | CV_8UC1
    int dims = 0;
    int rows = 0, cols = 0;
    uchar* data = nullptr;
    const uchar* datastart = nullptr;
    const uchar* dataend = nullptr;
    const uchar* datalimit = nullptr;
    MatAllocator* allocator = nullptr;
    UMatData* u = nullptr;
    MatSize size;
    MatStep step;

    Mat() {}
    // rows x cols 8-bit image (channels 1 or 3) owning zeroed pixels
    Mat(int r, int c, int type_) : flags(0x42FF0000 | type_), dims(2), rows(r), cols(c) {
        const int ch = type_ == CV_8UC3 ? 3 : 1;
        step[0] = (size_t)c * ch;
        step[1] = (size_t)ch;
        auto* h = new std::shared_ptr<std::vector<uchar>>(std::make_shared<std::vector<uchar>>((size_t)r * step[0]));
        data = (*h)->data();
        datastart = data;
        dataend = datalimit = data + (*h)->size();
        u = reinterpret_cast<UMatData*>(h);   // the pixel owner rides in the UMatData* slot: OpenCV's layout kept
    }
    Mat(const Mat& o) { copy_from(o); }
    Mat& operator=(const Mat& o) {
        if (this != &o) { release(); copy_from(o); }
        return *this;
    }
    ~Mat() { release(); }
    // a view of a rectangle (shares the pixels)
    Mat operator()(const Rect& r) const {
        Mat m(*this);
        m.rows = r.height;
        m.cols = r.width;
        m.data = data + (size_t)r.y * step[0] + (size_t)r.x * step[1];
        return m;
    }
    bool empty() const { return data == nullptr || rows <= 0 || cols <= 0; }
    int type() const { return flags & CV_MAT_TYPE_MASK; }

private:
    std::shared_ptr<std::vector<uchar>> owner_handle() const {
        return u ? *reinterpret_cast<std::shared_ptr<std::vector<uchar>>*>(u) : nullptr;
    }
    void copy_from(const Mat& o) {
        flags = o.flags; dims = o.dims; rows = o.rows; cols = o.cols; data = o.data;
        datastart = o.datastart; dataend = o.dataend; datalimit = o.datalimit; step = o.step;
        u = o.u ? reinterpret_cast<UMatData*>(new std::shared_ptr<std::vector<uchar>>(o.owner_handle())) : nullptr;
    }
    void release() {
        delete reinterpret_cast<std::shared_ptr<std::vector<uchar>>*>(u);
        u = nullptr;
    }
};

// declared for the reference's inline s_BlockMax (DataStructures.h:150-246); not used by the drop-in
void minMaxLoc(const Mat& src, double* minVal, double* maxVal = nullptr, Point* minLoc = nullptr,
               Point* maxLoc = nullptr, const Mat& mask = Mat());

}  // namespace cv
