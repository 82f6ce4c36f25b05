// TEST-ONLY stand-in for the few OpenCV core types the GPU adapters touch (adapter/*.cc), so that
// adapter/ORBextractor_gpu.cc and adapter/Frame_gpu.cc compile and run here, where OpenCV is absent
// (tests/cpp/adapter_e2e.cpp). It is not OpenCV: a cv::Mat that owns or views a 2-D buffer, the
// cv::KeyPoint record in OpenCV's field order (28 bytes, which the adapters reinterpret as
// orbfe_keypoint), and the InputArray / OutputArray proxies over a Mat. Nothing in the product
// includes it.
#ifndef ORBFE_TEST_CVSTUB_CORE_HPP
#define ORBFE_TEST_CVSTUB_CORE_HPP

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>

#define CV_8U 0
#define CV_32F 5
#define CV_8UC1 CV_8U
#define CV_32FC1 CV_32F

namespace cv {

typedef unsigned char uchar;

struct Point2f {
  float x = 0.f, y = 0.f;
  Point2f() = default;
  Point2f(float x_, float y_) : x(x_), y(y_) {}
};

// cv::KeyPoint: pt, size, angle, response, octave, class_id
struct KeyPoint {
  Point2f pt;
  float size = 0.f, angle = -1.f, response = 0.f;
  int octave = 0, class_id = -1;
  KeyPoint() = default;
  KeyPoint(float x, float y, float size_, float angle_ = -1.f, float response_ = 0.f, int octave_ = 0,
           int class_id_ = -1)
      : pt(x, y), size(size_), angle(angle_), response(response_), octave(octave_), class_id(class_id_) {}
};
static_assert(sizeof(KeyPoint) == 28, "cv::KeyPoint is 28 bytes");

inline size_t elem_size(int type) {
  if (type == CV_8U) return 1;
  if (type == CV_32F) return 4;
  throw std::invalid_argument("cvstub: only CV_8UC1 and CV_32FC1");
}

class Mat {
 public:
  int rows = 0, cols = 0;
  uchar* data = nullptr;
  size_t step = 0;

  Mat() = default;
  Mat(int r, int c, int type) { create(r, c, type); }
  // a header over caller memory (no ownership), as cv::Mat(rows, cols, type, data, step)
  Mat(int r, int c, int type, void* p, size_t step_) : rows(r), cols(c), data((uchar*)p), step(step_), type_(type) {}

  void create(int r, int c, int type) {
    if (owned_ && rows == r && cols == c && type_ == type) return;
    type_ = type;
    rows = r;
    cols = c;
    step = (size_t)c * elem_size(type);
    owned_.reset(new uchar[(size_t)r * step + 1], std::default_delete<uchar[]>());
    data = owned_.get();
  }
  void release() {
    owned_.reset();
    data = nullptr;
    rows = cols = 0;
    step = 0;
  }
  bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
  int type() const { return type_; }
  Mat clone() const {
    Mat m(rows, cols, type_);
    for (int y = 0; y < rows; y++) std::memcpy(m.data + y * m.step, data + y * step, (size_t)cols * elem_size(type_));
    return m;
  }
  template <typename T>
  T* ptr(int row = 0) {
    return reinterpret_cast<T*>(data + (size_t)row * step);
  }
  template <typename T>
  const T* ptr(int row = 0) const {
    return reinterpret_cast<const T*>(data + (size_t)row * step);
  }
  template <typename T>
  T& at(int r, int c) {
    return ptr<T>(r)[c];
  }
  template <typename T>
  const T& at(int r, int c) const {
    return ptr<T>(r)[c];
  }
  // element i of a continuous single-row or single-column matrix
  template <typename T>
  T& at(int i) {
    return reinterpret_cast<T*>(data)[i];
  }
  template <typename T>
  const T& at(int i) const {
    return reinterpret_cast<const T*>(data)[i];
  }
  bool isContinuous() const { return rows <= 1 || step == (size_t)cols * elem_size(type_); }
  static Mat zeros(int r, int c, int type) {
    Mat m(r, c, type);
    std::memset(m.data, 0, (size_t)r * m.step);
    return m;
  }
  static Mat eye(int r, int c, int type) {
    Mat m = zeros(r, c, type);
    for (int i = 0; i < r && i < c; i++) m.at<float>(i, i) = 1.f;
    return m;
  }

 private:
  int type_ = CV_8U;
  std::shared_ptr<uchar> owned_;
};

class _InputArray {
 public:
  _InputArray(const Mat& m) : m_(&m) {}  // NOLINT: implicit, as OpenCV's proxy
  Mat getMat() const { return *m_; }
  bool empty() const { return m_->empty(); }

 private:
  const Mat* m_;
};
typedef const _InputArray& InputArray;

class _OutputArray {
 public:
  _OutputArray(Mat& m) : m_(&m) {}  // NOLINT: implicit, as OpenCV's proxy
  void create(int r, int c, int type) const { m_->create(r, c, type); }
  void release() const { m_->release(); }
  Mat getMat() const { return *m_; }

 private:
  Mat* m_;
};
typedef const _OutputArray& OutputArray;

// CV_32F matrix product and sum (the adapter's epipole, ORBmatcher.cc:678-681): each product
// element accumulated in double and rounded once, as OpenCV's small-matrix gemm does
inline Mat operator*(const Mat& a, const Mat& b) {
  if (a.type() != CV_32F || b.type() != CV_32F || a.cols != b.rows) throw std::invalid_argument("cvstub: gemm");
  Mat c(a.rows, b.cols, CV_32F);
  for (int i = 0; i < a.rows; i++)
    for (int j = 0; j < b.cols; j++) {
      double s = 0.0;
      for (int k = 0; k < a.cols; k++) s += (double)a.at<float>(i, k) * (double)b.at<float>(k, j);
      c.at<float>(i, j) = (float)s;
    }
  return c;
}
inline Mat operator+(const Mat& a, const Mat& b) {
  if (a.type() != CV_32F || b.type() != CV_32F || a.rows != b.rows || a.cols != b.cols)
    throw std::invalid_argument("cvstub: add");
  Mat c(a.rows, a.cols, CV_32F);
  for (int i = 0; i < a.rows; i++)
    for (int j = 0; j < a.cols; j++) c.at<float>(i, j) = a.at<float>(i, j) + b.at<float>(i, j);
  return c;
}

}  // namespace cv

#endif
