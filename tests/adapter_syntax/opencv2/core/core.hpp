// OpenCV 3.3 cv::Mat / cv::KeyPoint subset (modules/core/include/opencv2/core/mat.hpp, types.hpp).
#pragma once
#define CV_32F 5
namespace cv {
class Mat {
 public:
  Mat();
  Mat(int rows, int cols, int type);
  Mat(int rows, int cols, int type, void *data, unsigned long step = 0);
  template <typename T> T &at(int i0);
  template <typename T> const T &at(int i0) const;
  template <typename T> T &at(int row, int col);
  template <typename T> const T &at(int row, int col) const;
  Mat inv(int method = 0) const;
  Mat clone() const;
  void create(int rows, int cols, int type);
  void copyTo(Mat &m) const;
  bool empty() const;
};
struct Point2f {
  float x, y;
};
struct Point3f {
  float x, y, z;
};
class KeyPoint {
 public:
  Point2f pt;
  float size, angle, response;
  int octave, class_id;
};
}  // namespace cv
