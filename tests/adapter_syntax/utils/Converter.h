// include/utils/Converter.h:54-193 (the members the adapter calls).
#pragma once
#include "Eigen/Dense"
#include "opencv2/core/core.hpp"
namespace ORB_SLAM2 {
class Converter {
 public:
  static cv::Mat toCvMat(const Eigen::Matrix<double, 3, 1> &m);
  static cv::Mat toCvSE3(const Eigen::Matrix<double, 3, 3> &R, const Eigen::Matrix<double, 3, 1> &t);
  static Eigen::Matrix<double, 3, 1> toVector3d(const cv::Mat &cvVector);
  static Eigen::Matrix<double, 3, 3> toMatrix3d(const cv::Mat &cvMat3);
};
}  // namespace ORB_SLAM2
