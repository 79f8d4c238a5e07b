// Thirdparty/g2o/g2o/types/sim3.h:52-290 (the value type's interface).
#pragma once
#include "Eigen/Geometry"
namespace g2o {
using Eigen::Matrix3d;
using Eigen::Quaterniond;
using Eigen::Vector3d;
struct Sim3 {
  Sim3();
  Sim3(const Quaterniond &r, const Vector3d &t, double s);
  Sim3(const Matrix3d &R, const Vector3d &t, double s);
  Vector3d map(const Vector3d &xyz) const;
  Sim3 inverse() const;
  Sim3 operator*(const Sim3 &other) const;
  const Vector3d &translation() const;
  const Quaterniond &rotation() const;
  const double &scale() const;
};
}  // namespace g2o
