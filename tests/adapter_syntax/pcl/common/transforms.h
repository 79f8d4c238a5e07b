#pragma once
#include "../point_cloud.h"
#include "Eigen/Geometry"
namespace pcl {
template <typename PointT>
void transformPointCloud(const PointCloud<PointT> &in, PointCloud<PointT> &out, const Eigen::Affine3d &transform);
}
