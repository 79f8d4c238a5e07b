#pragma once
#include <vector>
#include "../point_cloud.h"
namespace pcl {
template <typename PointT>
class KdTreeFLANN {
 public:
  void setInputCloud(const typename PointCloud<PointT>::ConstPtr &cloud);
  int nearestKSearch(const PointT &point, int k, std::vector<int> &k_indices, std::vector<float> &k_sqr_distances) const;
};
}  // namespace pcl
