// PCL 1.x pcl::PointXYZI / pcl::PointCloud subset (common/include/pcl/point_cloud.h).
#pragma once
#include <cstddef>
#include <memory>
#include <vector>
namespace pcl {
struct PointXYZI {
  float x, y, z, intensity;
};
template <typename PointT>
class PointCloud {
 public:
  typedef std::shared_ptr<PointCloud<PointT>> Ptr;
  typedef std::shared_ptr<const PointCloud<PointT>> ConstPtr;
  std::vector<PointT> points;
  Ptr makeShared() const;
  void push_back(const PointT &);
  bool empty() const;
  size_t size() const;
  PointT &operator[](size_t);
  const PointT &operator[](size_t) const;
  typename std::vector<PointT>::iterator begin();
  typename std::vector<PointT>::iterator end();
  typename std::vector<PointT>::const_iterator begin() const;
  typename std::vector<PointT>::const_iterator end() const;
  PointCloud &operator+=(const PointCloud &);
};
}  // namespace pcl
