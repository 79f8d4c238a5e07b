// include/data_structure/point_types.h:16-54 (types only).
#pragma once
#include <cstdint>
#include "pcl/point_cloud.h"
struct PointXYZIRT {
  float x, y, z;
  uint8_t intensity;
  uint16_t ring;
  double timestamp;
};
typedef pcl::PointXYZI PointI;
typedef pcl::PointCloud<PointI> PointICloud;
typedef pcl::PointCloud<PointI>::Ptr PointICloudPtr;
typedef PointXYZIRT PointIRT;
typedef pcl::PointCloud<PointIRT> PointIRTCloud;
typedef pcl::PointCloud<PointIRT>::Ptr PointIRTCloudPtr;
