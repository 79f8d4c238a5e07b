// include/data_structure/Map.h:38-144 (the members the adapter touches).
#pragma once
#include <mutex>
#include <vector>
#include "KeyFrame.h"
#include "MapPoint.h"
namespace ORB_SLAM2 {
class Map {
 public:
  std::vector<KeyFrame *> GetAllKeyFrames();
  std::vector<MapPoint *> GetAllMapPoints();
  long unsigned int GetMaxKFid();
  std::mutex mMutexMapUpdate;
};
}  // namespace ORB_SLAM2
