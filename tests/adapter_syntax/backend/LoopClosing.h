// include/backend/LoopClosing.h:58-65 (the KeyFrameAndPose map type).
#pragma once
#include <map>
#include "KeyFrame.h"
#include "Map.h"
#include "Thirdparty/g2o/g2o/types/sim3.h"
namespace ORB_SLAM2 {
class LoopClosing {
 public:
  typedef std::map<KeyFrame *, g2o::Sim3, std::less<KeyFrame *>,
                   Eigen::aligned_allocator<std::pair<KeyFrame *const, g2o::Sim3>>>
      KeyFrameAndPose;
};
}  // namespace ORB_SLAM2
