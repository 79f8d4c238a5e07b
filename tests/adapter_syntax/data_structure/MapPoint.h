// include/data_structure/MapPoint.h:53-287 (the members the adapter touches).
#pragma once
#include <map>
#include "opencv2/core/core.hpp"
namespace ORB_SLAM2 {
class KeyFrame;
class MapPoint {
 public:
  void SetWorldPos(const cv::Mat &Pos);
  cv::Mat GetWorldPos();
  KeyFrame *GetReferenceKeyFrame();
  std::map<KeyFrame *, size_t> GetObservations();
  void EraseObservation(KeyFrame *pKF);
  bool IsInKeyFrame(KeyFrame *pKF);
  bool isBad();
  void UpdateNormalAndDepth();
  long unsigned int mnId;
  long unsigned int mnBALocalForKF;
  long unsigned int mnCorrectedByKF;
  long unsigned int mnCorrectedReference;
  cv::Mat mPosGBA;
  long unsigned int mnBAGlobalForKF;
};
}  // namespace ORB_SLAM2
