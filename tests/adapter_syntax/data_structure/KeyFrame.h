// include/data_structure/KeyFrame.h:64-442 (the members the adapter touches).
#pragma once
#include <set>
#include <vector>
#include "opencv2/core/core.hpp"
#include "point_types.h"
namespace ORB_SLAM2 {
class MapPoint;
class KeyFrame {
 public:
  void SetPose(const cv::Mat &Tcw);
  cv::Mat GetPose();
  cv::Mat GetRotation();
  cv::Mat GetTranslation();
  std::vector<KeyFrame *> GetVectorCovisibleKeyFrames();
  std::vector<KeyFrame *> GetCovisiblesByWeight(const int &w);
  int GetWeight(KeyFrame *pKF);
  KeyFrame *GetParent();
  bool hasChild(KeyFrame *pKF);
  std::set<KeyFrame *> GetLoopEdges();
  void EraseMapPointMatch(MapPoint *pMP);
  std::vector<MapPoint *> GetMapPointMatches();
  bool isBad();
  long unsigned int mnId;
  long unsigned int mnBALocalForKF;
  long unsigned int mnBAFixedForKF;
  cv::Mat mTcwGBA;
  long unsigned int mnBAGlobalForKF;
  const float fx, fy, cx, cy, invfx, invfy, mbf, mb, mThDepth;
  const std::vector<cv::KeyPoint> mvKeysUn;
  const std::vector<float> mvuRight;
  const std::vector<float> mvInvLevelSigma2;
  PointIRTCloud surface_points_less_flat_;
  PointIRTCloud surface_points_less_flat_normal_;
};
}  // namespace ORB_SLAM2
