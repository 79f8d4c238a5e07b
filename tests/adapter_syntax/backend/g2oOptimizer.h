// include/backend/g2oOptimizer.h:52-162 (the entry points the dispatch and the adapter call).
#pragma once
#include <map>
#include <set>
#include <vector>
#include "KeyFrame.h"
#include "LoopClosing.h"
#include "Map.h"
#include "lidarconfig.h"
namespace ORB_SLAM2 {
class g2oOptimizer {
 public:
  void static BundleAdjustment(const std::vector<KeyFrame *> &vpKF, const std::vector<MapPoint *> &vpMP,
                               int nIterations = 5, bool *pbStopFlag = NULL, const unsigned long nLoopKF = 0,
                               const bool bRobust = true);
  void static GlobalBundleAdjustemnt(Map *pMap, int nIterations = 5, bool *pbStopFlag = NULL,
                                     const unsigned long nLoopKF = 0, const bool bRobust = true);
  void static LocalBundleAdjustment(KeyFrame *pKF, bool *pbStopFlag, Map *pMap, const lidarConfig *lidarconfig);
  void static OptimizeEssentialGraph(Map *pMap, KeyFrame *pLoopKF, KeyFrame *pCurKF,
                                     const LoopClosing::KeyFrameAndPose &NonCorrectedSim3,
                                     const LoopClosing::KeyFrameAndPose &CorrectedSim3,
                                     const std::map<KeyFrame *, std::set<KeyFrame *> > &LoopConnections,
                                     const bool &bFixScale);
};
}  // namespace ORB_SLAM2
