// hipOptimizer.h — libsqrtlm behind the reference's Optimizer seam.
//
// Drop-in sibling of g2oOptimizer (src/backend/g2oOptimizer.cc) for the
// calls the MI355X backend implements: LocalBundleAdjustment,
// BundleAdjustment, GlobalBundleAdjustemnt and OptimizeEssentialGraph
// (include/backend/Optimizer.h:50-65).
// It is meant to be added to the reference tree as include/backend/hipOptimizer.h
// + src/backend/hipOptimizer.cc and selected in Optimizer.cc's dispatch
// (see INTEGRATION.md §4); it builds against the reference's own headers and
// links libsqrtlm.so. It is not compiled in this repository: the reference's
// dependencies (OpenCV, PCL, Eigen, ROS) are absent here.
//
// Capture: with SQLM_CAPTURE_DIR set, every call also writes its seam inputs
// (and, in capture mode, the g2o backend's write-back) as a sqrtlm_capture.h
// file, replayable on a GPU box with tools/sqlm_replay.
#ifndef HIP_OPTIMIZER_H
#define HIP_OPTIMIZER_H

#include <map>
#include <set>
#include <vector>

#include "Eigen/Core"
#include "LoopClosing.h"

// global, as in the reference (include/utils/lidarconfig.h:7 declares it
// outside namespace ORB_SLAM2; a forward declaration inside the namespace
// would name a different, incomplete type)
struct lidarConfig;

namespace ORB_SLAM2 {

class KeyFrame;
class MapPoint;
class Map;

class hipOptimizer {
 public:
  // g2oOptimizer::LocalBundleAdjustment (g2oOptimizer.cc:704-1191) on the GPU.
  static void LocalBundleAdjustment(KeyFrame* pKF, bool* pbStopFlag, Map* pMap, const lidarConfig* cfg);
  // g2oOptimizer::BundleAdjustment (g2oOptimizer.cc:110-362) on the GPU.
  static void BundleAdjustment(const std::vector<KeyFrame*>& vpKFs, const std::vector<MapPoint*>& vpMP,
                               int nIterations, bool* pbStopFlag, unsigned long nLoopKF, bool bRobust);
  // g2oOptimizer::GlobalBundleAdjustemnt (g2oOptimizer.cc:80-95): every KF and MP of the map.
  static void GlobalBundleAdjustemnt(Map* pMap, int nIterations, bool* pbStopFlag, unsigned long nLoopKF,
                                     bool bRobust);
  // g2oOptimizer::OptimizeEssentialGraph (g2oOptimizer.cc:1212-1534) on the GPU
  // (sqlm_eg_*): same vertices, edges, insertion order and write-back.
  static void OptimizeEssentialGraph(Map* pMap, KeyFrame* pLoopKF, KeyFrame* pCurKF,
                                     const LoopClosing::KeyFrameAndPose& NonCorrectedSim3,
                                     const LoopClosing::KeyFrameAndPose& CorrectedSim3,
                                     const std::map<KeyFrame*, std::set<KeyFrame*> >& LoopConnections,
                                     const bool& bFixScale);

  // Capture mode around the g2o backend (Optimizer.cc dispatch): Begin*
  // records the seam inputs, End* the g2o write-back, then the file is written.
  static void BeginCaptureLBA(KeyFrame* pKF);
  static void EndCaptureLBA();
  static void BeginCaptureBA(const std::vector<KeyFrame*>& vpKFs, const std::vector<MapPoint*>& vpMP,
                             int nIterations, bool bRobust);
  static void EndCaptureBA(unsigned long nLoopKF);
  // One-line hook for g2oOptimizer.cc:1062-1070 in capture mode: the LiDAR
  // flat pair the reference's kd-tree found for pass 3.
  static void CaptureLidarFlat(const Eigen::Vector3d& p_cam, const Eigen::Vector3d& p_world,
                               const Eigen::Vector3d& normal, double weight);
  static bool CaptureEnabled();
};

}  // namespace ORB_SLAM2

#endif
