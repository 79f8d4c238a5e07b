// Optimizer_hip_dispatch.cc — the reference's Optimizer dispatch
// (src/backend/Optimizer.cc:29-100) with the libsqrtlm backend selected by
// `solver == Optimizer::HIP` (eSolver gains HIP = 3 in
// include/backend/Optimizer.h). A maintainer merges these four bodies into
// Optimizer.cc; the Ceres / MyOptimizer branches and the timing prints of the
// original stay as they are (elided here). Outside HIP mode the g2o calls are
// bracketed by the capture hooks (no-ops unless SQLM_CAPTURE_DIR is set).
// Syntax-checked against declaration-only reference headers by
// tests/test_adapter_syntax.py.
#include "backend/Optimizer.h"
#include "backend/g2oOptimizer.h"
#include "backend/hipOptimizer.h"

namespace ORB_SLAM2 {

Optimizer::eSolver solver = Optimizer::HIP;  // Optimizer.cc:26 (G2O in the reference)

void Optimizer::GlobalBundleAdjustemnt(Map* pMap, int nIterations, bool* pbStopFlag, const unsigned long nLoopKF,
                                       const bool bRobust) {
  if (solver == Optimizer::HIP) {
    hipOptimizer::GlobalBundleAdjustemnt(pMap, nIterations, pbStopFlag, nLoopKF, bRobust);
    return;
  }
  const std::vector<KeyFrame*> kfs = pMap->GetAllKeyFrames();
  const std::vector<MapPoint*> mps = pMap->GetAllMapPoints();
  hipOptimizer::BeginCaptureBA(kfs, mps, nIterations, bRobust);
  g2oOptimizer::GlobalBundleAdjustemnt(pMap, nIterations, pbStopFlag, nLoopKF, bRobust);
  hipOptimizer::EndCaptureBA(nLoopKF);
}

void Optimizer::BundleAdjustment(const std::vector<KeyFrame*>& vpKFs, const std::vector<MapPoint*>& vpMP,
                                 int nIterations, bool* pbStopFlag, const unsigned long nLoopKF, const bool bRobust) {
  if (solver == Optimizer::HIP) {
    hipOptimizer::BundleAdjustment(vpKFs, vpMP, nIterations, pbStopFlag, nLoopKF, bRobust);
    return;
  }
  hipOptimizer::BeginCaptureBA(vpKFs, vpMP, nIterations, bRobust);
  g2oOptimizer::BundleAdjustment(vpKFs, vpMP, nIterations, pbStopFlag, nLoopKF, bRobust);
  hipOptimizer::EndCaptureBA(nLoopKF);
}

void Optimizer::LocalBundleAdjustment(KeyFrame* pKF, bool* pbStopFlag, Map* pMap, const lidarConfig* lidarconfig) {
  if (solver == Optimizer::HIP) {
    hipOptimizer::LocalBundleAdjustment(pKF, pbStopFlag, pMap, lidarconfig);
    return;
  }
  hipOptimizer::BeginCaptureLBA(pKF);
  g2oOptimizer::LocalBundleAdjustment(pKF, pbStopFlag, pMap, lidarconfig);
  hipOptimizer::EndCaptureLBA();
}

void Optimizer::OptimizeEssentialGraph(Map* pMap, KeyFrame* pLoopKF, KeyFrame* pCurKF,
                                       const LoopClosing::KeyFrameAndPose& NonCorrectedSim3,
                                       const LoopClosing::KeyFrameAndPose& CorrectedSim3,
                                       const std::map<KeyFrame*, std::set<KeyFrame*> >& LoopConnections,
                                       const bool& bFixScale) {
  if (solver == Optimizer::HIP) {
    hipOptimizer::OptimizeEssentialGraph(pMap, pLoopKF, pCurKF, NonCorrectedSim3, CorrectedSim3, LoopConnections,
                                         bFixScale);
    return;
  }
  g2oOptimizer::OptimizeEssentialGraph(pMap, pLoopKF, pCurKF, NonCorrectedSim3, CorrectedSim3, LoopConnections,
                                       bFixScale);
}

}  // namespace ORB_SLAM2
