// hipOptimizer.cc — libsqrtlm behind the reference's Optimizer seam (see
// hipOptimizer.h). Builds inside the reference tree only: it uses the
// reference's KeyFrame / MapPoint / Map / lidarConfig types, OpenCV and PCL.
//
// Every call flattens the map objects into the seam graph of
// include/sqrtlm_capture.h (float32, exactly what g2oOptimizer reads), runs
// it through libsqrtlm and writes back as g2oOptimizer does. Ordering rules
// that make the result equal g2o's: poses and points in
// ascending mnId (g2o vertex ids mnId / mnId + maxKFid + 1), edges in
// insertion order (point list order, then GetObservations() map order).
#include "backend/hipOptimizer.h"
#include "backend/g2oOptimizer.h"  // fallback for the configurations libsqrtlm does not cover

#include <pcl/common/transforms.h>
#include <pcl/kdtree/kdtree_flann.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <map>
#include <mutex>
#include <set>
#include <string>

#include "Converter.h"
#include "Thirdparty/g2o/g2o/types/sim3.h"  // value type only (the solve runs in libsqrtlm)
#include "KeyFrame.h"
#include "Map.h"
#include "MapPoint.h"
#include "sqrtlm.h"
#include "sqrtlm_capture.h"

namespace ORB_SLAM2 {

// Defined in src/backend/g2oOptimizer.cc:59-66 (namespace ORB_SLAM2, external
// linkage) and declared in no reference header.
PointI PointIRT2PointI(const PointIRT &Pirt);

namespace {

// ---------------------------------------------------------------- context

struct CtxHolder {
  sqlm_ctx* ctx = nullptr;
  ~CtxHolder() {
    if (ctx) sqlm_ctx_destroy(ctx);
  }
};

// One context per calling thread (LocalMapping, LoopClosing, the GBA thread).
sqlm_ctx* thread_ctx() {
  thread_local CtxHolder h;
  if (!h.ctx) {
    const char* dev = std::getenv("SQLM_DEVICE");
    const int s = sqlm_ctx_create(dev ? std::atoi(dev) : -1, &h.ctx);
    if (s != SQLM_OK) {
      std::cerr << "hipOptimizer: sqlm_ctx_create failed: " << sqlm_status_string(s) << std::endl;
      h.ctx = nullptr;
    }
  }
  return h.ctx;
}

bool report(int s, const char* what) {
  if (s == SQLM_OK) return true;
  std::cerr << "hipOptimizer: " << what << ": " << sqlm_status_string(s) << std::endl;
  return false;
}

const volatile uint8_t* stop_ptr(bool* p) { return reinterpret_cast<const volatile uint8_t*>(p); }
bool stopped(const bool* p) { return p && *p; }

// ---------------------------------------------------------------- seam graph

// The g2o graph of one call in its float32 input form; view() exposes it as a
// sqlm_capture (no copies) for sqlm_capture_replay / sqlm_capture_write.
struct SeamGraph {
  uint32_t kind = SQLM_CAP_LBA;
  int iterations = 0;
  bool robust = false;
  std::vector<KeyFrame*> kfs;   // pose index -> keyframe (ascending mnId)
  std::vector<MapPoint*> mps;   // point index -> map point (ascending mnId)
  std::map<KeyFrame*, int> kf_index;
  std::map<MapPoint*, int> mp_index;
  std::vector<float> Tcw, intr, bf, pt, uv, ur, isig2, delta;
  std::vector<uint8_t> fixed;
  std::vector<uint64_t> kf_id, mp_id;
  std::vector<int32_t> op, ol;
  std::vector<KeyFrame*> edge_kf;  // edge -> (keyframe, map point), for tags and erasure
  std::vector<MapPoint*> edge_mp;
  std::vector<int32_t> lid_pose;
  std::vector<double> lid_pc, lid_pw, lid_n, lid_info;
  // reference write-back (capture mode)
  std::vector<float> res_Tcw, res_pt;
  std::vector<uint8_t> res_outlier;

  void set_poses(std::vector<KeyFrame*> v, const std::vector<uint8_t>& fix_by_input) {
    std::vector<std::pair<KeyFrame*, uint8_t>> s;
    for (size_t i = 0; i < v.size(); ++i) s.emplace_back(v[i], fix_by_input[i]);
    std::sort(s.begin(), s.end(), [](const auto& a, const auto& b) { return a.first->mnId < b.first->mnId; });
    for (auto& [kf, f] : s) {
      kf_index[kf] = (int)kfs.size();
      kfs.push_back(kf);
      const cv::Mat T = kf->GetPose();  // CV_32F 4x4 (KeyFrame.cc:127-131)
      for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) Tcw.push_back(T.at<float>(r, c));
      intr.insert(intr.end(), {kf->fx, kf->fy, kf->cx, kf->cy});
      bf.push_back(kf->mbf);
      fixed.push_back(f);
      kf_id.push_back(kf->mnId);
    }
  }
  void set_points(std::vector<MapPoint*> v) {
    std::sort(v.begin(), v.end(), [](MapPoint* a, MapPoint* b) { return a->mnId < b->mnId; });
    for (MapPoint* mp : v) {
      mp_index[mp] = (int)mps.size();
      mps.push_back(mp);
      const cv::Mat X = mp->GetWorldPos();  // CV_32F 3x1
      pt.insert(pt.end(), {X.at<float>(0), X.at<float>(1), X.at<float>(2)});
      mp_id.push_back(mp->mnId);
    }
  }
  // EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ for observation idx of kf
  void add_edge(KeyFrame* kf, MapPoint* mp, size_t idx, float huber) {
    const cv::KeyPoint& kp = kf->mvKeysUn[idx];
    op.push_back(kf_index.at(kf));
    ol.push_back(mp_index.at(mp));
    uv.insert(uv.end(), {kp.pt.x, kp.pt.y});
    ur.push_back(kf->mvuRight[idx]);
    isig2.push_back(kf->mvInvLevelSigma2[kp.octave]);
    delta.push_back(huber);
    edge_kf.push_back(kf);
    edge_mp.push_back(mp);
  }
  sqlm_capture view() {
    sqlm_capture c{};
    c.kind = kind;
    c.gba_iterations = iterations;
    c.gba_robust = robust;
    c.n_pose = (int32_t)kfs.size();
    c.Tcw = Tcw.data(); c.pose_fixed = fixed.data(); c.intr = intr.data(); c.bf = bf.data(); c.kf_id = kf_id.data();
    c.n_pt = (int32_t)mps.size();
    c.pt = pt.data(); c.mp_id = mp_id.data();
    c.n_obs = (int64_t)op.size();
    c.obs_pose = op.data(); c.obs_pt = ol.data(); c.obs_uv = uv.data(); c.obs_ur = ur.data();
    c.obs_inv_sigma2 = isig2.data(); c.obs_delta = delta.data();
    c.n_lid = (int64_t)lid_pose.size();
    c.lid_pose = lid_pose.data(); c.lid_pc = lid_pc.data(); c.lid_pw = lid_pw.data(); c.lid_n = lid_n.data();
    c.lid_info = lid_info.data();
    c.has_result = !res_Tcw.empty();
    c.res_Tcw = res_Tcw.empty() ? nullptr : res_Tcw.data();
    c.res_pt = res_pt.empty() ? nullptr : res_pt.data();
    c.res_outlier = res_outlier.empty() ? nullptr : res_outlier.data();
    c.res_chi2 = nullptr;  // g2o's edges are gone when the backend returns
    return c;
  }
};

// g2oOptimizer.cc:709-781: local keyframes (pKF + covisible), local map
// points, fixed cameras, in the reference's list order. mark = true sets
// mnBALocalForKF / mnBAFixedForKF as the reference does; capture mode (mark =
// false, before g2o's own selection runs) de-duplicates with sets instead so
// the markers g2o relies on stay untouched.
void select_local(KeyFrame* pKF, std::vector<KeyFrame*>& local, std::vector<MapPoint*>& points,
                  std::vector<KeyFrame*>& fixed_cams, bool mark) {
  const unsigned long id = pKF->mnId;
  std::set<KeyFrame*> is_local, is_fixed;
  std::set<MapPoint*> seen;
  auto local_tag = [&](KeyFrame* k) {
    if (mark) k->mnBALocalForKF = id;
    else is_local.insert(k);
  };
  local_tag(pKF);
  local.push_back(pKF);
  for (KeyFrame* k : pKF->GetVectorCovisibleKeyFrames()) {
    local_tag(k);  // bad covisible KFs are tagged too, so they never become fixed cameras
    if (!k->isBad()) local.push_back(k);
  }
  for (KeyFrame* k : local)
    for (MapPoint* mp : k->GetMapPointMatches()) {
      if (!mp || mp->isBad()) continue;
      const bool fresh = mark ? mp->mnBALocalForKF != id : seen.insert(mp).second;
      if (!fresh) continue;
      points.push_back(mp);
      if (mark) mp->mnBALocalForKF = id;
    }
  for (MapPoint* mp : points)
    for (const auto& ob : mp->GetObservations()) {
      KeyFrame* k = ob.first;
      const bool skip = mark ? (k->mnBALocalForKF == id || k->mnBAFixedForKF == id)
                             : (is_local.count(k) || !is_fixed.insert(k).second);
      if (skip) continue;
      if (mark) k->mnBAFixedForKF = id;
      if (!k->isBad()) fixed_cams.push_back(k);
    }
}

// The LBA seam graph (g2oOptimizer.cc:805-912): local KFs fixed iff mnId == 0,
// fixed cameras fixed; mono edges only (the stereo branch :914-916 adds none),
// Huber (float)sqrt(5.991). Edge order = point list order x observation map order.
void build_lba(KeyFrame* pKF, SeamGraph& g, std::vector<KeyFrame*>& local, std::vector<MapPoint*>& points,
               bool mark) {
  std::vector<KeyFrame*> fixed_cams;
  select_local(pKF, local, points, fixed_cams, mark);
  std::vector<KeyFrame*> all(local);
  std::vector<uint8_t> fix;
  for (KeyFrame* k : local) fix.push_back(k->mnId == 0);
  for (KeyFrame* k : fixed_cams) { all.push_back(k); fix.push_back(1); }
  g.kind = SQLM_CAP_LBA;
  g.set_poses(all, fix);
  g.set_points(points);
  const float th = std::sqrt(5.991);
  for (MapPoint* mp : points)
    for (const auto& ob : mp->GetObservations()) {
      KeyFrame* k = ob.first;
      if (!k->isBad() && k->mvuRight[ob.second] < 0) g.add_edge(k, mp, ob.second, th);
    }
}

// LBA pass 3 association (g2oOptimizer.cc:978-1062): the flat points of the
// other local KFs, moved to the world by their pass-2 poses, form a kd-tree;
// pKF's flat points, moved by its pass-2 pose, take their nearest neighbour
// within distance_sq_threshold. Same float pose path as the reference
// (Converter::toCvMat then cv::Mat::inv()).
void lidar_pairs(KeyFrame* pKF, const std::vector<KeyFrame*>& local, const SeamGraph& g,
                 const std::vector<double>& q, const std::vector<double>& t, const lidarConfig* cfg,
                 SeamGraph& out) {
  if (!cfg || !cfg->using_flat_point) return;  // corner points: LocalBundleAdjustment routes to g2o
  auto world_of = [&](KeyFrame* k) {
    const int i = g.kf_index.at(k);
    float T[16];
    sqlm_pose_to_Tcw_f32(&q[4 * i], &t[3 * i], T);
    const cv::Mat Twc = cv::Mat(4, 4, CV_32F, T).inv();
    Eigen::Matrix4d M = Eigen::Matrix4d::Identity();
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 4; ++c) M(r, c) = Twc.at<float>(r, c);
    return Eigen::Affine3d(M);
  };
  PointIRTCloudPtr flat_map = PointIRTCloud().makeShared();
  for (KeyFrame* k : local) {
    if (k->mnId == pKF->mnId) continue;
    PointIRTCloud pts = k->surface_points_less_flat_;
    pcl::transformPointCloud(pts, pts, world_of(k));
    *flat_map += pts;
  }
  pcl::PointCloud<PointI>::Ptr cloud = PointICloud().makeShared();
  for (const PointIRT& p : *flat_map) cloud->push_back(PointIRT2PointI(p));
  if (cloud->empty()) return;
  pcl::KdTreeFLANN<PointI> tree;
  tree.setInputCloud(cloud);
  PointIRTCloud cur;
  pcl::transformPointCloud(pKF->surface_points_less_flat_, cur, world_of(pKF));
  std::vector<int> idx;
  std::vector<float> d2;
  const int pose = g.kf_index.at(pKF);
  for (size_t i = 0; i < cur.size(); ++i) {
    tree.nearestKSearch(PointIRT2PointI(cur[i]), 1, idx, d2);
    if (d2[0] >= cfg->distance_sq_threshold) continue;
    const auto& pc = pKF->surface_points_less_flat_.points[i];
    const auto& pw = cloud->points[idx[0]];
    const auto& nm = pKF->surface_points_less_flat_normal_.points[i];
    out.lid_pose.push_back(pose);
    out.lid_pc.insert(out.lid_pc.end(), {pc.x, pc.y, pc.z});
    out.lid_pw.insert(out.lid_pw.end(), {pw.x, pw.y, pw.z});
    out.lid_n.insert(out.lid_n.end(), {nm.x, nm.y, nm.z});
    out.lid_info.push_back(cfg->flat_optimized_weight);
  }
}

// ---------------------------------------------------------------- capture

std::atomic<unsigned> g_capture_seq{0};
thread_local SeamGraph* t_capture = nullptr;
thread_local std::vector<KeyFrame*> t_capture_local;

const char* capture_dir() { return std::getenv("SQLM_CAPTURE_DIR"); }

void write_capture(SeamGraph& g, const char* tag, unsigned long id) {
  const char* dir = capture_dir();
  if (!dir) return;
  char path[1024];
  std::snprintf(path, sizeof(path), "%s/%s_%lu_%u.sqcap", dir, tag, id, g_capture_seq.fetch_add(1));
  sqlm_capture c = g.view();
  report(sqlm_capture_write(path, &c), "sqlm_capture_write");
}

// (q, t) in double from the seam graph's float poses, Converter::toSE3Quat
void poses_to_double(const SeamGraph& g, std::vector<double>& q, std::vector<double>& t) {
  q.resize(4 * g.kfs.size());
  t.resize(3 * g.kfs.size());
  for (size_t i = 0; i < g.kfs.size(); ++i) sqlm_pose_from_Tcw_f32(&g.Tcw[16 * i], &q[4 * i], &t[3 * i]);
}

}  // namespace

bool hipOptimizer::CaptureEnabled() { return capture_dir() != nullptr; }

// ---------------------------------------------------------------- LBA

void hipOptimizer::LocalBundleAdjustment(KeyFrame* pKF, bool* pbStopFlag, Map* pMap, const lidarConfig* cfg) {
  if (cfg && cfg->using_sharp_point) {
    // EdgeLidarCornerPoint (pass 3 with using_sharp_point, lidarOdom.cc's ROS
    // default) is not implemented by libsqrtlm: run the reference backend for
    // this call instead of silently dropping the corner constraints
    static bool warned = false;
    if (!warned) {
      std::cerr << "hipOptimizer: using_sharp_point=1 -> g2oOptimizer::LocalBundleAdjustment "
                   "(EdgeLidarCornerPoint not implemented by libsqrtlm)" << std::endl;
      warned = true;
    }
    g2oOptimizer::LocalBundleAdjustment(pKF, pbStopFlag, pMap, cfg);
    return;
  }
  sqlm_ctx* ctx = thread_ctx();
  if (!ctx) return;
  SeamGraph g;
  std::vector<KeyFrame*> local;
  std::vector<MapPoint*> points;
  build_lba(pKF, g, local, points, true);
  const int64_t E = (int64_t)g.op.size();
  std::vector<double> q, t, intr(g.intr.begin(), g.intr.end()), X(g.pt.begin(), g.pt.end());
  std::vector<double> uv(g.uv.begin(), g.uv.end()), info(g.isig2.begin(), g.isig2.end());
  std::vector<double> delta(g.delta.begin(), g.delta.end());
  poses_to_double(g, q, t);
  if (!report(sqlm_set_problem(ctx, (int)g.kfs.size(), q.data(), t.data(), g.fixed.data(), intr.data(),
                               (int)g.mps.size(), X.data(), E, g.op.data(), g.ol.data(), uv.data(), info.data(),
                               delta.data(), nullptr),
              "sqlm_set_problem"))
    return;
  if (stopped(pbStopFlag)) return;  // :923-928
  sqlm_stats st;
  int n = 0;
  if (!report(sqlm_optimize(ctx, 0, 5, 0.0, stop_ptr(pbStopFlag), &st, &n), "pass 1")) return;
  std::vector<double> chi2(E);
  std::vector<uint8_t> pos(E), level(E, 0);
  if (!stopped(pbStopFlag)) {  // :939-975; edges of points gone bad keep level 0 and their kernel
    sqlm_get_edge_chi2(ctx, chi2.data());
    sqlm_get_edge_depth_positive(ctx, pos.data());
    for (int64_t e = 0; e < E; ++e) {
      if (g.edge_mp[e]->isBad()) continue;
      if (chi2[e] > 5.991 || !pos[e]) level[e] = 1;
      delta[e] = 0.0;
    }
    sqlm_set_edge_level(ctx, level.data());
    sqlm_set_robust(ctx, delta.data());
    if (!report(sqlm_optimize(ctx, 0, 10, 0.0, stop_ptr(pbStopFlag), &st, &n), "pass 2")) return;
  }
  // pass 3 (:978-1114): LiDAR flat pairs at the pass-2 poses, 20 iterations
  sqlm_get_poses(ctx, q.data(), t.data());
  SeamGraph lid;
  lidar_pairs(pKF, local, g, q, t, cfg, lid);
  if (!lid.lid_pose.empty())
    report(sqlm_set_lidar(ctx, (int64_t)lid.lid_pose.size(), lid.lid_pose.data(), lid.lid_pc.data(),
                          lid.lid_pw.data(), lid.lid_n.data(), lid.lid_info.data()),
           "sqlm_set_lidar");
  if (!report(sqlm_optimize(ctx, 0, 20, 0.0, stop_ptr(pbStopFlag), &st, &n), "pass 3")) return;
  // outliers (:1119-1136) and write-back under the map mutex (:1145-1189)
  sqlm_get_edge_chi2(ctx, chi2.data());
  sqlm_get_edge_depth_positive(ctx, pos.data());
  sqlm_get_poses(ctx, q.data(), t.data());
  sqlm_get_points(ctx, X.data());
  std::vector<std::pair<KeyFrame*, MapPoint*>> erase;
  for (int64_t e = 0; e < E; ++e)
    if (!g.edge_mp[e]->isBad() && (chi2[e] > 5.991 || !pos[e])) erase.emplace_back(g.edge_kf[e], g.edge_mp[e]);
  std::unique_lock<std::mutex> lock(pMap->mMutexMapUpdate);
  for (auto& [k, mp] : erase) {
    k->EraseMapPointMatch(mp);
    mp->EraseObservation(k);
  }
  for (KeyFrame* k : local) {
    const int i = g.kf_index.at(k);
    float T[16];
    sqlm_pose_to_Tcw_f32(&q[4 * i], &t[3 * i], T);  // Converter::toCvMat(SE3Quat)
    k->SetPose(cv::Mat(4, 4, CV_32F, T).clone());
  }
  for (MapPoint* mp : points) {
    const int i = g.mp_index.at(mp);
    cv::Mat P(3, 1, CV_32F);
    for (int k = 0; k < 3; ++k) P.at<float>(k) = (float)X[3 * i + k];
    mp->SetWorldPos(P);
    mp->UpdateNormalAndDepth();
  }
}

// ---------------------------------------------------------------- GBA

namespace {

// g2oOptimizer.cc:142-296: non-bad KFs (KF 0 fixed); non-bad points; an edge
// per observation by a non-bad KF with mnId <= maxKFid, mono or stereo, Huber
// (float)sqrt(5.99) / (float)sqrt(7.815) when bRobust. Points without edges
// are removed (the replay compacts them and writes them back unchanged).
void build_ba(const std::vector<KeyFrame*>& vpKFs, const std::vector<MapPoint*>& vpMP, int iters, bool robust,
              SeamGraph& g) {
  std::vector<KeyFrame*> kfs;
  std::vector<uint8_t> fix;
  unsigned long maxKFid = 0;
  for (KeyFrame* k : vpKFs) {
    if (k->isBad()) continue;
    kfs.push_back(k);
    fix.push_back(k->mnId == 0);
    maxKFid = std::max<unsigned long>(maxKFid, k->mnId);
  }
  std::vector<MapPoint*> mps;
  for (MapPoint* mp : vpMP)
    if (!mp->isBad()) mps.push_back(mp);
  g.kind = SQLM_CAP_GBA;
  g.iterations = iters;
  g.robust = robust;
  g.set_poses(kfs, fix);
  g.set_points(mps);
  const float th2 = std::sqrt(5.99), th3 = std::sqrt(7.815);
  for (MapPoint* mp : mps)
    for (const auto& ob : mp->GetObservations()) {
      KeyFrame* k = ob.first;
      if (k->isBad() || k->mnId > maxKFid) continue;
      const bool stereo = k->mvuRight[ob.second] >= 0;
      g.add_edge(k, mp, ob.second, robust ? (stereo ? th3 : th2) : 0.f);
    }
}

}  // namespace

void hipOptimizer::BundleAdjustment(const std::vector<KeyFrame*>& vpKFs, const std::vector<MapPoint*>& vpMP,
                                    int nIterations, bool* pbStopFlag, unsigned long nLoopKF, bool bRobust) {
  sqlm_ctx* ctx = thread_ctx();
  if (!ctx) return;
  SeamGraph g;
  build_ba(vpKFs, vpMP, nIterations, bRobust, g);
  std::vector<float> Tcw(g.Tcw.size()), P(g.pt.size());
  sqlm_replay_out out{};
  out.Tcw = Tcw.data();
  out.pt = P.data();
  sqlm_capture c = g.view();
  if (!report(sqlm_capture_replay(ctx, &c, stop_ptr(pbStopFlag), &out), "sqlm_capture_replay")) return;
  std::vector<uint8_t> has_edge(g.mps.size(), 0);
  for (int32_t l : g.ol) has_edge[l] = 1;
  // write-back (:306-360): SetPose / SetWorldPos, or mTcwGBA / mPosGBA after a loop
  for (size_t i = 0; i < g.kfs.size(); ++i) {
    KeyFrame* k = g.kfs[i];
    const cv::Mat T = cv::Mat(4, 4, CV_32F, &Tcw[16 * i]).clone();
    if (nLoopKF == 0) {
      k->SetPose(T);
    } else {
      k->mTcwGBA.create(4, 4, CV_32F);
      T.copyTo(k->mTcwGBA);
      k->mnBAGlobalForKF = nLoopKF;
    }
  }
  for (size_t i = 0; i < g.mps.size(); ++i) {
    if (!has_edge[i]) continue;  // vbNotIncludedMP
    MapPoint* mp = g.mps[i];
    const cv::Mat X = cv::Mat(3, 1, CV_32F, &P[3 * i]).clone();
    if (nLoopKF == 0) {
      mp->SetWorldPos(X);
      mp->UpdateNormalAndDepth();
    } else {
      mp->mPosGBA.create(3, 1, CV_32F);
      X.copyTo(mp->mPosGBA);
      mp->mnBAGlobalForKF = nLoopKF;
    }
  }
}

void hipOptimizer::GlobalBundleAdjustemnt(Map* pMap, int nIterations, bool* pbStopFlag, unsigned long nLoopKF,
                                          bool bRobust) {
  const std::vector<KeyFrame*> kfs = pMap->GetAllKeyFrames();
  const std::vector<MapPoint*> mps = pMap->GetAllMapPoints();
  BundleAdjustment(kfs, mps, nIterations, pbStopFlag, nLoopKF, bRobust);
}

// ---------------------------------------------------------------- capture mode around g2o

void hipOptimizer::BeginCaptureLBA(KeyFrame* pKF) {
  if (!CaptureEnabled()) return;
  delete t_capture;
  t_capture = new SeamGraph();
  t_capture_local.clear();
  std::vector<MapPoint*> points;
  build_lba(pKF, *t_capture, t_capture_local, points, false);
}

void hipOptimizer::CaptureLidarFlat(const Eigen::Vector3d& pc, const Eigen::Vector3d& pw, const Eigen::Vector3d& n,
                                    double w) {
  if (!t_capture || t_capture->kfs.empty() || t_capture_local.empty()) return;
  SeamGraph& g = *t_capture;
  g.lid_pose.push_back(g.kf_index.at(t_capture_local.front()));  // the current KF
  g.lid_pc.insert(g.lid_pc.end(), {pc.x(), pc.y(), pc.z()});
  g.lid_pw.insert(g.lid_pw.end(), {pw.x(), pw.y(), pw.z()});
  g.lid_n.insert(g.lid_n.end(), {n.x(), n.y(), n.z()});
  g.lid_info.push_back(w);
}

namespace {
void capture_results(SeamGraph& g) {
  g.res_Tcw.clear();
  g.res_pt.clear();
  for (KeyFrame* k : g.kfs) {
    const cv::Mat T = k->GetPose();
    for (int r = 0; r < 4; ++r)
      for (int c = 0; c < 4; ++c) g.res_Tcw.push_back(T.at<float>(r, c));
  }
  for (MapPoint* mp : g.mps) {
    const cv::Mat X = mp->GetWorldPos();
    g.res_pt.insert(g.res_pt.end(), {X.at<float>(0), X.at<float>(1), X.at<float>(2)});
  }
  // an edge whose observation the backend erased was tagged an outlier
  g.res_outlier.assign(g.op.size(), 0);
  for (size_t e = 0; e < g.op.size(); ++e) g.res_outlier[e] = !g.edge_mp[e]->IsInKeyFrame(g.edge_kf[e]);
}
}  // namespace

void hipOptimizer::EndCaptureLBA() {
  if (!t_capture) return;
  capture_results(*t_capture);
  write_capture(*t_capture, "lba", t_capture->kfs.empty() ? 0 : t_capture_local.front()->mnId);
  delete t_capture;
  t_capture = nullptr;
}

void hipOptimizer::BeginCaptureBA(const std::vector<KeyFrame*>& vpKFs, const std::vector<MapPoint*>& vpMP,
                                  int nIterations, bool bRobust) {
  if (!CaptureEnabled()) return;
  delete t_capture;
  t_capture = new SeamGraph();
  build_ba(vpKFs, vpMP, nIterations, bRobust, *t_capture);
}

void hipOptimizer::EndCaptureBA(unsigned long nLoopKF) {
  if (!t_capture) return;
  if (nLoopKF == 0) {  // results are in the map; after a loop they sit in mTcwGBA / mPosGBA
    capture_results(*t_capture);
  } else {
    SeamGraph& g = *t_capture;
    g.res_Tcw.clear();
    g.res_pt.clear();
    for (KeyFrame* k : g.kfs)
      for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) g.res_Tcw.push_back(k->mTcwGBA.at<float>(r, c));
    for (MapPoint* mp : g.mps) {
      const cv::Mat X = mp->mPosGBA.empty() ? mp->GetWorldPos() : mp->mPosGBA;
      g.res_pt.insert(g.res_pt.end(), {X.at<float>(0), X.at<float>(1), X.at<float>(2)});
    }
  }
  t_capture->res_outlier.clear();  // GBA erases nothing
  write_capture(*t_capture, "ba", nLoopKF);
  delete t_capture;
  t_capture = nullptr;
}



// ---------------------------------------------------------------- essential graph
namespace {

// g2o::Sim3 <-> the ABI's [qx qy qz qw tx ty tz s] (sqrtlm.h, sqlm_eg_set_problem)
void sim3_pack(const g2o::Sim3& S, double* o) {
  const Eigen::Quaterniond& q = S.rotation();
  o[0] = q.x(); o[1] = q.y(); o[2] = q.z(); o[3] = q.w();
  o[4] = S.translation()[0]; o[5] = S.translation()[1]; o[6] = S.translation()[2];
  o[7] = S.scale();
}
g2o::Sim3 sim3_unpack(const double* o) {
  return g2o::Sim3(Eigen::Quaterniond(o[3], o[0], o[1], o[2]), Eigen::Vector3d(o[4], o[5], o[6]), o[7]);
}

}  // namespace

void hipOptimizer::OptimizeEssentialGraph(Map* pMap, KeyFrame* pLoopKF, KeyFrame* pCurKF,
                                          const LoopClosing::KeyFrameAndPose& NonCorrectedSim3,
                                          const LoopClosing::KeyFrameAndPose& CorrectedSim3,
                                          const std::map<KeyFrame*, std::set<KeyFrame*> >& LoopConnections,
                                          const bool& bFixScale) {
  sqlm_ctx* ctx = thread_ctx();
  if (!ctx) return;
  const std::vector<KeyFrame*> vpKFs = pMap->GetAllKeyFrames();
  const std::vector<MapPoint*> vpMPs = pMap->GetAllMapPoints();
  const unsigned int nMaxKFid = pMap->GetMaxKFid();
  std::vector<g2o::Sim3, Eigen::aligned_allocator<g2o::Sim3> > vScw(nMaxKFid + 1);
  std::vector<g2o::Sim3, Eigen::aligned_allocator<g2o::Sim3> > vCorrectedSwc(nMaxKFid + 1);
  const int minFeat = 100;
  // vertices (g2oOptimizer.cc:1240-1278): one per good keyframe; the ABI wants
  // them in g2o id order, so vertex v <-> mnId through a dense index
  std::vector<int> vidx(nMaxKFid + 1, -1);
  std::vector<KeyFrame*> order;
  for (KeyFrame* pKF : vpKFs)
    if (!pKF->isBad()) order.push_back(pKF);
  std::sort(order.begin(), order.end(), [](KeyFrame* a, KeyFrame* b) { return a->mnId < b->mnId; });
  std::vector<double> Siw(8 * order.size());
  std::vector<uint8_t> fixed(order.size(), 0);
  for (size_t v = 0; v < order.size(); ++v) {
    KeyFrame* pKF = order[v];
    const int nIDi = pKF->mnId;
    auto it = CorrectedSim3.find(pKF);
    if (it != CorrectedSim3.end()) {
      vScw[nIDi] = it->second;
    } else {
      const Eigen::Matrix<double, 3, 3> Rcw = Converter::toMatrix3d(pKF->GetRotation());
      const Eigen::Matrix<double, 3, 1> tcw = Converter::toVector3d(pKF->GetTranslation());
      vScw[nIDi] = g2o::Sim3(Rcw, tcw, 1.0);
    }
    sim3_pack(vScw[nIDi], &Siw[8 * v]);
    fixed[v] = pKF == pLoopKF;
    vidx[nIDi] = (int)v;
  }
  // edges in the reference's insertion order (:1280-1417); an edge whose vertex
  // is missing (a bad keyframe) is rejected by g2o's addEdge, so it is skipped
  std::vector<int32_t> ei, ej;
  std::vector<double> Sji;
  auto add = [&](unsigned long i, unsigned long j, const g2o::Sim3& S) {
    if (i > nMaxKFid || j > nMaxKFid || vidx[i] < 0 || vidx[j] < 0) return;
    ei.push_back(vidx[i]);
    ej.push_back(vidx[j]);
    Sji.resize(Sji.size() + 8);
    sim3_pack(S, &Sji[Sji.size() - 8]);
  };
  auto ncs = [&](KeyFrame* k) -> g2o::Sim3 {
    auto f = NonCorrectedSim3.find(k);
    return f != NonCorrectedSim3.end() ? f->second : vScw[k->mnId];
  };
  std::set<std::pair<long unsigned int, long unsigned int> > sInsertedEdges;
  for (auto mit = LoopConnections.begin(); mit != LoopConnections.end(); ++mit) {
    KeyFrame* pKF = mit->first;
    const long unsigned int nIDi = pKF->mnId;
    const g2o::Sim3 Swi = vScw[nIDi].inverse();
    for (KeyFrame* pKFj : mit->second) {
      const long unsigned int nIDj = pKFj->mnId;
      if ((nIDi != pCurKF->mnId || nIDj != pLoopKF->mnId) && pKF->GetWeight(pKFj) < minFeat) continue;
      add(nIDi, nIDj, vScw[nIDj] * Swi);
      sInsertedEdges.insert(std::make_pair(std::min(nIDi, nIDj), std::max(nIDi, nIDj)));
    }
  }
  for (KeyFrame* pKF : vpKFs) {
    const long unsigned int nIDi = pKF->mnId;
    const g2o::Sim3 Swi = ncs(pKF).inverse();
    KeyFrame* pParentKF = pKF->GetParent();
    if (pParentKF) add(nIDi, pParentKF->mnId, ncs(pParentKF) * Swi);  // spanning tree
    const std::set<KeyFrame*> sLoopEdges = pKF->GetLoopEdges();
    for (KeyFrame* pLKF : sLoopEdges)
      if (pLKF->mnId < pKF->mnId) add(nIDi, pLKF->mnId, ncs(pLKF) * Swi);
    for (KeyFrame* pKFn : pKF->GetCovisiblesByWeight(minFeat)) {  // covisibility
      if (pKFn && pKFn != pParentKF && !pKF->hasChild(pKFn) && !sLoopEdges.count(pKFn) && !pKFn->isBad() &&
          pKFn->mnId < pKF->mnId) {
        if (sInsertedEdges.count(std::make_pair(std::min(pKF->mnId, pKFn->mnId), std::max(pKF->mnId, pKFn->mnId))))
          continue;
        add(nIDi, pKFn->mnId, ncs(pKFn) * Swi);
      }
    }
  }
  // initializeOptimization(); setUserLambdaInit(1e-16); optimize(20), identity information
  if (!report(sqlm_eg_set_problem(ctx, (int)order.size(), Siw.data(), fixed.data(), bFixScale ? 1 : 0,
                                  (int64_t)ei.size(), ei.data(), ej.data(), Sji.data(), nullptr),
              "sqlm_eg_set_problem"))
    return;
  sqlm_stats st;
  int n_iter = 0;
  if (!report(sqlm_eg_optimize(ctx, 20, 1e-16, nullptr, &st, &n_iter), "sqlm_eg_optimize")) return;
  if (!report(sqlm_eg_get_poses(ctx, Siw.data()), "sqlm_eg_get_poses")) return;
  // write-back (:1427-1531): SE3 poses from the corrected Sim3, map points
  // through their reference keyframe's correction
  std::unique_lock<std::mutex> lock(pMap->mMutexMapUpdate);
  for (size_t v = 0; v < order.size(); ++v) {
    KeyFrame* pKFi = order[v];
    const g2o::Sim3 CorrectedSiw = sim3_unpack(&Siw[8 * v]);
    vCorrectedSwc[pKFi->mnId] = CorrectedSiw.inverse();
    const Eigen::Matrix3d eigR = CorrectedSiw.rotation().toRotationMatrix();
    Eigen::Vector3d eigt = CorrectedSiw.translation();
    eigt *= (1. / CorrectedSiw.scale());
    pKFi->SetPose(Converter::toCvSE3(eigR, eigt));
  }
  for (MapPoint* pMP : vpMPs) {
    if (pMP->isBad()) continue;
    const int nIDr = pMP->mnCorrectedByKF == pCurKF->mnId ? (int)pMP->mnCorrectedReference
                                                          : (int)pMP->GetReferenceKeyFrame()->mnId;
    const Eigen::Matrix<double, 3, 1> P = Converter::toVector3d(pMP->GetWorldPos());
    pMP->SetWorldPos(Converter::toCvMat(vCorrectedSwc[nIDr].map(vScw[nIDr].map(P))));
    pMP->UpdateNormalAndDepth();
  }
}

}  // namespace ORB_SLAM2
