/*
 * sqrtlm_orb.h — C ABI of the ORB front-end path of libsqrtlm.so (SURVEY.md
 * §8 row f3): ORB FAST + steered-BRIEF extraction and Hamming matching on the
 * GPU, behind the reference's ORBextractor / ORBmatcher interfaces.
 *
 * Seam: ORB_SLAM2::ORBextractor::operator()(image, keypoints, descriptors)
 * (src/frontend/ORBextractor.cc:1284-1399, declared include/frontend/
 * ORBextractor.h) and ORBmatcher::SearchForInitialization / DescriptorDistance
 * (src/frontend/ORBmatcher.cc:573-718, :2096-2116). Frame::ExtractORB
 * (src/data_structure/Frame.cc) calls the extractor once per image; the
 * adapter replaces that call with sqlm_orb_extract and copies the arrays into
 * cv::KeyPoint / cv::Mat.
 *
 * Contexts come from sqrtlm.h (sqlm_ctx_create); the calls run on the
 * context's HIP stream. Status codes as in sqrtlm.h.
 */
#ifndef SQRTLM_ORB_H
#define SQRTLM_ORB_H

#include <stdint.h>

#include "sqrtlm.h"

#ifdef __cplusplus
extern "C" {
#endif

/* cv::KeyPoint fields the reference uses: pt.x, pt.y, size, angle (degrees,
 * [0,360)), response (FAST score), octave (pyramid level). */
typedef struct sqlm_keypoint {
  float x, y, size, angle, response;
  int32_t octave;
} sqlm_keypoint;

/* ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)
 * (ORBextractor.cc:474-560; cfg/KITTI00-02.yaml: 2000, 1.2, 8, 20, 7). */
typedef struct sqlm_orb_params {
  int32_t nfeatures;
  float scale_factor;
  int32_t nlevels;
  int32_t ini_th_fast;
  int32_t min_th_fast;
} sqlm_orb_params;

/* ORBextractor::operator()(image, keypoints, descriptors): 8-bit grey image
 * (w x h, row stride in bytes, host memory) -> keypoints in level-0
 * coordinates and 32-byte descriptors, level after level in the reference's
 * order. Writes at most `cap` entries; *n_out = the full count (> cap means
 * the arrays were too small: nothing beyond cap is written).
 * SQLM_ERR_UNSUPPORTED: a pyramid level narrower / shorter than one 30-pixel
 * cell (the reference divides by zero there) or wider than 4096. */
int sqlm_orb_extract(sqlm_ctx *ctx, const sqlm_orb_params *p, const uint8_t *image, int w, int h, int stride,
                     sqlm_keypoint *kps, uint8_t *desc, int cap, int *n_out);

/* The pyramid image of `level` from the last sqlm_orb_extract (ORBextractor::
 * mvImagePyramid[level], GetImagePyramid) into out [lh][lw]; *lw / *lh its size. */
int sqlm_orb_get_level(sqlm_ctx *ctx, int level, uint8_t *out, int cap, int *lw, int *lh);

/* Brute-force Hamming matching (DescriptorDistance, ORBmatcher.cc:2096-2116,
 * over every train descriptor): for each query, the best distance, its first
 * train index in increasing order (strict <, the reference's tie-breaking)
 * and the second-best distance (INT_MAX when nt < 2). */
int sqlm_orb_match_bf(sqlm_ctx *ctx, const uint8_t *query, int nq, const uint8_t *train, int nt, int32_t *best_idx,
                      int32_t *best_dist, int32_t *second_dist);

/* Frame grid bounds of the second frame (Frame::mnMinX, mnMaxX, mnMinY, mnMaxY). */
typedef struct sqlm_frame_bounds {
  float min_x, max_x, min_y, max_y;
} sqlm_frame_bounds;

/* ORBmatcher(nnratio, check_ori).SearchForInitialization(F1, F2, prev,
 * matches12, window) (ORBmatcher.cc:573-718): k1/d1 = F1.mvKeysUn /
 * mDescriptors, k2/d2 = F2's, prev [n1][2] = vbPrevMatched (updated in place),
 * m12 [n1] = vnMatches12; *n_matches = the return value. */
int sqlm_orb_search_for_init(sqlm_ctx *ctx, const sqlm_keypoint *k1, const uint8_t *d1, int n1,
                             const sqlm_keypoint *k2, const uint8_t *d2, int n2, const sqlm_frame_bounds *f2,
                             float *prev, int32_t *m12, int window, float nnratio, int check_ori, int *n_matches);

/* The Frame fields the projection searches read and write
 * (include/data_structure/Frame.h): kps = mvKeysUn, desc = mDescriptors
 * [n][32], uright = mvuRight (NULL: monocular), bounds = mnMinX..mnMaxY,
 * scale_factors = mvScaleFactors [n_levels], fx fy cx cy, bf = mbf, mb, and
 * the keypoint slots mvpMapPoints as map-point ids (slot_mp, -1 = NULL) with
 * slot_obs = that point's Observations() > 0 — both updated by the call. */
typedef struct sqlm_orb_frame {
  const sqlm_keypoint *kps;
  const uint8_t *desc;
  const float *uright;
  int32_t n;
  sqlm_frame_bounds bounds;
  const float *scale_factors;
  int32_t n_levels;
  float fx, fy, cx, cy, bf, mb;
  int32_t *slot_mp;
  uint8_t *slot_obs;
} sqlm_orb_frame;

/* A local map point as Tracking::SearchLocalPoints leaves it (MapPoint.h:
 * mnId, mTrackProjX/Y/XR, mTrackViewCos, mnTrackScaleLevel, mbTrackInView,
 * isBad(), Observations() > 0). */
typedef struct sqlm_track_point {
  int32_t id;
  float proj_x, proj_y, proj_xr, view_cos;
  int32_t level;
  uint8_t in_view, bad, has_obs, pad;
} sqlm_track_point;

/* One LastFrame keypoint slot: mvpMapPoints[i] (id, -1 = NULL), the point's
 * GetWorldPos(), mvKeys[i].octave, mvKeysUn[i].angle, mvbOutlier[i] and the
 * point's Observations() > 0. */
typedef struct sqlm_last_point {
  int32_t id;
  float x, y, z;
  int32_t octave;
  float angle;
  uint8_t outlier, has_obs, pad[2];
} sqlm_last_point;

/* ORBmatcher(nnratio).SearchByProjection(F, vpMapPoints, th)
 * (ORBmatcher.cc:67-181): mps [n_mp] with their descriptors mp_desc [n_mp][32]
 * (GetDescriptor()). Candidate windows (GetFeaturesInArea, Frame.cc:1463) and
 * their Hamming distances on the GPU; the order-dependent acceptance (a slot
 * taken by an earlier point is skipped) on the host over those lists.
 * *n_matches = the return value. */
int sqlm_orb_search_by_projection_local(sqlm_ctx *ctx, sqlm_orb_frame *F, const sqlm_track_point *mps,
                                        const uint8_t *mp_desc, int n_mp, float th, float nnratio, int *n_matches);

/* ORBmatcher(., check_ori).SearchByProjection(CurrentFrame, LastFrame, th,
 * bMono) (ORBmatcher.cc:1717-1883): F = CurrentFrame, Tcw / Tlw = the 3x4
 * rows of CurrentFrame.mTcw / LastFrame.mTcw (float, row-major), lp / ldesc =
 * LastFrame's n_last slots and their points' descriptors. */
int sqlm_orb_search_by_projection_last(sqlm_ctx *ctx, sqlm_orb_frame *F, const float *Tcw, const float *Tlw,
                                       const sqlm_last_point *lp, const uint8_t *ldesc, int n_last, float th,
                                       int mono, int check_ori, int *n_matches);

/* A map point as the keyframe searches read it (MapPoint.h): mnId,
 * GetWorldPos(), GetNormal(), mfMinDistance / mfMaxDistance (the searches
 * apply the 0.8 / 1.2 invariance factors themselves) and the caller's
 * pre-filter `skip` (isBad(), or the point is already found / already in the
 * keyframe — each search's own first test). */
typedef struct sqlm_map_point {
  int32_t id;
  float x, y, z, nx, ny, nz, min_dist, max_dist;
  uint8_t skip, pad[3];
} sqlm_map_point;

/* ORBmatcher::SearchByProjection(pKF, Scw, vpPoints, vpMatched, th)
 * (ORBmatcher.cc:423-571): F = pKF with F->slot_mp = vpMatched (ids, updated);
 * Scw = 3x4 rows of the Sim3 [sR | t]. */
int sqlm_orb_search_by_projection_sim3(sqlm_ctx *ctx, sqlm_orb_frame *F, const float *Scw, const sqlm_map_point *mps,
                                       const uint8_t *mp_desc, int n, int th, int *n_matches);

/* ORBmatcher::Fuse(pKF, vpMapPoints, th) (:1109-1294; sim3 = 0, T = pKF's
 * 3x4 Tcw) and Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) (:1296-1446;
 * sim3 = 1, T = Scw): fuse_idx [n] = the keypoint of pKF each point fuses
 * into (-1: none). The map edit that follows (MapPoint::Replace /
 * AddObservation / vpReplacePoint) is the caller's, in point order; it
 * does not feed back into the searches of later points. *n_fused = nFused. */
int sqlm_orb_fuse(sqlm_ctx *ctx, const sqlm_orb_frame *F, const float *T, int sim3, const sqlm_map_point *mps,
                  const uint8_t *mp_desc, int n, float th, int32_t *fuse_idx, int *n_fused);

/* ORBmatcher::SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th,
 * ORBdist) (:1902-2046): F = CurrentFrame (slot_mp updated), Tcw its 3x4
 * pose; mps / mp_desc / kf_angle = pKF's map-point slots
 * (GetMapPointMatches; NULL, bad or already-found slots have skip set) and
 * pKF->mvKeysUn[i].angle. */
int sqlm_orb_search_by_projection_kf(sqlm_ctx *ctx, sqlm_orb_frame *F, const float *Tcw, const sqlm_map_point *mps,
                                     const uint8_t *mp_desc, const float *kf_angle, int n, float th, int orb_dist,
                                     int check_ori, int *n_matches);

/* ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th)
 * (ORBmatcher.cc:1448-1608): K1 / K2 the two keyframes (K1's fx fy cx cy
 * project both ways, as the reference does), T1w / T2w their 3x4 poses,
 * mp1 / mp2 their map-point slots (id -1: NULL, skip: isBad()) with
 * descriptors; R12 row-major, t12 [3]. matches12 [K1->n]: in = vpMatches12
 * as ids (-1: NULL), out = with the mutual matches added. *n_found = nFound. */
int sqlm_orb_search_by_sim3(sqlm_ctx *ctx, const sqlm_orb_frame *K1, const sqlm_orb_frame *K2, const float *T1w,
                            const float *T2w, const sqlm_map_point *mp1, const uint8_t *md1, const sqlm_map_point *mp2,
                            const uint8_t *md2, float s12, const float *R12, const float *t12, float th,
                            int32_t *matches12, int *n_found);

/* A keyframe (or Frame) as the BoW searches read it: mvKeysUn, mDescriptors
 * [n][32], the DBoW2 FeatureVector as the node id of each feature (-1: the
 * feature is not in mFeatVec), GetMapPointMatches() ids (-1: NULL), their
 * isBad() (NULL: none bad) and mvuRight (NULL: monocular). */
typedef struct sqlm_bow_frame {
  const sqlm_keypoint *kps;
  const uint8_t *desc;
  const int32_t *node;
  const int32_t *mp;
  const uint8_t *mp_bad;
  const float *uright;
  int32_t n;
} sqlm_bow_frame;

/* ORBmatcher(nnratio, check_ori).SearchByBoW(pKF, F, vpMapPointMatches)
 * (:246-403): matches [F->n] = map-point ids (-1: NULL). */
int sqlm_orb_search_by_bow_kf_frame(sqlm_ctx *ctx, const sqlm_bow_frame *KF, const sqlm_bow_frame *F, float nnratio,
                                    int check_ori, int32_t *matches, int *n_matches);

/* SearchByBoW(pKF1, pKF2, vpMatches12) (:731-869): matches12 [K1->n] = ids
 * of pKF2's map points (-1: NULL). */
int sqlm_orb_search_by_bow_kf_kf(sqlm_ctx *ctx, const sqlm_bow_frame *K1, const sqlm_bow_frame *K2, float nnratio,
                                 int check_ori, int32_t *matches12, int *n_matches);

/* SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, bOnlyStereo)
 * (:887-1096): m12 [K1->n] = the matched pKF2 keypoint (-1: none; the
 * reference's vMatchedPairs are the (i, m12[i]) with m12[i] >= 0, in i
 * order). C1 = pKF1->GetCameraCenter(), T2w = pKF2's 3x4 pose, cam2 = pKF2's
 * fx fy cx cy, scale_factors2 = pKF2->mvScaleFactors (mvLevelSigma2 = its
 * squares), F12 row-major 3x3. */
int sqlm_orb_search_for_triangulation(sqlm_ctx *ctx, const sqlm_bow_frame *K1, const sqlm_bow_frame *K2,
                                      const float *C1, const float *T2w, const float *cam2,
                                      const float *scale_factors2, int n_levels2, const float *F12, int only_stereo,
                                      int check_ori, int32_t *m12, int *n_matches);

/* Bench helper: time `reps` extractions of one image (input uploaded once;
 * timed region = the whole device pipeline incl. the host quadtree step).
 * ms_per_frame, and per-stage device milliseconds [6]: pyramid, fast,
 * compact, blur, describe, host quadtree (wall). */
int sqlm_orb_bench_extract(sqlm_ctx *ctx, const sqlm_orb_params *p, const uint8_t *image, int w, int h, int stride,
                           int reps, double *ms_per_frame, double *stage_ms);

#ifdef __cplusplus
}
#endif
#endif
