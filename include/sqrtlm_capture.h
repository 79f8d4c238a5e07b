/*
 * sqrtlm_capture.h — BA problem capture / replay at the Optimizer seam
 * (SURVEY.md §8 row f1).
 *
 * A capture is the exact input the reference's g2o path receives at the seam
 * `Optimizer::LocalBundleAdjustment` / `Optimizer::GlobalBundleAdjustemnt`
 * (src/backend/Optimizer.cc:67-98), in the reference's own float32 form
 * (KeyFrame::GetPose, MapPoint::GetWorldPos, undistorted keypoints, octave
 * invSigma2, mvuRight), plus, optionally, what the reference's g2o backend
 * wrote back (poses, points, outlier tags, edge chi2). The adapter
 * (adapter/hipOptimizer.cc) writes one file per call when SQLM_CAPTURE_DIR is
 * set; `sqlm_capture_replay` runs the same schedule on the GPU so KITTI
 * problems can be compared without ROS / OpenCV / PCL on the GPU box.
 *
 * File layout (little endian, version 1):
 *   char magic[8] = "SQLMCAP1"; uint32 version; uint32 kind;
 *   then tagged sections until EOF, each
 *   uint32 tag (fourcc); uint32 elem_bytes; uint64 count; payload[count*elem_bytes].
 * Readers skip unknown tags, so later versions can add sections.
 *
 * Conversions on replay are the reference's own: Tcw float 4x4 ->
 * SE3Quat by Converter::toSE3Quat (Converter.cc:55-68); float -> double
 * widening for points, pixels, invSigma2 and Huber deltas
 * (g2oOptimizer.cc:880-907); results back to float through
 * Converter::toCvMat (Converter.cc:73-79,98-109).
 */
#ifndef SQRTLM_CAPTURE_H
#define SQRTLM_CAPTURE_H

#include <stdint.h>

#include "sqrtlm.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SQLM_CAP_LBA 1 /* g2oOptimizer::LocalBundleAdjustment (g2oOptimizer.cc:704-1191) */
#define SQLM_CAP_GBA 2 /* g2oOptimizer::BundleAdjustment (g2oOptimizer.cc:110-362)       */

typedef struct sqlm_capture {
  uint32_t kind;       /* SQLM_CAP_*                                                 */
  int32_t gba_iterations; /* GBA: optimize(n) (LoopClosing.cc:987-991 passes 10)     */
  uint8_t gba_robust;  /* GBA: bRobust (Huber sqrt(5.991) mono edges)               */
  /* vertices: keyframe poses (VertexSE3Expmap), id order */
  int32_t n_pose;
  float *Tcw;          /* [n_pose][16] row-major T_cw (KeyFrame::GetPose)            */
  uint8_t *pose_fixed; /* [n_pose] setFixed                                          */
  float *intr;         /* [n_pose][4] fx fy cx cy (KeyFrame members)                 */
  float *bf;           /* [n_pose] mbf (stereo edges only; may be NULL)              */
  uint64_t *kf_id;     /* [n_pose] KeyFrame::mnId (bookkeeping; may be NULL)         */
  /* map points (VertexSBAPointXYZ, marginalised) */
  int32_t n_pt;
  float *pt;           /* [n_pt][3] MapPoint::GetWorldPos                            */
  uint64_t *mp_id;     /* [n_pt] MapPoint::mnId (may be NULL)                        */
  /* observations = edges in insertion order */
  int64_t n_obs;
  int32_t *obs_pose, *obs_pt; /* [n_obs] indices into the arrays above               */
  float *obs_uv;       /* [n_obs][2] kpUn.pt                                         */
  float *obs_ur;       /* [n_obs] mvuRight (< 0: mono edge); NULL = all mono         */
  float *obs_inv_sigma2; /* [n_obs] mvInvLevelSigma2[octave]                         */
  float *obs_delta;    /* [n_obs] Huber delta as set (0 = no kernel); NULL = none    */
  /* LiDAR flat-point pairs joined in LBA pass 3 (g2oOptimizer.cc:1034-1114),
   * as the reference's kd-tree found them at the pass-2 poses */
  int64_t n_lid;
  int32_t *lid_pose;
  double *lid_pc, *lid_pw, *lid_n; /* [n_lid][3]                                     */
  double *lid_info;    /* [n_lid] flat_optimized_weight                              */
  /* reference results (what the g2o backend wrote back), optional */
  uint8_t has_result;
  float *res_Tcw;      /* [n_pose][16]                                               */
  float *res_pt;       /* [n_pt][3]                                                  */
  uint8_t *res_outlier; /* [n_obs] LBA erase tags (chi2 > 5.991 || depth <= 0)      */
  double *res_chi2;    /* [n_obs] e->chi2() after the last pass                      */
} sqlm_capture;

/* Write / read a capture file. Read allocates every array (sqlm_capture_free
 * releases them); absent optional sections stay NULL. */
int sqlm_capture_write(const char *path, const sqlm_capture *cap);
int sqlm_capture_read(const char *path, sqlm_capture **out);
void sqlm_capture_free(sqlm_capture *cap);

typedef struct sqlm_replay_out {
  float *Tcw;          /* [n_pose][16] caller-allocated, or NULL                     */
  float *pt;           /* [n_pt][3]                                                  */
  uint8_t *outlier;    /* [n_obs] (LBA)                                              */
  double *chi2;        /* [n_obs]                                                    */
  sqlm_stats stats[3]; /* per LBA pass; GBA uses stats[0]                            */
  int ran;             /* LBA: 0 if the stop flag was already set                    */
} sqlm_replay_out;

/* Run the captured call on ctx's GPU with the reference's schedule and
 * conversions. Stereo observations (obs_ur >= 0) become 3-D stereo edges in
 * GBA; LBA drops them as the reference does (its stereo branch is empty,
 * g2oOptimizer.cc:914-916). */
int sqlm_capture_replay(sqlm_ctx *ctx, const sqlm_capture *cap, const volatile uint8_t *stop,
                        sqlm_replay_out *out);

/* System::SaveTrajectoryKITTI (src/System.cc:503-560): one line per tracked
 * frame, the 3x4 [Rwc | twc] of its camera-to-world pose, "%.9f" fixed, space
 * separated, in the origin keyframe's frame. Frame f's pose is Tcr[f] (its
 * pose relative to its reference keyframe, Tracking::mlRelativeFramePoses)
 * times the reference keyframe's pose; a bad reference keyframe is replaced by
 * its parent, accumulating Tcp (KeyFrame::mTcp), as the reference does. All
 * products in float (cv::Mat CV_32F); Two = the origin keyframe's pose
 * inverse as KeyFrame::SetPose forms it ([R^T | -R^T t]).
 *   Tcr     [n_frames][16] row-major 4x4   frame_ref [n_frames] keyframe index
 *   Tcw     [n_kf][16] keyframe poses      Tcp [n_kf][16], parent [n_kf] (-1 none)
 *   bad     [n_kf] (may be NULL)           origin_kf: index of the first keyframe (lowest mnId)
 * Returns SQLM_ERR_INVALID_ARG for bad arguments or an unwritable path, or a
 * bad keyframe without a good ancestor. */
int sqlm_save_trajectory_kitti(const char *path, int n_frames, const float *Tcr, const int32_t *frame_ref, int n_kf,
                               const float *Tcw, const float *Tcp, const int32_t *parent, const uint8_t *bad,
                               int origin_kf);

#ifdef __cplusplus
}
#endif
#endif
