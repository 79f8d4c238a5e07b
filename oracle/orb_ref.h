/* TEST INFRASTRUCTURE — CPU restatement of the reference's ORB front end
 * (SURVEY.md §8 row f3): ORBextractor::operator() (src/frontend/ORBextractor.cc)
 * and ORBmatcher::DescriptorDistance / SearchForInitialization /
 * SearchByProjection (src/frontend/ORBmatcher.cc). Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg use it, as the checker.
 *
 * PARITY: the extractor calls OpenCV 3.3.1 (cv::FAST, cv::resize INTER_LINEAR,
 * cv::GaussianBlur, copyMakeBorder), which is absent here; those are restated
 * from OpenCV's documented scalar / SSE2 fixed-point formulas (see orb_ref.c),
 * with no IPP path, so the pyramid and FAST stages are "parity unpinned"
 * against the reference binary. Everything the reference implements itself
 * (cell grid, FAST thresholds fallback, quadtree distribution, IC_Angle,
 * steered BRIEF, Hamming distance, SearchForInitialization with its
 * tie-breaking, rotation histogram and ComputeThreeMaxima, GetFeaturesInArea
 * and the projection searches' acceptance rules) follows its source line for
 * line, cited per function; the projection searches are cross-checked against
 * a second, pure-Python transliteration (tests/test_orb_oracle.py). The one
 * cv::Mat product they use (3x3 * 3x1 + 3x1 in SearchByProjection(Frame,
 * Frame)) is restated from OpenCV's small-matrix gemm and is unpinned. */
#ifndef ORC_ORB_REF_H
#define ORC_ORB_REF_H
#include <stdint.h>

#define ORC_ORB_MAX_LEVELS 16

/* cv::KeyPoint fields the reference uses. */
typedef struct orc_kp {
  float x, y, size, angle, response;
  int octave;
} orc_kp;

typedef struct orc_orb_params {
  int nfeatures;      /* ORBextractor.nFeatures (cfg/KITTI00-02.yaml: 2000) */
  float scale_factor; /* 1.2 */
  int nlevels;        /* 8 */
  int ini_th_fast;    /* 20 */
  int min_th_fast;    /* 7 */
} orc_orb_params;

/* Level geometry (ORBextractor ctor :474-560, ComputePyramid :1224-1282). */
int orc_orb_levels(const orc_orb_params *p, int cols, int rows, int *lw, int *lh, int *nfeat, float *scale);
/* cv::resize(INTER_LINEAR) of an 8-bit image, OpenCV 3.3.1 fixed point. */
void orc_orb_resize(const uint8_t *src, int sw, int sh, int sstride, uint8_t *dst, int dw, int dh, int dstride);
/* cv::FAST(view, kps, th, nonmax=true) on the w x h view at img; corner
 * coordinates relative to the view, in OpenCV's emission order. */
int orc_orb_fast(const uint8_t *img, int stride, int w, int h, int th, orc_kp *out, int cap);
/* Candidates of one level (ComputeKeyPointsOctTree :1045-1135 cell loop),
 * coordinates relative to (minBorderX, minBorderY) like vToDistributeKeys. */
int orc_orb_level_candidates(const orc_orb_params *p, const uint8_t *img, int w, int h, int stride, orc_kp *out,
                             int cap);
/* ORBextractor::DistributeOctTree (:692-1043). */
int orc_orb_distribute(const orc_kp *keys, int n, int minX, int maxX, int minY, int maxY, int N, orc_kp *out);
/* cv::GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101) of an 8-bit image. */
void orc_orb_blur(const uint8_t *src, int w, int h, int sstride, uint8_t *dst, int dstride);
/* IC_Angle (:92-141) and computeOrbDescriptor (:155-206). */
float orc_orb_ic_angle(const uint8_t *img, int stride, float x, float y);
void orc_orb_describe(const uint8_t *img, int stride, const orc_kp *kp, uint8_t *desc);
/* ORBextractor::operator() (:1284-1399): keypoints (level-0 coordinates) and
 * 32-byte descriptors; returns the count (<= cap) or -1. levels_out, when
 * non-null, receives the pyramid images packed level after level. */
int orc_orb_extract(const orc_orb_params *p, const uint8_t *img, int w, int h, int stride, orc_kp *kps,
                    uint8_t *desc, int cap, uint8_t *levels_out);

/* ORBmatcher::DescriptorDistance (ORBmatcher.cc:2096-2116). */
int orc_hamming(const uint8_t *a, const uint8_t *b);

/* Frame grid (Frame.cc:1268-1285 AssignFeaturesToGrid, :1554-1565 PosInGrid,
 * :1463-1552 GetFeaturesInArea) of the second frame. */
typedef struct orc_frame_grid {
  float min_x, max_x, min_y, max_y; /* mnMinX .. mnMaxY */
} orc_frame_grid;

/* ORBmatcher(nnratio, check_ori).SearchForInitialization(F1, F2, prev, m12,
 * window) (ORBmatcher.cc:573-718). prev [n1][2] is updated in place. */
int orc_search_for_init(const orc_kp *k1, const uint8_t *d1, int n1, const orc_kp *k2, const uint8_t *d2, int n2,
                        const orc_frame_grid *g2, float *prev, int *m12, int window, float nnratio, int check_ori);
/* The Frame fields ORBmatcher's projection searches read and write
 * (include/data_structure/Frame.h): mvKeysUn, mDescriptors, mvuRight (NULL:
 * monocular, every entry < 0), the grid bounds, mvScaleFactors, the
 * intrinsics and mb / mbf, and mvpMapPoints as map-point ids (slot_mp, -1 =
 * NULL) with slot_obs = that point's Observations() > 0. Layout equal to
 * sqlm_orb_frame (include/sqrtlm_orb.h). */
typedef struct orc_frame {
  const orc_kp *kps;
  const uint8_t *desc;
  const float *uright;
  int n;
  orc_frame_grid bounds;
  const float *scale_factors;
  int n_levels;
  float fx, fy, cx, cy, bf, mb;
  int *slot_mp;
  uint8_t *slot_obs;
} orc_frame;

/* MapPoint tracking fields (MapPoint.h mnId, mTrackProjX/Y/XR, mTrackViewCos,
 * mnTrackScaleLevel, mbTrackInView, isBad(), Observations() > 0). */
typedef struct orc_track_point {
  int id;
  float proj_x, proj_y, proj_xr, view_cos;
  int level;
  uint8_t in_view, bad, has_obs, pad;
} orc_track_point;

/* One LastFrame keypoint slot: mvpMapPoints[i] (id, -1 = NULL), its world
 * position GetWorldPos(), mvKeys[i].octave, mvKeysUn[i].angle, mvbOutlier[i],
 * the point's Observations() > 0. */
typedef struct orc_last_point {
  int id;
  float x, y, z;
  int octave;
  float angle;
  uint8_t outlier, has_obs, pad[2];
} orc_last_point;

/* Frame::GetFeaturesInArea(x, y, r, minLevel, maxLevel) (Frame.cc:1463-1552)
 * over F's grid (built by AssignFeaturesToGrid, :1268-1285); writes the
 * indices in the reference's order into out (capacity F->n), returns the count. */
int orc_features_in_area(const orc_frame *F, float x, float y, float r, int min_level, int max_level, int *out);

/* ORBmatcher(nnratio).SearchByProjection(F, vpMapPoints, th)
 * (ORBmatcher.cc:67-181): F->slot_mp / slot_obs updated; returns nmatches. */
int orc_search_by_projection_local(orc_frame *F, const orc_track_point *mps, const uint8_t *mp_desc, int n_mp,
                                   float th, float nnratio);

/* ORBmatcher(., check_ori).SearchByProjection(CurrentFrame, LastFrame, th,
 * bMono) (ORBmatcher.cc:1717-1883). Tcw / Tlw: the 3x4 rows of
 * CurrentFrame.mTcw / LastFrame.mTcw (float, row-major). */
int orc_search_by_projection_last(orc_frame *F, const float *Tcw, const float *Tlw, const orc_last_point *lp,
                                  const uint8_t *ldesc, int n_last, float th, int mono, int check_ori);

/* A map point as the keyframe searches read it (MapPoint.h): mnId,
 * GetWorldPos(), GetNormal(), mfMinDistance / mfMaxDistance and the caller's
 * pre-filter (isBad(), already found / already in the keyframe). Layout equal
 * to sqlm_map_point. */
typedef struct orc_map_point {
  int id;
  float x, y, z, nx, ny, nz, min_dist, max_dist;
  uint8_t skip, pad[3];
} orc_map_point;

/* SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) (ORBmatcher.cc:423-571):
 * F = pKF (slot_mp = vpMatched, updated). Returns nmatches. */
int orc_search_by_projection_sim3(orc_frame *F, const float *Scw, const orc_map_point *mps, const uint8_t *mp_desc,
                                  int n, int th);
/* Fuse(pKF, vpMapPoints, th) (:1109-1294) and Fuse(pKF, Scw, vpPoints, th,
 * vpReplacePoint) (:1296-1446): the keypoint each point fuses into (-1: none)
 * in fuse_idx; the caller applies Replace / AddMapPoint in point order.
 * Returns nFused. sim3 = 0: T is pKF's Tcw; 1: T is Scw. */
int orc_fuse(const orc_frame *F, const float *T, int sim3, const orc_map_point *mps, const uint8_t *mp_desc, int n,
             float th, int *fuse_idx);
/* SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist)
 * (:1902-2046): F = CurrentFrame with Tcw; mps / kf_angle = pKF's slots. */
int orc_search_by_projection_kf(orc_frame *F, const float *Tcw, const orc_map_point *mps, const uint8_t *mp_desc,
                                const float *kf_angle, int n, float th, int orb_dist, int check_ori);

/* A keyframe as the BoW searches read it: mvKeysUn, mDescriptors, the node of
 * each feature in mFeatVec (DBoW2 FeatureVector; -1: not in it),
 * GetMapPointMatches() ids (-1: NULL), their isBad() (NULL: none bad),
 * mvuRight (NULL: monocular). Layout equal to sqlm_bow_frame. */
typedef struct orc_bow_frame {
  const orc_kp *kps;
  const uint8_t *desc;
  const int *node;
  const int *mp;
  const uint8_t *mp_bad;
  const float *uright;
  int n;
} orc_bow_frame;

/* SearchByBoW(pKF, F, vpMapPointMatches) (:246-403): matches [F.n] = map-point ids. */
int orc_search_by_bow_kf_frame(const orc_bow_frame *KF, const orc_bow_frame *F, float nnratio, int check_ori,
                               int *matches);
/* SearchByBoW(pKF1, pKF2, vpMatches12) (:731-869): matches12 [KF1.n] = KF2 map-point ids. */
int orc_search_by_bow_kf_kf(const orc_bow_frame *K1, const orc_bow_frame *K2, float nnratio, int check_ori,
                            int *matches12);
/* SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, bOnlyStereo)
 * (:887-1096): m12 [K1.n] = matched KF2 keypoint (-1: none); C1 = pKF1's
 * camera centre, T2w = pKF2's 3x4 pose, cam2 = fx fy cx cy, F12 row-major. */
int orc_search_for_triangulation(const orc_bow_frame *K1, const orc_bow_frame *K2, const float *C1, const float *T2w,
                                 const float *cam2, const float *scale_factors2, const float *F12, int only_stereo,
                                 int check_ori, int *m12);

/* SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th)
 * (ORBmatcher.cc:1448-1608): K1 / K2 with their 3x4 poses T1w / T2w and
 * map-point slots mp1 / mp2 (id -1: NULL; skip: isBad()); matches12 [K1.n]
 * in: vpMatches12 as ids, out: with the mutual matches added. R12 row-major. */
int orc_search_by_sim3(const orc_frame *K1, const orc_frame *K2, const float *T1w, const float *T2w,
                       const orc_map_point *mp1, const uint8_t *md1, const orc_map_point *mp2, const uint8_t *md2,
                       float s12, const float *R12, const float *t12, float th, int *matches12);
#endif
