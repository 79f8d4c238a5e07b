/* TEST INFRASTRUCTURE — CPU restatement of the reference's ORB front end
 * (SURVEY.md §8 row f3): ORBextractor::operator() (src/frontend/ORBextractor.cc)
 * and ORBmatcher::DescriptorDistance / SearchForInitialization
 * (src/frontend/ORBmatcher.cc). Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg use it, as the checker.
 *
 * PARITY: the extractor calls OpenCV 3.3.1 (cv::FAST, cv::resize INTER_LINEAR,
 * cv::GaussianBlur, copyMakeBorder), which is absent here; those are restated
 * from OpenCV's documented scalar / SSE2 fixed-point formulas (see orb_ref.c),
 * with no IPP path, so the pyramid and FAST stages are "parity unpinned"
 * against the reference binary. Everything the reference implements itself
 * (cell grid, FAST thresholds fallback, quadtree distribution, IC_Angle,
 * steered BRIEF, Hamming distance, SearchForInitialization with its
 * tie-breaking, rotation histogram and ComputeThreeMaxima) follows its source
 * line for line, cited per function. */
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
#endif
