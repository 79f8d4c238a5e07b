/* TEST INFRASTRUCTURE — CPU restatement of the reference's ORB front end
 * (SURVEY.md §8 row f3). See orb_ref.h for scope and the parity statement.
 * Built with -ffp-contract=off like the reference (-std=c++11 / c++14 is ISO
 * mode for GCC, which disables FMA contraction; CMakeLists.txt:4,44,50). */
#include "orb_ref.h"

#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "orb_pattern.h"

#define EDGE_THRESHOLD 19 /* ORBextractor.cc:78 */
#define PATCH_SIZE 31     /* :76 */
#define HALF_PATCH_SIZE 15
#define ORC_CV_PI 3.1415926535897932384626433832795 /* CV_PI */

/* OpenCV cvRound / cvFloor / cvCeil on x86-64 (SSE2 cvtss2si: round half to even). */
static int cv_round(float v) { return (int)lrintf(v); }
static int cv_roundd(double v) { return (int)lrint(v); }
static int cv_floor(float v) {
  int i = (int)v;
  return i - (i > v);
}

static int imin(int a, int b) { return a < b ? a : b; }
static int imax(int a, int b) { return a > b ? a : b; }

/* ---- level geometry (ORBextractor ctor :474-560, ComputePyramid :1224-1282) ---- */
int orc_orb_levels(const orc_orb_params *p, int cols, int rows, int *lw, int *lh, int *nfeat, float *scale) {
  const int L = p->nlevels;
  if (L < 1 || L > ORC_ORB_MAX_LEVELS) return -1;
  float sf[ORC_ORB_MAX_LEVELS];
  sf[0] = 1.0f;
  for (int i = 1; i < L; ++i) sf[i] = sf[i - 1] * p->scale_factor;
  for (int i = 0; i < L; ++i) {
    const float inv = 1.0f / sf[i];
    lw[i] = cv_round((float)cols * inv);
    lh[i] = cv_round((float)rows * inv);
    scale[i] = sf[i];
  }
  const float factor = 1.0f / p->scale_factor;
  float nd = p->nfeatures * (1 - factor) / (1 - (float)pow((double)factor, (double)L));
  int sum = 0;
  for (int l = 0; l < L - 1; ++l) {
    nfeat[l] = cv_round(nd);
    sum += nfeat[l];
    nd *= factor;
  }
  nfeat[L - 1] = imax(p->nfeatures - sum, 0);
  /* the cell grid needs at least one 30-pixel cell per axis on every level */
  for (int i = 0; i < L; ++i)
    if (lw[i] - 2 * (EDGE_THRESHOLD - 3) < 30 || lh[i] - 2 * (EDGE_THRESHOLD - 3) < 30) return -2;
  for (int i = 0; i < L; ++i) /* DistributeOctTree needs round(width / height) >= 1 */
    if ((int)roundf((float)(lw[i] - 2 * (EDGE_THRESHOLD - 3)) / (lh[i] - 2 * (EDGE_THRESHOLD - 3))) < 1) return -3;
  return 0;
}

/* ---- cv::resize INTER_LINEAR, 8U (OpenCV 3.3.1 imgproc/resize.cpp) ----
 * Coefficients: fx = (float)((dx+0.5)*scale_x - 0.5), sx = cvFloor(fx), short
 * weights saturate_cast<short>((1-fx)*2048), (fx*2048); x clamped at the
 * borders (xmax: pure copy S[sx]*2048), rows clipped. Horizontal pass in int.
 * Vertical pass: SSE2 VResizeLinearVec_32s8u for x below the vector end
 * (((S0>>4)*b0 >> 16) + ((S1>>4)*b1 >> 16) + 2) >> 2, then the scalar
 * FixedPtCast (b0*S0 + b1*S1 + 2^21) >> 22 for the tail. */
static short sat_short(float v) {
  int r = cv_round(v);
  return (short)(r < SHRT_MIN ? SHRT_MIN : r > SHRT_MAX ? SHRT_MAX : r);
}
static int sat16(int v) { return v < -32768 ? -32768 : v > 32767 ? 32767 : v; }
static uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

int orc_resize_vec_end(int width) {
  int x = 0;
  for (; x <= width - 16; x += 16) {
  }
  for (; x < width - 4; x += 4) {
  }
  return x;
}

void orc_orb_resize(const uint8_t *src, int sw, int sh, int sstride, uint8_t *dst, int dw, int dh, int dstride) {
  const double inv_sx = (double)dw / sw, inv_sy = (double)dh / sh;
  const double scale_x = 1. / inv_sx, scale_y = 1. / inv_sy;
  int *xofs = (int *)malloc(sizeof(int) * dw);
  short *ialpha = (short *)malloc(sizeof(short) * 2 * dw);
  int xmax = dw;
  for (int dx = 0; dx < dw; ++dx) {
    float fx = (float)((dx + 0.5) * scale_x - 0.5);
    int sx = cv_floor(fx);
    fx -= sx;
    if (sx < 0) fx = 0, sx = 0;
    if (sx + 1 >= sw) {
      xmax = imin(xmax, dx);
      if (sx >= sw - 1) fx = 0, sx = sw - 1;
    }
    xofs[dx] = sx;
    ialpha[2 * dx] = sat_short((1.f - fx) * 2048);
    ialpha[2 * dx + 1] = sat_short(fx * 2048);
  }
  int *r0 = (int *)malloc(sizeof(int) * dw), *r1 = (int *)malloc(sizeof(int) * dw);
  const int vend = orc_resize_vec_end(dw);
  for (int dy = 0; dy < dh; ++dy) {
    float fy = (float)((dy + 0.5) * scale_y - 0.5);
    int sy = cv_floor(fy);
    fy -= sy;
    const short b0 = sat_short((1.f - fy) * 2048), b1 = sat_short(fy * 2048);
    const int y0 = imin(imax(sy, 0), sh - 1), y1 = imin(imax(sy + 1, 0), sh - 1);
    for (int k = 0; k < 2; ++k) {
      const uint8_t *S = src + (size_t)(k ? y1 : y0) * sstride;
      int *D = k ? r1 : r0;
      for (int dx = 0; dx < dw; ++dx) {
        const int sx = xofs[dx];
        D[dx] = dx < xmax ? S[sx] * ialpha[2 * dx] + S[sx + 1] * ialpha[2 * dx + 1] : S[sx] * 2048;
      }
    }
    uint8_t *out = dst + (size_t)dy * dstride;
    for (int x = 0; x < dw; ++x) {
      if (x < vend) {
        const int a = sat16(r0[x] >> 4), c = sat16(r1[x] >> 4);
        const int m = sat16(((a * b0) >> 16) + ((c * b1) >> 16));
        out[x] = sat_u8(sat16(m + 2) >> 2);
      } else {
        out[x] = sat_u8((r0[x] * b0 + r1[x] * b1 + (1 << 21)) >> 22);
      }
    }
  }
  free(xofs);
  free(ialpha);
  free(r0);
  free(r1);
}

/* ---- cv::FAST, TYPE_9_16, nonmax suppression (OpenCV 3.3.1 features2d/fast.cpp) ---- */
static const int kFastOff[16][2] = {{0, 3},  {1, 3},  {2, 2},  {3, 1},  {3, 0},   {3, -1}, {2, -2}, {1, -3},
                                    {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

/* cornerScore<16>: the largest threshold for which the pixel stays a corner, minus one. */
static int corner_score16(const uint8_t *ptr, const int *pixel, int threshold) {
  const int K = 8, N = K * 3 + 1;
  int k, v = ptr[0];
  short d[25];
  for (k = 0; k < N; k++) d[k] = (short)(v - ptr[pixel[k]]);
  int a0 = threshold;
  for (k = 0; k < 16; k += 2) {
    int a = imin((int)d[k + 1], (int)d[k + 2]);
    a = imin(a, (int)d[k + 3]);
    if (a <= a0) continue;
    a = imin(a, (int)d[k + 4]);
    a = imin(a, (int)d[k + 5]);
    a = imin(a, (int)d[k + 6]);
    a = imin(a, (int)d[k + 7]);
    a = imin(a, (int)d[k + 8]);
    a0 = imax(a0, imin(a, (int)d[k]));
    a0 = imax(a0, imin(a, (int)d[k + 9]));
  }
  int b0 = -a0;
  for (k = 0; k < 16; k += 2) {
    int b = imax((int)d[k + 1], (int)d[k + 2]);
    b = imax(b, (int)d[k + 3]);
    b = imax(b, (int)d[k + 4]);
    b = imax(b, (int)d[k + 5]);
    if (b >= b0) continue;
    b = imax(b, (int)d[k + 6]);
    b = imax(b, (int)d[k + 7]);
    b = imax(b, (int)d[k + 8]);
    b0 = imin(b0, imax(b, (int)d[k]));
    b0 = imin(b0, imax(b, (int)d[k + 9]));
  }
  return -b0 - 1;
}

int orc_orb_fast(const uint8_t *img, int stride, int w, int h, int threshold, orc_kp *out, int cap) {
  const int K = 8, N = 16 + K + 1;
  int pixel[25];
  for (int k = 0; k < 16; ++k) pixel[k] = kFastOff[k][0] + kFastOff[k][1] * stride;
  for (int k = 16; k < 25; ++k) pixel[k] = pixel[k - 16];
  threshold = imin(imax(threshold, 0), 255);
  uint8_t tab[512];
  for (int i = -255; i <= 255; i++) tab[i + 255] = (uint8_t)(i < -threshold ? 1 : i > threshold ? 2 : 0);
  uint8_t *buf[3];
  int *cpbuf[3];
  uint8_t *bmem = (uint8_t *)calloc((size_t)3 * w + 1, 1);
  int *cmem = (int *)calloc((size_t)3 * (w + 1), sizeof(int));
  for (int b = 0; b < 3; ++b) {
    buf[b] = bmem + (size_t)b * w;
    cpbuf[b] = cmem + (size_t)b * (w + 1) + 1;
  }
  int n = 0;
  for (int i = 3; i < h - 2; i++) {
    const uint8_t *ptr = img + (size_t)i * stride + 3;
    uint8_t *curr = buf[(i - 3) % 3];
    int *cornerpos = cpbuf[(i - 3) % 3];
    memset(curr, 0, w);
    int ncorners = 0;
    if (i < h - 3) {
      for (int j = 3; j < w - 3; j++, ptr++) {
        const int v = ptr[0];
        const uint8_t *t = &tab[0] - v + 255;
        int d = t[ptr[pixel[0]]] | t[ptr[pixel[8]]];
        if (d == 0) continue;
        d &= t[ptr[pixel[2]]] | t[ptr[pixel[10]]];
        d &= t[ptr[pixel[4]]] | t[ptr[pixel[12]]];
        d &= t[ptr[pixel[6]]] | t[ptr[pixel[14]]];
        if (d == 0) continue;
        d &= t[ptr[pixel[1]]] | t[ptr[pixel[9]]];
        d &= t[ptr[pixel[3]]] | t[ptr[pixel[11]]];
        d &= t[ptr[pixel[5]]] | t[ptr[pixel[13]]];
        d &= t[ptr[pixel[7]]] | t[ptr[pixel[15]]];
        if (d & 1) {
          const int vt = v - threshold;
          int count = 0;
          for (int k = 0; k < N; k++) {
            const int x = ptr[pixel[k]];
            if (x < vt) {
              if (++count > K) {
                cornerpos[ncorners++] = j;
                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                break;
              }
            } else
              count = 0;
          }
        }
        if (d & 2) {
          const int vt = v + threshold;
          int count = 0;
          for (int k = 0; k < N; k++) {
            const int x = ptr[pixel[k]];
            if (x > vt) {
              if (++count > K) {
                cornerpos[ncorners++] = j;
                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                break;
              }
            } else
              count = 0;
          }
        }
      }
    }
    cornerpos[-1] = ncorners;
    if (i == 3) continue;
    const uint8_t *prev = buf[(i - 4 + 3) % 3];
    const uint8_t *pprev = buf[(i - 5 + 3) % 3];
    cornerpos = cpbuf[(i - 4 + 3) % 3];
    ncorners = cornerpos[-1];
    for (int k = 0; k < ncorners; k++) {
      const int j = cornerpos[k];
      const int score = prev[j];
      if (score > prev[j + 1] && score > prev[j - 1] && score > pprev[j - 1] && score > pprev[j] &&
          score > pprev[j + 1] && score > curr[j - 1] && score > curr[j] && score > curr[j + 1]) {
        if (n < cap) {
          out[n].x = (float)j;
          out[n].y = (float)(i - 1);
          out[n].size = 7.f;
          out[n].angle = -1.f;
          out[n].response = (float)score;
          out[n].octave = 0;
        }
        ++n;
      }
    }
  }
  free(bmem);
  free(cmem);
  return n;
}

/* ComputeKeyPointsOctTree cell loop (ORBextractor.cc:1045-1135): FAST with
 * iniThFAST on each 30-px cell (+6 overlap), minThFAST when the cell is empty. */
int orc_orb_level_candidates(const orc_orb_params *p, const uint8_t *img, int cols, int rows, int stride,
                             orc_kp *out, int cap) {
  const float W = 30;
  const int minBorderX = EDGE_THRESHOLD - 3, minBorderY = minBorderX;
  const int maxBorderX = cols - EDGE_THRESHOLD + 3, maxBorderY = rows - EDGE_THRESHOLD + 3;
  const float width = (float)(maxBorderX - minBorderX), height = (float)(maxBorderY - minBorderY);
  const int nCols = (int)(width / W), nRows = (int)(height / W);
  const int wCell = (int)ceilf(width / nCols), hCell = (int)ceilf(height / nRows);
  int n = 0;
  orc_kp *cell = (orc_kp *)malloc(sizeof(orc_kp) * 4096);
  for (int i = 0; i < nRows; i++) {
    const float iniY = (float)(minBorderY + i * hCell);
    float maxY = iniY + hCell + 6;
    if (iniY >= maxBorderY - 3) continue;
    if (maxY > maxBorderY) maxY = (float)maxBorderY;
    for (int j = 0; j < nCols; j++) {
      const float iniX = (float)(minBorderX + j * wCell);
      float maxX = iniX + wCell + 6;
      if (iniX >= maxBorderX - 3) continue;
      if (maxX > maxBorderX) maxX = (float)maxBorderX;
      const uint8_t *view = img + (size_t)(int)iniY * stride + (int)iniX;
      const int vw = (int)maxX - (int)iniX, vh = (int)maxY - (int)iniY;
      int c = orc_orb_fast(view, stride, vw, vh, p->ini_th_fast, cell, 4096);
      if (c == 0) c = orc_orb_fast(view, stride, vw, vh, p->min_th_fast, cell, 4096);
      if (c > 4096) c = 4096;
      for (int k = 0; k < c; ++k) {
        orc_kp kp = cell[k];
        kp.x += j * wCell;
        kp.y += i * hCell;
        if (n < cap) out[n] = kp;
        ++n;
      }
    }
  }
  free(cell);
  return n;
}

/* ---- DistributeOctTree (ORBextractor.cc:606-1043) ---- */
typedef struct onode {
  int ulx, uly, urx, ury, blx, bly, brx, bry;
  orc_kp *keys;
  int nkeys;
  int nomore;
  struct onode *prev, *next;
} onode;

typedef struct olist {
  onode *head;
  int size;
  onode **pool;
  int npool, cpool;
} olist;

static onode *onode_new(olist *L, int cap) {
  onode *n = (onode *)calloc(1, sizeof(onode));
  n->keys = (orc_kp *)malloc(sizeof(orc_kp) * (cap > 0 ? cap : 1));
  if (L->npool == L->cpool) {
    L->cpool = L->cpool ? 2 * L->cpool : 64;
    L->pool = (onode **)realloc(L->pool, sizeof(onode *) * L->cpool);
  }
  L->pool[L->npool++] = n;
  return n;
}
static void olist_push_front(olist *L, onode *n) {
  n->prev = NULL;
  n->next = L->head;
  if (L->head) L->head->prev = n;
  L->head = n;
  L->size++;
}
static onode *olist_erase(olist *L, onode *n) {
  onode *nx = n->next;
  if (n->prev) n->prev->next = nx;
  else L->head = nx;
  if (nx) nx->prev = n->prev;
  L->size--;
  return nx;
}

/* ExtractorNode::DivideNode (:606-690) */
static void divide_node(olist *L, const onode *p, onode **c) {
  const int halfX = (int)ceilf((float)(p->urx - p->ulx) / 2);
  const int halfY = (int)ceilf((float)(p->bry - p->uly) / 2);
  for (int k = 0; k < 4; ++k) c[k] = onode_new(L, p->nkeys);
  c[0]->ulx = p->ulx; c[0]->uly = p->uly;
  c[0]->urx = p->ulx + halfX; c[0]->ury = p->uly;
  c[0]->blx = p->ulx; c[0]->bly = p->uly + halfY;
  c[0]->brx = p->ulx + halfX; c[0]->bry = p->uly + halfY;
  c[1]->ulx = c[0]->urx; c[1]->uly = c[0]->ury;
  c[1]->urx = p->urx; c[1]->ury = p->ury;
  c[1]->blx = c[0]->brx; c[1]->bly = c[0]->bry;
  c[1]->brx = p->urx; c[1]->bry = p->uly + halfY;
  c[2]->ulx = c[0]->blx; c[2]->uly = c[0]->bly;
  c[2]->urx = c[0]->brx; c[2]->ury = c[0]->bry;
  c[2]->blx = p->blx; c[2]->bly = p->bly;
  c[2]->brx = c[0]->brx; c[2]->bry = p->bly;
  c[3]->ulx = c[2]->urx; c[3]->uly = c[2]->ury;
  c[3]->urx = c[1]->brx; c[3]->ury = c[1]->bry;
  c[3]->blx = c[2]->brx; c[3]->bly = c[2]->bry;
  c[3]->brx = p->brx; c[3]->bry = p->bry;
  for (int i = 0; i < p->nkeys; ++i) {
    const orc_kp *kp = &p->keys[i];
    int t;
    if (kp->x < c[0]->urx) t = kp->y < c[0]->bry ? 0 : 2;
    else t = kp->y < c[0]->bry ? 1 : 3;
    c[t]->keys[c[t]->nkeys++] = *kp;
  }
  for (int k = 0; k < 4; ++k)
    if (c[k]->nkeys == 1) c[k]->nomore = 1;
}

typedef struct {
  int size;
  onode *node;
} size_node;

/* stable ascending sort by size (std::stable_sort in :900-906) */
static void stable_sort_sizes(size_node *v, int n) {
  for (int i = 1; i < n; ++i) {
    size_node x = v[i];
    int j = i - 1;
    while (j >= 0 && v[j].size > x.size) {
      v[j + 1] = v[j];
      --j;
    }
    v[j + 1] = x;
  }
}

int orc_orb_distribute(const orc_kp *keys, int n, int minX, int maxX, int minY, int maxY, int N, orc_kp *out) {
  const int nIni = (int)roundf((float)(maxX - minX) / (maxY - minY));
  const float hX = (float)(maxX - minX) / nIni;
  olist L = {0};
  onode **ini = (onode **)malloc(sizeof(onode *) * (nIni > 0 ? nIni : 1));
  /* lNodes.push_back in order: build back to front with push_front */
  for (int i = 0; i < nIni; i++) {
    onode *ni = onode_new(&L, n);
    ni->ulx = (int)(hX * (float)i); ni->uly = 0;
    ni->urx = (int)(hX * (float)(i + 1)); ni->ury = 0;
    ni->blx = ni->ulx; ni->bly = maxY - minY;
    ni->brx = ni->urx; ni->bry = maxY - minY;
    ini[i] = ni;
  }
  for (int i = nIni - 1; i >= 0; --i) olist_push_front(&L, ini[i]);
  for (int i = 0; i < n; i++) {
    onode *t = ini[(size_t)(keys[i].x / hX)];
    t->keys[t->nkeys++] = keys[i];
  }
  for (onode *it = L.head; it;) {
    if (it->nkeys == 1) {
      it->nomore = 1;
      it = it->next;
    } else if (it->nkeys == 0) it = olist_erase(&L, it);
    else it = it->next;
  }
  int cap_sz = 1024;
  size_node *vs = (size_node *)malloc(sizeof(size_node) * cap_sz);
  size_node *vp = (size_node *)malloc(sizeof(size_node) * cap_sz);
  int nvs = 0;
#define PUSH_SZ(cnt, nd)                                                     \
  do {                                                                            \
    if (cnt == cap_sz) {                                                          \
      cap_sz *= 2;                                                                \
      vs = (size_node *)realloc(vs, sizeof(size_node) * cap_sz);                  \
      vp = (size_node *)realloc(vp, sizeof(size_node) * cap_sz);                  \
    }                                                                             \
    vs[cnt].size = (nd)->nkeys;                                                   \
    vs[cnt].node = (nd);                                                          \
    cnt++;                                                                        \
  } while (0)
  int bFinish = 0;
  while (!bFinish) {
    int prevSize = L.size;
    int nToExpand = 0;
    nvs = 0;
    for (onode *it = L.head; it;) {
      if (it->nomore) {
        it = it->next;
        continue;
      }
      onode *c[4];
      divide_node(&L, it, c);
      for (int k = 0; k < 4; ++k) {
        if (c[k]->nkeys > 0) {
          olist_push_front(&L, c[k]);
          if (c[k]->nkeys > 1) {
            nToExpand++;
            PUSH_SZ(nvs, c[k]);
          }
        }
      }
      it = olist_erase(&L, it);
    }
    if (L.size >= N || L.size == prevSize) {
      bFinish = 1;
    } else if ((L.size + nToExpand * 3) > N) {
      while (!bFinish) {
        prevSize = L.size;
        const int nprev = nvs;
        memcpy(vp, vs, sizeof(size_node) * nprev);
        nvs = 0;
        stable_sort_sizes(vp, nprev);
        for (int j = nprev - 1; j >= 0; j--) {
          onode *c[4];
          divide_node(&L, vp[j].node, c);
          for (int k = 0; k < 4; ++k) {
            if (c[k]->nkeys > 0) {
              olist_push_front(&L, c[k]);
              if (c[k]->nkeys > 1) PUSH_SZ(nvs, c[k]);
            }
          }
          olist_erase(&L, vp[j].node);
          if (L.size >= N) break;
        }
        if (L.size >= N || L.size == prevSize) bFinish = 1;
      }
    }
  }
#undef PUSH_SZ
  int nout = 0;
  for (onode *it = L.head; it; it = it->next) {
    const orc_kp *best = &it->keys[0];
    float maxResponse = best->response;
    for (int k = 1; k < it->nkeys; k++)
      if (it->keys[k].response > maxResponse) {
        best = &it->keys[k];
        maxResponse = it->keys[k].response;
      }
    out[nout++] = *best;
  }
  for (int i = 0; i < L.npool; ++i) {
    free(L.pool[i]->keys);
    free(L.pool[i]);
  }
  free(L.pool);
  free(ini);
  free(vs);
  free(vp);
  return nout;
}

/* ---- cv::GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101), 8U (OpenCV 3.3.1) ----
 * getGaussianKernel(7, 2, CV_32F): t_i = exp(-0.5/4 x_i^2) rounded to float,
 * normalised in double, rounded to float; the 8U path converts both kernels to
 * int (x256, cvRound). Row pass: exact int sums. Column pass: SSE2
 * SymmColumnVec_32s8u (float kernel k/65536, s = k0*R0; s += k_k*(R+k + R-k);
 * round half even) for x below width & ~3, scalar (s + 2^15) >> 16 after. */
void orc_orb_gauss_kernel(int ik[7]) {
  const double scale2X = -0.5 / (2.0 * 2.0);
  float cf[7];
  double sum = 0;
  for (int i = 0; i < 7; i++) {
    const double x = i - (7 - 1) * 0.5;
    const double t = exp(scale2X * x * x);
    cf[i] = (float)t;
    sum += cf[i];
  }
  sum = 1. / sum;
  for (int i = 0; i < 7; i++) {
    cf[i] = (float)(cf[i] * sum);
    ik[i] = cv_round(cf[i] * 256.0f);
  }
}

static int refl101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
  return i;
}

void orc_orb_blur(const uint8_t *src, int w, int h, int sstride, uint8_t *dst, int dstride) {
  int ik[7];
  orc_orb_gauss_kernel(ik);
  float fk[4];
  for (int k = 0; k < 4; ++k) fk[k] = (float)((double)ik[3 + k] / 65536.0);
  int *R = (int *)malloc(sizeof(int) * (size_t)w * h);
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      int s = 0;
      for (int i = 0; i < 7; ++i) s += ik[i] * src[(size_t)y * sstride + refl101(x + i - 3, w)];
      R[(size_t)y * w + x] = s;
    }
  const int vend = w & ~3;
  for (int y = 0; y < h; ++y) {
    const int *rows[7];
    for (int k = -3; k <= 3; ++k) rows[k + 3] = R + (size_t)refl101(y + k, h) * w;
    for (int x = 0; x < w; ++x) {
      int v;
      if (x < vend) {
        float s = (float)rows[3][x] * fk[0];
        s = s + 0.0f;
        for (int k = 1; k <= 3; ++k) s = s + (float)(rows[3 + k][x] + rows[3 - k][x]) * fk[k];
        v = (int)lrintf(s);
        v = sat16(v);
      } else {
        int s = ik[3] * rows[3][x];
        for (int k = 1; k <= 3; ++k) s += ik[3 + k] * (rows[3 + k][x] + rows[3 - k][x]);
        v = (s + (1 << 15)) >> 16;
      }
      dst[(size_t)y * dstride + x] = sat_u8(v);
    }
  }
  free(R);
}

/* ---- IC_Angle (:92-141) with OpenCV's fastAtan2 (core/mathfuncs_core) ---- */
static void orb_umax(int umax[HALF_PATCH_SIZE + 1]) {
  int v, v0, vmax = (int)floorf(HALF_PATCH_SIZE * sqrtf(2.f) / 2 + 1);
  int vmin = (int)ceilf(HALF_PATCH_SIZE * sqrtf(2.f) / 2);
  const double hp2 = HALF_PATCH_SIZE * HALF_PATCH_SIZE;
  for (v = 0; v <= vmax; ++v) umax[v] = cv_roundd(sqrt(hp2 - v * v));
  for (v = HALF_PATCH_SIZE, v0 = 0; v >= vmin; --v) {
    while (umax[v0] == umax[v0 + 1]) ++v0;
    umax[v] = v0;
    ++v0;
  }
}

float orc_fast_atan2(float y, float x) {
  const float p1 = 0.9997878412794807f * (float)(180 / ORC_CV_PI);
  const float p3 = -0.3258083974640975f * (float)(180 / ORC_CV_PI);
  const float p5 = 0.1555786518463281f * (float)(180 / ORC_CV_PI);
  const float p7 = -0.04432655554792128f * (float)(180 / ORC_CV_PI);
  const float ax = fabsf(x), ay = fabsf(y);
  float a, c, c2;
  if (ax >= ay) {
    c = ay / (ax + (float)2.2204460492503131e-16);
    c2 = c * c;
    a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  } else {
    c = ax / (ay + (float)2.2204460492503131e-16);
    c2 = c * c;
    a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  }
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

float orc_orb_ic_angle(const uint8_t *image, int step, float px, float py) {
  int umax[HALF_PATCH_SIZE + 1];
  orb_umax(umax);
  int m_01 = 0, m_10 = 0;
  const uint8_t *center = image + (size_t)cv_round(py) * step + cv_round(px);
  for (int u = -HALF_PATCH_SIZE; u <= HALF_PATCH_SIZE; ++u) m_10 += u * center[u];
  for (int v = 1; v <= HALF_PATCH_SIZE; ++v) {
    int v_sum = 0;
    const int d = umax[v];
    for (int u = -d; u <= d; ++u) {
      const int val_plus = center[u + v * step], val_minus = center[u - v * step];
      v_sum += (val_plus - val_minus);
      m_10 += u * (val_plus + val_minus);
    }
    m_01 += v * v_sum;
  }
  return orc_fast_atan2((float)m_01, (float)m_10);
}

/* computeOrbDescriptor (:155-206). cos / sin: the double functions rounded to
 * float (the correctly rounded cosf/sinf; the reference's glibc cosf agrees
 * except where its < 1 ulp error bound is not correctly rounded). */
void orc_orb_describe(const uint8_t *img, int step, const orc_kp *kpt, uint8_t *desc) {
  const float factorPI = (float)(ORC_CV_PI / 180.f);
  const float angle = (float)kpt->angle * factorPI;
  const float a = (float)cos((double)angle), b = (float)sin((double)angle);
  const uint8_t *center = img + (size_t)cv_round(kpt->y) * step + cv_round(kpt->x);
  const signed char *pattern = kOrbPattern;
#define GET_VALUE(idx)                                                                                        \
  center[cv_round((float)pattern[2 * (idx)] * b + (float)pattern[2 * (idx) + 1] * a) * step +               \
         cv_round((float)pattern[2 * (idx)] * a - (float)pattern[2 * (idx) + 1] * b)]
  for (int i = 0; i < 32; ++i, pattern += 32) {
    int val = 0;
    for (int bit = 0; bit < 8; ++bit) {
      const int t0 = GET_VALUE(2 * bit), t1 = GET_VALUE(2 * bit + 1);
      val |= (t0 < t1) << bit;
    }
    desc[i] = (uint8_t)val;
  }
#undef GET_VALUE
}

/* ---- ORBextractor::operator() (:1284-1399) ---- */
int orc_orb_extract(const orc_orb_params *p, const uint8_t *img, int w, int h, int stride, orc_kp *kps,
                    uint8_t *desc, int cap, uint8_t *levels_out) {
  int lw[ORC_ORB_MAX_LEVELS], lh[ORC_ORB_MAX_LEVELS], nf[ORC_ORB_MAX_LEVELS];
  float sc[ORC_ORB_MAX_LEVELS];
  if (orc_orb_levels(p, w, h, lw, lh, nf, sc)) return -1;
  const int L = p->nlevels;
  uint8_t *lev[ORC_ORB_MAX_LEVELS];
  for (int l = 0; l < L; ++l) {
    lev[l] = (uint8_t *)malloc((size_t)lw[l] * lh[l]);
    if (l == 0)
      for (int y = 0; y < h; ++y) memcpy(lev[0] + (size_t)y * w, img + (size_t)y * stride, w);
    else
      orc_orb_resize(lev[l - 1], lw[l - 1], lh[l - 1], lw[l - 1], lev[l], lw[l], lh[l], lw[l]);
  }
  int umax[HALF_PATCH_SIZE + 1];
  orb_umax(umax);
  (void)umax;
  int total = 0;
  const int border = EDGE_THRESHOLD - 3;
  orc_kp *cand = (orc_kp *)malloc(sizeof(orc_kp) * 200000);
  orc_kp *sel = (orc_kp *)malloc(sizeof(orc_kp) * 200000);
  uint8_t *blur = (uint8_t *)malloc((size_t)w * h);
  for (int l = 0; l < L; ++l) {
    int nc = orc_orb_level_candidates(p, lev[l], lw[l], lh[l], lw[l], cand, 200000);
    if (nc > 200000) nc = 200000;
    const int ns = orc_orb_distribute(cand, nc, border, lw[l] - EDGE_THRESHOLD + 3, border,
                                      lh[l] - EDGE_THRESHOLD + 3, nf[l], sel);
    const int scaledPatchSize = (int)(PATCH_SIZE * sc[l]);
    for (int i = 0; i < ns; ++i) {
      sel[i].x += border;
      sel[i].y += border;
      sel[i].octave = l;
      sel[i].size = (float)scaledPatchSize;
      sel[i].angle = orc_orb_ic_angle(lev[l], lw[l], sel[i].x, sel[i].y);
    }
    if (ns > 0) orc_orb_blur(lev[l], lw[l], lh[l], lw[l], blur, lw[l]);
    for (int i = 0; i < ns; ++i) {
      if (total + i < cap) orc_orb_describe(blur, lw[l], &sel[i], desc + (size_t)32 * (total + i));
      if (l != 0) {
        sel[i].x *= sc[l];
        sel[i].y *= sc[l];
      }
      if (total + i < cap) kps[total + i] = sel[i];
    }
    total += ns;
  }
  if (levels_out) {
    size_t off = 0;
    for (int l = 0; l < L; ++l) {
      memcpy(levels_out + off, lev[l], (size_t)lw[l] * lh[l]);
      off += (size_t)lw[l] * lh[l];
    }
  }
  for (int l = 0; l < L; ++l) free(lev[l]);
  free(cand);
  free(sel);
  free(blur);
  return total;
}

/* ---- ORBmatcher ---- */
int orc_hamming(const uint8_t *a8, const uint8_t *b8) {
  int dist = 0;
  for (int i = 0; i < 8; i++) {
    uint32_t pa, pb;
    memcpy(&pa, a8 + 4 * i, 4);
    memcpy(&pb, b8 + 4 * i, 4);
    unsigned int v = pa ^ pb;
    v = v - ((v >> 1) & 0x55555555);
    v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
    dist += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
  }
  return dist;
}

#define GRID_COLS 64
#define GRID_ROWS 48
#define HISTO_LENGTH 30
#define TH_LOW 50

/* PosInGrid (Frame.cc:1554-1565): std::round of float. */
static int pos_in_grid(const orc_frame_grid *g, const orc_kp *kp, int *px, int *py) {
  const float wi = (float)GRID_COLS / (g->max_x - g->min_x), hi = (float)GRID_ROWS / (g->max_y - g->min_y);
  *px = (int)roundf((kp->x - g->min_x) * wi);
  *py = (int)roundf((kp->y - g->min_y) * hi);
  return !(*px < 0 || *px >= GRID_COLS || *py < 0 || *py >= GRID_ROWS);
}

int orc_search_for_init(const orc_kp *k1, const uint8_t *d1, int n1, const orc_kp *k2, const uint8_t *d2, int n2,
                        const orc_frame_grid *g2, float *prev, int *m12, int window, float nnratio, int check_ori) {
  /* AssignFeaturesToGrid (Frame.cc:1268-1285): cell lists in keypoint order */
  int *cnt = (int *)calloc(GRID_COLS * GRID_ROWS + 1, sizeof(int));
  int *cell = (int *)malloc(sizeof(int) * (n2 > 0 ? n2 : 1));
  for (int i = 0; i < n2; ++i) {
    int px, py;
    cell[i] = pos_in_grid(g2, &k2[i], &px, &py) ? px * GRID_ROWS + py : -1;
    if (cell[i] >= 0) cnt[cell[i] + 1]++;
  }
  for (int c = 0; c < GRID_COLS * GRID_ROWS; ++c) cnt[c + 1] += cnt[c];
  int *fill = (int *)malloc(sizeof(int) * (GRID_COLS * GRID_ROWS));
  memcpy(fill, cnt, sizeof(int) * GRID_COLS * GRID_ROWS);
  int *lst = (int *)malloc(sizeof(int) * (n2 > 0 ? n2 : 1));
  for (int i = 0; i < n2; ++i)
    if (cell[i] >= 0) lst[fill[cell[i]]++] = i;
  const float wi = (float)GRID_COLS / (g2->max_x - g2->min_x), hi = (float)GRID_ROWS / (g2->max_y - g2->min_y);

  int nmatches = 0;
  for (int i = 0; i < n1; ++i) m12[i] = -1;
  int *rot = (int *)malloc(sizeof(int) * (n1 > 0 ? n1 : 1));
  int *rotbin = (int *)malloc(sizeof(int) * (n1 > 0 ? n1 : 1));
  int hist[HISTO_LENGTH] = {0};
  int nrot = 0;
  const float factor = HISTO_LENGTH / 360.0f;
  int *vMatchedDistance = (int *)malloc(sizeof(int) * (n2 > 0 ? n2 : 1));
  int *vnMatches21 = (int *)malloc(sizeof(int) * (n2 > 0 ? n2 : 1));
  for (int i = 0; i < n2; ++i) {
    vMatchedDistance[i] = INT_MAX;
    vnMatches21[i] = -1;
  }
  for (int i1 = 0; i1 < n1; i1++) {
    const int level1 = k1[i1].octave;
    if (level1 > 0) continue;
    /* GetFeaturesInArea(prev.x, prev.y, window, level1, level1) (Frame.cc:1463-1552) */
    const float x = prev[2 * i1], y = prev[2 * i1 + 1], r = (float)window;
    const int nMinCellX = imax(0, (int)floorf((x - g2->min_x - r) * wi));
    if (nMinCellX >= GRID_COLS) continue;
    const int nMaxCellX = imin(GRID_COLS - 1, (int)ceilf((x - g2->min_x + r) * wi));
    if (nMaxCellX < 0) continue;
    const int nMinCellY = imax(0, (int)floorf((y - g2->min_y - r) * hi));
    if (nMinCellY >= GRID_ROWS) continue;
    const int nMaxCellY = imin(GRID_ROWS - 1, (int)ceilf((y - g2->min_y + r) * hi));
    if (nMaxCellY < 0) continue;
    const int bCheckLevels = (level1 > 0) || (level1 >= 0);
    int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1, any = 0;
    for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
      for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
        const int c = ix * GRID_ROWS + iy;
        for (int q = cnt[c]; q < cnt[c + 1]; ++q) {
          const int i2 = lst[q];
          const orc_kp *kpUn = &k2[i2];
          if (bCheckLevels) {
            if (kpUn->octave < level1) continue;
            if (level1 >= 0 && kpUn->octave > level1) continue;
          }
          const float distx = kpUn->x - x, disty = kpUn->y - y;
          if (!(fabsf(distx) < r && fabsf(disty) < r)) continue;
          any = 1;
          /* ORBmatcher.cc:620-641 */
          const int dist = orc_hamming(d1 + 32 * (size_t)i1, d2 + 32 * (size_t)i2);
          if (vMatchedDistance[i2] <= dist) continue;
          if (dist < bestDist) {
            bestDist2 = bestDist;
            bestDist = dist;
            bestIdx2 = i2;
          } else if (dist < bestDist2) {
            bestDist2 = dist;
          }
        }
      }
    if (!any) continue;
    if (bestDist <= TH_LOW) {
      if (bestDist < (float)bestDist2 * nnratio) {
        if (vnMatches21[bestIdx2] >= 0) {
          m12[vnMatches21[bestIdx2]] = -1;
          nmatches--;
        }
        m12[i1] = bestIdx2;
        vnMatches21[bestIdx2] = i1;
        vMatchedDistance[bestIdx2] = bestDist;
        nmatches++;
        if (check_ori) {
          float rr = k1[i1].angle - k2[bestIdx2].angle;
          if (rr < 0.0) rr += 360.0f;
          int bin = (int)roundf(rr * factor);
          if (bin == HISTO_LENGTH) bin = 0;
          rot[nrot] = i1;
          rotbin[nrot] = bin;
          nrot++;
          hist[bin]++;
        }
      }
    }
  }
  if (check_ori) {
    /* ComputeThreeMaxima (ORBmatcher.cc:2048-2090) */
    int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
    for (int i = 0; i < HISTO_LENGTH; i++) {
      const int s = hist[i];
      if (s > max1) {
        max3 = max2; max2 = max1; max1 = s;
        ind3 = ind2; ind2 = ind1; ind1 = i;
      } else if (s > max2) {
        max3 = max2; max2 = s;
        ind3 = ind2; ind2 = i;
      } else if (s > max3) {
        max3 = s;
        ind3 = i;
      }
    }
    if (max2 < 0.1f * (float)max1) {
      ind2 = -1;
      ind3 = -1;
    } else if (max3 < 0.1f * (float)max1) {
      ind3 = -1;
    }
    for (int q = 0; q < nrot; ++q) {
      const int b = rotbin[q];
      if (b == ind1 || b == ind2 || b == ind3) continue;
      if (m12[rot[q]] >= 0) {
        m12[rot[q]] = -1;
        nmatches--;
      }
    }
  }
  for (int i1 = 0; i1 < n1; i1++)
    if (m12[i1] >= 0) {
      prev[2 * i1] = k2[m12[i1]].x;
      prev[2 * i1 + 1] = k2[m12[i1]].y;
    }
  free(cnt); free(cell); free(fill); free(lst); free(rot); free(rotbin); free(vMatchedDistance); free(vnMatches21);
  return nmatches;
}

/* ---- projection searches (SearchByProjection overloads) ---- */
typedef struct {
  int *cnt, *lst; /* cell CSR (cell = ix * GRID_ROWS + iy), keypoint order inside a cell */
  float wi, hi;   /* mfGridElementWidthInv / HeightInv */
} orc_grid;

/* Frame::AssignFeaturesToGrid (Frame.cc:1268-1285). */
static void grid_build(const orc_frame *F, orc_grid *G) {
  const int n = F->n;
  G->cnt = (int *)calloc(GRID_COLS * GRID_ROWS + 1, sizeof(int));
  G->lst = (int *)malloc(sizeof(int) * (n > 0 ? n : 1));
  int *cell = (int *)malloc(sizeof(int) * (n > 0 ? n : 1));
  for (int i = 0; i < n; ++i) {
    int px, py;
    cell[i] = pos_in_grid(&F->bounds, &F->kps[i], &px, &py) ? px * GRID_ROWS + py : -1;
    if (cell[i] >= 0) G->cnt[cell[i] + 1]++;
  }
  for (int c = 0; c < GRID_COLS * GRID_ROWS; ++c) G->cnt[c + 1] += G->cnt[c];
  int *fill = (int *)malloc(sizeof(int) * GRID_COLS * GRID_ROWS);
  memcpy(fill, G->cnt, sizeof(int) * GRID_COLS * GRID_ROWS);
  for (int i = 0; i < n; ++i)
    if (cell[i] >= 0) G->lst[fill[cell[i]]++] = i;
  G->wi = (float)GRID_COLS / (F->bounds.max_x - F->bounds.min_x);
  G->hi = (float)GRID_ROWS / (F->bounds.max_y - F->bounds.min_y);
  free(cell);
  free(fill);
}

static void grid_free(orc_grid *G) {
  free(G->cnt);
  free(G->lst);
}

/* Frame::GetFeaturesInArea (Frame.cc:1463-1552), bCheckLevels as written. */
static int area(const orc_frame *F, const orc_grid *G, float x, float y, float r, int minLevel, int maxLevel,
                int *out) {
  const orc_frame_grid *g = &F->bounds;
  const int nMinCellX = imax(0, (int)floorf((x - g->min_x - r) * G->wi));
  if (nMinCellX >= GRID_COLS) return 0;
  const int nMaxCellX = imin(GRID_COLS - 1, (int)ceilf((x - g->min_x + r) * G->wi));
  if (nMaxCellX < 0) return 0;
  const int nMinCellY = imax(0, (int)floorf((y - g->min_y - r) * G->hi));
  if (nMinCellY >= GRID_ROWS) return 0;
  const int nMaxCellY = imin(GRID_ROWS - 1, (int)ceilf((y - g->min_y + r) * G->hi));
  if (nMaxCellY < 0) return 0;
  const int bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
  int n = 0;
  for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
    for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
      const int c = ix * GRID_ROWS + iy;
      for (int q = G->cnt[c]; q < G->cnt[c + 1]; ++q) {
        const orc_kp *kpUn = &F->kps[G->lst[q]];
        if (bCheckLevels) {
          if (kpUn->octave < minLevel) continue;
          if (maxLevel >= 0)
            if (kpUn->octave > maxLevel) continue;
        }
        const float distx = kpUn->x - x, disty = kpUn->y - y;
        if (fabsf(distx) < r && fabsf(disty) < r) out[n++] = G->lst[q];
      }
    }
  return n;
}

int orc_features_in_area(const orc_frame *F, float x, float y, float r, int min_level, int max_level, int *out) {
  orc_grid G;
  grid_build(F, &G);
  const int n = area(F, &G, x, y, r, min_level, max_level, out);
  grid_free(&G);
  return n;
}

#define TH_HIGH 100

/* ORBmatcher::RadiusByViewingCos (ORBmatcher.cc:183-190). */
static float radius_by_viewing_cos(float viewCos) { return viewCos > 0.998 ? 2.5f : 4.0f; }

int orc_search_by_projection_local(orc_frame *F, const orc_track_point *mps, const uint8_t *mp_desc, int n_mp,
                                   float th, float nnratio) {
  orc_grid G;
  grid_build(F, &G);
  int *vIndices = (int *)malloc(sizeof(int) * (F->n > 0 ? F->n : 1));
  int nmatches = 0;
  const int bFactor = th != 1.0;
  for (int iMP = 0; iMP < n_mp; iMP++) {
    const orc_track_point *pMP = &mps[iMP];
    if (!pMP->in_view) continue; /* :78-83 */
    if (pMP->bad) continue;
    const int nPredictedLevel = pMP->level;
    float r = radius_by_viewing_cos(pMP->view_cos);
    if (bFactor) r *= th;
    const float scale = F->scale_factors[nPredictedLevel];
    const int nI = area(F, &G, pMP->proj_x, pMP->proj_y, r * scale, nPredictedLevel - 1, nPredictedLevel, vIndices);
    if (nI == 0) continue;
    int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
    for (int v = 0; v < nI; ++v) { /* :118-155 */
      const int idx = vIndices[v];
      if (F->slot_mp[idx] >= 0)
        if (F->slot_obs[idx]) continue;
      if (F->uright && F->uright[idx] > 0) {
        const float er = fabsf(pMP->proj_xr - F->uright[idx]);
        if (er > r * scale) continue;
      }
      const int dist = orc_hamming(mp_desc + 32 * (size_t)iMP, F->desc + 32 * (size_t)idx);
      if (dist < bestDist) {
        bestDist2 = bestDist;
        bestDist = dist;
        bestLevel2 = bestLevel;
        bestLevel = F->kps[idx].octave;
        bestIdx = idx;
      } else if (dist < bestDist2) {
        bestLevel2 = F->kps[idx].octave;
        bestDist2 = dist;
      }
    }
    if (bestDist <= TH_HIGH) { /* :160-175 */
      if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;
      F->slot_mp[bestIdx] = pMP->id;
      F->slot_obs[bestIdx] = pMP->has_obs;
      nmatches++;
    }
  }
  free(vIndices);
  grid_free(&G);
  return nmatches;
}

/* cv::Mat 3x3 * 3x1 (+ 3x1) on CV_32F, OpenCV's small-matrix gemm path: float
 * products summed left to right, then alpha * t + beta * c in double — with
 * alpha = beta = 1 that is one float addition. OpenCV is absent here, so this
 * step is "parity unpinned" like the extractor's OpenCV stages. */
static void mat3_mul_add(const float *T, int transpose, const float *x, const float *c, float sign, float *out) {
  for (int i = 0; i < 3; ++i) {
    const float a0 = transpose ? T[0 * 4 + i] : T[i * 4 + 0];
    const float a1 = transpose ? T[1 * 4 + i] : T[i * 4 + 1];
    const float a2 = transpose ? T[2 * 4 + i] : T[i * 4 + 2];
    const float t0 = a0 * x[0] + a1 * x[1] + a2 * x[2];
    out[i] = c ? (float)((double)t0 * sign + (double)c[i]) : (float)((double)t0 * sign);
  }
}

/* ComputeThreeMaxima (ORBmatcher.cc:2048-2090) over bin sizes. */
static void three_maxima(const int *hist, int *i1, int *i2, int *i3) {
  int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
  for (int i = 0; i < HISTO_LENGTH; i++) {
    const int s = hist[i];
    if (s > max1) {
      max3 = max2; max2 = max1; max1 = s;
      ind3 = ind2; ind2 = ind1; ind1 = i;
    } else if (s > max2) {
      max3 = max2; max2 = s;
      ind3 = ind2; ind2 = i;
    } else if (s > max3) {
      max3 = s;
      ind3 = i;
    }
  }
  if (max2 < 0.1f * (float)max1) {
    ind2 = -1;
    ind3 = -1;
  } else if (max3 < 0.1f * (float)max1) {
    ind3 = -1;
  }
  *i1 = ind1;
  *i2 = ind2;
  *i3 = ind3;
}

int orc_search_by_projection_last(orc_frame *F, const float *Tcw, const float *Tlw, const orc_last_point *lp,
                                  const uint8_t *ldesc, int n_last, float th, int mono, int check_ori) {
  orc_grid G;
  grid_build(F, &G);
  int *vIndices2 = (int *)malloc(sizeof(int) * (F->n > 0 ? F->n : 1));
  /* rotHist[bin] lists in push order: (bin, slot) records, replayed per bin */
  int *rot_bin = (int *)malloc(sizeof(int) * (n_last > 0 ? n_last : 1));
  int *rot_idx = (int *)malloc(sizeof(int) * (n_last > 0 ? n_last : 1));
  int nrot = 0, hist[HISTO_LENGTH] = {0};
  const float factor = HISTO_LENGTH / 360.0f;
  int nmatches = 0;
  const float tcw[3] = {Tcw[3], Tcw[7], Tcw[11]}, tlw[3] = {Tlw[3], Tlw[7], Tlw[11]};
  float twc[3], tlc[3];
  mat3_mul_add(Tcw, 1, tcw, NULL, -1.0f, twc); /* twc = -Rcw.t()*tcw (:1730) */
  mat3_mul_add(Tlw, 0, twc, tlw, 1.0f, tlc);   /* tlc = Rlw*twc+tlw (:1735) */
  const int bForward = tlc[2] > F->mb && !mono;
  const int bBackward = -tlc[2] > F->mb && !mono;
  for (int i = 0; i < n_last; i++) {
    const orc_last_point *pMP = &lp[i];
    if (pMP->id < 0 || pMP->outlier) continue;
    const float x3Dw[3] = {pMP->x, pMP->y, pMP->z};
    float x3Dc[3];
    mat3_mul_add(Tcw, 0, x3Dw, tcw, 1.0f, x3Dc);
    const float xc = x3Dc[0], yc = x3Dc[1];
    const float invzc = (float)(1.0 / (double)x3Dc[2]);
    if (invzc < 0) continue;
    const float u = F->fx * xc * invzc + F->cx, v = F->fy * yc * invzc + F->cy;
    if (u < F->bounds.min_x || u > F->bounds.max_x) continue;
    if (v < F->bounds.min_y || v > F->bounds.max_y) continue;
    const int nLastOctave = pMP->octave;
    const float radius = th * F->scale_factors[nLastOctave];
    int nI;
    if (bForward)
      nI = area(F, &G, u, v, radius, nLastOctave, -1, vIndices2);
    else if (bBackward)
      nI = area(F, &G, u, v, radius, 0, nLastOctave, vIndices2);
    else
      nI = area(F, &G, u, v, radius, nLastOctave - 1, nLastOctave + 1, vIndices2);
    if (nI == 0) continue;
    int bestDist = 256, bestIdx2 = -1;
    for (int q = 0; q < nI; ++q) { /* :1806-1836 */
      const int i2 = vIndices2[q];
      if (F->slot_mp[i2] >= 0)
        if (F->slot_obs[i2]) continue;
      if (F->uright && F->uright[i2] > 0) {
        const float ur = u - F->bf * invzc;
        const float er = fabsf(ur - F->uright[i2]);
        if (er > radius) continue;
      }
      const int dist = orc_hamming(ldesc + 32 * (size_t)i, F->desc + 32 * (size_t)i2);
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx2 = i2;
      }
    }
    if (bestDist <= TH_HIGH) { /* :1839-1858 */
      F->slot_mp[bestIdx2] = pMP->id;
      F->slot_obs[bestIdx2] = pMP->has_obs;
      nmatches++;
      if (check_ori) {
        float rot = pMP->angle - F->kps[bestIdx2].angle;
        if (rot < 0.0) rot += 360.0f;
        int bin = (int)roundf(rot * factor);
        if (bin == HISTO_LENGTH) bin = 0;
        rot_bin[nrot] = bin;
        rot_idx[nrot++] = bestIdx2;
        hist[bin]++;
      }
    }
  }
  if (check_ori) { /* :1862-1880: every entry of a rejected bin is cleared */
    int ind1, ind2, ind3;
    three_maxima(hist, &ind1, &ind2, &ind3);
    for (int b = 0; b < HISTO_LENGTH; b++) {
      if (b == ind1 || b == ind2 || b == ind3) continue;
      for (int q = 0; q < nrot; ++q)
        if (rot_bin[q] == b) {
          F->slot_mp[rot_idx[q]] = -1;
          F->slot_obs[rot_idx[q]] = 0;
          nmatches--;
        }
    }
  }
  free(vIndices2);
  free(rot_bin);
  free(rot_idx);
  grid_free(&G);
  return nmatches;
}

/* ---- keyframe projection searches ---- */
typedef struct {
  float T[12];  /* [R | t], rows */
  float Ow[3];  /* -R^T t */
} orc_pose;

static void pose_finish(orc_pose *P) {
  const float t[3] = {P->T[3], P->T[7], P->T[11]};
  mat3_mul_add(P->T, 1, t, NULL, -1.0f, P->Ow);
}

/* pKF->GetRotation() / GetTranslation() / GetCameraCenter() of a 3x4 Tcw. */
static void pose_from_T(const float *T, orc_pose *P) {
  memcpy(P->T, T, sizeof(float) * 12);
  pose_finish(P);
}

/* Scw -> s = sqrt(row0 . row0) (Mat::dot in double), R = sR / s, t = t / s
 * (Mat / double: a float scale by (float)(1 / s)) — ORBmatcher.cc:434-441;
 * OpenCV's convertTo scaling, "parity unpinned" with the other cv::Mat steps. */
static void pose_from_sim3(const float *S, orc_pose *P) {
  const double d = (double)S[0] * S[0] + (double)S[1] * S[1] + (double)S[2] * S[2];
  const float scw = (float)sqrt(d);
  const float inv = (float)(1.0 / (double)scw);
  for (int i = 0; i < 12; ++i) P->T[i] = S[i] * inv;
  pose_finish(P);
}

/* cv::norm of a 3x1 CV_32F (double sum of squares, sqrt) and Mat::dot (double). */
static float norm3(const float *v) {
  double s = 0;
  for (int i = 0; i < 3; ++i) s += (double)v[i] * v[i];
  return (float)sqrt(s);
}
static double dot3(const float *a, const float *b) {
  double s = 0;
  for (int i = 0; i < 3; ++i) s += (double)a[i] * b[i];
  return s;
}

/* MapPoint::PredictScale (MapPoint.cc:610-650). */
static int predict_scale(float max_dist, float dist, float log_scale, int n_levels) {
  const float ratio = max_dist / dist;
  int nScale = (int)ceilf(logf(ratio) / log_scale);
  if (nScale < 0)
    nScale = 0;
  else if (nScale >= n_levels)
    nScale = n_levels - 1;
  return nScale;
}

/* The keyframe-side projection of ORBmatcher.cc:447-489 / :1132-1180 /
 * :1327-1372: camera point, z >= 0, (u, v) = (fx x/z + cx, ...) inside
 * IsInImage, distance invariance band, viewing angle within 60 degrees,
 * predicted level. Returns 0 when the point is rejected. */
static int project_kf(const orc_frame *F, const orc_pose *P, const orc_map_point *p, float *u, float *v, float *invz,
                      int *level) {
  const float X[3] = {p->x, p->y, p->z}, t[3] = {P->T[3], P->T[7], P->T[11]};
  float Xc[3];
  mat3_mul_add(P->T, 0, X, t, 1.0f, Xc);
  if (Xc[2] < 0.0f) return 0;
  *invz = 1 / Xc[2];
  const float x = Xc[0] * *invz, y = Xc[1] * *invz;
  *u = F->fx * x + F->cx;
  *v = F->fy * y + F->cy;
  if (!(*u >= F->bounds.min_x && *u < F->bounds.max_x && *v >= F->bounds.min_y && *v < F->bounds.max_y)) return 0;
  const float maxDistance = 1.2f * p->max_dist, minDistance = 0.8f * p->min_dist;
  const float PO[3] = {X[0] - P->Ow[0], X[1] - P->Ow[1], X[2] - P->Ow[2]};
  const float dist = norm3(PO);
  if (dist < minDistance || dist > maxDistance) return 0;
  const float Pn[3] = {p->nx, p->ny, p->nz};
  if (dot3(PO, Pn) < 0.5 * dist) return 0;
  *level = predict_scale(p->max_dist, dist, logf(F->scale_factors[1]), F->n_levels);
  return 1;
}

int orc_search_by_projection_sim3(orc_frame *F, const float *Scw, const orc_map_point *mps, const uint8_t *mp_desc,
                                  int n, int th) {
  orc_grid G;
  grid_build(F, &G);
  orc_pose P;
  pose_from_sim3(Scw, &P);
  int *vIndices = (int *)malloc(sizeof(int) * (F->n > 0 ? F->n : 1));
  int nmatches = 0;
  for (int iMP = 0; iMP < n; iMP++) {
    const orc_map_point *p = &mps[iMP];
    if (p->skip) continue;
    float u, v, invz;
    int pl;
    if (!project_kf(F, &P, p, &u, &v, &invz, &pl)) continue;
    const float radius = th * F->scale_factors[pl];
    /* KeyFrame::GetFeaturesInArea (KeyFrame.cc:809-853) + the level test of :518-520 */
    const int nI = area(F, &G, u, v, radius, pl - 1, pl, vIndices);
    int bestDist = 256, bestIdx = -1;
    for (int q = 0; q < nI; ++q) {
      const int idx = vIndices[q];
      if (F->slot_mp[idx] >= 0) continue;
      const int dist = orc_hamming(mp_desc + 32 * (size_t)iMP, F->desc + 32 * (size_t)idx);
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx = idx;
      }
    }
    if (bestDist <= TH_LOW) {
      F->slot_mp[bestIdx] = p->id;
      nmatches++;
    }
  }
  free(vIndices);
  grid_free(&G);
  return nmatches;
}

int orc_fuse(const orc_frame *F, const float *T, int sim3, const orc_map_point *mps, const uint8_t *mp_desc, int n,
             float th, int *fuse_idx) {
  orc_grid G;
  grid_build(F, &G);
  orc_pose P;
  if (sim3)
    pose_from_sim3(T, &P);
  else
    pose_from_T(T, &P);
  int *vIndices = (int *)malloc(sizeof(int) * (F->n > 0 ? F->n : 1));
  int nFused = 0;
  for (int i = 0; i < n; i++) {
    fuse_idx[i] = -1;
    const orc_map_point *p = &mps[i];
    if (p->skip) continue;
    float u, v, invz;
    int pl;
    if (!project_kf(F, &P, p, &u, &v, &invz, &pl)) continue;
    const float ur = u - F->bf * invz;
    const float radius = th * F->scale_factors[pl];
    const int nI = area(F, &G, u, v, radius, pl - 1, pl, vIndices);
    int bestDist = sim3 ? INT_MAX : 256, bestIdx = -1;
    for (int q = 0; q < nI; ++q) {
      const int idx = vIndices[q];
      const orc_kp *kp = &F->kps[idx];
      const int kpLevel = kp->octave;
      if (!sim3) { /* :1209-1237: reprojection gate, 3 dof (stereo) or 2 dof */
        const float s2 = F->scale_factors[kpLevel] * F->scale_factors[kpLevel];
        const float inv_s2 = 1.0f / s2;
        if (F->uright && F->uright[idx] >= 0) {
          const float ex = u - kp->x, ey = v - kp->y, er = ur - F->uright[idx];
          const float e2 = ex * ex + ey * ey + er * er;
          if (e2 * inv_s2 > 7.8) continue;
        } else {
          const float ex = u - kp->x, ey = v - kp->y;
          const float e2 = ex * ex + ey * ey;
          if (e2 * inv_s2 > 5.99) continue;
        }
      }
      const int dist = orc_hamming(mp_desc + 32 * (size_t)i, F->desc + 32 * (size_t)idx);
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx = idx;
      }
    }
    if (bestDist <= TH_LOW) {
      fuse_idx[i] = bestIdx;
      nFused++;
    }
  }
  free(vIndices);
  grid_free(&G);
  return nFused;
}

int orc_search_by_projection_kf(orc_frame *F, const float *Tcw, const orc_map_point *mps, const uint8_t *mp_desc,
                                const float *kf_angle, int n, float th, int orb_dist, int check_ori) {
  orc_grid G;
  grid_build(F, &G);
  orc_pose P;
  pose_from_T(Tcw, &P);
  int *vIndices2 = (int *)malloc(sizeof(int) * (F->n > 0 ? F->n : 1));
  int *rot_bin = (int *)malloc(sizeof(int) * (n > 0 ? n : 1));
  int *rot_idx = (int *)malloc(sizeof(int) * (n > 0 ? n : 1));
  int nrot = 0, hist[HISTO_LENGTH] = {0}, nmatches = 0;
  const float factor = HISTO_LENGTH / 360.0f;
  const float t[3] = {P.T[3], P.T[7], P.T[11]};
  for (int i = 0; i < n; i++) {
    const orc_map_point *p = &mps[i];
    if (p->skip) continue;
    const float X[3] = {p->x, p->y, p->z};
    float Xc[3];
    mat3_mul_add(P.T, 0, X, t, 1.0f, Xc);
    const float xc = Xc[0], yc = Xc[1];
    const float invzc = (float)(1.0 / (double)Xc[2]);
    const float u = F->fx * xc * invzc + F->cx, v = F->fy * yc * invzc + F->cy;
    if (u < F->bounds.min_x || u > F->bounds.max_x) continue;
    if (v < F->bounds.min_y || v > F->bounds.max_y) continue;
    const float PO[3] = {X[0] - P.Ow[0], X[1] - P.Ow[1], X[2] - P.Ow[2]};
    const float dist3D = norm3(PO);
    const float maxDistance = 1.2f * p->max_dist, minDistance = 0.8f * p->min_dist;
    if (dist3D < minDistance || dist3D > maxDistance) continue;
    const int pl = predict_scale(p->max_dist, dist3D, logf(F->scale_factors[1]), F->n_levels);
    const float radius = th * F->scale_factors[pl];
    const int nI = area(F, &G, u, v, radius, pl - 1, pl + 1, vIndices2);
    int bestDist = 256, bestIdx2 = -1;
    for (int q = 0; q < nI; ++q) {
      const int i2 = vIndices2[q];
      if (F->slot_mp[i2] >= 0) continue;
      const int dist = orc_hamming(mp_desc + 32 * (size_t)i, F->desc + 32 * (size_t)i2);
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx2 = i2;
      }
    }
    if (bestDist <= orb_dist) {
      F->slot_mp[bestIdx2] = p->id;
      nmatches++;
      if (check_ori) {
        float rot = kf_angle[i] - F->kps[bestIdx2].angle;
        if (rot < 0.0) rot += 360.0f;
        int bin = (int)roundf(rot * factor);
        if (bin == HISTO_LENGTH) bin = 0;
        rot_bin[nrot] = bin;
        rot_idx[nrot++] = bestIdx2;
        hist[bin]++;
      }
    }
  }
  if (check_ori) {
    int ind1, ind2, ind3;
    three_maxima(hist, &ind1, &ind2, &ind3);
    for (int b = 0; b < HISTO_LENGTH; b++) {
      if (b == ind1 || b == ind2 || b == ind3) continue;
      for (int q = 0; q < nrot; ++q)
        if (rot_bin[q] == b) {
          F->slot_mp[rot_idx[q]] = -1;
          nmatches--;
        }
    }
  }
  free(vIndices2);
  free(rot_bin);
  free(rot_idx);
  grid_free(&G);
  return nmatches;
}

/* ---- BoW searches: DBoW2 FeatureVector (std::map<NodeId, vector<unsigned>>,
 * features pushed in index order) as node-sorted index runs ---- */
typedef struct {
  int *idx; /* feature indices sorted by (node, index) */
  int n;    /* features present */
} orc_featvec;

static const int *g_sort_node;
static int cmp_node_idx(const void *a, const void *b) {
  const int ia = *(const int *)a, ib = *(const int *)b;
  if (g_sort_node[ia] != g_sort_node[ib]) return g_sort_node[ia] < g_sort_node[ib] ? -1 : 1;
  return ia < ib ? -1 : ia > ib;
}

static void featvec_build(const orc_bow_frame *K, orc_featvec *V) {
  V->idx = (int *)malloc(sizeof(int) * (K->n > 0 ? K->n : 1));
  V->n = 0;
  for (int i = 0; i < K->n; ++i)
    if (K->node[i] >= 0) V->idx[V->n++] = i;
  g_sort_node = K->node;
  qsort(V->idx, V->n, sizeof(int), cmp_node_idx);
}

/* The common nodes in increasing order (the KFit / Fit merge with lower_bound,
 * ORBmatcher.cc:280-382): calls visit(node run of side 1, node run of side 2). */
typedef void (*orc_node_visit)(void *ctx, const int *r1, int n1, const int *r2, int n2);
static void featvec_merge(const orc_bow_frame *K1, const orc_featvec *V1, const orc_bow_frame *K2,
                          const orc_featvec *V2, orc_node_visit visit, void *ctx) {
  int a = 0, b = 0;
  while (a < V1->n && b < V2->n) {
    const int na = K1->node[V1->idx[a]], nb = K2->node[V2->idx[b]];
    if (na == nb) {
      int ea = a, eb = b;
      while (ea < V1->n && K1->node[V1->idx[ea]] == na) ea++;
      while (eb < V2->n && K2->node[V2->idx[eb]] == nb) eb++;
      visit(ctx, V1->idx + a, ea - a, V2->idx + b, eb - b);
      a = ea;
      b = eb;
    } else if (na < nb) {
      while (a < V1->n && K1->node[V1->idx[a]] < nb) a++;
    } else {
      while (b < V2->n && K2->node[V2->idx[b]] < na) b++;
    }
  }
}

typedef struct {
  const orc_bow_frame *K1, *K2;
  float nnratio;
  int check_ori, nmatches, nrot, hist[HISTO_LENGTH];
  int *out, *rot_bin, *rot_idx;
  uint8_t *matched2;
  /* SearchForTriangulation */
  float ex, ey;
  const float *F12, *sf2;
  int only_stereo;
} orc_bow_ctx;

static void rot_push(orc_bow_ctx *c, float a1, float a2, int idx) {
  const float factor = HISTO_LENGTH / 360.0f;
  float rot = a1 - a2;
  if (rot < 0.0) rot += 360.0f;
  int bin = (int)roundf(rot * factor);
  if (bin == HISTO_LENGTH) bin = 0;
  c->rot_bin[c->nrot] = bin;
  c->rot_idx[c->nrot++] = idx;
  c->hist[bin]++;
}

/* the rejected bins' entries, bin by bin (ORBmatcher.cc:384-400 and alike);
 * clear(ctx, idx) undoes one match. */
static void rot_reject(orc_bow_ctx *c, void (*clear)(orc_bow_ctx *, int)) {
  int ind1, ind2, ind3;
  three_maxima(c->hist, &ind1, &ind2, &ind3);
  for (int b = 0; b < HISTO_LENGTH; b++) {
    if (b == ind1 || b == ind2 || b == ind3) continue;
    for (int q = 0; q < c->nrot; ++q)
      if (c->rot_bin[q] == b) {
        clear(c, c->rot_idx[q]);
        c->nmatches--;
      }
  }
}

static void visit_kf_frame(void *vc, const int *r1, int n1, const int *r2, int n2) {
  orc_bow_ctx *c = (orc_bow_ctx *)vc;
  for (int i = 0; i < n1; ++i) { /* :296-362 */
    const int realIdxKF = r1[i];
    if (c->K1->mp[realIdxKF] < 0) continue;
    if (c->K1->mp_bad && c->K1->mp_bad[realIdxKF]) continue;
    int bestDist1 = 256, bestIdxF = -1, bestDist2 = 256;
    for (int j = 0; j < n2; ++j) {
      const int realIdxF = r2[j];
      if (c->out[realIdxF] >= 0) continue;
      const int dist = orc_hamming(c->K1->desc + 32 * (size_t)realIdxKF, c->K2->desc + 32 * (size_t)realIdxF);
      if (dist < bestDist1) {
        bestDist2 = bestDist1;
        bestDist1 = dist;
        bestIdxF = realIdxF;
      } else if (dist < bestDist2) {
        bestDist2 = dist;
      }
    }
    if (bestDist1 <= TH_LOW) {
      if ((float)bestDist1 < c->nnratio * (float)bestDist2) {
        c->out[bestIdxF] = c->K1->mp[realIdxKF];
        if (c->check_ori) rot_push(c, c->K1->kps[realIdxKF].angle, c->K2->kps[bestIdxF].angle, bestIdxF);
        c->nmatches++;
      }
    }
  }
}

static void clear_out(orc_bow_ctx *c, int idx) { c->out[idx] = -1; }

int orc_search_by_bow_kf_frame(const orc_bow_frame *KF, const orc_bow_frame *F, float nnratio, int check_ori,
                               int *matches) {
  orc_bow_ctx c;
  memset(&c, 0, sizeof(c));
  c.K1 = KF;
  c.K2 = F;
  c.nnratio = nnratio;
  c.check_ori = check_ori;
  c.out = matches;
  for (int i = 0; i < F->n; ++i) matches[i] = -1;
  c.rot_bin = (int *)malloc(sizeof(int) * (KF->n > 0 ? KF->n : 1));
  c.rot_idx = (int *)malloc(sizeof(int) * (KF->n > 0 ? KF->n : 1));
  orc_featvec V1, V2;
  featvec_build(KF, &V1);
  featvec_build(F, &V2);
  featvec_merge(KF, &V1, F, &V2, visit_kf_frame, &c);
  if (check_ori) rot_reject(&c, clear_out);
  free(V1.idx);
  free(V2.idx);
  free(c.rot_bin);
  free(c.rot_idx);
  return c.nmatches;
}

static void visit_kf_kf(void *vc, const int *r1, int n1, const int *r2, int n2) {
  orc_bow_ctx *c = (orc_bow_ctx *)vc;
  for (int i = 0; i < n1; ++i) { /* :775-845 */
    const int idx1 = r1[i];
    if (c->K1->mp[idx1] < 0) continue;
    if (c->K1->mp_bad && c->K1->mp_bad[idx1]) continue;
    int bestDist1 = 256, bestIdx2 = -1, bestDist2 = 256;
    for (int j = 0; j < n2; ++j) {
      const int idx2 = r2[j];
      if (c->matched2[idx2] || c->K2->mp[idx2] < 0) continue;
      if (c->K2->mp_bad && c->K2->mp_bad[idx2]) continue;
      const int dist = orc_hamming(c->K1->desc + 32 * (size_t)idx1, c->K2->desc + 32 * (size_t)idx2);
      if (dist < bestDist1) {
        bestDist2 = bestDist1;
        bestDist1 = dist;
        bestIdx2 = idx2;
      } else if (dist < bestDist2) {
        bestDist2 = dist;
      }
    }
    if (bestDist1 < TH_LOW) {
      if ((float)bestDist1 < c->nnratio * (float)bestDist2) {
        c->out[idx1] = c->K2->mp[bestIdx2];
        c->matched2[bestIdx2] = 1;
        if (c->check_ori) rot_push(c, c->K1->kps[idx1].angle, c->K2->kps[bestIdx2].angle, idx1);
        c->nmatches++;
      }
    }
  }
}

int orc_search_by_bow_kf_kf(const orc_bow_frame *K1, const orc_bow_frame *K2, float nnratio, int check_ori,
                            int *matches12) {
  orc_bow_ctx c;
  memset(&c, 0, sizeof(c));
  c.K1 = K1;
  c.K2 = K2;
  c.nnratio = nnratio;
  c.check_ori = check_ori;
  c.out = matches12;
  for (int i = 0; i < K1->n; ++i) matches12[i] = -1;
  c.matched2 = (uint8_t *)calloc(K2->n > 0 ? K2->n : 1, 1);
  c.rot_bin = (int *)malloc(sizeof(int) * (K1->n > 0 ? K1->n : 1));
  c.rot_idx = (int *)malloc(sizeof(int) * (K1->n > 0 ? K1->n : 1));
  orc_featvec V1, V2;
  featvec_build(K1, &V1);
  featvec_build(K2, &V2);
  featvec_merge(K1, &V1, K2, &V2, visit_kf_kf, &c);
  if (check_ori) rot_reject(&c, clear_out); /* vbMatched2 is not reset (:855-866) */
  free(V1.idx);
  free(V2.idx);
  free(c.matched2);
  free(c.rot_bin);
  free(c.rot_idx);
  return c.nmatches;
}

/* CheckDistEpipolarLine (ORBmatcher.cc:203-229). */
static int check_epipolar(const orc_kp *kp1, const orc_kp *kp2, const float *F, const float *sf2) {
  const float a = kp1->x * F[0] + kp1->y * F[3] + F[6];
  const float b = kp1->x * F[1] + kp1->y * F[4] + F[7];
  const float c = kp1->x * F[2] + kp1->y * F[5] + F[8];
  const float num = a * kp2->x + b * kp2->y + c;
  const float den = a * a + b * b;
  if (den == 0) return 0;
  const float dsqr = num * num / den;
  const float sigma2 = sf2[kp2->octave] * sf2[kp2->octave];
  return dsqr < 3.84 * sigma2;
}

static void visit_triangulation(void *vc, const int *r1, int n1, const int *r2, int n2) {
  orc_bow_ctx *c = (orc_bow_ctx *)vc;
  for (int i = 0; i < n1; ++i) { /* :936-1030 */
    const int idx1 = r1[i];
    if (c->K1->mp[idx1] >= 0) continue;
    const int bStereo1 = c->K1->uright && c->K1->uright[idx1] >= 0;
    if (c->only_stereo && !bStereo1) continue;
    const orc_kp *kp1 = &c->K1->kps[idx1];
    int bestDist = TH_LOW, bestIdx2 = -1;
    for (int j = 0; j < n2; ++j) {
      const int idx2 = r2[j];
      if (c->matched2[idx2] || c->K2->mp[idx2] >= 0) continue;
      const int bStereo2 = c->K2->uright && c->K2->uright[idx2] >= 0;
      if (c->only_stereo && !bStereo2) continue;
      const int dist = orc_hamming(c->K1->desc + 32 * (size_t)idx1, c->K2->desc + 32 * (size_t)idx2);
      if (dist > TH_LOW || dist > bestDist) continue;
      const orc_kp *kp2 = &c->K2->kps[idx2];
      if (!bStereo1 && !bStereo2) {
        const float distex = c->ex - kp2->x, distey = c->ey - kp2->y;
        if (distex * distex + distey * distey < 100 * c->sf2[kp2->octave]) continue;
      }
      if (check_epipolar(kp1, kp2, c->F12, c->sf2)) {
        bestIdx2 = idx2;
        bestDist = dist;
      }
    }
    if (bestIdx2 >= 0) {
      c->out[idx1] = bestIdx2;
      c->matched2[bestIdx2] = 1;
      c->nmatches++;
      if (c->check_ori) rot_push(c, kp1->angle, c->K2->kps[bestIdx2].angle, idx1);
    }
  }
}

static void clear_tri(orc_bow_ctx *c, int idx1) {
  c->matched2[c->out[idx1]] = 0; /* :1073 */
  c->out[idx1] = -1;
}

int orc_search_for_triangulation(const orc_bow_frame *K1, const orc_bow_frame *K2, const float *C1, const float *T2w,
                                 const float *cam2, const float *scale_factors2, const float *F12, int only_stereo,
                                 int check_ori, int *m12) {
  orc_bow_ctx c;
  memset(&c, 0, sizeof(c));
  c.K1 = K1;
  c.K2 = K2;
  c.check_ori = check_ori;
  c.out = m12;
  c.F12 = F12;
  c.sf2 = scale_factors2;
  c.only_stereo = only_stereo;
  for (int i = 0; i < K1->n; ++i) m12[i] = -1;
  /* epipole: C2 = R2w * Cw + t2w, (ex, ey) (:903-913) */
  const float t2[3] = {T2w[3], T2w[7], T2w[11]};
  float C2[3];
  mat3_mul_add(T2w, 0, C1, t2, 1.0f, C2);
  const float invz = 1.0f / C2[2];
  c.ex = cam2[0] * C2[0] * invz + cam2[2];
  c.ey = cam2[1] * C2[1] * invz + cam2[3];
  c.matched2 = (uint8_t *)calloc(K2->n > 0 ? K2->n : 1, 1);
  c.rot_bin = (int *)malloc(sizeof(int) * (K1->n > 0 ? K1->n : 1));
  c.rot_idx = (int *)malloc(sizeof(int) * (K1->n > 0 ? K1->n : 1));
  orc_featvec V1, V2;
  featvec_build(K1, &V1);
  featvec_build(K2, &V2);
  featvec_merge(K1, &V1, K2, &V2, visit_triangulation, &c);
  if (check_ori) rot_reject(&c, clear_tri);
  free(V1.idx);
  free(V2.idx);
  free(c.matched2);
  free(c.rot_bin);
  free(c.rot_idx);
  return c.nmatches;
}

/* ---- SearchBySim3 (ORBmatcher.cc:1448-1608) ---- */
/* One direction: points of `src` (in src's camera via Tsw, then by [sR | t]
 * into dst's camera) searched in dst (fx.. of pKF1 for both, :1455-1458). */
static void sim3_direction(const orc_frame *cam, const orc_frame *dst, const float *Tsw, const float *sR,
                           const float *t, const orc_map_point *mp, const uint8_t *md, int n, const uint8_t *already,
                           float th, int *vnMatch) {
  orc_grid G;
  grid_build(dst, &G);
  int *vIndices = (int *)malloc(sizeof(int) * (dst->n > 0 ? dst->n : 1));
  const float ts[3] = {Tsw[3], Tsw[7], Tsw[11]};
  float sRT[12];
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c) sRT[r * 4 + c] = sR[r * 3 + c];
    sRT[r * 4 + 3] = 0.f;
  }
  for (int i = 0; i < n; i++) {
    vnMatch[i] = -1;
    const orc_map_point *p = &mp[i];
    if (p->id < 0 || already[i] || p->skip) continue;
    const float X[3] = {p->x, p->y, p->z};
    float Xs[3], Xd[3];
    mat3_mul_add(Tsw, 0, X, ts, 1.0f, Xs);
    mat3_mul_add(sRT, 0, Xs, t, 1.0f, Xd);
    if (Xd[2] < 0.0) continue;
    const float invz = (float)(1.0 / (double)Xd[2]);
    const float x = Xd[0] * invz, y = Xd[1] * invz;
    const float u = cam->fx * x + cam->cx, v = cam->fy * y + cam->cy;
    if (!(u >= dst->bounds.min_x && u < dst->bounds.max_x && v >= dst->bounds.min_y && v < dst->bounds.max_y))
      continue;
    const float maxDistance = 1.2f * p->max_dist, minDistance = 0.8f * p->min_dist;
    const float dist3D = norm3(Xd);
    if (dist3D < minDistance || dist3D > maxDistance) continue;
    const int pl = predict_scale(p->max_dist, dist3D, logf(dst->scale_factors[1]), dst->n_levels);
    const float radius = th * dst->scale_factors[pl];
    const int nI = area(dst, &G, u, v, radius, pl - 1, pl, vIndices);
    int bestDist = INT_MAX, bestIdx = -1;
    for (int q = 0; q < nI; ++q) {
      const int idx = vIndices[q];
      const int dist = orc_hamming(md + 32 * (size_t)i, dst->desc + 32 * (size_t)idx);
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx = idx;
      }
    }
    if (bestDist <= TH_HIGH) vnMatch[i] = bestIdx;
  }
  free(vIndices);
  grid_free(&G);
}

int orc_search_by_sim3(const orc_frame *K1, const orc_frame *K2, const float *T1w, const float *T2w,
                       const orc_map_point *mp1, const uint8_t *md1, const orc_map_point *mp2, const uint8_t *md2,
                       float s12, const float *R12, const float *t12, float th, int *matches12) {
  const int N1 = K1->n, N2 = K2->n;
  /* sR12 = s12 * R12, sR21 = (1 / s12) * R12^T, t21 = -sR21 * t12 (:1466-1469) */
  float sR12[9], sR21[9], t21[3];
  const float inv_s = (float)(1.0 / (double)s12);
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      sR12[r * 3 + c] = R12[r * 3 + c] * s12;
      sR21[r * 3 + c] = R12[c * 3 + r] * inv_s;
    }
  {
    float sR21T[12];
    for (int r = 0; r < 3; ++r) {
      for (int c = 0; c < 3; ++c) sR21T[r * 4 + c] = sR21[r * 3 + c];
      sR21T[r * 4 + 3] = 0.f;
    }
    mat3_mul_add(sR21T, 0, t12, NULL, -1.0f, t21);
  }
  /* vbAlreadyMatched1 / 2 (:1480-1494): pMP->GetIndexInKeyFrame(pKF2) is the
   * slot of pKF2 holding the same point */
  uint8_t *am1 = (uint8_t *)calloc(N1 > 0 ? N1 : 1, 1), *am2 = (uint8_t *)calloc(N2 > 0 ? N2 : 1, 1);
  for (int i = 0; i < N1; i++)
    if (matches12[i] >= 0) {
      am1[i] = 1;
      for (int j = 0; j < N2; ++j)
        if (mp2[j].id == matches12[i]) am2[j] = 1;
    }
  int *vnMatch1 = (int *)malloc(sizeof(int) * (N1 > 0 ? N1 : 1));
  int *vnMatch2 = (int *)malloc(sizeof(int) * (N2 > 0 ? N2 : 1));
  sim3_direction(K1, K2, T1w, sR21, t21, mp1, md1, N1, am1, th, vnMatch1);
  sim3_direction(K1, K1, T2w, sR12, t12, mp2, md2, N2, am2, th, vnMatch2);
  int nFound = 0;
  for (int i1 = 0; i1 < N1; i1++) { /* :1592-1606 */
    const int idx2 = vnMatch1[i1];
    if (idx2 >= 0 && vnMatch2[idx2] == i1) {
      matches12[i1] = mp2[idx2].id;
      nFound++;
    }
  }
  free(am1);
  free(am2);
  free(vnMatch1);
  free(vnMatch2);
  return nFound;
}
