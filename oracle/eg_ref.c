/*
 * eg_ref.c — TEST INFRASTRUCTURE (oracle). CPU restatement of the reference's
 * essential-graph optimisation (g2oOptimizer::OptimizeEssentialGraph,
 * src/backend/g2oOptimizer.cc:1212-1534): VertexSim3Expmap vertices
 * (Thirdparty/g2o/g2o/types/types_seven_dof_expmap.h:48-94), EdgeSim3 edges
 * (:99-122) with g2o's numeric Jacobians (core/base_binary_edge.hpp:131-205),
 * BlockSolver_7_3 without landmarks and the Levenberg-Marquardt loop of
 * optimization_algorithm_levenberg.cpp:61-189. Sim3 algebra follows
 * types/sim3.h. Only tests/ use this; PARITY UNPINNED (see oracle.h).
 */
#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"
#include "se3_ref.h"
#include "sqlm_libm.h" /* exp / log / sin / cos / acos, the same bits as the GPU (include/) */
#ifdef ORC_GLIBC_LIBM
/* liboracle_glibc.so: the platform libm instead, i.e. the arithmetic the
 * reference's g2o (sim3.h through std::sin / cos / exp / log / acos) runs on
 * -- pins the shared-libm oracle and the GPU to the reference's own libm
 * (tests/test_eg_oracle.py, tests/test_eg_gpu.py) */
#define sqlm_exp exp
#define sqlm_log log
#define sqlm_sin sin
#define sqlm_cos cos
#define sqlm_acos acos
#endif
#include "skyline_ref.h"

/* ------------------------------------------------------------ Sim3 (sim3.h) */

/* S = [qx qy qz qw tx ty tz s] */

static inline void skew3(const double w[3], double O[9]) {
  O[0] = 0.0;   O[1] = -w[2]; O[2] = w[1];
  O[3] = w[2];  O[4] = 0.0;   O[5] = -w[0];
  O[6] = -w[1]; O[7] = w[0];  O[8] = 0.0;
}

/* se3_ops.h:40-47 */
static inline void delta_r(const double R[9], double v[3]) {
  v[0] = R[7] - R[5];
  v[1] = R[2] - R[6];
  v[2] = R[3] - R[1];
}

/* Eigen Vector3d::norm(): sqrt of the pairwise-reduced squared norm. */
static inline double norm3(const double w[3]) { return sqrt((w[0] * w[0] + w[1] * w[1]) + w[2] * w[2]); }

/* Sim3(const Vector7d& update) (sim3.h:61-139). */
void orc_sim3_from_update(const double u[7], double S[8]) {
  const double omega[3] = {u[0], u[1], u[2]}, ups[3] = {u[3], u[4], u[5]}, sigma = u[6];
  const double theta = norm3(omega);
  double O[9], O2[9], R[9];
  skew3(omega, O);
  const double s = sqlm_exp(sigma);
  o3_matmul(O, O, O2);
  const double eps = 0.00001;
  double A, B, C;
  if (fabs(sigma) < eps) {
    C = 1;
    if (theta < eps) {
      A = 1. / 2.;
      B = 1. / 6.;
      for (int k = 0; k < 9; ++k) R[k] = ((k % 4 == 0 ? 1.0 : 0.0) + O[k]) + O2[k];
    } else {
      const double theta2 = theta * theta;
      A = (1 - sqlm_cos(theta)) / (theta2);
      B = (theta - sqlm_sin(theta)) / (theta2 * theta);
      const double a = sqlm_sin(theta) / theta, b = (1 - sqlm_cos(theta)) / (theta * theta);
      for (int k = 0; k < 9; ++k) R[k] = ((k % 4 == 0 ? 1.0 : 0.0) + a * O[k]) + b * O2[k];
    }
  } else {
    C = (s - 1) / sigma;
    if (theta < eps) {
      const double sigma2 = sigma * sigma;
      A = ((sigma - 1) * s + 1) / sigma2;
      B = ((0.5 * sigma2 - sigma + 1) * s) / (sigma2 * sigma);
      for (int k = 0; k < 9; ++k) R[k] = ((k % 4 == 0 ? 1.0 : 0.0) + O[k]) + O2[k];
    } else {
      const double ra = sqlm_sin(theta) / theta, rb = (1 - sqlm_cos(theta)) / (theta * theta);
      for (int k = 0; k < 9; ++k) R[k] = ((k % 4 == 0 ? 1.0 : 0.0) + ra * O[k]) + rb * O2[k];
      const double a = s * sqlm_sin(theta), b = s * sqlm_cos(theta);
      const double theta2 = theta * theta, sigma2 = sigma * sigma, c = theta2 + sigma2;
      A = (a * sigma + (1 - b) * theta) / (theta * c);
      B = (C - ((b - 1) * sigma + a * theta) / (c)) * 1. / (theta2);
    }
  }
  oq_from_mat(R, S);
  double W[9];
  for (int k = 0; k < 9; ++k) W[k] = (A * O[k] + B * O2[k]) + C * (k % 4 == 0 ? 1.0 : 0.0);
  for (int r = 0; r < 3; ++r) S[4 + r] = (W[3 * r] * ups[0] + W[3 * r + 1] * ups[1]) + W[3 * r + 2] * ups[2];
  S[7] = s;
}

/* W.lu().solve(t): Eigen PartialPivLU (unblocked, first maximum as pivot). */
static void lu_solve3(const double Win[9], const double b[3], double x[3]) {
  double a[9];
  int perm[3] = {0, 1, 2};
  memcpy(a, Win, sizeof(a));
  for (int k = 0; k < 3; ++k) {
    int piv = k;
    double big = fabs(a[3 * k + k]);
    for (int i = k + 1; i < 3; ++i)
      if (fabs(a[3 * i + k]) > big) { big = fabs(a[3 * i + k]); piv = i; }
    if (big != 0.0) {
      if (piv != k) {
        for (int c = 0; c < 3; ++c) { double t = a[3 * k + c]; a[3 * k + c] = a[3 * piv + c]; a[3 * piv + c] = t; }
        int t = perm[k]; perm[k] = perm[piv]; perm[piv] = t;
      }
      for (int i = k + 1; i < 3; ++i) a[3 * i + k] /= a[3 * k + k];
    }
    for (int i = k + 1; i < 3; ++i)
      for (int c = k + 1; c < 3; ++c) a[3 * i + c] -= a[3 * i + k] * a[3 * k + c];
  }
  double y[3];
  for (int i = 0; i < 3; ++i) {
    double v = b[perm[i]];
    for (int j = 0; j < i; ++j) v -= a[3 * i + j] * y[j];
    y[i] = v;
  }
  for (int i = 2; i >= 0; --i) {
    double v = y[i];
    for (int j = i + 1; j < 3; ++j) v -= a[3 * i + j] * x[j];
    x[i] = v / a[3 * i + i];
  }
}

/* Sim3::log (sim3.h:147-237). */
void orc_libm(int fn, const double *x, double *y, int n) {
  for (int i = 0; i < n; ++i)
    y[i] = fn == 0 ? sqlm_exp(x[i]) : fn == 1 ? sqlm_log(x[i]) : fn == 2 ? sqlm_sin(x[i])
         : fn == 3 ? sqlm_cos(x[i]) : sqlm_acos(x[i]);
}

void orc_sim3_log(const double S[8], double out[7]) {
  const double s = S[7];
  const double sigma = sqlm_log(s);
  double R[9], omega[3], O[9], dr[3];
  oq_to_mat(S, R);
  const double d = 0.5 * (R[0] + R[4] + R[8] - 1);
  const double eps = 0.00001;
  double A, B, C;
  delta_r(R, dr);
  if (fabs(sigma) < eps) {
    C = 1;
    if (d > 1 - eps) {
      for (int k = 0; k < 3; ++k) omega[k] = 0.5 * dr[k];
      A = 1. / 2.;
      B = 1. / 6.;
    } else {
      const double theta = sqlm_acos(d), theta2 = theta * theta;
      const double f = theta / (2 * sqrt(1 - d * d));
      for (int k = 0; k < 3; ++k) omega[k] = f * dr[k];
      A = (1 - sqlm_cos(theta)) / (theta2);
      B = (theta - sqlm_sin(theta)) / (theta2 * theta);
    }
  } else {
    C = (s - 1) / sigma;
    if (d > 1 - eps) {
      const double sigma2 = sigma * sigma;
      for (int k = 0; k < 3; ++k) omega[k] = 0.5 * dr[k];
      A = ((sigma - 1) * s + 1) / (sigma2);
      B = ((0.5 * sigma2 - sigma + 1) * s) / (sigma2 * sigma);
    } else {
      const double theta = sqlm_acos(d);
      const double f = theta / (2 * sqrt(1 - d * d));
      for (int k = 0; k < 3; ++k) omega[k] = f * dr[k];
      const double theta2 = theta * theta;
      const double a = s * sqlm_sin(theta), b = s * sqlm_cos(theta);
      const double c = theta2 + sigma * sigma;
      A = (a * sigma + (1 - b) * theta) / (theta * c);
      B = (C - ((b - 1) * sigma + a * theta) / (c)) * 1. / (theta2);
    }
  }
  skew3(omega, O);
  double O2[9], W[9];
  o3_matmul(O, O, O2);
  for (int k = 0; k < 9; ++k) W[k] = (A * O[k] + B * O2[k]) + C * (k % 4 == 0 ? 1.0 : 0.0);
  double ups[3];
  lu_solve3(W, S + 4, ups);
  for (int k = 0; k < 3; ++k) { out[k] = omega[k]; out[3 + k] = ups[k]; }
  out[6] = sigma;
}

/* Sim3::operator* (sim3.h:266-272). */
void orc_sim3_mul(const double a[8], const double b[8], double o[8]) {
  double q[4], rt[3];
  oq_mul(a, b, q);
  oq_rotate(a, b + 4, rt);
  o[4] = a[7] * rt[0] + a[4];
  o[5] = a[7] * rt[1] + a[5];
  o[6] = a[7] * rt[2] + a[6];
  o[7] = a[7] * b[7];
  memcpy(o, q, sizeof(q));
}

/* Sim3::inverse (sim3.h:239-242). */
void orc_sim3_inverse(const double a[8], double o[8]) {
  const double qc[4] = {-a[0], -a[1], -a[2], a[3]};
  const double k = -1. / a[7];
  const double v[3] = {k * a[4], k * a[5], k * a[6]};
  oq_rotate(qc, v, o + 4);
  memcpy(o, qc, sizeof(qc));
  o[7] = 1. / a[7];
}

/* VertexSim3Expmap::oplusImpl (types_seven_dof_expmap.h:60-66): S <- Sim3(u) * S,
 * the scale component of u zeroed when the scale is fixed. */
static void sim3_oplus(double S[8], const double upd[7], int fix_scale) {
  double u[7], E[8], o[8];
  memcpy(u, upd, sizeof(u));
  if (fix_scale) u[6] = 0;
  orc_sim3_from_update(u, E);
  orc_sim3_mul(E, S, o);
  memcpy(S, o, sizeof(o));
}

/* EdgeSim3::computeError (types_seven_dof_expmap.h:106-114): log(C * Si * Sj^-1). */
void orc_eg_edge_error(const double Si[8], const double Sj[8], const double C[8], double e[7]) {
  double a[8], b[8], jinv[8];
  orc_sim3_mul(C, Si, a);
  orc_sim3_inverse(Sj, jinv);
  orc_sim3_mul(a, jinv, b);
  orc_sim3_log(b, e);
}

/* BaseBinaryEdge::linearizeOplus, numeric (base_binary_edge.hpp:131-205):
 * central differences with delta = 1e-9 through oplus; Ji (d e / d Si) and Jj
 * column-major as g2o fills them column by column, stored row-major [7][7]. */
void orc_eg_edge_jacobians(const double Si[8], const double Sj[8], const double C[8], int fix_scale, int free_i,
                           int free_j, double Ji[49], double Jj[49]) {
  const double delta = 1e-9, scalar = 1.0 / (2 * delta);
  for (int side = 0; side < 2; ++side) {
    if (!(side == 0 ? free_i : free_j)) continue;
    double *J = side == 0 ? Ji : Jj;
    double add[7] = {0, 0, 0, 0, 0, 0, 0};
    for (int d = 0; d < 7; ++d) {
      double P[8], M[8], ep[7], em[7];
      memcpy(P, side == 0 ? Si : Sj, sizeof(P));
      add[d] = delta;
      sim3_oplus(P, add, fix_scale);
      if (side == 0) orc_eg_edge_error(P, Sj, C, ep);
      else orc_eg_edge_error(Si, P, C, ep);
      memcpy(M, side == 0 ? Si : Sj, sizeof(M));
      add[d] = -delta;
      sim3_oplus(M, add, fix_scale);
      if (side == 0) orc_eg_edge_error(M, Sj, C, em);
      else orc_eg_edge_error(Si, M, C, em);
      add[d] = 0.0;
      for (int r = 0; r < 7; ++r) {
        double bak = ep[r];
        bak -= em[r];
        J[7 * r + d] = scalar * bak;
      }
    }
  }
}

/* --------------------------------------------------- LM on the pose graph */

typedef struct {
  orc_eg_graph *g;
  int nP;
  int *hid, *pose_of;
  int64_t *ae, n_ae;
  double *Hd;            /* [nP][49] diagonal blocks */
  double *Ho;            /* [n_ae][49] off-diagonal block of each edge (hid order) */
  double *b, *x;         /* [7 nP] */
  double *bk;            /* [nP][8] backup */
  skyline sky;
} eg_ws;

static int cmp_int(const void *a, const void *b) { return *(const int *)a - *(const int *)b; }

static int eg_init(eg_ws *w, orc_eg_graph *g) {
  memset(w, 0, sizeof(*w));
  w->g = g;
  const int n = g->n_kf;
  uint8_t *act = calloc(n ? n : 1, 1);
  w->ae = malloc(sizeof(int64_t) * (g->n_edge ? g->n_edge : 1));
  for (int64_t e = 0; e < g->n_edge; ++e) {
    const int i = g->ei[e], j = g->ej[e];
    if (g->fixed[i] && g->fixed[j]) continue; /* all-fixed edges are not active */
    w->ae[w->n_ae++] = e;
    act[i] = act[j] = 1;
  }
  w->hid = malloc(sizeof(int) * (n ? n : 1));
  w->pose_of = malloc(sizeof(int) * (n ? n : 1));
  for (int p = 0; p < n; ++p) {
    if (act[p] && !g->fixed[p]) { w->hid[p] = w->nP; w->pose_of[w->nP++] = p; }
    else w->hid[p] = -1;
  }
  free(act);
  if (w->nP == 0) return 0;
  /* skyline profile in hidx order: first block row of column block c = min neighbour */
  const int nd = 7 * w->nP;
  int *firstblk = malloc(sizeof(int) * w->nP);
  for (int i = 0; i < w->nP; ++i) firstblk[i] = i;
  for (int64_t k = 0; k < w->n_ae; ++k) {
    const int64_t e = w->ae[k];
    const int a = w->hid[g->ei[e]], b = w->hid[g->ej[e]];
    if (a < 0 || b < 0) continue;
    const int lo = a < b ? a : b, hi = a < b ? b : a;
    if (firstblk[hi] > lo) firstblk[hi] = lo;
  }
  w->sky.n = nd;
  w->sky.first = malloc(sizeof(int) * nd);
  w->sky.cptr = malloc(sizeof(int64_t) * (nd + 1));
  w->sky.cptr[0] = 0;
  for (int c = 0; c < nd; ++c) {
    w->sky.first[c] = 7 * firstblk[c / 7];
    w->sky.cptr[c + 1] = w->sky.cptr[c] + (c - w->sky.first[c] + 1);
  }
  w->sky.val = malloc(sizeof(double) * w->sky.cptr[nd]);
  free(firstblk);
  w->Hd = malloc(sizeof(double) * 49 * w->nP);
  w->Ho = malloc(sizeof(double) * 49 * (w->n_ae ? w->n_ae : 1));
  w->b = malloc(sizeof(double) * nd);
  w->x = calloc(nd, sizeof(double));
  w->bk = malloc(sizeof(double) * 8 * w->nP);
  (void)cmp_int;
  return 1;
}

static void eg_free(eg_ws *w) {
  free(w->ae); free(w->hid); free(w->pose_of); free(w->Hd); free(w->Ho); free(w->b); free(w->x); free(w->bk);
  free(w->sky.first); free(w->sky.cptr); free(w->sky.val);
}

static void eg_errors(eg_ws *w) {
  orc_eg_graph *g = w->g;
  for (int64_t k = 0; k < w->n_ae; ++k) {
    const int64_t e = w->ae[k];
    orc_eg_edge_error(g->Siw + 8 * g->ei[e], g->Siw + 8 * g->ej[e], g->Sji + 8 * e, g->err + 7 * e);
  }
}

static inline double eg_info(const orc_eg_graph *g, int64_t e, int r, int c) {
  return g->info ? g->info[49 * e + 7 * r + c] : (r == c ? 1.0 : 0.0);
}

/* BaseEdge::chi2 = e^T Omega e, summed in edge-id order. */
static double eg_chi2(eg_ws *w) {
  orc_eg_graph *g = w->g;
  double chi = 0.0;
  for (int64_t k = 0; k < w->n_ae; ++k) {
    const int64_t e = w->ae[k];
    const double *er = g->err + 7 * e;
    double c = 0.0;
    for (int r = 0; r < 7; ++r) {
      double oe = 0.0;
      for (int s = 0; s < 7; ++s) oe += eg_info(g, e, r, s) * er[s];
      c += er[r] * oe;
    }
    chi += c;
  }
  return chi;
}

/* buildSystem with BaseBinaryEdge::constructQuadraticForm (base_binary_edge.hpp:55-120). */
static void eg_build(eg_ws *w) {
  orc_eg_graph *g = w->g;
  memset(w->Hd, 0, sizeof(double) * 49 * w->nP);
  memset(w->Ho, 0, sizeof(double) * 49 * w->n_ae);
  memset(w->b, 0, sizeof(double) * 7 * w->nP);
  for (int64_t k = 0; k < w->n_ae; ++k) {
    const int64_t e = w->ae[k];
    const int vi = g->ei[e], vj = g->ej[e], hi = w->hid[vi], hj = w->hid[vj];
    double A[49], B[49], om[7], AtO[49], BtO[49];
    orc_eg_edge_jacobians(g->Siw + 8 * vi, g->Siw + 8 * vj, g->Sji + 8 * e, g->fix_scale, hi >= 0, hj >= 0, A, B);
    const double *er = g->err + 7 * e;
    for (int r = 0; r < 7; ++r) {
      double v = 0.0;
      for (int s = 0; s < 7; ++s) v += eg_info(g, e, r, s) * er[s];
      om[r] = -v;
    }
    if (hi >= 0) {
      for (int r = 0; r < 7; ++r)
        for (int c = 0; c < 7; ++c) {
          double v = 0.0;
          for (int s = 0; s < 7; ++s) v += A[7 * s + r] * eg_info(g, e, s, c);
          AtO[7 * r + c] = v;
        }
      double *bi = w->b + 7 * hi, *H = w->Hd + 49 * hi;
      for (int r = 0; r < 7; ++r) {
        double v = 0.0;
        for (int s = 0; s < 7; ++s) v += A[7 * s + r] * om[s];
        bi[r] += v;
        for (int c = 0; c < 7; ++c) {
          double h = 0.0;
          for (int s = 0; s < 7; ++s) h += AtO[7 * r + s] * A[7 * s + c];
          H[7 * r + c] += h;
        }
      }
      if (hj >= 0) /* H_ij = AtO * B, kept as block (row hi, col hj) */
        for (int r = 0; r < 7; ++r)
          for (int c = 0; c < 7; ++c) {
            double h = 0.0;
            for (int s = 0; s < 7; ++s) h += AtO[7 * r + s] * B[7 * s + c];
            w->Ho[49 * k + 7 * r + c] = h;
          }
    }
    if (hj >= 0) {
      for (int r = 0; r < 7; ++r)
        for (int c = 0; c < 7; ++c) {
          double v = 0.0;
          for (int s = 0; s < 7; ++s) v += B[7 * s + r] * eg_info(g, e, s, c);
          BtO[7 * r + c] = v;
        }
      double *bj = w->b + 7 * hj, *H = w->Hd + 49 * hj;
      for (int r = 0; r < 7; ++r) {
        double v = 0.0;
        for (int s = 0; s < 7; ++s) v += B[7 * s + r] * om[s];
        bj[r] += v;
        for (int c = 0; c < 7; ++c) {
          double h = 0.0;
          for (int s = 0; s < 7; ++s) h += BtO[7 * r + s] * B[7 * s + c];
          H[7 * r + c] += h;
        }
      }
    }
  }
}

static double eg_maxdiag(eg_ws *w) {
  double m = 0.0;
  for (int i = 0; i < w->nP; ++i)
    for (int j = 0; j < 7; ++j) m = fmax(fabs(w->Hd[49 * i + 8 * j]), m);
  return m;
}

/* (H + lambda I) x = b by the skyline LDL^T (stand-in for SimplicialLDLT). */
static int eg_solve(eg_ws *w, double lambda) {
  orc_eg_graph *g = w->g;
  skyline *s = &w->sky;
  memset(s->val, 0, sizeof(double) * s->cptr[s->n]);
  for (int i = 0; i < w->nP; ++i)
    for (int c = 0; c < 7; ++c)
      for (int r = 0; r <= c; ++r)
        *sky_at(s, 7 * i + r, 7 * i + c) = w->Hd[49 * i + 7 * r + c] + (r == c ? lambda : 0.0);
  for (int64_t k = 0; k < w->n_ae; ++k) {
    const int64_t e = w->ae[k];
    const int hi = w->hid[g->ei[e]], hj = w->hid[g->ej[e]];
    if (hi < 0 || hj < 0 || hi == hj) continue;
    const double *Hb = w->Ho + 49 * k;
    for (int r = 0; r < 7; ++r)
      for (int c = 0; c < 7; ++c) {
        if (hi < hj) *sky_at(s, 7 * hi + r, 7 * hj + c) += Hb[7 * r + c];
        else *sky_at(s, 7 * hj + c, 7 * hi + r) += Hb[7 * r + c];
      }
  }
  if (!sky_factor(s)) return 0;
  sky_solve(s, w->b, w->x);
  return 1;
}

static int stopped_(const volatile uint8_t *stop) { return stop ? (*stop != 0) : 0; }

int orc_eg_optimize(orc_eg_graph *g, int iterations, double user_lambda, const volatile uint8_t *stop,
                    orc_stats *st) {
  orc_stats dummy;
  if (!st) st = &dummy;
  memset(st, 0, sizeof(*st));
  eg_ws w;
  if (!eg_init(&w, g)) { eg_free(&w); return -1; }
  st->n_active_edges = (int)w.n_ae;
  double lambda = -1., ni = 2.;
  int nbad = 0, its = 0, result = 0;
  for (int it = 0; it < iterations && !stopped_(stop) && result == 0; ++it) {
    eg_errors(&w);
    double currentChi = eg_chi2(&w), tempChi;
    const double iniChi = currentChi;
    if (it == 0) st->chi2_begin = currentChi;
    eg_build(&w);
    if (it == 0) {
      lambda = user_lambda > 0 ? user_lambda : 1e-5 * eg_maxdiag(&w);
      ni = 2;
      nbad = 0;
    }
    double rho = 0;
    int qmax = 0;
    do {
      for (int i = 0; i < w.nP; ++i) memcpy(w.bk + 8 * i, g->Siw + 8 * w.pose_of[i], 8 * sizeof(double));
      const int ok = eg_solve(&w, lambda);
      if (!ok) memset(w.x, 0, sizeof(double) * 7 * w.nP);
      for (int i = 0; i < w.nP; ++i) sim3_oplus(g->Siw + 8 * w.pose_of[i], w.x + 7 * i, g->fix_scale);
      eg_errors(&w);
      tempChi = eg_chi2(&w);
      if (!ok || (isnan(tempChi) && isfinite(currentChi))) tempChi = DBL_MAX;  // NaN: a failed trial (g2o_ref.c)
      rho = (currentChi - tempChi);
      double scale = 0.;
      for (int j = 0; j < 7 * w.nP; ++j) scale += w.x[j] * (lambda * w.x[j] + w.b[j]);
      scale += 1e-3;
      rho /= scale;
      if (rho > 0 && isfinite(tempChi)) {
        double alpha = 1. - pow((2 * rho - 1), 3);
        alpha = fmin(alpha, 2. / 3.);
        lambda *= fmax(1. / 3., alpha);
        ni = 2;
        currentChi = tempChi;
      } else {
        lambda *= ni;
        ni *= 2;
        for (int i = 0; i < w.nP; ++i) memcpy(g->Siw + 8 * w.pose_of[i], w.bk + 8 * i, 8 * sizeof(double));
      }
      qmax++;
      st->trials++;
    } while (rho < 0 && qmax < 10 && !stopped_(stop));
    if (qmax == 10 || rho == 0) result = 1;
    else {
      if ((iniChi - currentChi) * 1e3 < iniChi) nbad++;
      else nbad = 0;
      if (nbad >= 3) result = 1;
    }
    if (its < ORC_TRACE_MAX) {
      st->trace_chi2[its] = currentChi;
      st->trace_lambda[its] = lambda;
      st->trace_trials[its] = qmax;
      st->trace_len = its + 1;
    }
    st->chi2_end = currentChi;
    st->lambda_end = lambda;
    ++its;
  }
  st->iterations = its; /* err keeps g2o's stale-_error semantics (last computed, maybe rejected) */
  st->result = result;
  eg_free(&w);
  return its;
}
