/*
 * g2o_ref.c — TEST INFRASTRUCTURE (oracle). CPU restatement of the reference
 * g2o bundle-adjustment path. See oracle.h for the file:line map and the
 * "parity unpinned" note. Single-threaded by default: the reference builds g2o
 * with G2O_USE_OPENMP=OFF (Thirdparty/g2o/build/CMakeCache.txt:175), so this is
 * also the CPU baseline ("kind": "port") timed by bench.py. Built with
 * -fopenmp -DORC_OMP (liboracle_omp.so) it is the labelled all-cores variant:
 * the loops g2o parallelises under G2O_OPENMP (sparse_optimizer.cpp:71,
 * block_solver.hpp:379,527) run on every core, each accumulator owned by one
 * thread and summed in the serial order, so its results equal the serial
 * build's bit for bit (tests/test_oracle.py).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
 * this library; the product path (libsqrtlm.so) never links or calls it.
 */
#include "oracle.h"
#include "se3_ref.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef ORC_OMP
#include <omp.h>
#endif

/* threads the OpenMP loops of this build run on (1 for the serial build) */
int orc_omp_threads(void) {
#ifdef ORC_OMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* ------------------------------------------------------------------ edges */

/* SE3Quat::map (se3quat.h:217-220): _r*xyz + _t. */
static inline void se3_map(const double q[4], const double t[3], const double X[3], double o[3]) {
  double r[3];
  oq_rotate(q, X, r);
  o[0] = r[0] + t[0]; o[1] = r[1] + t[1]; o[2] = r[2] + t[2];
}

/* EdgeSE3ProjectXYZ::computeError (types_six_dof_expmap.h:90-95), cam_project
 * (.cpp:141-147) and project2d (.cpp:37-42): e = obs - (fx x/z + cx, fy y/z + cy). */
static void mono_error(const orc_graph *g, int64_t e, double err[2]) {
  const int p = g->obs_pose[e], l = g->obs_pt[e];
  const double *in = g->intr + 4 * p;
  double xc[3];
  se3_map(g->pose_q + 4 * p, g->pose_t + 3 * p, g->pt + 3 * l, xc);
  double u = (xc[0] / xc[2]) * in[0] + in[2];
  double v = (xc[1] / xc[2]) * in[1] + in[3];
  err[0] = g->obs_uv[2 * e + 0] - u;
  err[1] = g->obs_uv[2 * e + 1] - v;
}

void orc_mono_jacobians(const double q[4], const double t[3], const double in[4], const double X[3],
                        double Jl[6], double Jp[12]) {
  /* EdgeSE3ProjectXYZ::linearizeOplus (types_six_dof_expmap.cpp:103-139). */
  double xc[3], R[9];
  se3_map(q, t, X, xc);
  const double x = xc[0], y = xc[1], z = xc[2], z_2 = z * z;
  const double fx = in[0], fy = in[1];
  double tmp[6] = {fx, 0.0, -x / z * fx, 0.0, fy, -y / z * fy};
  oq_to_mat(q, R);
  const double s = -1. / z;
  for (int r = 0; r < 2; ++r)
    for (int c = 0; c < 3; ++c)
      Jl[r * 3 + c] = (s * tmp[r * 3 + 0]) * R[0 * 3 + c] + (s * tmp[r * 3 + 1]) * R[1 * 3 + c] +
                      (s * tmp[r * 3 + 2]) * R[2 * 3 + c];
  Jp[0] = x * y / z_2 * fx;
  Jp[1] = -(1 + (x * x / z_2)) * fx;
  Jp[2] = y / z * fx;
  Jp[3] = -1. / z * fx;
  Jp[4] = 0;
  Jp[5] = x / z_2 * fx;
  Jp[6] = (1 + y * y / z_2) * fy;
  Jp[7] = -x * y / z_2 * fy;
  Jp[8] = -x / z * fy;
  Jp[9] = 0;
  Jp[10] = -1. / z * fy;
  Jp[11] = y / z_2 * fy;
}

/* EdgeStereoSE3ProjectXYZ::cam_project (types_six_dof_expmap.cpp:150-157):
 * invz is a float (1/z rounded to single), bf arrives through a float
 * parameter and bf*invz is a single-precision product. */
void orc_stereo_project(const double q[4], const double t[3], const double in[4], double bf, const double X[3],
                        double proj[3]) {
  double xc[3];
  se3_map(q, t, X, xc);
  const float invz = (float)(1.0f / xc[2]);
  const float bff = (float)bf;
  proj[0] = xc[0] * invz * in[0] + in[2];
  proj[1] = xc[1] * invz * in[1] + in[3];
  const float bz = bff * invz;
  proj[2] = proj[0] - bz;
}

/* EdgeStereoSE3ProjectXYZ::linearizeOplus (types_six_dof_expmap.cpp:188-234). */
void orc_stereo_jacobians(const double q[4], const double t[3], const double in[4], double bf, const double X[3],
                          double Jl[9], double Jp[18]) {
  double xc[3], R[9];
  se3_map(q, t, X, xc);
  oq_to_mat(q, R);
  const double x = xc[0], y = xc[1], z = xc[2], z_2 = z * z, fx = in[0], fy = in[1];
  for (int c = 0; c < 3; ++c) {
    Jl[c] = -fx * R[c] / z + fx * x * R[6 + c] / z_2;
    Jl[3 + c] = -fy * R[3 + c] / z + fy * y * R[6 + c] / z_2;
    Jl[6 + c] = Jl[c] - bf * R[6 + c] / z_2;
  }
  Jp[0] = x * y / z_2 * fx;
  Jp[1] = -(1 + (x * x / z_2)) * fx;
  Jp[2] = y / z * fx;
  Jp[3] = -1. / z * fx;
  Jp[4] = 0;
  Jp[5] = x / z_2 * fx;
  Jp[6] = (1 + y * y / z_2) * fy;
  Jp[7] = -x * y / z_2 * fy;
  Jp[8] = -x / z * fy;
  Jp[9] = 0;
  Jp[10] = -1. / z * fy;
  Jp[11] = y / z_2 * fy;
  Jp[12] = Jp[0] - bf * y / z_2;
  Jp[13] = Jp[1] + bf * x / z_2;
  Jp[14] = Jp[2];
  Jp[15] = Jp[3];
  Jp[16] = 0;
  Jp[17] = Jp[5] - bf / z_2;
}

static inline int is_stereo(const orc_graph *g, int64_t e) { return g->obs_ur && g->obs_ur[e] >= 0.0; }

/* EdgeStereoSE3ProjectXYZ::computeError (types_six_dof_expmap.h:122-127). */
static void stereo_error(const orc_graph *g, int64_t e, double err[3]) {
  const int p = g->obs_pose[e];
  double proj[3];
  orc_stereo_project(g->pose_q + 4 * p, g->pose_t + 3 * p, g->intr + 4 * p, g->pose_bf[p], g->pt + 3 * g->obs_pt[e],
                     proj);
  err[0] = g->obs_uv[2 * e + 0] - proj[0];
  err[1] = g->obs_uv[2 * e + 1] - proj[1];
  err[2] = g->obs_ur[e] - proj[2];
}

/* computeError of edge e (mono or stereo) into obs_err / obs_err3. */
static void edge_error(orc_graph *g, int64_t e) {
  if (is_stereo(g, e)) {
    double er[3];
    stereo_error(g, e, er);
    g->obs_err[2 * e] = er[0];
    g->obs_err[2 * e + 1] = er[1];
    g->obs_err3[e] = er[2];
  } else {
    mono_error(g, e, g->obs_err + 2 * e);
  }
}

/* EdgeLidarFlatPoint::computeError (types_six_dof_expmap.h:217-229). The
 * reference forms T_wc = (T_cw)^-1 through a 4x4 inverse and then applies
 * R_wc^-1 (p_w - t_wc); algebraically that is T_cw.map(p_w), which is what is
 * restated here (identical up to ~1 ulp; Eigen's 4x4 inverse is unpinned). */
double orc_lidar_error(const double q[4], const double t[3], const double pc[3], const double pw[3],
                       const double n[3]) {
  double c[3];
  se3_map(q, t, pw, c);
  double d0 = c[0] - pc[0], d1 = c[1] - pc[1], d2 = c[2] - pc[2];
  return (d0 * n[0] + d1 * n[1]) + d2 * n[2];
}

/* BaseUnaryEdge::linearizeOplus numeric central difference, delta = 1e-9,
 * applied through oplus (base_unary_edge.hpp:82-122). */
void orc_lidar_jacobian(const double q[4], const double t[3], const double pc[3], const double pw[3],
                        const double n[3], double J[6]) {
  const double delta = 1e-9, scalar = 1.0 / (2 * delta);
  double add[6] = {0, 0, 0, 0, 0, 0};
  for (int d = 0; d < 6; ++d) {
    double qa[4] = {q[0], q[1], q[2], q[3]}, ta[3] = {t[0], t[1], t[2]};
    add[d] = delta;
    ose3_oplus(qa, ta, add);
    double e1 = orc_lidar_error(qa, ta, pc, pw, n);
    double qb[4] = {q[0], q[1], q[2], q[3]}, tb[3] = {t[0], t[1], t[2]};
    add[d] = -delta;
    ose3_oplus(qb, tb, add);
    double e2 = orc_lidar_error(qb, tb, pc, pw, n);
    add[d] = 0.0;
    J[d] = scalar * (e1 - e2);
  }
}

static void lidar_error(const orc_graph *g, int64_t e, double *err) {
  const int p = g->lid_pose[e];
  *err = orc_lidar_error(g->pose_q + 4 * p, g->pose_t + 3 * p, g->lid_pc + 3 * e, g->lid_pw + 3 * e,
                         g->lid_n + 3 * e);
}

/* RobustKernelHuber::robustify (robust_kernel_impl.cpp:78-90). */
static inline void huber(double delta, double e, double rho[2]) {
  const double dsqr = delta * delta;
  if (e <= dsqr) {
    rho[0] = e; rho[1] = 1.;
  } else {
    double sqrte = sqrt(e);
    rho[0] = 2 * sqrte * delta - dsqr;
    rho[1] = delta / sqrte;
  }
}

/* BaseEdge::chi2 = e^T (I info) e, 2-D or 3-D. */
static inline double mono_chi2(const orc_graph *g, int64_t e) {
  const double *er = g->obs_err + 2 * e, w = g->obs_info[e];
  double c = er[0] * (w * er[0]) + er[1] * (w * er[1]);
  if (is_stereo(g, e)) c += g->obs_err3[e] * (w * g->obs_err3[e]);
  return c;
}

/* Outlier threshold of the LBA tags: chi2(0.95) with 2 DoF for mono edges
 * (g2oOptimizer.cc:956,1123). The reference's LBA never adds stereo edges
 * (:914-916 is empty); 3 DoF, 7.815, is the ORB-SLAM2 value for them. */
static inline double tag_threshold(const orc_graph *g, int64_t e) { return is_stereo(g, e) ? 7.815 : 5.991; }

void orc_compute_mono_errors(orc_graph *g) {
  for (int64_t e = 0; e < g->n_obs; ++e) edge_error(g, e);
}

void orc_edge_chi2(const orc_graph *g, double *out) {
  for (int64_t e = 0; e < g->n_obs; ++e) out[e] = mono_chi2(g, e);
}

void orc_depth_positive(const orc_graph *g, uint8_t *out) {
  for (int64_t e = 0; e < g->n_obs; ++e) {
    double xc[3];
    const int p = g->obs_pose[e];
    se3_map(g->pose_q + 4 * p, g->pose_t + 3 * p, g->pt + 3 * g->obs_pt[e], xc);
    out[e] = xc[2] > 0.0;
  }
}

#include "skyline_ref.h"

/* --------------------------------------------------------- the optimizer */

typedef struct {
  orc_graph *g;
  int nP, nL;
  int *phid, *lhid, *pose_of, *pt_of;
  int64_t *ae, n_ae;     /* active mono edges, id order */
  int64_t *al, n_al;     /* active lidar edges, id order */
  /* Hpl CCS: per landmark column, blocks sorted by pose hidx */
  int64_t *col_ptr;      /* [nL+1] */
  int *blk_row;          /* [nblk] pose hidx */
  double *blk;           /* [nblk][18] 6x3 row-major */
  int64_t nblk;
  int64_t *edge_blk;     /* [n_obs] block of edge, -1 if none */
  double *Hpp;           /* [nP][36] */
  double *Hll;           /* [nL][9]  */
  double *b;             /* [6 nP + 3 nL] */
  double *x;             /* [6 nP + 3 nL] */
  double *Dinv;          /* [nL][9] */
  double *coeff;         /* [6 nP] */
  double *bschur;        /* [6 nP] */
  skyline sky;
  double *bk_q, *bk_t, *bk_X; /* push/pop backup */
#ifdef ORC_OMP
  /* owner-computes lists (ORC_OMP): active mono edges per landmark / per free
   * pose in id order; per free pose i2 the (landmark, block) pairs with that
   * row, landmarks ascending; per-landmark Dinv b_l and per-block B Dinv */
  int64_t *le_ptr, *le, *pe_ptr, *pe, *pl_ptr, *pl_blk;
  int *pl_lm;
  double *db, *BDinv, *chi_e;
#endif
} lm_ws;

static int cmp_blk(const void *a, const void *b) {
  const int64_t *x = (const int64_t *)a, *y = (const int64_t *)b;
  return (x[0] > y[0]) - (x[0] < y[0]);
}

/* initializeOptimization(level) + BlockSolver::buildStructure. */
static int ws_init(lm_ws *w, orc_graph *g, int level) {
  memset(w, 0, sizeof(*w));
  w->g = g;
  uint8_t *pose_act = calloc(g->n_pose ? g->n_pose : 1, 1);
  uint8_t *pt_act = calloc(g->n_pt ? g->n_pt : 1, 1);
  w->ae = malloc(sizeof(int64_t) * (g->n_obs ? g->n_obs : 1));
  w->al = malloc(sizeof(int64_t) * (g->n_lid ? g->n_lid : 1));
  for (int64_t e = 0; e < g->n_obs; ++e) {
    if (g->obs_level[e] != level) continue;
    /* points are never fixed, so a mono edge is never all-fixed */
    w->ae[w->n_ae++] = e;
    pose_act[g->obs_pose[e]] = 1;
    pt_act[g->obs_pt[e]] = 1;
  }
  for (int64_t e = 0; e < g->n_lid; ++e) {
    if (g->lid_level[e] != level || g->pose_fixed[g->lid_pose[e]]) continue;
    w->al[w->n_al++] = e;
    pose_act[g->lid_pose[e]] = 1;
  }
  /* buildIndexMapping (sparse_optimizer.cpp:166-190): free poses by id, then points */
  w->phid = malloc(sizeof(int) * (g->n_pose ? g->n_pose : 1));
  w->lhid = malloc(sizeof(int) * (g->n_pt ? g->n_pt : 1));
  w->pose_of = malloc(sizeof(int) * (g->n_pose ? g->n_pose : 1));
  w->pt_of = malloc(sizeof(int) * (g->n_pt ? g->n_pt : 1));
  for (int p = 0; p < g->n_pose; ++p) {
    if (pose_act[p] && !g->pose_fixed[p]) { w->phid[p] = w->nP; w->pose_of[w->nP++] = p; }
    else w->phid[p] = -1;
  }
  for (int l = 0; l < g->n_pt; ++l) {
    if (pt_act[l]) { w->lhid[l] = w->nL; w->pt_of[w->nL++] = l; }
    else w->lhid[l] = -1;
  }
  free(pose_act); free(pt_act);
  if (w->nP + w->nL == 0) return 0;

  /* Hpl blocks: (landmark hidx, pose hidx) pairs, unique */
  int64_t *keys = malloc(sizeof(int64_t) * 2 * (w->n_ae ? w->n_ae : 1));
  int64_t nk = 0;
  for (int64_t i = 0; i < w->n_ae; ++i) {
    int64_t e = w->ae[i];
    int ph = w->phid[g->obs_pose[e]];
    if (ph < 0) continue;
    keys[2 * nk] = (int64_t)w->lhid[g->obs_pt[e]] * (int64_t)(w->nP + 1) + ph;
    keys[2 * nk + 1] = e;
    nk++;
  }
  qsort(keys, nk, 2 * sizeof(int64_t), cmp_blk);
  w->edge_blk = malloc(sizeof(int64_t) * (g->n_obs ? g->n_obs : 1));
  for (int64_t e = 0; e < g->n_obs; ++e) w->edge_blk[e] = -1;
  w->col_ptr = calloc(w->nL + 1, sizeof(int64_t));
  w->blk_row = malloc(sizeof(int) * (nk ? nk : 1));
  w->blk = calloc(18 * (nk ? nk : 1), sizeof(double));
  int64_t nb = 0, prev = -1;
  for (int64_t i = 0; i < nk; ++i) {
    if (keys[2 * i] != prev) {
      prev = keys[2 * i];
      int l = (int)(prev / (w->nP + 1));
      w->blk_row[nb] = (int)(prev % (w->nP + 1));
      w->col_ptr[l + 1]++;
      nb++;
    }
    w->edge_blk[keys[2 * i + 1]] = nb - 1;
  }
  w->nblk = nb;
  for (int l = 0; l < w->nL; ++l) w->col_ptr[l + 1] += w->col_ptr[l];
  free(keys);

  /* Schur pattern (block_solver.hpp:262-292) -> skyline profile: first block
   * row of every block column = min pose hidx co-observing a landmark. */
  const int n = 6 * w->nP;
  int *firstblk = malloc(sizeof(int) * (w->nP ? w->nP : 1));
  for (int i = 0; i < w->nP; ++i) firstblk[i] = i;
  for (int l = 0; l < w->nL; ++l) {
    if (w->col_ptr[l + 1] == w->col_ptr[l]) continue;
    int mn = w->blk_row[w->col_ptr[l]]; /* sorted */
    for (int64_t k = w->col_ptr[l]; k < w->col_ptr[l + 1]; ++k)
      if (firstblk[w->blk_row[k]] > mn) firstblk[w->blk_row[k]] = mn;
  }
  w->sky.n = n;
  w->sky.first = malloc(sizeof(int) * (n ? n : 1));
  w->sky.cptr = malloc(sizeof(int64_t) * (n + 1));
  w->sky.cptr[0] = 0;
  for (int c = 0; c < n; ++c) {
    w->sky.first[c] = 6 * firstblk[c / 6];
    w->sky.cptr[c + 1] = w->sky.cptr[c] + (c - w->sky.first[c] + 1);
  }
  w->sky.val = malloc(sizeof(double) * (w->sky.cptr[n] ? w->sky.cptr[n] : 1));
  free(firstblk);

  const int dim = 6 * w->nP + 3 * w->nL;
  w->Hpp = malloc(sizeof(double) * 36 * (w->nP ? w->nP : 1));
  w->Hll = malloc(sizeof(double) * 9 * (w->nL ? w->nL : 1));
  w->b = malloc(sizeof(double) * dim);
  w->x = calloc(dim, sizeof(double));
  w->Dinv = malloc(sizeof(double) * 9 * (w->nL ? w->nL : 1));
  w->coeff = malloc(sizeof(double) * (n ? n : 1));
  w->bschur = malloc(sizeof(double) * (n ? n : 1));
  w->bk_q = malloc(sizeof(double) * 4 * (w->nP ? w->nP : 1));
  w->bk_t = malloc(sizeof(double) * 3 * (w->nP ? w->nP : 1));
  w->bk_X = malloc(sizeof(double) * 3 * (w->nL ? w->nL : 1));
#ifdef ORC_OMP
  {
    const int64_t ne = w->n_ae;
    w->le_ptr = calloc(w->nL + 1, sizeof(int64_t));
    w->pe_ptr = calloc(w->nP + 1, sizeof(int64_t));
    w->pl_ptr = calloc(w->nP + 1, sizeof(int64_t));
    w->le = malloc(sizeof(int64_t) * (ne ? ne : 1));
    w->pe = malloc(sizeof(int64_t) * (ne ? ne : 1));
    w->pl_blk = malloc(sizeof(int64_t) * (w->nblk ? w->nblk : 1));
    w->pl_lm = malloc(sizeof(int) * (w->nblk ? w->nblk : 1));
    for (int64_t i = 0; i < ne; ++i) {
      const int64_t e = w->ae[i];
      w->le_ptr[w->lhid[g->obs_pt[e]] + 1]++;
      if (w->phid[g->obs_pose[e]] >= 0) w->pe_ptr[w->phid[g->obs_pose[e]] + 1]++;
    }
    for (int64_t k = 0; k < w->nblk; ++k) w->pl_ptr[w->blk_row[k] + 1]++;
    for (int l = 0; l < w->nL; ++l) w->le_ptr[l + 1] += w->le_ptr[l];
    for (int i = 0; i < w->nP; ++i) { w->pe_ptr[i + 1] += w->pe_ptr[i]; w->pl_ptr[i + 1] += w->pl_ptr[i]; }
    int64_t *fl = malloc(sizeof(int64_t) * (w->nL + 1)), *fp = malloc(sizeof(int64_t) * (w->nP + 1));
    memcpy(fl, w->le_ptr, sizeof(int64_t) * (w->nL + 1));
    memcpy(fp, w->pe_ptr, sizeof(int64_t) * (w->nP + 1));
    for (int64_t i = 0; i < ne; ++i) {
      const int64_t e = w->ae[i];
      w->le[fl[w->lhid[g->obs_pt[e]]]++] = e;
      if (w->phid[g->obs_pose[e]] >= 0) w->pe[fp[w->phid[g->obs_pose[e]]]++] = e;
    }
    memcpy(fp, w->pl_ptr, sizeof(int64_t) * (w->nP + 1));
    for (int l = 0; l < w->nL; ++l)
      for (int64_t k = w->col_ptr[l]; k < w->col_ptr[l + 1]; ++k) {
        const int64_t o = fp[w->blk_row[k]]++;
        w->pl_blk[o] = k;
        w->pl_lm[o] = l;
      }
    free(fl); free(fp);
    w->db = malloc(sizeof(double) * 3 * (w->nL ? w->nL : 1));
    w->BDinv = malloc(sizeof(double) * 18 * (w->nblk ? w->nblk : 1));
    w->chi_e = malloc(sizeof(double) * (ne ? ne : 1));
  }
#endif
  return 1;
}

static void ws_free(lm_ws *w) {
  free(w->phid); free(w->lhid); free(w->pose_of); free(w->pt_of); free(w->ae); free(w->al);
  free(w->col_ptr); free(w->blk_row); free(w->blk); free(w->edge_blk); free(w->Hpp); free(w->Hll);
  free(w->b); free(w->x); free(w->Dinv); free(w->coeff); free(w->bschur);
  free(w->sky.first); free(w->sky.cptr); free(w->sky.val);
  free(w->bk_q); free(w->bk_t); free(w->bk_X);
#ifdef ORC_OMP
  free(w->le_ptr); free(w->le); free(w->pe_ptr); free(w->pe); free(w->pl_ptr); free(w->pl_blk); free(w->pl_lm);
  free(w->db); free(w->BDinv); free(w->chi_e);
#endif
}

/* SparseOptimizer::computeActiveErrors (sparse_optimizer.cpp:61-88). */
static void compute_active_errors(lm_ws *w) {
  orc_graph *g = w->g;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < w->n_ae; ++i) edge_error(g, w->ae[i]);
  for (int64_t i = 0; i < w->n_al; ++i) lidar_error(g, w->al[i], g->lid_err + w->al[i]);
}

/* SparseOptimizer::activeRobustChi2 (sparse_optimizer.cpp:100-114), edge id order. */
static double active_robust_chi2(lm_ws *w) {
  orc_graph *g = w->g;
  double chi = 0.0, rho[2];
#ifdef ORC_OMP
  /* per-edge terms in parallel, summed in id order (the serial sum's bits) */
#pragma omp parallel for schedule(static) private(rho)
  for (int64_t i = 0; i < w->n_ae; ++i) {
    int64_t e = w->ae[i];
    double c = mono_chi2(g, e);
    if (g->obs_delta[e] > 0.0) { huber(g->obs_delta[e], c, rho); c = rho[0]; }
    w->chi_e[i] = c;
  }
  for (int64_t i = 0; i < w->n_ae; ++i) chi += w->chi_e[i];
#else
  for (int64_t i = 0; i < w->n_ae; ++i) {
    int64_t e = w->ae[i];
    double c = mono_chi2(g, e);
    if (g->obs_delta[e] > 0.0) { huber(g->obs_delta[e], c, rho); chi += rho[0]; }
    else chi += c;
  }
#endif
  for (int64_t i = 0; i < w->n_al; ++i) {
    int64_t e = w->al[i];
    double er = g->lid_err[e];
    chi += er * (g->lid_info[e] * er);
  }
  return chi;
}

#ifdef ORC_OMP
/* One mono / stereo edge linearised as in build_system: Jacobians A (point),
 * B (pose), -(rho' info) e and the robust weight. */
static int edge_lin(const orc_graph *g, int64_t e, double A[9], double B[18], double omega_r[3], double *wgt) {
  const int p = g->obs_pose[e], l = g->obs_pt[e];
  const int nr = is_stereo(g, e) ? 3 : 2;
  double er[3];
  if (nr == 3)
    orc_stereo_jacobians(g->pose_q + 4 * p, g->pose_t + 3 * p, g->intr + 4 * p, g->pose_bf[p], g->pt + 3 * l, A, B);
  else
    orc_mono_jacobians(g->pose_q + 4 * p, g->pose_t + 3 * p, g->intr + 4 * p, g->pt + 3 * l, A, B);
  er[0] = g->obs_err[2 * e];
  er[1] = g->obs_err[2 * e + 1];
  er[2] = nr == 3 ? g->obs_err3[e] : 0.0;
  const double info = g->obs_info[e];
  for (int r = 0; r < nr; ++r) omega_r[r] = -(info * er[r]);
  *wgt = info;
  if (g->obs_delta[e] > 0.0) {
    double rho[2];
    huber(g->obs_delta[e], mono_chi2(g, e), rho);
    *wgt = rho[1] * info;
    for (int r = 0; r < nr; ++r) omega_r[r] *= rho[1];
  }
  return nr;
}

/* build_system with one owner per accumulator: landmark blocks (H_ll, b_l,
 * H_pl) by landmark, pose blocks (H_pp, b_p) by pose, each over its edges in
 * id order -- the serial loop's summation order, so the same bits. */
static void build_system_omp(lm_ws *w) {
  orc_graph *g = w->g;
  const int np6 = 6 * w->nP;
  memset(w->Hpp, 0, sizeof(double) * 36 * w->nP);
  memset(w->Hll, 0, sizeof(double) * 9 * w->nL);
  memset(w->blk, 0, sizeof(double) * 18 * w->nblk);
  memset(w->b, 0, sizeof(double) * (np6 + 3 * w->nL));
#pragma omp parallel for schedule(dynamic, 256)
  for (int lh = 0; lh < w->nL; ++lh) {
    double *bl = w->b + np6 + 3 * lh, *H = w->Hll + 9 * lh;
    for (int64_t k = w->le_ptr[lh]; k < w->le_ptr[lh + 1]; ++k) {
      const int64_t e = w->le[k];
      double A[9], B[18], omega_r[3], wgt;
      const int nr = edge_lin(g, e, A, B, omega_r, &wgt);
      for (int r = 0; r < 3; ++r) {
        double sb = 0.0;
        for (int q = 0; q < nr; ++q) sb += A[q * 3 + r] * omega_r[q];
        bl[r] += sb;
        for (int c = 0; c < 3; ++c) {
          double sh = 0.0;
          for (int q = 0; q < nr; ++q) sh += (A[q * 3 + r] * wgt) * A[q * 3 + c];
          H[r * 3 + c] += sh;
        }
      }
      if (w->phid[g->obs_pose[e]] >= 0) {
        double *Bl = w->blk + 18 * w->edge_blk[e];
        for (int r = 0; r < 6; ++r)
          for (int c = 0; c < 3; ++c) {
            double sh = 0.0;
            for (int q = 0; q < nr; ++q) sh += (B[q * 6 + r] * wgt) * A[q * 3 + c];
            Bl[r * 3 + c] += sh;
          }
      }
    }
  }
#pragma omp parallel for schedule(dynamic, 16)
  for (int ph = 0; ph < w->nP; ++ph) {
    double *bp = w->b + 6 * ph, *Hp = w->Hpp + 36 * ph;
    for (int64_t k = w->pe_ptr[ph]; k < w->pe_ptr[ph + 1]; ++k) {
      double A[9], B[18], omega_r[3], wgt;
      const int nr = edge_lin(g, w->pe[k], A, B, omega_r, &wgt);
      for (int r = 0; r < 6; ++r) {
        double sb = 0.0;
        for (int q = 0; q < nr; ++q) sb += B[q * 6 + r] * omega_r[q];
        bp[r] += sb;
        for (int c = 0; c < 6; ++c) {
          double sh = 0.0;
          for (int q = 0; q < nr; ++q) sh += (B[q * 6 + r] * wgt) * B[q * 6 + c];
          Hp[r * 6 + c] += sh;
        }
      }
    }
  }
  for (int64_t i = 0; i < w->n_al; ++i) {  /* after every mono edge, as in the serial loop */
    const int64_t e = w->al[i];
    const int p = g->lid_pose[e], ph = w->phid[p];
    double J[6];
    orc_lidar_jacobian(g->pose_q + 4 * p, g->pose_t + 3 * p, g->lid_pc + 3 * e, g->lid_pw + 3 * e,
                       g->lid_n + 3 * e, J);
    const double info = g->lid_info[e], er = g->lid_err[e];
    double *bp = w->b + 6 * ph, *Hp = w->Hpp + 36 * ph;
    for (int r = 0; r < 6; ++r) {
      bp[r] -= (J[r] * info) * er;
      for (int c = 0; c < 6; ++c) Hp[r * 6 + c] += (J[r] * info) * J[c];
    }
  }
}
#endif

/* BlockSolver::buildSystem (block_solver.hpp:502-560) with
 * BaseBinaryEdge / BaseUnaryEdge::constructQuadraticForm. */
static void build_system(lm_ws *w) {
  orc_graph *g = w->g;
  const int np6 = 6 * w->nP;
#ifdef ORC_OMP
  build_system_omp(w);
  return;
#endif
  memset(w->Hpp, 0, sizeof(double) * 36 * w->nP);
  memset(w->Hll, 0, sizeof(double) * 9 * w->nL);
  memset(w->blk, 0, sizeof(double) * 18 * w->nblk);
  memset(w->b, 0, sizeof(double) * (np6 + 3 * w->nL));
  for (int64_t i = 0; i < w->n_ae; ++i) {
    const int64_t e = w->ae[i];
    const int p = g->obs_pose[e], l = g->obs_pt[e];
    const int ph = w->phid[p], lh = w->lhid[l];
    double A[9], B[18], er[3];
    const int nr = is_stereo(g, e) ? 3 : 2;
    if (nr == 3)
      orc_stereo_jacobians(g->pose_q + 4 * p, g->pose_t + 3 * p, g->intr + 4 * p, g->pose_bf[p], g->pt + 3 * l, A, B);
    else
      orc_mono_jacobians(g->pose_q + 4 * p, g->pose_t + 3 * p, g->intr + 4 * p, g->pt + 3 * l, A, B);
    er[0] = g->obs_err[2 * e];
    er[1] = g->obs_err[2 * e + 1];
    er[2] = nr == 3 ? g->obs_err3[e] : 0.0;
    const double info = g->obs_info[e];
    double omega_r[3];
    for (int r = 0; r < nr; ++r) omega_r[r] = -(info * er[r]); /* -(I info) e, off-diagonal zeros exact */
    double wgt = info; /* diagonal of (robust) information */
    if (g->obs_delta[e] > 0.0) {
      double rho[2];
      huber(g->obs_delta[e], mono_chi2(g, e), rho);
      wgt = rho[1] * info;
      for (int r = 0; r < nr; ++r) omega_r[r] *= rho[1];
    }
    /* from = point (vertex 0, never fixed) */
    double *bl = w->b + np6 + 3 * lh;
    double *H = w->Hll + 9 * lh;
    for (int r = 0; r < 3; ++r) {
      double sb = 0.0;
      for (int k = 0; k < nr; ++k) sb += A[k * 3 + r] * omega_r[k];
      bl[r] += sb;
      for (int c = 0; c < 3; ++c) {
        double sh = 0.0;
        for (int k = 0; k < nr; ++k) sh += (A[k * 3 + r] * wgt) * A[k * 3 + c];
        H[r * 3 + c] += sh;
      }
    }
    if (ph >= 0) {
      double *Bl = w->blk + 18 * w->edge_blk[e]; /* H_pl(pose, point) = B^T W A */
      for (int r = 0; r < 6; ++r)
        for (int c = 0; c < 3; ++c) {
          double sh = 0.0;
          for (int k = 0; k < nr; ++k) sh += (B[k * 6 + r] * wgt) * A[k * 3 + c];
          Bl[r * 3 + c] += sh;
        }
      double *bp = w->b + 6 * ph;
      double *Hp = w->Hpp + 36 * ph;
      for (int r = 0; r < 6; ++r) {
        double sb = 0.0;
        for (int k = 0; k < nr; ++k) sb += B[k * 6 + r] * omega_r[k];
        bp[r] += sb;
        for (int c = 0; c < 6; ++c) {
          double sh = 0.0;
          for (int k = 0; k < nr; ++k) sh += (B[k * 6 + r] * wgt) * B[k * 6 + c];
          Hp[r * 6 + c] += sh;
        }
      }
    }
  }
  for (int64_t i = 0; i < w->n_al; ++i) {
    const int64_t e = w->al[i];
    const int p = g->lid_pose[e], ph = w->phid[p];
    double J[6];
    orc_lidar_jacobian(g->pose_q + 4 * p, g->pose_t + 3 * p, g->lid_pc + 3 * e, g->lid_pw + 3 * e,
                       g->lid_n + 3 * e, J);
    const double info = g->lid_info[e], er = g->lid_err[e];
    double *bp = w->b + 6 * ph, *Hp = w->Hpp + 36 * ph;
    for (int r = 0; r < 6; ++r) {
      bp[r] -= (J[r] * info) * er;
      for (int c = 0; c < 6; ++c) Hp[r * 6 + c] += (J[r] * info) * J[c];
    }
  }
}

/* OptimizationAlgorithmLevenberg::computeLambdaInit (levenberg.cpp:166-180). */
static double max_diagonal(lm_ws *w) {
  double m = 0.0;
  for (int i = 0; i < w->nP; ++i)
    for (int j = 0; j < 6; ++j) m = fmax(fabs(w->Hpp[36 * i + 7 * j]), m);
  for (int i = 0; i < w->nL; ++i)
    for (int j = 0; j < 3; ++j) m = fmax(fabs(w->Hll[9 * i + 4 * j]), m);
  return m;
}

#ifdef ORC_OMP
/* schur_solve with owners: per landmark Dinv, Dinv b_l and B Dinv (parallel);
 * S block column i2 (and coeff row i2) by one thread, over the landmarks that
 * touch it in ascending order -- each entry sums in the serial loop's order. */
static int schur_solve_omp(lm_ws *w, double lambda) {
  skyline *s = &w->sky;
  const int np6 = 6 * w->nP;
  memset(s->val, 0, sizeof(double) * s->cptr[s->n]);
  for (int i = 0; i < w->nP; ++i)
    for (int c = 0; c < 6; ++c)
      for (int r = 0; r <= c; ++r)
        *sky_at(s, 6 * i + r, 6 * i + c) = w->Hpp[36 * i + r * 6 + c] + (r == c ? lambda : 0.0);
  memset(w->coeff, 0, sizeof(double) * np6);
#pragma omp parallel for schedule(dynamic, 256)
  for (int l = 0; l < w->nL; ++l) {
    double D[9];
    for (int k = 0; k < 9; ++k) D[k] = w->Hll[9 * l + k] + ((k % 4 == 0) ? lambda : 0.0);
    double *Dinv = w->Dinv + 9 * l;
    o3_inverse(D, Dinv);
    const double *bl = w->b + np6 + 3 * l;
    double *db = w->db + 3 * l;
    for (int r = 0; r < 3; ++r) db[r] = Dinv[r * 3 + 0] * bl[0] + Dinv[r * 3 + 1] * bl[1] + Dinv[r * 3 + 2] * bl[2];
    for (int64_t ko = w->col_ptr[l]; ko < w->col_ptr[l + 1]; ++ko) {
      const double *Bi = w->blk + 18 * ko;
      double *BDinv = w->BDinv + 18 * ko;
      for (int r = 0; r < 6; ++r)
        for (int c = 0; c < 3; ++c)
          BDinv[r * 3 + c] = Bi[r * 3 + 0] * Dinv[0 * 3 + c] + Bi[r * 3 + 1] * Dinv[1 * 3 + c] + Bi[r * 3 + 2] * Dinv[2 * 3 + c];
    }
  }
#pragma omp parallel for schedule(dynamic, 4)
  for (int i2 = 0; i2 < w->nP; ++i2) {
    for (int64_t q = w->pl_ptr[i2]; q < w->pl_ptr[i2 + 1]; ++q) {
      const int l = w->pl_lm[q];
      const int64_t ki = w->pl_blk[q];
      const double *Bj = w->blk + 18 * ki, *db = w->db + 3 * l;
      for (int r = 0; r < 6; ++r) w->coeff[6 * i2 + r] += Bj[r * 3 + 0] * db[0] + Bj[r * 3 + 1] * db[1] + Bj[r * 3 + 2] * db[2];
      for (int64_t ko = w->col_ptr[l]; ko <= ki; ++ko) {
        const int i1 = w->blk_row[ko];
        const double *BDinv = w->BDinv + 18 * ko;
        for (int c = 0; c < 6; ++c)
          for (int r = 0; r < 6; ++r) {
            if (i1 == i2 && r > c) continue;
            double v = BDinv[r * 3 + 0] * Bj[c * 3 + 0] + BDinv[r * 3 + 1] * Bj[c * 3 + 1] + BDinv[r * 3 + 2] * Bj[c * 3 + 2];
            *sky_at(s, 6 * i1 + r, 6 * i2 + c) -= v;
          }
      }
    }
  }
  for (int i = 0; i < np6; ++i) w->bschur[i] = w->b[i] - w->coeff[i];
  if (!sky_factor(s)) return 0;
  sky_solve(s, w->bschur, w->x);
#pragma omp parallel for schedule(static)
  for (int l = 0; l < w->nL; ++l) {
    double cl[3] = {w->b[np6 + 3 * l], w->b[np6 + 3 * l + 1], w->b[np6 + 3 * l + 2]};
    for (int64_t k = w->col_ptr[l]; k < w->col_ptr[l + 1]; ++k) {
      const double *Bk = w->blk + 18 * k, *xp = w->x + 6 * w->blk_row[k];
      for (int c = 0; c < 3; ++c) {
        double acc = 0.0;
        for (int r = 0; r < 6; ++r) acc += Bk[r * 3 + c] * (-xp[r]);
        cl[c] += acc;
      }
    }
    const double *Dinv = w->Dinv + 9 * l;
    for (int r = 0; r < 3; ++r)
      w->x[np6 + 3 * l + r] = Dinv[r * 3 + 0] * cl[0] + Dinv[r * 3 + 1] * cl[1] + Dinv[r * 3 + 2] * cl[2];
  }
  return 1;
}
#endif

/* BlockSolver::solve (block_solver.hpp:369-483) on the lambda-damped system. */
static int schur_solve(lm_ws *w, double lambda) {
  skyline *s = &w->sky;
  const int np6 = 6 * w->nP;
#ifdef ORC_OMP
  return schur_solve_omp(w, lambda);
#endif
  /* _Hschur = _Hpp (damped diagonal blocks), off-diagonal pattern zero */
  memset(s->val, 0, sizeof(double) * s->cptr[s->n]);
  for (int i = 0; i < w->nP; ++i)
    for (int c = 0; c < 6; ++c)
      for (int r = 0; r <= c; ++r)
        *sky_at(s, 6 * i + r, 6 * i + c) = w->Hpp[36 * i + r * 6 + c] + (r == c ? lambda : 0.0);
  memset(w->coeff, 0, sizeof(double) * np6);
  for (int l = 0; l < w->nL; ++l) {
    double D[9];
    for (int k = 0; k < 9; ++k) D[k] = w->Hll[9 * l + k] + ((k % 4 == 0) ? lambda : 0.0);
    double *Dinv = w->Dinv + 9 * l;
    o3_inverse(D, Dinv);
    const double *bl = w->b + np6 + 3 * l;
    double db[3];
    for (int r = 0; r < 3; ++r) db[r] = Dinv[r * 3 + 0] * bl[0] + Dinv[r * 3 + 1] * bl[1] + Dinv[r * 3 + 2] * bl[2];
    for (int64_t ko = w->col_ptr[l]; ko < w->col_ptr[l + 1]; ++ko) {
      const int i1 = w->blk_row[ko];
      const double *Bi = w->blk + 18 * ko;
      double BDinv[18];
      for (int r = 0; r < 6; ++r)
        for (int c = 0; c < 3; ++c)
          BDinv[r * 3 + c] = Bi[r * 3 + 0] * Dinv[0 * 3 + c] + Bi[r * 3 + 1] * Dinv[1 * 3 + c] + Bi[r * 3 + 2] * Dinv[2 * 3 + c];
      for (int r = 0; r < 6; ++r)
        w->coeff[6 * i1 + r] += Bi[r * 3 + 0] * db[0] + Bi[r * 3 + 1] * db[1] + Bi[r * 3 + 2] * db[2];
      for (int64_t ki = ko; ki < w->col_ptr[l + 1]; ++ki) {
        const int i2 = w->blk_row[ki];
        const double *Bj = w->blk + 18 * ki;
        for (int c = 0; c < 6; ++c)
          for (int r = 0; r < 6; ++r) {
            if (i1 == i2 && r > c) continue; /* LDL^T reads the upper triangle only */
            double v = BDinv[r * 3 + 0] * Bj[c * 3 + 0] + BDinv[r * 3 + 1] * Bj[c * 3 + 1] + BDinv[r * 3 + 2] * Bj[c * 3 + 2];
            *sky_at(s, 6 * i1 + r, 6 * i2 + c) -= v;
          }
      }
    }
  }
  for (int i = 0; i < np6; ++i) w->bschur[i] = w->b[i] - w->coeff[i];
  if (!sky_factor(s)) return 0;
  sky_solve(s, w->bschur, w->x);
  /* landmarks: cl = bl - Hpl^T xp ; xl = Dinv cl */
  for (int l = 0; l < w->nL; ++l) {
    double cl[3] = {w->b[np6 + 3 * l], w->b[np6 + 3 * l + 1], w->b[np6 + 3 * l + 2]};
    for (int64_t k = w->col_ptr[l]; k < w->col_ptr[l + 1]; ++k) {
      const double *Bk = w->blk + 18 * k, *xp = w->x + 6 * w->blk_row[k];
      for (int c = 0; c < 3; ++c) {
        double acc = 0.0;
        for (int r = 0; r < 6; ++r) acc += Bk[r * 3 + c] * (-xp[r]);
        cl[c] += acc;
      }
    }
    const double *Dinv = w->Dinv + 9 * l;
    for (int r = 0; r < 3; ++r)
      w->x[np6 + 3 * l + r] = Dinv[r * 3 + 0] * cl[0] + Dinv[r * 3 + 1] * cl[1] + Dinv[r * 3 + 2] * cl[2];
  }
  return 1;
}

static void push_state(lm_ws *w) {
  orc_graph *g = w->g;
  for (int i = 0; i < w->nP; ++i) {
    memcpy(w->bk_q + 4 * i, g->pose_q + 4 * w->pose_of[i], 4 * sizeof(double));
    memcpy(w->bk_t + 3 * i, g->pose_t + 3 * w->pose_of[i], 3 * sizeof(double));
  }
#pragma omp parallel for schedule(static)
  for (int l = 0; l < w->nL; ++l) memcpy(w->bk_X + 3 * l, g->pt + 3 * w->pt_of[l], 3 * sizeof(double));
}

static void pop_state(lm_ws *w) {
  orc_graph *g = w->g;
  for (int i = 0; i < w->nP; ++i) {
    memcpy(g->pose_q + 4 * w->pose_of[i], w->bk_q + 4 * i, 4 * sizeof(double));
    memcpy(g->pose_t + 3 * w->pose_of[i], w->bk_t + 3 * i, 3 * sizeof(double));
  }
#pragma omp parallel for schedule(static)
  for (int l = 0; l < w->nL; ++l) memcpy(g->pt + 3 * w->pt_of[l], w->bk_X + 3 * l, 3 * sizeof(double));
}

/* SparseOptimizer::update (sparse_optimizer.cpp:422-435): poses then points. */
static void apply_update(lm_ws *w) {
  orc_graph *g = w->g;
  const int np6 = 6 * w->nP;
  for (int i = 0; i < w->nP; ++i) {
    int p = w->pose_of[i];
    ose3_oplus(g->pose_q + 4 * p, g->pose_t + 3 * p, w->x + 6 * i);
  }
#pragma omp parallel for schedule(static)
  for (int l = 0; l < w->nL; ++l) {
    double *X = g->pt + 3 * w->pt_of[l];
    X[0] += w->x[np6 + 3 * l]; X[1] += w->x[np6 + 3 * l + 1]; X[2] += w->x[np6 + 3 * l + 2];
  }
}

/* OptimizationAlgorithmLevenberg::computeScale (levenberg.cpp:182-189). */
static double compute_scale(lm_ws *w, double lambda) {
  const int dim = 6 * w->nP + 3 * w->nL;
  double scale = 0.;
  for (int j = 0; j < dim; ++j) scale += w->x[j] * (lambda * w->x[j] + w->b[j]);
  return scale;
}

static inline int stopped(const volatile uint8_t *stop) { return stop ? (*stop != 0) : 0; }

int orc_optimize(orc_graph *g, int level, int iterations, double user_lambda, const volatile uint8_t *stop,
                 orc_stats *st) {
  orc_stats dummy;
  if (!st) st = &dummy;
  memset(st, 0, sizeof(*st));
  lm_ws w;
  if (!ws_init(&w, g, level)) { ws_free(&w); return -1; } /* "0 vertices to optimize" */
  st->n_active_edges = (int)(w.n_ae + w.n_al);

  double lambda = -1., ni = 2.;
  int nbad = 0, its = 0, result = 0;
  for (int it = 0; it < iterations && !stopped(stop) && result == 0; ++it) {
    /* ---- OptimizationAlgorithmLevenberg::solve (levenberg.cpp:61-164) ---- */
    compute_active_errors(&w);
    double currentChi = active_robust_chi2(&w);
    double tempChi = currentChi;
    const double iniChi = currentChi;
    if (it == 0) st->chi2_begin = currentChi;
    build_system(&w);
    if (it == 0) {
      lambda = user_lambda > 0 ? user_lambda : 1e-5 * max_diagonal(&w);
      ni = 2;
      nbad = 0;
    }
    double rho = 0;
    int qmax = 0;
    do {
      push_state(&w);
      int ok2 = schur_solve(&w, lambda);
      if (!ok2) memset(w.x, 0, sizeof(double) * (6 * w.nP + 3 * w.nL));
      apply_update(&w);
      compute_active_errors(&w);
      tempChi = active_robust_chi2(&w);
      // a NaN chi2 (our sin / cos past 2^20 pi / 2, where glibc's stay finite and
      // the reference's chi2 is astronomically large) is a failed trial, as in
      // the library's lm_decide
      // (only when currentChi is finite: NaN input keeps g2o's rho = NaN)
      if (!ok2 || (isnan(tempChi) && isfinite(currentChi))) tempChi = DBL_MAX;
      rho = (currentChi - tempChi);
      double scale = compute_scale(&w, lambda);
      scale += 1e-3;
      rho /= scale;
      if (rho > 0 && isfinite(tempChi)) {
        double alpha = 1. - pow((2 * rho - 1), 3);
        alpha = fmin(alpha, 2. / 3.);
        double scaleFactor = fmax(1. / 3., alpha);
        lambda *= scaleFactor;
        ni = 2;
        currentChi = tempChi;
      } else {
        lambda *= ni;
        ni *= 2;
        pop_state(&w);
      }
      qmax++;
      st->trials++;
    } while (rho < 0 && qmax < 10 && !stopped(stop));

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
  st->iterations = its;
  st->result = result;
  ws_free(&w);
  return its;
}

/* ----------------------------------------------------- reference drivers */

int orc_local_ba(orc_graph *g, const volatile uint8_t *stop, uint8_t *outlier, orc_stats st[3]) {
  orc_stats tmp[3];
  if (!st) st = tmp;
  memset(st, 0, 3 * sizeof(orc_stats));
  /* g2oOptimizer.cc:923-928: abort before pass 1 leaves the map untouched */
  if (stopped(stop)) return 0;
  /* LiDAR edges are only added for pass 3 */
  for (int64_t e = 0; e < g->n_lid; ++e) g->lid_level[e] = 255;
  orc_optimize(g, 0, 5, 0.0, stop, &st[0]);
  int more = !stopped(stop);
  if (more) {
    /* :952-970 tag outliers from the stale chi2 and fresh depth, drop kernels */
    uint8_t *dp = malloc(g->n_obs ? g->n_obs : 1);
    orc_depth_positive(g, dp);
    for (int64_t e = 0; e < g->n_obs; ++e) {
      if (mono_chi2(g, e) > tag_threshold(g, e) || !dp[e]) g->obs_level[e] = 1;
      g->obs_delta[e] = 0.0;
    }
    free(dp);
    orc_optimize(g, 0, 10, 0.0, stop, &st[1]);
  }
  /* pass 3 (:1113-1114): LiDAR flat edges on the current KF join, 20 iterations */
  for (int64_t e = 0; e < g->n_lid; ++e) g->lid_level[e] = 0;
  orc_optimize(g, 0, 20, 0.0, stop, &st[2]);
  /* :1119-1136 final outlier tags */
  if (outlier) {
    uint8_t *dp = malloc(g->n_obs ? g->n_obs : 1);
    orc_depth_positive(g, dp);
    for (int64_t e = 0; e < g->n_obs; ++e) outlier[e] = (mono_chi2(g, e) > tag_threshold(g, e) || !dp[e]);
    free(dp);
  }
  return 1;
}

int orc_global_ba(orc_graph *g, int iterations, const volatile uint8_t *stop, orc_stats *st) {
  return orc_optimize(g, 0, iterations, 0.0, stop, st);
}

/* ------------------------------------------------- boundary conversions */

void orc_se3_from_Tcw_f32(const float T[16], double q[4], double t[3]) {
  double R[9];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) R[r * 3 + c] = (double)T[r * 4 + c];
  oq_from_mat(R, q);
  oq_normalize_rotation(q);
  for (int r = 0; r < 3; ++r) t[r] = (double)T[r * 4 + 3];
}

void orc_se3_to_Tcw_f32(const double q[4], const double t[3], float T[16]) {
  double R[9];
  oq_to_mat(q, R);
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c) T[r * 4 + c] = (float)R[r * 3 + c];
    T[r * 4 + 3] = (float)t[r];
  }
  T[12] = 0.f; T[13] = 0.f; T[14] = 0.f; T[15] = 1.f;
}

void orc_se3_exp(const double upd[6], double q[4], double t[3]) { ose3_exp(upd, q, t); }
void orc_se3_oplus(double q[4], double t[3], const double d[6]) { ose3_oplus(q, t, d); }
void orc_quat_rotate(const double q[4], const double v[3], double o[3]) { oq_rotate(q, v, o); }
