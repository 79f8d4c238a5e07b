/*
 * oracle.h — TEST INFRASTRUCTURE. CPU restatement of the reference's g2o
 * bundle-adjustment path (Levenberg–Marquardt + BlockSolver_6_3 Schur +
 * sparse LDL^T), used ONLY by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py as the checker. Never linked into the product.
 *
 * PARITY UNPINNED: the reference ships no tests, fixtures or golden vectors
 * for this path and cannot be compiled here (needs Eigen3,
 * OpenCV, PCL, ROS). The restatement is pinned by independent checks instead
 * (tests/test_oracle.py): central-difference Jacobians, Schur == dense normal
 * equations, noise-free convergence to ground truth.
 *
 * Semantics followed (all paths relative to /root/reference):
 *   LM control        Thirdparty/g2o/g2o/core/optimization_algorithm_levenberg.cpp:43-189
 *   optimize loop     Thirdparty/g2o/g2o/core/sparse_optimizer.cpp:354-419
 *   active set        sparse_optimizer.cpp:166-267 (level, all-fixed, index mapping)
 *   buildSystem       Thirdparty/g2o/g2o/core/block_solver.hpp:502-560
 *   Schur solve       block_solver.hpp:369-483
 *   set/restore diag  block_solver.hpp:564-604
 *   linear solve      Thirdparty/g2o/g2o/solvers/linear_solver_eigen.h:94-124
 *   mono edge         Thirdparty/g2o/g2o/types/types_six_dof_expmap.h:90-101, .cpp:103-147
 *   stereo edge       types_six_dof_expmap.h:112-145, .cpp:150-157 (float invz), :188-234
 *   binary quad form  Thirdparty/g2o/g2o/core/base_binary_edge.hpp:55-120
 *   LiDAR flat edge   types_six_dof_expmap.h:206-234; base_unary_edge.hpp:43-122
 *   Huber             Thirdparty/g2o/g2o/core/robust_kernel_impl.cpp:78-90
 *   local BA schedule src/backend/g2oOptimizer.cc:704-1191
 *   global BA         src/backend/g2oOptimizer.cc:80-362
 *   essential graph   g2oOptimizer.cc:1212-1534; types_seven_dof_expmap.h:48-122; sim3.h (eg_ref.c)
 */
#ifndef SQLM_ORACLE_H
#define SQLM_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_TRACE_MAX 256

typedef struct orc_graph {
  /* VertexSE3Expmap: vertex id = pose index (ids ascending = g2o id order). */
  int n_pose;
  double *pose_q;            /* [n_pose][4] qx qy qz qw (in/out)            */
  double *pose_t;            /* [n_pose][3]            (in/out)             */
  const uint8_t *pose_fixed; /* [n_pose] setFixed                           */
  const double *intr;        /* [n_pose][4] fx fy cx cy (edge copies)       */
  /* VertexSBAPointXYZ (marginalised), ids follow the poses. */
  int n_pt;
  double *pt;                /* [n_pt][3] (in/out)                          */
  /* EdgeSE3ProjectXYZ, internal id = index (insertion order). */
  int64_t n_obs;
  const int32_t *obs_pose, *obs_pt;
  const double *obs_uv;      /* [n_obs][2]                                  */
  const double *obs_info;    /* [n_obs] invSigma2 (information = I*info)    */
  double *obs_delta;         /* [n_obs] Huber delta, 0 = no kernel (in/out) */
  uint8_t *obs_level;        /* [n_obs] (in/out)                            */
  double *obs_err;           /* [n_obs][2] last computed _error (stale)     */
  /* EdgeLidarFlatPoint (unary), inserted after all mono edges. */
  int64_t n_lid;
  const int32_t *lid_pose;
  const double *lid_pc, *lid_pw, *lid_n; /* [n_lid][3] camera pt, world pt, normal */
  const double *lid_info;    /* [n_lid] information (1x1)                   */
  uint8_t *lid_level;        /* [n_lid] (in/out)                            */
  double *lid_err;           /* [n_lid] last computed _error                */
  /* EdgeStereoSE3ProjectXYZ: an edge with obs_ur[e] >= 0 is a stereo edge
   * (3-D error u, v, u_r; information = I3*info), else mono. */
  const double *obs_ur;      /* [n_obs] right-image u, NULL = all mono      */
  const double *pose_bf;     /* [n_pose] bf (mbf) of the edge's keyframe     */
  double *obs_err3;          /* [n_obs] third error component (stereo), may be NULL if no stereo */
} orc_graph;

typedef struct orc_stats {
  int iterations;            /* value optimize() returns                    */
  int trials;                /* total inner LM trials                       */
  int result;                /* last SolverResult: 0 OK, 1 Terminate, 2 Fail */
  int n_active_edges;
  double chi2_begin;         /* robust chi2 at iteration 0 start            */
  double chi2_end;           /* currentChi after the last iteration         */
  double lambda_end;
  int trace_len;
  double trace_chi2[ORC_TRACE_MAX];   /* currentChi after iteration i       */
  double trace_lambda[ORC_TRACE_MAX]; /* lambda after iteration i           */
  int trace_trials[ORC_TRACE_MAX];
} orc_stats;

/* initializeOptimization(level); optimize(iterations). user_lambda > 0 sets
 * setUserLambdaInit. stop may be NULL. Returns optimize()'s return value. */
int orc_optimize(orc_graph *g, int level, int iterations, double user_lambda,
                 const volatile uint8_t *stop, orc_stats *st);

/* EdgeSE3ProjectXYZ::computeError for every mono edge (writes obs_err). */
void orc_compute_mono_errors(orc_graph *g);
/* e->chi2() from the stored (possibly stale) error. */
void orc_edge_chi2(const orc_graph *g, double *out);
/* e->isDepthPositive() at the current estimate. */
void orc_depth_positive(const orc_graph *g, uint8_t *out);

/* g2oOptimizer::LocalBundleAdjustment schedule on an assembled graph
 * (g2oOptimizer.cc:923-1136). obs_delta must hold the pass-1 Huber deltas.
 * LiDAR edges (if any) join in pass 3. outlier[n_obs] receives the final
 * chi2>5.991 || depth<=0 tags. Returns 1 if it ran, 0 if aborted before pass 1. */
int orc_local_ba(orc_graph *g, const volatile uint8_t *stop, uint8_t *outlier, orc_stats st[3]);

/* g2oOptimizer::BundleAdjustment (g2oOptimizer.cc:110-362): optimize(level 0, n). */
int orc_global_ba(orc_graph *g, int iterations, const volatile uint8_t *stop, orc_stats *st);
/* OpenMP threads of the loops of this build (1 for the serial build) */
int orc_omp_threads(void);

/* Converter::toSE3Quat (Converter.cc:55-68): float 4x4 Tcw -> q (x,y,z,w), t. */
void orc_se3_from_Tcw_f32(const float T[16], double q[4], double t[3]);
/* Converter::toCvMat(SE3Quat) (Converter.cc:73-79,98-109): q,t -> float 4x4. */
void orc_se3_to_Tcw_f32(const double q[4], const double t[3], float T[16]);

/* ---- essential graph (eg_ref.c) ------------------------------------------
 * VertexSim3Expmap per keyframe, S = [qx qy qz qw tx ty tz s] (Sim3 S_iw),
 * EdgeSim3 e: vertex 0 = ei[e], vertex 1 = ej[e], measurement S_ji,
 * error log(S_ji * S_i * S_j^-1), information Omega (NULL = identity). */
typedef struct orc_eg_graph {
  int n_kf;
  double *Siw;               /* [n_kf][8] (in/out)                          */
  const uint8_t *fixed;      /* [n_kf] setFixed (the loop keyframe)         */
  int fix_scale;             /* VertexSim3Expmap::_fix_scale (bFixScale)    */
  int64_t n_edge;
  const int32_t *ei, *ej;    /* [n_edge]                                    */
  const double *Sji;         /* [n_edge][8]                                 */
  const double *info;        /* [n_edge][49] row-major or NULL = identity   */
  double *err;               /* [n_edge][7] last computed _error            */
} orc_eg_graph;

/* optimizer.optimize(iterations) with setUserLambdaInit(user_lambda) (the
 * reference uses 1e-16, g2oOptimizer.cc:1226). Returns iterations done. */
int orc_eg_optimize(orc_eg_graph *g, int iterations, double user_lambda, const volatile uint8_t *stop,
                    orc_stats *st);
void orc_sim3_from_update(const double u[7], double S[8]);
void orc_sim3_log(const double S[8], double out[7]);
/* include/sqlm_libm.h on n arguments: fn 0 exp, 1 log, 2 sin, 3 cos, 4 acos */
void orc_libm(int fn, const double *x, double *y, int n);
void orc_sim3_mul(const double a[8], const double b[8], double out[8]);
void orc_sim3_inverse(const double a[8], double out[8]);
void orc_eg_edge_error(const double Si[8], const double Sj[8], const double C[8], double e[7]);
void orc_eg_edge_jacobians(const double Si[8], const double Sj[8], const double C[8], int fix_scale, int free_i,
                           int free_j, double Ji[49], double Jj[49]);

/* Building blocks exposed for the known-answer tests. */
void orc_se3_exp(const double upd[6], double q[4], double t[3]);
void orc_se3_oplus(double q[4], double t[3], const double d[6]);
void orc_quat_rotate(const double q[4], const double v[3], double o[3]);
void orc_mono_jacobians(const double q[4], const double t[3], const double intr[4],
                        const double X[3], double Jl[6], double Jp[12]);
/* EdgeStereoSE3ProjectXYZ::cam_project / linearizeOplus: proj[3], Jl 3x3, Jp 3x6. */
void orc_stereo_project(const double q[4], const double t[3], const double intr[4], double bf,
                        const double X[3], double proj[3]);
void orc_stereo_jacobians(const double q[4], const double t[3], const double intr[4], double bf,
                          const double X[3], double Jl[9], double Jp[18]);
double orc_lidar_error(const double q[4], const double t[3], const double pc[3],
                       const double pw[3], const double n[3]);
void orc_lidar_jacobian(const double q[4], const double t[3], const double pc[3],
                        const double pw[3], const double n[3], double J[6]);

#ifdef __cplusplus
}
#endif
#endif
