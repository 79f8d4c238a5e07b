/*
 * sqrtlm.h — C ABI of the MI355X square-root Levenberg–Marquardt
 * bundle-adjustment backend (libsqrtlm.so).
 *
 * Drop-in seam: the reference dispatches every BA call through the static
 * façade `Optimizer` (include/backend/Optimizer.h:42-71, solver switch
 * src/backend/Optimizer.cc:26-28) into `g2oOptimizer`, which assembles a g2o
 * graph and calls `SparseOptimizer::optimize`. A host adapter (see
 * INTEGRATION.md) replaces that g2o graph with the plain arrays below and
 * calls this library instead; the Tracking / LocalMapping / LoopClosing
 * threads are untouched.
 *
 * Conventions (all mirror the g2o path):
 *   - poses are T_cw as SE3Quat: q = (qx,qy,qz,qw) unit, qw >= 0, t (3);
 *     tangent order [omega; upsilon], left update T <- exp(d) T
 *     (Thirdparty/g2o/g2o/types/types_six_dof_expmap.h:73-76);
 *   - observations are EdgeSE3ProjectXYZ in insertion order (edge id = index);
 *     error = obs - project(T X) (types_six_dof_expmap.h:90-95);
 *     information = I * info; Huber delta per edge, 0 = no robust kernel;
 *   - every call is FP64 end to end.
 * Error model: every entry point returns an int status (SQLM_OK = 0, < 0 on
 * error); nothing throws across the ABI. A non-SPD damped system is NOT an
 * error: the LM step is rejected, as g2o does (levenberg.cpp:126-127).
 * Threading: one context per calling thread (LBA, loop-closing and GBA threads
 * may each own one); a context owns its HIP stream and device memory.
 */
#ifndef SQRTLM_H
#define SQRTLM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SQLM_OK 0
#define SQLM_ERR_INVALID_ARG (-1)
#define SQLM_ERR_HIP (-2)
#define SQLM_ERR_NOT_SPD (-3)
#define SQLM_ERR_OOM (-4)
#define SQLM_ERR_ABORTED (-5)
#define SQLM_ERR_NO_DEVICE (-6)
#define SQLM_ERR_STATE (-7)
#define SQLM_ERR_UNSUPPORTED (-8)
#define SQLM_ERR_COMM (-9)

#define SQLM_TRACE_MAX 256

typedef struct sqlm_ctx sqlm_ctx;

/* Per optimize() statistics; field meaning follows g2o's loop
 * (sparse_optimizer.cpp:354-419, optimization_algorithm_levenberg.cpp:61-164). */
typedef struct sqlm_stats {
  int iterations;     /* value SparseOptimizer::optimize returns               */
  int trials;         /* inner LM trials, all iterations                         */
  int result;         /* last SolverResult: 0 OK, 1 Terminate, 2 Fail          */
  int n_active_edges;
  double chi2_begin;  /* robust chi2 at the start of iteration 0               */
  double chi2_end;    /* currentChi after the last iteration                   */
  double lambda_end;
  int trace_len;
  double trace_chi2[SQLM_TRACE_MAX];
  double trace_lambda[SQLM_TRACE_MAX];
  int trace_trials[SQLM_TRACE_MAX];
  /* wall time split (ms, host clock around stream syncs) */
  double ms_total, ms_setup, ms_linearize, ms_trials;
} sqlm_stats;

const char *sqlm_version(void);
const char *sqlm_status_string(int status);

/* Context / device. Replaces `new g2o::SparseOptimizer` + solver setup
 * (g2oOptimizer.cc:784-798). device_id < 0 picks the current HIP device. */
int sqlm_ctx_create(int device_id, sqlm_ctx **out);
int sqlm_ctx_destroy(sqlm_ctx *ctx);

/* Graph assembly: replaces the addVertex/addEdge loops of
 * g2oOptimizer::LocalBundleAdjustment (g2oOptimizer.cc:805-912) and
 * ::BundleAdjustment (:142-296). Arrays are copied (caller keeps ownership).
 *   pose_q [n_pose][4], pose_t [n_pose][3], pose_fixed [n_pose], intr [n_pose][4]
 *   pt [n_pt][3]
 *   obs_pose/obs_pt [n_obs], obs_uv [n_obs][2], obs_info [n_obs] (invSigma2),
 *   obs_delta [n_obs] Huber delta (0 = none; NULL = none), obs_level [n_obs] (NULL = 0). */
int sqlm_set_problem(sqlm_ctx *ctx, int n_pose, const double *pose_q, const double *pose_t,
                     const uint8_t *pose_fixed, const double *intr, int n_pt, const double *pt,
                     int64_t n_obs, const int32_t *obs_pose, const int32_t *obs_pt, const double *obs_uv,
                     const double *obs_info, const double *obs_delta, const uint8_t *obs_level);

/* EdgeStereoSE3ProjectXYZ (types_six_dof_expmap.h:112-145): edges with
 * obs_ur[e] >= 0 become stereo edges, error (u, v, u_right) - cam_project
 * (float invz, float bf*invz, .cpp:150-157), information info*I3; the Huber
 * delta set for the edge applies to its 3-D chi2. pose_bf [n_pose] = mbf.
 * obs_ur = NULL (or all < 0) makes every edge mono again. Call after
 * sqlm_set_problem (which resets it). GBA stereo branch: g2oOptimizer.cc:247-281. */
int sqlm_set_stereo(sqlm_ctx *ctx, const double *obs_ur, const double *pose_bf);

/* EdgeLidarFlatPoint unary pose edges (types_six_dof_expmap.h:206-234), added
 * after the mono edges (g2oOptimizer.cc:1062-1070). Level 0, no kernel. */
int sqlm_set_lidar(sqlm_ctx *ctx, int64_t n, const int32_t *pose, const double *p_cam,
                   const double *p_world, const double *normal, const double *info);

/* e->setLevel / e->setRobustKernel for every mono edge (NULL delta = none). */
int sqlm_set_edge_level(sqlm_ctx *ctx, const uint8_t *level);
int sqlm_set_robust(sqlm_ctx *ctx, const double *delta);
int sqlm_set_lidar_level(sqlm_ctx *ctx, const uint8_t *level);

/* optimizer.initializeOptimization(level); optimizer.optimize(iterations).
 * user_lambda > 0 mirrors setUserLambdaInit. stop mirrors setForceStopFlag
 * (polled before each iteration and each trial; may be NULL).
 * *n_iter receives optimize()'s return value. */
int sqlm_optimize(sqlm_ctx *ctx, int level, int iterations, double user_lambda,
                  const volatile uint8_t *stop, sqlm_stats *stats, int *n_iter);

/* The whole g2oOptimizer::LocalBundleAdjustment schedule on the set problem
 * (g2oOptimizer.cc:923-1136): pass 1 optimize(5) with the set Huber kernels;
 * unless stopped, tag chi2 > 5.991 || depth <= 0 edges to level 1, drop the
 * kernels, pass 2 optimize(10); pass 3 optimize(20) with the LiDAR edges;
 * outlier[n_obs] receives the final erase tags. *ran = 0 when the stop flag
 * was already set (the reference returns before pass 1). */
int sqlm_local_ba(sqlm_ctx *ctx, const volatile uint8_t *stop, uint8_t *outlier,
                  sqlm_stats stats[3], int *ran);

/* g2oOptimizer::BundleAdjustment core (g2oOptimizer.cc:299-301): optimize
 * level 0 for `iterations`, kernels as set. */
int sqlm_global_ba(sqlm_ctx *ctx, int iterations, const volatile uint8_t *stop, sqlm_stats *stats,
                   int *n_iter);

/* Essential graph: g2oOptimizer::OptimizeEssentialGraph (g2oOptimizer.cc:1212-1534).
 * Vertices VertexSim3Expmap (types_seven_dof_expmap.h:48-94), one per keyframe in
 * g2o id order: Siw [n_kf][8] = qx qy qz qw tx ty tz s (Sim3 S_iw), fixed [n_kf]
 * (the loop keyframe), fix_scale = bFixScale (VertexSim3Expmap::_fix_scale).
 * Edges EdgeSim3 (:99-122) in insertion order: vertex 0 = edge_i, vertex 1 =
 * edge_j, measurement Sji [n_edge][8], error log(S_ji * S_i * S_j^-1),
 * information info [n_edge][49] row-major (NULL = identity, as the reference).
 * Numeric Jacobians (central differences, delta 1e-9, base_binary_edge.hpp:131-205). */
int sqlm_eg_set_problem(sqlm_ctx *ctx, int n_kf, const double *Siw, const uint8_t *fixed, int fix_scale,
                        int64_t n_edge, const int32_t *edge_i, const int32_t *edge_j, const double *Sji,
                        const double *info);
/* optimizer.setUserLambdaInit(user_lambda) (the reference: 1e-16); optimize(iterations). */
int sqlm_eg_optimize(sqlm_ctx *ctx, int iterations, double user_lambda, const volatile uint8_t *stop,
                     sqlm_stats *stats, int *n_iter);
int sqlm_eg_get_poses(sqlm_ctx *ctx, double *Siw);
/* e->chi2() from the last computed error (g2o semantics). */
int sqlm_eg_get_edge_chi2(sqlm_ctx *ctx, double *chi2);
/* The numeric Jacobians EdgeSim3::linearizeOplus computes at the current
 * estimates (BaseBinaryEdge, base_binary_edge.hpp:131-205: central differences
 * through oplus, delta 1e-9), on the GPU with the arithmetic of the optimizer's
 * k_eg_linearize: J [n_edge][2][7][7] row-major, [e][0] = d e / d S_i,
 * [e][1] = d e / d S_j, zero for a fixed vertex. Diagnostics / parity tests. */
int sqlm_eg_get_jacobians(sqlm_ctx *ctx, double *J);

/* Results (write-back inputs, g2oOptimizer.cc:1167-1189, :306-360). */
int sqlm_get_poses(sqlm_ctx *ctx, double *pose_q, double *pose_t);
int sqlm_get_points(sqlm_ctx *ctx, double *pt);
/* e->chi2() from the last computed error (g2o semantics: may belong to a
 * rejected trial, and level-1 edges keep their pass-1 value). */
int sqlm_get_edge_chi2(sqlm_ctx *ctx, double *chi2);
/* e->isDepthPositive() evaluated at the current estimate. */
int sqlm_get_edge_depth_positive(sqlm_ctx *ctx, uint8_t *positive);
int sqlm_get_edge_level(sqlm_ctx *ctx, uint8_t *level);

/* Layout the last optimize() chose for the reduced camera system S (the
 * replacement of SimplicialLDLT + AMD, linear_solver_eigen.h:60-75):
 * out[0] = 0 none (no free camera), 1 banded (block cyclic reduction),
 * 2 band + border (loop closure: cameras coupled far off the band eliminated
 * last, launch_arrow_solve), 3 dense Cholesky; out[1] = cameras per
 * superblock B, out[2] = superblocks p, out[3] = superblock rows n,
 * out[4] = border cameras, out[5] = border rows (16-padded), out[6] = free
 * cameras, out[7] = superblocks carrying band-border coupling. */
int sqlm_get_rcs_layout(sqlm_ctx *ctx, int out[8]);

/* Device paths the last optimize() ran (introspection for tests and tools; no
 * reference counterpart): out[0] = 1 if the observation inputs (u, v,
 * invSigma2, Huber delta) were all float32 values and travelled as float4,
 * 0 if they took the double arrays; out[1] = reduced-camera solve: 0 none,
 * 1 cyclic reduction (per-level launches), 3 band + border, 4 dense
 * Cholesky (2 and 5 retired); out[2..7] = 0 (reserved). */
int sqlm_get_exec_info(sqlm_ctx *ctx, int out[8]);

/* Converter::toSE3Quat / toCvMat(SE3Quat) (src/utils/Converter.cc:55-79,98-109):
 * float32 row-major 4x4 T_cw <-> (q, t). */
void sqlm_pose_from_Tcw_f32(const float T[16], double q[4], double t[3]);
void sqlm_pose_to_Tcw_f32(const double q[4], const double t[3], float T[16]);

/* Multi-GPU: landmark-sharded global BA, one context per rank. Each rank
 * calls sqlm_set_problem with ALL poses and ITS landmarks/observations; the
 * reduced camera system, gradient and scalars are summed over RCCL (xGMI).
 * Rank 0 creates the id; the caller broadcasts it (e.g. torch.distributed). */
int sqlm_comm_id_size(void);
int sqlm_comm_get_unique_id(char *id_out);
int sqlm_ctx_set_comm(sqlm_ctx *ctx, const char *unique_id, int rank, int nranks);
/* What the context's exchange actually runs on: *transport = SQLM_COMM_NONE,
 * _RCCL, _RCCL_SELFLOOP or _HOST; for RCCL *rank / *nranks are the ones the
 * communicator itself reports (ncclCommUserRank / ncclCommCount), otherwise
 * the ones the caller set. No reference counterpart (bench / test hook). */
#define SQLM_COMM_NONE 0
#define SQLM_COMM_RCCL 1
#define SQLM_COMM_RCCL_SELFLOOP 2
#define SQLM_COMM_HOST 3
int sqlm_ctx_comm_info(const sqlm_ctx *ctx, int *transport, int *rank, int *nranks);
/* RCCL transport checks on ONE GPU (no reference counterpart; test hooks).
 * sqlm_ctx_set_comm_selfloop: a one-rank RCCL communicator on which the
 * context takes the sharded code path (every all-reduce, the rank-0 gather and
 * the dx broadcast run through RCCL with one rank).
 * sqlm_comm_selftest: on `device`, a one-rank communicator drives the three
 * exchange primitives — a grouped send/recv to self of `count` doubles, an
 * in-place broadcast and sum / max all-reduces (f64, i32, u8) — and writes
 * the largest deviation from the expected buffers to *max_err. */
int sqlm_ctx_set_comm_selfloop(sqlm_ctx *ctx, const char *unique_id);
int sqlm_comm_selftest(int device, const char *unique_id, int64_t count, double *max_err);

/* Same sharded algorithm over a caller-provided host collective (for example
 * torch.distributed gloo): the library stages each exchange through host
 * memory and calls fn(user, buf, count, dtype, op), which must all-reduce
 * `count` elements of `buf` in place across the ranks and return 0. Used to
 * run several ranks on one GPU (tests); production uses sqlm_ctx_set_comm.
 * LiDAR unary edges are owned by rank 0 (ignored on other ranks). */
#define SQLM_DT_F64 0
#define SQLM_DT_U8 1
#define SQLM_DT_I32 2
#define SQLM_OP_SUM 0
#define SQLM_OP_MAX 1
typedef int (*sqlm_allreduce_fn)(void *user, void *buf, int64_t count, int dtype, int op);
int sqlm_ctx_set_host_comm(sqlm_ctx *ctx, int rank, int nranks, sqlm_allreduce_fn fn, void *user);
/* Point-to-point half of the host transport (the per-trial gather of the
 * reduced camera system to rank 0 and the broadcast of its solution):
 * fn(user, buf, count, dtype, peer, op) with op SQLM_P2P_SEND (buf -> peer),
 * SQLM_P2P_RECV (peer -> buf) or SQLM_P2P_BCAST (in place from root = peer).
 * Required with sqlm_ctx_set_host_comm for nranks > 1; set it first. */
#define SQLM_P2P_SEND 0
#define SQLM_P2P_RECV 1
#define SQLM_P2P_BCAST 2
typedef int (*sqlm_p2p_fn)(void *user, void *buf, int64_t count, int dtype, int peer, int op);
int sqlm_ctx_set_host_p2p(sqlm_ctx *ctx, sqlm_p2p_fn fn, void *user);

/* Device-resident benchmarking hooks: time `n` LM iterations on the set
 * problem with data already in HBM (bench.py). Per-kernel averaged durations
 * (HIP events on the context stream) are returned through kernel_ms
 * [SQLM_NKERNEL_TIMERS] when non-NULL. */
#define SQLM_NKERNEL_TIMERS 9
int sqlm_bench_iterations(sqlm_ctx *ctx, int warmup, int n, double *ms_per_iter, double *kernel_ms,
                          sqlm_stats *stats);
const char *sqlm_kernel_timer_name(int i);

#ifdef __cplusplus
}
#endif
#endif
