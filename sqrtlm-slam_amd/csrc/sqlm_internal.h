// sqlm_internal.h — shared between the host LM driver (sqlm_api.cpp) and the
// HIP kernels (sqlm_kernels.hip). Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cfloat>
#include <cmath>
#include <vector>

#include "../../include/sqrtlm.h"

namespace sqlm {

#ifndef SQLM_TILE_MAXCAMS
#define SQLM_TILE_MAXCAMS 24
#endif
#ifndef SQLM_TILE_MAXLM
#define SQLM_TILE_MAXLM 128
#endif
// tile window cap of the greedy cut (a single landmark may exceed it up to kTileHardCams)
constexpr int kTileMaxCams = SQLM_TILE_MAXCAMS, kTileHardCams = 24, kTileMaxLm = SQLM_TILE_MAXLM, kTileMaxK = 1 << 20;
constexpr int kTileNtMax = (6 * kTileHardCams + 15) / 16;  // widest tile class (9)

constexpr int kBlock = 256;

// ---- Levenberg-Marquardt control (optimization_algorithm_levenberg.cpp:61-164
// inside sparse_optimizer.cpp:376-414), host side -------------------------
struct LMCtl {
  double lambda, ni, currentChi, iniChi;
  double chi2_end, lambda_end;
  int qmax, nbad, its, result, trials, iterations, bench;
  int done;  // the run is over
  double trace_chi2[SQLM_TRACE_MAX], trace_lambda[SQLM_TRACE_MAX];
  int trace_trials[SQLM_TRACE_MAX];
};

// One trial's outcome (computeActiveErrors chi2 at the trial state, the
// predicted reduction scale, the solve status) applied to the LM state:
// levenberg.cpp:110-160 (rho, lambda update, accept) and the iteration end of
// sparse_optimizer.cpp:376-414 with levenberg.cpp:150-163 (Terminate on
// qmax == 10 or rho == 0, Raul's criterion). Returns true if the trial state
// is accepted (the caller swaps the state buffers).
inline bool lm_decide(LMCtl &c, double chi_cur, double chi_new, double scale, bool ok, bool stop) {
  if (c.qmax == 0 && c.its > 0) {  // a fresh linearization's computeActiveErrors
    c.currentChi = chi_cur;
    c.iniChi = chi_cur;
  }
  // a NaN trial chi2 is a failed trial: our sin / cos (include/sqlm_libm.h)
  // return NaN past fdlibm's medium-range reduction (a rotation step of
  // > 2^20 pi / 2 rad), where glibc's stay finite and the reference's chi2 is
  // astronomically large -- rejected with a larger lambda either way. Only
  // when the current chi2 is finite: NaN input (a NaN measurement or state)
  // keeps g2o's arithmetic, rho = NaN, and the iteration ends after this one
  // trial (levenberg.cpp:124-160; tests/test_gpu_parity.py::test_nan_measurement)
  const double tempChi = ok && !(std::isnan(chi_new) && std::isfinite(c.currentChi)) ? chi_new : DBL_MAX;
  double rho = c.currentChi - tempChi;
  const double scl = (ok ? scale : 0.0) + 1e-3;
  rho /= scl;
  bool acc = false;
  if (rho > 0 && std::isfinite(tempChi)) {
    double alpha = 1. - std::pow(2 * rho - 1, 3);  // levenberg.cpp:136, the same libm call
    alpha = (2. / 3. < alpha) ? 2. / 3. : alpha;         // std::min(alpha, 2/3)
    const double sf = (1. / 3. < alpha) ? alpha : 1. / 3.;  // std::max(1/3, alpha)
    c.lambda *= sf;
    c.ni = 2;
    c.currentChi = tempChi;
    acc = true;
  } else {
    c.lambda *= c.ni;
    c.ni *= 2;
  }
  c.qmax++;
  c.trials++;
  if (!(rho < 0 && c.qmax < 10 && !stop)) {  // the iteration ends
    if (c.qmax == 10 || rho == 0) {
      c.result = 1;
    } else {
      if ((c.iniChi - c.currentChi) * 1e3 < c.iniChi) c.nbad++;
      else c.nbad = 0;
      if (c.nbad >= 3) c.result = 1;
    }
    if (c.its < SQLM_TRACE_MAX) {
      c.trace_chi2[c.its] = c.currentChi;
      c.trace_lambda[c.its] = c.lambda;
      c.trace_trials[c.its] = c.qmax;
    }
    c.chi2_end = c.currentChi;
    c.lambda_end = c.lambda;
    c.its++;
    c.qmax = 0;
    c.done = c.its >= c.iterations || stop || (c.result != 0 && !c.bench);
  }
  return acc;
}

// HBM layout of one optimize() call. Everything is FP64 except indices.
//   poses     : all problem poses, index = pose id (ascending id = g2o order)
//   landmarks : ACTIVE points only, in "device slot" order: bucketed by track
//               length into segments of width W in {2,4,8,16,32,64}
//   obs       : ACTIVE mono edges only, contiguous per landmark slot
//   cameras   : free active poses, hidx = g2o hessianIndex order
struct DevProblem {
  int n_pose = 0, nP = 0, nL = 0;
  int sharded = 0, rank = 0;               // landmark-sharded multi-GPU run
  int64_t nE = 0;
  // pose state, double-buffered (cur = 0 / trial = 1 swapped on accept)
  double *pose_qt[2] = {nullptr, nullptr};  // [n_pose][8]  qx qy qz qw tx ty tz 0
  double *pose_rt[2] = {nullptr, nullptr};  // [n_pose][16] R(9) t(3) fx fy cx cy
  double *intr = nullptr;                   // [n_pose][4]
  int *pose_hidx = nullptr;                 // [n_pose] free hidx or -1
  int *hidx_pose = nullptr;                 // [nP]
  // landmarks
  double *X[2] = {nullptr, nullptr};        // [nL][4]
  int *lm_begin = nullptr;                  // [nL+1]
  double *lm_R = nullptr;                   // [nL][8]  R upper (6) of QR(J_l)
  double *lm_b = nullptr;                   // [nL][4]  b_l = -J_l^T W r
  // speculative linearization at the trial state (k_landmark_update<SPEC>),
  // swapped with lm_R / lm_b / obs_s / Hpp / bp when the trial is accepted
  double *lm_R_nx = nullptr, *lm_b_nx = nullptr, *obs_s_nx = nullptr, *Hpp_nx = nullptr, *bp_nx = nullptr;
  double *lm_M = nullptr;                   // [nL][8]  (H_ll + lambda I)^-1, sym (6)
  double *lm_v = nullptr;                   // [nL][4]  M b_l
  // observations
  int *obs_lm = nullptr;                    // [nE] landmark slot
  int *obs_cam = nullptr;                   // [nE] pose id
  int *obs_camh = nullptr;                  // [nE] free hidx or -1
  double *obs_uv = nullptr;                 // [nE][2]
  double *obs_info = nullptr;               // [nE]
  double *obs_delta = nullptr;              // [nE] Huber delta, 0 = none
  // obs_f32: every u, v, info and delta of the problem is a float32 value (the
  // reference's inputs are: kpUn.pt, mvInvLevelSigma2, the Huber thresholds),
  // so they travel as one float4 per edge (u v info delta, 16 B instead of 32 B
  // in three loads) and widen to the same doubles; obs_uv / info / delta null
  int obs_f32 = 0;
  float *obs_q = nullptr;                   // [nE][4] (obs_f32)
  float *cam_q = nullptr;                   // [cam_obs][4] camera order (obs_f32)
  double *obs_s = nullptr;                  // [nE] sqrt(rho' info) at the linearization point
  double *obs_P = nullptr;                  // [18][nE] H_lp blocks, SoA: row-kernel fallback only (else null)
  double *obs_err = nullptr;                // [nE][2] last computed error (g2o _error)
  // stereo edges (EdgeStereoSE3ProjectXYZ): has_stereo selects the ST kernels
  int has_stereo = 0;
  double *obs_ur = nullptr;                 // [nE] right-image u, < 0 = mono edge
  double *obs_err3 = nullptr;               // [nE] third error component (0 for mono)
  double *pose_bf = nullptr;                // [n_pose] bf
  double *cam_ur = nullptr;                 // [cam_obs] obs_ur in camera order
  // cameras
  int *cam_obs_ptr = nullptr;               // [nP+1]
  int *cam_obs = nullptr;                   // device obs ids per camera, landmark order
  int *cam_slot = nullptr;                  // [cam_obs] landmark slot, camera order (camera pass)
  double *cam_uv = nullptr;                 // [cam_obs][4] u v info delta, camera order
  double *Hpp = nullptr;                    // [nP][36]
  double *bp = nullptr;                     // [nP][8]
  // lidar unary edges (grouped by camera)
  int64_t nLid = 0;
  int *lid_cam_ptr = nullptr;               // [nP+1]
  double *lid_data = nullptr;               // [nLid][12] pc(3) pw(3) n(3) info pad pad
  int *lid_pose = nullptr;                  // [nLid]
  double *lid_err = nullptr;                // [nLid]
  // reduced camera system, BSR upper, row i = free camera i
  int64_t nnzb = 0;
  int *s_row_ptr = nullptr;                 // [nP+1]
  int *s_col = nullptr;                     // [nnzb]
  int *s_row = nullptr;                     // [nnzb] block row (direct CR assembly)
  double *S = nullptr;                      // [nnzb][36]
  double *g = nullptr;                      // [6 nP]
  double *dx = nullptr;                     // [6 nP + 1] (+ the solve flag in sharded runs)
  double *hdiag = nullptr;                  // [6 nP] pose Hessian diagonals (sharded lambda_0)
  double *xstage = nullptr;                 // rank 0 of a sharded run: gathered S / g row ranges
  // dense path (S not block-banded enough for the CR solver, e.g. a real LBA
  // window in keyframe-id order): n_pad = 6 nP rounded up to kCRMaxN
  int dense_n = 0;
  double *dense = nullptr;                  // [n_pad][n_pad] A (lower), factored in place
  double *dense_L = nullptr;                // [n_pad][n_pad] L
  double *dense_Linv = nullptr;             // [n_pad / kCRMaxN][kCRMaxN][kCRMaxN]
  double *dense_r = nullptr, *dense_x = nullptr;  // [n_pad]
  // tiled RCS assembly (landmark tiles with a small camera window)
  int n_tiles = 0;
  // tiles grouped by accumulator width nt = ceil(6 cp / 16) (one launch per
  // class, compiled for that width); tile_order[cls_off[nt] ..] = their ids
  int *tile_order = nullptr;
  int tile_cls_off[kTileNtMax + 2] = {}, tile_cls_cnt[kTileNtMax + 1] = {};
  int *tile_lm_ptr = nullptr;               // [T+1] landmark slot ranges
  int *tile_cam_ptr = nullptr;              // [T+1] into tile_cams / g partials
  int *tile_cams = nullptr;                 // free hidx, sorted within a tile
  int64_t *tile_part_ptr = nullptr;         // [T+1] offset (doubles) of the tile's ld x ld partial
  int64_t *tile_gpart_ptr = nullptr;        // [T+1] offset (doubles) of the tile's g partial
  int *tile_ld = nullptr;                   // [T] 16 * ceil(6 cp / 16)
  int2 *lm_urange = nullptr;                // [nL] local camera span (min, max), -1 if none free
  int *obs_local = nullptr;                 // [nE] local camera index in its tile (-1 fixed)
  double *part = nullptr;                   // tile partial Gram matrices
  double *gpart = nullptr;                  // tile partial g
  int *red_ptr = nullptr;                   // [nnzb+1] S block -> contributions
  int64_t *red_off = nullptr;               //   offset in part of the contribution's 36-double block
  int *gred_ptr = nullptr;                  // [nP+1] camera -> contributions
  int64_t *gred_off = nullptr;              //   offset in gpart of the contribution's 6 doubles
  // S blocks / g rows with more than kRedLong contributions (loop-closure
  // cameras: hundreds) are summed by a whole workgroup each
  int n_long_s = 0, n_long_g = 0;
  // per-landmark kernels: pose id range [x, y] of each block tile's
  // observations (tiles of kBlock / W consecutive slots, buckets concatenated)
  int2 *upd_rng = nullptr;
  int *long_s = nullptr, *long_g = nullptr;
  int tile_dups = 0;                        // some landmark observed twice by one camera
  int tile_maxk = 0;                        // longest track (staging fast path needs <= kTileFastK = 64)
  int tile_prod = 1;                        // mono tiles: producer / consumer k_rcs_tile_p (SQLM_TILE_PROD=0: k_rcs_tile)
  // block-tridiagonal cyclic reduction workspace (sqlm_rcs_solve.hip)
  double *cr_D = nullptr, *cr_E = nullptr;  // [p][n][n]
  double *cr_L = nullptr;                   // [p][n][n] Linv_I of the factored superblocks
  double *cr_A = nullptr, *cr_C = nullptr;  // [p][n][n]
  double *cr_g = nullptr, *cr_x = nullptr;  // [p][n]
  int cr_direct = 0;                        // k_rcs_reduce writes D/E/g in CR layout (no BSR S)
  int cr_B = 0, cr_n = 0, cr_p = 0;
  // band + border ("arrow") layout of a loop-closed S (CRPlan.R > 0): cameras
  // covering every block far off the band are eliminated last as a dense
  // border; the band cameras keep the CR superblocks in camera order
  int cr_nband = 0;                         // band cameras (= nP without a border)
  int arw_R = 0, arw_Rp = 0;                // border rows padded to 16 / to kCRMaxN (0 = no border)
  int *cam_pos = nullptr;                   // [nP] band position, or -(1 + border index)
  double *arw_G = nullptr, *arw_Z = nullptr;  // [p][n][R] band-border coupling F^T, and Linv F^T
  double *bd_A = nullptr, *bd_L = nullptr;  // [Rp][Rp] border system (lower) / its factor
  double *bd_Linv = nullptr;                // [Rp / kCRMaxN][kCRMaxN][kCRMaxN]
  double *bd_r = nullptr, *bd_x = nullptr;  // [Rp]
  // reductions
  double *partials = nullptr;               // [kMaxPartials]
  int pc_lm = 0, pc_lid = 0;                // chi2 partial regions of the current linearization
  int px_lm = 0, px_lid = 0;                //   ... and of the speculative one (swapped on accept)
  double *scalars = nullptr;                // [8] see Scalar
  unsigned long long *maxdiag = nullptr;    // bit pattern of a non-negative double
  int *flags = nullptr;                     // [4] solve_ok, device error, ...
  // device-side LM loop (trials enqueued ahead of their decisions): the trial
  // kernels take lambda, the state parity and the done flag from here
};

enum Scalar { kChiCur = 0, kChiNew = 1, kScale = 2, kMaxDiag = 3, kSolveOk = 4, kDevErr = 5, kNScalars = 8 };
constexpr int kMboxSeq = 7;  // host mailbox: the scalars, then the sequence number in slot 7

// partial-sum slots
enum PartialRegion {
  kPartChiCurLm = 0,         // landmark linearize blocks       (<= 16384)
  kPartChiCurLid = 16384,    // camera pass, one per free camera (<= 131072)
  kPartChiNewLm = 147456,    // landmark update blocks          (<= 16384)
  kPartChiNewLid = 163840,   // lidar chi2 at trial state blocks (<= 16384)
  kPartScaleCam = 180224,    // pose part of computeScale blocks (<= 16384)
  kPartScaleLm = 196608,     // landmark part                   (<= 16384)
  kPartChiCurLm2 = 212992,   // second chi-cur landmark region (speculative linearization)
  kPartChiCurLid2 = 229376,  // second chi-cur camera region
  kPartEnd = 360448
};
constexpr int kMaxPartials = kPartEnd;
constexpr int kMaxFreePoses = 131072;

// Superblock plan of the reduced camera system: B cameras per superblock
// (B = block bandwidth + 1), p superblocks of n = roundup(6B, 16) rows.
// With a border (R > 0) the band's cyclic reduction also carries the sparse
// right-hand sides F^T (the band-border coupling): only superblocks whose F^T
// block can be nonzero are touched, per level (host-built lists in `sched`).
struct CRPlan {
  bool enabled = false;
  int B = 0, p = 0, n = 0;
  int nband = 0;                 // band cameras
  int R = 0, Rp = 0, nbc = 0;    // border width (16-padded, kCRMaxN-padded), border cameras
  std::vector<int> sched;        // concatenated lists (host); dev copy below
  const int *sched_dev = nullptr;
  // per level h = 1, 2, 4, ...: [fwd_off, fwd_cnt, upd_off, upd_cnt]
  std::vector<int> lvl;
  int init_off = 0, init_cnt = 0;  // superblocks with a nonzero F^T block (cleared per trial)
  int elim_off = 0, elim_cnt = 0;  // superblocks whose Z = Linv F^T is formed (Gram, correction)
  bool top_active = false;         // superblock 0 carries F^T after the last level
};
constexpr int kCRMaxN = 112;  // LDS: L (n x n+1) + Dinv (16n) + W (16n) <= 160 KiB
constexpr int kBandMaxCams = kCRMaxN / 6 - 1;  // S blocks farther off the diagonal go to the border
// update-list entries: superblock | flags
constexpr int kUpdHad = 1 << 28, kUpdRight = 1 << 29, kUpdLeft = 1 << 30, kUpdMask = (1 << 28) - 1;

// Tile partials are stored block-major: the upper 6x6 camera blocks (u <= w)
// of a tile's cp cameras, packed row by row, 36 contiguous doubles each (the
// reduction reads every contribution as one 288-byte run).
__host__ __device__ inline int tile_blk(int u, int w, int cp) { return u * (2 * cp - u + 1) / 2 + (w - u); }

// Observations per lane in the per-landmark kernels (k_linearize,
// k_landmark_update): a segment of W lanes serves tracks of up to
// kObsPerLane * W observations. A serial chain of Givens rows per lane is
// cheaper than more lanes and butterfly rounds (config 4: 1 / 2 / 3 / 4 per
// lane -> 0.43 / 0.33 / 0.30 / 0.31 ms for the speculative landmark update,
// two of them preloaded).
#ifndef SQLM_OBS_PER_LANE
#define SQLM_OBS_PER_LANE 3
#endif
constexpr int kObsPerLane = SQLM_OBS_PER_LANE;
// loaded up front (the rest of a lane's observations stream in a loop): 3
// would push the speculative landmark update to 130 VGPRs, 3 waves per SIMD
#ifndef SQLM_OBS_PRELOAD
#define SQLM_OBS_PRELOAD 2
#endif
constexpr int kObsPreload = SQLM_OBS_PRELOAD;

// k_landmark_update stages a block tile's pose window in LDS when it spans at
// most kUpdWin poses (wider: loop-closure landmarks, global reads)
constexpr int kUpdWin = 64;
struct Bucket {
  int W;            // segment width
  int slot_begin;   // first landmark slot
  int slot_end;
  int rng_off = 0;  // first entry of this bucket's tiles in DevProblem::upd_rng
  bool wide = false;  // some block tile's pose window is wider than kUpdWin
};

// kernel launchers (sqlm_kernels.hip). All asynchronous on `st`.
void launch_pose_prep(const DevProblem &d, int buf, hipStream_t st);
void launch_linearize(const DevProblem &d, const Bucket &b, int part_off, hipStream_t st);
void launch_camera_pass(const DevProblem &d, hipStream_t st, bool spec = false);
void launch_pose_maxdiag(const DevProblem &d, hipStream_t st);
void launch_pose_diag(const DevProblem &d, hipStream_t st);
void launch_cam_gather(const DevProblem &d, int64_t n_cam_obs, hipStream_t st);
// camera CSR of the device observations (stable: observation order within a camera)
size_t cam_csr_temp_bytes(int64_t n, int nP);
int launch_cam_csr(const int *camh, int64_t n, int nP, unsigned *keys_in, unsigned *keys_out, int *vals_in,
                   int *cam_obs, int *cam_ptr, void *temp, size_t temp_bytes, hipStream_t st);
// rank 0 of a sharded run: destination / source ranges of the gathered rows
constexpr int kMaxRanks = 16;
struct GatherTab {
  int n = 0;
  int64_t s_lo[kMaxRanks], s_hi[kMaxRanks], s_src[kMaxRanks];
  int64_t g_lo[kMaxRanks], g_hi[kMaxRanks], g_src[kMaxRanks];
};
void launch_gather_add(const DevProblem &d, const GatherTab &t, hipStream_t st);
void launch_flag_pack(const DevProblem &d, bool unpack, hipStream_t st);
void launch_damp(const DevProblem &d, double lambda, hipStream_t st);
void launch_rcs(const DevProblem &d, double lambda, int max_row_blocks, hipStream_t st);
// extra streams for the RCS tile classes (null: everything on st)
struct TileStreams {
  hipStream_t s[2] = {nullptr, nullptr};
  hipEvent_t fork = nullptr, join[2] = {nullptr, nullptr};
};
void launch_rcs_tiles(const DevProblem &d, double lambda, int max_cp, int max_k, hipStream_t st,
                      const TileStreams *ts = nullptr);
void launch_rcs_reduce(const DevProblem &d, double lambda, hipStream_t st);
#ifdef SQLM_TILE_PROF
int tile_profile_read(long long *out);  // diagnostic build: k_rcs_tile phase counters
#endif
constexpr int kRedLong = 24;
int launch_dense_solve(const DevProblem &d, hipStream_t st);  // returns SQLM status for setup errors
// completion words of the one-launch back substitution (k_cr_back_all): one
// per superblock, zeroed when allocated; every solve publishes a new epoch
struct CRSync {
  int *done = nullptr;
  int cap = 0, epoch = 0;
};
int launch_cr_solve(const DevProblem &d, const CRPlan &pl, hipStream_t st, bool gather = true,
                    CRSync *sync = nullptr);  // zeroes + scatters unless cr_direct
// band + border layout: clear F^T / the border system before S is assembled into it
void launch_arrow_clear(const DevProblem &d, const CRPlan &pl, hipStream_t st);
// CR levels + top + back substitution on blocks already in CR layout
// (sync: every back-substitution level in one launch; null: one launch per level)
void launch_cr_core(double *D, double *L, double *E, double *A, double *C, double *g, double *x, int *flags, int p, int n,
                    hipStream_t st, CRSync *sync = nullptr);
// Dense SPD solve (sqlm_rcs_solve.hip): A (n x n, lower, n % kCRMaxN == 0) is
// factored in place into L (+ diagonal block inverses Linv), r is consumed,
// x = A^-1 r; flags[0] is cleared on a non-positive pivot. band > 0: A is a
// block arrow — its first `band` blocks of kCRMaxN form a block-tridiagonal
// band, the rest a dense border — and only the blocks the factor fills are
// touched (band = 0: fully dense).
int launch_dense_spd_solve(double *A, double *L, double *Linv, double *r, double *x, int *flags, int n,
                           hipStream_t st, int band = 0, int n_last = 0);
// Block-tridiagonal SPD solve with R right-hand sides by cyclic reduction:
// D / E [p][n][n] (D_I lower, E_I = S(I, I+1)), G [p][n][R] right-hand sides
// (overwritten), X [p][n][R] solution; A, C, Z scratch of the same shapes, gs /
// xs [p][n] scratch. n <= kCRMaxN, n and R multiples of 16. flags[0] = 0 if a
// pivot is not positive.
int launch_cr_multi(double *D, double *L, double *E, double *A, double *C, double *gs, double *xs, double *G, double *Z,
                    double *X, int *flags, int p, int n, int R, hipStream_t st);
// P_I = A_I^T B_I for I < p, A_I / B_I [n][R] row-major, P_I [R][R] (R % 16 == 0).
int launch_batched_atb(const double *A, const double *B, double *P, int p, int n, int R, hipStream_t st);
// from_cr: dx taken from the cyclic-reduction solution (launch_cr_solve with
// gather = false), written to d.dx on the way
void launch_pose_update(const DevProblem &d, double lambda, hipStream_t st, bool from_cr = false);
// fuse_pose: the launch also does launch_pose_update(from_cr = true)'s work
// (band / border CR solves, a bucket without wide windows)
void launch_landmark_update(const DevProblem &d, const Bucket &b, double lambda, int part_off, hipStream_t st,
                            bool spec = false, bool fuse_pose = false);
// every bucket's landmark update in one launch (by value: the block ranges,
// heaviest bucket first); upd_launch_plan fails past kMaxUpdBuckets buckets
constexpr int kMaxUpdBuckets = 6;
struct UpdLaunch {
  int nb = 0, grid = 0;
  int W[kMaxUpdBuckets], slot_begin[kMaxUpdBuckets], slot_end[kMaxUpdBuckets], part_off[kMaxUpdBuckets],
      rng_off[kMaxUpdBuckets], nblk[kMaxUpdBuckets], blk0[kMaxUpdBuckets];
};
int upd_launch_plan(const std::vector<Bucket> &bk, const std::vector<int> &part_off, UpdLaunch &u);
void launch_landmark_update_all(const DevProblem &d, const UpdLaunch &u, double lambda, hipStream_t st, bool spec);
void launch_lidar_chi2(const DevProblem &d, hipStream_t st);
void launch_reduce(const DevProblem &d, int n_lm_parts_cur, int n_lm_parts_new, int n_cam_parts,
                   int n_lid_parts, hipStream_t st, double *mbox = nullptr, unsigned long long seq = 0);
void launch_depth_positive(const DevProblem &d, uint8_t *out_dev, hipStream_t st);

int linearize_blocks(const Bucket &b);

// Essential graph (sqlm_eg.hip): one solver per context, on the context's stream.
struct EGSolver;
EGSolver *eg_create(hipStream_t st);
void eg_destroy(EGSolver *s);
int eg_set_problem(EGSolver *s, int n_kf, const double *Siw, const uint8_t *fixed, int fix_scale, int64_t n_edge,
                   const int32_t *ei, const int32_t *ej, const double *Sji, const double *info);
int eg_optimize(EGSolver *s, int iterations, double user_lambda, const volatile uint8_t *stop, struct sqlm_stats *st,
                int *n_iter);
int eg_get_poses(const EGSolver *s, double *Siw);
int eg_get_edge_chi2(const EGSolver *s, double *chi2);
int eg_get_jacobians(EGSolver *s, double *J);

// ORB front end (sqlm_orb.hip): one engine per context, on the context's stream.
struct OrbEngine;
OrbEngine *orb_create(hipStream_t st);
void orb_destroy(OrbEngine *e);
int orb_extract(OrbEngine *e, const struct sqlm_orb_params *p, const uint8_t *image, int w, int h, int stride,
                struct sqlm_keypoint *kps, uint8_t *desc, int cap, int *n_out);
int orb_get_level(OrbEngine *e, int level, uint8_t *out, int cap, int *w, int *h);
int orb_bench_extract(OrbEngine *e, const struct sqlm_orb_params *p, const uint8_t *image, int w, int h, int stride,
                      int reps, double *ms_per_frame, double *stage_ms);
int orb_match_bf(OrbEngine *e, const uint8_t *query, int nq, const uint8_t *train, int nt, int32_t *best_idx,
                 int32_t *best_dist, int32_t *second_dist);
int orb_search_for_init(OrbEngine *e, const struct sqlm_keypoint *k1, const uint8_t *d1, int n1,
                        const struct sqlm_keypoint *k2, const uint8_t *d2, int n2,
                        const struct sqlm_frame_bounds *f2, float *prev, int32_t *m12, int window, float nnratio,
                        int check_ori, int *n_matches);
int orb_search_by_projection_local(OrbEngine *e, struct sqlm_orb_frame *F, const struct sqlm_track_point *mps,
                                   const uint8_t *mp_desc, int n_mp, float th, float nnratio, int *n_matches);
int orb_search_by_projection_last(OrbEngine *e, struct sqlm_orb_frame *F, const float *Tcw, const float *Tlw,
                                  const struct sqlm_last_point *lp, const uint8_t *ldesc, int n_last, float th,
                                  int mono, int check_ori, int *n_matches);
int orb_search_by_projection_sim3(OrbEngine *e, struct sqlm_orb_frame *F, const float *Scw,
                                  const struct sqlm_map_point *mps, const uint8_t *mp_desc, int n, int th,
                                  int *n_matches);
int orb_fuse(OrbEngine *e, const struct sqlm_orb_frame *F, const float *T, int sim3, const struct sqlm_map_point *mps,
             const uint8_t *mp_desc, int n, float th, int32_t *fuse_idx, int *n_fused);
int orb_search_by_projection_kf(OrbEngine *e, struct sqlm_orb_frame *F, const float *Tcw,
                                const struct sqlm_map_point *mps, const uint8_t *mp_desc, const float *kf_angle, int n,
                                float th, int orb_dist, int check_ori, int *n_matches);
int orb_search_by_sim3(OrbEngine *e, const struct sqlm_orb_frame *K1, const struct sqlm_orb_frame *K2, const float *T1w,
                       const float *T2w, const struct sqlm_map_point *mp1, const uint8_t *md1,
                       const struct sqlm_map_point *mp2, const uint8_t *md2, float s12, const float *R12,
                       const float *t12, float th, int32_t *matches12, int *n_found);
int orb_search_by_bow_kf_frame(OrbEngine *e, const struct sqlm_bow_frame *KF, const struct sqlm_bow_frame *F,
                               float nnratio, int check_ori, int32_t *matches, int *n_matches);
int orb_search_by_bow_kf_kf(OrbEngine *e, const struct sqlm_bow_frame *K1, const struct sqlm_bow_frame *K2,
                            float nnratio, int check_ori, int32_t *matches12, int *n_matches);
int orb_search_for_triangulation(OrbEngine *e, const struct sqlm_bow_frame *K1, const struct sqlm_bow_frame *K2,
                                 const float *C1, const float *T2w, const float *cam2, const float *sf2,
                                 int n_levels2, const float *F12, int only_stereo, int check_ori, int32_t *m12,
                                 int *n_matches);

}  // namespace sqlm
