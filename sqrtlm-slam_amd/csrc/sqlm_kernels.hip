// sqlm_kernels.hip — hand-written CDNA4 (gfx950) kernels of the square-root
// LM bundle-adjustment step. FP64 throughout. One wavefront = 64 lanes.
//
// Pipeline of one LM iteration (reference counterparts in brackets):
//   k_pose_prep        quaternion -> rotation matrix per pose
//   k_linearize<W>     per landmark segment of W lanes: residual, robust weight,
//                      Jacobians, TSQR of the landmark Jacobian, H_pl blocks
//                      [computeActiveErrors + linearizeOplus + constructQuadraticForm,
//                       sparse_optimizer.cpp:73-76, block_solver.hpp:502-560]
//   k_camera_pass      per free camera: H_pp, b_p, LiDAR unary edges
//   --- per LM trial ---
//   k_damp             Givens-damp R with sqrt(lambda) I -> M = (H_ll+lambda)^-1
//                      [setLambda + D->inverse(), block_solver.hpp:564-589, :389]
//   k_rcs              reduced camera system rows S_i*, g_i
//                      [Schur loop, block_solver.hpp:381-439]
//   launch_dense_solve S dx = g  [LinearSolverEigen::solve] when S is not banded
//   k_pose_update      T <- exp(dx) T, pose part of computeScale
//   k_landmark_update<W> back-substitution, X += dl, new residuals + chi2
//                      [block_solver.hpp:459-483, sparse_optimizer.cpp:422-435]
//   k_reduce           deterministic fixed-order sums of the block partials
#include <hip/hip_runtime.h>

#include <type_traits>

#include <algorithm>

#include <cstring>
#ifdef SQLM_TILE_HTRACE
#include <chrono>
#include <cstdio>
#endif
#include <rocprim/device/device_radix_sort.hpp>

#include "se3_dev.h"
#include "sqlm_internal.h"

namespace sqlm {

// ---------------------------------------------------------------- helpers

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  return v;
}

// Deterministic block sum (blockDim = 256): wave butterflies then waves in order.
__device__ double block_sum(double v, double *red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double r = 0.0;
  if (threadIdx.x == 0) r = ((red[0] + red[1]) + red[2]) + red[3];
  return r;
}

__device__ double block_max(double v, double *red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double r = 0.0;
  if (threadIdx.x == 0) r = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
  return r;
}

// Givens-rotate row a = (a0,a1,a2) into upper-triangular R (r00 r01 r02 r11 r12 r22).
// Diagonal of R stays >= 0, so the factor is canonical. Each rotation uses
// one reciprocal square root (v_rsq_f64 + a Newton step): r = h y, c = R y,
// s = a y with y = 1/sqrt(h), h = R^2 + a^2 -- no divides.
__device__ __forceinline__ double rsqrt_nr(double h) {
  double y = __builtin_amdgcn_rsq(h);
  const double t = 0.5 * h * y;
  return fma(y, fma(-t, y, 0.5), y);
}

__device__ __forceinline__ void givens_add_row(double R[6], double a0, double a1, double a2) {
  if (a0 != 0.0) {
    const double h = R[0] * R[0] + a0 * a0, y = rsqrt_nr(h);
    const double c = R[0] * y, s = a0 * y;
    R[0] = h * y;
    const double t1 = c * R[1] + s * a1; a1 = c * a1 - s * R[1]; R[1] = t1;
    const double t2 = c * R[2] + s * a2; a2 = c * a2 - s * R[2]; R[2] = t2;
  }
  if (a1 != 0.0) {
    const double h = R[3] * R[3] + a1 * a1, y = rsqrt_nr(h);
    const double c = R[3] * y, s = a1 * y;
    R[3] = h * y;
    const double t2 = c * R[4] + s * a2; a2 = c * a2 - s * R[4]; R[4] = t2;
  }
  if (a2 != 0.0) R[5] = sqrt(R[5] * R[5] + a2 * a2);
}

// EdgeSE3ProjectXYZ at one observation (types_six_dof_expmap.h:90-95, .cpp:103-147),
// with the Huber weight folded in as sqrt(rho' * info) (robust_kernel_impl.cpp:78-90).
struct MonoEval {
  double e0, e1;      // raw error obs - proj
  double e2;          // stereo edges: right-image error
  double chi_rob;     // rho(chi2) (robust) or chi2
  double s;           // sqrt(rho' * info)
  double x, y, z;     // camera-frame point
};

__device__ __forceinline__ void mono_error(const double *__restrict__ prt, double X0, double X1, double X2,
                                           double u, double v, double info, double delta, MonoEval &m) {
  m.x = prt[0] * X0 + prt[1] * X1 + prt[2] * X2 + prt[9];
  m.y = prt[3] * X0 + prt[4] * X1 + prt[5] * X2 + prt[10];
  m.z = prt[6] * X0 + prt[7] * X1 + prt[8] * X2 + prt[11];
  const double iz = 1.0 / m.z;
  const double pu = (m.x * iz) * prt[12] + prt[14];
  const double pv = (m.y * iz) * prt[13] + prt[15];
  m.e0 = u - pu;
  m.e1 = v - pv;
  const double chi2 = m.e0 * (info * m.e0) + m.e1 * (info * m.e1);
  double rho1 = 1.0;
  m.chi_rob = chi2;
  if (delta > 0.0) {
    const double dsqr = delta * delta;
    if (chi2 > dsqr) {
      const double sq = sqrt(chi2);
      m.chi_rob = 2 * sq * delta - dsqr;
      rho1 = delta / sq;
    }
  }
  m.s = sqrt(rho1 * info);
}

// EdgeStereoSE3ProjectXYZ (types_six_dof_expmap.h:122-127, .cpp:150-157): the
// projection uses invz = (float)(1/z) and the single-precision product
// bf*invz, as the reference's `const float invz` / `const float &bf` do; chi2
// adds the right-image component (information = info I3).
__device__ __forceinline__ void stereo_error(const double *__restrict__ prt, double X0, double X1, double X2,
                                             double u, double v, double ur, double bf, double info, double delta,
                                             MonoEval &m) {
  m.x = prt[0] * X0 + prt[1] * X1 + prt[2] * X2 + prt[9];
  m.y = prt[3] * X0 + prt[4] * X1 + prt[5] * X2 + prt[10];
  m.z = prt[6] * X0 + prt[7] * X1 + prt[8] * X2 + prt[11];
  const float izf = (float)(1.0 / m.z);
  const double iz = (double)izf;
  const double pu = (m.x * iz) * prt[12] + prt[14];
  const double pv = (m.y * iz) * prt[13] + prt[15];
  const float bz = (float)bf * izf;
  m.e0 = u - pu;
  m.e1 = v - pv;
  m.e2 = ur - (pu - (double)bz);
  const double chi2 = m.e0 * (info * m.e0) + m.e1 * (info * m.e1) + m.e2 * (info * m.e2);
  double rho1 = 1.0;
  m.chi_rob = chi2;
  if (delta > 0.0) {
    const double dsqr = delta * delta;
    if (chi2 > dsqr) {
      const double sq = sqrt(chi2);
      m.chi_rob = 2 * sq * delta - dsqr;
      rho1 = delta / sq;
    }
  }
  m.s = sqrt(rho1 * info);
}

// Weighted Jacobians: jl (2x3, row-major) d e / d X, jp (2x6) d e / d [omega; upsilon]
// (types_six_dof_expmap.cpp:103-139), written with one reciprocal iz = 1/z:
// g2o's x/z, 1/z, x/z^2 ... become products of xz = x iz, yz = y iz and iz.
__device__ __forceinline__ void mono_jac(const double *__restrict__ prt, const MonoEval &m, double jl[6],
                                         double jp[12]) {
  const double iz = 1.0 / m.z, xz = m.x * iz, yz = m.y * iz;
  const double fx = prt[12], fy = prt[13];
  const double t00 = -iz * fx, t02 = (xz * iz) * fx;
  const double t11 = -iz * fy, t12 = (yz * iz) * fy;
  const double s = m.s;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    jl[c] = s * (t00 * prt[c] + t02 * prt[6 + c]);
    jl[3 + c] = s * (t11 * prt[3 + c] + t12 * prt[6 + c]);
  }
  jp[0] = s * ((xz * yz) * fx);
  jp[1] = s * (-(1 + xz * xz) * fx);
  jp[2] = s * (yz * fx);
  jp[3] = s * (-iz * fx);
  jp[4] = 0.0;
  jp[5] = s * ((xz * iz) * fx);
  jp[6] = s * ((1 + yz * yz) * fy);
  jp[7] = s * (-(xz * yz) * fy);
  jp[8] = s * (-xz * fy);
  jp[9] = 0.0;
  jp[10] = s * (-iz * fy);
  jp[11] = s * ((yz * iz) * fy);
}

// Third (right-image) row of a stereo edge, weighted: d e2 / d X = row 0 -
// bf R(2,:) / z^2, d e2 / d xi = row 0 + bf (-y, x, 0, 0, 0, -1) / z^2
// (types_six_dof_expmap.cpp:206-233).
__device__ __forceinline__ void stereo_row(const double *__restrict__ prt, const MonoEval &m, double bf,
                                           const double jl[6], const double jp[12], double jl3[3], double jp3[6]) {
  const double iz = 1.0 / m.z, k = m.s * (bf * (iz * iz));
#pragma unroll
  for (int c = 0; c < 3; ++c) jl3[c] = jl[c] - k * prt[6 + c];
  jp3[0] = jp[0] - k * m.y;
  jp3[1] = jp[1] + k * m.x;
  jp3[2] = jp[2];
  jp3[3] = jp[3];
  jp3[4] = 0.0;
  jp3[5] = jp[5] - k;
}

// Column c of an observation's H_lp block P = jl^T jp (3 values), recomputed
// from the linearization point (pose prt, landmark X, stored weight s) by the
// same device code k_linearize used, so the consumers need not store P.
template <bool ST = false>
__device__ __forceinline__ void hlp_col(const double *prt, double X0, double X1, double X2, double s, int c,
                                        double out[3], bool stereo = false, double bf = 0.0) {
  MonoEval m;
  m.x = prt[0] * X0 + prt[1] * X1 + prt[2] * X2 + prt[9];
  m.y = prt[3] * X0 + prt[4] * X1 + prt[5] * X2 + prt[10];
  m.z = prt[6] * X0 + prt[7] * X1 + prt[8] * X2 + prt[11];
  m.s = s;
  double jl[6], jp[12];
  mono_jac(prt, m, jl, jp);
  double p0 = jp[0], p1 = jp[6];
#pragma unroll
  for (int k = 1; k < 6; ++k) {
    p0 = c == k ? jp[k] : p0;
    p1 = c == k ? jp[6 + k] : p1;
  }
#pragma unroll
  for (int a = 0; a < 3; ++a) out[a] = jl[a] * p0 + jl[3 + a] * p1;
  if (ST && stereo) {
    double jl3[3], jp3[6];
    stereo_row(prt, m, bf, jl, jp, jl3, jp3);
    double p2 = jp3[0];
#pragma unroll
    for (int k = 1; k < 6; ++k) p2 = c == k ? jp3[k] : p2;
#pragma unroll
    for (int a = 0; a < 3; ++a) out[a] += jl3[a] * p2;
  }
}

// Workgroup barrier that orders LDS only: global loads issued before it stay in
// flight (a __syncthreads() fence would wait vmcnt(0) and drain the prefetch).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ void store2(double *p, double a, double b) {
  *reinterpret_cast<double2 *>(p) = make_double2(a, b);
}

// The per-observation inputs of one edge, loaded up front: every lane of a
// segment owns at most kObsPerLane observations (W >= k / kObsPerLane,
// seg_width); the first kObsPreload of them are requested before any is used.
struct ObsIn {
  int cam, camh;
  double u, v, info, delta, ur, s;
};

template <bool ST, bool WANT_S>
__device__ __forceinline__ ObsIn load_obs(const DevProblem &d, int e, bool ok) {
  ObsIn o{0, -1, 0.0, 0.0, 0.0, 0.0, -1.0, 0.0};
  if (ok) {
    o.cam = d.obs_cam[e];
    o.camh = d.obs_camh[e];
    if (d.obs_f32) {
      const float4 q = *reinterpret_cast<const float4 *>(d.obs_q + 4 * (int64_t)e);
      o.u = q.x;
      o.v = q.y;
      o.info = q.z;
      o.delta = q.w;
    } else {
      const double2 uv = *reinterpret_cast<const double2 *>(d.obs_uv + 2 * e);
      o.u = uv.x;
      o.v = uv.y;
      o.info = d.obs_info[e];
      o.delta = d.obs_delta[e];
    }
    if (ST) o.ur = d.obs_ur[e];
    if (WANT_S) o.s = d.obs_s[e];
  }
  return o;
}

// ---------------------------------------------------------------- pose prep

__global__ void k_pose_prep(const double *__restrict__ qt, const double *__restrict__ intr,
                            double *__restrict__ rt, int n) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  double q[4] = {qt[8 * p], qt[8 * p + 1], qt[8 * p + 2], qt[8 * p + 3]};
  double R[9];
  q_to_mat(q, R);
  double *o = rt + 16 * p;
#pragma unroll
  for (int i = 0; i < 9; ++i) o[i] = R[i];
  o[9] = qt[8 * p + 4]; o[10] = qt[8 * p + 5]; o[11] = qt[8 * p + 6];
  o[12] = intr[4 * p]; o[13] = intr[4 * p + 1]; o[14] = intr[4 * p + 2]; o[15] = intr[4 * p + 3];
}

void launch_pose_prep(const DevProblem &d, int buf, hipStream_t st) {
  if (d.n_pose == 0) return;
  hipLaunchKernelGGL(k_pose_prep, dim3((d.n_pose + 255) / 256), dim3(256), 0, st, d.pose_qt[buf], d.intr,
                     d.pose_rt[buf], d.n_pose);
}

// One edge of the landmark linearization at the state (prt_all, X): residual
// and robust weight (to obs_err / s_out), the weighted Jacobian rows folded into
// the landmark's R by Givens rotations, b_l, the Hessian diagonal g, chi2.
// k_linearize and the speculative pass of k_landmark_update call it in the same
// order, so both produce the same bits.
template <bool ST>
__device__ __forceinline__ void lin_edge(const DevProblem &d, const ObsIn &o, int e, const double *prt_all, double X0,
                                         double X1, double X2, double *s_out, bool want_P, double R[6], double &b0,
                                         double &b1, double &b2, double &g0, double &g1, double &g2, double &chi) {
  const int cam = o.cam;
  const double *prt = prt_all + 16 * cam;
  MonoEval m;
  const double bf = ST ? d.pose_bf[cam] : 0.0;
  const bool st = ST && o.ur >= 0.0;
  if (st) stereo_error(prt, X0, X1, X2, o.u, o.v, o.ur, bf, o.info, o.delta, m);
  else mono_error(prt, X0, X1, X2, o.u, o.v, o.info, o.delta, m);
  store2(d.obs_err + 2 * e, m.e0, m.e1);
  if (ST) d.obs_err3[e] = st ? m.e2 : 0.0;
  s_out[e] = m.s;
  chi += m.chi_rob;
  double jl[6], jp[12], jl3[3] = {0, 0, 0}, jp3[6] = {0, 0, 0, 0, 0, 0};
  mono_jac(prt, m, jl, jp);
  const double r0 = m.s * m.e0, r1 = m.s * m.e1;
  b0 -= jl[0] * r0 + jl[3] * r1;
  b1 -= jl[1] * r0 + jl[4] * r1;
  b2 -= jl[2] * r0 + jl[5] * r1;
  g0 += jl[0] * jl[0] + jl[3] * jl[3];
  g1 += jl[1] * jl[1] + jl[4] * jl[4];
  g2 += jl[2] * jl[2] + jl[5] * jl[5];
  givens_add_row(R, jl[0], jl[1], jl[2]);
  givens_add_row(R, jl[3], jl[4], jl[5]);
  if (st) {
    stereo_row(prt, m, bf, jl, jp, jl3, jp3);
    const double r2 = m.s * m.e2;
    b0 -= jl3[0] * r2; b1 -= jl3[1] * r2; b2 -= jl3[2] * r2;
    g0 += jl3[0] * jl3[0]; g1 += jl3[1] * jl3[1]; g2 += jl3[2] * jl3[2];
    givens_add_row(R, jl3[0], jl3[1], jl3[2]);
  }
  if (want_P && d.obs_P && o.camh >= 0) {
    // row-kernel fallback only: H_lp block jl^T jp (3x6), SoA, entry (a,c) at P[(6a+c) nE + e]
    double *P = d.obs_P + e;
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int c = 0; c < 6; ++c)
        P[(6 * a + c) * d.nE] = jl[a] * jp[c] + jl[3 + a] * jp[6 + c] + (st ? jl3[a] * jp3[c] : 0.0);
  }
}

// Exchange with the partner group of a segment butterfly level OFF. Within a
// row of 16 lanes this is a DPP move (quad_perm for 1 and 2, half-row / row
// mirror for 4 and 8: after the lower levels every lane of a group holds the
// same value, so the mirror partner is as good as lane ^ OFF), else ds_bpermute.
template <int OFF>
__device__ __forceinline__ double seg_xor(double v) {
  if constexpr (OFF <= 8) {
    constexpr int ctrl = OFF == 1 ? 0xB1 : OFF == 2 ? 0x4E : OFF == 4 ? 0x141 : 0x140;
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, ctrl, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), ctrl, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
  } else {
    return __shfl_xor(v, OFF, 64);
  }
}

// Sum over a W-lane segment, the same tree in every lane (bitwise equal results).
template <int W, int OFF = 1>
__device__ __forceinline__ double seg_sum(double v) {
  if constexpr (OFF < W) return seg_sum<W, 2 * OFF>(v + seg_xor<OFF>(v));
  else return v;
}

// TSQR butterfly inside a W-lane segment (canonical: the lower lane's R absorbs
// the upper's rows), with the sums of b, g and chi2.
template <int W, int OFF = 1>
__device__ __forceinline__ void lin_butterfly(int lane, double R[6], double &b0, double &b1, double &b2, double &g0,
                                              double &g1, double &g2, double &chi) {
  if constexpr (OFF < W) {
    double o[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) o[i] = seg_xor<OFF>(R[i]);
    const bool lo = (lane & OFF) == 0;
    double A[6], B[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) { A[i] = lo ? R[i] : o[i]; B[i] = lo ? o[i] : R[i]; }
    givens_add_row(A, B[0], B[1], B[2]);
    givens_add_row(A, 0.0, B[3], B[4]);
    givens_add_row(A, 0.0, 0.0, B[5]);
#pragma unroll
    for (int i = 0; i < 6; ++i) R[i] = A[i];
    b0 += seg_xor<OFF>(b0); b1 += seg_xor<OFF>(b1); b2 += seg_xor<OFF>(b2);
    g0 += seg_xor<OFF>(g0); g1 += seg_xor<OFF>(g1); g2 += seg_xor<OFF>(g2);
    chi += seg_xor<OFF>(chi);
    lin_butterfly<W, 2 * OFF>(lane, R, b0, b1, b2, g0, g1, g2, chi);
  }
}

// ---------------------------------------------------------------- linearize

// per-landmark kernels: at most this many blocks per bucket launch (grid-stride
// beyond; 1024 / 4096 measured within noise, profiles/r03 + r04/ab_split_grid.log)
static int max_grid() { return 2048; }

int linearize_blocks(const Bucket &b) {
  const int nseg = b.slot_end - b.slot_begin;
  const int segs_per_block = kBlock / b.W;
  int tiles = (nseg + segs_per_block - 1) / segs_per_block;
  return tiles < max_grid() ? tiles : max_grid();
}

// One landmark per W-lane segment. Each lane folds its observations' two
// weighted Jacobian rows into a private 3x3 R by Givens rotations; a butterfly
// over the segment merges the R's (TSQR), so every lane ends with the QR
// factor of the landmark's stacked 2k x 3 Jacobian without forming J^T J.
// ST: some edges are stereo (obs_ur >= 0) and add a third row.
template <int W, bool ST>
__global__ __launch_bounds__(256) void k_linearize(DevProblem d, int slot_begin, int slot_end, int part_off) {
  __shared__ double red[4];
  constexpr int SPB = kBlock / W;
  const int lane = threadIdx.x & (W - 1);
  const int nseg = slot_end - slot_begin;
  const int ntiles = (nseg + SPB - 1) / SPB;
  const double *__restrict__ prt_all = d.pose_rt[0];
  double chi_acc = 0.0, dmax = 0.0;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int seg = tile * SPB + threadIdx.x / W;
    const int slot = slot_begin + seg;
    const bool valid = seg < nseg;
    double R[6] = {0, 0, 0, 0, 0, 0};
    double b0 = 0, b1 = 0, b2 = 0, g0 = 0, g1 = 0, g2 = 0, chi = 0;
    if (valid) {
      const double X0 = d.X[0][4 * slot], X1 = d.X[0][4 * slot + 1], X2 = d.X[0][4 * slot + 2];
      const int beg = d.lm_begin[slot], end = d.lm_begin[slot + 1];
      ObsIn o[kObsPreload];
#pragma unroll
      for (int i = 0; i < kObsPreload; ++i) o[i] = load_obs<ST, false>(d, beg + lane + i * W, beg + lane + i * W < end);
#pragma unroll
      for (int i = 0; i < kObsPreload; ++i) {
        const int e = beg + lane + i * W;
        if (e < end) lin_edge<ST>(d, o[i], e, prt_all, X0, X1, X2, d.obs_s, true, R, b0, b1, b2, g0, g1, g2, chi);
      }
      for (int e = beg + lane + kObsPreload * W; e < end; e += W)  // the rest of the lane's observations
        lin_edge<ST>(d, load_obs<ST, false>(d, e, true), e, prt_all, X0, X1, X2, d.obs_s, true, R, b0, b1, b2, g0, g1,
                     g2, chi);
    }
    lin_butterfly<W>(lane, R, b0, b1, b2, g0, g1, g2, chi);
    if (valid && lane == 0) {
      double *Ro = d.lm_R + 8 * slot;
      store2(Ro, R[0], R[1]); store2(Ro + 2, R[2], R[3]); store2(Ro + 4, R[4], R[5]);
      double *bo = d.lm_b + 4 * slot;
      store2(bo, b0, b1); store2(bo + 2, b2, 0.0);
      chi_acc += chi;
      dmax = fmax(dmax, fmax(g0, fmax(g1, g2)));
    }
  }
  const double s = block_sum(chi_acc, red);
  const double mx = block_max(dmax, red);
  if (threadIdx.x == 0) {
    d.partials[d.pc_lm + part_off + blockIdx.x] = s;
    atomicMax(d.maxdiag, (unsigned long long)__double_as_longlong(mx));
  }
}

void launch_linearize(const DevProblem &d, const Bucket &b, int part_off, hipStream_t st) {
  const int nb = linearize_blocks(b);
  if (nb <= 0) return;
  switch (b.W) {
#define SQLM_CASE(WW)                                                                                          \
  case WW:                                                                                                     \
    if (d.has_stereo)                                                                                          \
      hipLaunchKernelGGL((k_linearize<WW, true>), dim3(nb), dim3(kBlock), 0, st, d, b.slot_begin, b.slot_end,  \
                         part_off);                                                                            \
    else                                                                                                       \
      hipLaunchKernelGGL((k_linearize<WW, false>), dim3(nb), dim3(kBlock), 0, st, d, b.slot_begin, b.slot_end, \
                         part_off);                                                                            \
    break;
    SQLM_CASE(2) SQLM_CASE(4) SQLM_CASE(8) SQLM_CASE(16) SQLM_CASE(32) SQLM_CASE(64)
#undef SQLM_CASE
    default: break;
  }
}

// ---------------------------------------------------------------- camera pass

// One wave per free camera: H_pp = sum jp^T jp, b_p = -sum jp^T r with the
// weighted pose Jacobian recomputed from the inputs (the same device code as
// k_linearize, so bit-identical), plus the camera's LiDAR unary edges
// (numeric Jacobian, base_unary_edge.hpp:82-122).
// spec: the speculative pass at the trial state (pose / landmark buffers 1)
// into Hpp_nx / bp_nx, launched after k_landmark_update<SPEC>.
// LID: the instantiation with LiDAR edges. Their numeric Jacobian needs
// ~2.5x the registers; without it the pass is compiled for 5 waves per SIMD
// (96 VGPRs, a dozen spilled), which holds the whole config-4 grid -- 5000
// waves -- resident at once: 0.095 -> 0.061 ms beside the tiles, 748 -> 760
// it/s (one observation prefetched ahead at 4 waves per SIMD: 0.073 ms,
// profiles/r05/ab_cam_pass_r5h.log).
#ifndef SQLM_CAM_OCC
#define SQLM_CAM_OCC 5
#endif
template <bool ST, bool LID>
__global__ __launch_bounds__(256, LID ? 1 : SQLM_CAM_OCC) void k_camera_pass(DevProblem d, int spec) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const double *pose_rt_s = spec ? d.pose_rt[1] : d.pose_rt[0], *X_s = spec ? d.X[1] : d.X[0];
  const double *pose_qt_s = spec ? d.pose_qt[1] : d.pose_qt[0];
  // the camera index is wave-uniform: said so, its pose is read with scalar
  // loads into SGPRs (32 VGPRs less)
  const int i = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + wave);
  double H[21], b[6], chi = 0.0;
#pragma unroll
  for (int k = 0; k < 21; ++k) H[k] = 0.0;
#pragma unroll
  for (int k = 0; k < 6; ++k) b[k] = 0.0;
  if (i < d.nP) {
    const double *prt = pose_rt_s + 16 * d.hidx_pose[i];
    const double bf = ST ? d.pose_bf[d.hidx_pose[i]] : 0.0;
    for (int t = d.cam_obs_ptr[i] + lane; t < d.cam_obs_ptr[i + 1]; t += 64) {
      const double *X = X_s + 4 * d.cam_slot[t];
      double2 uv, id;
      if (d.obs_f32) {
        const float4 q = *reinterpret_cast<const float4 *>(d.cam_q + 4 * (int64_t)t);
        uv = make_double2(q.x, q.y);
        id = make_double2(q.z, q.w);
      } else {
        uv = *reinterpret_cast<const double2 *>(d.cam_uv + 4 * t);
        id = *reinterpret_cast<const double2 *>(d.cam_uv + 4 * t + 2);
      }
      const double ur = ST ? d.cam_ur[t] : -1.0;
      const bool st = ST && ur >= 0.0;
      MonoEval m;
      if (st) stereo_error(prt, X[0], X[1], X[2], uv.x, uv.y, ur, bf, id.x, id.y, m);
      else mono_error(prt, X[0], X[1], X[2], uv.x, uv.y, id.x, id.y, m);
      double jl[6], j[14];
      mono_jac(prt, m, jl, j);
      j[12] = m.s * m.e0;
      j[13] = m.s * m.e1;
      int k = 0;
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        b[r] -= j[r] * j[12] + j[6 + r] * j[13];
#pragma unroll
        for (int c = r; c < 6; ++c) H[k++] += j[r] * j[c] + j[6 + r] * j[6 + c];
      }
      if (st) {
        double jl3[3], jp3[6];
        stereo_row(prt, m, bf, jl, j, jl3, jp3);
        const double r2 = m.s * m.e2;
        k = 0;
#pragma unroll
        for (int r = 0; r < 6; ++r) {
          b[r] -= jp3[r] * r2;
#pragma unroll
          for (int c = r; c < 6; ++c) H[k++] += jp3[r] * jp3[c];
        }
      }
    }
    if (LID) {
      const int p = d.hidx_pose[i];
      const double *qt = pose_qt_s + 8 * p;
      const double q[4] = {qt[0], qt[1], qt[2], qt[3]}, t3[3] = {qt[4], qt[5], qt[6]};
      for (int t = d.lid_cam_ptr[i] + lane; t < d.lid_cam_ptr[i + 1]; t += 64) {
        const double *L = d.lid_data + 12 * t;
        const double e = lidar_error(q, t3, L, L + 3, L + 6);
        d.lid_err[t] = e;
        const double info = L[9];
        chi += e * (info * e);
        double J[6];
        lidar_jacobian(q, t3, L, L + 3, L + 6, J);
        int k = 0;
#pragma unroll
        for (int r = 0; r < 6; ++r) {
          b[r] -= (J[r] * info) * e;
#pragma unroll
          for (int c = r; c < 6; ++c) H[k++] += (J[r] * info) * J[c];
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 21; ++k) H[k] = wave_sum(H[k]);
#pragma unroll
  for (int k = 0; k < 6; ++k) b[k] = wave_sum(b[k]);
  chi = wave_sum(chi);
  if (i < d.nP && lane == 0) {
    double *Ho = (spec ? d.Hpp_nx : d.Hpp) + 36 * i;
    int k = 0;
    double mx = 0.0;
    for (int r = 0; r < 6; ++r)
      for (int c = r; c < 6; ++c) {
        Ho[r * 6 + c] = H[k];
        Ho[c * 6 + r] = H[k];
        if (r == c) mx = fmax(mx, fabs(H[k]));
        ++k;
      }
    double *bo = spec ? d.bp_nx : d.bp;
    for (int r = 0; r < 6; ++r) bo[8 * i + r] = b[r];
    d.partials[(spec ? d.px_lid : d.pc_lid) + i] = chi;
    if (!d.sharded && !spec) atomicMax(d.maxdiag, (unsigned long long)__double_as_longlong(mx));
  }
}

void launch_camera_pass(const DevProblem &d, hipStream_t st, bool spec) {
  if (d.nP == 0) return;
  const dim3 g((d.nP + 3) / 4);
  if (d.nLid > 0) {
    if (d.has_stereo) hipLaunchKernelGGL((k_camera_pass<true, true>), g, dim3(256), 0, st, d, (int)spec);
    else hipLaunchKernelGGL((k_camera_pass<false, true>), g, dim3(256), 0, st, d, (int)spec);
  } else {
    if (d.has_stereo) hipLaunchKernelGGL((k_camera_pass<true, false>), g, dim3(256), 0, st, d, (int)spec);
    else hipLaunchKernelGGL((k_camera_pass<false, false>), g, dim3(256), 0, st, d, (int)spec);
  }
}

// Sharded runs, iteration 0: the pose Hessian diagonals of this rank (summed
// across ranks by the caller), then their max |.| for lambda_0.
__global__ __launch_bounds__(256) void k_pose_diag(DevProblem d) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < 6 * d.nP) d.hdiag[k] = d.Hpp[36 * (k / 6) + 7 * (k % 6)];
}

__global__ __launch_bounds__(256) void k_pose_maxdiag(DevProblem d) {
  __shared__ double red[4];
  double mx = 0.0;
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < 6 * d.nP; k += gridDim.x * blockDim.x)
    mx = fmax(mx, fabs(d.hdiag[k]));
  mx = block_max(mx, red);
  if (threadIdx.x == 0) atomicMax(d.maxdiag, (unsigned long long)__double_as_longlong(mx));
}

// setup: camera-ordered copies of the camera pass inputs, gathered from the
// slot-ordered observation arrays (saves uploading them a second time)
__global__ __launch_bounds__(256) void k_cam_gather(DevProblem d, int64_t n) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int o = d.cam_obs[t];
  d.cam_slot[t] = d.obs_lm[o];
  if (d.obs_f32) {
    *reinterpret_cast<float4 *>(d.cam_q + 4 * t) = *reinterpret_cast<const float4 *>(d.obs_q + 4 * (int64_t)o);
  } else {
    double *u = d.cam_uv + 4 * t;
    u[0] = d.obs_uv[2 * (int64_t)o];
    u[1] = d.obs_uv[2 * (int64_t)o + 1];
    u[2] = d.obs_info[o];
    u[3] = d.obs_delta[o];
  }
  if (d.cam_ur) d.cam_ur[t] = d.obs_ur[o];
}

// ---- camera CSR on the device: the observations of every free camera in
// observation (slot) order, = the host's stable counting sort. Keys are the
// free camera id (fixed cameras -> nP, sorted last), values the observation;
// a stable radix sort over the key bits, then each camera's start by binary
// search over the sorted keys.
__global__ __launch_bounds__(256) void k_cam_keys(const int *__restrict__ camh, int64_t n, int nP,
                                                  unsigned *__restrict__ keys, int *__restrict__ vals) {
  const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= n) return;
  const int h = camh[o];
  keys[o] = h >= 0 ? (unsigned)h : (unsigned)nP;
  vals[o] = (int)o;
}

__global__ __launch_bounds__(256) void k_cam_ptr(const unsigned *__restrict__ keys, int64_t n, int nP,
                                                 int *__restrict__ ptr) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > nP) return;
  int64_t lo = 0, hi = n;  // first position with key >= i
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (keys[mid] < (unsigned)i) lo = mid + 1;
    else hi = mid;
  }
  ptr[i] = (int)lo;
}

static unsigned cam_key_bits(int nP) {
  unsigned b = 1;
  while ((1u << b) <= (unsigned)nP) ++b;
  return b;
}

size_t cam_csr_temp_bytes(int64_t n, int nP) {
  size_t bytes = 0;
  (void)rocprim::radix_sort_pairs(nullptr, bytes, (unsigned *)nullptr, (unsigned *)nullptr, (int *)nullptr,
                                  (int *)nullptr, (size_t)n, 0u, cam_key_bits(nP));
  return std::max<size_t>(bytes, 16);
}

int launch_cam_csr(const int *camh, int64_t n, int nP, unsigned *keys_in, unsigned *keys_out, int *vals_in,
                   int *cam_obs, int *cam_ptr, void *temp, size_t temp_bytes, hipStream_t st) {
  if (n > 0) {
    hipLaunchKernelGGL(k_cam_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, camh, n, nP, keys_in, vals_in);
    size_t bytes = temp_bytes;
    if (rocprim::radix_sort_pairs(temp, bytes, keys_in, keys_out, vals_in, cam_obs, (size_t)n, 0u, cam_key_bits(nP),
                                  st) != hipSuccess)
      return -2;
  }
  hipLaunchKernelGGL(k_cam_ptr, dim3((unsigned)((nP + 1 + 255) / 256)), dim3(256), 0, st, keys_out, n, nP, cam_ptr);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

void launch_cam_gather(const DevProblem &d, int64_t n, hipStream_t st) {
  if (n > 0) hipLaunchKernelGGL(k_cam_gather, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, d, n);
}

void launch_pose_diag(const DevProblem &d, hipStream_t st) {
  if (d.nP == 0) return;
  hipLaunchKernelGGL(k_pose_diag, dim3((6 * d.nP + 255) / 256), dim3(256), 0, st, d);
}

void launch_pose_maxdiag(const DevProblem &d, hipStream_t st) {
  if (d.nP == 0) return;
  hipLaunchKernelGGL(k_pose_maxdiag, dim3(std::min(64, (6 * d.nP + 255) / 256)), dim3(256), 0, st, d);
}

// Sharded runs, rank 0: S / g += the row ranges gathered from the other ranks
// (staged contiguously). Each destination entry sums its sources in rank
// order, so the result is deterministic and no two threads write one entry.
__global__ __launch_bounds__(256) void k_gather_add(DevProblem d, GatherTab t) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nS = 36 * d.nnzb;
  if (i < nS) {
    double v = d.S[i];
    for (int r = 0; r < t.n; ++r)
      if (i >= t.s_lo[r] && i < t.s_hi[r]) v += d.xstage[t.s_src[r] + (i - t.s_lo[r])];
    d.S[i] = v;
  } else if (i < nS + 6 * d.nP) {
    const int64_t k = i - nS;
    double v = d.g[k];
    for (int r = 0; r < t.n; ++r)
      if (k >= t.g_lo[r] && k < t.g_hi[r]) v += d.xstage[t.g_src[r] + (k - t.g_lo[r])];
    d.g[k] = v;
  }
}

void launch_gather_add(const DevProblem &d, const GatherTab &t, hipStream_t st) {
  const int64_t n = 36 * d.nnzb + 6 * (int64_t)d.nP;
  if (n > 0) hipLaunchKernelGGL(k_gather_add, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, d, t);
}

// The solve flag rides in the dx broadcast (slot 6 nP).
__global__ void k_flag_pack(DevProblem d, int unpack) {
  if (unpack) d.flags[0] = d.dx[6 * d.nP] > 0.5 ? 1 : 0;
  else d.dx[6 * d.nP] = (double)d.flags[0];
}

void launch_flag_pack(const DevProblem &d, bool unpack, hipStream_t st) {
  hipLaunchKernelGGL(k_flag_pack, dim3(1), dim3(1), 0, st, d, unpack ? 1 : 0);
}

// ---------------------------------------------------------------- damping

// Damped landmark factor: R' = QR([R; sqrt(lambda) I]) by three Givens
// sweeps, its inverse R'^-1 (upper: i00 i01 i02 i11 i12 i22) and
// w = R'^-T b_l. Computed where it is consumed (the RCS tile staging and the
// landmark update, same code => same bits), not stored per trial.
__device__ __forceinline__ void damp_factor(const double *__restrict__ Rl, const double *__restrict__ bl,
                                            double lambda, double Ri[6], double w[3]) {
  double R[6] = {Rl[0], Rl[1], Rl[2], Rl[3], Rl[4], Rl[5]};
  const double sl = sqrt(lambda);
  givens_add_row(R, sl, 0.0, 0.0);
  givens_add_row(R, 0.0, sl, 0.0);
  givens_add_row(R, 0.0, 0.0, sl);
  const double i00 = 1.0 / R[0], i11 = 1.0 / R[3], i22 = 1.0 / R[5];
  const double i01 = -(R[1] * i11) * i00;
  const double i12 = -(R[4] * i22) * i11;
  const double i02 = -(R[1] * i12 + R[2] * i22) * i00;
  Ri[0] = i00; Ri[1] = i01; Ri[2] = i02; Ri[3] = i11; Ri[4] = i12; Ri[5] = i22;
  w[0] = i00 * bl[0];
  w[1] = i01 * bl[0] + i11 * bl[1];
  w[2] = i02 * bl[0] + i12 * bl[1] + i22 * bl[2];
}

// Row-kernel RCS fallback only: M = (R'^T R')^-1 = R'^-1 R'^-T and M b_l.
__global__ void k_damp(DevProblem d, double lambda) {
  const int l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= d.nL) return;
  double Ri[6], w[3];
  const double *bl = d.lm_b + 4 * l;
  damp_factor(d.lm_R + 8 * l, bl, lambda, Ri, w);
  const double i00 = Ri[0], i01 = Ri[1], i02 = Ri[2], i11 = Ri[3], i12 = Ri[4], i22 = Ri[5];
  const double m00 = i00 * i00 + i01 * i01 + i02 * i02;
  const double m01 = i01 * i11 + i02 * i12;
  const double m02 = i02 * i22;
  const double m11 = i11 * i11 + i12 * i12;
  const double m12 = i12 * i22;
  const double m22 = i22 * i22;
  double *M = d.lm_M + 8 * l;
  store2(M, m00, m01); store2(M + 2, m02, m11); store2(M + 4, m12, m22);
  const double v0 = m00 * bl[0] + m01 * bl[1] + m02 * bl[2];
  const double v1 = m01 * bl[0] + m11 * bl[1] + m12 * bl[2];
  const double v2 = m02 * bl[0] + m12 * bl[1] + m22 * bl[2];
  double *v = d.lm_v + 4 * l;
  store2(v, v0, v1); store2(v + 2, v2, 0.0);
}

void launch_damp(const DevProblem &d, double lambda, hipStream_t st) {
  if (d.nL == 0 || !d.obs_P) return;  // the tiled path damps where it consumes
  hipLaunchKernelGGL(k_damp, dim3((d.nL + 255) / 256), dim3(256), 0, st, d, lambda);
}

// ---------------------------------------------------------------- RCS

// Row i of the reduced camera system. Each wave walks a share of camera i's
// landmarks and accumulates -P_i^T M P_j into a wave-private LDS copy of the
// row (one observation j at a time, so no two lanes touch one entry); the four
// copies are summed in wave order at the end => bitwise deterministic.
__global__ __launch_bounds__(256) void k_rcs(DevProblem d, double lambda, int nslot_max) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int i = blockIdx.x;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int rb = d.s_row_ptr[i], nslot = d.s_row_ptr[i + 1] - rb;
  double *acc = smem + wave * nslot_max * 36;
  double *gw = smem + 4 * nslot_max * 36;                 // [4][8]
  int *cols = reinterpret_cast<int *>(gw + 32);           // [nslot_max]
  for (int k = lane; k < nslot * 36; k += 64) acc[k] = 0.0;
  for (int k = threadIdx.x; k < nslot; k += 256) cols[k] = d.s_col[rb + k];
  __syncthreads();
  const int r = lane / 6, c = lane % 6;  // entry owned by lanes 0..35
  double gacc = 0.0;                     // lanes 0..5: g_r partial
  for (int t = d.cam_obs_ptr[i] + wave; t < d.cam_obs_ptr[i + 1]; t += 4) {
    const int oi = d.cam_obs[t];
    const int l = d.obs_lm[oi];
    const double *Ml = d.lm_M + 8 * l;
    const double M00 = Ml[0], M01 = Ml[1], M02 = Ml[2], M11 = Ml[3], M12 = Ml[4], M22 = Ml[5];
    const double *Pi = d.obs_P + oi;  // SoA: entry (a,c) at Pi[(6a+c) nE]
    // lanes 0..17 compute Z[zr][zc] = (P_i^T M)[zr][zc], zr in 0..5, zc in 0..2
    double zval = 0.0;
    if (lane < 18) {
      const int zr = lane / 3, zc = lane % 3;
      const double p0 = Pi[zr * d.nE], p1 = Pi[(6 + zr) * d.nE], p2 = Pi[(12 + zr) * d.nE];
      const double m0 = zc == 0 ? M00 : (zc == 1 ? M01 : M02);
      const double m1 = zc == 0 ? M01 : (zc == 1 ? M11 : M12);
      const double m2 = zc == 0 ? M02 : (zc == 1 ? M12 : M22);
      zval = p0 * m0 + p1 * m1 + p2 * m2;
    }
    if (lane < 6) {
      const double *v = d.lm_v + 4 * l;
      gacc -= Pi[lane * d.nE] * v[0] + Pi[(6 + lane) * d.nE] * v[1] + Pi[(12 + lane) * d.nE] * v[2];
    }
    const int rr = lane < 36 ? r : 0;
    const double z0 = __shfl(zval, 3 * rr, 64);
    const double z1 = __shfl(zval, 3 * rr + 1, 64);
    const double z2 = __shfl(zval, 3 * rr + 2, 64);
    const int beg = d.lm_begin[l], end = d.lm_begin[l + 1];
    for (int o = beg; o < end; ++o) {
      const int cj = d.obs_camh[o];
      if (cj < i) continue;  // fixed (-1) or lower triangle
      // binary search slot of cj in the sorted row pattern
      int lo = 0, hi = nslot - 1;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cols[mid] < cj) lo = mid + 1; else hi = mid;
      }
      if (lane < 36) {
        const double *Pj = d.obs_P + o;
        const double v = z0 * Pj[c * d.nE] + z1 * Pj[(6 + c) * d.nE] + z2 * Pj[(12 + c) * d.nE];
        acc[lo * 36 + lane] -= v;
      }
    }
  }
  if (lane < 6) gw[wave * 8 + lane] = gacc;
  __syncthreads();
  double *Srow = d.S + (int64_t)rb * 36;
  for (int k = threadIdx.x; k < nslot * 36; k += 256) {
    const int nsm = nslot_max * 36;
    double v = ((smem[k] + smem[nsm + k]) + smem[2 * nsm + k]) + smem[3 * nsm + k];
    if (k < 36) {  // slot 0 = diagonal block (cols[0] == i); sharded: this rank's H_pp share
      v += d.Hpp[36 * i + k];
      if (k % 7 == 0 && (!d.sharded || d.rank == 0)) v += lambda;
    }
    Srow[k] = v;
  }
  if (threadIdx.x < 6) {
    const int rr = threadIdx.x;
    const double bpv = d.bp[8 * i + rr];  // sharded: this rank's b_p share
    d.g[6 * i + rr] = bpv + (((gw[rr] + gw[8 + rr]) + gw[16 + rr]) + gw[24 + rr]);
  }
}

void launch_rcs(const DevProblem &d, double lambda, int max_row_blocks, hipStream_t st) {
  if (d.nP == 0) return;
  const size_t lds = (size_t)4 * max_row_blocks * 36 * sizeof(double) + 32 * sizeof(double) +
                     (size_t)max_row_blocks * sizeof(int) + 16;
  hipLaunchKernelGGL(k_rcs, dim3(d.nP), dim3(256), lds, st, d, lambda, max_row_blocks);
}

// Tiled RCS on the FP64 matrix cores. With Y_o = R'^-T P_o (3x6 per
// observation) and w_l = R'^-T b_l:
//   S_ij = H_pp,i d_ij + lambda I d_ij - sum_l Y_li^T Y_lj,  g_i = b_p,i - sum_l Y_li^T w_l.
// A tile is a run of consecutive landmark slots whose free cameras form a small
// sorted window C_t (|C_t| <= 24, 6|C_t| <= 144 columns). One workgroup of
// kTileWaves wavefronts owns a tile: per landmark it stages the dense
// 3 x 6|C_t| row block Y_l (plus a zero 4th row) in LDS and accumulates
// G_t += Y_l^T Y_l with v_mfma_f64_16x16x4_f64 into NT(NT+1)/2 upper 16x16
// accumulator tiles held in AGPRs (tile q owned by wave q % kTileWaves),
// skipping the tiles outside the landmark's column span. Fixed ownership
// means no atomics and a fixed summation order (bitwise deterministic).
typedef double d4v __attribute__((ext_vector_type(4)));

// Landmarks are consumed in batches of 4: landmark li of a batch occupies rows
// 3li..3li+2 of the staged block, so one batch = 3 K-steps of
// v_mfma_f64_16x16x4_f64 per 16x16 tile (no padding rows).
// The raw P columns of the next batch are prefetched into registers while the
// current batch runs on the matrix cores.
#ifndef SQLM_TILE_WAVES
#define SQLM_TILE_WAVES 4
#endif
constexpr int kTileWaves = SQLM_TILE_WAVES, kTileThreads = 64 * kTileWaves;
// waves per SIMD the tile kernel is compiled for (VGPR budget 512 / this)
constexpr int kTileOcc = kTileWaves == 4 ? 3 : 4;

// Phase cycle counters of the first kTileProfTiles tiles (diagnostic build
// -DSQLM_TILE_PROF only; read with sqlm_debug_tile_profile).
#ifdef SQLM_TILE_PROF
constexpr int kTileProfTiles = 64, kTileProfSlots = 8;
__device__ long long g_tile_prof[kTileProfTiles][kTileProfSlots];
#define TP_DECL                \
  long long tp_acc[kTileProfSlots] = {}; \
  long long tp_last = clock64();
#define TP(slot)                          \
  do {                                    \
    const long long tp_now = clock64();   \
    tp_acc[slot] += tp_now - tp_last;     \
    tp_last = tp_now;                     \
  } while (0)
#define TP_STORE                                                        \
  do {                                                                  \
    if (threadIdx.x == 0 && blockIdx.x < kTileProfTiles)                \
      for (int i_ = 0; i_ < kTileProfSlots; ++i_) g_tile_prof[blockIdx.x][i_] += tp_acc[i_]; \
  } while (0)
// one role's stamps, stored by thread `who` (k_rcs_tile_p: producer lane 0, first consumer lane 0)
#define TP_STORE_BY(who)                                                \
  do {                                                                  \
    if (threadIdx.x == (who) && blockIdx.x < kTileProfTiles)            \
      for (int i_ = 0; i_ < kTileProfSlots; ++i_) g_tile_prof[blockIdx.x][i_] += tp_acc[i_]; \
  } while (0)
#else
#define TP_STORE_BY(who) \
  do {                   \
  } while (0)
#define TP_DECL
#define TP(slot) \
  do {           \
  } while (0)
#define TP_STORE \
  do {           \
  } while (0)
#endif
// A batch of kTileBL landmarks fills 3 kTileBL rows of the staged block
// (landmark li in rows 3li..3li+2), i.e. kTileKS K-steps of 4 rows.
constexpr int kTileBL = 4, kTileKS = (3 * kTileBL + 3) / 4, kTileRows = 4 * kTileKS;
// fast path: one thread per observation of a batch, so tracks up to
// kTileThreads / kTileBL = 64 observations and no camera seen twice by a landmark
constexpr int kTileFastK = kTileThreads / kTileBL;

// MFMA phase of one batch for the accumulator tiles q = P (mod kTileWaves):
// acc[q/W] += sum_ks Y[4ks..4ks+3][ti-tile]^T Y[4ks..4ks+3][tj-tile].
// Both operands of every MFMA are entries Y[4ks + (lane>>4)][16t + (lane&15)],
// so the lane's NT x 4 values are read from LDS once and the MFMAs then issue
// back to back from registers.
// The pair loop runs over the union span [tmin, tmax] of the batch with all K
// steps branch-free (per-landmark spans would save MFMAs but split the chain
// into basic blocks the compiler cannot interleave: measured slower).
template <int NT, int P, int NC>
__device__ __forceinline__ void tile_mfma(d4v *acc, const double (*Y)[NC], int tmin, int tmax, int nks, int r16,
                                          int k4) {
  double op[NT][kTileKS];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int ks = 0; ks < kTileKS; ++ks) op[t][ks] = Y[4 * ks + k4][t * 16 + r16];
  int q = 0;
#pragma unroll
  for (int ti = 0; ti < NT; ++ti) {
#pragma unroll
    for (int tj = ti; tj < NT; ++tj, ++q) {
      if (q % kTileWaves == P && ti >= tmin && tj <= tmax) {
#pragma unroll
        for (int ks = 0; ks < kTileKS; ++ks)
          if (ks < nks)
            acc[q / kTileWaves] =
                __builtin_amdgcn_mfma_f64_16x16x4f64(op[ti][ks], op[tj][ks], acc[q / kTileWaves], 0, 0, 0);
      }
    }
  }
}

// tile_mfma for this wave's accumulator tiles (P = wave, a compile-time constant)
template <int NT, int P = 0, int NC>
__device__ __forceinline__ void tile_mfma_wave(int wave, d4v *acc, const double (*Y)[NC], int tmin, int tmax, int nks,
                                               int r16, int k4) {
  if constexpr (P + 1 < kTileWaves) {
    if (wave != P) return tile_mfma_wave<NT, P + 1>(wave, acc, Y, tmin, tmax, nks, r16, k4);
  }
  tile_mfma<NT, P>(acc, Y, tmin, tmax, nks, r16, k4);
}

// Y block of one mono observation into rows Y[0..2] (row stride ld) at
// column col: Y = R'^-T P with P = jl^T jp (types_six_dof_expmap.cpp:103-139)
// factored as P = [-B' [X_c]x | B'], B' = R^T A, A = s^2 J_pi^T J_pi (five
// distinct entries) -- ~45 % fewer FP64 operations than forming jl, jp and
// their 18 products. pr: the camera's R t fx fy, xl: the landmark, r: R'^-1
// (upper: r0 r1 r2 / r3 r4 / r5), ps: sqrt(rho' info).
__device__ __forceinline__ void stage_mono_y(const double *pr, const double *xl, const double *r, double ps,
                                             double *Y, int ld, int col) {
  MonoEval m;
  m.x = pr[0] * xl[0] + pr[1] * xl[1] + pr[2] * xl[2] + pr[9];
  m.y = pr[3] * xl[0] + pr[4] * xl[1] + pr[5] * xl[2] + pr[10];
  m.z = pr[6] * xl[0] + pr[7] * xl[1] + pr[8] * xl[2] + pr[11];
  const double iz = 1.0 / m.z, xz = m.x * iz, yz = m.y * iz, fx = pr[12], fy = pr[13];
  const double t00 = -iz * fx, t02 = (xz * iz) * fx, t11 = -iz * fy, t12 = (yz * iz) * fy;
  const double s2 = ps * ps;
  const double A00 = s2 * (t00 * t00), A02 = s2 * (t00 * t02), A11 = s2 * (t11 * t11),
               A12 = s2 * (t11 * t12), A22 = s2 * (t02 * t02 + t12 * t12);
  double Q[3][3];  // R^T A
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    Q[i][0] = pr[i] * A00 + pr[6 + i] * A02;
    Q[i][1] = pr[3 + i] * A11 + pr[6 + i] * A12;
    Q[i][2] = pr[i] * A02 + pr[3 + i] * A12 + pr[6 + i] * A22;
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {  // B = R'^-T Q
    const double b0 = r[0] * Q[0][j], b1 = r[1] * Q[0][j] + r[3] * Q[1][j],
                 b2 = r[2] * Q[0][j] + r[4] * Q[1][j] + r[5] * Q[2][j];
    Q[0][j] = b0;
    Q[1][j] = b1;
    Q[2][j] = b2;
  }
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    double *yr = Y + (size_t)q * ld + col;
    yr[0] = Q[q][2] * m.y - Q[q][1] * m.z;
    yr[1] = Q[q][0] * m.z - Q[q][2] * m.x;
    yr[2] = Q[q][1] * m.x - Q[q][0] * m.y;
    yr[3] = Q[q][0];
    yr[4] = Q[q][1];
    yr[5] = Q[q][2];
  }
}

// occupancy the mono kernel of width NT is compiled for (its accumulators and
// LDS shrink with NT, so the narrower classes fit more workgroups per CU)
#ifndef SQLM_TILE_OCC_NARROW
#define SQLM_TILE_OCC_NARROW 5
#endif
#ifndef SQLM_TILE_OCC_MID
#define SQLM_TILE_OCC_MID 4
#endif
#ifndef SQLM_TILE_OCC_WIDE8
#define SQLM_TILE_OCC_WIDE8 3
#endif
template <int NT>
constexpr int tile_occ() {
  return NT <= 4 ? SQLM_TILE_OCC_NARROW : NT <= 6 ? SQLM_TILE_OCC_MID : NT <= 8 ? SQLM_TILE_OCC_WIDE8 : kTileOcc;
}

template <int NT, bool ST>
__global__ __launch_bounds__(kTileThreads, ST ? 2 : tile_occ<NT>()) void k_rcs_tile(DevProblem d, double lambda,
                                                                                   int cls_off) {
  // wave w owns the accumulator tiles q with q % kTileWaves == w; 3 waves per SIMD
  // for mono problems (167 VGPRs), 2 with the stereo row (spill-free)
  constexpr int TH = kTileThreads, NQ = NT * (NT + 1) / 2, NQW = (NQ + kTileWaves - 1) / kTileWaves;
  constexpr int NC = NT * 16;
  constexpr int BL = kTileBL;
  __shared__ double Ys[2][kTileRows][NC];
  // per-landmark data of the whole tile, loaded once: offsets, camera span, w, R'^-1
  __shared__ int Lb[kTileMaxLm + 1];
  __shared__ int2 Lu[kTileMaxLm];
  __shared__ double Lw[kTileMaxLm][3];
  __shared__ double Lr[kTileMaxLm][6];
  __shared__ double Lx[kTileMaxLm][3];            // landmarks at the linearization point
  __shared__ double Lc[kTileHardCams][16];        // window cameras: R t fx fy cx cy
  __shared__ double Lbf[ST ? kTileHardCams : 1];  // window cameras: bf (stereo edges)
  __shared__ int2 Bs[(kTileMaxLm + kTileBL - 1) / kTileBL];  // column span of every batch (cmin, cmax)
  const int t = d.tile_order[cls_off + blockIdx.x], tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int cp = d.tile_cam_ptr[t + 1] - d.tile_cam_ptr[t];
  const int ncol = 6 * cp, nt = (ncol + 15) >> 4;
  const int r16 = lane & 15, k4 = lane >> 4;
  d4v acc[NQW];
#pragma unroll
  for (int q = 0; q < NQW; ++q) acc[q] = d4v{0.0, 0.0, 0.0, 0.0};
  // gradient column tid - 64 of the tile (waves 1.., while wave 0, which
  // stages the common batch alone, moves on)
  static_assert(NT * 16 <= kTileThreads - 64, "one gradient column per thread of waves 1..");
  const int gcol = tid - 64;
  double gacc = 0.0;
  for (int k = tid; k < 2 * kTileRows * NC; k += TH) (&Ys[0][0][0])[k] = 0.0;
  const int l0 = d.tile_lm_ptr[t], l1 = d.tile_lm_ptr[t + 1], ntl = l1 - l0;
  const int nbatch = (ntl + BL - 1) / BL;
  const bool slow = d.tile_dups || d.tile_maxk > kTileFastK;
  for (int k = tid; k <= ntl; k += TH) Lb[k] = d.lm_begin[l0 + k];
  for (int k = tid; k < ntl; k += TH) Lu[k] = d.lm_urange[l0 + k];
  for (int li = tid; li < ntl; li += TH) damp_factor(d.lm_R + 8 * (l0 + li), d.lm_b + 4 * (l0 + li), lambda, Lr[li], Lw[li]);
  for (int k = tid; k < 3 * ntl; k += TH) {
    const int li = k / 3, c = k - 3 * li;
    Lx[li][c] = d.X[0][4 * (l0 + li) + c];
  }
  {
    const int cb = d.tile_cam_ptr[t];
    for (int k = tid; k < 16 * cp; k += TH) {
      const int u = k >> 4, c = k & 15;
      Lc[u][c] = d.pose_rt[0][16 * d.hidx_pose[d.tile_cams[cb + u]] + c];
    }
    if (ST)
      for (int u = tid; u < cp; u += TH) Lbf[u] = d.pose_bf[d.hidx_pose[d.tile_cams[cb + u]]];
  }
  for (int bt = tid; bt < nbatch; bt += TH) {  // batch spans from the landmarks' camera ranges
    int cmin = 1 << 30, cmax = -1;
    for (int li = BL * bt; li < min(BL * bt + BL, ntl); ++li) {
      const int2 ur = d.lm_urange[l0 + li];
      if (ur.x >= 0) { cmin = min(cmin, 6 * ur.x); cmax = max(cmax, 6 * ur.y + 6); }
    }
    Bs[bt] = int2{cmin, cmax};
  }
  __syncthreads();
  // prefetched raw inputs of one batch (fast path): thread tid owns observation b0 + tid
  double ps = 0.0, pur = -1.0;
  int pu = -1, pli = 0;
  auto fetch = [&](int bt) {
    const int lb = BL * bt, nl = min(BL, ntl - lb);
    const int b0 = Lb[lb], bn = Lb[lb + nl];
    const int e1 = nl > 1 ? Lb[lb + 1] : bn, e2 = nl > 2 ? Lb[lb + 2] : bn, e3 = nl > 3 ? Lb[lb + 3] : bn;
    const int o = b0 + tid;
    pu = -1;
    if (!slow && o < bn) {
      pli = lb + (o >= e1) + (o >= e2) + (o >= e3);  // tile-local landmark
      pu = d.obs_local[o];
      ps = d.obs_s[o];
      if (ST) pur = d.obs_ur[o];
    }
  };
  if (nbatch > 0) fetch(0);
  int2 prev = int2{-1, -1};  // column span of the previous batch (its buffer is cleared next)
  lds_barrier();
  TP_DECL
  for (int bt = 0; bt < nbatch; ++bt) {
    const int buf = bt & 1, lb = BL * bt, nl = min(BL, ntl - lb);
    double (*Y)[NC] = Ys[buf];
    // ---- stage Y rows 4li..4li+2 = R'^-T P for every landmark li of the batch;
    // meanwhile the waves without observations clear the previous batch's
    // columns in the other buffer (read by the MFMAs before the last barrier)
    if (!slow) {
      if (pu >= 0) {  // Y block of the observation: (R'^-1)^T jl^T jp, Jacobians recomputed once
        const double *pr = Lc[pu], *xl = Lx[pli], *r = Lr[pli];
        MonoEval m;
        m.x = pr[0] * xl[0] + pr[1] * xl[1] + pr[2] * xl[2] + pr[9];
        m.y = pr[3] * xl[0] + pr[4] * xl[1] + pr[5] * xl[2] + pr[10];
        m.z = pr[6] * xl[0] + pr[7] * xl[1] + pr[8] * xl[2] + pr[11];
        m.s = ps;
        const int row = 3 * (pli - lb), col = 6 * pu;
        if (!(ST && pur >= 0.0)) {
          // mono: jl = s J_pi R and jp = s J_pi [-[X_c]x | I] (types_six_dof_expmap.cpp:
          // 103-139), so P = jl^T jp = [-B' [X_c]x | B'] with B' = R^T A,
          // A = s^2 J_pi^T J_pi (3x3, five distinct entries), and Y = R'^-T P =
          // [-B [X_c]x | B], B = R'^-T R^T A: ~45 % fewer FP64 operations than
          // forming jl, jp and their 18 products
          const double iz = 1.0 / m.z, xz = m.x * iz, yz = m.y * iz, fx = pr[12], fy = pr[13];
          const double t00 = -iz * fx, t02 = (xz * iz) * fx, t11 = -iz * fy, t12 = (yz * iz) * fy;
          const double s2 = ps * ps;
          const double A00 = s2 * (t00 * t00), A02 = s2 * (t00 * t02), A11 = s2 * (t11 * t11),
                       A12 = s2 * (t11 * t12), A22 = s2 * (t02 * t02 + t12 * t12);
          double Q[3][3];  // R^T A
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            Q[i][0] = pr[i] * A00 + pr[6 + i] * A02;
            Q[i][1] = pr[3 + i] * A11 + pr[6 + i] * A12;
            Q[i][2] = pr[i] * A02 + pr[3 + i] * A12 + pr[6 + i] * A22;
          }
#pragma unroll
          for (int j = 0; j < 3; ++j) {  // B = R'^-T Q (R'^-1 upper: r0 r1 r2 / r3 r4 / r5)
            const double b0 = r[0] * Q[0][j], b1 = r[1] * Q[0][j] + r[3] * Q[1][j],
                         b2 = r[2] * Q[0][j] + r[4] * Q[1][j] + r[5] * Q[2][j];
            Q[0][j] = b0;
            Q[1][j] = b1;
            Q[2][j] = b2;
          }
#pragma unroll
          for (int q = 0; q < 3; ++q) {
            double *yr = &Y[row + q][col];
            yr[0] = Q[q][2] * m.y - Q[q][1] * m.z;
            yr[1] = Q[q][0] * m.z - Q[q][2] * m.x;
            yr[2] = Q[q][1] * m.x - Q[q][0] * m.y;
            yr[3] = Q[q][0];
            yr[4] = Q[q][1];
            yr[5] = Q[q][2];
          }
        } else {  // stereo: the third row's Jacobians join the products
          double jl[6], jp[12], jl3[3], jp3[6];
          mono_jac(pr, m, jl, jp);
          stereo_row(pr, m, Lbf[pu], jl, jp, jl3, jp3);
#pragma unroll
          for (int c = 0; c < 6; ++c) {
            const double p0 = jl[0] * jp[c] + jl[3] * jp[6 + c] + jl3[0] * jp3[c];
            const double p1 = jl[1] * jp[c] + jl[4] * jp[6 + c] + jl3[1] * jp3[c];
            const double p2 = jl[2] * jp[c] + jl[5] * jp[6 + c] + jl3[2] * jp3[c];
            Y[row][col + c] = r[0] * p0;
            Y[row + 1][col + c] = r[1] * p0 + r[3] * p1;
            Y[row + 2][col + c] = r[2] * p0 + r[4] * p1 + r[5] * p2;
          }
        }
      }
    } else if (tid < 6) {  // repeated cameras / long tracks: serial, observation order
      for (int li = 0; li < nl; ++li) {
        const double *Rp = Lr[lb + li];
        for (int o = Lb[lb + li]; o < Lb[lb + li + 1]; ++o) {
          const int u = d.obs_local[o];
          if (u < 0) continue;
          double pcol[3];
          const double *xl = Lx[lb + li];
          const double our = ST ? d.obs_ur[o] : -1.0;
          hlp_col<ST>(Lc[u], xl[0], xl[1], xl[2], d.obs_s[o], tid, pcol, our >= 0.0, ST ? Lbf[u] : 0.0);
          const double p0 = pcol[0], p1 = pcol[1], p2 = pcol[2];
          const double y0 = Rp[0] * p0;
          const double y1 = Rp[1] * p0 + Rp[3] * p1;
          const double y2 = Rp[2] * p0 + Rp[4] * p1 + Rp[5] * p2;
          Y[3 * li][6 * u + tid] += y0; Y[3 * li + 1][6 * u + tid] += y1; Y[3 * li + 2][6 * u + tid] += y2;
        }
      }
    }
    if (prev.x >= 0 && tid >= 64) {  // waves 1.. (wave 0 stages the common case alone)
#pragma unroll
      for (int row = 0; row < kTileRows; ++row)
        for (int col = prev.x + tid - 64; col < prev.y; col += TH - 64) Ys[buf ^ 1][row][col] = 0.0;
    }
    TP(0);
    lds_barrier();  // (A) batch staged, the other buffer clear
    TP(1);
    if (bt + 1 < nbatch) fetch(bt + 1);  // in flight during the MFMAs below
    TP(2);
    const int2 bsp = Bs[bt];
    const int cmin = bsp.x, cmax = bsp.y;
    TP(3);
    if (cmax > 0) {
      const int tmin = cmin >> 4, tmax = (cmax - 1) >> 4;
      tile_mfma_wave<NT>(wave, acc, Y, tmin, tmax, (3 * nl + 3) >> 2, r16, k4);
      TP(4);
      if (gcol >= cmin && gcol < cmax) {
        double gs = 0.0;
        for (int li = 0; li < nl; ++li)
          gs += Y[3 * li][gcol] * Lw[lb + li][0] + Y[3 * li + 1][gcol] * Lw[lb + li][1] +
                Y[3 * li + 2][gcol] * Lw[lb + li][2];
        gacc -= gs;
      }
      prev = int2{cmin, cmax};
    } else {
      prev = int2{-1, -1};
    }
    TP(5);
    lds_barrier();  // (B) every wave is done with this buffer before it is cleared
    TP(6);
  }
  TP_STORE;
  if (d.cr_direct) {  // this tile's share of clearing the CR superblocks that k_rcs_reduce fills next
    const int64_t tot = (int64_t)d.cr_p * d.cr_n * d.cr_n;  // doubles per array (even: n % 16 == 0)
    const int64_t per = ((tot + d.n_tiles - 1) / d.n_tiles + 1) & ~(int64_t)1;
    const int64_t a0 = (int64_t)t * per, a1 = min(tot, a0 + per);
    for (int64_t k = a0 + 2 * tid; k < a1; k += 2 * TH) {
      store2(d.cr_D + k, 0.0, 0.0);
      store2(d.cr_E + k, 0.0, 0.0);
    }
  }
  // write -G_t as the tile's partial, block-major (tile_blk): element (R, C) of
  // an upper 16x16 tile goes to block (R/6, C/6) if that block is upper; a
  // diagonal block straddling two tiles also gets the mirror of the elements
  // whose transpose falls in the (never computed) lower tile
  double *out = d.part + d.tile_part_ptr[t];
  const int n6 = 6 * cp;
  int q = 0;
#pragma unroll
  for (int ti = 0; ti < NT; ++ti)
#pragma unroll
    for (int tj = ti; tj < NT; ++tj, ++q) {
      if (q % kTileWaves == wave && tj < nt) {
        const int C = tj * 16 + r16, w = C / 6, c = C - 6 * w;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int R = ti * 16 + k4 + 4 * j, u = R / 6, r = R - 6 * u;
          if (R < n6 && C < n6 && u <= w) {
            double *blk = out + 36 * tile_blk(u, w, cp);
            const double v = -acc[q / kTileWaves][j];
            blk[6 * r + c] = v;
            if (u == w && ti < tj) blk[6 * c + r] = v;
          }
        }
      }
    }
  double *go = d.gpart + d.tile_gpart_ptr[t];
  if (gcol >= 0 && gcol < ncol) go[gcol] = gacc;
}

// ---- producer / consumer RCS tiles (mono, no repeated cameras) ----
// k_rcs_tile runs every batch in two barrier-separated phases that all four
// waves take part in: wave 0 stages the batch while waves 1-3 clear, then
// every wave runs its quarter of the MFMAs. The phase profile
// (scripts/tile_prof.py) puts wave 0 at 31 % staging, 32 % MFMA and 20 %
// parked at the two barriers. Here wave 0 only produces: while waves 1-3 run
// batch b's MFMAs (tiles q with q % 3 == wave - 1) and gradient columns from
// one LDS buffer, wave 0 clears the entries it staged two batches ago in the
// other buffer and stages batch b + 1 there (two observations per lane, so a
// batch of up to 128 observations is one pass, and the two chains give the
// lone wave some ILP); ONE barrier per batch hands the buffers over. Every
// accumulator tile sums the same products in the same order as k_rcs_tile
// (only its owner wave changes) and the gradient code is the same: the
// partials are bitwise identical to k_rcs_tile's.
constexpr int kTileCons = kTileWaves - 1;  // consumer waves
// Wide classes (NT >= 8) one K step at a time (its NT operand tiles in
// registers, then every owned pair of the span): each accumulator still adds
// its K steps in order, so the sums are the same bits as k_rcs_tile's, with a
// third of the operand registers (NT = 8: 155 -> 124 VGPRs, 4 waves per SIMD;
// NT = 9 fits 3). The narrow classes keep all operands loaded at once (the
// stepped form of NT = 4 spilled).
#ifndef SQLM_TILE_KS_STEP_MIN
#define SQLM_TILE_KS_STEP_MIN 8
#endif
template <int NT, int P, int NC>
__device__ __forceinline__ void tile_mfma_cons(d4v *acc, const double (*Y)[NC], int tmin, int tmax, int nks, int r16,
                                               int k4) {
  if constexpr (NT >= SQLM_TILE_KS_STEP_MIN) {
#pragma unroll
  for (int ks = 0; ks < kTileKS; ++ks) {
    if (ks < nks) {
      double op[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) op[t] = Y[4 * ks + k4][t * 16 + r16];
      int q = 0;
#pragma unroll
      for (int ti = 0; ti < NT; ++ti) {
#pragma unroll
        for (int tj = ti; tj < NT; ++tj, ++q) {
          if (q % kTileCons == P && ti >= tmin && tj <= tmax)
            acc[q / kTileCons] = __builtin_amdgcn_mfma_f64_16x16x4f64(op[ti], op[tj], acc[q / kTileCons], 0, 0, 0);
        }
      }
    }
  }
  } else {
    double op[NT][kTileKS];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int ks = 0; ks < kTileKS; ++ks) op[t][ks] = Y[4 * ks + k4][t * 16 + r16];
    int q = 0;
#pragma unroll
    for (int ti = 0; ti < NT; ++ti) {
#pragma unroll
      for (int tj = ti; tj < NT; ++tj, ++q) {
        if (q % kTileCons == P && ti >= tmin && tj <= tmax) {
#pragma unroll
          for (int ks = 0; ks < kTileKS; ++ks)
            if (ks < nks)
              acc[q / kTileCons] =
                  __builtin_amdgcn_mfma_f64_16x16x4f64(op[ti][ks], op[tj][ks], acc[q / kTileCons], 0, 0, 0);
        }
      }
    }
  }
}

// observations a producer lane stages per batch (lane, lane + 64): batches of
// up to kProdObs observations take the producer path
constexpr int kProdPer = 2, kProdObs = 64 * kProdPer;

// Consumer wave P (wave P + 1) of k_rcs_tile_p: one instantiation per wave,
// so its accumulator tiles (q % 3 == P) are compile-time registers that live
// in this branch only. After each batch's MFMAs and gradient column it joins
// the batch barrier; at the end it writes its tiles of the partial.
template <int NT, int P, int NC>
__device__ __forceinline__ void tile_consumer(const DevProblem &d, int t, int cp, int ntl, int nbatch,
                                              const double (*Ys)[kTileRows][NC], const double (*Lw)[3],
                                              const int2 *Bs, int tid) {
  constexpr int NQ = NT * (NT + 1) / 2, NQW = (NQ + kTileCons - 1) / kTileCons, BL = kTileBL;
  const int lane = tid & 63, r16 = lane & 15, k4 = lane >> 4, gcol = tid - 64;
  const int ncol = 6 * cp, nt = (ncol + 15) >> 4;
  d4v acc[NQW];
#pragma unroll
  for (int q = 0; q < NQW; ++q) acc[q] = d4v{0.0, 0.0, 0.0, 0.0};
  double gacc = 0.0;
  TP_DECL
  lds_barrier();  // batch 0 staged
  TP(3);
  for (int bt = 0; bt < nbatch; ++bt) {
    const int lb = BL * bt, nl = min(BL, ntl - lb);
    const double(*Y)[NC] = Ys[bt & 1];
    const int2 bsp = Bs[bt];
    const int cmin = __builtin_amdgcn_readfirstlane(bsp.x), cmax = __builtin_amdgcn_readfirstlane(bsp.y);
    if (cmax > 0) {
      const int tmin = cmin >> 4, tmax = (cmax - 1) >> 4;
      tile_mfma_cons<NT, P>(acc, Y, tmin, tmax, (3 * nl + 3) >> 2, r16, k4);
      if (gcol >= cmin && gcol < cmax) {
        double gs = 0.0;
        for (int li = 0; li < nl; ++li)
          gs += Y[3 * li][gcol] * Lw[lb + li][0] + Y[3 * li + 1][gcol] * Lw[lb + li][1] +
                Y[3 * li + 2][gcol] * Lw[lb + li][2];
        gacc -= gs;
      }
    }
    TP(2);  // consumer: MFMAs + gradient
    lds_barrier();  // batch bt + 1 staged, batch bt's buffer free
    TP(3);  // consumer: waiting for the producer
  }
  if (P == 0) TP_STORE_BY(64);
  // -G_t as the tile's partial, block-major (as k_rcs_tile)
  double *out = d.part + d.tile_part_ptr[t];
  const int n6 = 6 * cp;
  int q = 0;
#pragma unroll
  for (int ti = 0; ti < NT; ++ti)
#pragma unroll
    for (int tj = ti; tj < NT; ++tj, ++q) {
      if (q % kTileCons == P && tj < nt) {
        const int C = tj * 16 + r16, w = C / 6, c = C - 6 * w;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int R = ti * 16 + k4 + 4 * j, u = R / 6, r = R - 6 * u;
          if (R < n6 && C < n6 && u <= w) {
            double *blk = out + 36 * tile_blk(u, w, cp);
            const double v = -acc[q / kTileCons][j];
            blk[6 * r + c] = v;
            if (u == w && ti < tj) blk[6 * c + r] = v;
          }
        }
      }
    }
  double *go = d.gpart + d.tile_gpart_ptr[t];
  if (gcol >= 0 && gcol < ncol) go[gcol] = gacc;
}

// waves per SIMD k_rcs_tile_p is compiled for: the consumer waves' registers
// without spills (NT = 8: 124 VGPRs, 6: 84, 9: 150)
#ifndef SQLM_TILE_P_OCC_MID
#define SQLM_TILE_P_OCC_MID 4
#endif
template <int NT>
constexpr int tile_p_occ() {
  return NT <= 3 ? 5 : NT <= 8 ? SQLM_TILE_P_OCC_MID : 3;
}
template <int NT>
__global__ __launch_bounds__(kTileThreads, tile_p_occ<NT>()) void k_rcs_tile_p(DevProblem d, double lambda, int cls_off) {
  constexpr int TH = kTileThreads, NC = NT * 16, BL = kTileBL;
  __shared__ double Ys[2][kTileRows][NC];
  __shared__ int Lb[kTileMaxLm + 1];
  __shared__ double Lw[kTileMaxLm][3];
  __shared__ double Lr[kTileMaxLm][6];
  __shared__ double Lx[kTileMaxLm][3];
  __shared__ double Lc[kTileHardCams][16];
  __shared__ int2 Bs[(kTileMaxLm + kTileBL - 1) / kTileBL];
  const int t = d.tile_order[cls_off + blockIdx.x], tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: the role branches are scalar
  const int cp = d.tile_cam_ptr[t + 1] - d.tile_cam_ptr[t];
  static_assert(NT * 16 <= kTileThreads - 64, "one gradient column per thread of waves 1..");
  static_assert(kTileHardCams <= 32, "the producer's staged-position code holds a camera in 5 bits");
  for (int k = tid; k < 2 * kTileRows * NC; k += TH) (&Ys[0][0][0])[k] = 0.0;
  const int l0 = d.tile_lm_ptr[t], l1 = d.tile_lm_ptr[t + 1], ntl = l1 - l0;
  const int nbatch = (ntl + BL - 1) / BL;
  for (int k = tid; k <= ntl; k += TH) Lb[k] = d.lm_begin[l0 + k];
  for (int li = tid; li < ntl; li += TH) damp_factor(d.lm_R + 8 * (l0 + li), d.lm_b + 4 * (l0 + li), lambda, Lr[li], Lw[li]);
  for (int k = tid; k < 3 * ntl; k += TH) {
    const int li = k / 3, c = k - 3 * li;
    Lx[li][c] = d.X[0][4 * (l0 + li) + c];
  }
  {
    const int cb = d.tile_cam_ptr[t];
    for (int k = tid; k < 16 * cp; k += TH) {
      const int u = k >> 4, c = k & 15;
      Lc[u][c] = d.pose_rt[0][16 * d.hidx_pose[d.tile_cams[cb + u]] + c];
    }
  }
  for (int bt = tid; bt < nbatch; bt += TH) {  // batch spans from the landmarks' camera ranges
    int cmin = 1 << 30, cmax = -1;
    for (int li = BL * bt; li < min(BL * bt + BL, ntl); ++li) {
      const int2 ur = d.lm_urange[l0 + li];
      if (ur.x >= 0) { cmin = min(cmin, 6 * ur.x); cmax = max(cmax, 6 * ur.y + 6); }
    }
    Bs[bt] = int2{cmin, cmax};
  }
  if (d.cr_direct) {  // this tile's share of clearing the CR superblocks that k_rcs_reduce fills next
    const int64_t tot = (int64_t)d.cr_p * d.cr_n * d.cr_n;
    const int64_t per = ((tot + d.n_tiles - 1) / d.n_tiles + 1) & ~(int64_t)1;
    const int64_t a0 = (int64_t)t * per, a1 = min(tot, a0 + per);
    for (int64_t k = a0 + 2 * tid; k < a1; k += 2 * TH) {
      store2(d.cr_D + k, 0.0, 0.0);
      store2(d.cr_E + k, 0.0, 0.0);
    }
  }
  __syncthreads();
  // Two role loops with the same number of barriers (nbatch + 1): between
  // barriers b - 1 and b the producer stages batch b into buffer b & 1 while
  // the consumers work on batch b - 1 in the other buffer. Each role keeps
  // only its own state live (the accumulators exist in the consumer branch).
  if (wave == 0) {
    // the prefetched raw inputs of the next batch (two observations per lane),
    // and where this lane staged in each buffer: 32 row + camera, -1: nothing
    // (separate registers per buffer, selected by value: a runtime index into
    // a register array would put it in scratch)
    int pu0 = -1, pu1 = -1, pl0 = 0, pl1 = 0, w00 = -1, w01 = -1, w10 = -1, w11 = -1;
    double ps0 = 0.0, ps1 = 0.0;
    auto fetch_in = [&](int sb) {
      const int lb = BL * sb, nl = min(BL, ntl - lb);
      const int b0 = Lb[lb], bn = Lb[lb + nl];
      const int e1 = nl > 1 ? Lb[lb + 1] : bn, e2 = nl > 2 ? Lb[lb + 2] : bn, e3 = nl > 3 ? Lb[lb + 3] : bn;
      const int o0 = b0 + lane, o1 = o0 + 64;
      pu0 = o0 < bn ? d.obs_local[o0] : -1;
      pu1 = o1 < bn ? d.obs_local[o1] : -1;
      ps0 = o0 < bn ? d.obs_s[o0] : 0.0;
      ps1 = o1 < bn ? d.obs_s[o1] : 0.0;
      pl0 = lb + (o0 >= e1) + (o0 >= e2) + (o0 >= e3);
      pl1 = lb + (o1 >= e1) + (o1 >= e2) + (o1 >= e3);
    };
    if (nbatch > 0) fetch_in(0);
    TP_DECL
    for (int sb = 0; sb <= nbatch; ++sb) {
      if (sb < nbatch) {
        const int buf = sb & 1, lb = BL * sb;
        double(*Y)[NC] = Ys[buf];
        // clear what this lane staged in this buffer two batches ago
        const int c0 = buf ? w10 : w00, c1 = buf ? w11 : w01;
        if (c0 >= 0) {
#pragma unroll
          for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 6; c += 2) store2(&Y[(c0 >> 5) + r][6 * (c0 & 31) + c], 0.0, 0.0);
        }
        if (c1 >= 0) {
#pragma unroll
          for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 6; c += 2) store2(&Y[(c1 >> 5) + r][6 * (c1 & 31) + c], 0.0, 0.0);
        }
        int n0 = -1, n1 = -1;
        if (pu0 >= 0) {
          const int row = 3 * (pl0 - lb);
          stage_mono_y(Lc[pu0], Lx[pl0], Lr[pl0], ps0, &Y[row][0], NC, 6 * pu0);
          n0 = 32 * row + pu0;  // (cp <= 24 cameras)
        }
        if (pu1 >= 0) {
          const int row = 3 * (pl1 - lb);
          stage_mono_y(Lc[pu1], Lx[pl1], Lr[pl1], ps1, &Y[row][0], NC, 6 * pu1);
          n1 = 32 * row + pu1;
        }
        if (buf) {
          w10 = n0;
          w11 = n1;
        } else {
          w00 = n0;
          w01 = n1;
        }
        if (sb + 1 < nbatch) fetch_in(sb + 1);  // in flight across the barrier (LDS-only)
      }
      TP(0);  // producer: clear + stage + prefetch issue
      lds_barrier();
      TP(1);  // producer: waiting for the consumers
    }
    TP_STORE_BY(0);
  } else if (wave == 1) {
    tile_consumer<NT, 0>(d, t, cp, ntl, nbatch, Ys, Lw, Bs, tid);
  } else if (wave == 2) {
    tile_consumer<NT, 1>(d, t, cp, ntl, nbatch, Ys, Lw, Bs, tid);
  } else {
    tile_consumer<NT, 2>(d, t, cp, ntl, nbatch, Ys, Lw, Bs, tid);
  }
}

// S block s = sum of its tile partials + H_pp + lambda I on the diagonal; g
// row i likewise. Each contribution is one 36-double block of a tile's
// block-major partial (tile_blk), or 6 doubles of its g partial, at a
// host-precomputed offset. With cr_direct the sums go straight into the
// block-tridiagonal superblocks of the CR solver (D_I and its mirror,
// E_I = S(I, I+1), g_I, identity on padded rows) or, on a band + border layout,
// into F^T / the border system, replacing the BSR copy and its scatter.
//
// Summation order is fixed (deterministic, no atomics): a list of up to
// kRedLong contributions is summed by one thread in list order, eight loads in
// flight; a longer one (the cameras of a loop closure collect hundreds) by a
// workgroup, groups of threads taking every G-th contribution, the group sums
// then added in group order.
__device__ __forceinline__ void rcs_put_s(const DevProblem &d, int s, int e, double v, double lambda) {
  const int r = e / 6, c = e % 6;
  const bool own = !d.sharded || d.rank == 0;
  const int j = d.s_col[s];
  if (s == d.s_row_ptr[j]) {  // diagonal block (first block of row j); sharded: this rank's share
    v += d.Hpp[36 * j + e];
    if (r == c && own) v += lambda;
  }
  if (!d.cr_direct) {
    d.S[(int64_t)s * 36 + e] = v;
    return;
  }
  const int i = d.s_row[s], n = d.cr_n, B = d.cr_B;
  const int pi = d.cam_pos ? d.cam_pos[i] : i, pj = d.cam_pos ? d.cam_pos[j] : j;
  if (pi >= 0 && pj >= 0) {  // band (positions ascend with the camera index)
    const int I = pi / B, li = pi - I * B, J = pj / B, lj = pj - J * B;
    double *base = (J == I ? d.cr_D : d.cr_E) + (size_t)I * n * n;
    base[(6 * li + r) * n + 6 * lj + c] = v;
    if (J == I && j != i) base[(6 * lj + c) * n + 6 * li + r] = v;
  } else if (pi >= 0) {  // band row, border column: F^T
    const int I = pi / B, li = pi - I * B;
    d.arw_G[((size_t)I * n + 6 * li + r) * d.arw_R + 6 * (-1 - pj) + c] = v;
  } else if (pj >= 0) {
    const int J = pj / B, lj = pj - J * B;
    d.arw_G[((size_t)J * n + 6 * lj + c) * d.arw_R + 6 * (-1 - pi) + r] = v;
  } else {  // border system, both triangles
    const int bi = -1 - pi, bj = -1 - pj;
    d.bd_A[(size_t)(6 * bi + r) * d.arw_Rp + 6 * bj + c] = v;
    d.bd_A[(size_t)(6 * bj + c) * d.arw_Rp + 6 * bi + r] = v;
  }
}

__device__ __forceinline__ void rcs_put_g(const DevProblem &d, int i, int r, double v) {
  v += d.bp[8 * i + r];
  d.g[6 * i + r] = v;
  if (d.cr_direct) {
    const int pi = d.cam_pos ? d.cam_pos[i] : i;
    if (pi >= 0) {
      const int I = pi / d.cr_B, li = pi - I * d.cr_B;
      d.cr_g[(size_t)I * d.cr_n + 6 * li + r] = v;
    } else {
      d.bd_r[6 * (-1 - pi) + r] = v;
    }
  }
}

// sum of src[off[k] + e] over k = k0, k0 + step, ... < k1 in that order, eight loads in flight
__device__ __forceinline__ double red_sum(const double *src, const int64_t *off, int k0, int k1, int step, int e) {
  double v = 0.0;
  if (step == 1 && k1 - k0 <= kRedLong) {  // short list: offsets first (see red_sumv)
    int64_t o[kRedLong];
#pragma unroll
    for (int u = 0; u < kRedLong; ++u) o[u] = k0 + u < k1 ? off[k0 + u] : -1;
#pragma unroll
    for (int g = 0; g < kRedLong; g += 8) {
      if (k0 + g >= k1) break;
      double p8[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) p8[u] = o[g + u] >= 0 ? src[o[g + u] + e] : 0.0;
#pragma unroll
      for (int u = 0; u < 8; ++u) v += p8[u];
    }
    return v;
  }
  for (int k = k0; k < k1; k += 8 * step) {
    double p8[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) p8[u] = k + u * step < k1 ? src[off[k + u * step] + e] : 0.0;
#pragma unroll
    for (int u = 0; u < 8; ++u) v += p8[u];
  }
  return v;
}

// the same sum for the entries e .. e + V - 1 (V = 2 or 4, e a multiple of V):
// 16-byte loads per contribution (every contribution starts at a multiple of 36 doubles)
// A short list (<= kRedLong contributions): every offset is loaded first, in
// one round trip, then the values in groups of eight -- two dependent memory
// round trips in all instead of two per group (the sum keeps list order).
template <int V>
__device__ __forceinline__ void red_sumv(const double *src, const int64_t *off, int k0, int k1, int e, double *v) {
#pragma unroll
  for (int j = 0; j < V; ++j) v[j] = 0.0;
  if (k1 - k0 <= kRedLong) {
    int64_t o[kRedLong];
#pragma unroll
    for (int u = 0; u < kRedLong; ++u) o[u] = k0 + u < k1 ? off[k0 + u] : -1;
#pragma unroll
    for (int g = 0; g < kRedLong; g += 8) {
      if (k0 + g >= k1) break;
      double2 p8[8][V / 2];
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int j = 0; j < V / 2; ++j)
          p8[u][j] = o[g + u] >= 0 ? *reinterpret_cast<const double2 *>(src + o[g + u] + e + 2 * j) : make_double2(0.0, 0.0);
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int j = 0; j < V / 2; ++j) {
          v[2 * j] += p8[u][j].x;
          v[2 * j + 1] += p8[u][j].y;
        }
    }
    return;
  }
  for (int k = k0; k < k1; k += 8) {
    double2 p8[8][V / 2];
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int j = 0; j < V / 2; ++j)
        p8[u][j] = k + u < k1 ? *reinterpret_cast<const double2 *>(src + off[k + u] + e + 2 * j) : make_double2(0.0, 0.0);
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int j = 0; j < V / 2; ++j) {
        v[2 * j] += p8[u][j].x;
        v[2 * j + 1] += p8[u][j].y;
      }
  }
}

// S entries per thread of k_rcs_reduce (2 or 4; A/B: -DSQLM_RED_V=4)
#ifndef SQLM_RED_V
#define SQLM_RED_V 2
#endif
constexpr int kRedV = SQLM_RED_V, kRedPer = 36 / kRedV;

// threads per k_rcs_reduce workgroup: a long list (the cameras of a loop
// closure, every block of a small local-BA system) is summed by kRedThreads / 36
// groups, so the width sets that critical path (A/B: -DSQLM_RED_THREADS=1024)
#ifndef SQLM_RED_THREADS
#define SQLM_RED_THREADS 256
#endif
constexpr int kRedThreads = SQLM_RED_THREADS;
constexpr int kRedGroupsS = kRedThreads / 36, kRedGroupsG = kRedThreads / 6;

__global__ __launch_bounds__(kRedThreads) void k_rcs_reduce(DevProblem d, double lambda, int short_blocks) {
  if ((int)blockIdx.x >= short_blocks) {  // one long S block or g row per workgroup
    __shared__ double part[kRedThreads];
    const int w = blockIdx.x - short_blocks, tid = threadIdx.x;
    if (w < d.n_long_s) {
      const int s = d.long_s[w], e = tid % 36, grp = tid / 36;
      const int k0 = d.red_ptr[s], k1 = d.red_ptr[s + 1];
      if (grp < kRedGroupsS) part[tid] = red_sum(d.part, d.red_off, k0 + grp, k1, kRedGroupsS, e);
      __syncthreads();
      if (tid < 36) {
        double v = 0.0;
        for (int g = 0; g < kRedGroupsS; ++g) v += part[36 * g + tid];
        rcs_put_s(d, s, tid, v, lambda);
      }
    } else {
      const int i = d.long_g[w - d.n_long_s], e = tid % 6, grp = tid / 6;
      const int k0 = d.gred_ptr[i], k1 = d.gred_ptr[i + 1];
      if (grp < kRedGroupsG) part[tid] = red_sum(d.gpart, d.gred_off, k0 + grp, k1, kRedGroupsG, e);
      __syncthreads();
      if (tid < 6) {
        double v = 0.0;
        for (int g = 0; g < kRedGroupsG; ++g) v += part[6 * g + tid];
        rcs_put_g(d, i, tid, v);
      }
    }
    return;
  }
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid < d.nnzb * kRedPer) {  // kRedV consecutive entries of the 6x6 block
    const int s = (int)(gid / kRedPer), e = kRedV * (int)(gid % kRedPer);
    const int k0 = d.red_ptr[s], k1 = d.red_ptr[s + 1];
    if (k1 - k0 <= kRedLong) {
      double v[kRedV];
      red_sumv<kRedV>(d.part, d.red_off, k0, k1, e, v);
#pragma unroll
      for (int j = 0; j < kRedV; ++j) rcs_put_s(d, s, e + j, v[j], lambda);
    }
  }
  const int64_t g2 = gid - d.nnzb * kRedPer;
  if (g2 >= 0 && g2 < (int64_t)d.nP * 6) {
    const int i = (int)(g2 / 6), r = (int)(g2 % 6);
    const int k0 = d.gred_ptr[i], k1 = d.gred_ptr[i + 1];
    if (k1 - k0 <= kRedLong) rcs_put_g(d, i, r, red_sum(d.gpart, d.gred_off, k0, k1, 1, r));
  }
  if (d.cr_direct) {  // identity on the padded rows of every superblock; solve flag
    const int64_t g3 = g2 - (int64_t)d.nP * 6;
    if (g3 >= 0 && g3 < (int64_t)d.cr_p * d.cr_n) {
      const int I = (int)(g3 / d.cr_n), rr = (int)(g3 % d.cr_n);
      const int used = min(d.cr_B, d.cr_nband - I * d.cr_B);
      if (rr >= 6 * used) {
        d.cr_D[((size_t)I * d.cr_n + rr) * d.cr_n + rr] = 1.0;
        d.cr_g[(size_t)I * d.cr_n + rr] = 0.0;
      }
    }
    if (gid == 0) d.flags[0] = 1;
  }
}

// the producer / consumer kernel for classes up to 8 tiles wide (the
// 9-wide class keeps k_rcs_tile: 15 accumulator tiles per consumer wave would
// not fit its 3 waves per SIMD)
#ifndef SQLM_TILE_PROD_MAXNT
#define SQLM_TILE_PROD_MAXNT 9
#endif
template <int NTT>
void launch_tile_p(int cnt, hipStream_t S, const DevProblem &d, double lambda, int off) {
  if constexpr (NTT <= SQLM_TILE_PROD_MAXNT)
    hipLaunchKernelGGL((k_rcs_tile_p<NTT>), dim3(cnt), dim3(kTileThreads), 0, S, d, lambda, off);
  else
    hipLaunchKernelGGL((k_rcs_tile<NTT, false>), dim3(cnt), dim3(kTileThreads), 0, S, d, lambda, off);
}

void launch_rcs_tiles(const DevProblem &d, double lambda, int max_cp, int max_k, hipStream_t st,
                      const TileStreams *ts) {
  if (d.nP == 0) return;
  (void)max_k;
  (void)max_cp;
  if (d.n_tiles > 0) {
    // one launch per accumulator-width class (4, 6, 8, 9); the classes go to
    // three streams so that no launch's tail leaves the chip idle: 8 (the
    // most work) on st, 6 on the first tile stream, the few widest tiles (9,
    // one round of long-running workgroups) then 4 on the second
    int ncls = 0;
    for (int k = 0; k <= kTileNtMax; ++k) ncls += d.tile_cls_cnt[k] > 0;
    // one class (small windows): no fork / join (one stream for all classes
    // measured 687 -> 624 it/s, profiles/r03/ab_tile_serial_grid.log)
    const bool par = ts && ts->s[0] && ts->s[1] && ncls > 1;
#ifdef SQLM_TILE_HTRACE
    static double acc[8] = {};
    static int nacc = 0;
    auto tnow = [] { return std::chrono::steady_clock::now(); };
    auto tp0 = tnow();
    int tk = 0;
    auto tm = [&] {
      const auto n = tnow();
      acc[tk++] += std::chrono::duration<double, std::micro>(n - tp0).count();
      tp0 = n;
    };
#define TH_MARK tm()
#else
#define TH_MARK
#endif
    if (par) {
      (void)hipEventRecord(ts->fork, st);
      TH_MARK;
    }
    // mono tiles without repeated cameras whose batches fit the producer wave:
    // the producer / consumer kernel
    const bool prod_tiles = !d.has_stereo && !d.tile_dups && d.tile_maxk * kTileBL <= kProdObs && d.tile_prod;
#define SQLM_TILE(NTT, S)                                                                                     \
  do {                                                                                                        \
    const int cnt = d.tile_cls_cnt[NTT], off = d.tile_cls_off[NTT];                                            \
    if (cnt > 0) {                                                                                            \
      if (d.has_stereo)                                                                                       \
        hipLaunchKernelGGL((k_rcs_tile<NTT, true>), dim3(cnt), dim3(kTileThreads), 0, S, d, lambda, off);      \
      else if (prod_tiles)                                                                                    \
        launch_tile_p<NTT>(cnt, S, d, lambda, off);                                                           \
      else                                                                                                    \
        hipLaunchKernelGGL((k_rcs_tile<NTT, false>), dim3(cnt), dim3(kTileThreads), 0, S, d, lambda, off);     \
    }                                                                                                         \
  } while (0)
    // (the chain 9, 4, 3 on the context stream instead, so that the reduce
    // follows its last kernel in-queue: within noise, profiles/r05/
    // ab_stream_order_rejected.log)
    const hipStream_t sm = par ? ts->s[0] : st, sn = par ? ts->s[1] : st;
    SQLM_TILE(8, st);
    // the side streams' waits (≈10 us of host time each) after the first
    // class is on its way: the fork event already marks st's position before it
    // (tile phase 0.520 -> 0.516 ms, profiles/r05/ab_tile_first8_r5p.log)
    if (par) {
      (void)hipStreamWaitEvent(ts->s[0], ts->fork, 0);
      (void)hipStreamWaitEvent(ts->s[1], ts->fork, 0);
    }
    TH_MARK;
    // (4 behind 6, or behind 8: config 4 777 -> 776 / 761 it/s,
    // profiles/r05/ab_tile_stream_assign_rejected.log)
    SQLM_TILE(6, sm);
    TH_MARK;
    SQLM_TILE(9, sn); SQLM_TILE(4, sn); SQLM_TILE(3, sn);
    TH_MARK;
#undef SQLM_TILE
    if (par) {
      (void)hipEventRecord(ts->join[0], ts->s[0]);
      (void)hipEventRecord(ts->join[1], ts->s[1]);
      TH_MARK;
      (void)hipStreamWaitEvent(st, ts->join[0], 0);
      (void)hipStreamWaitEvent(st, ts->join[1], 0);
      TH_MARK;
    }
#ifdef SQLM_TILE_HTRACE
    if (++nacc % 20 == 0) {
      std::fprintf(stderr, "tile launch host us (fork rec, -, cls8 + fork waits, cls6, cls9/4/3, join recs, join waits):");
      for (int k = 0; k < tk; ++k) std::fprintf(stderr, " %.1f", acc[k] / nacc);
      std::fprintf(stderr, "\n");
    }
#endif
#undef TH_MARK
  }
}

#ifdef SQLM_TILE_PROF
int tile_profile_read(long long *out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tile_prof), sizeof(g_tile_prof)) == hipSuccess ? 0 : -2;
}
#endif

void launch_rcs_reduce(const DevProblem &d, double lambda, hipStream_t st) {
  if (d.nP == 0) return;
  const int64_t items = d.nnzb * kRedPer + (int64_t)d.nP * 6 + (d.cr_direct ? (int64_t)d.cr_p * d.cr_n : 0);
  const int short_blocks = (int)((items + kRedThreads - 1) / kRedThreads);
  hipLaunchKernelGGL(k_rcs_reduce, dim3((unsigned)(short_blocks + d.n_long_s + d.n_long_g)), dim3(kRedThreads), 0, st,
                     d, lambda, short_blocks);
}

// ---------------------------------------------------------------- dense solve

// BSR upper blocks of S -> lower triangle of the padded dense matrix (row-major,
// ld n_pad, zeroed beforehand): one thread per BSR entry writes its transposed
// position; then identity on the padded rows and r = g (zero padded).
__global__ __launch_bounds__(256) void k_dense_scatter(DevProblem d) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int np_ = d.dense_n, n = 6 * d.nP;
  if (k < d.nnzb * 36) {
    const int s = (int)(k / 36), e = (int)(k % 36);
    const int r = 6 * d.s_row[s] + e / 6, c = 6 * d.s_col[s] + e % 6;  // upper entry (r, c)
    if (r <= c) d.dense[(int64_t)c * np_ + r] = d.S[k];
  } else if (k < d.nnzb * 36 + np_) {
    const int r = (int)(k - d.nnzb * 36);
    d.dense_r[r] = r < n ? d.g[r] : 0.0;
    if (r >= n) d.dense[(int64_t)r * np_ + r] = 1.0;
  }
}

__global__ void k_dense_copy_dx(DevProblem d) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < 6 * d.nP) d.dx[k] = d.flags[0] ? d.dense_x[k] : 0.0;
}

// LinearSolverEigen::solve on a dense S: blocked right-looking Cholesky with
// 112-wide LDS diagonal factors and MFMA panel / trailing updates, then the two
// block triangular solves. A non-positive pivot clears flags[0] (rejected trial).
int launch_dense_solve(const DevProblem &d, hipStream_t st) {
  const int n = 6 * d.nP;
  if (n == 0) return 0;
  const int64_t nn = (int64_t)d.dense_n * d.dense_n;
  if (hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d.flags), 1, 1, st) != hipSuccess) return -2;
  if (hipMemsetAsync(d.dense, 0, sizeof(double) * nn, st) != hipSuccess) return -2;
  const int64_t items = d.nnzb * 36 + d.dense_n;
  hipLaunchKernelGGL(k_dense_scatter, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, st, d);
  // the last block's real rows (16-rounded; identity padding after them is not factored)
  const int n_last = ((n - (d.dense_n - kCRMaxN)) + 15) / 16 * 16;
  if (launch_dense_spd_solve(d.dense, d.dense_L, d.dense_Linv, d.dense_r, d.dense_x, d.flags, d.dense_n, st, 0,
                             n_last))
    return -2;
  hipLaunchKernelGGL(k_dense_copy_dx, dim3((n + 255) / 256), dim3(256), 0, st, d);
  return 0;
}

// ---------------------------------------------------------------- updates

// CR: the pose's dx is read from the cyclic-reduction solution (band position
// or border slot; 0 if the solve flagged a non-positive pivot) and written to
// dx for the landmark update -- the k_cr_gather step folded into this launch.
// The trial pose of pose p (VertexSE3Expmap::oplusImpl, exp(dx) * T) into q, t;
// dd = its dx (zero for a fixed pose), h = its free index or -1.
template <bool CR>
__device__ __forceinline__ void trial_pose(const DevProblem &d, int p, double q[4], double t[3], double dd[6], int &h) {
  const double *qt = d.pose_qt[0] + 8 * p;
  q[0] = qt[0]; q[1] = qt[1]; q[2] = qt[2]; q[3] = qt[3];
  t[0] = qt[4]; t[1] = qt[5]; t[2] = qt[6];
  h = d.pose_hidx[p];
#pragma unroll
  for (int k = 0; k < 6; ++k) dd[k] = 0.0;
  if (h < 0) return;
  if (CR) {
    const int pi = d.cam_pos ? d.cam_pos[h] : h;
    const double *x = pi >= 0 ? d.cr_x + (size_t)(pi / d.cr_B) * d.cr_n + 6 * (pi % d.cr_B) : d.bd_x + 6 * (-1 - pi);
    const bool ok = d.flags[0] != 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) dd[k] = ok ? x[k] : 0.0;
  } else {
    const double *dx = d.dx + 6 * h;
#pragma unroll
    for (int k = 0; k < 6; ++k) dd[k] = dx[k];
  }
  se3_oplus(q, t, dd);
}

// k_pose_update's work for pose p: the trial pose rows, dx (CR), and this
// pose's computeScale term dx^T (lambda dx + b) (sharded: b_p is summed over
// ranks and lambda counted once)
template <bool CR>
__device__ __forceinline__ double pose_update_item(const DevProblem &d, double lambda, int p) {
  double q[4], t[3], dd[6];
  int h;
  trial_pose<CR>(d, p, q, t, dd, h);
  double sc = 0.0;
  if (h >= 0) {
    if (CR) {
      double *dx = d.dx + 6 * h;
      store2(dx, dd[0], dd[1]); store2(dx + 2, dd[2], dd[3]); store2(dx + 4, dd[4], dd[5]);
    }
    const double lam = (!d.sharded || d.rank == 0) ? lambda : 0.0;
    for (int k = 0; k < 6; ++k) sc += dd[k] * (lam * dd[k] + d.bp[8 * h + k]);
  }
  double *o = d.pose_qt[1] + 8 * p;
  store2(o, q[0], q[1]); store2(o + 2, q[2], q[3]); store2(o + 4, t[0], t[1]); store2(o + 6, t[2], 0.0);
  double R[9];
  q_to_mat(q, R);
  double *rt = d.pose_rt[1] + 16 * p;
#pragma unroll
  for (int k = 0; k < 9; ++k) rt[k] = R[k];
  rt[9] = t[0]; rt[10] = t[1]; rt[11] = t[2];
  rt[12] = d.intr[4 * p]; rt[13] = d.intr[4 * p + 1]; rt[14] = d.intr[4 * p + 2]; rt[15] = d.intr[4 * p + 3];
  return sc;
}

template <bool CR>
__global__ __launch_bounds__(256) void k_pose_update(DevProblem d, double lambda) {
  __shared__ double red[4];
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  double sc = 0.0;
  if (p < d.n_pose) sc = pose_update_item<CR>(d, lambda, p);
  const double s = block_sum(sc, red);
  if (threadIdx.x == 0) d.partials[kPartScaleCam + blockIdx.x] = s;
}

void launch_pose_update(const DevProblem &d, double lambda, hipStream_t st, bool from_cr) {
  if (d.n_pose == 0) return;
  if (from_cr)
    hipLaunchKernelGGL(k_pose_update<true>, dim3((d.n_pose + 255) / 256), dim3(256), 0, st, d, lambda);
  else
    hipLaunchKernelGGL(k_pose_update<false>, dim3((d.n_pose + 255) / 256), dim3(256), 0, st, d, lambda);
}

// Back-substitution dl = M (b_l - sum_i H_lp,i dx_i), X' = X + dl, then the
// residuals of the landmark's edges at the trial state (computeActiveErrors).
// A block's landmarks are consecutive slots (trajectory order), so their
// observations see a short window of cameras (host-computed per tile, `rng`):
// the window's poses at both states and its dx are staged in LDS once per
// tile, and the per-observation gathers read LDS instead of L2. Tiles whose
// window is wider (loop-closure landmarks) read the global arrays.
#ifndef SQLM_UPD_OCC
#define SQLM_UPD_OCC 1
#endif
// fuse_pose (first bucket of a band solve, no window wider than kUpdWin): the
// blocks past nlm_blocks do k_pose_update<true>'s work, and every block tile
// forms its window's trial poses and dx itself (the same trial_pose code, so
// the same bits) instead of reading them -- one launch less per trial.
// waves per SIMD the mono variants are compiled for (A/B: -DSQLM_UPD_OCC_MONO=3)
#ifndef SQLM_UPD_OCC_MONO
#define SQLM_UPD_OCC_MONO 4
#endif
// The observations a lane streams after its kObsPreload preloaded ones are
// read twice, by the back substitution and then by the trial evaluation /
// speculative linearization; a tile's inputs do not stay in L2 in between
// (the re-reads were ~100 MB of the pass's 342 MB, profiles/r05/pmc_gba.json).
// The first pass parks the first kUpdCache of them in LDS (camera + the f32
// measurement, as loaded: the same doubles come back) for the second.
// Depth 3 measured best: 1 / 2 / 4 entries (6 / 5 / 3 workgroups per CU by
// LDS) gave 0.155 / 0.153 / 0.156 ms against 0.150 (profiles/r06/ab_upd_cache_depth.log).
#ifndef SQLM_UPD_NCACHE
#define SQLM_UPD_NCACHE 3
#endif
constexpr int kUpdCache = SQLM_UPD_NCACHE;
#ifndef SQLM_UPD_CACHE  // A/B: -DSQLM_UPD_CACHE=0 reads them twice
#define SQLM_UPD_CACHE 1
#endif
struct UpdCache {
  int cam[kUpdCache][kBlock];
  float4 q[kUpdCache][kBlock];
};
template <int W, bool ST, bool SPEC, bool FUSE>
__device__ __forceinline__ void landmark_update_body(const DevProblem &d, int slot_begin, int slot_end, double lambda,
                                                    int part_off, const int2 *rng, int nlm_blocks, int bid,
                                                    double *red, double *Wp0, double *Wp1, double *Wdx,
                                                    UpdCache *oc) {
  constexpr bool fuse_pose = FUSE;
  if (fuse_pose && bid >= nlm_blocks) {  // k_pose_update<true>
    const int pb = bid - nlm_blocks;
    const int p = pb * blockDim.x + threadIdx.x;
    double sc = 0.0;
    if (p < d.n_pose) sc = pose_update_item<true>(d, lambda, p);
    const double s = block_sum(sc, red);
    if (threadIdx.x == 0) d.partials[kPartScaleCam + pb] = s;
    return;
  }
  constexpr int SPB = kBlock / W;
  const int lane = threadIdx.x & (W - 1);
  const int nseg = slot_end - slot_begin;
  const int ntiles = (nseg + SPB - 1) / SPB;
  double chi_acc = 0.0, sc_acc = 0.0;
  // one tile: P0 / P1 = pose rows (R t fx fy cx cy) at the linearization / trial
  // state indexed by pose id, DX = dx rows (by pose id in the window, by free
  // camera otherwise)
  // The tile's own first inputs (track bounds, the landmark's position) are
  // requested before the window is staged, so their latency overlaps the
  // window's instead of following it; the observations follow the window.
  struct TileIn {
    int slot, beg, end;
    bool valid;
    double L0, L1, L2;
  };
  auto tile_load = [&](int tile) {
    TileIn t;
    const int seg = tile * SPB + threadIdx.x / W;
    t.slot = slot_begin + seg;
    t.valid = seg < nseg;
    t.beg = t.end = 0;
    t.L0 = t.L1 = t.L2 = 0.0;
    if (t.valid) {
      t.beg = d.lm_begin[t.slot];
      t.end = d.lm_begin[t.slot + 1];
      const double *Xl = d.X[0] + 4 * t.slot;
      t.L0 = Xl[0]; t.L1 = Xl[1]; t.L2 = Xl[2];
    }
    return t;
  };
  auto tile_body = [&](const TileIn &tin, const double *P0, const double *P1, const double *DX, auto in_win) {
    constexpr bool WIN = decltype(in_win)::value;
    const int slot = tin.slot, beg = tin.beg, end = tin.end;
    const bool valid = tin.valid;
    ObsIn o[kObsPreload];
#pragma unroll
    for (int i = 0; i < kObsPreload; ++i) o[i] = load_obs<ST, true>(d, beg + lane + i * W, beg + lane + i * W < end);
    double a0 = 0, a1 = 0, a2 = 0;
    const double L0 = tin.L0, L1 = tin.L1, L2 = tin.L2;
    // H_lp dx_cam = jl^T (jp dx_cam), Jacobians recomputed at the linearization point
    auto hlp_dx = [&](const ObsIn &o) {
      if (o.camh < 0) return;
      const double *prt = P0 + 16 * o.cam, *dx = WIN ? DX + 8 * o.cam : DX + 6 * o.camh;
      double x[6];
#pragma unroll
      for (int k = 0; k < 6; ++k) x[k] = dx[k];
      MonoEval m;
      m.x = prt[0] * L0 + prt[1] * L1 + prt[2] * L2 + prt[9];
      m.y = prt[3] * L0 + prt[4] * L1 + prt[5] * L2 + prt[10];
      m.z = prt[6] * L0 + prt[7] * L1 + prt[8] * L2 + prt[11];
      m.s = o.s;
      double jl[6], jp[12];
      mono_jac(prt, m, jl, jp);
      const double t0 = jp[0] * x[0] + jp[1] * x[1] + jp[2] * x[2] + jp[3] * x[3] + jp[5] * x[5];
      const double t1 = jp[6] * x[0] + jp[7] * x[1] + jp[8] * x[2] + jp[10] * x[4] + jp[11] * x[5];
      a0 += jl[0] * t0 + jl[3] * t1;
      a1 += jl[1] * t0 + jl[4] * t1;
      a2 += jl[2] * t0 + jl[5] * t1;
      if (ST && o.ur >= 0.0) {
        double jl3[3], jp3[6];
        stereo_row(prt, m, d.pose_bf[o.cam], jl, jp, jl3, jp3);
        const double t2 = jp3[0] * x[0] + jp3[1] * x[1] + jp3[2] * x[2] + jp3[3] * x[3] + jp3[5] * x[5];
        a0 += jl3[0] * t2;
        a1 += jl3[1] * t2;
        a2 += jl3[2] * t2;
      }
    };
#pragma unroll
    for (int i = 0; i < kObsPreload; ++i) hlp_dx(o[i]);  // camh = -1 for lanes past the track
    // (mono, f32 measurements: the streamed ones are parked for the second pass)
    const bool park = SQLM_UPD_CACHE && !ST && oc != nullptr && d.obs_f32;
    {
      int j = 0;
      for (int e = beg + lane + kObsPreload * W; e < end; e += W, ++j) {
        if (park && j < kUpdCache) {  // the raw inputs straight into the cache, then only what hlp_dx reads
          const int cam = d.obs_cam[e];
          oc->cam[j][threadIdx.x] = cam;
          oc->q[j][threadIdx.x] = *reinterpret_cast<const float4 *>(d.obs_q + 4 * (int64_t)e);
          ObsIn oi{cam, d.obs_camh[e], 0.0, 0.0, 0.0, 0.0, -1.0, d.obs_s[e]};
          hlp_dx(oi);
        } else {
          hlp_dx(load_obs<ST, true>(d, e, true));
        }
      }
    }
    // a parked observation for the second pass (j < kUpdCache)
    auto parked = [&](int j) {
      ObsIn oi{0, -1, 0.0, 0.0, 0.0, 0.0, -1.0, 0.0};
      oi.cam = oc->cam[j][threadIdx.x];
      const float4 q = oc->q[j][threadIdx.x];
      oi.u = q.x;
      oi.v = q.y;
      oi.info = q.z;
      oi.delta = q.w;
      return oi;
    };
    // the second pass over the streamed observations: the parked ones from LDS
    // (a loop of their own: one loop choosing per observation spilled), then
    // any further ones loaded again
    auto stream2 = [&](auto &&use) {
      int e = beg + lane + kObsPreload * W;
      if (park) {
#pragma unroll 1
        for (int j = 0; j < kUpdCache && e < end; ++j, e += W) use(parked(j), e);
      }
      for (; e < end; e += W) use(load_obs<ST, true>(d, e, true), e);
    };
    a0 = seg_sum<W>(a0); a1 = seg_sum<W>(a1); a2 = seg_sum<W>(a2);
    double chi = 0.0;
    double R[6] = {0, 0, 0, 0, 0, 0};  // SPEC: QR of the landmark's rows at the trial state
    double b0 = 0, b1 = 0, b2 = 0, g0 = 0, g1 = 0, g2 = 0;
    if (valid) {
      // dl = (H_ll + lambda I)^-1 c = R'^-1 (R'^-T c), R'^-1 upper (i00 i01 i02 i11 i12 i22)
      const double *bl = d.lm_b + 4 * slot;
      double Ri[6], wl[3];
      damp_factor(d.lm_R + 8 * slot, bl, lambda, Ri, wl);
      const double c0 = bl[0] - a0, c1 = bl[1] - a1, c2 = bl[2] - a2;
      const double y0 = Ri[0] * c0, y1 = Ri[1] * c0 + Ri[3] * c1, y2 = Ri[2] * c0 + Ri[4] * c1 + Ri[5] * c2;
      const double dl0 = Ri[0] * y0 + Ri[1] * y1 + Ri[2] * y2;
      const double dl1 = Ri[3] * y1 + Ri[4] * y2;
      const double dl2 = Ri[5] * y2;
      const double X0 = L0 + dl0, X1 = L1 + dl1, X2 = L2 + dl2;
      if (lane == 0) {
        double *Xo = d.X[1] + 4 * slot;
        store2(Xo, X0, X1); store2(Xo + 2, X2, 0.0);
        sc_acc += dl0 * (lambda * dl0 + bl[0]) + dl1 * (lambda * dl1 + bl[1]) + dl2 * (lambda * dl2 + bl[2]);
      }
      if (SPEC) {  // the next linearization at the trial state (used if the trial is accepted)
#pragma unroll
        for (int i = 0; i < kObsPreload; ++i) {
          const int e = beg + lane + i * W;
          if (e < end) lin_edge<ST>(d, o[i], e, P1, X0, X1, X2, d.obs_s_nx, false, R, b0, b1, b2, g0, g1, g2, chi);
        }
        stream2([&](const ObsIn &oi, int e) {
          lin_edge<ST>(d, oi, e, P1, X0, X1, X2, d.obs_s_nx, false, R, b0, b1, b2, g0, g1, g2, chi);
        });
      } else {
        auto trial_err = [&](const ObsIn &o, int e) {
          MonoEval m;
          const double *prt = P1 + 16 * o.cam;
          if (ST && o.ur >= 0.0) stereo_error(prt, X0, X1, X2, o.u, o.v, o.ur, d.pose_bf[o.cam], o.info, o.delta, m);
          else mono_error(prt, X0, X1, X2, o.u, o.v, o.info, o.delta, m);
          store2(d.obs_err + 2 * e, m.e0, m.e1);
          if (ST) d.obs_err3[e] = o.ur >= 0.0 ? m.e2 : 0.0;
          chi += m.chi_rob;
        };
#pragma unroll
        for (int i = 0; i < kObsPreload; ++i)
          if (beg + lane + i * W < end) trial_err(o[i], beg + lane + i * W);
        stream2([&](const ObsIn &oi, int e) { trial_err(oi, e); });
      }
    }
    if (SPEC) {
      lin_butterfly<W>(lane, R, b0, b1, b2, g0, g1, g2, chi);
      if (valid && lane == 0) {
        double *Ro = d.lm_R_nx + 8 * slot;
        store2(Ro, R[0], R[1]); store2(Ro + 2, R[2], R[3]); store2(Ro + 4, R[4], R[5]);
        double *bo = d.lm_b_nx + 4 * slot;
        store2(bo, b0, b1); store2(bo + 2, b2, 0.0);
      }
    } else {
      chi = seg_sum<W>(chi);
    }
    if (valid && lane == 0) chi_acc += chi;
  };
  for (int tile = bid; tile < ntiles; tile += nlm_blocks) {
    const int2 rg = rng[tile];  // pose id range of the tile's observations (x > y: none)
    // (the fused variant, which forms the window's trial poses itself, keeps
    // them after the window: hoisted there they spill)
    TileIn tin;
    if constexpr (!FUSE) tin = tile_load(tile);
    const int nw = rg.y - rg.x + 1;
    if (nw <= kUpdWin) {
      lds_barrier();  // the previous tile's readers are done with the window (the loads above stay in flight)
      if constexpr (FUSE) {
        for (int k = threadIdx.x; k < 16 * nw; k += blockDim.x) Wp0[k] = d.pose_rt[0][16 * rg.x + k];
        for (int c = threadIdx.x; c < nw; c += blockDim.x) {
          const int p = rg.x + c;
          double q[4], t3[3], dd[6], R[9];
          int h;
          trial_pose<true>(d, p, q, t3, dd, h);
          q_to_mat(q, R);
          double *w1 = Wp1 + 16 * c, *wd = Wdx + 8 * c;
#pragma unroll
          for (int k = 0; k < 9; ++k) w1[k] = R[k];
          w1[9] = t3[0]; w1[10] = t3[1]; w1[11] = t3[2];
          w1[12] = d.intr[4 * p]; w1[13] = d.intr[4 * p + 1]; w1[14] = d.intr[4 * p + 2]; w1[15] = d.intr[4 * p + 3];
#pragma unroll
          for (int k = 0; k < 6; ++k) wd[k] = dd[k];
          wd[6] = wd[7] = 0.0;
        }
      } else {
        for (int k = threadIdx.x; k < 16 * nw; k += blockDim.x) {
          Wp0[k] = d.pose_rt[0][16 * rg.x + k];
          Wp1[k] = d.pose_rt[1][16 * rg.x + k];
        }
        for (int k = threadIdx.x; k < 8 * nw; k += blockDim.x) {
          const int c = k >> 3, r = k & 7, h = d.pose_hidx[rg.x + c];
          Wdx[k] = (h >= 0 && r < 6) ? d.dx[6 * h + r] : 0.0;
        }
      }
      lds_barrier();
      if constexpr (FUSE) tin = tile_load(tile);
      tile_body(tin, Wp0 - 16 * rg.x, Wp1 - 16 * rg.x, Wdx - 8 * rg.x, std::true_type{});
    } else {
      if constexpr (FUSE) tin = tile_load(tile);
      tile_body(tin, d.pose_rt[0], d.pose_rt[1], d.dx, std::false_type{});
    }
  }
  const double s1 = block_sum(chi_acc, red);
  const double s2 = block_sum(sc_acc, red);
  if (threadIdx.x == 0) {
    d.partials[kPartChiNewLm + part_off + bid] = s1;
    d.partials[kPartScaleLm + part_off + bid] = s2;
    if (SPEC) d.partials[d.px_lm + part_off + bid] = s1;  // chi2 of the next linearization
  }
}

template <int W, bool ST, bool SPEC, bool FUSE = false>
__global__ __launch_bounds__(256, ST ? SQLM_UPD_OCC : SQLM_UPD_OCC_MONO) void k_landmark_update(DevProblem d, int slot_begin, int slot_end,
                                                         double lambda, int part_off, const int2 *rng, int nlm_blocks) {
  __shared__ double red[4];
  __shared__ double Wp0[kUpdWin * 16], Wp1[kUpdWin * 16], Wdx[kUpdWin * 8];
  // (no observation cache here: the per-bucket launches serve small problems,
  // where it measured slower -- local BA 0.0143 -> 0.0152 ms, profiles/r06/)
  landmark_update_body<W, ST, SPEC, FUSE>(d, slot_begin, slot_end, lambda, part_off, rng, nlm_blocks, blockIdx.x, red,
                                          Wp0, Wp1, Wdx, nullptr);
}

// Every bucket of a trial in one launch: the block range [blk0[b], blk0[b] +
// nblk[b]) runs bucket b exactly as its own launch would (same tiles, same
// partial slots), so the results are the same bits; one launch instead of
// one per bucket, the heaviest bucket's blocks dispatched first, and no
// bucket's tail idles the chip before the next starts (config 4: 0.205 ->
// 0.178 ms, profiles/r05/ab_upd_merged_r5o.log). The fused-pose form (every
// bucket forming its trial poses, small problems) measured slower than the
// fused single bucket (local BA 7.33k -> 7.21k it/s, ab_upd_merged_fused_rejected.log).
template <bool ST, bool SPEC>
__global__ __launch_bounds__(256, ST ? SQLM_UPD_OCC : SQLM_UPD_OCC_MONO) void k_landmark_update_all(DevProblem d,
                                                                                                 double lambda,
                                                                                                 UpdLaunch u) {
  __shared__ double red[4];
  __shared__ double Wp0[kUpdWin * 16], Wp1[kUpdWin * 16], Wdx[kUpdWin * 8];
  __shared__ UpdCache oc;
  const int bx = blockIdx.x;
  int b = 0;
#pragma unroll
  for (int k = 1; k < kMaxUpdBuckets; ++k)
    if (k < u.nb && bx >= u.blk0[k]) b = k;
  const int bid = bx - u.blk0[b];
  const int2 *rng = d.upd_rng + u.rng_off[b];
#define SQLM_UCASE(WW)                                                                                       \
  case WW:                                                                                                   \
    landmark_update_body<WW, ST, SPEC, false>(d, u.slot_begin[b], u.slot_end[b], lambda, u.part_off[b], rng, \
                                              u.nblk[b], bid, red, Wp0, Wp1, Wdx, ST ? nullptr : &oc);       \
    break;
  switch (u.W[b]) {
    SQLM_UCASE(2) SQLM_UCASE(4) SQLM_UCASE(8) SQLM_UCASE(16) SQLM_UCASE(32) SQLM_UCASE(64)
    default: break;
  }
#undef SQLM_UCASE
}

int upd_launch_plan(const std::vector<Bucket> &bk, const std::vector<int> &part_off, UpdLaunch &u) {
  u = UpdLaunch{};
  if (bk.size() > (size_t)kMaxUpdBuckets) return -1;
  std::vector<int> ord(bk.size());
  for (size_t b = 0; b < ord.size(); ++b) ord[b] = (int)b;
  std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return bk[x].W > bk[y].W; });
  for (int b : ord) {
    const int nb = linearize_blocks(bk[b]);
    if (nb <= 0) continue;
    const int k = u.nb++;
    u.W[k] = bk[b].W;
    u.slot_begin[k] = bk[b].slot_begin;
    u.slot_end[k] = bk[b].slot_end;
    u.part_off[k] = part_off[b];
    u.rng_off[k] = bk[b].rng_off;
    u.nblk[k] = nb;
    u.blk0[k] = u.grid;
    u.grid += nb;
  }
  return 0;
}

void launch_landmark_update_all(const DevProblem &d, const UpdLaunch &u, double lambda, hipStream_t st, bool spec) {
  if (u.nb <= 0 || u.grid <= 0) return;
  if (d.has_stereo) {
    if (spec) hipLaunchKernelGGL((k_landmark_update_all<true, true>), dim3(u.grid), dim3(kBlock), 0, st, d, lambda, u);
    else hipLaunchKernelGGL((k_landmark_update_all<true, false>), dim3(u.grid), dim3(kBlock), 0, st, d, lambda, u);
  } else {
    if (spec) hipLaunchKernelGGL((k_landmark_update_all<false, true>), dim3(u.grid), dim3(kBlock), 0, st, d, lambda, u);
    else hipLaunchKernelGGL((k_landmark_update_all<false, false>), dim3(u.grid), dim3(kBlock), 0, st, d, lambda, u);
  }
}

void launch_landmark_update(const DevProblem &d, const Bucket &b, double lambda, int part_off, hipStream_t st,
                            bool spec, bool fuse_pose) {
  const int nb = linearize_blocks(b);
  if (nb <= 0) return;
  if (fuse_pose && !spec) return;  // instantiated for the speculative schedule only: the caller must not ask
  const int grid = nb + (fuse_pose ? (d.n_pose + kBlock - 1) / kBlock : 0);
#define SQLM_LAUNCH(WW, STT, SP, FU) \
  hipLaunchKernelGGL((k_landmark_update<WW, STT, SP, FU>), dim3(grid), dim3(kBlock), 0, st, d, b.slot_begin, \
                     b.slot_end, lambda, part_off, d.upd_rng + b.rng_off, nb)
#define SQLM_CASE(WW)                                            \
  case WW:                                                       \
    if (d.has_stereo) {                                          \
      if (fuse_pose) SQLM_LAUNCH(WW, true, true, true);          \
      else if (spec) SQLM_LAUNCH(WW, true, true, false);         \
      else SQLM_LAUNCH(WW, true, false, false);                  \
    } else {                                                     \
      if (fuse_pose) SQLM_LAUNCH(WW, false, true, true);         \
      else if (spec) SQLM_LAUNCH(WW, false, true, false);        \
      else SQLM_LAUNCH(WW, false, false, false);                 \
    }                                                            \
    break;
  switch (b.W) {
    SQLM_CASE(2) SQLM_CASE(4) SQLM_CASE(8) SQLM_CASE(16) SQLM_CASE(32) SQLM_CASE(64)
    default: break;
  }
#undef SQLM_CASE
#undef SQLM_LAUNCH
}

__global__ __launch_bounds__(256) void k_lidar_chi2(DevProblem d) {
  __shared__ double red[4];
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  double chi = 0.0;
  if (t < d.nLid) {
    const double *qt = d.pose_qt[1] + 8 * d.lid_pose[t];
    const double q[4] = {qt[0], qt[1], qt[2], qt[3]}, t3[3] = {qt[4], qt[5], qt[6]};
    const double *L = d.lid_data + 12 * t;
    const double e = lidar_error(q, t3, L, L + 3, L + 6);
    d.lid_err[t] = e;
    chi = e * (L[9] * e);
  }
  const double s = block_sum(chi, red);
  if (threadIdx.x == 0) d.partials[kPartChiNewLid + blockIdx.x] = s;
}

void launch_lidar_chi2(const DevProblem &d, hipStream_t st) {
  if (d.nLid == 0) return;
  hipLaunchKernelGGL(k_lidar_chi2, dim3((d.nLid + 255) / 256), dim3(256), 0, st, d);
}

// ---------------------------------------------------------------- reductions

// The six partial regions, one wavefront each (fixed order: bitwise deterministic).
// The six partial regions folded into the trial scalars by one 1024-thread
// block: every thread loads its strided share of all regions with the loads
// of four strides in flight together (one memory latency per 4096 partials,
// not one per 64), then fixed-order wave and block sums (deterministic).
constexpr int kReduceThreads = 1024;
// mbox (optional): the host's mailbox in page-locked host memory; the scalars
// are written there too, then seq (a fence apart), so the host can poll it
// instead of copying and synchronizing the stream.
__global__ __launch_bounds__(kReduceThreads) void k_reduce(DevProblem d, int n_lm_cur, int n_lm_new, int n_cam,
                                                          int n_lid, double *mbox, unsigned long long seq) {
  __shared__ double red[6][kReduceThreads / 64];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const double *p = d.partials;
  const double *base[6] = {p + d.pc_lm, p + d.pc_lid, p + kPartChiNewLm, p + kPartChiNewLid, p + kPartScaleCam,
                           p + kPartScaleLm};
  const int n[6] = {n_lm_cur, d.nP, n_lm_new, n_lid, n_cam, n_lm_new};
  int nmax = 0;
#pragma unroll
  for (int r = 0; r < 6; ++r) nmax = max(nmax, n[r]);
  // the words thread 0 publishes, requested with the partials (not after the barrier)
  unsigned long long md = 0ull;
  int f0 = 0, f1 = 0;
  if (tid == 0) {
    md = *d.maxdiag;
    f0 = d.flags[0];
    f1 = d.flags[1];
  }
  double acc[6] = {0, 0, 0, 0, 0, 0};
  // groups of four strides, two groups' loads in flight together (8192
  // partials per memory round trip); each group summed as its own step, in order
  for (int k0 = tid; k0 < nmax; k0 += 8 * kReduceThreads) {
    double v[8][6];
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        const int k = k0 + u * kReduceThreads;
        v[u][r] = k < n[r] ? base[r][k] : 0.0;
      }
#pragma unroll
    for (int r = 0; r < 6; ++r) acc[r] += (v[0][r] + v[1][r]) + (v[2][r] + v[3][r]);
    if (k0 + 4 * kReduceThreads < nmax) {
#pragma unroll
      for (int r = 0; r < 6; ++r) acc[r] += (v[4][r] + v[5][r]) + (v[6][r] + v[7][r]);
    }
  }
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    const double w = wave_sum(acc[r]);
    if (lane == 0) red[r][wave] = w;
  }
  __syncthreads();
  if (tid == 0) {
    double part[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      double t = 0.0;
      for (int w = 0; w < kReduceThreads / 64; ++w) t += red[r][w];
      part[r] = t;
    }
    d.scalars[kChiCur] = part[0] + part[1];
    d.scalars[kChiNew] = part[2] + part[3];
    d.scalars[kScale] = part[4] + part[5];
    d.scalars[kMaxDiag] = __longlong_as_double((long long)md);
    *d.maxdiag = 0ull;  // ready for the next linearization's atomicMax
    d.scalars[kSolveOk] = (double)f0;
    d.scalars[kDevErr] = (double)f1;
    if (mbox) {
      mbox[kChiCur] = part[0] + part[1];
      mbox[kChiNew] = part[2] + part[3];
      mbox[kScale] = part[4] + part[5];
      mbox[kMaxDiag] = __longlong_as_double((long long)md);
      mbox[kSolveOk] = (double)f0;
      mbox[kDevErr] = (double)f1;
      __threadfence_system();
      __hip_atomic_store(reinterpret_cast<unsigned long long *>(mbox + kMboxSeq), seq, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

void launch_reduce(const DevProblem &d, int n_lm_parts_cur, int n_lm_parts_new, int n_cam_parts, int n_lid_parts,
                   hipStream_t st, double *mbox, unsigned long long seq) {
  hipLaunchKernelGGL(k_reduce, dim3(1), dim3(kReduceThreads), 0, st, d, n_lm_parts_cur, n_lm_parts_new, n_cam_parts,
                     n_lid_parts, mbox, seq);
}

}  // namespace sqlm
