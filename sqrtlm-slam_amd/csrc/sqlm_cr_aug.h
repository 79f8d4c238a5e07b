// sqlm_cr_aug.h — the cyclic-reduction block factorization as one augmented
// right-looking Cholesky on the FP64 matrix cores (included by
// sqlm_rcs_solve.hip; the factor of linear_solver_eigen.h:94-124's SimplicialLDLT
// restated for the block-tridiagonal reduced camera system).
//
// For odd superblock I at level h the cyclic reduction needs, with D_I = L L^T:
//   A_I = L^-1 E_{I-h}^T,  C_I = L^-1 E_I,  z_I = L^-1 g_I,
// and, for the back substitution, either Linv_I = L^-1 (LINV, the layouts
// that carry extra right-hand sides: band + border, essential graph) or the
// factor itself, U = L^T, with the inverses T_k = L_kk^-1 of its 16x16
// diagonal blocks (plain band). All of them are block rows of one forward
// substitution, so this kernel runs a blocked Cholesky of the augmented matrix
// [D | E^T | E | g (| I)] in upper form and reads the results off the columns.
//
// Layout: every 16x16 tile lives in registers in the f64 MFMA accumulator
// layout (lane l holds column l & 15, rows (l >> 4) + 4 j in element j). In
// that layout a tile is ALSO the A and B operand of an MFMA that sums over
// its row index, so the trailing update T_IJ -= U_kI^T U_kJ is four
// v_mfma_f64_16x16x4f64 on the tiles as they stand, with no data movement.
//
// Roles (16 waves; a workgroup's waves w, w+4, w+8, w+12 share one SIMD):
//   wave 0        the diagonal wave. Step k: diagonal tile k in four rank-4
//                 groups (a 4x4 Cholesky on uniform values from readlane,
//                 W = L44^-1 per lane, the finished rows X = W M4 by one MFMA,
//                 the rank-4 update by one MFMA). In the pipe beside that scalar
//                 chain the same groups turn an identity tile into T_k = L_kk^-1
//                 (published for the workers), finish P = (k, k+1) -> U_k,k+1 and
//                 apply its piece to the next diagonal Q = (k+1, k+1). At the end
//                 of the step it takes column k+2's tiles (k+1, k+2), (k+2, k+2)
//                 (handed over through step k-1) and U_k,k+2, and forms the next
//                 step's P and Q. Waves 4, 8, 12 stay idle: any MFMA-busy wave on
//                 this SIMD triples the chain, whatever the priorities
//                 (tools/group_probe).
//   workers       the other 12 waves own one column of tiles each: D column J
//                 (the U tiles above the diagonal; rows J-1 and J go to wave 0
//                 at step J-2; in LINV mode continued below the diagonal by
//                 identity column J+1), identity column 0 (LINV), g, and the
//                 E^T / E columns dealt over the `split` workgroups that share
//                 the superblock (each repeats the factorization: it is the
//                 latency, the E columns are the parallel work).
// Step k on a worker: row-k tile <- T_k tile (four MFMAs), D columns publish
// U_kJ; trailing tile(I, col) -= U_kI^T X_k,col for I > k, row k+1 at once, the
// rest deferred into the next step. Hand-offs are LDS flags (no barrier after
// the start).
#pragma once

namespace sqlm {
namespace aug {

// wave 0: the diagonal chain; waves 1 and 2 (other SIMDs) its off-chain MFMAs:
// the PQ wave (U_k,k+1 and the next diagonal) and the T wave (T_k); waves 4,
// 8, 12 (wave 0's SIMD) idle; the other 10 are column workers.
// SQLM_AUG_SOLO (A/B builds): wave 0 alone, 12 workers.
#ifdef SQLM_AUG_SOLO
constexpr bool kPipe = false;
#else
constexpr bool kPipe = true;
#endif

constexpr int kWaves = 16, kThreads = 64 * kWaves, kMaxNt = kCRMaxN / 16, kWorkers = kPipe ? 10 : 12;
constexpr int kPairs = kMaxNt * (kMaxNt - 1) / 2;
enum : int { kNone = 0, kColD = 1, kColI0 = 3, kColEt = 4, kColE = 5, kColG = 6 };

#ifndef SQLM_SPIN_LIMIT
#define SQLM_SPIN_LIMIT (1 << 20)
#endif
constexpr int kSpinLimit = SQLM_SPIN_LIMIT;
constexpr int kTp = 17;  // padded row stride of the T_k images
struct Shared {
  double T[kMaxNt][16 * kTp];  // T_k = L_kk^-1 of step k, row-major (the workers read it as an A operand)
  double U[kPairs][256];    // U_kJ (k < J), accumulator layout: element j of lane l at [64 j + l]
  double Hp[kMaxNt][256];   // column J's tiles (J-1, J) and (J, J): through step J-3 to wave 0 (solo), through step J-2 to the PQ wave
  double Hq[kMaxNt][256];
  int fT[kMaxNt], fU[kPairs], fH[kMaxNt];
  // diagonal wave -> pipe wave: group a's A operand (W) and rank-4 rows (op),
  // one slot per group reused every step (flag value = step + 1); pipe wave ->
  // diagonal wave: the next diagonal tile (flag value = its step)
  double Ga[2][4][64], Go[2][4][64], Dn[256];  // slots by step parity (two consumer waves)
  int fA[2][4], fO[2][4], fD;
  double by[kCRMaxN], bx[kCRMaxN], br[16];  // BACK: y, x and one block row's right-hand side
};

// (k, J), k < J < kMaxNt -> 0 .. kPairs-1
__device__ __forceinline__ constexpr int pair_id(int k, int J) { return k * (2 * kMaxNt - k - 1) / 2 + (J - k - 1); }

__device__ __forceinline__ double rl(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// 1/sqrt(x) by v_rsq_f64 and one Newton step; a non-positive pivot is flagged
// (off the chain: the value is not guarded -- a flagged factor is discarded
// whole, and a NaN or inf in it changes no control flow)
__device__ __forceinline__ double rsqn(double x, bool &bad) {
  bad |= !(x > 0.0);
  double y = __builtin_amdgcn_rsq(x);
  const double hh = 0.5 * x * y;
  return fma(y, fma(-hh, y, 0.5), y);
}

// per-lane select of two values (a v_cndmask pair: the operands are plain
// values, so the front end emits a select, never a branch on the lane)
__device__ __forceinline__ double sel(bool c, double x, double y) { return c ? x : y; }

__device__ __forceinline__ d4 mfma(double a, double b, const d4 &c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ d4 identity_tile(int lane) {
  const int k4 = lane >> 4, c = lane & 15;
  d4 t;
#pragma unroll
  for (int j = 0; j < 4; ++j) t[j] = (k4 + 4 * j == c) ? 1.0 : 0.0;
  return t;
}

// phase stamps for tools/cr_bench (-DSQLM_CR_PROF): slot i of this workgroup
#ifdef SQLM_CR_PROF
#define AUG_PROF(i)                                                                               \
  do {                                                                                            \
    if ((threadIdx.x & 63) == 0 && g_cr_prof) g_cr_prof[blockIdx.x * 1024 + (i)] = clock64(); \
  } while (0)
// per wave / step / event stamps and the wave's hardware id (SIMD placement)
#define AUG_STAMP(w, k, e) AUG_PROF(64 + 32 * (w) + 4 * (k) + (e))
#define AUG_HWID(w)                                                                                       \
  do {                                                                                                    \
    if ((threadIdx.x & 63) == 0 && g_cr_prof)                                                             \
      g_cr_prof[blockIdx.x * 1024 + 900 + (w)] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)); \
  } while (0)
#else
#define AUG_PROF(i) \
  do {              \
  } while (0)
#define AUG_STAMP(w, k, e) AUG_PROF(0)
#define AUG_HWID(w) AUG_PROF(0)
#endif

// LDS flags between the waves of the workgroup, accessed through address-space
// 3 pointers so they compile to ds_read / ds_write (a generic volatile pointer
// becomes a flat access with system scope and a vmcnt wait).
typedef __attribute__((address_space(3))) int lds_int;

// Wait for a flag raised by another wave of the workgroup. Bounded (tens of
// ms): a wave can never hang the device, whatever the schedule does. Returns
// false when the wait gave up: the caller then fails the solve (cr_fail) --
// the data it goes on with is not the factor, and the trial must not use it.
// -DSQLM_SPIN_FORCE_TIMEOUT (tests only): every wait reports a timeout after
// it has completed, so the failure path runs on a correct factor.
// SQLM_SPIN_SLEEP (build, A/B): s_sleep units between polls (0: poll back to back)
#ifndef SQLM_SPIN_SLEEP
#define SQLM_SPIN_SLEEP 1
#endif
__device__ __forceinline__ bool spin(int *f) {
  lds_int *p = (lds_int *)f;
  int it = 0;
  for (; __atomic_load_n(p, __ATOMIC_RELAXED) == 0 && it < kSpinLimit; ++it)
    if (SQLM_SPIN_SLEEP > 0) __builtin_amdgcn_s_sleep(SQLM_SPIN_SLEEP);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#ifdef SQLM_SPIN_DEBUG
  if (it >= kSpinLimit && (threadIdx.x & 63) == 0)
    printf("spin timeout: block %d wave %d lds offset %u\n", (int)blockIdx.x, (int)(threadIdx.x >> 6),
           (unsigned)(uintptr_t)p);
#endif
#ifdef SQLM_SPIN_FORCE_TIMEOUT
  return false;
#else
  return it < kSpinLimit;
#endif
}
// Producer side: the DS instructions of one wave execute in order, so the flag
// store lands after the data stores issued before it; only the compiler must
// not move them (no s_waitcnt: the wave goes on while the stores drain).
__device__ __forceinline__ void raise_flag(int *f, int lane, int val = 1) {
  __asm__ volatile("" ::: "memory");
  if (lane == 0) __atomic_store_n((lds_int *)f, val, __ATOMIC_RELAXED);
}
// Wait until a step-numbered flag reaches val; no sleep between polls (the
// hand-offs between the diagonal wave and its pipe wave are the chain itself).
// Bounded and fail-loud like spin().
__device__ __forceinline__ bool spin_to(int *f, int val) {
  lds_int *p = (lds_int *)f;
  int it = 0;
  for (; __atomic_load_n(p, __ATOMIC_RELAXED) < val && it < 16 * kSpinLimit; ++it) {
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#ifdef SQLM_SPIN_FORCE_TIMEOUT
  return false;
#else
  return it < 16 * kSpinLimit;
#endif
}

__device__ __forceinline__ void put_tile(double *dst, const d4 &t, int lane) {
#pragma unroll
  for (int j = 0; j < 4; ++j) dst[64 * j + lane] = t[j];
}
__device__ __forceinline__ d4 get_tile(const double *src, int lane) {
  d4 t;
#pragma unroll
  for (int j = 0; j < 4; ++j) t[j] = src[64 * j + lane];
  return t;
}

// The 4x4 pivot block of group a of a diagonal tile Dg (rows / columns
// 4a .. 4a+3, element a of lanes 16 r + 4a + c) as uniform values from
// readlane: m00 m01 m02 m03 m11 m12 m13 m22 m23 m33.
__device__ __forceinline__ void pivot_block(const d4 &Dg, int a, double (&m)[10]) {
  m[0] = rl(Dg[a], 4 * a), m[1] = rl(Dg[a], 4 * a + 1), m[2] = rl(Dg[a], 4 * a + 2), m[3] = rl(Dg[a], 4 * a + 3);
  m[4] = rl(Dg[a], 16 + 4 * a + 1), m[5] = rl(Dg[a], 16 + 4 * a + 2), m[6] = rl(Dg[a], 16 + 4 * a + 3);
  m[7] = rl(Dg[a], 32 + 4 * a + 2), m[8] = rl(Dg[a], 32 + 4 * a + 3);
  m[9] = rl(Dg[a], 48 + 4 * a + 3);
}

// The Cholesky of a group's 4x4 pivot block on uniform values, and W =
// (U44^T)^-1 as the A operand of the group's MFMAs: lane (b, i) holds W[i][b]
// (column b; zero for i >= 4).
__device__ __forceinline__ double group_pivot_m(const double (&m)[10], int lane, bool &bad) {
  const int b = lane >> 4, i = lane & 15;
  const bool b0 = b == 0, b1 = b == 1, b2 = b == 2, b3 = b == 3, i3 = i == 3;
  const double m00 = m[0], m01 = m[1], m02 = m[2], m03 = m[3], m11 = m[4], m12 = m[5], m13 = m[6], m22 = m[7],
               m23 = m[8], m33 = m[9];
  // U44 (upper, U44^T U44 = M44) with d_r = 1 / U44[r][r]
  const double d0 = rsqn(m00, bad);
  const double u01 = m01 * d0, u02 = m02 * d0, u03 = m03 * d0;
  const double d1 = rsqn(fma(-u01, u01, m11), bad);
  const double u12 = fma(-u01, u02, m12) * d1, u13 = fma(-u01, u03, m13) * d1;
  const double d2 = rsqn(fma(-u12, u12, fma(-u02, u02, m22)), bad);
  const double u23 = fma(-u12, u13, fma(-u02, u03, m23)) * d2;
  const double d3 = rsqn(fma(-u23, u23, fma(-u13, u13, fma(-u03, u03, m33))), bad);
  // Every entry of W is a uniform value (column cb below, cb a constant); the
  // lane picks its own by selects, so the wave never branches on its lane.
  double W[4][4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const double w0 = cb == 0 ? d0 : 0.0;
    const double w1 = cb == 1 ? d1 : (cb < 1 ? -d1 * (u01 * w0) : 0.0);
    const double w2 = cb == 2 ? d2 : (cb < 2 ? -d2 * fma(u12, w1, u02 * w0) : 0.0);
    W[0][cb] = w0;
    W[1][cb] = w1;
    W[2][cb] = w2;
    W[3][cb] = cb == 3 ? d3 : -d3 * fma(u23, w2, fma(u13, w1, u03 * w0));
  }
  // rows 0..2 first (ready before d3), row 3 -- the chain's last -- selected last
  double r012 = 0.0;
#pragma unroll
  for (int r = 2; r >= 0; --r) {
    const double wr = sel(b0, W[r][0], sel(b1, W[r][1], sel(b2, W[r][2], W[r][3])));
    r012 = sel(i == r, wr, r012);
  }
  const double w3b = sel(b3, W[3][3], sel(b2, W[3][2], sel(b1, W[3][1], W[3][0])));
  return sel(i3, w3b, r012);
}

// Group a of a diagonal step: pivot block from Dg, then group_pivot_m.
__device__ __forceinline__ double group_pivot(const d4 &Dg, int a, int lane, bool &bad) {
  double m[10];
  pivot_block(Dg, a, m);
  return group_pivot_m(m, lane, bad);
}

// Step k on the diagonal tile Dg, in four rank-4 groups, all on one wave
// (SQLM_AUG_SOLO builds, A/B only); T_k = L_kk^-1 in Tt. With PQ the same
// groups also finish P = tile (k, k+1) -> U_k,k+1 and take the step-k piece of
// the next diagonal tile Q = (k+1, k+1) -= U_k,k+1^T U_k,k+1.
template <bool PQ>
__device__ __forceinline__ void diag_groups(d4 Dg, d4 &P, d4 &Q, d4 &Tt, int lane, bool &bad) {
  const int c = lane & 15;
  const d4 zero = {0.0, 0.0, 0.0, 0.0};
  Tt = identity_tile(lane);
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const double aop = group_pivot(Dg, a, lane, bad);
    // finished rows 4a .. 4a+3 = W M4 (rows 0..3 of the product, element 0);
    // the rank-4 update of the rows and columns past the group
    const d4 Xd = mfma(aop, Dg[a], zero);
    const double op = c >= 4 * a + 4 ? Xd[0] : 0.0;
    Dg = mfma(-op, op, Dg);
    __builtin_amdgcn_sched_barrier(0);  // the chain's update is issued first
    // off the chain: T_k = the same groups on the identity; with PQ, P = (k, k+1)
    // -> U_k,k+1 and the step-k piece of the next diagonal Q = (k+1, k+1) -= U^T U
    const d4 Xt = mfma(aop, Tt[a], zero);
    Tt[a] = Xt[0];
    Tt = mfma(-op, Xt[0], Tt);
    if (PQ) {
      const d4 Xp = mfma(aop, P[a], zero);
      P[a] = Xp[0];
      P = mfma(-op, Xp[0], P);
      Q = mfma(-Xp[0], Xp[0], Q);
    }
  }
}

// Row-k tile t <- T_k t (T_k = L_kk^-1 from wave 0, read from LDS as the A
// operand: lane 16 b + i holds T_k[i][4 s + b] for K-step s).
__device__ __forceinline__ void tile_trsm(Shared &sh, int k, d4 &t, int lane, bool &tmo) {
  const int b = lane >> 4, i = lane & 15;
  tmo |= !spin(&sh.fT[k]);
  double ta[4];
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4) ta[s4] = sh.T[k][i * kTp + 4 * s4 + b];
  d4 x = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4) x = mfma(ta[s4], t[s4], x);
  t = x;
}

// tile loads in the accumulator layout: (r0, c0) = first row / column in P
__device__ __forceinline__ d4 load_tile(const double *P, int n, int r0, int c0, int lane) {
  const int k4 = lane >> 4, c = lane & 15;
  d4 t;
#pragma unroll
  for (int j = 0; j < 4; ++j) t[j] = P[(size_t)(r0 + k4 + 4 * j) * n + c0 + c];
  return t;
}
// tile (r0, c0) of P^T
__device__ __forceinline__ d4 load_tile_t(const double *P, int n, int r0, int c0, int lane) {
  const int k4 = lane >> 4, c = lane & 15;
  d4 t;
#pragma unroll
  for (int j = 0; j < 4; ++j) t[j] = P[(size_t)(c0 + c) * n + r0 + k4 + 4 * j];
  return t;
}
// diagonal tile (r0, r0) from its lower triangle (the dense solvers keep only
// that one; a symmetric block gives the same bits as load_tile)
__device__ __forceinline__ d4 load_tile_sym(const double *P, int n, int r0, int lane) {
  const int k4 = lane >> 4, c = lane & 15;
  const d4 lo = load_tile(P, n, r0, r0, lane), up = load_tile_t(P, n, r0, r0, lane);
  d4 t;
#pragma unroll
  for (int j = 0; j < 4; ++j) t[j] = k4 + 4 * j >= c ? lo[j] : up[j];
  return t;
}
__device__ __forceinline__ void store_tile(double *P, int n, int r0, int c0, const d4 &t, int lane) {
  const int k4 = lane >> 4, c = lane & 15;
#pragma unroll
  for (int j = 0; j < 4; ++j) st_d(P + (size_t)(r0 + k4 + 4 * j) * n + c0 + c, t[j]);
}

// D columns carried by workers: J = 1 .. nt-1 (LINV: 0 .. nt-1, column 0 then
// carries identity column 1)
__host__ __device__ __forceinline__ int d_columns(int nt, bool linv) { return linv ? nt : nt - 1; }
// E / g columns of a superblock: E_{I-h}^T (left, a level step), E_I (right)
// and g
__host__ __device__ __forceinline__ int extra_columns(int nt, bool left, bool right) {
  return (left ? nt : 0) + (right ? nt : 0) + 1;
}
// workers left for the E / g columns (LINV also carries identity column 0)
__host__ __device__ __forceinline__ int fixed_columns(int nt, bool linv) { return d_columns(nt, linv) + (linv ? 1 : 0); }
inline int min_split(int nt, bool linv, int ne) {
  const int cap = kWorkers - fixed_columns(nt, linv);
  return (ne + cap - 1) / cap;
}

// role of a worker (q = 0 .. kWorkers-1) of a workgroup serving one superblock
__device__ __forceinline__ void column_of(int q, int nt, bool linv, bool left, bool right, int split, int sidx,
                                          int &type, int &J) {
  J = 0;
  const int nd = d_columns(nt, linv);
  if (q < nd) {
    type = kColD;
    J = linv ? q : q + 1;
    return;
  }
  if (linv && q == nd) {
    type = kColI0;
    return;
  }
  const int e = (q - fixed_columns(nt, linv)) * split + sidx;
  const int net = left ? nt : 0, nee = right ? nt : 0;
  if (e < net) {
    type = kColEt;
    J = e;
  } else if (e < net + nee) {
    type = kColE;
    J = e - net;
  } else {
    type = e == net + nee ? kColG : kNone;
  }
}

// Does column (type, J) take the trailing update of row I from step k (k < I)?
// D column J keeps its rows J-1 and J only through step J-3: at step J-2 it
// hands them to wave 0, which applies the rest.
template <bool LINV>
__device__ __forceinline__ bool takes_update(int type, int J, int k, int I) {
  if (type == kColD) return (I <= J && (I <= J - 2 || k <= J - 3)) || (LINV && I > J && k >= J + 1);
  return type == kColI0 || type == kColEt || type == kColE || type == kColG;
}

}  // namespace aug

// BACK (MODE 1, U layout, one superblock: the top of the cyclic reduction):
// the g worker goes on to x = U^-1 y with U's tiles and the T_k still in LDS --
// the arithmetic of k_cr_back_u<true> in the same order (bitwise equal), one
// launch less per solve. Wave (block row) k's step in k_cr_back_u becomes
// step k of a loop from the bottom: lane (q, r) sums U_kj[r][4q..4q+3] x_j over
// j > k (j descending), the quarter sums are added by two xor shuffles, and
// x_k = T_k^T (y_k - that).
__device__ __forceinline__ void top_back(aug::Shared &sh, const CRView &v, int I, int nt, const d4 *t, int lane) {
  using namespace aug;
  const int n = v.n, q = lane >> 4, r = lane & 15, k4 = lane >> 4;
#pragma unroll
  for (int rr = 0; rr < kMaxNt; ++rr)
    if (rr < nt && r == 0)
#pragma unroll
      for (int j = 0; j < 4; ++j) sh.by[16 * rr + k4 + 4 * j] = t[rr][j];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  for (int i = nt - 1; i >= 0; --i) {
    double acc = 0.0;
    for (int j = nt - 1; j > i; --j) {
      const double *U = sh.U[pair_id(i, j)];  // U_ij[row][col] at [64 (row >> 2) + 16 (row & 3) + col]
#pragma unroll
      for (int m = 0; m < 4; ++m) acc = fma(U[64 * (r >> 2) + 16 * (r & 3) + 4 * q + m], sh.bx[16 * j + 4 * q + m], acc);
    }
    acc += __shfl_xor(acc, 16, 64);
    acc += __shfl_xor(acc, 32, 64);
    if (q == 0) sh.br[r] = sh.by[16 * i + r] - acc;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double x = 0.0;
#pragma unroll
    for (int m = 0; m < 4; ++m) x = fma(sh.T[i][(4 * q + m) * kTp + r], sh.br[4 * q + m], x);  // T_i[4q+m][r]
    x += __shfl_xor(x, 16, 64);
    x += __shfl_xor(x, 32, 64);
    if (q == 0) {
      sh.bx[16 * i + r] = x;
      st_d(v.x + (size_t)I * n + 16 * i + r, x);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// A wait gave up (aug::spin / spin_to): the solve is marked failed (flags[0]
// = 0: the trial is rejected, as for a non-positive pivot) and flags[1] keeps
// the error for the host, which returns SQLM_ERR_HIP (never a silently wrong
// factor).
constexpr int kCrErrTimeout = 1;
__device__ __forceinline__ void cr_fail(const CRView &v, int lane) {
  if (lane == 0) {
    __hip_atomic_store(v.flags, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(v.flags + 1, kCrErrTimeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// MODE 0: level step (A_I, C_I, z_I and the back-substitution factor).
// MODE 1: factor only (z_I and the factor). LINV: the factor is Linv_I
// (lower, dense tiles); otherwise the upper U tiles with T_k on the diagonal.
// Superblock I, workgroup sidx of the split that serve it. Every thread of the
// workgroup enters; waves return as their role ends (no barrier after the
// first).
template <int MODE, bool LINV, bool BACK>
__device__ __forceinline__ void aug_body(aug::Shared &sh, const CRView &v, int h, int I, int split, int sidx) {
  using namespace aug;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = v.n, nt = n >> 4;
  const bool left = MODE == 0, right = MODE != 1 && I + h < v.p, first = sidx == 0;
  bool tmo = false;
  for (int t = threadIdx.x; t < 2 * kMaxNt + kPairs + 17; t += blockDim.x) {
    if (t < kMaxNt) sh.fT[t] = 0;
    else if (t < kMaxNt + kPairs) sh.fU[t - kMaxNt] = 0;
    else if (t < 2 * kMaxNt + kPairs) sh.fH[t - kMaxNt - kPairs] = 0;
    else if (t < 2 * kMaxNt + kPairs + 8) (&sh.fA[0][0])[t - 2 * kMaxNt - kPairs] = 0;
    else if (t < 2 * kMaxNt + kPairs + 16) (&sh.fO[0][0])[t - 2 * kMaxNt - kPairs - 8] = 0;
    else sh.fD = 0;
  }
  __syncthreads();
#ifdef SQLM_SPIN_DEBUG
  if (lane == 0 && (wave == 0 || wave == 9))
    printf("aug blk %d wave %d I %d mode %d past zeroing, fT0 %d\n", (int)blockIdx.x, wave, I, MODE, sh.fT[0]);
#endif
  if (threadIdx.x == 0) AUG_PROF(0);
  AUG_HWID(wave);
  // MODE 1 with v.ld: one diagonal block of a larger dense matrix (row stride ld)
  // (its diagonal tiles are read from their lower triangles: the dense solver
  // keeps only that one; the CR superblocks are stored whole)
  const bool dense = MODE == 1 && v.ld;
  const int ldd = dense ? v.ld : n;
  const double *Dblk = dense ? v.D : blk(v.D, I, n);
  bool bad = false;
  if (kPipe && wave == 0) {  // ---- the diagonal wave: the chain only
    __builtin_amdgcn_s_setprio(3);
    AUG_PROF(1);
    const int c = lane & 15;
    const d4 zero = {0.0, 0.0, 0.0, 0.0};
    d4 Dg = dense ? load_tile_sym(Dblk, ldd, 0, lane) : load_tile(Dblk, n, 0, 0, lane);
    for (int k = 0; k < nt; ++k) {
      AUG_STAMP(0, k, 0);
      const int pk = k & 1;
      if (k > 0) {  // diagonal tile k, updated through step k-1 by the PQ wave
        tmo |= !spin_to(&sh.fD, k);
        Dg = get_tile(sh.Dn, lane);
      }
      // this step's slots held step k-2's groups: the T wave must be past that step
      if (k >= 2) tmo |= !spin(&sh.fT[k - 2]);
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        AUG_PROF(600 + 16 * k + 4 * a);  // (cr_bench stamps: group start, pivot done, X ready)
        const double aop = group_pivot(Dg, a, lane, bad);
        AUG_PROF(601 + 16 * k + 4 * a);
        sh.Ga[pk][a][lane] = aop;
        raise_flag(&sh.fA[pk][a], lane, k + 1);
        if (a == 3) {  // the last group updates nothing past the tile
          AUG_STAMP(0, k, 1);
          break;
        }
        // finished rows 4a .. 4a+3 = W M4 (element 0); the rank-4 update of the
        // rows and columns past the group
        const d4 Xd = mfma(aop, Dg[a], zero);
        const double op = c >= 4 * a + 4 ? Xd[0] : 0.0;
        AUG_PROF(602 + 16 * k + 4 * a);
        Dg = mfma(-op, op, Dg);
        sh.Go[pk][a][lane] = op;
        raise_flag(&sh.fO[pk][a], lane, k + 1);
      }
    }
    if (bad && lane == 0) v.flags[0] = 0;
    if (tmo) cr_fail(v, lane);
    return;
  }
  if (kPipe && wave == 1) {  // ---- the PQ wave: U_k,k+1 and the next diagonal
    __builtin_amdgcn_s_setprio(3);
    double *Lb = blk(v.L, I, n);
    const d4 zero = {0.0, 0.0, 0.0, 0.0};
    d4 P = zero, Q = zero;
    if (nt > 1) {
      P = load_tile_t(Dblk, ldd, 0, 16, lane);  // U tile (0, 1) from the lower block (1, 0)
      Q = dense ? load_tile_sym(Dblk, ldd, 16, lane) : load_tile(Dblk, n, 16, 16, lane);
    }
    for (int k = 0; k + 1 < nt; ++k) {
      const int pk = k & 1;
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        tmo |= !spin_to(&sh.fA[pk][a], k + 1);
        const double aop = sh.Ga[pk][a][lane];
        const d4 Xp = mfma(aop, P[a], zero);
        Q = mfma(-Xp[0], Xp[0], Q);
        double op = 0.0;  // the last group's rows update nothing (the diagonal wave's op is 0 there)
        if (a < 3) {
          tmo |= !spin_to(&sh.fO[pk][a], k + 1);
          op = sh.Go[pk][a][lane];
        }
        P[a] = Xp[0];
        P = mfma(-op, Xp[0], P);
      }
      AUG_STAMP(1, k, 0);
      put_tile(sh.Dn, Q, lane);  // the next diagonal first: it is the chain
      raise_flag(&sh.fD, lane, k + 1);
      // U_k,k+1 feeds the trailing updates of row k+1
      put_tile(sh.U[pair_id(k, k + 1)], P, lane);
      raise_flag(&sh.fU[pair_id(k, k + 1)], lane);
      if (!LINV && first) store_tile(Lb, n, 16 * k, 16 * (k + 1), P, lane);
      if (k + 2 < nt) {  // the next step's P = (k+1, k+2) and Q = (k+2, k+2) through step k
        tmo |= !spin(&sh.fU[pair_id(k, k + 2)]);  // U_k,k+2 from column k+2's worker
        const d4 X = get_tile(sh.U[pair_id(k, k + 2)], lane);
        tmo |= !spin(&sh.fH[k + 2]);  // its Q, and its P through step k-1
        d4 P2 = get_tile(sh.Hp[k + 2], lane);
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) P2 = mfma(-P[s4], X[s4], P2);
        P = P2;
        Q = get_tile(sh.Hq[k + 2], lane);
      }
      AUG_STAMP(1, k, 1);
    }
    if (tmo) cr_fail(v, lane);
    return;
  }
  if (kPipe && wave == 2) {  // ---- the T wave: T_k = L_kk^-1 (the same groups on the identity)
    __builtin_amdgcn_s_setprio(3);
    double *Lb = blk(v.L, I, n);
    const d4 zero = {0.0, 0.0, 0.0, 0.0};
    for (int k = 0; k < nt; ++k) {
      const int pk = k & 1;
      d4 Tt = identity_tile(lane);
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        tmo |= !spin_to(&sh.fA[pk][a], k + 1);
        const double aop = sh.Ga[pk][a][lane];
        const d4 Xt = mfma(aop, Tt[a], zero);
        double op = 0.0;
        if (a < 3) {
          tmo |= !spin_to(&sh.fO[pk][a], k + 1);
          op = sh.Go[pk][a][lane];
        }
        Tt[a] = Xt[0];
        Tt = mfma(-op, Xt[0], Tt);
      }
      AUG_STAMP(2, k, 0);
      {  // T_k for the workers (row-major) and, U/T layout, for the back substitution
        const int k4 = lane >> 4, c = lane & 15;
#pragma unroll
        for (int j = 0; j < 4; ++j) sh.T[k][(k4 + 4 * j) * kTp + c] = Tt[j];
        raise_flag(&sh.fT[k], lane);
        if (!LINV && first) store_tile(Lb, n, 16 * k, 16 * k, Tt, lane);
      }
      AUG_PROF(2 + k);
    }
    if (tmo) cr_fail(v, lane);
    return;
  }
  if (!kPipe && wave == 0) {  // ---- the diagonal wave alone (SQLM_AUG_SOLO)
    __builtin_amdgcn_s_setprio(3);
    AUG_PROF(1);
    double *Lb = blk(v.L, I, n);
    d4 Dg = dense ? load_tile_sym(Dblk, ldd, 0, lane) : load_tile(Dblk, n, 0, 0, lane), P = {0.0, 0.0, 0.0, 0.0}, Q = P;
    if (nt > 1) {
      P = load_tile_t(Dblk, ldd, 0, 16, lane);  // U tile (0, 1) from the lower block (1, 0)
      Q = dense ? load_tile_sym(Dblk, ldd, 16, lane) : load_tile(Dblk, n, 16, 16, lane);
    }
    for (int k = 0; k < nt; ++k) {
      AUG_STAMP(0, k, 0);
#ifdef SQLM_SPIN_DEBUG
      if (lane == 0) printf("w0 blk %d I %d step %d t %lld\n", (int)blockIdx.x, I, k, (long long)clock64());
#endif
      d4 Tt;
      if (k + 1 < nt) diag_groups<true>(Dg, P, Q, Tt, lane, bad);
      else diag_groups<false>(Dg, P, Q, Tt, lane, bad);
      {  // T_k for the workers (row-major) and, U/T layout, for the back substitution
        const int k4 = lane >> 4, c = lane & 15;
#pragma unroll
        for (int j = 0; j < 4; ++j) sh.T[k][(k4 + 4 * j) * kTp + c] = Tt[j];
        raise_flag(&sh.fT[k], lane);
        if (!LINV && first) store_tile(Lb, n, 16 * k, 16 * k, Tt, lane);
      }
      AUG_PROF(2 + k);
      if (k + 1 < nt) {  // U_k,k+1 feeds the trailing updates of row k+1
        put_tile(sh.U[pair_id(k, k + 1)], P, lane);
        raise_flag(&sh.fU[pair_id(k, k + 1)], lane);
        if (!LINV && first) store_tile(Lb, n, 16 * k, 16 * (k + 1), P, lane);
      }
      if (k + 2 < nt) {  // the next step's P = (k+1, k+2) and Q = (k+2, k+2) through step k
        tmo |= !spin(&sh.fH[k + 2]);
        d4 P2 = get_tile(sh.Hp[k + 2], lane), Q2 = get_tile(sh.Hq[k + 2], lane);
        tmo |= !spin(&sh.fU[pair_id(k, k + 2)]);
        const d4 X = get_tile(sh.U[pair_id(k, k + 2)], lane);
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) Q2 = mfma(-X[s4], X[s4], Q2);
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) P2 = mfma(-P[s4], X[s4], P2);
        Dg = Q;
        P = P2;
        Q = Q2;
      } else {
        Dg = Q;
      }
    }
    if (bad && lane == 0) v.flags[0] = 0;
    if (tmo) cr_fail(v, lane);
#ifdef SQLM_SPIN_DEBUG
    if (lane == 0) printf("w0 blk %d I %d done t %lld\n", (int)blockIdx.x, I, (long long)clock64());
#endif
    return;
  }
  if ((wave & 3) == 0) return;  // the diagonal wave's SIMD partners stay idle
  const int q = wave - (wave >> 2) - (kPipe ? 3 : 1);
  int type, J;
  column_of(q, nt, LINV, left, right, split, sidx, type, J);
  if (type == kNone) return;
  // ---- load this wave's column
  d4 t[kMaxNt];
#pragma unroll
  for (int r = 0; r < kMaxNt; ++r) {
    t[r] = d4{0.0, 0.0, 0.0, 0.0};
    if (r >= nt) continue;
    if (type == kColD) {
      if (r < J) t[r] = load_tile_t(Dblk, ldd, 16 * r, 16 * J, lane);  // U tile (r, J) from the lower block (J, r)
      else if (r == J) t[r] = dense ? load_tile_sym(Dblk, ldd, 16 * r, lane) : load_tile(Dblk, n, 16 * r, 16 * J, lane);
      else if (LINV && r == J + 1) t[r] = identity_tile(lane);
    } else if (type == kColI0) {
      if (r == 0) t[r] = identity_tile(lane);
    } else if (type == kColEt) {
      t[r] = load_tile_t(blk(v.E, I - h, n), n, 16 * r, 16 * J, lane);
    } else if (type == kColE) {
      t[r] = load_tile(blk(v.E, I, n), n, 16 * r, 16 * J, lane);
    } else if (type == kColG) {
      const int k4 = lane >> 4, c = lane & 15;
#pragma unroll
      for (int j = 0; j < 4; ++j) t[r][j] = c == 0 ? v.g[(size_t)I * n + 16 * r + k4 + 4 * j] : 0.0;
    }
  }
  // ---- steps
#pragma unroll
  for (int k = 0; k < kMaxNt; ++k) {
    if (k >= nt) break;
    // deferred trailing of step k-1: rows k+1 .. (rows handed to wave 0 excluded)
    if (k >= 1) {
#pragma unroll
      for (int r = k + 1; r < kMaxNt; ++r) {
        if (r >= nt || !takes_update<LINV>(type, J, k - 1, r)) continue;
        const int pid = pair_id(k - 1, r);
        tmo |= !spin(&sh.fU[pid]);
        const double *U = sh.U[pid];
#pragma unroll
        for (int s = 0; s < 4; ++s) t[r] = mfma(-U[64 * s + lane], t[k - 1][s], t[r]);
      }
    }
    if (!kPipe && type == kColD && k == J - 2 && k + 2 < kMaxNt) {  // rows J-1, J through step J-3: to wave 0
      put_tile(sh.Hp[k + 2], t[k + 1], lane);
      put_tile(sh.Hq[k + 2], t[k + 2], lane);
      raise_flag(&sh.fH[k + 2], lane);
    }
    // the column that hands the next P / Q over is the chain: its MFMAs go first
    // on the SIMD it shares with other workers
    if (kPipe && type == kColD && k == J - 2) __builtin_amdgcn_s_setprio(2);
    AUG_STAMP(wave, k, 0);
    // row k: U_kJ (D column, k <= J-2), identity column J+1 (LINV, k > J), T, I0, E, g
    const bool dtile = type == kColD && k <= J - 2;
    const bool rowk = type == kColD ? (dtile || (LINV && k > J)) : type != kNone;
    if (rowk) {
      tile_trsm(sh, k, t[k], lane, tmo);
      if (dtile) {  // U_kJ feeds the trailing updates of row J
        put_tile(sh.U[pair_id(k, J)], t[k], lane);
        raise_flag(&sh.fU[pair_id(k, J)], lane);
      }
    }
    if (kPipe && type == kColD && k == J - 2 && k + 2 < kMaxNt) {
      // the PQ wave's next Q = tile (J, J) with step J-2's piece (the MFMAs
      // wave 0 applied in the one-wave layout, same operands and order), and
      // tile (J-1, J) through step J-3 (the PQ wave applies its step J-2 piece
      // with U_J-2,J-1, which it holds)
      d4 Q2 = t[k + 2];
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) Q2 = mfma(-t[k][s4], t[k][s4], Q2);
      put_tile(sh.Hp[k + 2], t[k + 1], lane);
      put_tile(sh.Hq[k + 2], Q2, lane);
      raise_flag(&sh.fH[k + 2], lane);
      __builtin_amdgcn_s_setprio(0);
    }
    AUG_STAMP(wave, k, 1);
    // trailing of step k, row k+1 (the next step's row)
    if (k + 1 < nt && rowk && takes_update<LINV>(type, J, k, k + 1)) {
      const int pid = pair_id(k, k + 1);
      tmo |= !spin(&sh.fU[pid]);
      const double *U = sh.U[pid];
#pragma unroll
      for (int s = 0; s < 4; ++s) t[k + 1] = mfma(-U[64 * s + lane], t[k][s], t[k + 1]);
    }
  }
  // ---- results
  double *Lb = blk(v.L, I, n);
#pragma unroll
  for (int r = 0; r < kMaxNt; ++r) {
    if (r >= nt) continue;
    if (type == kColD) {
      if (LINV) {
        if (first && r > J) store_tile(Lb, n, 16 * r, 16 * (J + 1), t[r], lane);  // Linv block column J+1
      } else {
        if (first && r <= J - 2) store_tile(Lb, n, 16 * r, 16 * J, t[r], lane);  // U tile (r, J); (J-1, J): wave 0
      }
    } else if (type == kColI0) {
      if (first) store_tile(Lb, n, 16 * r, 0, t[r], lane);
    } else if (type == kColEt) {
      store_tile(blk(v.A, I, n), n, 16 * r, 16 * J, t[r], lane);
    } else if (type == kColE) {
      store_tile(blk(v.C, I, n), n, 16 * r, 16 * J, t[r], lane);
    } else if (type == kColG) {
      const int k4 = lane >> 4, c = lane & 15;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (c == 0) st_d(v.g + (size_t)I * n + 16 * r + k4 + 4 * j, t[r][j]);
    }
  }
  if (BACK && type == kColG) top_back(sh, v, I, nt, t, lane);
  if (tmo) cr_fail(v, lane);
  AUG_PROF(16 + wave);
}

// Superblock I = I0 + stride * (blockIdx.x / split); workgroup sidx = blockIdx.x % split.
template <int MODE, bool LINV, bool BACK = false>
__global__ __launch_bounds__(aug::kThreads) void k_cr_aug(CRView v, int h, int I0, int stride, int split) {
  extern __shared__ __attribute__((aligned(16))) unsigned char aug_lds[];
  const int ob = blockIdx.x / split, sidx = blockIdx.x - ob * split;
  aug_body<MODE, LINV, BACK>(*reinterpret_cast<aug::Shared *>(aug_lds), v, h, I0 + stride * ob, split, sidx);
}

// Workgroups per odd superblock for the augmented factor: enough to hold the
// superblock's E / g columns in the spare workers, then as many as spread the
// level over the chip (the E columns are the parallel part; every workgroup
// repeats the factorization, which is the latency).
// SQLM_CR_SPLIT=s: exactly max(s, the minimum) workgroups per superblock (tests:
// the split must not change a bit).
inline int aug_split(int n_odd, int nt, bool linv, int ne) {
  static const int forced = std::getenv("SQLM_CR_SPLIT") ? std::atoi(std::getenv("SQLM_CR_SPLIT")) : 0;
  const int s = aug::min_split(nt, linv, ne);
  if (forced > 0) return std::max(s, std::min(ne, forced));
  return std::max(s, std::min(ne, 256 / std::max(1, n_odd)));
}

}  // namespace sqlm
