// sqlm_rcs_solve.hip — reduced-camera-system solve S dx = g on gfx950.
//
// Replaces LinearSolverEigen (SimplicialLDLT + AMD, Thirdparty/g2o/g2o/solvers/
// linear_solver_eigen.h:94-124). The camera ordering of g2o (pose id) makes S
// block-banded for sequential trajectories: with block bandwidth bw (cameras),
// grouping B = bw+1 consecutive cameras into one "superblock" makes S block
// TRIDIAGONAL with p superblocks of n = 6B (padded to a multiple of 16) rows.
// That system is solved by block cyclic reduction (an odd-even nested
// dissection): log2(p) levels, each eliminating every other superblock in
// parallel, so the critical path is O(log p) dense block operations instead of
// the O(p) of a banded Cholesky.
//
// The solve is latency-bound (≈3.4 GFLOP at config 4, spread over 9 levels),
// so every kernel is shaped for a short critical path:
//   * k_cr_factor: Cholesky + triangular inverse of one n x n block in LDS.
//     16x16 diagonal blocks are factored by one wavefront with readlane
//     broadcasts; the panel solve is row-parallel; the trailing update runs on
//     the FP64 matrix cores while wave 0 already factors the next diagonal
//     block (look-ahead); the diagonal inverses are formed in parallel.
//   * k_cr_factor_elim: every level runs the factor and the A_I / C_I tiles
//     in one launch with Linv_I still in LDS: one workgroup per odd
//     superblock on wide levels (>= 128), several on the deep ones, each
//     factoring redundantly and forming a share of the strips (the tiles
//     spread over the idle CUs without a second launch).
//   * k_cr_elim_gemm / k_cr_update_gemm: one wavefront per 16x16 output tile
//     (v_mfma_f64_16x16x4f64), workgroups remapped so that the tiles of one
//     superblock run on one XCD and share its L2; only the lower triangle of
//     the symmetric diagonal blocks is formed.
//   * matrix-vector steps (right-hand side, back substitution) are VALU dot
//     products with the 16x4 lane map of the MFMA tiles and a two-step
//     cross-lane reduction.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdlib>

#include "sqlm_internal.h"

namespace sqlm {

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st_d(double *p, double v) { *p = v; }

// Phase timestamps for tools/cr_bench (compiled with -DSQLM_CR_PROF only).
#ifdef SQLM_CR_PROF
__device__ long long *g_cr_prof;
#define CR_PROF(i)                                                                    \
  do {                                                                                \
    if (threadIdx.x == 0 && g_cr_prof) g_cr_prof[blockIdx.x * 64 + (i)] = clock64(); \
  } while (0)
#else
#define CR_PROF(i) \
  do {             \
  } while (0)
#endif

__device__ __forceinline__ double readlane_d(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// Dot-product helpers: k runs over 4u + k4 < kCRMaxN with the index clamped
// to n-1 and a zero weight past n, so every load is unconditional and the
// compiler issues them all before the first use.
__device__ __forceinline__ int kclamp(int k, int n) { return k < n ? k : n - 1; }

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

// sum over the four k4 groups of a wave (lanes r16, r16+16, r16+32, r16+48)
__device__ __forceinline__ double k4_sum(double s) {
  s += __shfl_xor(s, 16, 64);
  s += __shfl_xor(s, 32, 64);
  return s;
}

// Logical block id with the workgroups that the dispatcher sends to one XCD
// (hardware id mod 8) made contiguous, so a superblock's tiles share one L2.
__device__ __forceinline__ int xcd_block(int total) {
  const int b = blockIdx.x, chunk = (total + 7) >> 3;
  return (b & 7) * chunk + (b >> 3);
}
inline unsigned xcd_grid(int total) { return (unsigned)((total + 7) & ~7); }

// ---- dense block factorization in LDS --------------------------------------

constexpr int kT = 17;  // row stride of the 16x16 LDS scratch tiles (odd: conflict free)
constexpr int kTile = 16 * kT;

// Panel factorization of block column kb (columns c0 .. c0+15, rows c0 .. n-1):
// right-looking Cholesky of the 16x16 diagonal block fused with the solve of
// the rows below it. Wave w holds the 16 diagonal rows in lanes 0..15
// (redundantly in every participating wave, so no cross-wave traffic) and the
// rows c0+16+48w .. +48 in lanes 16..63. Column k is broadcast with readlane;
// 1/l_kk comes from v_rsq_f64 plus one Newton step (no divides).
__device__ __forceinline__ void panel_factor(double *L, int ld, int n, int c0, double *invd, int *fail, int wave) {
  const int lane = threadIdx.x & 63;
  const int i = lane < 16 ? lane : 16 + 48 * wave + (lane - 16);  // row within the panel
  const bool has = c0 + i < n;
  double *Lr = L + (c0 + i) * ld + c0;
  double row[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) row[j] = has ? Lr[j] : 0.0;
  bool bad = false;
  double myinv = 0.0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const double piv = readlane_d(row[k], k);
    double col[16];
#pragma unroll
    for (int j = k + 1; j < 16; ++j) col[j] = readlane_d(row[k], j);
    bad |= !(piv > 0.0);
    const double pv = piv > 0.0 ? piv : 1.0;
    double y = __builtin_amdgcn_rsq(pv);
    const double h = 0.5 * pv * y;
    y = fma(y, fma(-h, y, 0.5), y);  // one Newton step on 1/sqrt
    // row[j] -= l_ik l_jk = (a_ik y)(a_jk y); entries (i, j > i) of the diagonal rows
    // collect garbage here, they are never read
    const double t = row[k] * (y * y);
#pragma unroll
    for (int j = k + 1; j < 16; ++j) row[j] = fma(-t, col[j], row[j]);
    // selects, not branches: l_kk = piv y on the pivot row, l_ik = a_ik y below
    const double scaled = (i == k ? pv : row[k]) * y;
    row[k] = i >= k ? scaled : row[k];
    myinv = lane == k ? y : myinv;
  }
  if (lane < 16) {
    if (wave == 0) {
#pragma unroll
      for (int j = 0; j < 16; ++j) Lr[j] = j <= i ? row[j] : 0.0;
      invd[c0 + lane] = myinv;
      if (lane == 0 && bad) *fail = 1;
    }
  } else if (has) {
#pragma unroll
    for (int j = 0; j < 16; ++j) Lr[j] = row[j];
  }
}

__device__ __forceinline__ int panel_waves(int n, int c0) {
  const int below = n - c0 - 16;
  return below <= 48 ? 1 : (below + 47) / 48;
}

// Inverses of the lower-triangular 16x16 diagonal blocks of L into Dinv, four
// blocks per wave: lane quarter q takes block 4 wave + q and lane c of it owns
// column c of X (forward substitution, rows of L read from LDS). Quarters of
// one wave read different blocks, so no lane fetches a duplicate broadcast.
__device__ __forceinline__ void diag_trtri16x4(const double *L, int ld, int nt, const double *invd, double *Dinv,
                                               int wave) {
  const int lane = threadIdx.x & 63, c = lane & 15, kb = 4 * wave + (lane >> 4);
  if (kb >= nt) return;
  const int c0 = 16 * kb;
  double x[16];
#pragma unroll
  for (int rr = 0; rr < 16; ++rr) {
    const double *lr = L + (c0 + rr) * ld + c0;
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < rr; ++k) s += lr[k] * x[k];
    const double inv = invd[c0 + rr];
    x[rr] = rr == c ? inv : (rr > c ? -s * inv : 0.0);
  }
  double *X = Dinv + kb * kTile;
#pragma unroll
  for (int rr = 0; rr < 16; ++rr) X[rr * kT + c] = x[rr];
}

// One 16x16 trailing-update tile: L[I][J] -= L[I][kb] L[J][kb]^T (one wavefront).
__device__ __forceinline__ void syrk_tile(double *L, int ld, int c0, int I, int J) {
  const int lane = threadIdx.x & 63, r16 = lane & 15, k4 = lane >> 4;
  double a[4], b[4];
  d4 acc;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    a[s] = -L[(16 * I + r16) * ld + c0 + 4 * s + k4];
    b[s] = L[(16 * J + r16) * ld + c0 + 4 * s + k4];
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = L[(16 * I + k4 + 4 * j) * ld + 16 * J + r16];
#pragma unroll
  for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[s], acc, 0, 0, 0);
#pragma unroll
  for (int j = 0; j < 4; ++j) L[(16 * I + k4 + 4 * j) * ld + 16 * J + r16] = acc[j];
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// In-LDS Cholesky L L^T = A (lower block triangle of A read, n = 16 nt <=
// kCRMaxN, odd leading dim ld), then L <- L^-1 in place (blocked, LAPACK
// dtrtri lower order). The strict upper block triangle is left undefined.
// Needs 8 waves. Dinv, W: [nt][16][kT], invd: [n] LDS scratch.
// Returns false (for every thread) if a pivot is not positive.
__device__ __forceinline__ bool wg_potrf_trtri(double *L, int ld, int n, double *Dinv, double *W, double *invd,
                                               int *fail) {
  const int tid = threadIdx.x, nw = blockDim.x >> 6, wave = tid >> 6, lane = tid & 63;
  const int r16 = lane & 15, k4 = lane >> 4, nt = n >> 4;
  if (tid == 0) *fail = 0;
  __syncthreads();
  CR_PROF(1);
  if (wave < panel_waves(n, 0)) panel_factor(L, ld, n, 0, invd, fail, wave);
  __syncthreads();
  CR_PROF(2);
  for (int kb = 0; kb + 1 < nt; ++kb) {
    const int c0 = 16 * kb, m = nt - kb - 1;
    // (A) block column kb+1 absorbs column kb
    for (int t = wave; t < m; t += nw) syrk_tile(L, ld, c0, kb + 1 + t, kb + 1);
    __syncthreads();
    CR_PROF(3 + 2 * kb);
    // (B) panel kb+1, while the other waves apply column kb to the rest of the trailing matrix
    const int pw = panel_waves(n, c0 + 16);
    if (wave < pw) {
      panel_factor(L, ld, n, c0 + 16, invd, fail, wave);
    } else {
      const int mm = m - 1, ntile = mm * (mm + 1) / 2;
      for (int q = wave - pw; q < ntile; q += nw - pw) {
        int ib = 0, rem = q;
        while (rem > ib) { rem -= ib + 1; ++ib; }
        syrk_tile(L, ld, c0, kb + 2 + ib, kb + 2 + rem);
      }
    }
    __syncthreads();
    CR_PROF(4 + 2 * kb);
  }
  // diagonal inverses, one wave per block
  if (wave < (nt + 3) / 4) diag_trtri16x4(L, ld, nt, invd, Dinv, wave);
  __syncthreads();
  CR_PROF(31);
  // Linv by columns: L X = I gives X[ib][jb] = -Dinv_ib sum_{k=jb}^{ib-1} L[ib][k] X[k][jb]. Each
  // wave owns one block column (no barriers between columns; heavy columns on
  // distinct SIMDs) and parks X[ib][jb] in the unused upper block (jb, ib), since
  // the other waves keep reading the lower L.
  {
    const int jb = wave < 4 ? wave : wave == 4 ? 5 : wave == 5 ? 4 : wave;
    double *Wi = W + kTile * wave;
    for (int ib = jb + 1; ib < nt; ++ib) {
      double a[4 * (kCRMaxN / 16)], b[4 * (kCRMaxN / 16)];
#pragma unroll
      for (int t = 0; t < kCRMaxN / 16; ++t) {
        const int kb = jb + t;
        if (kb < ib) {
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            a[4 * t + s] = L[(16 * ib + r16) * ld + 16 * kb + 4 * s + k4];
            b[4 * t + s] = kb == jb ? Dinv[jb * kTile + (4 * s + k4) * kT + r16]
                                    : L[(16 * jb + 4 * s + k4) * ld + 16 * kb + r16];  // X[kb][jb] parked
          }
        }
      }
      d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int t = 0; t < kCRMaxN / 16; ++t)
        if (jb + t < ib) {
#pragma unroll
          for (int s = 0; s < 4; ++s)
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[4 * t + s], b[4 * t + s], acc, 0, 0, 0);
        }
#pragma unroll
      for (int j = 0; j < 4; ++j) Wi[(k4 + 4 * j) * kT + r16] = acc[j];
      wave_sync();
      double a2[4], b2[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        a2[s] = -Dinv[ib * kTile + r16 * kT + 4 * s + k4];
        b2[s] = Wi[(4 * s + k4) * kT + r16];
      }
      d4 acc2 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s = 0; s < 4; ++s) acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a2[s], b2[s], acc2, 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) L[(16 * jb + k4 + 4 * j) * ld + 16 * ib + r16] = acc2[j];
      wave_sync();
    }
  }
  __syncthreads();
  CR_PROF(32);
  return *fail == 0;
}

// Linv[r][c] of the factored LDS block: diagonal 16x16 blocks in Dinv, the
// block (ib, jb), ib > jb, parked untransposed at block position (jb, ib).
__device__ __forceinline__ double linv_at(const double *L, int ld, const double *Dinv, int r, int c) {
  const int ib = r >> 4, jb = c >> 4;
  if (ib > jb) return L[(16 * jb + (r & 15)) * ld + 16 * ib + (c & 15)];
  if (ib == jb) return Dinv[ib * kTile + (r & 15) * kT + (c & 15)];
  return 0.0;
}

// (Linv g) for the 16 rows of block ib (one wavefront; entry per lane r16 after
// the k-quarter sum). All loads are issued before the FMAs.
__device__ __forceinline__ double linv_gemv(const double *L, int ld, const double *Dinv, const double *g, int ib) {
  const int lane = threadIdx.x & 63, r16 = lane & 15, k4 = lane >> 4;
  double a[kCRMaxN / 4], b[kCRMaxN / 4];
#pragma unroll
  for (int t = 0; t < kCRMaxN / 16; ++t)
    if (t <= ib) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int k = 4 * s + k4;
        a[4 * t + s] = t < ib ? L[(16 * t + r16) * ld + 16 * ib + k] : Dinv[ib * kTile + r16 * kT + k];
        b[4 * t + s] = g[16 * t + k];
      }
    }
  double acc = 0.0;
#pragma unroll
  for (int t = 0; t < kCRMaxN / 16; ++t)
    if (t <= ib) {
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = fma(a[4 * t + s], b[4 * t + s], acc);
    }
  return k4_sum(acc);
}

// (Linv^T z) for the 16 rows of block jb.
__device__ __forceinline__ double linv_gemv_t(const double *L, int ld, const double *Dinv, const double *z, int jb,
                                              int nt) {
  const int lane = threadIdx.x & 63, r16 = lane & 15, k4 = lane >> 4;
  double a[kCRMaxN / 4], b[kCRMaxN / 4];
#pragma unroll
  for (int t = 0; t < kCRMaxN / 16; ++t)
    if (t >= jb && t < nt) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int k = 4 * s + k4;
        a[4 * t + s] = t > jb ? L[(16 * jb + k) * ld + 16 * t + r16] : Dinv[jb * kTile + k * kT + r16];
        b[4 * t + s] = z[16 * t + k];
      }
    }
  double acc = 0.0;
#pragma unroll
  for (int t = 0; t < kCRMaxN / 16; ++t)
    if (t >= jb && t < nt) {
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = fma(a[4 * t + s], b[4 * t + s], acc);
    }
  return k4_sum(acc);
}

struct CRView {
  int p, n, B, nP;
  double *D, *E, *A, *C, *g, *x;  // [p][n][n] x4, [p][n] x2
  int *flags;
  double *L;  // [p][n][n]: Linv_I of every factored superblock
  int ld;     // k_cr_aug<1, *> only: nonzero = D is one block with this row stride (dense solve)
  int *done = nullptr;  // k_cr_back_all: done[I] == epoch once x_I is published
  int epoch = 0;
};

__device__ __forceinline__ double *blk(double *base, int I, int n) { return base + (size_t)I * n * n; }

// LDS footprint of the factor kernels: L (n x (n+1)) + tmp (2n) + Dinv (17n) + W (17n) + invd (n)
inline size_t cr_factor_lds(int n) { return ((size_t)n * (n + 1) + 37 * (size_t)n) * sizeof(double); }

// BSR (upper, 6x6 blocks) -> superblock D_I (symmetric) and E_I = S(I, I+1); g -> g_I.
// With a border (d.cam_pos): band-border blocks -> F^T (arw_G), border-border
// blocks -> the border system bd_A (both triangles), border g -> bd_r.
__global__ __launch_bounds__(256) void k_cr_scatter(DevProblem d, CRView v) {
  const int i = blockIdx.x;  // free camera
  const int n = v.n, R = d.arw_R, Rp = d.arw_Rp;
  const int pi = d.cam_pos ? d.cam_pos[i] : i;
  const int I = pi >= 0 ? pi / v.B : 0, li = pi >= 0 ? pi - I * v.B : 0;
  for (int s = d.s_row_ptr[i]; s < d.s_row_ptr[i + 1]; ++s) {
    const int j = d.s_col[s];
    const int pj = d.cam_pos ? d.cam_pos[j] : j;
    const int J = pj >= 0 ? pj / v.B : 0, lj = pj >= 0 ? pj - J * v.B : 0;
    for (int e = threadIdx.x; e < 36; e += blockDim.x) {
      const int r = e / 6, c = e % 6;
      const double val = d.S[(size_t)s * 36 + e];
      if (pi >= 0 && pj >= 0) {
        if (J == I) {
          blk(v.D, I, n)[(6 * li + r) * n + 6 * lj + c] = val;
          if (j != i) blk(v.D, I, n)[(6 * lj + c) * n + 6 * li + r] = val;
        } else {  // J == I + 1 (block tridiagonal by construction)
          blk(v.E, I, n)[(6 * li + r) * n + 6 * lj + c] = val;
        }
      } else if (pi >= 0) {
        d.arw_G[((size_t)I * n + 6 * li + r) * R + 6 * (-1 - pj) + c] = val;
      } else if (pj >= 0) {
        d.arw_G[((size_t)J * n + 6 * lj + c) * R + 6 * (-1 - pi) + r] = val;
      } else {
        const int bi = -1 - pi, bj = -1 - pj;
        d.bd_A[(size_t)(6 * bi + r) * Rp + 6 * bj + c] = val;
        d.bd_A[(size_t)(6 * bj + c) * Rp + 6 * bi + r] = val;
      }
    }
  }
  if (threadIdx.x < 6) {
    if (pi >= 0) v.g[(size_t)I * n + 6 * li + threadIdx.x] = d.g[6 * i + threadIdx.x];
    else d.bd_r[6 * (-1 - pi) + threadIdx.x] = d.g[6 * i + threadIdx.x];
  }
  // identity on padded rows (cameras past the band in the last superblock, rows >= 6B)
  if (i < v.p && threadIdx.x < 64) {
    const int K = i, used = min(v.B, d.cr_nband - K * v.B);
    for (int r = 6 * used + threadIdx.x; r < n; r += 64) {
      blk(v.D, K, n)[r * n + r] = 1.0;
      v.g[(size_t)K * n + r] = 0.0;
    }
  }
  if (i == 0 && threadIdx.x == 0) v.flags[0] = 1;
}

// Factor superblock I into LDS: L <- chol(D_I)^-1; z = L g_I kept in LDS (tmp).
// Every wave returns; afterwards Linv is readable through linv_at() and tmp[0:n] = g_I.
__device__ __forceinline__ void cr_factor_block(const CRView &v, int I, double *lds, int *fail) {
  const int n = v.n, ld = n + 1, nw = blockDim.x >> 6, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double *L = lds, *tmp = lds + n * ld, *Dinv = tmp + 2 * n, *W = Dinv + 17 * n, *invd = W + 17 * n;
  const double *Dg = blk(v.D, I, n);
  CR_PROF(0);
  {  // lower block triangle only; all loads in flight before the LDS stores
    constexpr int kRows = (kCRMaxN + 7) / 8;
    double v0[kRows], v1[kRows];
#pragma unroll
    for (int t = 0; t < kRows; ++t) {
      const int r = wave + nw * t, cend = (r | 15) + 1;
      v0[t] = (r < n && lane < cend) ? Dg[r * n + lane] : 0.0;
      v1[t] = (r < n && lane + 64 < cend) ? Dg[r * n + lane + 64] : 0.0;
    }
#pragma unroll
    for (int t = 0; t < kRows; ++t) {
      const int r = wave + nw * t, cend = (r | 15) + 1;
      if (r < n && lane < cend) L[r * ld + lane] = v0[t];
      if (r < n && lane + 64 < cend) L[r * ld + lane + 64] = v1[t];
    }
  }
  for (int k = threadIdx.x; k < n; k += blockDim.x) tmp[k] = v.g[(size_t)I * n + k];
  if (!wg_potrf_trtri(L, ld, n, Dinv, W, invd, fail) && threadIdx.x == 0) v.flags[0] = 0;
}

}  // namespace sqlm
#include "sqlm_cr_aug.h"
namespace sqlm {

// Level h, step 1: every odd superblock I (I = h, 3h, 5h, ...) is factored:
// D_I <- Linv_I = chol(D_I)^-1 (lower block triangle, zero above), g_I <- z_I = Linv_I g_I.
__device__ __forceinline__ void cr_factor_store(const CRView &v, int I, double *lds, int *fail_p) {
  int &fail = *fail_p;
  const int n = v.n, ld = n + 1, nt = n >> 4;
  const int nw = blockDim.x >> 6, wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r16 = lane & 15, k4 = lane >> 4;
  cr_factor_block(v, I, lds, &fail);
  const double *L = lds, *tmp = lds + n * ld, *Dinv = tmp + 2 * n;
  double *Dg = blk(v.L, I, n);
  {  // dense Linv, one 16x16 tile per wave step; lane: row lane/4, 4 columns
    const int r = lane >> 2, c = 4 * (lane & 3);
    for (int q = wave; q < nt * nt; q += nw) {
      const int ib = q / nt, jb = q - ib * nt;
      double o[4];
      const double *src = ib > jb ? L + (16 * jb + r) * ld + 16 * ib + c : Dinv + ib * kTile + r * kT + c;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = ib >= jb ? src[e] : 0.0;
      double *dst = Dg + (16 * ib + r) * n + 16 * jb + c;
#pragma unroll
      for (int e = 0; e < 4; ++e) dst[e] = o[e];
    }
  }
  if (wave < nt) {  // z = Linv g, rows 16 wave .. +16
    const double s = linv_gemv(L, ld, Dinv, tmp, wave);
    if (k4 == 0) v.g[(size_t)I * n + 16 * wave + r16] = s;
  }
}

__global__ __launch_bounds__(512) void k_cr_factor(CRView v, int h) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ int fail;
  cr_factor_store(v, h + 2 * h * blockIdx.x, lds, &fail);
}

// One wavefront computes one 16x16 tile acc = op(A) op(B) over K = n,
// skipping K blocks that are zero because A is lower triangular (LA).
// CH: K pairs whose operands are loaded together (all of them by default; a
// smaller chunk changes the register budget only, not the MFMA order)
template <bool TA, bool TB, bool LA, int CH = kCRMaxN / 8>
__device__ __forceinline__ d4 tile_gemm(const double *A, const double *B, int n, int ti, int tj) {
  // K order within each pair of MFMA steps m: lane k4 feeds k = 8m + 2 k4 to the
  // first and k + 1 to the second, so row-contiguous operands (A untransposed,
  // B transposed) come in as one 16-byte load per lane and step pair.
  using d2 = HIP_vector_type<double, 2>;
  const int lane = threadIdx.x & 63, r16 = lane & 15, k4 = lane >> 4;
  const int ar = ti * 16 + r16, bc = tj * 16 + r16;
  const int kend = LA ? 16 * (ti + 1) : n;
  d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int m0 = 0; m0 < kCRMaxN / 8; m0 += CH) {
    d2 av[CH], bv[CH];
#pragma unroll
    for (int mm = 0; mm < CH; ++mm) {
      const int m = m0 + mm, k = 8 * m + 2 * k4;
      if (m < kCRMaxN / 8 && 8 * m < kend) {
        if (TA) {
          av[mm].x = A[k * n + ar];
          av[mm].y = A[(k + 1) * n + ar];
        } else {
          av[mm] = *reinterpret_cast<const d2 *>(A + ar * n + k);
        }
        if (TB) {
          bv[mm] = *reinterpret_cast<const d2 *>(B + bc * n + k);
        } else {
          bv[mm].x = B[k * n + bc];
          bv[mm].y = B[(k + 1) * n + bc];
        }
      }
    }
#pragma unroll
    for (int mm = 0; mm < CH; ++mm) {
      const int m = m0 + mm;
      if (m < kCRMaxN / 8 && 8 * m < kend) {
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[mm].x, bv[mm].x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[mm].y, bv[mm].y, acc, 0, 0, 0);
      }
    }
  }
  return acc;
}

__device__ __forceinline__ void tile_store(double *C, int n, int ti, int tj, const d4 &acc, double alpha,
                                           bool accumulate) {
  const int lane = threadIdx.x & 63, r16 = lane & 15, k4 = lane >> 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double *c = C + (ti * 16 + k4 + 4 * j) * n + tj * 16 + r16;
    st_d(c, accumulate ? *c + alpha * acc[j] : alpha * acc[j]);
  }
}

// Level h, step 2: A_I = Linv_I S(I, I-h) = Linv_I E_{I-h}^T and
// C_I = Linv_I S(I, I+h) = Linv_I E_I, one 16x16 tile per wavefront.
__device__ __forceinline__ void cr_elim_item(const CRView &v, int h, int lb) {
  const int n = v.n, nt = n >> 4, per = nt * nt;
  const int odd = lb / (2 * per), rem = lb - odd * 2 * per;
  const int which = rem / per, t = rem - which * per, ti = t / nt, tj = t - ti * nt;
  const int I = h + 2 * h * odd;
  if (which == 0) {
    const d4 acc = tile_gemm<false, true, true>(blk(v.L, I, n), blk(v.E, I - h, n), n, ti, tj);
    tile_store(blk(v.A, I, n), n, ti, tj, acc, 1.0, false);
  } else if (I + h < v.p) {
    const d4 acc = tile_gemm<false, false, true>(blk(v.L, I, n), blk(v.E, I, n), n, ti, tj);
    tile_store(blk(v.C, I, n), n, ti, tj, acc, 1.0, false);
  }
}

__global__ __launch_bounds__(64) void k_cr_elim_gemm(CRView v, int h, int total) {
  const int lb = xcd_block(total);
  if (lb < total) cr_elim_item(v, h, lb);
}

// One column strip of op(E) (rows 0..n, columns 16 tj .. +16) in registers, in
// tile_gemm's K order (lane k4 holds k = 8m + 2k4 and k + 1 of pair m).
template <bool TB>
__device__ __forceinline__ void load_strip(const double *B, int n, int tj, double (&bx)[kCRMaxN / 8],
                                           double (&by)[kCRMaxN / 8]) {
  using d2 = HIP_vector_type<double, 2>;
  const int lane = threadIdx.x & 63, r16 = lane & 15, k4 = lane >> 4, bc = tj * 16 + r16;
#pragma unroll
  for (int m = 0; m < kCRMaxN / 8; ++m) {
    const int k = 8 * m + 2 * k4;
    if (8 * m < n) {
      if (TB) {
        const d2 t = *reinterpret_cast<const d2 *>(B + bc * n + k);
        bx[m] = t.x;
        by[m] = t.y;
      } else {
        bx[m] = B[k * n + bc];
        by[m] = B[(k + 1) * n + bc];
      }
    }
  }
}

// Output tiles (ti, tj), ti = 0 .. nt-1, of Linv_I op(E) for one register strip,
// Linv_I read from the factor's LDS layout (linv_at): the K order of
// tile_gemm<false, TB, true>, so the same bits as k_cr_elim_gemm.
__device__ __forceinline__ void strip_tiles(const double *L, int ld, const double *Dinv, const double (&bx)[kCRMaxN / 8],
                                            const double (&by)[kCRMaxN / 8], double *out, int n, int tj) {
  const int lane = threadIdx.x & 63, r16 = lane & 15, k4 = lane >> 4, nt = n >> 4;
  for (int ti = 0; ti < nt; ++ti) {
    double ax[kCRMaxN / 8], ay[kCRMaxN / 8];
#pragma unroll
    for (int m = 0; m < kCRMaxN / 8; ++m) {
      const int k = 8 * m + 2 * k4, kb = m >> 1;  // k and k + 1 lie in block column kb
      if (kb <= ti) {
        const double *a =
            ti > kb ? L + (16 * kb + r16) * ld + 16 * ti + (k & 15) : Dinv + ti * kTile + r16 * kT + (k & 15);
        ax[m] = a[0];
        ay[m] = a[1];
      }
    }
    d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int m = 0; m < kCRMaxN / 8; ++m)
      if ((m >> 1) <= ti) {
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(ax[m], bx[m], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(ay[m], by[m], acc, 0, 0, 0);
      }
    tile_store(out, n, ti, tj, acc, 1.0, false);
  }
}

// Level h, steps 1 + 2 fused: the factor of k_cr_factor, then
// A_I = Linv_I E_{I-h}^T and C_I = Linv_I E_I with Linv_I still in LDS (one
// launch and one global read of Linv_I less per level). `split` workgroups
// serve one odd superblock: each factors it (redundantly: the deep levels
// leave the CUs idle, and the 112-pivot chain is the level's latency either
// way) and forms every split-th of the 2 n/16 output column strips; only the
// first stores Linv_I and z_I. Wave w of a workgroup owns its strips w and
// w + 8; both E strips are loaded before the first MFMA.
__global__ __launch_bounds__(512) void k_cr_factor_elim(CRView v, int h, int split) {
  static_assert(kCRMaxN / 16 <= 8, "two strips per wave of 8 cover at most 16 strips (kCRMaxN <= 128)");
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ int fail;
  const int ob = blockIdx.x / split, sidx = blockIdx.x - ob * split;
  const int I = h + 2 * h * ob;
  const int n = v.n, ld = n + 1, nt = n >> 4;
  const int nw = blockDim.x >> 6, wave = threadIdx.x >> 6;
  const int jobs = (I + h < v.p ? 2 : 1) * nt;
  const int q0 = sidx + split * wave, q1 = sidx + split * (wave + nw);
  double b0x[kCRMaxN / 8], b0y[kCRMaxN / 8], b1x[kCRMaxN / 8], b1y[kCRMaxN / 8];
  if (sidx == 0) cr_factor_store(v, I, lds, &fail);
  else cr_factor_block(v, I, lds, &fail);
  const double *L = lds, *Dinv = lds + n * ld + 2 * n;
  if (q0 < jobs) {
    if (q0 < nt) load_strip<true>(blk(v.E, I - h, n), n, q0, b0x, b0y);
    else load_strip<false>(blk(v.E, I, n), n, q0 - nt, b0x, b0y);
  }
  if (q1 < jobs) {
    if (q1 < nt) load_strip<true>(blk(v.E, I - h, n), n, q1, b1x, b1y);
    else load_strip<false>(blk(v.E, I, n), n, q1 - nt, b1x, b1y);
  }
  if (q0 < jobs) strip_tiles(L, ld, Dinv, b0x, b0y, q0 < nt ? blk(v.A, I, n) : blk(v.C, I, n), n, q0 % nt);
  if (q1 < jobs) strip_tiles(L, ld, Dinv, b1x, b1y, q1 < nt ? blk(v.A, I, n) : blk(v.C, I, n), n, q1 % nt);
}

// Workgroups per odd superblock of the fused factor + elimination: enough to
// spread a level's strips over the chip (one 134 KB-LDS workgroup per CU)
inline int cr_split(int n_odd, int nt) { return std::max(1, std::min(2 * nt, 256 / std::max(1, n_odd))); }

// Level h, step 3: every even superblock J absorbs its eliminated neighbours:
// D_J -= A_{J+h}^T A_{J+h} + C_{J-h}^T C_{J-h} (lower tiles only);
// E_J = -A_{J+h}^T C_{J+h}; g_J -= A_{J+h}^T z_{J+h} + C_{J-h}^T z_{J-h}.
// Work items per even block: nt(nt+1)/2 D tiles, nt^2 E tiles, nt g slices.
__device__ __forceinline__ void cr_update_item(const CRView &v, int h, int lb) {
  const int n = v.n, nt = n >> 4, nd = nt * (nt + 1) / 2, items = nd + nt * nt + nt;
  const int ev = lb / items, rem = lb - ev * items;
  const int J = 2 * h * ev;
  const bool right = J + h < v.p, left = J >= h;
  const int lane = threadIdx.x & 63, r16 = lane & 15, k4 = lane >> 4;
  if (rem < nd) {
    int ti = 0, tj = rem;
    while (tj > ti) { tj -= ti + 1; ++ti; }
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    if (right) acc = tile_gemm<true, false, false>(blk(v.A, J + h, n), blk(v.A, J + h, n), n, ti, tj);
    if (left) {
      const d4 a2 = tile_gemm<true, false, false>(blk(v.C, J - h, n), blk(v.C, J - h, n), n, ti, tj);
      acc += a2;
    }
    if (right || left) tile_store(blk(v.D, J, n), n, ti, tj, acc, -1.0, true);
  } else if (rem < nd + nt * nt) {
    const int t = rem - nd, ti = t / nt, tj = t - ti * nt;
    if (right && J + 2 * h < v.p) {
      const d4 acc = tile_gemm<true, false, false>(blk(v.A, J + h, n), blk(v.C, J + h, n), n, ti, tj);
      tile_store(blk(v.E, J, n), n, ti, tj, acc, -1.0, false);
    }
  } else {  // right-hand side rows 16 ti .. +16
    const int ar = 16 * (rem - nd - nt * nt) + r16;
    double s = 0.0;
    if (right) {
      const double *A = blk(v.A, J + h, n), *z = v.g + (size_t)(J + h) * n;
#pragma unroll
      for (int u = 0; u < kCRMaxN / 4; ++u) {
        const int k = kclamp(4 * u + k4, n);
        s += A[k * n + ar] * (4 * u < n ? z[k] : 0.0);
      }
    }
    if (left) {
      const double *C = blk(v.C, J - h, n), *z = v.g + (size_t)(J - h) * n;
#pragma unroll
      for (int u = 0; u < kCRMaxN / 4; ++u) {
        const int k = kclamp(4 * u + k4, n);
        s += C[k * n + ar] * (4 * u < n ? z[k] : 0.0);
      }
    }
    s = k4_sum(s);
    if (k4 == 0) st_d(v.g + (size_t)J * n + ar, v.g[(size_t)J * n + ar] - s);
  }
}

__global__ __launch_bounds__(64) void k_cr_update_gemm(CRView v, int h, int total) {
  const int lb = xcd_block(total);
  if (lb < total) cr_update_item(v, h, lb);
}

// Last remaining superblock 0: x_0 = D_0^-1 g_0 = Linv^T (Linv g).
__device__ __forceinline__ void cr_top_body(const CRView &v, double *lds, int *fail) {
  const int n = v.n, ld = n + 1, nt = n >> 4;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r16 = lane & 15, k4 = lane >> 4;
  cr_factor_block(v, 0, lds, fail);
  const double *L = lds;
  double *tmp = lds + n * ld, *z = tmp + n;
  const double *Dinv = tmp + 2 * n;
  const int ar = 16 * wave + r16;
  if (wave < nt) {
    const double s = linv_gemv(L, ld, Dinv, tmp, wave);
    if (k4 == 0) z[ar] = s;
  }
  __syncthreads();
  if (wave < nt) {
    const double s = linv_gemv_t(L, ld, Dinv, z, wave, nt);
    if (k4 == 0) v.x[ar] = s;
  }
  CR_PROF(34);
}

__global__ __launch_bounds__(512) void k_cr_top(CRView v) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ int fail;
  cr_top_body(v, lds, &fail);
}

// Back substitution at level h: x_I = Linv_I^T (z_I - A_I x_{I-h} - C_I x_{I+h}).
// One wave per 16-row slice (blockDim = 64 nt).
// Waves nt .. of a larger workgroup only join the barrier.
// LINV = false: only y = z_I - A_I x_{I-h} - C_I x_{I+h} into t (k_cr_back_u).
template <bool LINV>
__device__ __forceinline__ void cr_back_body(const CRView &v, int h, int I, double *t) {
  const int n = v.n;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, lo = lane & 7, hi = lane >> 3;
  const bool act = wave < (n >> 4);
  const bool right = I + h < v.p;
  // 16-byte loads, eight lanes per 128-byte line; every global load is issued
  // before the first use (one memory round trip, 56 loads in flight).
  // y = z - A x_{I-h} - C x_{I+h}: lane (hi, lo) takes rows 16 wave + hi (+8),
  // columns 16 u + 2 lo (+1); partial sums close over the eight lo lanes.
  // x_I = Linv^T y: lane takes columns 16 wave + 2 lo (+1), rows k = 16 wave + 8 u + hi
  // (Linv is lower triangular, rows below 16 wave are zero); sums close over hi.
  using d2 = HIP_vector_type<double, 2>;
  const int ca = 2 * lo;
  const d2 *A = reinterpret_cast<const d2 *>(blk(v.A, I, n)), *C = reinterpret_cast<const d2 *>(blk(v.C, I, n));
  const d2 *xl = reinterpret_cast<const d2 *>(v.x + (size_t)(I - h) * n);
  const d2 *xr = reinterpret_cast<const d2 *>(v.x + (size_t)(I + (right ? h : 0)) * n);
  const d2 *Li = reinterpret_cast<const d2 *>(blk(v.L, I, n));
  const int r0 = 16 * wave + hi, hn = n >> 1;
  d2 a0[kCRMaxN / 16], a1[kCRMaxN / 16], c0[kCRMaxN / 16], c1[kCRMaxN / 16], vl[kCRMaxN / 16], vr[kCRMaxN / 16];
  d2 li[kCRMaxN / 8];
  if (act) {
#pragma unroll
  for (int u = 0; u < kCRMaxN / 16; ++u) {
    const int c = kclamp(16 * u + ca, n) >> 1;
    a0[u] = A[r0 * hn + c];
    a1[u] = A[(r0 + 8) * hn + c];
    vl[u] = xl[c];
  }
  if (LINV) {
#pragma unroll
    for (int u = 0; u < kCRMaxN / 8; ++u) li[u] = Li[kclamp(16 * wave + 8 * u + hi, n) * hn + 8 * wave + lo];
  }
  if (right) {
#pragma unroll
    for (int u = 0; u < kCRMaxN / 16; ++u) {
      const int c = kclamp(16 * u + ca, n) >> 1;
      c0[u] = C[r0 * hn + c];
      c1[u] = C[(r0 + 8) * hn + c];
      vr[u] = xr[c];
    }
  }
  double s0 = 0.0, s1 = 0.0;
#pragma unroll
  for (int u = 0; u < kCRMaxN / 16; ++u)
    if (16 * u < n) {
      s0 += a0[u].x * vl[u].x + a0[u].y * vl[u].y;
      s1 += a1[u].x * vl[u].x + a1[u].y * vl[u].y;
      if (right) {
        s0 += c0[u].x * vr[u].x + c0[u].y * vr[u].y;
        s1 += c1[u].x * vr[u].x + c1[u].y * vr[u].y;
      }
    }
#pragma unroll
  for (int m = 1; m < 8; m <<= 1) {
    s0 += __shfl_xor(s0, m, 64);
    s1 += __shfl_xor(s1, m, 64);
  }
  if (lo == 0) {
    t[r0] = v.g[(size_t)I * n + r0] - s0;
    t[r0 + 8] = v.g[(size_t)I * n + r0 + 8] - s1;
  }
  }
  __syncthreads();
  if (!LINV || !act) return;
  double x0 = 0.0, x1 = 0.0;
#pragma unroll
  for (int u = 0; u < kCRMaxN / 8; ++u) {
    const int k = 16 * wave + 8 * u + hi;
    const double tk = k < n ? t[kclamp(k, n)] : 0.0;
    x0 += li[u].x * tk;
    x1 += li[u].y * tk;
  }
#pragma unroll
  for (int m = 8; m < 64; m <<= 1) {
    x0 += __shfl_xor(x0, m, 64);
    x1 += __shfl_xor(x1, m, 64);
  }
  if (hi == 0) {
    v.x[(size_t)I * n + 16 * wave + ca] = x0;
    v.x[(size_t)I * n + 16 * wave + ca + 1] = x1;
  }
}

__global__ __launch_bounds__(512) void k_cr_back(CRView v, int h) {
  extern __shared__ __attribute__((aligned(16))) double t[];
  cr_back_body<true>(v, h, h + 2 * h * blockIdx.x, t);
}

// Back substitution with the factor kept as U (upper tiles) and T_i = L_ii^-1
// on the diagonal (k_cr_aug<.., false>): x_I = U^-1 y with y = z_I - A_I x_{I-h}
// - C_I x_{I+h} (TOP: y = z_0), blocked from the bottom:
//   x_i = T_i^T (y_i - sum_{j>i} U_ij x_j),  i = nt-1 .. 0.
// Wave i owns block row i: its U tiles and T_i are loaded up front, each U_ij x_j
// term is added as soon as x_j is flagged in LDS, so after x_{i+1} only one
// 16x16 product, two 16-lane sums and T_i^T remain on the chain.
template <bool TOP>
__device__ __forceinline__ void back_u_body(double *sm, const CRView &v, int h, int I) {
  double *y = sm, *rr = sm + kCRMaxN, *xs = sm + 2 * kCRMaxN;
  int *fx = reinterpret_cast<int *>(sm + 3 * kCRMaxN);
  const int n = v.n, nt = n >> 4;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, q = lane >> 4, r = lane & 15;
  if (threadIdx.x < aug::kMaxNt) fx[threadIdx.x] = 0;
  // this wave's U row and T_i first: in flight during the right-hand side
  const int i = wave < nt ? wave : nt - 1;
  const double *Lb = blk(v.L, I, n);
  double u[aug::kMaxNt][4], tv[4];
#pragma unroll
  for (int j = 0; j < aug::kMaxNt; ++j)
    if (j > i && j < nt) {
#pragma unroll
      for (int m = 0; m < 4; ++m) u[j][m] = Lb[(size_t)(16 * i + r) * n + 16 * j + 4 * q + m];  // U_ij[r][4q+m]
    }
#pragma unroll
  for (int m = 0; m < 4; ++m) tv[m] = Lb[(size_t)(16 * i + 4 * q + m) * n + 16 * i + r];  // T_i[4q+m][r]
  if (TOP) {
    for (int k = threadIdx.x; k < n; k += blockDim.x) y[k] = v.g[(size_t)I * n + k];
    __syncthreads();
  } else {
    cr_back_body<false>(v, h, I, y);  // ends with a barrier (also covers fx)
  }
  if (wave >= nt) return;
  bool tmo = false;
  double acc = 0.0;
#pragma unroll
  for (int j = aug::kMaxNt - 1; j > 0; --j)
    if (j > i && j < nt) {
      tmo |= !aug::spin(&fx[j]);
#pragma unroll
      for (int m = 0; m < 4; ++m) acc = fma(u[j][m], xs[16 * j + 4 * q + m], acc);
    }
  acc += __shfl_xor(acc, 16, 64);
  acc += __shfl_xor(acc, 32, 64);
  if (q == 0) rr[16 * i + r] = y[16 * i + r] - acc;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  double x = 0.0;
#pragma unroll
  for (int m = 0; m < 4; ++m) x = fma(tv[m], rr[16 * i + 4 * q + m], x);  // lane (q, c = r)
  x += __shfl_xor(x, 16, 64);
  x += __shfl_xor(x, 32, 64);
  if (q == 0) {
    xs[16 * i + r] = x;
    st_d(v.x + (size_t)I * n + 16 * i + r, x);
  }
  aug::raise_flag(&fx[i], lane);
  if (tmo) cr_fail(v, lane);
}

template <bool TOP>
__global__ __launch_bounds__(512) void k_cr_back_u(CRView v, int h) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  back_u_body<TOP>(sm, v, h, TOP ? 0 : h + 2 * h * blockIdx.x);
}

// ---- every back-substitution level in one launch ----------------------------
// The levels of k_cr_back_u<false> are a chain of dependent launches whose
// work is tiny next to their launch and load latency (9 x 7-12 us on config
// 4's band for ~2 us of arithmetic each). Here one launch holds a workgroup per
// odd superblock of every level, coarsest level first: each loads its
// operands (A_I, C_I, z_I, U_I, T), written by earlier launches, at once, then
// waits for its neighbours' solutions x_{I-h}, x_{I+h} -- superblock 0 (the top
// solve, an earlier launch) or superblocks of coarser levels, i.e. workgroups
// with lower ids, dispatched before it, so the launch drains at any residency
// -- and runs k_cr_back_u's arithmetic in the same order (the same bits).
// Hand-off across the chip (per-XCD L2s): x_I is stored write-through (agent
// scope, sc1), drained (vmcnt(0)) by every storing wave, then after a barrier
// one lane stores done[I] = epoch (sc1; a per-solve counter, so nothing is
// reset); the consumer polls that word with sc1 loads and s_sleep and reads x
// with sc1 loads only. Bounded: a wait that gives up fails the solve
// (cr_fail -> SQLM_ERR_HIP), and every wave still reaches the end.
// Assumption: a workgroup is dispatched no earlier than every lower-numbered
// workgroup of the same launch (the command processor's in-order dispatch on
// gfx950; HIP does not promise it). If it ever fails, a waiting workgroup
// that holds the CU a producer needs times out and the solve fails loudly
// instead of hanging. -DSQLM_SPIN_FORCE_TIMEOUT (tests) makes this wait, like
// aug::spin / spin_to, report a timeout after it has completed, so
// tests/test_gpu_fail_loud.py runs this hand-off's give-up path too.
__device__ __forceinline__ bool wait_x(const CRView &v, int J) {
  bool ok = J == 0;  // the top superblock: solved by an earlier launch
  const int *f = v.done + J;
  for (int it = 0; !ok && it < aug::kSpinLimit; ++it) {
    if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == v.epoch) ok = true;
    else __builtin_amdgcn_s_sleep(2);
  }
#ifdef SQLM_SPIN_FORCE_TIMEOUT
  ok = false;
#endif
  return ok;
}
__device__ __forceinline__ double ld_x(const double *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void back_all_body(double *sm, const CRView &v, int h, int I) {
  double *y = sm, *rr = sm + kCRMaxN, *xs = sm + 2 * kCRMaxN;
  int *fx = reinterpret_cast<int *>(sm + 3 * kCRMaxN);
  __shared__ int tmo_s;
  const int n = v.n, nt = n >> 4;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, q = lane >> 4, r = lane & 15;
  const int lo = lane & 7, hi = lane >> 3;
  const bool right = I + h < v.p;
  if (threadIdx.x < aug::kMaxNt) fx[threadIdx.x] = 0;
  // this wave's U row and T_i (blockDim = 64 nt: wave i owns block row i)
  const int i = wave;
  const double *Lb = blk(v.L, I, n);
  double u[aug::kMaxNt][4], tv[4];
#pragma unroll
  for (int j = 0; j < aug::kMaxNt; ++j)
    if (j > i && j < nt) {
#pragma unroll
      for (int m = 0; m < 4; ++m) u[j][m] = Lb[(size_t)(16 * i + r) * n + 16 * j + 4 * q + m];  // U_ij[r][4q+m]
    }
#pragma unroll
  for (int m = 0; m < 4; ++m) tv[m] = Lb[(size_t)(16 * i + 4 * q + m) * n + 16 * i + r];  // T_i[4q+m][r]
  // A_I, C_I rows and z_I (cr_back_body's lane map: rows 16 wave + hi (+8),
  // columns 16 u + 2 lo (+1))
  using d2 = HIP_vector_type<double, 2>;
  const int ca = 2 * lo;
  const d2 *A = reinterpret_cast<const d2 *>(blk(v.A, I, n)), *C = reinterpret_cast<const d2 *>(blk(v.C, I, n));
  const int r0 = 16 * wave + hi, hn = n >> 1;
  d2 a0[kCRMaxN / 16], a1[kCRMaxN / 16], c0[kCRMaxN / 16], c1[kCRMaxN / 16];
#pragma unroll
  for (int uu = 0; uu < kCRMaxN / 16; ++uu) {
    const int c = kclamp(16 * uu + ca, n) >> 1;
    a0[uu] = A[r0 * hn + c];
    a1[uu] = A[(r0 + 8) * hn + c];
  }
  if (right) {
#pragma unroll
    for (int uu = 0; uu < kCRMaxN / 16; ++uu) {
      const int c = kclamp(16 * uu + ca, n) >> 1;
      c0[uu] = C[r0 * hn + c];
      c1[uu] = C[(r0 + 8) * hn + c];
    }
  }
  const double z0 = v.g[(size_t)I * n + r0], z1 = v.g[(size_t)I * n + r0 + 8];
  // the neighbours' solutions: every load of them is an sc1 load (ld_x) of
  // bytes stored sc1 and drained before the flag, so no acquire fence (an
  // L1 invalidate, ~1.7 us) is needed (MI355X_MICROARCH.md, hand-off table
  // row 1: one flag per storing workgroup, one workgroup per CU)
  if (threadIdx.x == 0) {
    bool ok = wait_x(v, I - h);
    if (right) ok = wait_x(v, I + h) && ok;
    tmo_s = ok ? 0 : 1;
  }
  __syncthreads();
  const bool tmo = tmo_s != 0;
  const double *xl = v.x + (size_t)(I - h) * n, *xr = v.x + (size_t)(I + (right ? h : 0)) * n;
  d2 vl[kCRMaxN / 16], vr[kCRMaxN / 16];
#pragma unroll
  for (int uu = 0; uu < kCRMaxN / 16; ++uu) {
    const int c = (kclamp(16 * uu + ca, n) >> 1) << 1;  // the pair cr_back_body's 16-byte load takes
    vl[uu].x = ld_x(xl + c);
    vl[uu].y = ld_x(xl + c + 1);
    if (right) {
      vr[uu].x = ld_x(xr + c);
      vr[uu].y = ld_x(xr + c + 1);
    }
  }
  // y = z - A x_{I-h} - C x_{I+h} (cr_back_body<false>, the same expressions)
  double s0 = 0.0, s1 = 0.0;
#pragma unroll
  for (int uu = 0; uu < kCRMaxN / 16; ++uu)
    if (16 * uu < n) {
      s0 += a0[uu].x * vl[uu].x + a0[uu].y * vl[uu].y;
      s1 += a1[uu].x * vl[uu].x + a1[uu].y * vl[uu].y;
      if (right) {
        s0 += c0[uu].x * vr[uu].x + c0[uu].y * vr[uu].y;
        s1 += c1[uu].x * vr[uu].x + c1[uu].y * vr[uu].y;
      }
    }
#pragma unroll
  for (int m = 1; m < 8; m <<= 1) {
    s0 += __shfl_xor(s0, m, 64);
    s1 += __shfl_xor(s1, m, 64);
  }
  if (lo == 0) {
    y[r0] = z0 - s0;
    y[r0 + 8] = z1 - s1;
  }
  __syncthreads();
  // x_I = U^-1 y from the bottom (back_u_body's chain)
  bool tw = false;
  double acc = 0.0;
#pragma unroll
  for (int j = aug::kMaxNt - 1; j > 0; --j)
    if (j > i && j < nt) {
      tw |= !aug::spin(&fx[j]);
#pragma unroll
      for (int m = 0; m < 4; ++m) acc = fma(u[j][m], xs[16 * j + 4 * q + m], acc);
    }
  acc += __shfl_xor(acc, 16, 64);
  acc += __shfl_xor(acc, 32, 64);
  if (q == 0) rr[16 * i + r] = y[16 * i + r] - acc;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  double x = 0.0;
#pragma unroll
  for (int m = 0; m < 4; ++m) x = fma(tv[m], rr[16 * i + 4 * q + m], x);  // lane (q, c = r)
  x += __shfl_xor(x, 16, 64);
  x += __shfl_xor(x, 32, 64);
  if (q == 0) {
    xs[16 * i + r] = x;
    __hip_atomic_store(v.x + (size_t)I * n + 16 * i + r, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  aug::raise_flag(&fx[i], lane);
  if (tmo || tw) cr_fail(v, lane);
  // publish x_I: every wave's stores drained, then the completion word
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(v.done + I, v.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// blockIdx -> (level h, odd superblock I), coarsest level (h_top) first
__global__ __launch_bounds__(512) void k_cr_back_all(CRView v, int h_top) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  int b = blockIdx.x, h = h_top;
  for (;;) {
    const int n_odd = (v.p - h + 2 * h - 1) / (2 * h);
    if (b < n_odd || h == 1) break;
    b -= n_odd;
    h >>= 1;
  }
  back_all_body(sm, v, h, h + 2 * h * b);
}


// ---- dense SPD solve (essential graph) --------------------------------------
// Blocked right-looking Cholesky of an n x n SPD matrix (n a multiple of
// kCRMaxN, lower triangle of A row-major), block size nb = kCRMaxN:
//   Linv_kk = chol(A_kk)^-1 (LDS factor), L_ik = A_ik Linv_kk^T,
//   A_ij -= L_ik L_jk^T (k < j <= i, MFMA tiles),
// then L L^T x = b by block forward / backward substitution.
struct DenseView {
  int n, nblk;
  double *A, *L, *Linv;  // [n][n], [n][n], [nblk][nb][nb]
  double *r, *x;         // [n] right-hand side (consumed), solution
  int *flags;
};

// nk: rows of the block that are not identity padding (a multiple of 16; the
// ragged last block of a padded system): only those are factored, the rest of
// Linv is the identity — the same bits as factoring the padded block.
__global__ __launch_bounds__(512) void k_dchol_diag(DenseView v, int k, int nk) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ int fail;
  constexpr int nb = kCRMaxN;
  const int ld = nb + 1, nw = blockDim.x >> 6, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double *L = lds, *tmp = lds + nb * ld, *Dinv = tmp + 2 * nb, *W = Dinv + 17 * nb, *invd = W + 17 * nb;
  const double *Ak = v.A + (size_t)k * nb * v.n + (size_t)k * nb;
  for (int r = wave; r < nk; r += nw)
    for (int c = lane; c < nk; c += 64)
      if (c <= (r | 15)) L[r * ld + c] = Ak[(size_t)r * v.n + c];
  __syncthreads();
  if (!wg_potrf_trtri(L, ld, nk, Dinv, W, invd, &fail) && threadIdx.x == 0) v.flags[0] = 0;
  double *Lo = v.Linv + (size_t)k * nb * nb;
  for (int r = wave; r < nb; r += nw)
    for (int c = lane; c < nb; c += 64)
      Lo[r * nb + c] = (r < nk && c < nk) ? linv_at(L, ld, Dinv, r, c) : (r == c ? 1.0 : 0.0);
  // fused forward step: y_k = Linv_kk r_k (r_k already holds every earlier
  // block's update) in place; thread (row, quarter), quarters summed in order
  constexpr int q = nb / 4;
  const int t = threadIdx.x, row = t % nb, h = t / nb;
  const double *rk = v.r + (size_t)k * nb;
  if (h < 4 && row < nk) {
    double s = 0.0;
#pragma unroll 4
    for (int i = 0; i < q; ++i) {
      const int m = h * q + i;
      if (m <= row) s += linv_at(L, ld, Dinv, row, m) * rk[m];
    }
    W[h * nb + row] = s;
  } else if (h < 4) {
    W[h * nb + row] = h == 0 ? rk[row] : 0.0;  // identity row
  }
  __syncthreads();
  if (t < nb) v.r[(size_t)k * nb + t] = ((W[t] + W[nb + t]) + W[2 * nb + t]) + W[3 * nb + t];
}

// 16x16 tile of X Y^T over K = kend (X, Y row-major with their own leading dims).
__device__ __forceinline__ d4 tile_xyt(const double *X, int ldx, const double *Y, int ldy, int kend) {
  using d2 = HIP_vector_type<double, 2>;
  const int lane = threadIdx.x & 63, r16 = lane & 15, k4 = lane >> 4;
  d2 av[kCRMaxN / 8], bv[kCRMaxN / 8];
#pragma unroll
  for (int m = 0; m < kCRMaxN / 8; ++m)
    if (8 * m < kend) {
      av[m] = *reinterpret_cast<const d2 *>(X + (size_t)r16 * ldx + 8 * m + 2 * k4);
      bv[m] = *reinterpret_cast<const d2 *>(Y + (size_t)r16 * ldy + 8 * m + 2 * k4);
    }
  d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int m = 0; m < kCRMaxN / 8; ++m)
    if (8 * m < kend) {
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[m].x, bv[m].x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[m].y, bv[m].y, acc, 0, 0, 0);
    }
  return acc;
}

// Block rows of L below block k that can be nonzero: an optional `extra` row
// (the next band block of a block-arrow matrix) then the range [r0, r1).
// Dense: extra = -1, [k+1, nblk). Arrow (block-tridiagonal band of `band`
// blocks, dense border after it), band block k: extra = k+1 (if in the band),
// range = the border.
struct RowSet {
  int extra, r0, r1;
  __host__ __device__ int count() const { return (extra >= 0) + (r1 - r0); }
  __host__ __device__ int at(int i) const { return extra >= 0 ? (i == 0 ? extra : r0 + i - 1) : r0 + i; }
};

inline RowSet rows_below(int k, int nblk, int band) {
  if (k >= band) return RowSet{-1, k + 1, nblk};
  return RowSet{k + 1 < band ? k + 1 : -1, band, nblk};
}

__global__ __launch_bounds__(64) void k_dchol_update_tiles(DenseView v, int k, RowSet rs, int total) {
  const int lb = xcd_block(total);
  if (lb >= total) return;
  constexpr int nb = kCRMaxN, nt = nb / 16;
  // block pair (bi, bj), bi >= bj, row-major over the lower triangle of rs; 49 tiles each
  const int pair = lb / (nt * nt), t = lb % (nt * nt);
  int ii = 0, rem = pair;
  while (rem > ii) { rem -= ii + 1; ++ii; }
  const int bi = rs.at(ii), bj = rs.at(rem), ti = t / nt, tj = t % nt;
  if (bi == bj && tj > ti) return;
  const double *X = v.L + (size_t)(bi * nb + 16 * ti) * v.n + (size_t)k * nb;
  const double *Y = v.L + (size_t)(bj * nb + 16 * tj) * v.n + (size_t)k * nb;
  const d4 acc = tile_xyt(X, v.n, Y, v.n, nb);
  const int lane = threadIdx.x & 63, r16 = lane & 15, k4 = lane >> 4;
  double *o = v.A + (size_t)(bi * nb + 16 * ti) * v.n + (size_t)bj * nb + 16 * tj;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[(size_t)(k4 + 4 * j) * v.n + r16] -= acc[j];
}

// L_ik = A_ik Linv_kk^T for the block rows i of rs; one wavefront per 16x16 tile.
__global__ __launch_bounds__(64) void k_dchol_panel(DenseView v, int k, RowSet rs, int total) {
  const int lb = xcd_block(total);
  if (lb >= total) return;
  constexpr int nb = kCRMaxN, nt = nb / 16;
  const int bi = rs.at(lb / (nt * nt)), t = lb % (nt * nt), ti = t / nt, tj = t % nt;
  const double *X = v.A + (size_t)(bi * nb + 16 * ti) * v.n + (size_t)k * nb;
  const double *Y = v.Linv + (size_t)k * nb * nb + (size_t)(16 * tj) * nb;  // Linv rows 16 tj..: lower, K <= 16 (tj+1)
  const d4 acc = tile_xyt(X, v.n, Y, nb, 16 * (tj + 1));
  const int lane = threadIdx.x & 63, r16 = lane & 15, k4 = lane >> 4;
  double *o = v.L + (size_t)(bi * nb + 16 * ti) * v.n + (size_t)k * nb + 16 * tj;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[(size_t)(k4 + 4 * j) * v.n + r16] = acc[j];
}

// A_ij -= L_ik L_jk^T for k < j <= i (diagonal blocks: lower tiles only).
// The same update with one wavefront per 16x16 tile and operands straight
// from L2 / HBM: more parallelism per pair, used when there are few pairs (the
// block-arrow band steps), where one workgroup per pair is latency-bound.
struct RowSet;
__global__ __launch_bounds__(64) void k_dchol_update_tiles(DenseView v, int k, RowSet rs, int total);

// A_ij -= L_ik L_jk^T for one 112x112 block pair (bi, bj), bi >= bj > k, per
// workgroup of 8 waves: the two 112 x 16 K-slices of L are staged in LDS (16-
// byte loads, double-buffered), waves 0..6 each accumulate one row of 16x16
// output tiles (lower 28 only on the diagonal pair) in registers with
// v_mfma_f64_16x16x4f64. Per pair: 1372 MFMAs on 200 KB of L2 reads, so the
// update runs on the matrix cores instead of the L2 (the one-wave-per-tile
// k_dchol_update re-reads both 16 x 112 slices for every tile).
constexpr int kUpdKC = 16, kUpdLd = kUpdKC + 2;  // row stride: 16-byte aligned, spreads the 16 rows over banks
__global__ __launch_bounds__(512) void k_dchol_update_blk(DenseView v, int k, RowSet rs, int npairs) {
  constexpr int nb = kCRMaxN, nt = nb / 16, nkc = nb / kUpdKC;
  __shared__ __attribute__((aligned(16))) double Xs[2][nb * kUpdLd];
  __shared__ __attribute__((aligned(16))) double Ys[2][nb * kUpdLd];
  const int lb = xcd_block(npairs);
  if (lb >= npairs) return;
  int ii = 0, rem = lb;
  while (rem > ii) { rem -= ii + 1; ++ii; }
  const int bi = rs.at(ii), bj = rs.at(rem);
  const bool diag = bi == bj;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r16 = lane & 15, k4 = lane >> 4;
  const double *X = v.L + (size_t)bi * nb * v.n + (size_t)k * nb;
  const double *Y = v.L + (size_t)bj * nb * v.n + (size_t)k * nb;
  // staging: 112 rows x 16 doubles = 896 double2 per operand; 512 threads, 2 passes
  auto stage = [&](int buf, int kc) {
    for (int e = tid; e < nb * kUpdKC / 2; e += 512) {
      const int r = e >> 3, c2 = (e & 7) * 2;
      const double2 xv = *reinterpret_cast<const double2 *>(X + (size_t)r * v.n + kc * kUpdKC + c2);
      *reinterpret_cast<double2 *>(&Xs[buf][r * kUpdLd + c2]) = xv;
      if (!diag) {
        const double2 yv = *reinterpret_cast<const double2 *>(Y + (size_t)r * v.n + kc * kUpdKC + c2);
        *reinterpret_cast<double2 *>(&Ys[buf][r * kUpdLd + c2]) = yv;
      }
    }
  };
  // wave w < 7 owns output tile row ti = w (tiles tj = 0..6, tj <= ti on the
  // diagonal pair): its A operand is read once per K step for all 7 tiles
  d4 acc[nt];
#pragma unroll
  for (int q = 0; q < nt; ++q) acc[q] = d4{0.0, 0.0, 0.0, 0.0};
  const int ti = wave, tjmax = diag ? ti : nt - 1;
  stage(0, 0);
  __syncthreads();
  for (int kc = 0; kc < nkc; ++kc) {
    const int buf = kc & 1;
    if (kc + 1 < nkc) stage(buf ^ 1, kc + 1);
    const double *Xb = Xs[buf], *Yb = diag ? Xs[buf] : Ys[buf];
    if (ti < nt) {
#pragma unroll
      for (int s = 0; s < kUpdKC / 4; ++s) {
        const double a = Xb[(16 * ti + r16) * kUpdLd + 4 * s + k4];
#pragma unroll
        for (int tj = 0; tj < nt; ++tj)
          if (tj <= tjmax) {
            const double b = Yb[(16 * tj + r16) * kUpdLd + 4 * s + k4];
            acc[tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[tj], 0, 0, 0);
          }
      }
    }
    __syncthreads();
  }
  if (ti < nt) {
#pragma unroll
    for (int tj = 0; tj < nt; ++tj)
      if (tj <= tjmax) {
        double *o = v.A + (size_t)(bi * nb + 16 * ti) * v.n + (size_t)bj * nb + 16 * tj;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[(size_t)(k4 + 4 * j) * v.n + r16] -= acc[tj][j];
      }
  }
}

// one wavefront per row of the block rows rs below block k: r_i -= L_i,k-block . y_k
// (y_k in r_k: the diagonal step forms it in place)
__global__ __launch_bounds__(256) void k_dtrsv_fwd_update(DenseView v, int k, RowSet rs) {
  constexpr int nb = kCRMaxN;
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (q >= rs.count() * nb) return;
  const int row = rs.at(q / nb) * nb + q % nb;
  const double *Lr = v.L + (size_t)row * v.n + (size_t)k * nb, *y = v.r + (size_t)k * nb;
  double s = 0.0;
  for (int m = lane; m < nb; m += 64) s += Lr[m] * y[m];
  s = wave_sum_d(s);
  if (lane == 0) v.r[row] -= s;
}

// backward: x_k = Linv_kk^T r_k: thread (c, part) sums rows m = c.. of its
// quarter for column c (consecutive threads read consecutive columns of one
// row: coalesced), the four quarters are added in LDS in a fixed order.
__global__ __launch_bounds__(512) void k_dtrsv_bwd_diag(DenseView v, int k) {
  constexpr int nb = kCRMaxN, q = nb / 4;
  __shared__ double part[4][nb];
  const int t = threadIdx.x, c = t % nb, h = t / nb;
  const double *Lk = v.Linv + (size_t)k * nb * nb, *rk = v.r + (size_t)k * nb;
  if (h < 4) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < q; ++i) {
      const int m = h * q + i;
      s += m >= c ? Lk[(size_t)m * nb + c] * rk[m] : 0.0;
    }
    part[h][c] = s;
  }
  __syncthreads();
  if (t < nb) v.x[(size_t)k * nb + t] = ((part[0][t] + part[1][t]) + part[2][t]) + part[3][t];
}

// columns [c0 nb, k nb) left of block k whose L_kj can be nonzero
__global__ __launch_bounds__(256) void k_dtrsv_bwd_update(DenseView v, int k, int c0) {
  constexpr int nb = kCRMaxN;
  const int c = c0 * nb + blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= k * nb) return;
  const double *Lk = v.L + (size_t)k * nb * v.n + c, *xk = v.x + (size_t)k * nb;
  double s[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 28
  for (int m = 0; m < nb; ++m) s[m & 3] += Lk[(size_t)m * v.n] * xk[m];
  v.r[c] -= (s[0] + s[1]) + (s[2] + s[3]);
}

inline bool cr_legacy();
static void launch_cr_factor(const CRView &v, int h, int I0, int stride, int count, bool linv, hipStream_t st);

int launch_dense_spd_solve(double *A, double *L, double *Linv, double *r, double *x, int *flags, int n,
                           hipStream_t st, int band, int n_last) {
  constexpr int nb = kCRMaxN, nt = nb / 16;
  if (n <= 0 || n % nb) return -1;
  if (n_last <= 0 || n_last > nb || n_last % 16) n_last = nb;
  const int nblk = n / nb;
  band = std::max(0, std::min(band, nblk));
  DenseView v{n, nblk, A, L, Linv, r, x, flags};
  const size_t lds = cr_factor_lds(nb);
  // factor + forward substitution in one sweep: block k's diagonal kernel also
  // forms y_k = Linv_kk r_k (in place), then the panel, the trailing update and
  // r_i -= L_ik y_k for the rows below. The diagonal factor is the augmented
  // MFMA Cholesky of sqlm_cr_aug.h on the block in place (row stride n; the
  // identity padding of a ragged last block factors to itself exactly).
  for (int k = 0; k < nblk; ++k) {
    if (cr_legacy()) {
      hipLaunchKernelGGL(k_dchol_diag, dim3(1), dim3(512), lds, st, v, k, k == nblk - 1 ? n_last : nb);
    } else {
      const CRView dv{1, nb, 0, 0, A + (size_t)k * nb * n + (size_t)k * nb, nullptr, nullptr, nullptr,
                      r + (size_t)k * nb, nullptr, flags, Linv + (size_t)k * nb * nb, n};
      launch_cr_factor(dv, 0, 0, 0, 1, true, st);
    }
    const RowSet rs = rows_below(k, nblk, band);
    const int m = rs.count();
    if (m == 0) continue;
    const int np = m * nt * nt, npairs = m * (m + 1) / 2;
    hipLaunchKernelGGL(k_dchol_panel, dim3(xcd_grid(np)), dim3(64), 0, st, v, k, rs, np);
    if (npairs < 128)  // few pairs: one wave per tile keeps every CU busy
      hipLaunchKernelGGL(k_dchol_update_tiles, dim3(xcd_grid(npairs * nt * nt)), dim3(64), 0, st, v, k, rs,
                         npairs * nt * nt);
    else
      hipLaunchKernelGGL(k_dchol_update_blk, dim3(xcd_grid(npairs)), dim3(512), 0, st, v, k, rs, npairs);
    hipLaunchKernelGGL(k_dtrsv_fwd_update, dim3((m * nb + 3) / 4), dim3(256), 0, st, v, k, rs);
  }
  // y (in r) is the right-hand side of the backward pass
  for (int k = nblk - 1; k >= 0; --k) {
    hipLaunchKernelGGL(k_dtrsv_bwd_diag, dim3(1), dim3(512), 0, st, v, k);
    // L_kj != 0: j = k - 1 for a band block, every j < k for a border block
    const int c0 = k < band ? std::max(k - 1, 0) : 0;
    if (k > c0)
      hipLaunchKernelGGL(k_dtrsv_bwd_update, dim3(((k - c0) * nb + 255) / 256), dim3(256), 0, st, v, k, c0);
  }
  return 0;
}

// ---- block-tridiagonal solve with many right-hand sides (essential graph) ----
// The elimination of launch_cr_core (k_cr_factor, k_cr_elim_gemm,
// k_cr_update_gemm on D / E; their single right-hand side runs on a scratch
// vector), with R right-hand sides G [p][n][R] carried by MFMA tile GEMMs
// (one wavefront per 16x16 tile):
//   odd I at level h:  Z_I = Linv_I G_I
//   even J:            G_J -= A_{J+h}^T Z_{J+h} + C_{J-h}^T Z_{J-h}
//   top (block 0):     X_0 = Linv_0^T (Linv_0 G_0)
//   back, odd I:       X_I = Linv_I^T (Z_I - A_I X_{I-h} - C_I X_{I+h}).
struct CRMView {
  int p, n, R;
  const double *D, *A, *C;  // D_I = Linv_I (lower) once block I is factored
  double *G, *Z, *X;        // [p][n][R]
};

// acc = op(A)[16 ti .. +16][k0 .. k1) B[k0 .. k1)[16 tj .. +16] (row-major;
// op(A) = A or A^T), k1 - k0 <= kCRMaxN; every operand load is issued before
// the first MFMA (clamped index, zero weight past k1).
template <bool TA>
__device__ __forceinline__ d4 mm_tile(const double *A, int lda, const double *B, int ldb, int ti, int tj, int k0,
                                      int k1) {
  const int lane = threadIdx.x & 63, r16 = lane & 15, k4 = lane >> 4;
  const int ar = 16 * ti + r16, bc = 16 * tj + r16;
  constexpr int S = kCRMaxN / 4;
  double a[S], b[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int k = k0 + 4 * s + k4, kc = k < k1 ? k : k1 - 1;
    a[s] = TA ? A[(size_t)kc * lda + ar] : A[(size_t)ar * lda + kc];
    b[s] = k < k1 ? B[(size_t)kc * ldb + bc] : 0.0;
  }
  d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int s = 0; s < S; ++s)
    if (k0 + 4 * s < k1) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[s], acc, 0, 0, 0);
  return acc;
}

__device__ __forceinline__ void mm_store(double *C, int ldc, int ti, int tj, const d4 &acc, double alpha, bool add) {
  const int lane = threadIdx.x & 63, r16 = lane & 15, k4 = lane >> 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double *c = C + (size_t)(16 * ti + k4 + 4 * j) * ldc + 16 * tj + r16;
    *c = add ? *c + alpha * acc[j] : alpha * acc[j];
  }
}

// Z_I = Linv_I G_I for I = I0 + stride q (Linv lower: K up to the tile row)
__device__ __forceinline__ void crm_fwd_item(const CRMView &v, int I0, int stride, int lb) {
  const int nt = v.n >> 4, rt = v.R >> 4, per = nt * rt;
  const int q = lb / per, t = lb - q * per, ti = t / rt, tj = t - ti * rt, I = I0 + stride * q;
  const size_t nn = (size_t)v.n * v.n, nr = (size_t)v.n * v.R;
  const d4 acc = mm_tile<false>(v.D + I * nn, v.n, v.G + I * nr, v.R, ti, tj, 0, 16 * (ti + 1));
  mm_store(v.Z + I * nr, v.R, ti, tj, acc, 1.0, false);
}

__global__ __launch_bounds__(64) void k_crm_fwd(CRMView v, int I0, int stride, int total) {
  const int lb = xcd_block(total);
  if (lb < total) crm_fwd_item(v, I0, stride, lb);
}

// even J = 2 h q: G_J -= A_{J+h}^T Z_{J+h} + C_{J-h}^T Z_{J-h}
__device__ __forceinline__ void crm_upd_item(const CRMView &v, int h, int lb) {
  const int n = v.n, nt = n >> 4, rt = v.R >> 4, per = nt * rt;
  const int q = lb / per, t = lb - q * per, ti = t / rt, tj = t - ti * rt, J = 2 * h * q;
  const size_t nn = (size_t)n * n, nr = (size_t)n * v.R;
  d4 acc = {0.0, 0.0, 0.0, 0.0};
  const bool right = J + h < v.p, left = J >= h;
  if (right) acc = mm_tile<true>(v.A + (J + h) * nn, n, v.Z + (J + h) * nr, v.R, ti, tj, 0, n);
  if (left) acc += mm_tile<true>(v.C + (J - h) * nn, n, v.Z + (J - h) * nr, v.R, ti, tj, 0, n);
  if (right || left) mm_store(v.G + J * nr, v.R, ti, tj, acc, -1.0, true);
}

// Level h of the many-right-hand-side CR in two launches after the factor:
// (1) the eliminations A_I / C_I and Z_I = Linv_I G_I (both read only Linv_I),
// (2) the even superblocks' update of D / E / g and of G (both read A / C / Z).
__global__ __launch_bounds__(64) void k_crm_elim(CRView v, CRMView m, int h, int nel, int total) {
  const int lb = xcd_block(total);
  if (lb >= total) return;
  if (lb < nel) cr_elim_item(v, h, lb);
  else crm_fwd_item(m, h, 2 * h, lb - nel);
}
__global__ __launch_bounds__(64) void k_crm_update(CRView v, CRMView m, int h, int nup, int total) {
  const int lb = xcd_block(total);
  if (lb >= total) return;
  if (lb < nup) cr_update_item(v, h, lb);
  else crm_upd_item(m, h, lb - nup);
}

// odd I = h + 2 h q: Z_I -= A_I X_{I-h} + C_I X_{I+h} (in place, tile by tile)
__global__ __launch_bounds__(64) void k_crm_back_rhs(CRMView v, int h, int total) {
  const int lb = xcd_block(total);
  if (lb >= total) return;
  const int n = v.n, nt = n >> 4, rt = v.R >> 4, per = nt * rt;
  const int q = lb / per, t = lb - q * per, ti = t / rt, tj = t - ti * rt, I = h + 2 * h * q;
  const size_t nn = (size_t)n * n, nr = (size_t)n * v.R;
  d4 acc = mm_tile<false>(v.A + I * nn, n, v.X + (I - h) * nr, v.R, ti, tj, 0, n);
  if (I + h < v.p) acc += mm_tile<false>(v.C + I * nn, n, v.X + (I + h) * nr, v.R, ti, tj, 0, n);
  mm_store(v.Z + I * nr, v.R, ti, tj, acc, -1.0, true);
}

// X_I = Linv_I^T Z_I for I = I0 + stride q (Linv^T upper: K from the tile row)
__global__ __launch_bounds__(64) void k_crm_bwd(CRMView v, int I0, int stride, int total) {
  const int lb = xcd_block(total);
  if (lb >= total) return;
  const int nt = v.n >> 4, rt = v.R >> 4, per = nt * rt;
  const int q = lb / per, t = lb - q * per, ti = t / rt, tj = t - ti * rt, I = I0 + stride * q;
  const size_t nn = (size_t)v.n * v.n, nr = (size_t)v.n * v.R;
  const d4 acc = mm_tile<true>(v.D + I * nn, v.n, v.Z + I * nr, v.R, ti, tj, 16 * ti, v.n);
  mm_store(v.X + I * nr, v.R, ti, tj, acc, 1.0, false);
}

// P_I = A_I^T B_I for p blocks of [n][R] (R x R results, one tile per wavefront)
__global__ __launch_bounds__(64) void k_batched_atb(const double *A, const double *B, double *P, int n, int R,
                                                    int total) {
  const int lb = xcd_block(total);
  if (lb >= total) return;
  const int rt = R >> 4, per = rt * rt, I = lb / per, t = lb - I * per, ti = t / rt, tj = t - ti * rt;
  const size_t nr = (size_t)n * R;
  const d4 acc = mm_tile<true>(A + I * nr, R, B + I * nr, R, ti, tj, 0, n);
  mm_store(P + (size_t)I * R * R, R, ti, tj, acc, 1.0, false);
}

int launch_batched_atb(const double *A, const double *B, double *P, int p, int n, int R, hipStream_t st) {
  if (p <= 0 || n % 4 || R % 16) return -1;
  const int total = p * (R / 16) * (R / 16);
  hipLaunchKernelGGL(k_batched_atb, dim3(xcd_grid(total)), dim3(64), 0, st, A, B, P, n, R, total);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

__global__ __launch_bounds__(512) void k_cr_factor_at(CRView v, int I) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ int fail;
  cr_factor_store(v, I, lds, &fail);
}

// A_I = L^-1 E_{I-h}^T and C_I = L^-1 E_I for the odd superblocks of level h
// by forward substitution with the factor k_cr_aug<1, false> left in L_I (U tiles
// above the diagonal, T_k = L_kk^-1 on it): for k = 0 .. nt-1, X_k = T_k M_k,
// then M_r -= U_kr^T X_k (r > k); tiles in the MFMA accumulator layout as in
// k_cr_aug. One wavefront per 16-column strip: the levels with many odd
// superblocks (the fused kernel would need more workgroups than CUs) run the
// factor and this kernel instead.
__device__ __forceinline__ void trsm_strip(const CRView &v, int h, int I, int s) {
  const int n = v.n, nt = n >> 4, lane = threadIdx.x & 63, b = lane >> 4, i16 = lane & 15;
  const bool et = s < nt;
  const int J = et ? s : s - nt;
  if (!et && I + h >= v.p) return;
  const double *Lb = blk(v.L, I, n);
  d4 t[aug::kMaxNt];
#pragma unroll
  for (int r = 0; r < aug::kMaxNt; ++r)
    if (r < nt)
      t[r] = et ? aug::load_tile_t(blk(v.E, I - h, n), n, 16 * r, 16 * J, lane)
                : aug::load_tile(blk(v.E, I, n), n, 16 * r, 16 * J, lane);
  // step k's operands (T_k and the U_kr row) are loaded during step k-1: the
  // strip's chain waits on one memory round trip in all, not one per step
  // (same MFMAs in the same order)
  double ta[4];
  d4 u[aug::kMaxNt];
  auto load_step = [&](int k, double (&a)[4], d4 (&uu)[aug::kMaxNt]) {
#pragma unroll
    for (int m = 0; m < 4; ++m) a[m] = Lb[(size_t)(16 * k + i16) * n + 16 * k + 4 * m + b];  // T_k[i][4m+b]
#pragma unroll
    for (int r = 1; r < aug::kMaxNt; ++r)
      if (r > k && r < nt) uu[r] = aug::load_tile(Lb, n, 16 * k, 16 * r, lane);  // U_kr
  };
  load_step(0, ta, u);
#pragma unroll
  for (int k = 0; k < aug::kMaxNt; ++k) {
    if (k >= nt) break;
    double ta_n[4];
    d4 u_n[aug::kMaxNt];
    if (k + 1 < nt) load_step(k + 1, ta_n, u_n);
    d4 x = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int m = 0; m < 4; ++m) x = aug::mfma(ta[m], t[k][m], x);
    t[k] = x;
#pragma unroll
    for (int r = k + 1; r < aug::kMaxNt; ++r)
      if (r < nt) {
#pragma unroll
        for (int m = 0; m < 4; ++m) t[r] = aug::mfma(-u[r][m], t[k][m], t[r]);
      }
    if (k + 1 < nt) {
#pragma unroll
      for (int m = 0; m < 4; ++m) ta[m] = ta_n[m];
#pragma unroll
      for (int r = 1; r < aug::kMaxNt; ++r) u[r] = u_n[r];
    }
  }
  double *out = blk(et ? v.A : v.C, I, n);
#pragma unroll
  for (int r = 0; r < aug::kMaxNt; ++r)
    if (r < nt) aug::store_tile(out, n, 16 * r, 16 * J, t[r], lane);
}

__global__ __launch_bounds__(256) void k_cr_trsm(CRView v, int h, int total) {
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (gw >= total) return;
  const int nt = v.n >> 4, ob = gw / (2 * nt), s = gw - ob * 2 * nt;
  trsm_strip(v, h, h + 2 * h * ob, s);
}

// SQLM_CR_LEGACY=1: the round-2 factor (panel Cholesky + explicit Linv in LDS,
// k_cr_factor / k_cr_factor_elim / k_cr_top) instead of k_cr_aug (A/B only).
// odd superblocks x minimum split above which a level runs factor + TRSM
// instead of the fused k_cr_aug (160 and 300 / 1000 measured, profiles/r04)
constexpr int kCrAugWideWGs = 160;

inline bool cr_legacy() {
  static const bool on = std::getenv("SQLM_CR_LEGACY") != nullptr;
  return on;
}

// Factor `count` superblocks I = I0 + stride q: z_I -> g_I, and Linv_I (linv)
// or U_I with T on the diagonal (k_cr_back_u) -> L_I. Legacy: always Linv.
static void launch_cr_factor(const CRView &v, int h, int I0, int stride, int count, bool linv, hipStream_t st) {
  if (cr_legacy()) {
    const size_t lds = cr_factor_lds(v.n);
    if (stride == 0) hipLaunchKernelGGL(k_cr_factor_at, dim3(1), dim3(512), lds, st, v, I0);
    else hipLaunchKernelGGL(k_cr_factor, dim3(count), dim3(512), lds, st, v, h);
    return;
  }
  if (linv) hipLaunchKernelGGL((k_cr_aug<1, true>), dim3(count), dim3(aug::kThreads), sizeof(aug::Shared), st, v, h, I0, stride, 1);
  else hipLaunchKernelGGL((k_cr_aug<1, false>), dim3(count), dim3(aug::kThreads), sizeof(aug::Shared), st, v, h, I0, stride, 1);
}

// A level with too many odd superblocks for the fused kernel's workgroups on
// one round of CUs: the factor alone, then the strips as a wide kernel.
static bool cr_level_wide(int n_odd, int nt, bool linv) {
  return !cr_legacy() &&
         (int64_t)n_odd * aug::min_split(nt, linv, aug::extra_columns(nt, true, true)) > kCrAugWideWGs;
}

// Level h, steps 1 + 2: every odd superblock factored, A_I / C_I / z_I formed.
static void launch_cr_level(const CRView &v, int h, int n_odd, bool linv, hipStream_t st) {
  const int nt = v.n / 16;
  if (!cr_legacy()) {
    const int sp = aug_split(n_odd, nt, linv, aug::extra_columns(nt, true, true));
    if (cr_level_wide(n_odd, nt, linv)) {
      // too many odd superblocks for the fused kernel's workgroups on one
      // round of CUs: the factor alone, then the strips as a wide kernel
      launch_cr_factor(v, h, h, 2 * h, n_odd, linv, st);
      if (linv) {
        const int per = nt * nt;
        hipLaunchKernelGGL(k_cr_elim_gemm, dim3(xcd_grid(n_odd * 2 * per)), dim3(64), 0, st, v, h, n_odd * 2 * per);
      } else {
        const int total = n_odd * 2 * nt;
        hipLaunchKernelGGL(k_cr_trsm, dim3((total + 3) / 4), dim3(256), 0, st, v, h, total);
      }
      return;
    }
    if (linv)
      hipLaunchKernelGGL((k_cr_aug<0, true>), dim3(n_odd * sp), dim3(aug::kThreads), sizeof(aug::Shared), st, v, h, h, 2 * h, sp);
    else
      hipLaunchKernelGGL((k_cr_aug<0, false>), dim3(n_odd * sp), dim3(aug::kThreads), sizeof(aug::Shared), st, v, h, h, 2 * h, sp);
    return;
  }
  // legacy: the fused factor + elimination, one workgroup per odd superblock
  // from 128 of them up, several below (round 2)
  const size_t lds = cr_factor_lds(v.n);
  const int sp = n_odd >= 128 ? 1 : cr_split(n_odd, nt);
  hipLaunchKernelGGL(k_cr_factor_elim, dim3(n_odd * sp), dim3(512), lds, st, v, h, sp);
}

int launch_cr_multi(double *D, double *L, double *E, double *A, double *C, double *gs, double *xs, double *G,
                    double *Z, double *X, int *flags, int p, int n, int R, hipStream_t st) {
  if (p <= 0 || n % 16 || n > kCRMaxN || R <= 0 || R % 16) return -1;
  CRView v{p, n, 0, 0, D, E, A, C, gs, xs, flags, L};
  CRMView m{p, n, R, L, A, C, G, Z, X};
  const int nt = n / 16, per = nt * nt, upd = nt * (nt + 1) / 2 + per + nt, rhs = nt * (R / 16);
  int h = 1;
  for (; h < p; h *= 2) {
    const int n_odd = (p - h + 2 * h - 1) / (2 * h);
    const int n_even = (p + 2 * h - 1) / (2 * h);
    launch_cr_factor(v, h, h, 2 * h, n_odd, true, st);
    const int nel = n_odd * 2 * per, t1 = nel + n_odd * rhs, nup = n_even * upd, t2 = nup + n_even * rhs;
    hipLaunchKernelGGL(k_crm_elim, dim3(xcd_grid(t1)), dim3(64), 0, st, v, m, h, nel, t1);
    hipLaunchKernelGGL(k_crm_update, dim3(xcd_grid(t2)), dim3(64), 0, st, v, m, h, nup, t2);
  }
  launch_cr_factor(v, 0, 0, 0, 1, true, st);
  hipLaunchKernelGGL(k_crm_fwd, dim3(xcd_grid(rhs)), dim3(64), 0, st, m, 0, 1, rhs);
  hipLaunchKernelGGL(k_crm_bwd, dim3(xcd_grid(rhs)), dim3(64), 0, st, m, 0, 1, rhs);
  for (h /= 2; h >= 1; h /= 2) {
    const int n_odd = (p - h + 2 * h - 1) / (2 * h);
    hipLaunchKernelGGL(k_crm_back_rhs, dim3(xcd_grid(n_odd * rhs)), dim3(64), 0, st, m, h, n_odd * rhs);
    hipLaunchKernelGGL(k_crm_bwd, dim3(xcd_grid(n_odd * rhs)), dim3(64), 0, st, m, h, 2 * h, n_odd * rhs);
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

__global__ void k_cr_gather(DevProblem d, CRView v) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= 6 * v.nP) return;
  const int i = k / 6, r = k % 6, pi = d.cam_pos ? d.cam_pos[i] : i;
  double x = 0.0;
  if (pi >= 0) {
    const int I = pi / v.B, li = pi - I * v.B;
    x = v.x[(size_t)I * v.n + 6 * li + r];
  } else {
    x = d.bd_x[6 * (-1 - pi) + r];
  }
  d.dx[k] = v.flags[0] ? x : 0.0;
}

// ---- band + border ("arrow") solve of a loop-closed reduced camera system ----
// Replaces SimplicialLDLT + AMD on S (linear_solver_eigen.h:60-75,94-124) when
// loop closures couple cameras far off the band. The border cameras (a greedy
// vertex cover of the blocks farther than kBandMaxCams cameras off the
// diagonal) are ordered last, so in the permuted camera order
//   S = [ B  F^T ]   B: block-tridiagonal band (CR superblocks),
//       [ F  G   ]   F: band-border coupling, G: border block.
// With the band's cyclic reduction written as a permuted block Cholesky
// B = P L L^T P^T (L's diagonal blocks are the CR factors, its off-diagonal
// blocks the A / C eliminations), the forward sweep applied to the columns of
// F^T gives W = L^-1 P^T F^T (blocks Z_I), applied to r_b gives w (the CR's
// z_I). Then
//   (G - W^T W) x_c = r_c - W^T w          (dense border system, MFMA Cholesky)
//   x_b = P L^-T (w - W x_c)               (correct z_I, back substitution)
// which is the exact block elimination of S (same math as g2o's LDL^T, another
// elimination order). F^T is nonzero only in the few superblocks next to the
// border cameras; the forward sweep keeps that sparsity (a superblock's
// right-hand side becomes nonzero only when an eliminated neighbour's is), so
// Z is formed for O(#coupled + log p) superblocks, from host-built lists.
struct ArwView {
  int p, n, R;
  const double *D, *A, *C;  // D_I = Linv_I once factored
  double *G, *Z;            // [p][n][R]
  double *g;                // [p][n]: z_I after the forward sweep
};

// Z_I = Linv_I G_I for the superblocks I of `list`
__device__ __forceinline__ void arw_fwd_item(const ArwView &a, const int *list, int lb) {
  const int nt = a.n >> 4, rt = a.R >> 4, per = nt * rt;
  const int q = lb / per, t = lb - q * per, ti = t / rt, tj = t - ti * rt, I = list[q];
  const size_t nn = (size_t)a.n * a.n, nr = (size_t)a.n * a.R;
  const d4 acc = mm_tile<false>(a.D + I * nn, a.n, a.G + I * nr, a.R, ti, tj, 0, 16 * (ti + 1));
  mm_store(a.Z + I * nr, a.R, ti, tj, acc, 1.0, false);
}

__global__ __launch_bounds__(64) void k_arw_fwd(ArwView a, const int *list, int total) {
  const int lb = xcd_block(total);
  if (lb < total) arw_fwd_item(a, list, lb);
}

// a wide level's eliminations A_I / C_I (cr_elim_item, items [0, nel)) and the
// border right-hand sides' Z_I (the rest) in one launch: both read only Linv_I
__global__ __launch_bounds__(64) void k_arw_elim(CRView v, ArwView a, int h, int nel, const int *list, int total) {
  const int lb = xcd_block(total);
  if (lb >= total) return;
  if (lb < nel) cr_elim_item(v, h, lb);
  else arw_fwd_item(a, list, lb - nel);
}

// even J of level h: G_J = [G_J] - A_{J+h}^T Z_{J+h} - C_{J-h}^T Z_{J-h}, the
// terms present per the entry's flags (a superblock without a right-hand side
// yet starts from zero)
__device__ __forceinline__ void arw_upd_item(const ArwView &a, int h, const int *list, int lb) {
  const int n = a.n, nt = n >> 4, rt = a.R >> 4, per = nt * rt;
  const int q = lb / per, t = lb - q * per, ti = t / rt, tj = t - ti * rt;
  const int e = list[q], J = e & kUpdMask;
  const size_t nn = (size_t)n * n, nr = (size_t)n * a.R;
  d4 acc = {0.0, 0.0, 0.0, 0.0};
  if (e & kUpdRight) acc = mm_tile<true>(a.A + (J + h) * nn, n, a.Z + (J + h) * nr, a.R, ti, tj, 0, n);
  if (e & kUpdLeft) acc += mm_tile<true>(a.C + (J - h) * nn, n, a.Z + (J - h) * nr, a.R, ti, tj, 0, n);
  mm_store(a.G + J * nr, a.R, ti, tj, acc, -1.0, (e & kUpdHad) != 0);
}

// Level h, step 3 of the band (cr_update_item, items [0, ncr)) and the border
// right-hand sides' update (arw_upd_item, the rest) in one launch: both read
// only the level's eliminations A / C / Z.
__global__ __launch_bounds__(64) void k_arw_update_gemm(CRView v, ArwView a, int h, int ncr, const int *list,
                                                        int total) {
  const int lb = xcd_block(total);
  if (lb >= total) return;
  if (lb < ncr) cr_update_item(v, h, lb);
  else arw_upd_item(a, h, list, lb - ncr);
}

// Border Schur complement, lower 16x16 tiles: Ab -= sum_{I in elim} Z_I^T Z_I
// (superblocks in list order: deterministic)
__global__ __launch_bounds__(64) void k_arw_gram(ArwView a, const int *elim, int ne, double *Ab, int ldb, int total) {
  const int lb = xcd_block(total);
  if (lb >= total) return;
  int ti = 0, tj = lb;
  while (tj > ti) { tj -= ti + 1; ++ti; }
  const size_t nr = (size_t)a.n * a.R;
  d4 acc = {0.0, 0.0, 0.0, 0.0};
  for (int q = 0; q < ne; ++q) {
    const double *Z = a.Z + elim[q] * nr;
    acc += mm_tile<true>(Z, a.R, Z, a.R, ti, tj, 0, a.n);
  }
  mm_store(Ab, ldb, ti, tj, acc, -1.0, true);
}

// rb -= sum_{I in elim} Z_I^T z_I: one wavefront per 16 columns (lane: column
// r16, k-quarter k4), a superblock's n / 4 loads per lane issued before its
// FMAs, superblocks in list order, the quarters summed at the end
__global__ __launch_bounds__(64) void k_arw_gvec(ArwView a, const int *elim, int ne, double *rb) {
  const int lane = threadIdx.x, r16 = lane & 15, k4 = lane >> 4, c = 16 * blockIdx.x + r16;
  constexpr int S = kCRMaxN / 4;
  double s = 0.0;
  for (int q = 0; q < ne; ++q) {
    const int I = elim[q];
    const double *Z = a.Z + (size_t)I * a.n * a.R, *z = a.g + (size_t)I * a.n;
    double zv[S], gv[S];
#pragma unroll
    for (int t = 0; t < S; ++t) {
      const int k = 4 * t + k4, kc = k < a.n ? k : a.n - 1;
      zv[t] = Z[(size_t)kc * a.R + c];
      gv[t] = k < a.n ? z[kc] : 0.0;
    }
#pragma unroll
    for (int t = 0; t < S; ++t) s = fma(zv[t], gv[t], s);
  }
  s = k4_sum(s);
  if (k4 == 0) rb[c] -= s;
}

// z_I -= Z_I x_c for I in elim: one wavefront per row
__global__ __launch_bounds__(256) void k_arw_correct(ArwView a, const int *elim, int ne, const double *xc) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (w >= ne * a.n) return;
  const int I = elim[w / a.n], k = w % a.n;
  const double *Zr = a.Z + ((size_t)I * a.n + k) * a.R;
  double s = 0.0;
  for (int c = lane; c < a.R; c += 64) s += Zr[c] * xc[c];
  s = wave_sum_d(s);
  if (lane == 0) a.g[(size_t)I * a.n + k] -= s;
}

// x_0 = Linv_0^T z_0 (the top superblock, factored with LINV): thread (c, h)
// sums its quarter of rows m >= c of column c, the quarters added in order
__global__ __launch_bounds__(512) void k_arw_top_back(ArwView a, double *x) {
  __shared__ double part[4][kCRMaxN];
  const int n = a.n, t = threadIdx.x, c = t % kCRMaxN, h = t / kCRMaxN, q = (n + 3) / 4;
  if (h < 4 && c < n) {
    double s = 0.0;
    for (int i = 0; i < q; ++i) {
      const int m = h * q + i;
      if (m >= c && m < n) s += a.D[(size_t)m * n + c] * a.g[m];
    }
    part[h][c] = s;
  }
  __syncthreads();
  if (t < n) x[t] = ((part[0][t] + part[1][t]) + part[2][t]) + part[3][t];
}

// Border system init per trial: clear F^T in the superblocks that carry it,
// the border matrix (identity on its padding rows) and its right-hand side.
__global__ __launch_bounds__(256) void k_arw_clear(DevProblem d, const int *init, int ninit) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nr = (int64_t)d.cr_n * d.arw_R, Rp = d.arw_Rp;
  if (gid < ninit * nr) {
    const int64_t q = gid / nr, e = gid - q * nr;
    d.arw_G[(int64_t)init[q] * nr + e] = 0.0;
    return;
  }
  const int64_t g2 = gid - ninit * nr;
  if (g2 < Rp * Rp) {
    const int64_t r = g2 / Rp, c = g2 - r * Rp;
    d.bd_A[g2] = (r == c && r >= 6 * (d.nP - d.cr_nband)) ? 1.0 : 0.0;
    if (c == 0) d.bd_r[r] = 0.0;
  }
}

void launch_arrow_clear(const DevProblem &d, const CRPlan &pl, hipStream_t st) {
  const int64_t items = (int64_t)pl.init_cnt * pl.n * pl.R + (int64_t)pl.Rp * pl.Rp;
  hipLaunchKernelGGL(k_arw_clear, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, st, d,
                     pl.sched_dev + pl.init_off, pl.init_cnt);
}

// The CR levels of launch_cr_core with the sparse right-hand sides F^T carried
// along, the border system, and the back substitution.
static void launch_arrow_solve(const DevProblem &d, const CRPlan &pl, hipStream_t st) {
  const int p = pl.p, n = pl.n, R = pl.R;
  CRView v{p, n, pl.B, d.nP, d.cr_D, d.cr_E, d.cr_A, d.cr_C, d.cr_g, d.cr_x, d.flags, d.cr_L};
  ArwView a{p, n, R, d.cr_L, d.cr_A, d.cr_C, d.arw_G, d.arw_Z, d.cr_g};
  const int nt = n / 16, per = nt * nt, upd = nt * (nt + 1) / 2 + per + nt, rhs = nt * (R / 16);
  const int *S = pl.sched_dev;
  int h = 1, lv = 0;
  for (; h < p; h *= 2, ++lv) {
    const int n_odd = (p - h + 2 * h - 1) / (2 * h);
    const int n_even = (p + 2 * h - 1) / (2 * h);
    const int fo = pl.lvl[4 * lv], fc = pl.lvl[4 * lv + 1], uo = pl.lvl[4 * lv + 2], uc = pl.lvl[4 * lv + 3];
    if (cr_level_wide(n_odd, nt, true)) {  // factor, then the eliminations with Z_I in one launch
      launch_cr_factor(v, h, h, 2 * h, n_odd, true, st);
      const int nel = n_odd * 2 * per, tot = nel + fc * rhs;
      hipLaunchKernelGGL(k_arw_elim, dim3(xcd_grid(tot)), dim3(64), 0, st, v, a, h, nel, S + fo, tot);
    } else {
      launch_cr_level(v, h, n_odd, true, st);
      if (fc) hipLaunchKernelGGL(k_arw_fwd, dim3(xcd_grid(fc * rhs)), dim3(64), 0, st, a, S + fo, fc * rhs);
    }
    const int ncr = n_even * upd, tot = ncr + uc * rhs;
    hipLaunchKernelGGL(k_arw_update_gemm, dim3(xcd_grid(tot)), dim3(64), 0, st, v, a, h, ncr, S + uo, tot);
  }
  // top superblock: factor (Linv_0 into L_0, z_0 into g_0) and its Z_0
  launch_cr_factor(v, 0, 0, 0, 1, true, st);
  const int *elim = S + pl.elim_off;
  if (pl.top_active)
    hipLaunchKernelGGL(k_arw_fwd, dim3(xcd_grid(rhs)), dim3(64), 0, st, a, elim + pl.elim_cnt - 1, rhs);
  // border system (G - W^T W) x_c = r_c - W^T w
  if (pl.elim_cnt) {
    const int rt = R / 16, lt = rt * (rt + 1) / 2;
    hipLaunchKernelGGL(k_arw_gram, dim3(xcd_grid(lt)), dim3(64), 0, st, a, elim, pl.elim_cnt, d.bd_A, pl.Rp, lt);
    hipLaunchKernelGGL(k_arw_gvec, dim3(R / 16), dim3(64), 0, st, a, elim, pl.elim_cnt, d.bd_r);
  }
  // the border's last block holds R - (Rp - kCRMaxN) real rows (identity padding after them)
  launch_dense_spd_solve(d.bd_A, d.bd_L, d.bd_Linv, d.bd_r, d.bd_x, d.flags, pl.Rp, st, 0, R - (pl.Rp - kCRMaxN));
  // x_b = P L^-T (w - W x_c)
  if (pl.elim_cnt)
    hipLaunchKernelGGL(k_arw_correct, dim3((pl.elim_cnt * n + 3) / 4), dim3(256), 0, st, a, elim, pl.elim_cnt, d.bd_x);
  hipLaunchKernelGGL(k_arw_top_back, dim3(1), dim3(512), 0, st, a, d.cr_x);
  for (h /= 2; h >= 1; h /= 2) {
    const int n_odd = (p - h + 2 * h - 1) / (2 * h);
    hipLaunchKernelGGL(k_cr_back, dim3(n_odd), dim3(64 * nt), (size_t)n * sizeof(double), st, v, h);
  }
}

// Levels, top solve and back substitution on D/E/g already in CR layout.
void launch_cr_core(double *D, double *L, double *E, double *A, double *C, double *g, double *x, int *flags, int p,
                    int n, hipStream_t st, CRSync *sync) {
  CRView v{p, n, 0, 0, D, E, A, C, g, x, flags, L};
  const size_t lds = cr_factor_lds(n);
  const int nt = n / 16, per = nt * nt, upd = nt * (nt + 1) / 2 + per + nt;
  int h = 1;
  for (; h < p; h *= 2) {
    const int n_odd = (p - h + 2 * h - 1) / (2 * h);
    const int n_even = (p + 2 * h - 1) / (2 * h);
    launch_cr_level(v, h, n_odd, false, st);
    // (two waves per workgroup, a D tile's A^T A and C^T C at once: solve
    // 0.458 -> 0.473 ms, profiles/r05/ab_upd_half_lanes_cr_upd2w.log)
    hipLaunchKernelGGL(k_cr_update_gemm, dim3(xcd_grid(n_even * upd)), dim3(64), 0, st, v, h, n_even * upd);
  }
  const size_t back_lds = 3 * kCRMaxN * sizeof(double) + aug::kMaxNt * sizeof(int);
  if (cr_legacy())
    hipLaunchKernelGGL(k_cr_top, dim3(1), dim3(512), lds, st, v);
  else  // x_0 = U_0^-1 z_0 by the top factor's workgroup
    hipLaunchKernelGGL((k_cr_aug<1, false, true>), dim3(1), dim3(aug::kThreads), sizeof(aug::Shared), st, v, 0, 0, 0, 1);
  if (!cr_legacy() && p > 1 && sync && sync->done && sync->cap >= p) {  // every back level in one launch
    if (sync->epoch == INT_MAX) {  // (never in practice) restart the completion words
      (void)hipMemsetAsync(sync->done, 0, (size_t)sync->cap * sizeof(int), st);
      sync->epoch = 0;
    }
    v.done = sync->done;
    v.epoch = ++sync->epoch;
    hipLaunchKernelGGL(k_cr_back_all, dim3(p - 1), dim3(64 * nt), back_lds, st, v, h / 2);
    return;
  }
  for (h /= 2; h >= 1; h /= 2) {
    const int n_odd = (p - h + 2 * h - 1) / (2 * h);
    if (cr_legacy())
      hipLaunchKernelGGL(k_cr_back, dim3(n_odd), dim3(64 * nt), (size_t)n * sizeof(double), st, v, h);
    else
      hipLaunchKernelGGL(k_cr_back_u<false>, dim3(n_odd), dim3(64 * nt), back_lds, st, v, h);
  }
}

int launch_cr_solve(const DevProblem &d, const CRPlan &pl, hipStream_t st, bool gather, CRSync *sync) {
  CRView v{pl.p, pl.n, pl.B, d.nP, d.cr_D, d.cr_E, d.cr_A, d.cr_C, d.cr_g, d.cr_x, d.flags, d.cr_L};
  if (!d.cr_direct) {  // BSR S (sharded runs / row-kernel RCS): zero the superblocks and scatter
    const size_t blkbytes = (size_t)pl.p * pl.n * pl.n * sizeof(double);
    if (hipMemsetAsync(d.cr_D, 0, blkbytes, st) != hipSuccess) return -2;
    if (hipMemsetAsync(d.cr_E, 0, blkbytes, st) != hipSuccess) return -2;
    if (pl.R) launch_arrow_clear(d, pl, st);
    hipLaunchKernelGGL(k_cr_scatter, dim3(d.nP), dim3(64), 0, st, d, v);
  }
  if (pl.R) launch_arrow_solve(d, pl, st);
  else launch_cr_core(d.cr_D, d.cr_L, d.cr_E, d.cr_A, d.cr_C, d.cr_g, d.cr_x, d.flags, pl.p, pl.n, st, sync);
  if (gather) hipLaunchKernelGGL(k_cr_gather, dim3((6 * d.nP + 255) / 256), dim3(256), 0, st, d, v);
  return 0;
}

}  // namespace sqlm
