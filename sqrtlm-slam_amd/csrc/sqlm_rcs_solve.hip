// sqlm_rcs_solve.hip — reduced-camera-system solve S dx = g on gfx950.
//
// Replaces LinearSolverEigen (SimplicialLDLT + AMD, Thirdparty/g2o/g2o/solvers/
// linear_solver_eigen.h:94-124). The camera ordering of g2o (pose id) makes S
// block-banded for sequential trajectories: with block bandwidth bw (cameras),
// grouping B = bw+1 consecutive cameras into one "superblock" makes S block
// TRIDIAGONAL with p superblocks of n = 6B (padded to a multiple of 16) rows.
// That system is solved by block cyclic reduction (an odd-even nested
// dissection): log2(p) levels, each eliminating every other superblock in
// parallel (one workgroup per superblock), so the critical path is
// O(log p) dense block operations instead of the O(p) of a banded Cholesky.
//
// Per superblock the dense work is Cholesky + triangular inverse in LDS and
// n x n x n products on the FP64 matrix cores (v_mfma_f64_16x16x4_f64).
#include <hip/hip_runtime.h>

#include "sqlm_internal.h"

namespace sqlm {

typedef double d4 __attribute__((ext_vector_type(4)));

// C = alpha * op(A) * op(B) + beta * C, n x n row-major; lda/ldb/ldc leading
// dimensions (LDS operands use an odd stride to stay bank-conflict free).
// Any number of waves; each wave owns 16x16 output tiles. MFMA f64 16x16x4
// operand map: lane l holds A[l&15][k + (l>>4)] and B[k + (l>>4)][l&15];
// result register j holds C[(l>>4) + 4j][l&15]. All K-step operands of a tile
// are fetched before the MFMA chain so the loads overlap.
template <bool TA, bool TB, int NMAX>
__device__ void wg_gemm(double *C, int ldc, const double *A, int lda, const double *B, int ldb, int n, double alpha,
                        double beta) {
  const int nw = blockDim.x >> 6, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nt = n >> 4, r16 = lane & 15, k4 = lane >> 4;
  for (int t = wave; t < nt * nt; t += nw) {
    const int ti = t / nt, tj = t - ti * nt;
    const int ar = ti * 16 + r16, bc = tj * 16 + r16;
    double av[NMAX / 4], bv[NMAX / 4];
#pragma unroll
    for (int s = 0; s < NMAX / 4; ++s) {
      const int k = 4 * s + k4;
      if (4 * s < n) {
        av[s] = TA ? A[k * lda + ar] : A[ar * lda + k];
        bv[s] = TB ? B[bc * ldb + k] : B[k * ldb + bc];
      }
    }
    d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < NMAX / 4; ++s)
      if (4 * s < n) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s], bv[s], acc, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      double *c = C + (ti * 16 + k4 + 4 * j) * ldc + bc;
      *c = beta == 0.0 ? alpha * acc[j] : alpha * acc[j] + beta * *c;
    }
  }
}

// y = alpha * op(A) x + beta * y (n x n), one thread per output row.
template <bool TA>
__device__ void wg_gemv(double *y, const double *A, int lda, const double *x, int n, double alpha, double beta) {
  for (int r = threadIdx.x; r < n; r += blockDim.x) {
    double s = 0.0;
    for (int k = 0; k < n; ++k) s += (TA ? A[k * lda + r] : A[r * lda + k]) * x[k];
    y[r] = beta == 0.0 ? alpha * s : alpha * s + beta * y[r];
  }
}

// ---- 16x16 diagonal-block helpers (one wavefront) -------------------------

// Cholesky of the 16x16 block at (c0, c0) of the LDS matrix L (row r held by
// lane r in registers), written back lower-triangular.
__device__ void diag_potrf16(double *L, int ld, int c0, int *fail) {
  const int lane = threadIdx.x & 63, r = lane & 15;
  double row[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) row[j] = L[(c0 + r) * ld + c0 + j];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const double piv = __shfl(row[k], k, 64);
    if (lane == 0 && !(piv > 0.0)) *fail = 1;
    const double lkk = piv > 0.0 ? sqrt(piv) : 1.0;
    if (r == k) row[k] = lkk;
    if (r > k) row[k] /= lkk;
    const double lk = row[k];
#pragma unroll
    for (int j = k + 1; j < 16; ++j) {
      const double ljk = __shfl(row[k], j, 64);
      if (r >= j) row[j] -= lk * ljk;
    }
  }
  if (lane < 16) {
#pragma unroll
    for (int j = 0; j < 16; ++j) L[(c0 + r) * ld + c0 + j] = j <= r ? row[j] : 0.0;
  }
}

// X = inverse of the lower-triangular 16x16 block at (c0, c0) of L; lane c
// owns column c of X (forward substitution, L rows read as LDS broadcasts).
__device__ void diag_trtri16(const double *L, int ld, int c0, double *X /*16x16*/) {
  const int lane = threadIdx.x & 63, c = lane & 15;
  double x[16];
#pragma unroll
  for (int rr = 0; rr < 16; ++rr) {
    const double *lr = L + (c0 + rr) * ld + c0;
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < rr; ++k) s += lr[k] * x[k];
    const double inv = 1.0 / lr[rr];
    x[rr] = rr == c ? inv : (rr > c ? -s * inv : 0.0);
  }
  if (lane < 16) {
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) X[rr * 16 + c] = x[rr];
  }
}

// In-LDS blocked Cholesky L L^T = A (lower, n = 16 nt, odd leading dim ld),
// then L <- L^-1 in place (LAPACK dtrtri lower-blocked order). Diagonal
// 16x16 blocks are factored / inverted by one wavefront in registers; panel
// solves, trailing SYRK updates and the off-diagonal inverse products run on
// the FP64 matrix cores. Dinv: [nt][16][16] LDS scratch, W: [n][16] scratch.
// Returns false (for every thread) if a pivot is not positive.
__device__ bool wg_potrf_trtri(double *L, int ld, int n, double *Dinv, double *W, int *fail) {
  const int tid = threadIdx.x, nw = blockDim.x >> 6, wave = tid >> 6, lane = tid & 63;
  const int r16 = lane & 15, k4 = lane >> 4, nt = n >> 4;
  if (tid == 0) *fail = 0;
  __syncthreads();
  for (int kb = 0; kb < nt; ++kb) {
    const int c0 = 16 * kb;
    if (wave == 0) {
      diag_potrf16(L, ld, c0, fail);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      diag_trtri16(L, ld, c0, Dinv + kb * 256);
    }
    __syncthreads();
    // panel: L[ib][kb] = A[ib][kb] * Dinv_kb^T  (ib > kb)
    for (int ib = kb + 1 + wave; ib < nt; ib += nw) {
      double a[4], b[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        a[s] = L[(16 * ib + r16) * ld + c0 + 4 * s + k4];
        b[s] = Dinv[kb * 256 + r16 * 16 + 4 * s + k4];  // B[k][col] = Dinv[col][k]
      }
      d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[s], acc, 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) L[(16 * ib + k4 + 4 * j) * ld + c0 + r16] = acc[j];
    }
    __syncthreads();
    // trailing SYRK: L[ib][jb] -= L[ib][kb] L[jb][kb]^T, kb < jb <= ib
    const int m = nt - kb - 1, ntile = m * (m + 1) / 2;
    for (int q = wave; q < ntile; q += nw) {
      int ib = 0, rem = q;
      while (rem > ib) { rem -= ib + 1; ++ib; }
      const int jb = rem;  // 0 <= jb <= ib within the trailing matrix
      const int I = kb + 1 + ib, J = kb + 1 + jb;
      double a[4], b[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        a[s] = -L[(16 * I + r16) * ld + c0 + 4 * s + k4];
        b[s] = L[(16 * J + r16) * ld + c0 + 4 * s + k4];
      }
      d4 acc;
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = L[(16 * I + k4 + 4 * j) * ld + 16 * J + r16];
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[s], acc, 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) L[(16 * I + k4 + 4 * j) * ld + 16 * J + r16] = acc[j];
    }
    __syncthreads();
  }
  for (int idx = tid; idx < n * n; idx += blockDim.x) {  // strict upper triangle -> 0
    const int i = idx / n, j = idx - i * n;
    if (j > i) L[i * ld + j] = 0.0;
  }
  __syncthreads();
  // inverse: for jb from last to first, Linv21 = -(Linv22 L21) Dinv_jb, Linv11 = Dinv_jb
  for (int jb = nt - 1; jb >= 0; --jb) {
    const int c0 = 16 * jb;
    for (int ib = jb + 1 + wave; ib < nt; ib += nw) {  // W[ib] = sum_{kb=jb+1..ib} Linv[ib][kb] L[kb][jb]
      d4 acc = {0.0, 0.0, 0.0, 0.0};
      for (int kb = jb + 1; kb <= ib; ++kb) {
        double a[4], b[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          a[s] = L[(16 * ib + r16) * ld + 16 * kb + 4 * s + k4];
          b[s] = L[(16 * kb + 4 * s + k4) * ld + c0 + r16];
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[s], acc, 0, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) W[(16 * ib + k4 + 4 * j) * 16 + r16] = acc[j];
    }
    __syncthreads();
    for (int ib = jb + 1 + wave; ib < nt; ib += nw) {  // L[ib][jb] = -W[ib] Dinv_jb
      double a[4], b[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        a[s] = -W[(16 * ib + r16) * 16 + 4 * s + k4];
        b[s] = Dinv[jb * 256 + (4 * s + k4) * 16 + r16];
      }
      d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[s], acc, 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) L[(16 * ib + k4 + 4 * j) * ld + c0 + r16] = acc[j];
    }
    for (int e = tid; e < 256; e += blockDim.x) L[(c0 + e / 16) * ld + c0 + e % 16] = Dinv[jb * 256 + e];
    __syncthreads();
  }
  return *fail == 0;
}

struct CRView {
  int p, n, B, nP;
  double *D, *E, *A, *C, *g, *x;  // [p][n][n] x4, [p][n] x2
  int *flags;
};

__device__ __forceinline__ double *blk(double *base, int I, int n) { return base + (size_t)I * n * n; }

// BSR (upper, 6x6 blocks) -> superblock D_I (symmetric) and E_I = S(I, I+1); g -> g_I.
__global__ __launch_bounds__(256) void k_cr_scatter(DevProblem d, CRView v) {
  const int i = blockIdx.x;  // free camera
  const int I = i / v.B, li = i - I * v.B, n = v.n;
  for (int s = d.s_row_ptr[i]; s < d.s_row_ptr[i + 1]; ++s) {
    const int j = d.s_col[s];
    const int J = j / v.B, lj = j - J * v.B;
    for (int e = threadIdx.x; e < 36; e += blockDim.x) {
      const int r = e / 6, c = e % 6;
      const double val = d.S[(size_t)s * 36 + e];
      if (J == I) {
        blk(v.D, I, n)[(6 * li + r) * n + 6 * lj + c] = val;
        if (j != i) blk(v.D, I, n)[(6 * lj + c) * n + 6 * li + r] = val;
      } else {  // J == I + 1 (block tridiagonal by construction)
        blk(v.E, I, n)[(6 * li + r) * n + 6 * lj + c] = val;
      }
    }
  }
  if (threadIdx.x < 6) v.g[(size_t)I * n + 6 * li + threadIdx.x] = d.g[6 * i + threadIdx.x];
  // identity on padded rows (cameras past nP in the last superblock, rows >= 6B)
  if (li == 0) {
    for (int r = 6 * v.B + threadIdx.x; r < n; r += blockDim.x) blk(v.D, I, n)[r * n + r] = 1.0;
    if (I == v.p - 1) {
      const int used = v.nP - I * v.B;
      for (int r = 6 * used + threadIdx.x; r < 6 * v.B; r += blockDim.x) blk(v.D, I, n)[r * n + r] = 1.0;
    }
  }
  if (i == 0 && threadIdx.x == 0) v.flags[0] = 1;
}

// Level h, step 1: every odd superblock I (I = h, 3h, 5h, ...) is factored:
// D_I <- Linv_I = chol(D_I)^-1 (in place), g_I <- z_I = Linv_I g_I.
__global__ __launch_bounds__(512) void k_cr_factor(CRView v, int h) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ int fail;
  const int I = h + 2 * h * blockIdx.x, n = v.n, ld = n + 1;
  double *L = lds, *tmp = lds + n * ld, *Dinv = tmp + 2 * n, *W = Dinv + 16 * n;
  double *Dg = blk(v.D, I, n);
  for (int k = threadIdx.x; k < n * n; k += blockDim.x) L[(k / n) * ld + k % n] = Dg[k];
  for (int k = threadIdx.x; k < n; k += blockDim.x) tmp[k] = v.g[(size_t)I * n + k];
  __syncthreads();
  if (!wg_potrf_trtri(L, ld, n, Dinv, W, &fail) && threadIdx.x == 0) v.flags[0] = 0;
  for (int k = threadIdx.x; k < n * n; k += blockDim.x) Dg[k] = L[(k / n) * ld + k % n];
  wg_gemv<false>(v.g + (size_t)I * n, L, ld, tmp, n, 1.0, 0.0);
}

// One wavefront computes one 16x16 tile C[ti][tj] (+)= alpha * op(A) op(B) over K = n,
// skipping K blocks that are zero because A is lower triangular (LA) or
// A^T is upper triangular... (lower-triangular A used un-transposed only).
template <bool TA, bool TB, bool LA>
__device__ __forceinline__ d4 tile_gemm(const double *A, const double *B, int n, int ti, int tj) {
  const int lane = threadIdx.x & 63, r16 = lane & 15, k4 = lane >> 4;
  const int ar = ti * 16 + r16, bc = tj * 16 + r16;
  const int kend = LA ? 16 * (ti + 1) : n;
  double av[kCRMaxN / 4], bv[kCRMaxN / 4];
#pragma unroll
  for (int s = 0; s < kCRMaxN / 4; ++s) {
    const int k = 4 * s + k4;
    if (4 * s < kend) {
      av[s] = TA ? A[k * n + ar] : A[ar * n + k];
      bv[s] = TB ? B[bc * n + k] : B[k * n + bc];
    }
  }
  d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int s = 0; s < kCRMaxN / 4; ++s)
    if (4 * s < kend) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s], bv[s], acc, 0, 0, 0);
  return acc;
}

__device__ __forceinline__ void tile_store(double *C, int n, int ti, int tj, const d4 &acc, double alpha,
                                           bool accumulate) {
  const int lane = threadIdx.x & 63, r16 = lane & 15, k4 = lane >> 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double *c = C + (ti * 16 + k4 + 4 * j) * n + tj * 16 + r16;
    *c = accumulate ? *c + alpha * acc[j] : alpha * acc[j];
  }
}

// Level h, step 2: A_I = Linv_I S(I, I-h) = Linv_I E_{I-h}^T and
// C_I = Linv_I S(I, I+h) = Linv_I E_I, one 16x16 tile per wavefront.
__global__ __launch_bounds__(64) void k_cr_elim_gemm(CRView v, int h) {
  const int n = v.n, nt = n >> 4, per = nt * nt;
  const int odd = blockIdx.x / (2 * per), rem = blockIdx.x - odd * 2 * per;
  const int which = rem / per, t = rem - which * per, ti = t / nt, tj = t - ti * nt;
  const int I = h + 2 * h * odd;
  if (which == 0) {
    const d4 acc = tile_gemm<false, true, true>(blk(v.D, I, n), blk(v.E, I - h, n), n, ti, tj);
    tile_store(blk(v.A, I, n), n, ti, tj, acc, 1.0, false);
  } else if (I + h < v.p) {
    const d4 acc = tile_gemm<false, false, true>(blk(v.D, I, n), blk(v.E, I, n), n, ti, tj);
    tile_store(blk(v.C, I, n), n, ti, tj, acc, 1.0, false);
  }
}

// Level h, step 3: every even superblock J absorbs its eliminated neighbours:
// D_J -= A_{J+h}^T A_{J+h} + C_{J-h}^T C_{J-h};  E_J = -A_{J+h}^T C_{J+h};
// g_J -= A_{J+h}^T z_{J+h} + C_{J-h}^T z_{J-h}. One wavefront per output tile
// (plus one per block for g).
__global__ __launch_bounds__(64) void k_cr_update_gemm(CRView v, int h) {
  const int n = v.n, nt = n >> 4, per = nt * nt;
  const int ev = blockIdx.x / (2 * per + 1), rem = blockIdx.x - ev * (2 * per + 1);
  const int J = 2 * h * ev;
  const bool right = J + h < v.p, left = J >= h;
  if (rem == 2 * per) {  // right-hand side
    double *gj = v.g + (size_t)J * n;
    for (int r = threadIdx.x; r < n; r += 64) {
      double s = gj[r];
      if (right) {
        const double *A = blk(v.A, J + h, n), *z = v.g + (size_t)(J + h) * n;
        for (int k = 0; k < n; ++k) s -= A[k * n + r] * z[k];
      }
      if (left) {
        const double *C = blk(v.C, J - h, n), *z = v.g + (size_t)(J - h) * n;
        for (int k = 0; k < n; ++k) s -= C[k * n + r] * z[k];
      }
      gj[r] = s;
    }
    return;
  }
  const int which = rem / per, t = rem - which * per, ti = t / nt, tj = t - ti * nt;
  if (which == 0) {
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    if (right) acc = tile_gemm<true, false, false>(blk(v.A, J + h, n), blk(v.A, J + h, n), n, ti, tj);
    if (left) {
      const d4 a2 = tile_gemm<true, false, false>(blk(v.C, J - h, n), blk(v.C, J - h, n), n, ti, tj);
      acc += a2;
    }
    if (right || left) tile_store(blk(v.D, J, n), n, ti, tj, acc, -1.0, true);
  } else if (right && J + 2 * h < v.p) {
    const d4 acc = tile_gemm<true, false, false>(blk(v.A, J + h, n), blk(v.C, J + h, n), n, ti, tj);
    tile_store(blk(v.E, J, n), n, ti, tj, acc, -1.0, false);
  }
}

// Last remaining superblock 0: x_0 = D_0^-1 g_0.
__global__ __launch_bounds__(512) void k_cr_top(CRView v) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ int fail;
  const int n = v.n, ld = n + 1;
  double *L = lds, *tmp = lds + n * ld, *Dinv = tmp + 2 * n, *W = Dinv + 16 * n;
  for (int k = threadIdx.x; k < n * n; k += blockDim.x) L[(k / n) * ld + k % n] = v.D[k];
  __syncthreads();
  if (!wg_potrf_trtri(L, ld, n, Dinv, W, &fail) && threadIdx.x == 0) v.flags[0] = 0;
  for (int k = threadIdx.x; k < n; k += blockDim.x) tmp[k] = v.g[k];
  __syncthreads();
  double *z = tmp + n;
  wg_gemv<false>(z, L, ld, tmp, n, 1.0, 0.0);
  __syncthreads();
  wg_gemv<true>(v.x, L, ld, z, n, 1.0, 0.0);
}

// Back substitution at level h: x_I = Linv_I^T (z_I - A_I x_{I-h} - C_I x_{I+h}).
__global__ __launch_bounds__(256) void k_cr_back(CRView v, int h) {
  extern __shared__ __attribute__((aligned(16))) double t[];
  const int I = h + 2 * h * blockIdx.x, n = v.n;
  for (int k = threadIdx.x; k < n; k += blockDim.x) t[k] = v.g[(size_t)I * n + k];
  __syncthreads();
  wg_gemv<false>(t, blk(v.A, I, n), n, v.x + (size_t)(I - h) * n, n, -1.0, 1.0);
  __syncthreads();
  if (I + h < v.p) wg_gemv<false>(t, blk(v.C, I, n), n, v.x + (size_t)(I + h) * n, n, -1.0, 1.0);
  __syncthreads();
  wg_gemv<true>(v.x + (size_t)I * n, blk(v.D, I, n), n, t, n, 1.0, 0.0);
}

__global__ void k_cr_gather(DevProblem d, CRView v) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= 6 * v.nP) return;
  const int i = k / 6, r = k % 6, I = i / v.B, li = i - I * v.B;
  d.dx[k] = v.flags[0] ? v.x[(size_t)I * v.n + 6 * li + r] : 0.0;
}

int launch_cr_solve(const DevProblem &d, const CRPlan &pl, hipStream_t st) {
  CRView v{pl.p, pl.n, pl.B, d.nP, d.cr_D, d.cr_E, d.cr_A, d.cr_C, d.cr_g, d.cr_x, d.flags};
  const size_t blkbytes = (size_t)pl.p * pl.n * pl.n * sizeof(double);
  if (hipMemsetAsync(d.cr_D, 0, blkbytes, st) != hipSuccess) return -2;
  if (hipMemsetAsync(d.cr_E, 0, blkbytes, st) != hipSuccess) return -2;
  hipLaunchKernelGGL(k_cr_scatter, dim3(d.nP), dim3(64), 0, st, d, v);
  // L (n x (n+1)) + tmp (2n) + Dinv (nt x 256 = 16n) + W (16n)
  const size_t lds = ((size_t)pl.n * (pl.n + 1) + 2 * pl.n + 32 * (size_t)pl.n) * sizeof(double);
  int h = 1;
  for (; h < pl.p; h *= 2) {
    const int n_odd = (pl.p - h + 2 * h - 1) / (2 * h);
    const int n_even = (pl.p + 2 * h - 1) / (2 * h);
    const int per = (pl.n / 16) * (pl.n / 16);
    hipLaunchKernelGGL(k_cr_factor, dim3(n_odd), dim3(512), lds, st, v, h);
    hipLaunchKernelGGL(k_cr_elim_gemm, dim3(n_odd * 2 * per), dim3(64), 0, st, v, h);
    hipLaunchKernelGGL(k_cr_update_gemm, dim3(n_even * (2 * per + 1)), dim3(64), 0, st, v, h);
  }
  hipLaunchKernelGGL(k_cr_top, dim3(1), dim3(512), lds, st, v);
  for (h /= 2; h >= 1; h /= 2) {
    const int n_odd = (pl.p - h + 2 * h - 1) / (2 * h);
    hipLaunchKernelGGL(k_cr_back, dim3(n_odd), dim3(256), (size_t)pl.n * sizeof(double), st, v, h);
  }
  hipLaunchKernelGGL(k_cr_gather, dim3((6 * d.nP + 255) / 256), dim3(256), 0, st, d, v);
  return 0;
}

}  // namespace sqlm
