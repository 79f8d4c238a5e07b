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

// C = alpha * op(A) * op(B) + beta * C, all n x n row-major (ld = n), n % 16 == 0.
// Workgroup of 256 threads (4 waves); each wave owns 16x16 output tiles.
// MFMA f64 16x16x4 operand map: lane l holds A[l&15][k + (l>>4)] and
// B[k + (l>>4)][l&15]; result register j holds C[(l>>4) + 4j][l&15].
template <bool TA, bool TB>
__device__ void wg_gemm(double *C, const double *A, const double *B, int n, double alpha, double beta) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nt = n >> 4, r16 = lane & 15, k4 = lane >> 4;
  for (int t = wave; t < nt * nt; t += 4) {
    const int ti = t / nt, tj = t - ti * nt;
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    const int ar = ti * 16 + r16, bc = tj * 16 + r16;

    for (int kk = 0; kk < n; kk += 4) {
      const int k = kk + k4;
      const double a = TA ? A[k * n + ar] : A[ar * n + k];
      const double b = TB ? B[bc * n + k] : B[k * n + bc];
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = ti * 16 + k4 + 4 * j;
      double *c = C + row * n + bc;
      *c = beta == 0.0 ? alpha * acc[j] : alpha * acc[j] + beta * *c;
    }
  }
}

// y = alpha * op(A) x + beta * y (n x n), one thread per output row.
template <bool TA>
__device__ void wg_gemv(double *y, const double *A, const double *x, int n, double alpha, double beta) {
  for (int r = threadIdx.x; r < n; r += blockDim.x) {
    double s = 0.0;
    for (int k = 0; k < n; ++k) s += (TA ? A[k * n + r] : A[r * n + k]) * x[k];
    y[r] = beta == 0.0 ? alpha * s : alpha * s + beta * y[r];
  }
}

// In-LDS Cholesky L L^T = A (lower, in place), then L <- L^-1 (LAPACK trti2
// order). Returns false (for every thread) if a pivot is not positive.
__device__ bool wg_potrf_trtri(double *L, double *tmp, int n, int *fail) {
  const int tid = threadIdx.x;
  if (tid == 0) *fail = 0;
  __syncthreads();
  for (int k = 0; k < n; ++k) {
    if (tid == 0) {
      const double d = L[k * n + k];
      if (!(d > 0.0)) *fail = 1;
      L[k * n + k] = d > 0.0 ? sqrt(d) : 1.0;
    }
    __syncthreads();
    const double lkk = L[k * n + k];
    for (int i = k + 1 + tid; i < n; i += blockDim.x) L[i * n + k] /= lkk;
    __syncthreads();
    const int m = n - k - 1;
    for (int idx = tid; idx < m * m; idx += blockDim.x) {
      const int i = k + 1 + idx / m, j = k + 1 + idx % m;
      if (j <= i) L[i * n + j] -= L[i * n + k] * L[j * n + k];
    }
    __syncthreads();
  }
  for (int idx = tid; idx < n * n; idx += blockDim.x) {
    const int i = idx / n, j = idx % n;
    if (j > i) L[idx] = 0.0;
  }
  __syncthreads();
  for (int j = n - 1; j >= 0; --j) {
    if (tid == 0) L[j * n + j] = 1.0 / L[j * n + j];
    const int m = n - j - 1;
    for (int i = tid; i < m; i += blockDim.x) tmp[i] = L[(j + 1 + i) * n + j];
    __syncthreads();
    const double ajj = -L[j * n + j];
    for (int i = tid; i < m; i += blockDim.x) {
      double s = 0.0;
      const double *row = L + (j + 1 + i) * n + (j + 1);
      for (int k = 0; k <= i; ++k) s += row[k] * tmp[k];
      L[(j + 1 + i) * n + j] = ajj * s;
    }
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

// Level h: every odd superblock I (I = h, 3h, 5h, ...) is eliminated:
// Linv = chol(D_I)^-1, A_I = Linv S(I, I-h), C_I = Linv S(I, I+h), z_I = Linv g_I.
__global__ __launch_bounds__(256) void k_cr_elim(CRView v, int h) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ int fail;
  const int I = h + 2 * h * blockIdx.x, n = v.n;
  double *L = lds, *tmp = lds + n * n;
  double *Dg = blk(v.D, I, n);
  for (int k = threadIdx.x; k < n * n; k += blockDim.x) L[k] = Dg[k];
  __syncthreads();
  if (!wg_potrf_trtri(L, tmp, n, &fail) && threadIdx.x == 0) v.flags[0] = 0;
  for (int k = threadIdx.x; k < n * n; k += blockDim.x) Dg[k] = L[k];
  // S(I, I-h) = E_{I-h}^T
  wg_gemm<false, true>(blk(v.A, I, n), L, blk(v.E, I - h, n), n, 1.0, 0.0);
  if (I + h < v.p) wg_gemm<false, false>(blk(v.C, I, n), L, blk(v.E, I, n), n, 1.0, 0.0);
  __syncthreads();
  for (int k = threadIdx.x; k < n; k += blockDim.x) tmp[k] = v.g[(size_t)I * n + k];
  __syncthreads();
  wg_gemv<false>(v.g + (size_t)I * n, L, tmp, n, 1.0, 0.0);
}

// Level h: every even superblock J absorbs its eliminated neighbours:
// D_J -= A_{J+h}^T A_{J+h} + C_{J-h}^T C_{J-h};  E_J = -A_{J+h}^T C_{J+h};
// g_J -= A_{J+h}^T z_{J+h} + C_{J-h}^T z_{J-h}.
__global__ __launch_bounds__(256) void k_cr_update(CRView v, int h) {
  const int J = 2 * h * blockIdx.x, n = v.n;
  double *Dj = blk(v.D, J, n);
  const bool right = J + h < v.p, left = J >= h;
  if (right) wg_gemm<true, false>(Dj, blk(v.A, J + h, n), blk(v.A, J + h, n), n, -1.0, 1.0);
  __syncthreads();
  if (left) wg_gemm<true, false>(Dj, blk(v.C, J - h, n), blk(v.C, J - h, n), n, -1.0, 1.0);
  if (right && J + 2 * h < v.p) wg_gemm<true, false>(blk(v.E, J, n), blk(v.A, J + h, n), blk(v.C, J + h, n), n, -1.0, 0.0);
  double *gj = v.g + (size_t)J * n;
  if (right) wg_gemv<true>(gj, blk(v.A, J + h, n), v.g + (size_t)(J + h) * n, n, -1.0, 1.0);
  __syncthreads();
  if (left) wg_gemv<true>(gj, blk(v.C, J - h, n), v.g + (size_t)(J - h) * n, n, -1.0, 1.0);
}

// Last remaining superblock 0: x_0 = D_0^-1 g_0.
__global__ __launch_bounds__(256) void k_cr_top(CRView v) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ int fail;
  const int n = v.n;
  double *L = lds, *tmp = lds + n * n;
  for (int k = threadIdx.x; k < n * n; k += blockDim.x) L[k] = v.D[k];
  __syncthreads();
  if (!wg_potrf_trtri(L, tmp, n, &fail) && threadIdx.x == 0) v.flags[0] = 0;
  for (int k = threadIdx.x; k < n; k += blockDim.x) tmp[k] = v.g[k];
  __syncthreads();
  double *z = tmp + n;
  wg_gemv<false>(z, L, tmp, n, 1.0, 0.0);
  __syncthreads();
  wg_gemv<true>(v.x, L, z, n, 1.0, 0.0);
}

// Back substitution at level h: x_I = Linv_I^T (z_I - A_I x_{I-h} - C_I x_{I+h}).
__global__ __launch_bounds__(256) void k_cr_back(CRView v, int h) {
  extern __shared__ __attribute__((aligned(16))) double t[];
  const int I = h + 2 * h * blockIdx.x, n = v.n;
  for (int k = threadIdx.x; k < n; k += blockDim.x) t[k] = v.g[(size_t)I * n + k];
  __syncthreads();
  wg_gemv<false>(t, blk(v.A, I, n), v.x + (size_t)(I - h) * n, n, -1.0, 1.0);
  __syncthreads();
  if (I + h < v.p) wg_gemv<false>(t, blk(v.C, I, n), v.x + (size_t)(I + h) * n, n, -1.0, 1.0);
  __syncthreads();
  wg_gemv<true>(v.x + (size_t)I * n, blk(v.D, I, n), t, n, 1.0, 0.0);
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
  const size_t lds = ((size_t)pl.n * pl.n + 2 * pl.n) * sizeof(double);
  int h = 1;
  for (; h < pl.p; h *= 2) {
    const int n_odd = (pl.p - h + 2 * h - 1) / (2 * h);
    const int n_even = (pl.p + 2 * h - 1) / (2 * h);
    hipLaunchKernelGGL(k_cr_elim, dim3(n_odd), dim3(256), lds, st, v, h);
    hipLaunchKernelGGL(k_cr_update, dim3(n_even), dim3(256), 0, st, v, h);
  }
  hipLaunchKernelGGL(k_cr_top, dim3(1), dim3(256), lds, st, v);
  for (h /= 2; h >= 1; h /= 2) {
    const int n_odd = (pl.p - h + 2 * h - 1) / (2 * h);
    hipLaunchKernelGGL(k_cr_back, dim3(n_odd), dim3(256), (size_t)pl.n * sizeof(double), st, v, h);
  }
  hipLaunchKernelGGL(k_cr_gather, dim3((6 * d.nP + 255) / 256), dim3(256), 0, st, d, v);
  return 0;
}

}  // namespace sqlm
