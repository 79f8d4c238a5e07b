// sqlm_eg.hip — essential-graph optimisation on the GPU:
// g2oOptimizer::OptimizeEssentialGraph (src/backend/g2oOptimizer.cc:1212-1534)
// = LM over VertexSim3Expmap vertices and EdgeSim3 edges with numeric
// Jacobians, BlockSolver_7_3 without landmarks (the full 7n system).
//
// Per LM iteration: k_eg_errors (one thread per edge), k_eg_linearize (one
// wavefront per edge: 28 perturbed error evaluations in parallel lanes, the
// central-difference Jacobians and the edge's H / b blocks), k_eg_assemble
// (one wavefront per destination block, contributions summed in edge-id order
// like g2o's buildSystem). Per trial: damped copy, the dense blocked Cholesky
// of sqlm_rcs_solve.hip, the Sim3 update, the trial errors and the reductions.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <map>
#include <vector>

#include "../../include/sqrtlm.h"
#include "sim3_dev.h"
#include "sqlm_internal.h"

namespace sqlm {

namespace {

constexpr int kEGBlock = 256;
constexpr int kEGMaxParts = 8192;  // per partial region

struct EGDev {
  int nK = 0, nP = 0, n = 0, n_pad = 0, fix_scale = 0;
  // vertex slots: band vertices in slots [0, band_slots), border vertices in
  // [border0, border0 + border_slots); rows 7 slot .. 7 slot + 6; other rows
  // are padding (identity in A, zero in b and x)
  int band_slots = 0, border0 = 0, border_slots = 0;
  int64_t nE = 0;                       // active edges
  const int *act = nullptr;             // [nE] edge id
  const int *ei = nullptr, *ej = nullptr;  // [nE] vertex ids
  const int *hid = nullptr;             // [nK] free hidx or -1
  const double *C = nullptr;            // [nE][8]
  const double *info = nullptr;         // [nE][49] or null (identity)
  double *err = nullptr;                // [nE][7]
  double *jt = nullptr;                 // [nE][161]: Hii Hjj Hij (49 each), bi bj (7 each)
  double *H0 = nullptr;                 // [n_pad][n_pad] assembled (lower); dense / arrow-Cholesky path
  // cyclic-reduction path: the assembled lower system straight in block form
  // (no dense buffer): D0 [p][112][112] diagonal band blocks, E0 [p][112][112]
  // block (I+1, I), F0 [nb][112 p] border rows x band columns, B0 [nb][nb]
  int cr = 0, cr_p = 0, cr_nb = 0;
  double *D0 = nullptr, *E0 = nullptr, *F0 = nullptr, *B0 = nullptr;
  double *b = nullptr;                  // [n_pad]
  const int *dst = nullptr;             // [nD] destination: block row << 16 | block col, or -(v+1) for b_v
  const int *src_ptr = nullptr;         // [nD+1]
  const int *src = nullptr;             // (edge slot) << 2 | kind: 0 Hii, 1 Hjj, 2 Hij, 3 Hij^T; b: side in kind
  double *partials = nullptr;           // 3 regions of kEGMaxParts
  double *scalars = nullptr;            // chi_cur, chi_new, scale, maxdiag, ok
};

__device__ __forceinline__ bool row_valid(const EGDev &d, int r) {
  return r < 7 * d.band_slots || (r >= 7 * d.border0 && r < 7 * (d.border0 + d.border_slots));
}

// Entry (R, C), R >= C block-wise (the assembled lower part), of the system.
__device__ __forceinline__ double *h0_at(const EGDev &d, int R, int C) {
  if (!d.cr) return d.H0 + (size_t)R * d.n_pad + C;
  constexpr int n = kCRMaxN;
  const int vb = 7 * d.band_slots, b0 = 7 * d.border0;
  if (R < vb) {  // band row, band column in the same or the previous block
    const int I = R / n, J = C / n;
    double *blk = (I == J ? d.D0 + (size_t)I * n * n : d.E0 + (size_t)J * n * n);
    return blk + (size_t)(R - I * n) * n + (C - J * n);
  }
  const int k = R - b0;
  return C < vb ? d.F0 + (size_t)k * d.cr_p * n + C : d.B0 + (size_t)k * d.cr_nb + (C - b0);
}

__device__ __forceinline__ double info_at(const EGDev &d, int64_t k, int r, int c) {
  return d.info ? d.info[49 * k + 7 * r + c] : (r == c ? 1.0 : 0.0);
}

__device__ __forceinline__ void eg_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ double eg_block_sum(double v, double *red) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double r = 0.0;
  if (threadIdx.x == 0)
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) r += red[i];
  return r;
}

// EdgeSim3::computeError for every active edge at state S; chi2 = e^T Omega e.
__global__ __launch_bounds__(kEGBlock) void k_eg_errors(EGDev d, const double *__restrict__ S, int region) {
  __shared__ double red[kEGBlock / 64];
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double chi = 0.0;
  if (k < d.nE) {
    double e[7];
    eg_edge_error(S + 8 * d.ei[k], S + 8 * d.ej[k], d.C + 8 * k, e);
#pragma unroll
    for (int r = 0; r < 7; ++r) d.err[7 * k + r] = e[r];
#pragma unroll
    for (int r = 0; r < 7; ++r) {
      double oe = 0.0;
#pragma unroll
      for (int s = 0; s < 7; ++s) oe += info_at(d, k, r, s) * e[s];
      chi += e[r] * oe;
    }
  }
  const double s = eg_block_sum(chi, red);
  if (threadIdx.x == 0) d.partials[region * kEGMaxParts + blockIdx.x] = s;
}

// One wavefront per edge. Lanes 0..27: side = l / 14, dimension d = (l % 14) / 2,
// sign + / - for even / odd l; each applies its perturbation through oplus
// and evaluates the edge error. The Jacobian columns are (e+ - e-) / (2 delta)
// (base_binary_edge.hpp:131-205), then the quadratic form of
// BaseBinaryEdge::constructQuadraticForm (:55-120): H_ii += A^T O A,
// H_jj += B^T O B, H_ij += (A^T O) B, b_i += A^T (-O e), b_j += B^T (-O e).
__global__ __launch_bounds__(256) void k_eg_linearize(EGDev d, const double *__restrict__ S) {
  __shared__ double ers[4][28][7];
  __shared__ double J[4][2][49];  // row-major [r][c]
  __shared__ double AtO[4][2][49];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t k = (int64_t)blockIdx.x * 4 + w;
  const bool valid = k < d.nE;
  int vi = 0, vj = 0;
  bool free_i = false, free_j = false;
  if (valid) {
    vi = d.ei[k];
    vj = d.ej[k];
    free_i = d.hid[vi] >= 0;
    free_j = d.hid[vj] >= 0;
  }
  if (valid && lane < 28) {
    const int side = lane / 14, dim = (lane % 14) >> 1;
    const bool minus = lane & 1;
    if (side == 0 ? free_i : free_j) {
      double Si[8], Sj[8], add[7] = {0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int c = 0; c < 8; ++c) { Si[c] = S[8 * vi + c]; Sj[c] = S[8 * vj + c]; }
      add[dim] = minus ? -1e-9 : 1e-9;
      sim3_oplus(side == 0 ? Si : Sj, add, d.fix_scale != 0);
      double e[7];
      eg_edge_error(Si, Sj, d.C + 8 * k, e);
#pragma unroll
      for (int r = 0; r < 7; ++r) ers[w][lane][r] = e[r];
    }
  }
  eg_wave_sync();
  if (valid) {
    const double scalar = 1.0 / (2 * 1e-9);
    for (int q = lane; q < 98; q += 64) {
      const int side = q / 49, r = (q % 49) / 7, c = q % 7;
      double v = 0.0;
      if (side == 0 ? free_i : free_j) {
        double bak = ers[w][14 * side + 2 * c][r];
        bak -= ers[w][14 * side + 2 * c + 1][r];
        v = scalar * bak;
      }
      J[w][side][7 * r + c] = v;
    }
  }
  eg_wave_sync();
  if (valid) {  // AtO = J^T Omega for both sides
    for (int q = lane; q < 98; q += 64) {
      const int side = q / 49, r = (q % 49) / 7, c = q % 7;
      double v = 0.0;
#pragma unroll
      for (int s = 0; s < 7; ++s) v += J[w][side][7 * s + r] * info_at(d, k, s, c);
      AtO[w][side][7 * r + c] = v;
    }
  }
  eg_wave_sync();
  if (valid) {
    double *o = d.jt + 161 * k;
    const double *e = d.err + 7 * k;
    for (int q = lane; q < 161; q += 64) {
      double v = 0.0;
      if (q < 147) {  // 0: H_ii, 1: H_jj, 2: H_ij
        const int blk = q / 49, r = (q % 49) / 7, c = q % 7;
        const double *Ao = AtO[w][blk == 1 ? 1 : 0];
        const double *R = J[w][blk == 0 ? 0 : 1];
#pragma unroll
        for (int s = 0; s < 7; ++s) v += Ao[7 * r + s] * R[7 * s + c];
      } else {  // b_side[r] = sum_s J[s][r] * (-(Omega e)[s])
        const int side = (q - 147) / 7, r = (q - 147) % 7;
#pragma unroll
        for (int s = 0; s < 7; ++s) {
          double oe = 0.0;
#pragma unroll
          for (int t = 0; t < 7; ++t) oe += info_at(d, k, s, t) * e[t];
          v += J[w][side][7 * s + r] * (-oe);
        }
      }
      o[q] = v;
    }
  }
}

// sqlm_eg_get_jacobians: one thread per (edge, side, dimension), the same
// perturbation, error and difference arithmetic as k_eg_linearize's lanes.
__global__ __launch_bounds__(256) void k_eg_jacobians(const double *__restrict__ S, const int32_t *__restrict__ ei,
                                                      const int32_t *__restrict__ ej, const double *__restrict__ C,
                                                      const uint8_t *__restrict__ fixed, int fix_scale, int64_t nE,
                                                      double *__restrict__ J) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 14 * nE) return;
  const int64_t k = t / 14;
  const int side = (int)(t % 14) / 7, dim = (int)(t % 7);
  const int vi = ei[k], vj = ej[k];
  double *o = J + 98 * k + 49 * side;
  if (fixed[side == 0 ? vi : vj]) {
    for (int r = 0; r < 7; ++r) o[7 * r + dim] = 0.0;
    return;
  }
  double e2[2][7];
  for (int m = 0; m < 2; ++m) {
    double Si[8], Sj[8], add[7] = {0, 0, 0, 0, 0, 0, 0};
    for (int c = 0; c < 8; ++c) { Si[c] = S[8 * vi + c]; Sj[c] = S[8 * vj + c]; }
    add[dim] = m ? -1e-9 : 1e-9;
    sim3_oplus(side == 0 ? Si : Sj, add, fix_scale != 0);
    eg_edge_error(Si, Sj, C + 8 * k, e2[m]);
  }
  const double scalar = 1.0 / (2 * 1e-9);
  for (int r = 0; r < 7; ++r) {
    double bak = e2[0][r];
    bak -= e2[1][r];
    o[7 * r + dim] = scalar * bak;
  }
}

// One wavefront per destination: a 7x7 block of H0 (lower) or a b vector;
// contributions summed in edge order.
__global__ __launch_bounds__(64) void k_eg_assemble(EGDev d, int nD) {
  const int t = blockIdx.x, lane = threadIdx.x;
  if (t >= nD) return;
  const int dst = d.dst[t];
  const int beg = d.src_ptr[t], end = d.src_ptr[t + 1];
  if (dst >= 0) {
    if (lane >= 49) return;
    const int br = dst >> 16, bc = dst & 0xffff, r = lane / 7, c = lane % 7;
    double v = 0.0;
    for (int q = beg; q < end; ++q) {
      const int s = d.src[q], kind = s & 3;
      const double *blk = d.jt + 161 * (int64_t)(s >> 2);
      v += kind == 0 ? blk[lane] : kind == 1 ? blk[49 + lane] : kind == 2 ? blk[98 + lane] : blk[98 + 7 * c + r];
    }
    *h0_at(d, 7 * br + r, 7 * bc + c) = v;
  } else {
    if (lane >= 7) return;
    const int hv = -dst - 1;
    double v = 0.0;
    for (int q = beg; q < end; ++q) {
      const int s = d.src[q], side = s & 1;
      v += d.jt[161 * (int64_t)(s >> 2) + 147 + 7 * side + lane];
    }
    d.b[7 * hv + lane] = v;
  }
}

// A = H0 + lambda I on the problem's dimensions, identity on the padding (lower part).
__global__ __launch_bounds__(256) void k_eg_damp(EGDev d, double *A, double lambda) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t np = d.n_pad;
  if (g >= np * np) return;
  const int r = (int)(g / np), c = (int)(g % np);
  double v = 0.0;
  if (c <= r) {
    if (row_valid(d, r)) v = d.H0[g] + (r == c ? lambda : 0.0);
    else v = r == c ? 1.0 : 0.0;
  }
  A[g] = v;
}

__global__ __launch_bounds__(256) void k_eg_maxdiag(EGDev d) {
  __shared__ double red[4];
  double m = 0.0;
  for (int j = threadIdx.x; j < d.n_pad; j += blockDim.x)
    if (row_valid(d, j)) m = fmax(m, fabs(*h0_at(d, j, j)));
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) m = fmax(m, __shfl_xor(m, s, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) d.scalars[3] = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
}

// VertexSim3Expmap::oplusImpl on every free vertex: S1 = Sim3(x_v) * S0.
__global__ __launch_bounds__(256) void k_eg_update(EGDev d, const double *__restrict__ S0, double *__restrict__ S1,
                                                   const double *__restrict__ x) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= d.nK) return;
  double S[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) S[c] = S0[8 * p + c];
  const int h = d.hid[p];
  if (h >= 0) sim3_oplus(S, x + 7 * h, d.fix_scale != 0);
#pragma unroll
  for (int c = 0; c < 8; ++c) S1[8 * p + c] = S[c];
}

// computeScale: sum_j x_j (lambda x_j + b_j)
__global__ __launch_bounds__(kEGBlock) void k_eg_scale(EGDev d, const double *__restrict__ x, double lambda) {
  __shared__ double red[kEGBlock / 64];
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  double v = 0.0;
  if (j < d.n_pad && row_valid(d, j)) v = x[j] * (lambda * x[j] + d.b[j]);
  const double s = eg_block_sum(v, red);
  if (threadIdx.x == 0) d.partials[2 * kEGMaxParts + blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_eg_reduce(EGDev d, int n_err_parts, int n_scale_parts, int cur,
                                                   const int *flags) {
  __shared__ double red[4];
  for (int reg = 0; reg < 3; ++reg) {
    if (reg == 0 && !cur) continue;
    const int n = reg == 2 ? n_scale_parts : n_err_parts;
    double v = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) v += d.partials[reg * kEGMaxParts + i];
    const double s = eg_block_sum(v, red);
    if (threadIdx.x == 0) d.scalars[reg] = s;
    __syncthreads();
  }
  if (threadIdx.x == 0 && flags) d.scalars[4] = (double)flags[0];
}

// ---- band + border solve of the block-arrow layout (cyclic reduction) -------
// The band (p blocks of n = kCRMaxN rows) is block-tridiagonal and the border
// couples to any band block, so [B F^T; F G] [x_b; x_c] = [r_b; r_c] is solved as
//   B [Y | y] = [F^T | r_b]     cyclic reduction, R = nb + 1 right-hand sides
//   (G - F Y) x_c = r_c - F y   dense Cholesky of the nb x nb border system
//   x_b = y - Y x_c,
// i.e. log2(p) levels of 112-row block factorizations instead of p sequential
// block steps of the arrow Cholesky.
struct EGCR {
  int p = 0, n = 0, R = 0, nb = 0, nc = 0;
  double *D = nullptr, *E = nullptr, *A = nullptr, *Cm = nullptr, *gs = nullptr, *xs = nullptr;
  double *L = nullptr;  // Linv_I of the factored blocks
  double *G = nullptr, *Go = nullptr, *Z = nullptr, *X = nullptr, *P = nullptr;
  double *Sc = nullptr, *ScL = nullptr, *ScLinv = nullptr, *rc = nullptr, *xc = nullptr;
};

// D_I / E_I / G_I (and its copy Go) from the assembled lower H0 with lambda on
// the diagonal of the problem rows (identity on padding rows), the border
// system S_c = G + lambda I and r_c.
__global__ __launch_bounds__(256) void k_egcr_gather(EGDev d, EGCR c, double lambda) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int n = c.n, R = c.R;
  const int64_t nn = (int64_t)n * n, nD = (int64_t)c.p * nn, nG = (int64_t)c.p * n * R;
  const int64_t nS = (int64_t)c.nc * c.nc;
  const int vb = 7 * d.band_slots, b0 = 7 * d.border0;
  if (g < nD) {
    const int I = (int)(g / nn), rem = (int)(g - I * nn), r = rem / n, cc = rem - r * n;
    const int gr = I * n + r, gc = I * n + cc;
    const double *D0 = d.D0 + I * nn;
    double v;
    if (gr < vb && gc < vb) {
      v = cc <= r ? D0[r * n + cc] : D0[cc * n + r];
      if (r == cc) v += lambda;
    } else {
      v = r == cc ? 1.0 : 0.0;
    }
    c.D[g] = v;
    // E_I(r, cc) = S(I n + r, (I+1) n + cc), assembled as block (I+1, I) entry (cc, r)
    c.E[g] = (I + 1 < c.p && gr < vb && gc + n < vb) ? d.E0[I * nn + (int64_t)cc * n + r] : 0.0;
  } else if (g < nD + nG) {
    const int64_t g2 = g - nD;
    const int I = (int)(g2 / ((int64_t)n * R)), rem = (int)(g2 - (int64_t)I * n * R), r = rem / R, l = rem - r * R;
    const int gr = I * n + r;
    double v = 0.0;
    if (gr < vb) {
      if (l < c.nb) v = d.F0[(size_t)l * c.p * n + gr];
      else if (l == c.nb) v = d.b[gr];
    }
    c.G[g2] = v;
    c.Go[g2] = v;
  } else if (g < nD + nG + nS) {
    const int64_t g3 = g - nD - nG;
    const int k = (int)(g3 / c.nc), l = (int)(g3 - (int64_t)k * c.nc);
    double v;
    if (k < c.nb && l < c.nb) {
      v = l <= k ? d.B0[(size_t)k * c.nb + l] : d.B0[(size_t)l * c.nb + k];
      if (k == l) v += lambda;
    } else {
      v = k == l ? 1.0 : 0.0;
    }
    c.Sc[g3] = v;
    if (l == 0) c.rc[k] = k < c.nb ? d.b[b0 + k] : 0.0;
  }
}

// S_c -= F Y, r_c -= F y from the per-block products P_I = Go_I^T X_I, summed
// in block order (deterministic).
__global__ __launch_bounds__(256) void k_egcr_schur(EGCR c) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= c.nb * (c.nb + 1)) return;
  const int k = g / (c.nb + 1), l = g - k * (c.nb + 1);
  double s = 0.0;
  for (int I = 0; I < c.p; ++I) s += c.P[((size_t)I * c.R + k) * c.R + l];
  if (l < c.nb) c.Sc[(size_t)k * c.nc + l] -= s;
  else c.rc[k] -= s;
}

// x in the EG row layout: band rows y - Y x_c, border rows x_c, padding 0.
__global__ __launch_bounds__(256) void k_egcr_final(EGDev d, EGCR c, double *x) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= d.n_pad) return;
  const int vb = 7 * d.band_slots, b0 = 7 * d.border0;
  double v = 0.0;
  if (j < vb) {
    const double *Xr = c.X + (size_t)j * c.R;  // band row j = block j / n, row j % n
    v = Xr[c.nb];
    for (int l = 0; l < c.nb; ++l) v -= Xr[l] * c.xc[l];
  } else if (j >= b0 && j < b0 + c.nb) {
    v = c.xc[j - b0];
  }
  x[j] = v;
}

}  // namespace

// ---------------------------------------------------------------- host driver

struct EGSolver {
  hipStream_t st = nullptr;
  int nK = 0, fix_scale = 0;
  int64_t nE = 0;
  std::vector<double> S, C, info, err;
  std::vector<uint8_t> fixed;
  std::vector<int32_t> ei, ej;
  std::vector<void *> mem;
  double *h_scal = nullptr;

  ~EGSolver() { release(); if (h_scal) (void)hipHostFree(h_scal); }
  void release() {
    for (void *p : mem) (void)hipFree(p);
    mem.clear();
  }
  template <class T>
  T *alloc(size_t n) {
    void *p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) return nullptr;
    mem.push_back(p);
    return static_cast<T *>(p);
  }
  template <class T>
  T *upload(const std::vector<T> &v) {
    T *p = alloc<T>(v.size());
    if (p && !v.empty() && hipMemcpyAsync(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, st) != hipSuccess)
      return nullptr;
    return p;
  }

  int optimize(int iterations, double user_lambda, const volatile uint8_t *stop, sqlm_stats *stt, int *n_iter);
};

namespace {
inline bool stopped(const volatile uint8_t *s) { return s && *s; }
}

int EGSolver::optimize(int iterations, double user_lambda, const volatile uint8_t *stop, sqlm_stats *stt,
                       int *n_iter) {
  sqlm_stats local;
  if (!stt) stt = &local;
  std::memset(stt, 0, sizeof(*stt));
  if (n_iter) *n_iter = -1;
  // initializeOptimization: active edges (not all-fixed), active vertices, free hidx in id order
  std::vector<int> act, hid(nK, -1);
  std::vector<uint8_t> vact(nK, 0);
  for (int64_t e = 0; e < nE; ++e) {
    if (fixed[ei[e]] && fixed[ej[e]]) continue;
    act.push_back((int)e);
    vact[ei[e]] = vact[ej[e]] = 1;
  }
  int nP = 0;
  for (int p = 0; p < nK; ++p)
    if (vact[p] && !fixed[p]) hid[p] = nP++;
  if (nP == 0) return SQLM_OK;  // "0 vertices to optimize": optimize() returns -1
  const int64_t A_ = (int64_t)act.size();
  const int n = 7 * nP;
  // Block-arrow layout: g2o's id order keeps the essential graph banded except
  // for the loop edges. Vertices covering every edge longer than one 112-row
  // block (16 vertices) move to a dense border after the band, so the band is
  // block-tridiagonal and the factor only touches the band + border blocks.
  // Dense layout when the border would exceed a third of the system.
  constexpr int kVB = kCRMaxN / 7;
  std::vector<uint8_t> border(nP, 0);
  {
    std::vector<int> nlong(nP, 0);
    std::vector<std::pair<int, int>> longe;
    for (int e : act) {
      const int hi = hid[ei[e]], hj = hid[ej[e]];
      if (hi >= 0 && hj >= 0 && std::abs(hi - hj) > kVB) {
        longe.emplace_back(hi, hj);
        ++nlong[hi];
        ++nlong[hj];
      }
    }
    for (auto &pr : longe)
      if (!border[pr.first] && !border[pr.second])
        border[nlong[pr.first] > nlong[pr.second] || (nlong[pr.first] == nlong[pr.second] && pr.first > pr.second)
                   ? pr.first
                   : pr.second] = 1;
  }
  int nborder = 0;
  for (int h = 0; h < nP; ++h) nborder += border[h];
  const bool arrow = 3 * nborder <= nP && std::getenv("SQLM_EG_DENSE") == nullptr;
  int band_slots = nP, border0 = nP, band_blk = 0;
  {
    std::vector<int> slot(nP);
    if (arrow) {
      int nb = 0;
      for (int h = 0; h < nP; ++h)
        if (!border[h]) slot[h] = nb++;
      band_blk = (nb + kVB - 1) / kVB;
      band_slots = nb;
      border0 = band_blk * kVB;
      int q = 0;
      for (int h = 0; h < nP; ++h)
        if (border[h]) slot[h] = border0 + q++;
      nborder = q;
    } else {
      for (int h = 0; h < nP; ++h) slot[h] = h;
      nborder = 0;
    }
    for (int p = 0; p < nK; ++p)
      if (hid[p] >= 0) hid[p] = slot[hid[p]];
  }
  const int nslots = arrow ? border0 + nborder : nP;
  const int n_pad = std::max(kCRMaxN, (7 * nslots + kCRMaxN - 1) / kCRMaxN * kCRMaxN);
  if ((int64_t)n_pad * n_pad > (int64_t)1 << 31) return SQLM_ERR_UNSUPPORTED;  // dense path limit (~46k dims)
  if ((A_ + kEGBlock - 1) / kEGBlock > kEGMaxParts || (n_pad + kEGBlock - 1) / kEGBlock > kEGMaxParts)
    return SQLM_ERR_UNSUPPORTED;
  // assembly lists: diagonal blocks, off-diagonal pairs (lower), b vectors; sources in edge order
  std::vector<std::vector<int>> diag(nslots), bvec(nslots);
  std::vector<uint8_t> used(nslots, 0);
  for (int p = 0; p < nK; ++p)
    if (hid[p] >= 0) used[hid[p]] = 1;
  std::map<std::pair<int, int>, std::vector<int>> off;
  std::vector<int> aei(A_), aej(A_);
  std::vector<double> aC(8 * A_), ainfo(info.empty() ? 0 : 49 * A_);
  for (int64_t k = 0; k < A_; ++k) {
    const int e = act[k], i = ei[e], j = ej[e], hi = hid[i], hj = hid[j];
    aei[k] = i;
    aej[k] = j;
    std::memcpy(&aC[8 * k], &C[8 * e], 8 * sizeof(double));
    if (!info.empty()) std::memcpy(&ainfo[49 * k], &info[49 * e], 49 * sizeof(double));
    const int ks = (int)k << 2;
    if (hi >= 0) { diag[hi].push_back(ks | 0); bvec[hi].push_back(ks | 0); }
    if (hj >= 0) { diag[hj].push_back(ks | 1); bvec[hj].push_back(ks | 1); }
    if (hi >= 0 && hj >= 0 && hi != hj) {
      if (hi > hj) off[{hi, hj}].push_back(ks | 2);
      else off[{hj, hi}].push_back(ks | 3);
    }
  }
  std::vector<int> dst, sptr{0}, src;
  for (int v = 0; v < nslots; ++v) {
    if (!used[v]) continue;
    dst.push_back(v << 16 | v);
    src.insert(src.end(), diag[v].begin(), diag[v].end());
    sptr.push_back((int)src.size());
  }
  for (auto &kv : off) {
    dst.push_back(kv.first.first << 16 | kv.first.second);
    src.insert(src.end(), kv.second.begin(), kv.second.end());
    sptr.push_back((int)src.size());
  }
  for (int v = 0; v < nslots; ++v) {
    if (!used[v]) continue;
    dst.push_back(-(v + 1));
    src.insert(src.end(), bvec[v].begin(), bvec[v].end());
    sptr.push_back((int)src.size());
  }
  if (nslots > 0xffff) return SQLM_ERR_UNSUPPORTED;
  release();
  if (!h_scal && hipHostMalloc((void **)&h_scal, 8 * sizeof(double)) != hipSuccess) return SQLM_ERR_HIP;
  EGDev d;
  d.nK = nK; d.nP = nP; d.n = n; d.n_pad = n_pad; d.fix_scale = fix_scale; d.nE = A_;
  d.band_slots = band_slots; d.border0 = border0; d.border_slots = nborder;
  int *d_act = upload(act), *d_ei = upload(aei), *d_ej = upload(aej), *d_hid = upload(hid);
  double *d_C = upload(aC), *d_info = info.empty() ? nullptr : upload(ainfo);
  double *Sd[2] = {upload(S), alloc<double>(S.size())};
  d.err = alloc<double>(7 * A_);
  d.jt = alloc<double>(161 * A_);
  const size_t nn = (size_t)n_pad * n_pad;
  // arrow layout: the band by cyclic reduction with the border columns as extra
  // right-hand sides (EGCR) unless SQLM_EG_CR=0; else the arrow / dense Cholesky
  const int nbr = 7 * nborder;
  const char *cr_env = std::getenv("SQLM_EG_CR");
  const bool use_cr = arrow && band_blk >= 1 && nbr + 1 <= 512 && !(cr_env && std::atoi(cr_env) == 0);
  double *A = nullptr, *L = nullptr, *Linv = nullptr;
  EGCR c;
  size_t asm_n = nn;  // doubles of the assembly buffer (cleared every iteration)
  if (use_cr) {
    const size_t pnn = (size_t)band_blk * kCRMaxN * kCRMaxN;
    asm_n = 2 * pnn + (size_t)nbr * band_blk * kCRMaxN + (size_t)nbr * nbr;
    d.H0 = alloc<double>(asm_n);
    if (!d.H0) return SQLM_ERR_OOM;
    d.cr = 1; d.cr_p = band_blk; d.cr_nb = nbr;
    d.D0 = d.H0; d.E0 = d.D0 + pnn; d.F0 = d.E0 + pnn; d.B0 = d.F0 + (size_t)nbr * band_blk * kCRMaxN;
  } else {
    d.H0 = alloc<double>(nn);
  }
  if (use_cr) {
    c.p = band_blk;
    c.n = kCRMaxN;
    c.nb = nbr;
    c.R = (nbr + 1 + 15) / 16 * 16;
    c.nc = nbr > 0 ? (nbr + kCRMaxN - 1) / kCRMaxN * kCRMaxN : kCRMaxN;
    const size_t pnn = (size_t)c.p * c.n * c.n, pnr = (size_t)c.p * c.n * c.R, ncc = (size_t)c.nc * c.nc;
    c.D = alloc<double>(pnn); c.L = alloc<double>(pnn); c.E = alloc<double>(pnn); c.A = alloc<double>(pnn); c.Cm = alloc<double>(pnn);
    c.gs = alloc<double>((size_t)c.p * c.n); c.xs = alloc<double>((size_t)c.p * c.n);
    c.G = alloc<double>(pnr); c.Go = alloc<double>(pnr); c.Z = alloc<double>(pnr); c.X = alloc<double>(pnr);
    c.P = alloc<double>((size_t)c.p * c.R * c.R);
    c.Sc = alloc<double>(ncc); c.ScL = alloc<double>(ncc);
    c.ScLinv = alloc<double>((size_t)(c.nc / kCRMaxN) * kCRMaxN * kCRMaxN);
    c.rc = alloc<double>(c.nc); c.xc = alloc<double>(c.nc);
    if (!c.D || !c.L || !c.E || !c.A || !c.Cm || !c.gs || !c.xs || !c.G || !c.Go || !c.Z || !c.X || !c.P || !c.Sc || !c.ScL ||
        !c.ScLinv || !c.rc || !c.xc)
      return SQLM_ERR_OOM;
    // the scratch right-hand side of the reused single-RHS kernels: finite values
    if (hipMemsetAsync(c.gs, 0, sizeof(double) * c.p * c.n, st) != hipSuccess) return SQLM_ERR_HIP;
  } else {
    A = alloc<double>(nn);
    L = alloc<double>(nn);
    Linv = alloc<double>((size_t)(n_pad / kCRMaxN) * kCRMaxN * kCRMaxN);
  }
  d.b = alloc<double>(n_pad);
  double *r = alloc<double>(n_pad), *x = alloc<double>(n_pad);
  int *d_dst = upload(dst), *d_sptr = upload(sptr), *d_src = upload(src);
  d.partials = alloc<double>(3 * kEGMaxParts);
  d.scalars = alloc<double>(8);
  int *flags = alloc<int>(4);
  if (!d_act || !d_ei || !d_ej || !d_hid || !d_C || (!info.empty() && !d_info) || !Sd[0] || !Sd[1] || !d.err ||
      !d.jt || !d.H0 || (!use_cr && (!A || !L || !Linv)) || !d.b || !r || !x || !d_dst || !d_sptr || !d_src || !d.partials ||
      !d.scalars || !flags)
    return SQLM_ERR_OOM;
  d.act = d_act; d.ei = d_ei; d.ej = d_ej; d.hid = d_hid; d.C = d_C; d.info = d_info;
  d.dst = d_dst; d.src_ptr = d_sptr; d.src = d_src;
  if (hipMemsetAsync(d.b, 0, sizeof(double) * n_pad, st) != hipSuccess) return SQLM_ERR_HIP;
  const int nD = (int)dst.size();
  const int eb = (int)((A_ + kEGBlock - 1) / kEGBlock), sb = (n_pad + kEGBlock - 1) / kEGBlock;
  auto fetch = [&]() -> int {
    if (hipMemcpyAsync(h_scal, d.scalars, 8 * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess) return -1;
    return hipStreamSynchronize(st) == hipSuccess ? 0 : -1;
  };
  stt->n_active_edges = (int)A_;
  const bool debug = std::getenv("SQLM_EG_DEBUG") != nullptr;  // per-trial trace on stderr
  double lambda = -1., ni = 2.;
  int nbad = 0, its = 0, result = 0;
  for (int it = 0; it < iterations && !stopped(stop) && result == 0; ++it) {
    // computeActiveErrors + buildSystem
    hipLaunchKernelGGL(k_eg_errors, dim3(eb), dim3(kEGBlock), 0, st, d, Sd[0], 0);
    hipLaunchKernelGGL(k_eg_reduce, dim3(1), dim3(256), 0, st, d, eb, 0, 1, (const int *)nullptr);
    hipLaunchKernelGGL(k_eg_linearize, dim3((unsigned)((A_ + 3) / 4)), dim3(256), 0, st, d, Sd[0]);
    if (hipMemsetAsync(d.H0, 0, asm_n * sizeof(double), st) != hipSuccess) return SQLM_ERR_HIP;
    hipLaunchKernelGGL(k_eg_assemble, dim3(nD), dim3(64), 0, st, d, nD);
    if (it == 0) hipLaunchKernelGGL(k_eg_maxdiag, dim3(1), dim3(256), 0, st, d);
    if (fetch()) return SQLM_ERR_HIP;
    double currentChi = h_scal[0];
    const double iniChi = currentChi;
    if (it == 0) {
      stt->chi2_begin = currentChi;
      lambda = user_lambda > 0 ? user_lambda : 1e-5 * h_scal[3];
      ni = 2;
      nbad = 0;
    }
    double rho = 0;
    int qmax = 0;
    do {
      if (hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(flags), 1, 1, st) != hipSuccess) return SQLM_ERR_HIP;
      if (use_cr) {
        const int64_t tot = (int64_t)c.p * c.n * c.n + (int64_t)c.p * c.n * c.R + (int64_t)c.nc * c.nc;
        hipLaunchKernelGGL(k_egcr_gather, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, d, c, lambda);
        if (launch_cr_multi(c.D, c.L, c.E, c.A, c.Cm, c.gs, c.xs, c.G, c.Z, c.X, flags, c.p, c.n, c.R, st))
          return SQLM_ERR_HIP;
        if (c.nb > 0) {
          if (launch_batched_atb(c.Go, c.X, c.P, c.p, c.n, c.R, st)) return SQLM_ERR_HIP;
          hipLaunchKernelGGL(k_egcr_schur, dim3((c.nb * (c.nb + 1) + 255) / 256), dim3(256), 0, st, c);
          // the border complement's last block holds nb - (nc - kCRMaxN) real rows (identity after them)
          const int n_last = ((c.nb - (c.nc - kCRMaxN)) + 15) / 16 * 16;
          if (launch_dense_spd_solve(c.Sc, c.ScL, c.ScLinv, c.rc, c.xc, flags, c.nc, st, 0, n_last))
            return SQLM_ERR_HIP;
        }
        hipLaunchKernelGGL(k_egcr_final, dim3((n_pad + 255) / 256), dim3(256), 0, st, d, c, x);
      } else {
        hipLaunchKernelGGL(k_eg_damp, dim3((unsigned)((nn + 255) / 256)), dim3(256), 0, st, d, A, lambda);
        if (hipMemcpyAsync(r, d.b, sizeof(double) * n_pad, hipMemcpyDeviceToDevice, st) != hipSuccess)
          return SQLM_ERR_HIP;
        if (launch_dense_spd_solve(A, L, Linv, r, x, flags, n_pad, st, arrow ? band_blk : 0)) return SQLM_ERR_HIP;
      }
      hipLaunchKernelGGL(k_eg_update, dim3((nK + 255) / 256), dim3(256), 0, st, d, Sd[0], Sd[1], x);
      hipLaunchKernelGGL(k_eg_errors, dim3(eb), dim3(kEGBlock), 0, st, d, Sd[1], 1);
      hipLaunchKernelGGL(k_eg_scale, dim3(sb), dim3(kEGBlock), 0, st, d, x, lambda);
      hipLaunchKernelGGL(k_eg_reduce, dim3(1), dim3(256), 0, st, d, eb, sb, 0, flags);
      if (fetch()) return SQLM_ERR_HIP;
      const bool ok = h_scal[4] > 0.5;
      if (debug)
        std::fprintf(stderr, "eg it %d trial %d lambda %.6g chi_cur %.17g chi_new %.17g scale %.6g ok %d\n", it,
                     qmax, lambda, currentChi, h_scal[1], h_scal[2], (int)ok);
      // a NaN chi2 is a failed trial (lm_decide, sqlm_internal.h)
      double tempChi = ok && !(std::isnan(h_scal[1]) && std::isfinite(currentChi)) ? h_scal[1]
                                                                                   : std::numeric_limits<double>::max();
      rho = (currentChi - tempChi);
      double scale = ok ? h_scal[2] : 0.0;
      scale += 1e-3;
      rho /= scale;
      if (rho > 0 && std::isfinite(tempChi)) {
        double alpha = 1. - std::pow((2 * rho - 1), 3);
        alpha = std::min(alpha, 2. / 3.);
        lambda *= std::max(1. / 3., alpha);
        ni = 2;
        currentChi = tempChi;
        std::swap(Sd[0], Sd[1]);
      } else {
        lambda *= ni;
        ni *= 2;
      }
      qmax++;
      stt->trials++;
    } while (rho < 0 && qmax < 10 && !stopped(stop));
    if (qmax == 10 || rho == 0) result = 1;
    else {
      if ((iniChi - currentChi) * 1e3 < iniChi) nbad++;
      else nbad = 0;
      if (nbad >= 3) result = 1;
    }
    if (its < SQLM_TRACE_MAX) {
      stt->trace_chi2[its] = currentChi;
      stt->trace_lambda[its] = lambda;
      stt->trace_trials[its] = qmax;
      stt->trace_len = its + 1;
    }
    stt->chi2_end = currentChi;
    stt->lambda_end = lambda;
    ++its;
  }
  stt->iterations = its;
  stt->result = result;
  if (n_iter) *n_iter = its;
  // results: estimates and the last computed (g2o: possibly rejected-trial) errors
  std::vector<double> aerr(7 * A_);
  if (hipMemcpyAsync(S.data(), Sd[0], S.size() * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(aerr.data(), d.err, aerr.size() * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return SQLM_ERR_HIP;
  for (int64_t k = 0; k < A_; ++k) std::memcpy(&err[7 * (size_t)act[k]], &aerr[7 * k], 7 * sizeof(double));
  release();
  return SQLM_OK;
}

EGSolver *eg_create(hipStream_t st) {
  EGSolver *s = new (std::nothrow) EGSolver();
  if (s) s->st = st;
  return s;
}
void eg_destroy(EGSolver *s) { delete s; }

int eg_set_problem(EGSolver *s, int n_kf, const double *Siw, const uint8_t *fixed, int fix_scale, int64_t n_edge,
                   const int32_t *ei, const int32_t *ej, const double *Sji, const double *info) {
  if (n_kf < 0 || n_edge < 0 || (n_kf && (!Siw || !fixed)) || (n_edge && (!ei || !ej || !Sji)))
    return SQLM_ERR_INVALID_ARG;
  for (int64_t e = 0; e < n_edge; ++e)
    if (ei[e] < 0 || ei[e] >= n_kf || ej[e] < 0 || ej[e] >= n_kf) return SQLM_ERR_INVALID_ARG;
  for (int p = 0; p < n_kf; ++p)
    if (!(Siw[8 * p + 7] > 0.0)) return SQLM_ERR_INVALID_ARG;
  s->nK = n_kf;
  s->nE = n_edge;
  s->fix_scale = fix_scale ? 1 : 0;
  s->S.assign(Siw, Siw + 8 * (size_t)n_kf);
  s->fixed.assign(fixed, fixed + n_kf);
  s->ei.assign(ei, ei + n_edge);
  s->ej.assign(ej, ej + n_edge);
  s->C.assign(Sji, Sji + 8 * (size_t)n_edge);
  if (info) s->info.assign(info, info + 49 * (size_t)n_edge);
  else s->info.clear();
  s->err.assign(7 * (size_t)n_edge, 0.0);
  return SQLM_OK;
}

int eg_optimize(EGSolver *s, int iterations, double user_lambda, const volatile uint8_t *stop, sqlm_stats *st,
                int *n_iter) {
  return s->optimize(iterations, user_lambda, stop, st, n_iter);
}

int eg_get_poses(const EGSolver *s, double *Siw) {
  if (!Siw && s->nK) return SQLM_ERR_INVALID_ARG;
  std::memcpy(Siw, s->S.data(), s->S.size() * sizeof(double));
  return SQLM_OK;
}

int eg_get_jacobians(EGSolver *s, double *J) {
  if (!J && s->nE) return SQLM_ERR_INVALID_ARG;
  if (s->nE == 0) return SQLM_OK;
  std::vector<void *> keep;
  keep.swap(s->mem);  // the optimizer's buffers stay as they are
  int rc = SQLM_OK;
  double *dS = s->upload(s->S), *dC = s->upload(s->C);
  int32_t *dei = s->upload(s->ei), *dej = s->upload(s->ej);
  uint8_t *dfx = s->upload(s->fixed);
  double *dJ = s->alloc<double>(98 * (size_t)s->nE);
  if (!dS || !dC || !dei || !dej || !dfx || !dJ) {
    rc = SQLM_ERR_HIP;
  } else {
    const int64_t n = 14 * s->nE;
    hipLaunchKernelGGL(k_eg_jacobians, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s->st, dS, dei, dej, dC, dfx,
                       s->fix_scale, s->nE, dJ);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(J, dJ, 98 * sizeof(double) * (size_t)s->nE, hipMemcpyDeviceToHost, s->st) != hipSuccess ||
        hipStreamSynchronize(s->st) != hipSuccess)
      rc = SQLM_ERR_HIP;
  }
  s->release();
  s->mem.swap(keep);
  return rc;
}

int eg_get_edge_chi2(const EGSolver *s, double *chi2) {
  if (!chi2 && s->nE) return SQLM_ERR_INVALID_ARG;
  for (int64_t e = 0; e < s->nE; ++e) {
    const double *er = &s->err[7 * e];
    double c = 0.0;
    for (int r = 0; r < 7; ++r) {
      double oe = 0.0;
      for (int t = 0; t < 7; ++t) oe += (s->info.empty() ? (r == t ? 1.0 : 0.0) : s->info[49 * e + 7 * r + t]) * er[t];
      c += er[r] * oe;
    }
    chi2[e] = c;
  }
  return SQLM_OK;
}

}  // namespace sqlm
