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
//   wave 0        the diagonal wave: factors diagonal tile k at step k in four
//                 rank-4 groups (a 4x4 Cholesky on uniform values from
//                 readlane, W = L44^-1 per lane, the finished rows X = W M4 by
//                 one MFMA, the rank-4 update by one MFMA) and publishes each
//                 group's W and finished rows in LDS. Waves 4, 8, 12 stay idle
//                 so the critical path has its SIMD (matrix pipe and issue) to
//                 itself: any MFMA-busy partner triples its time (tools/
//                 group_probe).
//   workers       the other 12 waves own one column of tiles each: D column J
//                 (the U tiles above its diagonal, and its diagonal tile until
//                 step J, when it hands it to wave 0 through LDS; in LINV mode
//                 continued below the diagonal by identity column J+1), the T
//                 column (diagonal inverses; LINV: identity column 0), g, and
//                 the E^T / E columns dealt over the `split` workgroups that
//                 share the superblock (each repeats the factorization: it is
//                 the latency, the E columns are the parallel work).
// Step k: every row-k tile follows wave 0 one group behind (group_apply: the
// same two MFMAs per group); D columns publish U_kJ for the trailing updates
// tile(I, col) -= U_kI^T X_k,col (row k+1 first, the rest deferred into the
// next step). The owner of column k+1 folds the update of its diagonal tile
// into its group_apply (one MFMA per group) and hands the tile over.
// Hand-offs are LDS flags (no barrier after the start).
#pragma once

namespace sqlm {
namespace aug {

constexpr int kWaves = 16, kThreads = 64 * kWaves, kMaxNt = kCRMaxN / 16, kWorkers = 12;
constexpr int kPairs = kMaxNt * (kMaxNt - 1) / 2;
enum : int { kNone = 0, kColD = 1, kColT = 2, kColI0 = 3, kColEt = 4, kColE = 5, kColG = 6 };

struct Shared {
  double W[kMaxNt][4][64];  // group a of step k: A operand W[i][b] at lane 16 b + i (W = L44^-1)
  double O[kMaxNt][4][64];  // the group's finished rows U[4a+b][i] (i > 4a+3) at lane 16 b + i
  double U[kPairs][256];    // U_kJ (k < J), accumulator layout: element j of lane l at [64 j + l]
  double Dg[kMaxNt][256];   // diagonal tile k handed to wave 0, same layout
  int fG[kMaxNt][4], fU[kPairs], fD[kMaxNt];
};

// (k, J), k < J < kMaxNt -> 0 .. kPairs-1
__device__ __forceinline__ constexpr int pair_id(int k, int J) { return k * (2 * kMaxNt - k - 1) / 2 + (J - k - 1); }

__device__ __forceinline__ double rl(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// 1/sqrt(x) by v_rsq_f64 and one Newton step; a non-positive pivot is flagged
__device__ __forceinline__ double rsqn(double x, bool &bad) {
  bad |= !(x > 0.0);
  const double v = x > 0.0 ? x : 1.0;
  double y = __builtin_amdgcn_rsq(v);
  const double hh = 0.5 * v * y;
  return fma(y, fma(-hh, y, 0.5), y);
}

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
// ms): a wave can never hang the device, whatever the schedule does.
__device__ __forceinline__ void spin(int *f) {
  lds_int *p = (lds_int *)f;
  for (int it = 0; __atomic_load_n(p, __ATOMIC_RELAXED) == 0 && it < (1 << 20); ++it) __builtin_amdgcn_s_sleep(1);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
// Producer side: the DS instructions of one wave execute in order, so the flag
// store lands after the data stores issued before it; only the compiler must
// not move them (no s_waitcnt: the wave goes on while the stores drain).
__device__ __forceinline__ void raise_flag(int *f, int lane) {
  __asm__ volatile("" ::: "memory");
  if (lane == 0) __atomic_store_n((lds_int *)f, 1, __ATOMIC_RELAXED);
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

// Step k on the diagonal tile Dg, in four rank-4 groups. Each group publishes
// its A operand W (L44^-1) and its finished rows for group_apply.
__device__ __forceinline__ void diag_groups(Shared &sh, int k, d4 Dg, int lane, bool &bad) {
  const int b = lane >> 4, i = lane & 15, c = lane & 15;
  const d4 zero = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    // the group's 4x4 pivot block: rows / columns 4a .. 4a+3 sit in element a
    // of lanes 16 r + 4a + c (r = row - 4a, c = column - 4a)
    const double m00 = rl(Dg[a], 4 * a), m01 = rl(Dg[a], 4 * a + 1), m02 = rl(Dg[a], 4 * a + 2),
                 m03 = rl(Dg[a], 4 * a + 3);
    const double m11 = rl(Dg[a], 16 + 4 * a + 1), m12 = rl(Dg[a], 16 + 4 * a + 2), m13 = rl(Dg[a], 16 + 4 * a + 3);
    const double m22 = rl(Dg[a], 32 + 4 * a + 2), m23 = rl(Dg[a], 32 + 4 * a + 3);
    const double m33 = rl(Dg[a], 48 + 4 * a + 3);
    // U44 (upper, U44^T U44 = M44) with d_r = 1 / U44[r][r]
    const double d0 = rsqn(m00, bad);
    const double u01 = m01 * d0, u02 = m02 * d0, u03 = m03 * d0;
    const double d1 = rsqn(fma(-u01, u01, m11), bad);
    const double u12 = fma(-u01, u02, m12) * d1, u13 = fma(-u01, u03, m13) * d1;
    const double d2 = rsqn(fma(-u12, u12, fma(-u02, u02, m22)), bad);
    const double u23 = fma(-u12, u13, fma(-u02, u03, m23)) * d2;
    const double d3 = rsqn(fma(-u23, u23, fma(-u13, u13, fma(-u03, u03, m33))), bad);
    // W = (U44^T)^-1, lower; lane (b, i) of the A operand holds W[i][b] (column b)
    const double w0 = b == 0 ? d0 : 0.0;
    const double w1 = b == 1 ? d1 : (b < 1 ? -d1 * (u01 * w0) : 0.0);
    const double w2 = b == 2 ? d2 : (b < 2 ? -d2 * fma(u12, w1, u02 * w0) : 0.0);
    const double w3 = b == 3 ? d3 : -d3 * fma(u23, w2, fma(u13, w1, u03 * w0));
    const double aop = i == 0 ? w0 : i == 1 ? w1 : i == 2 ? w2 : i == 3 ? w3 : 0.0;
    sh.W[k][a][lane] = aop;
    // finished rows 4a .. 4a+3 = W M4 (rows 0..3 of the product, element 0);
    // the rank-4 update of the rows and columns past the group
    const d4 Xd = mfma(aop, Dg[a], zero);
    const double op = c >= 4 * a + 4 ? Xd[0] : 0.0;
    sh.O[k][a][lane] = op;
    Dg = mfma(-op, op, Dg);
    __builtin_amdgcn_sched_barrier(0);  // the update is issued before the flag's LDS wait
    raise_flag(&sh.fG[k][a], lane);
  }
}

// The same four groups on a tile of block row k: t <- L_kk^-1 t. With `diag`,
// the rank-4 pieces of the trailing update diag -= t^T t follow each group.
template <bool DIAG>
__device__ __forceinline__ void group_apply(Shared &sh, int k, d4 &t, d4 &diag, int lane) {
  const d4 zero = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    spin(&sh.fG[k][a]);
    const double aop = sh.W[k][a][lane], op = sh.O[k][a][lane];
    const d4 X = mfma(aop, t[a], zero);
    t[a] = X[0];
    t = mfma(-op, X[0], t);
    if (DIAG) diag = mfma(-X[0], X[0], diag);
  }
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
__device__ __forceinline__ void store_tile(double *P, int n, int r0, int c0, const d4 &t, int lane) {
  const int k4 = lane >> 4, c = lane & 15;
#pragma unroll
  for (int j = 0; j < 4; ++j) P[(size_t)(r0 + k4 + 4 * j) * n + c0 + c] = t[j];
}

// D columns carried by workers: J = 1 .. nt-1 (LINV: 0 .. nt-1, column 0 then
// carries identity column 1)
__host__ __device__ __forceinline__ int d_columns(int nt, bool linv) { return linv ? nt : nt - 1; }
// E / g columns of a superblock
__host__ __device__ __forceinline__ int extra_columns(int nt, bool level, bool right) {
  return (level ? nt : 0) + (level && right ? nt : 0) + 1;
}
inline int min_split(int nt, bool linv, int ne) {
  const int cap = kWorkers - d_columns(nt, linv) - 1;
  return (ne + cap - 1) / cap;
}

// role of a worker (q = 0 .. kWorkers-1) of a workgroup serving one superblock
__device__ __forceinline__ void column_of(int q, int nt, bool linv, bool level, bool right, int split, int sidx,
                                          int &type, int &J) {
  J = 0;
  const int nd = d_columns(nt, linv);
  if (q < nd) {
    type = kColD;
    J = linv ? q : q + 1;
    return;
  }
  if (q == nd) {
    type = linv ? kColI0 : kColT;
    return;
  }
  const int e = (q - nd - 1) * split + sidx;
  const int net = level ? nt : 0, nee = (level && right) ? nt : 0;
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
template <bool LINV>
__device__ __forceinline__ bool takes_update(int type, int J, int k, int I) {
  if (type == kColD) return I <= J || (LINV && k >= J + 1);  // U tile / diagonal, or identity column J+1
  return type == kColI0 || type == kColEt || type == kColE || type == kColG;
}

}  // namespace aug

// MODE 0: level step (A_I, C_I, z_I and the back-substitution factor).
// MODE 1: factor only (z_I and the factor). LINV: the factor is Linv_I
// (lower, dense tiles); otherwise the upper U tiles with T_k on the diagonal.
// Superblock I = I0 + stride * (blockIdx.x / split); workgroup sidx = blockIdx.x % split.
template <int MODE, bool LINV>
__global__ __launch_bounds__(aug::kThreads) void k_cr_aug(CRView v, int h, int I0, int stride, int split) {
  using namespace aug;
  extern __shared__ __attribute__((aligned(16))) unsigned char aug_lds[];
  Shared &sh = *reinterpret_cast<Shared *>(aug_lds);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ob = blockIdx.x / split, sidx = blockIdx.x - ob * split;
  const int I = I0 + stride * ob, n = v.n, nt = n >> 4;
  const bool level = MODE == 0, right = level && I + h < v.p, first = sidx == 0;
  for (int t = threadIdx.x; t < 4 * kMaxNt + kPairs + kMaxNt; t += blockDim.x) {
    if (t < 4 * kMaxNt) sh.fG[t >> 2][t & 3] = 0;
    else if (t < 4 * kMaxNt + kPairs) sh.fU[t - 4 * kMaxNt] = 0;
    else sh.fD[t - 4 * kMaxNt - kPairs] = 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) AUG_PROF(0);
  AUG_HWID(wave);
  const double *Dblk = blk(v.D, I, n);
  bool bad = false;
  if (wave == 0) {  // ---- the diagonal wave
    __builtin_amdgcn_s_setprio(3);
    AUG_PROF(1);
    for (int k = 0; k < nt; ++k) {
      d4 Dg;
      if (k == 0) {
        Dg = load_tile(Dblk, n, 0, 0, lane);
      } else {
        spin(&sh.fD[k]);
        Dg = get_tile(sh.Dg[k], lane);
      }
      AUG_STAMP(0, k, 0);
      diag_groups(sh, k, Dg, lane, bad);
      AUG_PROF(2 + k);
    }
    if (bad && lane == 0) v.flags[0] = 0;
    return;
  }
  if ((wave & 3) == 0) return;  // the diagonal wave's SIMD partners stay idle
  const int q = wave - (wave >> 2) - 1;
  int type, J;
  column_of(q, nt, LINV, level, right, split, sidx, type, J);
  if (type == kNone) return;
  // ---- load this wave's column
  d4 t[kMaxNt];
#pragma unroll
  for (int r = 0; r < kMaxNt; ++r) {
    t[r] = d4{0.0, 0.0, 0.0, 0.0};
    if (r >= nt) continue;
    if (type == kColD) {
      if (r < J) t[r] = load_tile_t(Dblk, n, 16 * r, 16 * J, lane);  // U tile (r, J) from the lower block (J, r)
      else if (r == J) t[r] = load_tile(Dblk, n, 16 * r, 16 * J, lane);
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
    // deferred trailing of step k-1: rows k+1 .. (the diagonal of column k+1
    // took its step-(k-1) piece inside group_apply)
    if (k >= 1) {
#pragma unroll
      for (int r = k + 1; r < kMaxNt; ++r) {
        if (r >= nt || !takes_update<LINV>(type, J, k - 1, r)) continue;
        const int pid = pair_id(k - 1, r);
        spin(&sh.fU[pid]);
        const double *U = sh.U[pid];
#pragma unroll
        for (int s = 0; s < 4; ++s) t[r] = mfma(-U[64 * s + lane], t[k - 1][s], t[r]);
      }
    }
    AUG_STAMP(wave, k, 0);
    // row k
    const bool dtile = type == kColD && k < J, next = type == kColD && J == k + 1;
    const bool rowk = type == kColT || (type == kColD ? (k < J || (LINV && k > J)) : true);
    if (rowk) {
      if (type == kColT) t[k] = identity_tile(lane);
      if (next) {
        __builtin_amdgcn_s_setprio(2);
        d4 dd = t[k + 1];
        group_apply<true>(sh, k, t[k], dd, lane);
        t[k + 1] = dd;
        put_tile(sh.U[pair_id(k, J)], t[k], lane);
        raise_flag(&sh.fU[pair_id(k, J)], lane);
        put_tile(sh.Dg[k + 1], t[k + 1], lane);  // the diagonal tile, complete: to wave 0
        raise_flag(&sh.fD[k + 1], lane);
        __builtin_amdgcn_s_setprio(0);
      } else {
        d4 none;
        group_apply<false>(sh, k, t[k], none, lane);
        if (dtile) {  // U_kJ feeds the trailing updates of row J
          put_tile(sh.U[pair_id(k, J)], t[k], lane);
          raise_flag(&sh.fU[pair_id(k, J)], lane);
        }
      }
    }
    AUG_STAMP(wave, k, 1);
    // trailing of step k, row k+1 (the next step's row)
    if (k + 1 < nt && rowk && type != kColT && !next && takes_update<LINV>(type, J, k, k + 1)) {
      const int pid = pair_id(k, k + 1);
      spin(&sh.fU[pid]);
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
        if (first && r < J) store_tile(Lb, n, 16 * r, 16 * J, t[r], lane);  // U tile (r, J)
      }
    } else if (type == kColT) {
      if (first) store_tile(Lb, n, 16 * r, 16 * r, t[r], lane);  // T_r on the diagonal
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
        if (c == 0) v.g[(size_t)I * n + 16 * r + k4 + 4 * j] = t[r][j];
    }
  }
  AUG_PROF(16 + wave);
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
