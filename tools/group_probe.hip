// group_probe — cycles of the CR factor's diagonal rank-4 groups
// (sqlm_cr_aug.h diag_groups) alone and beside other waves of a workgroup.
#include <hip/hip_runtime.h>

#include <cstdio>

#define SQLM_CR_PROF 1
#include "../sqrtlm-slam_amd/csrc/sqlm_rcs_solve.hip"

using sqlm::d4;

// mode 0: wave 0 alone; 1: 15 more waves spinning on an LDS flag (s_sleep);
// 2: 15 more waves running MFMA chains; 3: VALU/readlane part only (no MFMA)
__global__ __launch_bounds__(1024) void k_probe(double *out, long long *cyc, int mode) {
  __shared__ int done;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x == 0) done = 0;
  __syncthreads();
  if (wave == 0) {
    if (mode == 4) __builtin_amdgcn_s_setprio(3);
    d4 t;
    const int k4 = lane >> 4, c = lane & 15;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = k4 + 4 * j;
      t[j] = (r == c ? 16.0 : 0.0) + 0.01 * ((r * 7 + c * 7) % 5);
    }
    bool bad = false;
    long long t0 = clock64();
    for (int it = 0; it < 8; ++it) {
      d4 Tt;
      if (mode == 3) {
        double acc = 0.0;
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          const double m00 = sqlm::aug::rl(t[a], 4 * a), m01 = sqlm::aug::rl(t[a], 4 * a + 1);
          const double m11 = sqlm::aug::rl(t[a], 16 + 4 * a + 1), m22 = sqlm::aug::rl(t[a], 32 + 4 * a + 2);
          const double m33 = sqlm::aug::rl(t[a], 48 + 4 * a + 3), m02 = sqlm::aug::rl(t[a], 4 * a + 2);
          const double d0 = sqlm::aug::rsqn(m00, bad), u01 = m01 * d0, u02 = m02 * d0;
          const double d1 = sqlm::aug::rsqn(fma(-u01, u01, m11), bad);
          const double d2 = sqlm::aug::rsqn(fma(-u02, u02, m22), bad);
          const double d3 = sqlm::aug::rsqn(m33 - d2, bad);
          acc += d0 + d1 + d2 + d3;
          t[(a + 1) & 3] += acc * 1e-30;
        }
        Tt = t;
      } else {
        d4 P = t, Q = t, T2;
        if (mode == 4) sqlm::aug::diag_groups<true>(t, P, Q, T2, lane, bad);
        else sqlm::aug::diag_groups<false>(t, P, Q, T2, lane, bad);
        Tt = T2 + P + Q;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) t[j] += 1e-30 * Tt[j];
    }
    long long t1 = clock64();
    if (lane == 0) {
      cyc[0] = (t1 - t0) / 8;
      done = 1;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) out[lane * 4 + j] = t[j] + (bad ? 1.0 : 0.0);
  } else if (mode == 1) {
    sqlm::aug::spin(&done);
  } else if (mode == 2) {
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    double a = lane * 1e-3;
    for (int it = 0; it < 400; ++it) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, acc, 0, 0, 0);
    out[1024 + threadIdx.x] = acc[0] + acc[3];
  }
}

int main() {
  double *out;
  long long *cyc, h;
  if (hipMalloc(&out, 4096 * 8) != hipSuccess || hipMalloc(&cyc, 8) != hipSuccess) return 1;
  const char *names[] = {"alone", "with_15_spinning", "with_15_mfma", "valu_readlane_only",
                         "alone_with_PQ"};
  std::printf("{");
  for (int mode = 0; mode < 5; ++mode) {
    const int threads = mode == 0 || mode == 3 || mode == 4 ? 64 : 1024;
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(threads), 0, 0, out, cyc, mode);
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(threads), 0, 0, out, cyc, mode);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    if (hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost) != hipSuccess) return 3;
    std::printf("\"diag_groups_%s\": %lld%s", names[mode], h, mode < 4 ? ", " : "");
  }
  std::printf("}\n");
  return 0;
}
