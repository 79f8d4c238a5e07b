// mfma44_probe — v_mfma_f64_4x4x4f64 (four independent 4x4x4 blocks per
// instruction) on gfx950: (1) issue cycles per instruction on one SIMD for 1..8
// independent accumulation chains, next to v_mfma_f64_16x16x4f64; (2) the
// operand / result lane layout, found by one-hot experiments: wave w puts 1.0
// in lane la = w / 64 of A and lane lb = w % 64 of B, everything else 0; the
// lanes of D that become non-zero are where a_la * b_lb lands.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC, bool BIG>
__global__ __launch_bounds__(256) void k_rate(double *out, long long *cyc, int iters) {
  const int lane = threadIdx.x & 63;
  double a = 1e-3 * lane, b = 1e-3 * (64 - lane);
  double acc[NACC];
  d4 acc4[NACC];
#pragma unroll
  for (int q = 0; q < NACC; ++q) {
    acc[q] = q;
    acc4[q] = d4{0.0, 0.0, 0.0, (double)q};
  }
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int q = 0; q < NACC; ++q) {
      if (BIG) acc4[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc4[q], 0, 0, 0);
      else acc[q] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[q], 0, 0, 0);
    }
  }
  const long long t1 = clock64();
  double s = 0.0;
#pragma unroll
  for (int q = 0; q < NACC; ++q) s += acc[q] + acc4[q][0] + acc4[q][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ __launch_bounds__(64) void k_layout(double *out) {
  const int w = blockIdx.x, lane = threadIdx.x, la = w / 64, lb = w % 64;
  const double a = lane == la ? 1.0 : 0.0, b = lane == lb ? 1.0 : 0.0;
  out[64 * w + lane] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

template <int NACC, bool BIG>
int rate(double *out, long long *cyc) {
  const int iters = 4096;
  hipLaunchKernelGGL((k_rate<NACC, BIG>), dim3(1), dim3(64), 0, 0, out, cyc, iters);  // one wave
  CK(hipDeviceSynchronize());
  long long c = 0;
  CK(hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost));
  std::printf("{\"op\": \"%s\", \"chains\": %d, \"cycles_per_mfma\": %.2f}\n", BIG ? "f64_16x16x4" : "f64_4x4x4",
              NACC, (double)c / iters / NACC);
  return 0;
}

int main() {
  double *out = nullptr;
  long long *cyc = nullptr;
  CK(hipMalloc(&out, 4096 * 64 * sizeof(double)));
  CK(hipMalloc(&cyc, 64 * sizeof(long long)));
  if (rate<1, false>(out, cyc) || rate<2, false>(out, cyc) || rate<4, false>(out, cyc) || rate<8, false>(out, cyc) ||
      rate<1, true>(out, cyc) || rate<4, true>(out, cyc))
    return 1;
  hipLaunchKernelGGL(k_layout, dim3(4096), dim3(64), 0, 0, out);
  CK(hipDeviceSynchronize());
  std::vector<double> h(4096 * 64);
  CK(hipMemcpy(h.data(), out, h.size() * sizeof(double), hipMemcpyDeviceToHost));
  // per A lane: "la: lb->dlane ..." for every (lb, dlane) with D != 0
  for (int la = 0; la < 64; ++la) {
    std::printf("A%d:", la);
    for (int lb = 0; lb < 64; ++lb)
      for (int l = 0; l < 64; ++l)
        if (h[64 * (64 * la + lb) + l] != 0.0) std::printf(" %d>%d", lb, l);
    std::printf("\n");
  }
  return 0;
}
