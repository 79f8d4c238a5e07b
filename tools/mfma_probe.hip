// mfma_probe — cycles per v_mfma_f64_16x16x4f64 on one SIMD for 1, 2, 4 and 8
// independent accumulation chains per wave (SrcC dependence only), and for a
// chain whose next MFMA takes the previous result as its B operand (the
// factor's diagonal chain), one wave per SIMD (256-thread workgroup, 1 / CU).
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));
#define MF(a, b, c) __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0)

template <int NACC>
__global__ __launch_bounds__(1024) void k_chain(double *out, long long *cyc, int iters) {
  const int lane = threadIdx.x & 63;
  double a = 1e-3 * lane, b = 1e-3 * (64 - lane);
  d4 acc[NACC];
#pragma unroll
  for (int q = 0; q < NACC; ++q) acc[q] = d4{0.0, 0.0, 0.0, (double)q};
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int q = 0; q < NACC; ++q) acc[q] = MF(a, b, acc[q]);
  }
  const long long t1 = clock64();
  double s = 0.0;
#pragma unroll
  for (int q = 0; q < NACC; ++q) s += acc[q][0] + acc[q][3];
  out[blockIdx.x * 1024 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = (t1 - t0);
}

// result as the next MFMA's B operand (element 0), plus a VALU read of it
__global__ __launch_bounds__(256) void k_hop(double *out, long long *cyc, int iters) {
  const int lane = threadIdx.x & 63;
  double a = 1e-3 * lane, b = 1e-3 * (64 - lane);
  const d4 z = {0.0, 0.0, 0.0, 0.0};
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
    const d4 x = MF(a, b, z);
    b = x[0] * 0.5 + 1e-3;
  }
  const long long t1 = clock64();
  out[blockIdx.x * 256 + threadIdx.x] = b;
  if (threadIdx.x == 0) cyc[blockIdx.x] = (t1 - t0);
}

// f32 16x16x4 MFMA (the guide: 32 cycles / SIMD issue) and v_fma_f64: clock calibration
template <int NACC>
__global__ __launch_bounds__(256) void k_f32(double *out, long long *cyc, int iters) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63;
  float a = 1e-3f * lane, b = 1e-3f * (64 - lane);
  f4 acc[NACC];
#pragma unroll
  for (int q = 0; q < NACC; ++q) acc[q] = f4{0.f, 0.f, 0.f, (float)q};
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int q = 0; q < NACC; ++q) acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[q], 0, 0, 0);
  }
  const long long t1 = clock64();
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < NACC; ++q) s += acc[q][0] + acc[q][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = (t1 - t0);
}
__global__ __launch_bounds__(1024) void k_fma64(double *out, long long *cyc, int iters) {
  const int lane = threadIdx.x & 63;
  double x[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) x[q] = 1e-3 * (lane + q);
  const double m = 0.999, c = 1e-6;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int q = 0; q < 8; ++q) x[q] = fma(x[q], m, c);
  }
  const long long t1 = clock64();
  double s = 0.0;
#pragma unroll
  for (int q = 0; q < 8; ++q) s += x[q];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = (t1 - t0);
}
// clock rate: s_memtime ticks per s_memrealtime tick (100 MHz)
__global__ void k_clock(long long *o, int iters) {
  const long long a = __builtin_amdgcn_s_memtime(), ra = __builtin_amdgcn_s_memrealtime();
  double x = threadIdx.x;
  for (int i = 0; i < iters; ++i) x = fma(x, 0.9999, 1e-7);
  const long long b = __builtin_amdgcn_s_memtime(), rb = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { o[2 * blockIdx.x] = b - a; o[2 * blockIdx.x + 1] = rb - ra; }
  if (x == 12345.0) o[0] = 0;
}

int main() {
  double *out;
  long long *cyc, h[256];
  if (hipMalloc(&out, 1024 * 1024 * 8) != hipSuccess || hipMalloc(&cyc, 1024 * 8) != hipSuccess) return 1;
  const int iters = 2000;
  auto rep = [&](const char *name, int per_iter) {
    hipMemcpy(h, cyc, 256 * 8, hipMemcpyDeviceToHost);
    long long s = 0;
    for (int i = 0; i < 256; ++i) s += h[i];
    std::printf("\"%s\": %.1f, ", name, (double)s / 256 / iters / per_iter);
  };
  std::printf("{\"cycles_per_mfma\": {");
#define RUN(K, NAME, PER)                                                         \
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(K, dim3(256), dim3(256), 0, 0, out, cyc, iters); \
  hipDeviceSynchronize();                                                       \
  rep(NAME, PER);
  RUN(k_chain<1>, "srcC_chain_1acc", 1)
  RUN(k_chain<2>, "srcC_chain_2acc", 2)
  RUN(k_chain<4>, "srcC_chain_4acc", 4)
  RUN(k_chain<8>, "srcC_chain_8acc", 8)
  RUN(k_hop, "result_to_B_plus_valu", 1)
  RUN(k_f32<8>, "f32_16x16x4_8acc", 8)
  // several waves per SIMD: cycles per MFMA of the workgroup's first wave. It
  // runs at the lone-wave rate (the oldest wave wins the arbitration; the
  // others wait), so this is no SIMD throughput -- the chip test below is.
  for (int wps = 2; wps <= 4; wps *= 2) {
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k_chain<4>, dim3(256), dim3(256 * wps), 0, 0, out, cyc, iters);
    hipDeviceSynchronize();
    hipMemcpy(h, cyc, 256 * 8, hipMemcpyDeviceToHost);
    long long s2 = 0;
    for (int i = 0; i < 256; ++i) s2 += h[i];
    std::printf("\"f64_4acc_first_of_%d_waves_per_simd\": %.1f, ", wps, (double)s2 / 256 / iters / 4);
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k_chain<1>, dim3(256), dim3(256 * wps), 0, 0, out, cyc, iters);
    hipDeviceSynchronize();
    hipMemcpy(h, cyc, 256 * 8, hipMemcpyDeviceToHost);
    s2 = 0;
    for (int i = 0; i < 256; ++i) s2 += h[i];
    std::printf("\"f64_1acc_first_of_%d_waves_per_simd\": %.1f, ", wps, (double)s2 / 256 / iters / 1);
  }
  RUN(k_fma64, "v_fma_f64_8chains", 8)
  for (int wps = 2; wps <= 4; wps *= 2) {  // f64 VALU with several waves per SIMD: chip time per instruction per SIMD
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int it2 = 20000;
    hipLaunchKernelGGL(k_fma64, dim3(256), dim3(256 * wps), 0, 0, out, cyc, it2);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k_fma64, dim3(256), dim3(256 * wps), 0, 0, out, cyc, it2);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    // wave-instructions per SIMD = 4 * wps waves per CU / 4 SIMDs * it2 * 8
    const double inst = (double)wps * it2 * 8;
    std::printf("\"v_fma_f64_%d_waves_per_simd_cycles\": %.2f, ", wps, ms * 1e-3 * 2.39e9 / inst);
  }
  {
    long long *co, hc[512];
    hipMalloc(&co, 512 * 8);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k_clock, dim3(256), dim3(256), 0, 0, co, 2000000);
    hipDeviceSynchronize();
    hipMemcpy(hc, co, 512 * 8, hipMemcpyDeviceToHost);
    double r = 0;
    for (int i = 0; i < 256; ++i) r += (double)hc[2 * i] / (double)hc[2 * i + 1];
    std::printf("\"shader_clock_MHz\": %.0f, ", r / 256 * 100.0);
  }
  // chip throughput: hipEvent-timed grid of k_chain<4> (f64) and k_f32<8>
  {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int blocks : {256, 512, 1024}) {
      for (int thr : {256, 512, 1024}) {
        const int it2 = 4000;
        hipLaunchKernelGGL(k_chain<4>, dim3(blocks), dim3(thr), 0, 0, out, cyc, it2);
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k_chain<4>, dim3(blocks), dim3(thr), 0, 0, out, cyc, it2);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0.f;
        hipEventElapsedTime(&ms, e0, e1);
        const double fl = (double)blocks * (thr / 64) * it2 * 4 * 2048.0;
        std::printf("\"f64_TFLOPs_%dx%d\": %.1f, ", blocks, thr, fl / (ms * 1e-3) / 1e12);
      }
    }
  }
  std::printf("\"end\": 0}}\n");
  return 0;
}
