// lat_probe — per-instruction latency / issue probes on gfx950 for the CR
// factor redesign (one wave, clock64 around dependent or independent chains).
// Prints one JSON line of cycles per operation.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

#define N_IT 256

__device__ __forceinline__ double rl(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

__global__ void k_probe(double *out, long long *cyc, double seed) {
  const int lane = threadIdx.x;
  double x = seed + lane * 1e-3, a = 0.999999, b = 1e-7;
  d4 acc = {x, x, x, x}, acc2 = acc, acc3 = acc, acc4 = acc;
  long long t0, t1;
  int slot = 0;
  // 1. dependent f64 FMA chain
  t0 = clock64();
#pragma unroll 16
  for (int i = 0; i < N_IT; ++i) x = fma(x, a, b);
  t1 = clock64();
  if (lane == 0) cyc[slot] = t1 - t0;
  ++slot;
  // 2. 4 independent f64 FMA chains (issue rate)
  double y0 = x, y1 = x + 1, y2 = x + 2, y3 = x + 3;
  t0 = clock64();
#pragma unroll 16
  for (int i = 0; i < N_IT; ++i) {
    y0 = fma(y0, a, b); y1 = fma(y1, a, b); y2 = fma(y2, a, b); y3 = fma(y3, a, b);
  }
  t1 = clock64();
  if (lane == 0) cyc[slot] = t1 - t0;
  ++slot;
  x = y0 + y1 + y2 + y3;
  // 3. dependent f64 MFMA 16x16x4 (accumulator chain)
  t0 = clock64();
#pragma unroll 8
  for (int i = 0; i < 64; ++i) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  t1 = clock64();
  if (lane == 0) cyc[slot] = t1 - t0;
  ++slot;
  // 4. four independent MFMA accumulators
  t0 = clock64();
#pragma unroll 8
  for (int i = 0; i < 64; ++i) {
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc2, 0, 0, 0);
    acc3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc3, 0, 0, 0);
    acc4 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc4, 0, 0, 0);
  }
  t1 = clock64();
  if (lane == 0) cyc[slot] = t1 - t0;
  ++slot;
  // 5. MFMA result -> operand of the next MFMA (A operand from acc[0])
  double op = acc[0];
  t0 = clock64();
#pragma unroll 8
  for (int i = 0; i < 64; ++i) {
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(op, b, acc, 0, 0, 0);
    op = acc[1];
  }
  t1 = clock64();
  if (lane == 0) cyc[slot] = t1 - t0;
  ++slot;
  // 6. MFMA -> readlane -> fma -> MFMA operand (the per-group chain)
  t0 = clock64();
#pragma unroll 8
  for (int i = 0; i < 64; ++i) {
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(op, b, acc, 0, 0, 0);
    const double s = rl(acc[2], 5);
    op = fma(s, a, op);
  }
  t1 = clock64();
  if (lane == 0) cyc[slot] = t1 - t0;
  ++slot;
  // 7. dependent v_rsq_f64 + one Newton step chain
  double r = fabs(op) + 1.0;
  t0 = clock64();
#pragma unroll 8
  for (int i = 0; i < 64; ++i) {
    double y = __builtin_amdgcn_rsq(r);
    const double h = 0.5 * r * y;
    y = fma(y, fma(-h, y, 0.5), y);
    r = y + 1.0;
  }
  t1 = clock64();
  if (lane == 0) cyc[slot] = t1 - t0;
  ++slot;
  // 8. 32 independent readlanes (f64 = 2 each) summed
  double s8 = 0.0;
  t0 = clock64();
#pragma unroll
  for (int i = 0; i < 16; ++i) s8 += rl(r + i, i);
  t1 = clock64();
  if (lane == 0) cyc[slot] = t1 - t0;
  ++slot;
  // 9. dependent readlane chain (value -> readlane -> fma -> readlane ...)
  double c9 = s8;
  t0 = clock64();
#pragma unroll 8
  for (int i = 0; i < 64; ++i) c9 = fma(rl(c9, i & 63), a, lane * 1e-9);
  t1 = clock64();
  if (lane == 0) cyc[slot] = t1 - t0;
  ++slot;
  // 10. permlane32_swap dependent chain (f64 = 2 swaps)
  double c10 = c9;
  t0 = clock64();
#pragma unroll 8
  for (int i = 0; i < 64; ++i) {
    const int lo = __double2loint(c10), hi = __double2hiint(c10);
    const auto pl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto ph = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    c10 = fma(__hiloint2double(ph[0], pl[0]), a, b);
  }
  t1 = clock64();
  if (lane == 0) cyc[slot] = t1 - t0;
  ++slot;
  // 11. ds_bpermute (shfl) dependent chain on f64
  double c11 = c10;
  t0 = clock64();
#pragma unroll 8
  for (int i = 0; i < 64; ++i) c11 = fma(__shfl(c11, (lane + 16) & 63, 64), a, b);
  t1 = clock64();
  if (lane == 0) cyc[slot] = t1 - t0;
  ++slot;
  // 12. dependent f64 multiply chain
  double c12 = c11;
  t0 = clock64();
#pragma unroll 16
  for (int i = 0; i < N_IT; ++i) c12 = c12 * a;
  t1 = clock64();
  if (lane == 0) cyc[slot] = t1 - t0;
  ++slot;
  out[lane] = x + acc[0] + acc2[1] + acc3[2] + acc4[3] + r + s8 + c9 + c10 + c11 + c12;
}

// LDS round trip: one lane writes, barrier-free wave read-back (wave_barrier)
__global__ void k_lds(double *out, long long *cyc) {
  __shared__ double buf[64];
  const int lane = threadIdx.x;
  double v = lane;
  long long t0 = clock64();
  for (int i = 0; i < 64; ++i) {
    if (lane == (i & 15)) buf[0] = v;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    v = buf[0] * 0.5 + lane;
    __builtin_amdgcn_wave_barrier();
  }
  long long t1 = clock64();
  if (lane == 0) cyc[0] = t1 - t0;
  out[lane] = v;
}

// __syncthreads round trip in an 8-wave workgroup
__global__ void k_bar(double *out, long long *cyc) {
  __shared__ double buf[512];
  const int t = threadIdx.x;
  double v = t;
  long long t0 = clock64();
  for (int i = 0; i < 64; ++i) {
    buf[t] = v;
    __syncthreads();
    v = buf[(t + 64) & 511] * 0.5;
    __syncthreads();
  }
  long long t1 = clock64();
  if (t == 0) cyc[0] = t1 - t0;
  out[t] = v;
}

int main() {
  double *out;
  long long *cyc, h[16];
  hipMalloc(&out, 512 * 8);
  hipMalloc(&cyc, 16 * 8);
  hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, out, cyc, 0.5);
  hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, out, cyc, 0.5);
  hipDeviceSynchronize();
  hipMemcpy(h, cyc, 16 * 8, hipMemcpyDeviceToHost);
  const char *names[] = {"fma_f64_dep", "fma_f64_4indep", "mfma_f64_dep", "mfma_f64_4indep", "mfma_acc_to_operand",
                         "mfma_readlane_fma", "rsq_newton_dep", "readlane16_f64", "readlane_dep",
                         "permlane32_swap_f64_dep", "bpermute_f64_dep", "mul_f64_dep"};
  const double per[] = {N_IT, N_IT, 64, 64, 64, 64, 64, 16, 64, 64, 64, N_IT};
  std::printf("{");
  for (int i = 0; i < 12; ++i) std::printf("\"%s\": %.1f, ", names[i], h[i] / per[i]);
  hipLaunchKernelGGL(k_lds, dim3(1), dim3(64), 0, 0, out, cyc);
  hipDeviceSynchronize();
  hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost);
  std::printf("\"lds_roundtrip\": %.1f, ", h[0] / 64.0);
  hipLaunchKernelGGL(k_bar, dim3(1), dim3(512), 0, 0, out, cyc);
  hipDeviceSynchronize();
  hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost);
  std::printf("\"syncthreads_pair_8w\": %.1f}\n", h[0] / 64.0);
  return 0;
}
