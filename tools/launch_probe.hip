// launch_probe — host time per hipLaunchKernelGGL as a function of the size of
// the by-value kernel argument (64 B ... 2 KB, empty kernels, no sync inside
// the timed loop), and the GPU-side gap between back-to-back dispatches
// (events around a run of launches). Tells whether the per-launch host cost of
// the 984-byte DevProblem kernels comes from the argument size.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

template <int B>
struct Arg {
  long long v[B / 8];
};

template <int B>
__global__ void k_empty(Arg<B> a, int *out) {
  if (a.v[B / 8 - 1] == 12345 && threadIdx.x == 0) out[blockIdx.x] = 1;
}

template <int B>
void probe(int *out, hipStream_t st) {
  Arg<B> a{};
  const int n = 2000;
  for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(k_empty<B>, dim3(1), dim3(64), 0, st, a, out);
  (void)hipStreamSynchronize(st);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, st);
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) {
    a.v[0] = i;
    hipLaunchKernelGGL(k_empty<B>, dim3(1), dim3(64), 0, st, a, out);
  }
  const auto t1 = std::chrono::steady_clock::now();
  (void)hipEventRecord(e1, st);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double host_us = std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
  std::printf("{\"arg_bytes\": %d, \"host_us_per_launch\": %.2f, \"gpu_us_per_launch\": %.2f}\n", B, host_us,
              1e3 * ms / n);
}

int main() {
  int *out;
  if (hipMalloc(&out, 4096) != hipSuccess) return 1;
  hipStream_t st;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return 1;
  probe<64>(out, st);
  probe<128>(out, st);
  probe<256>(out, st);
  probe<512>(out, st);
  probe<1024>(out, st);
  probe<2048>(out, st);
  probe<64>(out, st);
  probe<1024>(out, st);
  return 0;
}
