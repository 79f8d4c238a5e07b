// dense_check — residual check of the dense blocked Cholesky solve
// (launch_dense_spd_solve, sqlm_rcs_solve.hip) on a random SPD system.
// Usage: dense_check [n] (a multiple of 112). Prints one JSON line.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../sqrtlm-slam_amd/csrc/sqlm_rcs_solve.hip"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 2; } } while (0)

int main(int argc, char **argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 336;
  if (n % sqlm::kCRMaxN) { std::printf("n must be a multiple of %d\n", sqlm::kCRMaxN); return 1; }
  std::mt19937_64 rng(5);
  std::uniform_real_distribution<double> U(-0.5, 0.5);
  std::vector<double> A((size_t)n * n), b(n);
  for (int r = 0; r < n; ++r)
    for (int c = 0; c <= r; ++c) A[(size_t)r * n + c] = A[(size_t)c * n + r] = (r == c ? 2.0 * std::sqrt((double)n) + 1 : 0.0) + U(rng) / std::sqrt((double)n);
  for (auto &v : b) v = U(rng);
  double *dA, *dL, *dLi, *dr, *dx;
  int *df;
  const int nblk = n / sqlm::kCRMaxN;
  CK(hipMalloc(&dA, A.size() * 8)); CK(hipMalloc(&dL, A.size() * 8));
  CK(hipMalloc(&dLi, (size_t)nblk * sqlm::kCRMaxN * sqlm::kCRMaxN * 8));
  CK(hipMalloc(&dr, n * 8)); CK(hipMalloc(&dx, n * 8)); CK(hipMalloc(&df, 16));
  CK(hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dr, b.data(), n * 8, hipMemcpyHostToDevice));
  const int one = 1;
  CK(hipMemcpy(df, &one, 4, hipMemcpyHostToDevice));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  if (sqlm::launch_dense_spd_solve(dA, dL, dLi, dr, dx, df, n, st)) { std::printf("launch failed\n"); return 2; }
  CK(hipStreamSynchronize(st));
  std::vector<double> x(n);
  int flag = 0;
  CK(hipMemcpy(x.data(), dx, n * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&flag, df, 4, hipMemcpyDeviceToHost));
  double res = 0, bn = 0;
  for (int r = 0; r < n; ++r) {
    double s = 0;
    for (int c = 0; c < n; ++c) s += A[(size_t)r * n + c] * x[c];
    res = std::fmax(res, std::fabs(s - b[r]));
    bn = std::fmax(bn, std::fabs(b[r]));
  }
  // per-block diagnosis: L_00 L_00^T == A_00 ?
  std::vector<double> Li((size_t)sqlm::kCRMaxN * sqlm::kCRMaxN);
  CK(hipMemcpy(Li.data(), dLi, Li.size() * 8, hipMemcpyDeviceToHost));
  double e0 = 0;  // (Linv A00 Linv^T) - I on block 0
  const int nb = sqlm::kCRMaxN;
  for (int i = 0; i < nb; ++i)
    for (int j = 0; j < nb; ++j) {
      double s = 0;
      for (int p = 0; p < nb; ++p) {
        double t = 0;
        for (int q = 0; q < nb; ++q) t += A[(size_t)p * n + q] * Li[(size_t)j * nb + q];
        s += Li[(size_t)i * nb + p] * t;
      }
      e0 = std::fmax(e0, std::fabs(s - (i == j ? 1.0 : 0.0)));
    }
  std::printf("{\"n\": %d, \"flag\": %d, \"rel_residual\": %.3e, \"block0_LinvALinvT_minus_I\": %.3e}\n", n, flag,
              res / bn, e0);
  return 0;
}
