// simd_probe — which SIMD each wave of a 4-wave workgroup lands on, with 3
// workgroups resident per CU (the tile kernel's shape: 256 threads, ~41 KB of
// LDS). If wave 0 of every workgroup shares one SIMD, work that only wave 0
// does (the tile kernel's batch staging) piles onto that SIMD.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ __launch_bounds__(256) void k_where(int *out, int iters) {
  __shared__ double pad[5000];  // ~40 KB: three workgroups per CU
  const int w = threadIdx.x >> 6;
  // HW_REG_HW_ID (id 4), all 32 bits: wave_id[3:0] simd_id[5:4] cu_id[11:8] se_id[15:13]
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4) & 0xFFFF;
  const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20) & 0xF;  // HW_REG_XCC_ID
  double x = threadIdx.x;
  for (int i = 0; i < iters; ++i) x = fma(x, 0.999, 1e-3);  // keep the workgroups resident together
  pad[threadIdx.x] = x;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + w] = (int)(hw | xcc << 16) + (pad[0] == 12345.0 ? 1 : 0);
}

int main() {
  const int nb = 768;
  int *d, h[nb * 4];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
  hipLaunchKernelGGL(k_where, dim3(nb), dim3(256), 0, 0, d, 200000);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  // histogram: wave index within the workgroup x SIMD id
  int hist[4][4] = {};
  int same_simd_wave0 = 0, groups = 0;
  for (int b = 0; b < nb; ++b)
    for (int w = 0; w < 4; ++w) hist[w][(h[4 * b + w] >> 4) & 3]++;
  // per CU (se, cu): the SIMDs of the wave-0s of its workgroups
  for (int b = 0; b < nb; ++b)
    for (int c = b + 1; c < nb; ++c) {
      // same CU: equal xcc, se, sh and cu fields (bits 8..19 of the packed id)
      if (((h[4 * b] ^ h[4 * c]) & 0xFFF00) == 0) {
        groups++;
        same_simd_wave0 += ((h[4 * b] >> 4) & 3) == ((h[4 * c] >> 4) & 3);
      }
    }
  std::printf("{\"wave_x_simd\": [");
  for (int w = 0; w < 4; ++w)
    std::printf("[%d, %d, %d, %d]%s", hist[w][0], hist[w][1], hist[w][2], hist[w][3], w < 3 ? ", " : "");
  std::printf("], \"same_cu_pairs\": %d, \"wave0_same_simd\": %d}\n", groups, same_simd_wave0);
  return 0;
}
