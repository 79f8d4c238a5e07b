// sqlm_orb.hip — ORB front end on gfx950:
// ORBextractor::operator() (src/frontend/ORBextractor.cc:1284-1399) and
// ORBmatcher::SearchForInitialization / DescriptorDistance
// (src/frontend/ORBmatcher.cc:573-718, :2096-2116), bit-exact with the CPU
// restatement in oracle/orb_ref.c.
//
// Extraction pipeline for one image (all levels in flight on one stream):
//   k_orb_resize    level l from level l-1, one thread per output pixel
//                   (OpenCV INTER_LINEAR fixed point, SSE2 vertical rounding
//                   below the vector end, scalar after — see orb_ref.c);
//   k_orb_fast      one workgroup per 30-px cell of every level: the cell view
//                   (<= 72x72) is staged in LDS, FAST-9/16 score per pixel,
//                   3x3 non-max suppression, the minThFAST retry when the cell
//                   is empty, and a ballot compaction that keeps OpenCV's
//                   row-major emission order;
//   k_orb_scan / k_orb_compact   cell counts -> one contiguous candidate list
//                   per level in the reference's cell order (4 B each);
//   host            DistributeOctTree (ORBextractor.cc:692-1043) on the
//                   candidates: a serial list algorithm whose output order is
//                   part of the result, so it stays a host step;
//   k_orb_blur      GaussianBlur 7x7 sigma 2 per level, LDS tile with halo
//                   (integer row pass, float column pass as OpenCV's SSE2);
//   k_orb_describe  one wavefront per keypoint: intensity-centroid moments
//                   (IC_Angle) by lane-parallel integer sums + fastAtan2, then
//                   256 steered-BRIEF tests, 4 per lane, nibbles merged by a
//                   lane shuffle.
// Matching: k_orb_bf (one thread per query, train descriptors staged through
// LDS, v_bcnt popcounts) and, for the windowed searches, k_area_list (one
// wavefront per query enumerates the frame grid window in the reference's
// order and emits (candidate, distance) pairs); the order-dependent
// acceptance loop (vMatchedDistance, vnMatches21, rotation histogram) runs on
// the host over those lists.
//
// Compiled with -ffp-contract=off: the reference is built in ISO C++ mode
// (CMakeLists.txt:4), where GCC does not contract a*b+c into an FMA.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstring>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/sqrtlm_orb.h"
#include "orb_pattern.h"
#include "sqlm_internal.h"

namespace sqlm {

namespace {

constexpr int kEdge = 19;       // EDGE_THRESHOLD (ORBextractor.cc:78)
constexpr int kPatch = 31;      // PATCH_SIZE (:76)
constexpr int kHalf = 15;       // HALF_PATCH_SIZE
constexpr int kCellMax = 72;    // largest FAST view side (cell <= 60 + 6 overlap)
constexpr int kCellCap = 1024;  // candidates per cell (3x3 NMS: <= 33 x 33)
constexpr int kMaxLevels = 16;
constexpr int kGridCols = 64, kGridRows = 48;  // FRAME_GRID_COLS / ROWS (Frame.h:70-75)
constexpr int kHistoLength = 30, kThLow = 50, kThHigh = 100;  // ORBmatcher.cc:46-48

struct OrbCell {
  int img_off, pitch;  // level image in the packed pyramid
  int x0, y0, w, h;    // FAST view
  int offx, offy;      // j*wCell, i*hCell (coordinates relative to minBorder)
};

struct OrbDescIn {
  float x, y, response;
  int level;
};

struct LevelTab {
  int off[kMaxLevels], pitch[kMaxLevels];
  float scale[kMaxLevels], size[kMaxLevels];
  int umax[kHalf + 1];
};

__device__ __forceinline__ int d_floor(float v) {
  const int i = (int)v;
  return i - (i > v);
}
__device__ __forceinline__ int d_round(float v) { return (int)__builtin_rintf(v); }  // cvRound: half to even
__device__ __forceinline__ int d_sat_short(float v) {
  const int r = d_round(v);
  return r < -32768 ? -32768 : r > 32767 ? 32767 : r;
}
__device__ __forceinline__ int d_sat16(int v) { return v < -32768 ? -32768 : v > 32767 ? 32767 : v; }
__device__ __forceinline__ int d_sat_u8(int v) { return v < 0 ? 0 : v > 255 ? 255 : v; }

// ---- pyramid ------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_orb_resize(const uint8_t *__restrict__ src, int sw, int sh,
                                                    uint8_t *__restrict__ dst, int dw, int dh, double scale_x,
                                                    double scale_y, int vend) {
  const int dx = blockIdx.x * blockDim.x + threadIdx.x, dy = blockIdx.y;
  if (dx >= dw || dy >= dh) return;
  float fx = (float)((dx + 0.5) * scale_x - 0.5);
  int sx = d_floor(fx);
  fx -= sx;
  if (sx < 0) fx = 0, sx = 0;
  const bool tail = sx + 1 >= sw;  // dx >= xmax (sx is monotone in dx)
  if (tail && sx >= sw - 1) fx = 0, sx = sw - 1;
  const int a0 = d_sat_short((1.f - fx) * 2048), a1 = d_sat_short(fx * 2048);
  float fy = (float)((dy + 0.5) * scale_y - 0.5);
  int sy = d_floor(fy);
  fy -= sy;
  const int b0 = d_sat_short((1.f - fy) * 2048), b1 = d_sat_short(fy * 2048);
  const int y0 = min(max(sy, 0), sh - 1), y1 = min(max(sy + 1, 0), sh - 1);
  const uint8_t *S0 = src + (size_t)y0 * sw, *S1 = src + (size_t)y1 * sw;
  const int r0 = tail ? S0[sx] * 2048 : S0[sx] * a0 + S0[sx + 1] * a1;
  const int r1 = tail ? S1[sx] * 2048 : S1[sx] * a0 + S1[sx + 1] * a1;
  int v;
  if (dx < vend) {
    const int a = d_sat16(r0 >> 4), c = d_sat16(r1 >> 4);
    const int m = d_sat16(((a * b0) >> 16) + ((c * b1) >> 16));
    v = d_sat16(m + 2) >> 2;
  } else {
    v = (r0 * b0 + r1 * b1 + (1 << 21)) >> 22;
  }
  dst[(size_t)dy * dw + dx] = (uint8_t)d_sat_u8(v);
}

// ---- FAST-9/16 per cell --------------------------------------------------------
__constant__ int c_fast_off[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},   {3, 0},  {3, -1}, {2, -2}, {1, -3},
                                      {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

// cornerScore<16> (OpenCV fast_score.cpp) on an LDS view with row pitch kCellMax.
__device__ int fast_corner_score(const uint8_t *ptr, const int *pixel, int threshold) {
  int d[25];
  const int v = ptr[0];
#pragma unroll
  for (int k = 0; k < 25; ++k) d[k] = v - ptr[pixel[k]];
  int a0 = threshold;
#pragma unroll
  for (int k = 0; k < 16; k += 2) {
    int a = min(d[k + 1], d[k + 2]);
    a = min(a, d[k + 3]);
    if (a <= a0) continue;
    a = min(a, d[k + 4]);
    a = min(a, d[k + 5]);
    a = min(a, d[k + 6]);
    a = min(a, d[k + 7]);
    a = min(a, d[k + 8]);
    a0 = max(a0, min(a, d[k]));
    a0 = max(a0, min(a, d[k + 9]));
  }
  int b0 = -a0;
#pragma unroll
  for (int k = 0; k < 16; k += 2) {
    int b = max(d[k + 1], d[k + 2]);
    b = max(b, d[k + 3]);
    b = max(b, d[k + 4]);
    b = max(b, d[k + 5]);
    if (b >= b0) continue;
    b = max(b, d[k + 6]);
    b = max(b, d[k + 7]);
    b = max(b, d[k + 8]);
    b0 = min(b0, max(b, d[k]));
    b0 = min(b0, max(b, d[k + 9]));
  }
  return -b0 - 1;
}

// The FAST test of OpenCV's FAST_t<16> for one pixel: 0 if not a corner, else
// its score (>= threshold - 1 > 0 for the thresholds used).
__device__ int fast_pixel(const uint8_t *ptr, const int *pixel, int threshold) {
  const int v = ptr[0];
  auto cls = [&](int x) { const int i = x - v; return i < -threshold ? 1 : i > threshold ? 2 : 0; };
  int d = cls(ptr[pixel[0]]) | cls(ptr[pixel[8]]);
  if (d == 0) return 0;
  d &= cls(ptr[pixel[2]]) | cls(ptr[pixel[10]]);
  d &= cls(ptr[pixel[4]]) | cls(ptr[pixel[12]]);
  d &= cls(ptr[pixel[6]]) | cls(ptr[pixel[14]]);
  if (d == 0) return 0;
  d &= cls(ptr[pixel[1]]) | cls(ptr[pixel[9]]);
  d &= cls(ptr[pixel[3]]) | cls(ptr[pixel[11]]);
  d &= cls(ptr[pixel[5]]) | cls(ptr[pixel[13]]);
  d &= cls(ptr[pixel[7]]) | cls(ptr[pixel[15]]);
  if (d & 1) {
    const int vt = v - threshold;
    int count = 0;
    for (int k = 0; k < 25; k++) {
      if (ptr[pixel[k]] < vt) {
        if (++count > 8) return fast_corner_score(ptr, pixel, threshold);
      } else
        count = 0;
    }
  }
  if (d & 2) {
    const int vt = v + threshold;
    int count = 0;
    for (int k = 0; k < 25; k++) {
      if (ptr[pixel[k]] > vt) {
        if (++count > 8) return fast_corner_score(ptr, pixel, threshold);
      } else
        count = 0;
    }
  }
  return 0;
}

__global__ __launch_bounds__(256) void k_orb_fast(const uint8_t *__restrict__ pyr, const OrbCell *__restrict__ cells,
                                                  int ini_th, int min_th, uint32_t *__restrict__ out,
                                                  int *__restrict__ cnt) {
  __shared__ uint8_t pix[kCellMax * kCellMax];
  __shared__ uint8_t sc[kCellMax * kCellMax];
  __shared__ int wsum[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const OrbCell c = cells[blockIdx.x];
  const int n = c.w * c.h;
  for (int p = tid; p < n; p += 256) {
    const int y = p / c.w, x = p - y * c.w;
    pix[y * kCellMax + x] = pyr[c.img_off + (size_t)(c.y0 + y) * c.pitch + c.x0 + x];
  }
  int pixel[25];
#pragma unroll
  for (int k = 0; k < 16; ++k) pixel[k] = c_fast_off[k][0] + c_fast_off[k][1] * kCellMax;
#pragma unroll
  for (int k = 16; k < 25; ++k) pixel[k] = pixel[k - 16];
  auto keep = [&](int p) -> bool {
    const int y = p / c.w, x = p - y * c.w;
    if (y < 3 || y >= c.h - 3 || x < 3 || x >= c.w - 3) return false;
    const uint8_t *s = &sc[y * kCellMax + x];
    const int v = s[0];
    return v > 0 && v > s[1] && v > s[-1] && v > s[-kCellMax - 1] && v > s[-kCellMax] && v > s[-kCellMax + 1] &&
           v > s[kCellMax - 1] && v > s[kCellMax] && v > s[kCellMax + 1];
  };
  int th = min(max(ini_th, 0), 255);
  for (int pass = 0; pass < 2; ++pass) {
    for (int p = tid; p < kCellMax * kCellMax; p += 256) sc[p] = 0;
    __syncthreads();
    for (int p = tid; p < n; p += 256) {
      const int y = p / c.w, x = p - y * c.w;
      if (y < 3 || y >= c.h - 3 || x < 3 || x >= c.w - 3) continue;
      sc[y * kCellMax + x] = (uint8_t)fast_pixel(&pix[y * kCellMax + x], pixel, th);
    }
    __syncthreads();
    int mine = 0;
    for (int p = tid; p < n; p += 256) mine += keep(p);
    for (int m = 32; m >= 1; m >>= 1) mine += __shfl_xor(mine, m, 64);
    if (lane == 0) wsum[wave] = mine;
    __syncthreads();
    const int total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
    if (total > 0 || pass == 1) break;
    th = min(max(min_th, 0), 255);
  }
  // emission in row-major order (OpenCV pushes row i-1 after scanning row i)
  int base = 0;
  for (int r0 = 0; r0 < n; r0 += 256) {
    const int p = r0 + tid;
    const bool k = p < n && keep(p);
    const unsigned long long m = __ballot(k);
    const int pre = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wave] = __popcll(m);
    __syncthreads();
    int off = base;
    for (int w = 0; w < wave; ++w) off += wsum[w];
    if (k && off + pre < kCellCap) {
      const int y = p / c.w, x = p - y * c.w;
      out[(size_t)blockIdx.x * kCellCap + off + pre] =
          (uint32_t)(x + c.offx) | ((uint32_t)(y + c.offy) << 12) | ((uint32_t)sc[y * kCellMax + x] << 24);
    }
    base += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
  }
  if (tid == 0) cnt[blockIdx.x] = min(base, kCellCap);
}

// exclusive scan of n counts (one workgroup of 1024)
__global__ __launch_bounds__(1024) void k_orb_scan(const int *__restrict__ cnt, int n, int *__restrict__ off) {
  __shared__ int part[1024];
  const int t = threadIdx.x, chunk = (n + 1023) / 1024, b = t * chunk, e = min(n, b + chunk);
  int s = 0;
  for (int i = b; i < e; ++i) s += cnt[i];
  part[t] = s;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    const int v = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int run = t ? part[t - 1] : 0;
  for (int i = b; i < e; ++i) {
    off[i] = run;
    run += cnt[i];
  }
  if (t == 1023) off[n] = part[1023];
}

__global__ __launch_bounds__(256) void k_orb_compact(const uint32_t *__restrict__ cellkp, const int *__restrict__ cnt,
                                                     const int *__restrict__ off, uint32_t *__restrict__ outc) {
  const int c = blockIdx.x, n = cnt[c], o = off[c];
  for (int i = threadIdx.x; i < n; i += 256) outc[o + i] = cellkp[(size_t)c * kCellCap + i];
}

// ---- GaussianBlur 7x7, sigma 2, BORDER_REFLECT_101 ----------------------------------
struct BlurK {
  int ik[4];    // center .. edge, x256 integers
  float fk[4];  // ik / 65536 (SSE2 column kernel)
};

__device__ __forceinline__ int refl101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
  return i;
}

constexpr int kBTX = 32, kBTY = 8;
// all levels in one launch: block b belongs to the level whose tile range holds it
struct BlurLevels {
  int n;
  int off[kMaxLevels], w[kMaxLevels], h[kMaxLevels], tx[kMaxLevels], tile0[kMaxLevels + 1];
};

__global__ __launch_bounds__(256) void k_orb_blur(const uint8_t *__restrict__ pyr, uint8_t *__restrict__ blur,
                                                  BlurLevels lv, BlurK k) {
  __shared__ uint8_t pix[kBTY + 6][kBTX + 6];
  __shared__ int R[kBTY + 6][kBTX];
  int L = 0;
  while (L + 1 < lv.n && (int)blockIdx.x >= lv.tile0[L + 1]) ++L;
  const int b = blockIdx.x - lv.tile0[L], w = lv.w[L], h = lv.h[L];
  const uint8_t *src = pyr + lv.off[L];
  uint8_t *dst = blur + lv.off[L];
  const int tx = threadIdx.x % kBTX, ty = threadIdx.x / kBTX;
  const int x0 = (b % lv.tx[L]) * kBTX, y0 = (b / lv.tx[L]) * kBTY;
  for (int p = threadIdx.x; p < (kBTY + 6) * (kBTX + 6); p += 256) {
    const int yy = p / (kBTX + 6), xx = p - yy * (kBTX + 6);
    pix[yy][xx] = src[(size_t)refl101(y0 + yy - 3, h) * w + refl101(x0 + xx - 3, w)];
  }
  __syncthreads();
  for (int p = threadIdx.x; p < (kBTY + 6) * kBTX; p += 256) {
    const int yy = p / kBTX, xx = p - yy * kBTX;
    const uint8_t *s = &pix[yy][xx + 3];
    R[yy][xx] = k.ik[0] * s[0] + k.ik[1] * (s[1] + s[-1]) + k.ik[2] * (s[2] + s[-2]) + k.ik[3] * (s[3] + s[-3]);
  }
  __syncthreads();
  const int x = x0 + tx, y = y0 + ty;
  if (x >= w || y >= h) return;
  // the row sums of rows beyond the image come from reflected pixel rows, as
  // OpenCV's filter engine reflects the row buffer index
  int v;
  if (x < (w & ~3)) {
    float s = (float)R[ty + 3][tx] * k.fk[0];
    s = s + 0.0f;
#pragma unroll
    for (int j = 1; j <= 3; ++j) s = s + (float)(R[ty + 3 + j][tx] + R[ty + 3 - j][tx]) * k.fk[j];
    v = d_sat16((int)__builtin_rintf(s));
  } else {
    int s = k.ik[0] * R[ty + 3][tx];
#pragma unroll
    for (int j = 1; j <= 3; ++j) s += k.ik[j] * (R[ty + 3 + j][tx] + R[ty + 3 - j][tx]);
    v = (s + (1 << 15)) >> 16;
  }
  dst[(size_t)y * w + x] = (uint8_t)d_sat_u8(v);
}

// ---- orientation + steered BRIEF, one wavefront per keypoint -----------------------
__device__ float fast_atan2_deg(float y, float x) {
  const float p1 = 0.9997878412794807f * (float)(180 / 3.1415926535897932384626433832795);
  const float p3 = -0.3258083974640975f * (float)(180 / 3.1415926535897932384626433832795);
  const float p5 = 0.1555786518463281f * (float)(180 / 3.1415926535897932384626433832795);
  const float p7 = -0.04432655554792128f * (float)(180 / 3.1415926535897932384626433832795);
  const float ax = fabsf(x), ay = fabsf(y);
  float a, c, c2;
  if (ax >= ay) {
    c = __fdiv_rn(ay, ax + (float)2.2204460492503131e-16);
    c2 = c * c;
    a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  } else {
    c = __fdiv_rn(ax, ay + (float)2.2204460492503131e-16);
    c2 = c * c;
    a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  }
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

__global__ __launch_bounds__(256) void k_orb_describe(const uint8_t *__restrict__ pyr, const uint8_t *__restrict__ blur,
                                                      LevelTab tab, const signed char *__restrict__ pattern,
                                                      const OrbDescIn *__restrict__ in, int n,
                                                      sqlm_keypoint *__restrict__ kout, uint8_t *__restrict__ dout) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  const OrbDescIn q = in[i];
  const int L = q.level, step = tab.pitch[L];
  const int cx = d_round(q.x), cy = d_round(q.y);
  // IC_Angle (ORBextractor.cc:92-141): m_10 = sum u I, m_01 = sum v I over the disc
  const uint8_t *center = pyr + tab.off[L] + (size_t)cy * step + cx;
  int m10 = 0, m01 = 0;
  for (int v = -kHalf; v <= kHalf; ++v) {
    const int d = tab.umax[v < 0 ? -v : v];
    for (int u = -d + lane; u <= d; u += 64) {
      const int val = center[v * step + u];
      m10 += u * val;
      m01 += v * val;
    }
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    m10 += __shfl_xor(m10, m, 64);
    m01 += __shfl_xor(m01, m, 64);
  }
  const float angle = fast_atan2_deg((float)m01, (float)m10);
  // computeOrbDescriptor (:155-206) on the blurred level
  const float factorPI = (float)(3.1415926535897932384626433832795 / 180.f);
  const float ang = angle * factorPI;
  const float a = (float)cos((double)ang), b = (float)sin((double)ang);
  const uint8_t *bc = blur + tab.off[L] + (size_t)cy * step + cx;
  int nib = 0;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const signed char *pp = pattern + 4 * (4 * lane + t);
    const float x0 = (float)pp[0], y0 = (float)pp[1], x1 = (float)pp[2], y1 = (float)pp[3];
    const int t0 = bc[d_round(x0 * b + y0 * a) * step + d_round(x0 * a - y0 * b)];
    const int t1 = bc[d_round(x1 * b + y1 * a) * step + d_round(x1 * a - y1 * b)];
    nib |= (t0 < t1) << t;
  }
  int byte = nib << (4 * (lane & 1));
  byte |= __shfl_xor(byte, 1, 64);
  if (!(lane & 1)) dout[(size_t)32 * i + (lane >> 1)] = (uint8_t)byte;
  if (lane == 0) {
    sqlm_keypoint k;
    k.x = q.x;
    k.y = q.y;
    if (L != 0) {
      k.x *= tab.scale[L];
      k.y *= tab.scale[L];
    }
    k.size = tab.size[L];
    k.angle = angle;
    k.response = q.response;
    k.octave = L;
    kout[i] = k;
  }
}

// ---- Hamming matching ------------------------------------------------------------
__global__ __launch_bounds__(256) void k_orb_bf(const uint32_t *__restrict__ q, int nq, const uint32_t *__restrict__ t,
                                                int nt, int *__restrict__ bidx, int *__restrict__ bd,
                                                int *__restrict__ bd2) {
  __shared__ uint32_t tile[256][9];  // +1 word: conflict-free column reads
  const int qi = blockIdx.x * 256 + threadIdx.x;
  uint32_t my[8];
#pragma unroll
  for (int w = 0; w < 8; ++w) my[w] = qi < nq ? q[(size_t)8 * qi + w] : 0u;
  int best = INT_MAX, best2 = INT_MAX, bi = -1;
  for (int t0 = 0; t0 < nt; t0 += 256) {
    __syncthreads();
    for (int p = threadIdx.x; p < 256 * 8; p += 256) {
      const int r = p >> 3, w = p & 7;
      tile[r][w] = t0 + r < nt ? t[(size_t)8 * (t0 + r) + w] : 0u;
    }
    __syncthreads();
    const int m = min(256, nt - t0);
    for (int r = 0; r < m; ++r) {
      int dist = 0;
#pragma unroll
      for (int w = 0; w < 8; ++w) dist += __builtin_popcount(my[w] ^ tile[r][w]);
      if (dist < best) {
        best2 = best;
        best = dist;
        bi = t0 + r;
      } else if (dist < best2) {
        best2 = dist;
      }
    }
  }
  if (qi < nq) {
    bidx[qi] = bi;
    bd[qi] = best;
    bd2[qi] = best2;
  }
}

// One GetFeaturesInArea query: window centre, half-size r, and the level
// range packed as (minLevel & 0xffff) | (maxLevel << 16) (both int16);
// kAreaSkip marks a query the caller skips before the area search.
constexpr int kAreaSkip = (int)0x80008000;
__host__ __device__ inline int area_levels(int min_level, int max_level) {
  return (int)(((unsigned)min_level & 0xffffu) | ((unsigned)max_level << 16));
}

struct AreaArgs {
  const float4 *q;         // [n1] x y r levels(int bits)
  const uint32_t *d1;      // [n1][8] query descriptors
  const float *k2;         // [n2][4] x y octave pad
  const uint32_t *d2;      // [n2][8]
  const int *cell_ptr;     // [64*48+1] grid CSR (cell = ix*48 + iy)
  const int *cell_idx;     // keypoint indices in cell order
  float min_x, min_y, wi, hi;
  int n1;
};

// GetFeaturesInArea (Frame.cc:1463-1552) + DescriptorDistance for one query
// per wave: pass 0 counts the candidates, pass 1 writes (i2, dist) in the
// reference's iteration order (cells ix-major, then cell insertion order).
template <int PASS>
__global__ __launch_bounds__(256) void k_area_list(AreaArgs A, int *__restrict__ cnt, const int *__restrict__ off,
                                                   int2 *__restrict__ pairs) {
  const int lane = threadIdx.x & 63;
  const int i1 = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i1 >= A.n1) return;
  const float4 qv = A.q[i1];
  const float x = qv.x, y = qv.y, r = qv.z;
  const int lv = __float_as_int(qv.w);
  const int minLevel = (int)(short)(lv & 0xffff), maxLevel = lv >> 16;
  const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
  int run = 0;
  bool ok = lv != kAreaSkip;
  int nMinCellX = 0, nMaxCellX = -1, nMinCellY = 0, nMaxCellY = -1;
  if (ok) {
    nMinCellX = max(0, (int)floorf((x - A.min_x - r) * A.wi));
    ok = nMinCellX < kGridCols;
  }
  if (ok) {
    nMaxCellX = min(kGridCols - 1, (int)ceilf((x - A.min_x + r) * A.wi));
    ok = nMaxCellX >= 0;
  }
  if (ok) {
    nMinCellY = max(0, (int)floorf((y - A.min_y - r) * A.hi));
    ok = nMinCellY < kGridRows;
  }
  if (ok) {
    nMaxCellY = min(kGridRows - 1, (int)ceilf((y - A.min_y + r) * A.hi));
    ok = nMaxCellY >= 0;
  }
  uint32_t my[8];
  if (PASS == 1) {
#pragma unroll
    for (int w = 0; w < 8; ++w) my[w] = A.d1[(size_t)8 * i1 + w];
  }
  const int base = PASS == 1 ? off[i1] : 0;
  if (ok) {
    for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
      for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
        const int c = ix * kGridRows + iy, b = A.cell_ptr[c], e = A.cell_ptr[c + 1];
        for (int j0 = b; j0 < e; j0 += 64) {
          const int j = j0 + lane;
          bool hit = false;
          int i2 = 0;
          if (j < e) {
            i2 = A.cell_idx[j];
            const float kx = A.k2[4 * i2], ky = A.k2[4 * i2 + 1];
            const int oct = __float_as_int(A.k2[4 * i2 + 2]);
            hit = !bCheckLevels || (!(oct < minLevel) && !(maxLevel >= 0 && oct > maxLevel));
            const float distx = kx - x, disty = ky - y;
            hit = hit && fabsf(distx) < r && fabsf(disty) < r;
          }
          const unsigned long long m = __ballot(hit);
          if (PASS == 1 && hit) {
            int dist = 0;
#pragma unroll
            for (int w = 0; w < 8; ++w) dist += __builtin_popcount(my[w] ^ A.d2[(size_t)8 * i2 + w]);
            pairs[base + run + __popcll(m & ((1ull << lane) - 1ull))] = make_int2(i2, dist);
          }
          run += __popcll(m);
        }
      }
  }
  if (PASS == 0 && lane == 0) cnt[i1] = run;
}

// BoW node runs (SearchByBoW / SearchForTriangulation): query q = (feature
// of side 1, run [b, e) of side-2 features in cand, output offset); one wave
// per query, one candidate per lane: dist[off + j] = Hamming(d1[f], d2[cand[b + j]]).
__global__ __launch_bounds__(256) void k_cand_dist(const int4 *__restrict__ q, int nq, const uint32_t *__restrict__ d1,
                                                   const uint32_t *__restrict__ d2, const int *__restrict__ cand,
                                                   int *__restrict__ dist) {
  const int lane = threadIdx.x & 63;
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= nq) return;
  const int4 Q = q[w];
  uint32_t my[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) my[k] = d1[(size_t)8 * Q.x + k];
  for (int j = Q.y + lane; j < Q.z; j += 64) {
    const int i2 = cand[j];
    int d = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) d += __builtin_popcount(my[k] ^ d2[(size_t)8 * i2 + k]);
    dist[Q.w + (j - Q.y)] = d;
  }
}

// ---- host: DistributeOctTree (ORBextractor.cc:606-1043) -----------------------------
struct Cand {
  float x, y, response;
};

// Node pool + index-linked list with the reference's std::list semantics
// (push_front, erase-returns-next, iterator kept per expandable node); each
// node owns a contiguous slice of a key-index arena, children are filled by a
// stable 4-way partition, so key order inside a node is the reference's.
struct QNode {
  int ulx, uly, urx, ury, blx, bly, brx, bry;
  int koff, kcnt;
  int prev, next;
  bool no_more;
};

struct QuadTree {
  std::vector<QNode> pool;
  std::vector<int> arena;  // key indices
  std::vector<uint8_t> tag;
  int head = -1, size = 0;

  void push_front(int n) {
    pool[n].prev = -1;
    pool[n].next = head;
    if (head >= 0) pool[head].prev = n;
    head = n;
    ++size;
  }
  int erase(int n) {
    const int nx = pool[n].next, pv = pool[n].prev;
    if (pv >= 0) pool[pv].next = nx;
    else head = nx;
    if (nx >= 0) pool[nx].prev = pv;
    --size;
    return nx;
  }
  // ExtractorNode::DivideNode (ORBextractor.cc:606-690): children c[0..3] = n1..n4
  void divide(int pi, const std::vector<Cand> &keys, int c[4]) {
    const QNode p = pool[pi];
    const int halfX = (int)std::ceil(static_cast<float>(p.urx - p.ulx) / 2);
    const int halfY = (int)std::ceil(static_cast<float>(p.bry - p.uly) / 2);
    QNode n[4];
    n[0] = QNode{p.ulx, p.uly, p.ulx + halfX, p.uly, p.ulx, p.uly + halfY, p.ulx + halfX, p.uly + halfY,
                 0, 0, -1, -1, false};
    n[1] = QNode{n[0].urx, n[0].ury, p.urx, p.ury, n[0].brx, n[0].bry, p.urx, p.uly + halfY, 0, 0, -1, -1, false};
    n[2] = QNode{n[0].blx, n[0].bly, n[0].brx, n[0].bry, p.blx, p.bly, n[0].brx, p.bly, 0, 0, -1, -1, false};
    n[3] = QNode{n[2].urx, n[2].ury, n[1].brx, n[1].bry, n[2].brx, n[2].bry, p.brx, p.bry, 0, 0, -1, -1, false};
    int cnt[4] = {0, 0, 0, 0};
    if ((int)tag.size() < p.kcnt) tag.resize(p.kcnt);
    for (int i = 0; i < p.kcnt; ++i) {
      const Cand &k = keys[arena[p.koff + i]];
      const int t = k.x < n[0].urx ? (k.y < n[0].bry ? 0 : 2) : (k.y < n[0].bry ? 1 : 3);
      tag[i] = (uint8_t)t;
      ++cnt[t];
    }
    int pos[4];
    int base = (int)arena.size();
    for (int t = 0; t < 4; ++t) {
      n[t].koff = base;
      n[t].kcnt = cnt[t];
      n[t].no_more = cnt[t] == 1;
      pos[t] = base;
      base += cnt[t];
    }
    arena.resize(base);
    for (int i = 0; i < p.kcnt; ++i) arena[pos[tag[i]]++] = arena[p.koff + i];
    for (int t = 0; t < 4; ++t) {
      c[t] = (int)pool.size();
      pool.push_back(n[t]);
    }
  }
};

std::vector<Cand> distribute_quadtree(const std::vector<Cand> &keys, int minX, int maxX, int minY, int maxY, int N) {
  const int nIni = (int)std::round(static_cast<float>(maxX - minX) / (maxY - minY));
  const float hX = static_cast<float>(maxX - minX) / nIni;
  QuadTree T;
  T.pool.reserve(4 * keys.size() + nIni + 16);
  T.arena.reserve(keys.size() * 6 + 16);
  // initial nodes (lNodes.push_back in order) and their keys in input order
  std::vector<int> which(keys.size()), cnt(nIni, 0);
  for (size_t i = 0; i < keys.size(); ++i) {
    which[i] = (int)(size_t)(keys[i].x / hX);
    ++cnt[which[i]];
  }
  std::vector<int> pos(nIni);
  int base = 0;
  for (int i = 0; i < nIni; i++) {
    QNode ni{(int)(hX * static_cast<float>(i)), 0, (int)(hX * static_cast<float>(i + 1)), 0, 0, maxY - minY, 0,
             maxY - minY, base, cnt[i], -1, -1, false};
    ni.blx = ni.ulx;
    ni.brx = ni.urx;
    pos[i] = base;
    base += cnt[i];
    T.pool.push_back(ni);
  }
  T.arena.resize(base);
  for (size_t i = 0; i < keys.size(); ++i) T.arena[pos[which[i]]++] = (int)i;
  for (int i = nIni - 1; i >= 0; --i) T.push_front(i);
  for (int it = T.head; it >= 0;) {
    if (T.pool[it].kcnt == 1) {
      T.pool[it].no_more = true;
      it = T.pool[it].next;
    } else if (T.pool[it].kcnt == 0)
      it = T.erase(it);
    else
      it = T.pool[it].next;
  }
  std::vector<std::pair<int, int>> expand, prev;  // (size, node)
  auto push_children = [&](const int c[4], int *n_to_expand) {
    for (int k = 0; k < 4; ++k) {
      if (T.pool[c[k]].kcnt == 0) continue;
      T.push_front(c[k]);
      if (T.pool[c[k]].kcnt > 1) {
        if (n_to_expand) ++*n_to_expand;
        expand.emplace_back(T.pool[c[k]].kcnt, c[k]);
      }
    }
  };
  bool finish = false;
  while (!finish) {
    int prev_size = T.size;
    int n_to_expand = 0;
    expand.clear();
    for (int it = T.head; it >= 0;) {
      if (T.pool[it].no_more) {
        it = T.pool[it].next;
        continue;
      }
      int c[4];
      T.divide(it, keys, c);
      push_children(c, &n_to_expand);
      it = T.erase(it);
    }
    if (T.size >= N || T.size == prev_size) {
      finish = true;
    } else if (T.size + n_to_expand * 3 > N) {
      while (!finish) {
        prev_size = T.size;
        prev = expand;
        expand.clear();
        std::stable_sort(prev.begin(), prev.end(),
                         [](const std::pair<int, int> &a, const std::pair<int, int> &b) { return a.first < b.first; });
        for (int j = (int)prev.size() - 1; j >= 0; j--) {
          int c[4];
          T.divide(prev[j].second, keys, c);
          push_children(c, nullptr);
          T.erase(prev[j].second);
          if (T.size >= N) break;
        }
        if (T.size >= N || T.size == prev_size) finish = true;
      }
    }
  }
  std::vector<Cand> out;
  out.reserve(T.size);
  for (int it = T.head; it >= 0; it = T.pool[it].next) {
    const QNode &nd = T.pool[it];
    const Cand *best = &keys[T.arena[nd.koff]];
    float max_resp = best->response;
    for (int k = 1; k < nd.kcnt; k++) {
      const Cand &c = keys[T.arena[nd.koff + k]];
      if (c.response > max_resp) {
        best = &c;
        max_resp = c.response;
      }
    }
    out.push_back(*best);
  }
  return out;
}

int resize_vec_end(int width) {  // VResizeLinearVec_32s8u loop bounds
  int x = 0;
  for (; x <= width - 16; x += 16) {
  }
  for (; x < width - 4; x += 4) {
  }
  return x;
}

BlurK gauss_kernel_7x7_s2() {  // getGaussianKernel(7, 2, CV_32F) -> x256 ints
  const double scale2X = -0.5 / (2.0 * 2.0);
  float cf[7];
  double sum = 0;
  for (int i = 0; i < 7; i++) {
    const double x = i - (7 - 1) * 0.5;
    cf[i] = (float)std::exp(scale2X * x * x);
    sum += cf[i];
  }
  sum = 1. / sum;
  BlurK k;
  for (int i = 0; i < 7; i++) {
    cf[i] = (float)(cf[i] * sum);
    if (i >= 3) k.ik[i - 3] = (int)std::lrint(cf[i] * 256.0f);
  }
  for (int j = 0; j < 4; ++j) k.fk[j] = (float)((double)k.ik[j] / 65536.0);
  return k;
}

}  // namespace

// ---------------------------------------------------------------------- engine

// Persistent host workers for the per-level quadtrees: run(n, f) calls f(i)
// for i = 1..n-1 on the workers and f(0) on the caller, then waits. Workers
// live as long as the engine (no thread start-up per frame).
class LevelPool {
 public:
  ~LevelPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      quit_ = true;
    }
    cv_.notify_all();
    for (auto &t : th_) t.join();
  }
  void run(int n, const std::function<void(int)> &f) {
    while ((int)th_.size() < n - 1) {
      const int id = (int)th_.size() + 1;
      th_.emplace_back([this, id] { worker(id); });
    }
    {
      std::lock_guard<std::mutex> g(m_);
      job_ = &f;
      n_ = n;
      pending_ = n - 1;
      ++gen_;
    }
    cv_.notify_all();
    f(0);
    std::unique_lock<std::mutex> lk(m_);
    done_.wait(lk, [this] { return pending_ == 0; });
    job_ = nullptr;
  }

 private:
  void worker(int id) {
    long seen = 0;
    for (;;) {
      const std::function<void(int)> *job = nullptr;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return quit_ || gen_ != seen; });
        if (quit_) return;
        seen = gen_;
        if (id < n_) job = job_;
      }
      if (!job) continue;
      (*job)(id);
      std::lock_guard<std::mutex> g(m_);
      if (--pending_ == 0) done_.notify_one();
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<void(int)> *job_ = nullptr;
  int n_ = 0, pending_ = 0;
  long gen_ = 0;
  bool quit_ = false;
};

struct OrbEngine {
  LevelPool pool;
  std::vector<int> cells_key;  // geometry of the uploaded cell table
  void *cells_ptr = nullptr;
  hipStream_t st = nullptr;
  struct Buf {
    void *p = nullptr;
    size_t bytes = 0;
  };
  Buf img, pyr, blur, cells, cellkp, cnt, off, cand, din, kout, dout, pattern, q, qd, t, td, bidx, bd, bd2, grid,
      gidx, pairs;
  std::vector<int> lw, lh, loff;
  float lscale[kMaxLevels] = {};
  hipEvent_t ev[8] = {};
  hipEvent_t ev_copy = nullptr;  // default flags: the host waits on it for a D2H copy
  double stage_ms[6] = {};
  bool timing = false;
  std::vector<int> h_off;
  std::vector<uint32_t> h_cand;

  ~OrbEngine() {
    for (Buf *b : {&img, &pyr, &blur, &cells, &cellkp, &cnt, &off, &cand, &din, &kout, &dout, &pattern, &q, &qd, &t,
                   &td, &bidx, &bd, &bd2, &grid, &gidx, &pairs})
      if (b->p) (void)hipFree(b->p);
    for (auto &e : ev)
      if (e) (void)hipEventDestroy(e);
    if (ev_copy) (void)hipEventDestroy(ev_copy);
  }
  template <class T>
  T *get(Buf &b, size_t n) {
    const size_t need = std::max<size_t>(n, 1) * sizeof(T);
    if (b.bytes < need) {
      if (b.p) (void)hipFree(b.p);
      b.p = nullptr;
      b.bytes = 0;
      if (hipMalloc(&b.p, need) != hipSuccess) return nullptr;
      b.bytes = need;
    }
    return static_cast<T *>(b.p);
  }
  void mark(int i) {
    if (timing) (void)hipEventRecord(ev[i], st);
  }

  int extract(const sqlm_orb_params *p, const uint8_t *image, int w, int h, int stride, bool upload,
              std::vector<sqlm_keypoint> &kps, std::vector<uint8_t> &desc);
  int extract_impl(const sqlm_orb_params *p, int w, int h, std::vector<sqlm_keypoint> &kps,
                   std::vector<uint8_t> &desc);
};

OrbEngine *orb_create(hipStream_t st) {
  OrbEngine *e = new (std::nothrow) OrbEngine();
  if (!e) return nullptr;
  e->st = st;
  for (auto &v : e->ev)
    if (hipEventCreateWithFlags(&v, hipEventDisableSystemFence) != hipSuccess) {
      delete e;
      return nullptr;
    }
  if (hipEventCreate(&e->ev_copy) != hipSuccess) {
    delete e;
    return nullptr;
  }
  signed char *pat = e->get<signed char>(e->pattern, 1024);
  if (!pat || hipMemcpy(pat, kOrbPattern, 1024, hipMemcpyHostToDevice) != hipSuccess) {
    delete e;
    return nullptr;
  }
  return e;
}

void orb_destroy(OrbEngine *e) { delete e; }

int OrbEngine::extract(const sqlm_orb_params *p, const uint8_t *image, int w, int h, int stride, bool upload,
                       std::vector<sqlm_keypoint> &kps, std::vector<uint8_t> &desc) {
  if (!p || !image || w <= 0 || h <= 0 || stride < w) return SQLM_ERR_INVALID_ARG;
  if (upload) {
    uint8_t *d = get<uint8_t>(img, (size_t)w * h);
    if (!d) return SQLM_ERR_OOM;
    if (hipMemcpy2DAsync(d, w, image, stride, w, h, hipMemcpyHostToDevice, st) != hipSuccess) return SQLM_ERR_HIP;
  }
  return extract_impl(p, w, h, kps, desc);
}

int OrbEngine::extract_impl(const sqlm_orb_params *p, int w, int h, std::vector<sqlm_keypoint> &kps,
                            std::vector<uint8_t> &desc) {
  const int L = p->nlevels;
  if (L < 1 || L > kMaxLevels || !(p->scale_factor > 1.0f) || p->nfeatures < 0) return SQLM_ERR_INVALID_ARG;
  // level geometry (ORBextractor ctor :474-560, ComputePyramid :1224-1282)
  float sf[kMaxLevels];
  sf[0] = 1.0f;
  for (int i = 1; i < L; ++i) sf[i] = sf[i - 1] * p->scale_factor;
  lw.assign(L, 0);
  lh.assign(L, 0);
  loff.assign(L + 1, 0);
  for (int i = 0; i < L; ++i) {
    const float inv = 1.0f / sf[i];
    lw[i] = (int)std::lrint((float)w * inv);
    lh[i] = (int)std::lrint((float)h * inv);
    lscale[i] = sf[i];
    if (lw[i] - 2 * (kEdge - 3) < 30 || lh[i] - 2 * (kEdge - 3) < 30 || lw[i] > 4096 || lh[i] > 4096)
      return SQLM_ERR_UNSUPPORTED;
    // DistributeOctTree needs >= 1 initial node (round(width / height) >= 1)
    if ((int)std::round(static_cast<float>(lw[i] - 2 * (kEdge - 3)) / (lh[i] - 2 * (kEdge - 3))) < 1)
      return SQLM_ERR_UNSUPPORTED;
    loff[i + 1] = loff[i] + lw[i] * lh[i];
  }
  std::vector<int> nfeat(L);
  {
    const float factor = 1.0f / p->scale_factor;
    float nd = p->nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)L));
    int sum = 0;
    for (int l = 0; l < L - 1; ++l) {
      nfeat[l] = (int)std::lrint(nd);
      sum += nfeat[l];
      nd *= factor;
    }
    nfeat[L - 1] = std::max(p->nfeatures - sum, 0);
  }
  // cells of every level (ComputeKeyPointsOctTree :1045-1110)
  std::vector<OrbCell> hc;
  std::vector<int> level_cell(L + 1, 0);
  for (int l = 0; l < L; ++l) {
    level_cell[l] = (int)hc.size();
    const float W = 30;
    const int minB = kEdge - 3, maxBX = lw[l] - kEdge + 3, maxBY = lh[l] - kEdge + 3;
    const float width = (float)(maxBX - minB), height = (float)(maxBY - minB);
    const int nCols = (int)(width / W), nRows = (int)(height / W);
    const int wCell = (int)std::ceil(width / nCols), hCell = (int)std::ceil(height / nRows);
    for (int i = 0; i < nRows; i++) {
      const float iniY = (float)(minB + i * hCell);
      float maxY = iniY + hCell + 6;
      if (iniY >= maxBY - 3) continue;
      if (maxY > maxBY) maxY = (float)maxBY;
      for (int j = 0; j < nCols; j++) {
        const float iniX = (float)(minB + j * wCell);
        float maxX = iniX + wCell + 6;
        if (iniX >= maxBX - 3) continue;
        if (maxX > maxBX) maxX = (float)maxBX;
        OrbCell c;
        c.img_off = loff[l];
        c.pitch = lw[l];
        c.x0 = (int)iniX;
        c.y0 = (int)iniY;
        c.w = (int)maxX - (int)iniX;
        c.h = (int)maxY - (int)iniY;
        c.offx = j * wCell;
        c.offy = i * hCell;
        if (c.w > kCellMax || c.h > kCellMax) return SQLM_ERR_UNSUPPORTED;
        hc.push_back(c);
      }
    }
  }
  level_cell[L] = (int)hc.size();
  const int ncell = (int)hc.size();
  uint8_t *d_pyr = get<uint8_t>(pyr, loff[L]), *d_blur = get<uint8_t>(blur, loff[L]);
  OrbCell *d_cells = get<OrbCell>(cells, ncell);
  uint32_t *d_cellkp = get<uint32_t>(cellkp, (size_t)ncell * kCellCap);
  int *d_cnt = get<int>(cnt, ncell), *d_off = get<int>(off, ncell + 1);
  uint32_t *d_cand = get<uint32_t>(cand, (size_t)ncell * kCellCap);
  if (!d_pyr || !d_blur || !d_cells || !d_cellkp || !d_cnt || !d_off || !d_cand) return SQLM_ERR_OOM;
  mark(0);
  if (hipMemcpyAsync(d_pyr, img.p, (size_t)w * h, hipMemcpyDeviceToDevice, st) != hipSuccess) return SQLM_ERR_HIP;
  for (int l = 1; l < L; ++l) {
    const double scale_x = 1. / ((double)lw[l] / lw[l - 1]), scale_y = 1. / ((double)lh[l] / lh[l - 1]);
    hipLaunchKernelGGL(k_orb_resize, dim3((lw[l] + 255) / 256, lh[l]), dim3(256), 0, st, d_pyr + loff[l - 1],
                       lw[l - 1], lh[l - 1], d_pyr + loff[l], lw[l], lh[l], scale_x, scale_y, resize_vec_end(lw[l]));
  }
  mark(1);
  // the cell table depends only on the geometry: upload it when it changes
  const std::vector<int> key = {w, h, L, (int)(p->scale_factor * 1e6f)};
  if (key != cells_key || cells.p != cells_ptr) {
    if (hipMemcpyAsync(d_cells, hc.data(), sizeof(OrbCell) * ncell, hipMemcpyHostToDevice, st) != hipSuccess)
      return SQLM_ERR_HIP;
    cells_key = key;
    cells_ptr = cells.p;
  }
  hipLaunchKernelGGL(k_orb_fast, dim3(ncell), dim3(256), 0, st, d_pyr, d_cells, p->ini_th_fast, p->min_th_fast,
                     d_cellkp, d_cnt);
  mark(2);
  hipLaunchKernelGGL(k_orb_scan, dim3(1), dim3(1024), 0, st, d_cnt, ncell, d_off);
  hipLaunchKernelGGL(k_orb_compact, dim3(ncell), dim3(256), 0, st, d_cellkp, d_cnt, d_off, d_cand);
  mark(3);
  h_off.resize(ncell + 1);
  if (hipMemcpyAsync(h_off.data(), d_off, sizeof(int) * (ncell + 1), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return SQLM_ERR_HIP;
  const int ncand = h_off[ncell];
  h_cand.resize(std::max(ncand, 1));
  if (ncand &&
      hipMemcpyAsync(h_cand.data(), d_cand, sizeof(uint32_t) * ncand, hipMemcpyDeviceToHost, st) != hipSuccess)
    return SQLM_ERR_HIP;
  if (hipEventRecord(ev_copy, st) != hipSuccess) return SQLM_ERR_HIP;
  // the blur does not depend on the quadtree: it runs while the host distributes
  const BlurK bk = gauss_kernel_7x7_s2();
  BlurLevels bl;
  bl.n = L;
  bl.tile0[0] = 0;
  for (int l = 0; l < L; ++l) {
    bl.off[l] = loff[l];
    bl.w[l] = lw[l];
    bl.h[l] = lh[l];
    bl.tx[l] = (lw[l] + kBTX - 1) / kBTX;
    bl.tile0[l + 1] = bl.tile0[l] + bl.tx[l] * ((lh[l] + kBTY - 1) / kBTY);
  }
  hipLaunchKernelGGL(k_orb_blur, dim3(bl.tile0[L]), dim3(256), 0, st, d_pyr, d_blur, bl, bk);
  mark(4);
  if (hipEventSynchronize(ev_copy) != hipSuccess) return SQLM_ERR_HIP;
  // quadtree per level (host)
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<std::vector<Cand>> sel(L);
  auto level_tree = [&](int l) {
    const int b = h_off[level_cell[l]], e = h_off[level_cell[l + 1]];
    std::vector<Cand> keys(e - b);
    for (int i = b; i < e; ++i) {
      const uint32_t v = h_cand[i];
      keys[i - b] = Cand{(float)(v & 4095u), (float)((v >> 12) & 4095u), (float)(v >> 24)};
    }
    const int minB = kEdge - 3;
    sel[l] = distribute_quadtree(keys, minB, lw[l] - kEdge + 3, minB, lh[l] - kEdge + 3, nfeat[l]);
  };
  // levels are independent: level 0 (the largest) here, the others on the pool
  pool.run(L, std::function<void(int)>(level_tree));
  std::vector<OrbDescIn> hin;
  for (int l = 0; l < L; ++l)
    for (const Cand &c : sel[l]) hin.push_back(OrbDescIn{c.x + (kEdge - 3), c.y + (kEdge - 3), c.response, l});
  stage_ms[5] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  const int n = (int)hin.size();
  kps.resize(n);
  desc.resize((size_t)32 * n);
  if (n == 0) return SQLM_OK;
  OrbDescIn *d_in = get<OrbDescIn>(din, n);
  sqlm_keypoint *d_kout = get<sqlm_keypoint>(kout, n);
  uint8_t *d_dout = get<uint8_t>(dout, (size_t)32 * n);
  if (!d_in || !d_kout || !d_dout) return SQLM_ERR_OOM;
  LevelTab tab;
  for (int l = 0; l < L; ++l) {
    tab.off[l] = loff[l];
    tab.pitch[l] = lw[l];
    tab.scale[l] = lscale[l];
    tab.size[l] = (float)(int)(kPatch * lscale[l]);
  }
  {  // umax (ORBextractor ctor :546-560)
    int v, v0, vmax = (int)std::floor(kHalf * std::sqrt(2.f) / 2 + 1);
    int vmin = (int)std::ceil(kHalf * std::sqrt(2.f) / 2);
    const double hp2 = kHalf * kHalf;
    for (v = 0; v <= vmax; ++v) tab.umax[v] = (int)std::lrint(std::sqrt(hp2 - v * v));
    for (v = kHalf, v0 = 0; v >= vmin; --v) {
      while (tab.umax[v0] == tab.umax[v0 + 1]) ++v0;
      tab.umax[v] = v0;
      ++v0;
    }
  }
  mark(5);
  if (hipMemcpyAsync(d_in, hin.data(), sizeof(OrbDescIn) * n, hipMemcpyHostToDevice, st) != hipSuccess)
    return SQLM_ERR_HIP;
  hipLaunchKernelGGL(k_orb_describe, dim3((n + 3) / 4), dim3(256), 0, st, d_pyr, d_blur, tab,
                     (const signed char *)pattern.p, d_in, n, d_kout, d_dout);
  mark(6);
  if (hipMemcpyAsync(kps.data(), d_kout, sizeof(sqlm_keypoint) * n, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(desc.data(), d_dout, (size_t)32 * n, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return SQLM_ERR_HIP;
  if (timing) {
    float ms;
    const int pairs_[5][2] = {{0, 1}, {1, 2}, {2, 3}, {3, 4}, {5, 6}};
    for (int s = 0; s < 5; ++s) {
      if (hipEventElapsedTime(&ms, ev[pairs_[s][0]], ev[pairs_[s][1]]) == hipSuccess) stage_ms[s] += ms;
    }
  }
  return SQLM_OK;
}

int orb_extract(OrbEngine *e, const sqlm_orb_params *p, const uint8_t *image, int w, int h, int stride,
                sqlm_keypoint *kps, uint8_t *desc, int cap, int *n_out) {
  std::vector<sqlm_keypoint> k;
  std::vector<uint8_t> d;
  const int r = e->extract(p, image, w, h, stride, true, k, d);
  if (r) return r;
  const int n = (int)k.size();
  if (n_out) *n_out = n;
  const int m = std::min(n, std::max(cap, 0));
  if (m > 0 && (!kps || !desc)) return SQLM_ERR_INVALID_ARG;
  if (m > 0) {
    std::memcpy(kps, k.data(), sizeof(sqlm_keypoint) * m);
    std::memcpy(desc, d.data(), (size_t)32 * m);
  }
  return SQLM_OK;
}

int orb_get_level(OrbEngine *e, int level, uint8_t *out, int cap, int *w, int *h) {
  if (level < 0 || level >= (int)e->lw.size()) return SQLM_ERR_STATE;
  if (w) *w = e->lw[level];
  if (h) *h = e->lh[level];
  const int n = e->lw[level] * e->lh[level];
  if (!out || cap < n) return SQLM_ERR_INVALID_ARG;
  if (hipMemcpyAsync(out, (uint8_t *)e->pyr.p + e->loff[level], n, hipMemcpyDeviceToHost, e->st) != hipSuccess ||
      hipStreamSynchronize(e->st) != hipSuccess)
    return SQLM_ERR_HIP;
  return SQLM_OK;
}

int orb_bench_extract(OrbEngine *e, const sqlm_orb_params *p, const uint8_t *image, int w, int h, int stride,
                      int reps, double *ms_per_frame, double *stage_ms) {
  std::vector<sqlm_keypoint> k;
  std::vector<uint8_t> d;
  int r = e->extract(p, image, w, h, stride, true, k, d);  // warm-up + upload
  if (r) return r;
  for (double &s : e->stage_ms) s = 0.0;
  e->timing = true;
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < reps && !r; ++i) r = e->extract_impl(p, w, h, k, d);
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  e->timing = false;
  if (r) return r;
  if (ms_per_frame) *ms_per_frame = ms / std::max(reps, 1);
  if (stage_ms)
    for (int s = 0; s < 6; ++s) stage_ms[s] = e->stage_ms[s] / std::max(reps, 1);
  return SQLM_OK;
}

int orb_match_bf(OrbEngine *e, const uint8_t *query, int nq, const uint8_t *train, int nt, int32_t *best_idx,
                 int32_t *best_dist, int32_t *second_dist) {
  if (nq < 0 || nt < 0 || (nq && (!query || !best_idx || !best_dist || !second_dist)) || (nt && !train))
    return SQLM_ERR_INVALID_ARG;
  if (nq == 0) return SQLM_OK;
  uint32_t *dq = e->get<uint32_t>(e->qd, (size_t)8 * nq), *dt = e->get<uint32_t>(e->td, (size_t)8 * std::max(nt, 1));
  int *bi = e->get<int>(e->bidx, nq), *b1 = e->get<int>(e->bd, nq), *b2 = e->get<int>(e->bd2, nq);
  if (!dq || !dt || !bi || !b1 || !b2) return SQLM_ERR_OOM;
  if (hipMemcpyAsync(dq, query, (size_t)32 * nq, hipMemcpyHostToDevice, e->st) != hipSuccess ||
      (nt && hipMemcpyAsync(dt, train, (size_t)32 * nt, hipMemcpyHostToDevice, e->st) != hipSuccess))
    return SQLM_ERR_HIP;
  hipLaunchKernelGGL(k_orb_bf, dim3((nq + 255) / 256), dim3(256), 0, e->st, dq, nq, dt, nt, bi, b1, b2);
  if (hipMemcpyAsync(best_idx, bi, sizeof(int) * nq, hipMemcpyDeviceToHost, e->st) != hipSuccess ||
      hipMemcpyAsync(best_dist, b1, sizeof(int) * nq, hipMemcpyDeviceToHost, e->st) != hipSuccess ||
      hipMemcpyAsync(second_dist, b2, sizeof(int) * nq, hipMemcpyDeviceToHost, e->st) != hipSuccess ||
      hipStreamSynchronize(e->st) != hipSuccess)
    return SQLM_ERR_HIP;
  return SQLM_OK;
}

// The candidate lists of n_q GetFeaturesInArea queries over frame 2's grid
// (AssignFeaturesToGrid, Frame.cc:1268-1285, with PosInGrid :1554-1565):
// hoff [n_q + 1] offsets into hp = (keypoint index, Hamming distance to the
// query's descriptor qdesc [n_q][32]) in the reference's candidate order.
static int area_search(OrbEngine *e, const sqlm_keypoint *k2, const uint8_t *d2, int n2, const sqlm_frame_bounds *f2,
                       const std::vector<float4> &hq, const uint8_t *qdesc, std::vector<int> &hoff,
                       std::vector<int2> &hp) {
  const int n1 = (int)hq.size();
  hoff.assign(n1 + 1, 0);
  hp.clear();
  if (n1 == 0) return SQLM_OK;
  const float wi = static_cast<float>(kGridCols) / static_cast<float>(f2->max_x - f2->min_x);
  const float hi = static_cast<float>(kGridRows) / static_cast<float>(f2->max_y - f2->min_y);
  std::vector<int> cell_of(n2), ptr(kGridCols * kGridRows + 1, 0), idx;
  for (int i = 0; i < n2; ++i) {
    const int px = (int)std::round((k2[i].x - f2->min_x) * wi), py = (int)std::round((k2[i].y - f2->min_y) * hi);
    cell_of[i] = (px < 0 || px >= kGridCols || py < 0 || py >= kGridRows) ? -1 : px * kGridRows + py;
    if (cell_of[i] >= 0) ptr[cell_of[i] + 1]++;
  }
  for (int c = 0; c < kGridCols * kGridRows; ++c) ptr[c + 1] += ptr[c];
  idx.resize(std::max(ptr.back(), 1));
  {
    std::vector<int> fill(ptr.begin(), ptr.end() - 1);
    for (int i = 0; i < n2; ++i)
      if (cell_of[i] >= 0) idx[fill[cell_of[i]]++] = i;
  }
  std::vector<float> hk2((size_t)4 * std::max(n2, 1));
  for (int i = 0; i < n2; ++i) {
    hk2[4 * i] = k2[i].x;
    hk2[4 * i + 1] = k2[i].y;
    std::memcpy(&hk2[4 * i + 2], &k2[i].octave, 4);
  }
  AreaArgs A;
  float4 *dq = e->get<float4>(e->q, n1);
  uint32_t *dd1 = e->get<uint32_t>(e->qd, (size_t)8 * n1);
  float *dk2 = e->get<float>(e->t, hk2.size());
  uint32_t *dd2 = e->get<uint32_t>(e->td, (size_t)8 * std::max(n2, 1));
  int *dptr = e->get<int>(e->grid, ptr.size()), *didx = e->get<int>(e->gidx, idx.size());
  int *dcnt = e->get<int>(e->bidx, n1), *doff = e->get<int>(e->bd, n1 + 1);
  if (!dq || !dd1 || !dk2 || !dd2 || !dptr || !didx || !dcnt || !doff) return SQLM_ERR_OOM;
  if (hipMemcpyAsync(dq, hq.data(), sizeof(float4) * n1, hipMemcpyHostToDevice, e->st) != hipSuccess ||
      hipMemcpyAsync(dd1, qdesc, (size_t)32 * n1, hipMemcpyHostToDevice, e->st) != hipSuccess ||
      hipMemcpyAsync(dk2, hk2.data(), sizeof(float) * hk2.size(), hipMemcpyHostToDevice, e->st) != hipSuccess ||
      (n2 && hipMemcpyAsync(dd2, d2, (size_t)32 * n2, hipMemcpyHostToDevice, e->st) != hipSuccess) ||
      hipMemcpyAsync(dptr, ptr.data(), sizeof(int) * ptr.size(), hipMemcpyHostToDevice, e->st) != hipSuccess ||
      hipMemcpyAsync(didx, idx.data(), sizeof(int) * idx.size(), hipMemcpyHostToDevice, e->st) != hipSuccess)
    return SQLM_ERR_HIP;
  A.q = dq;
  A.d1 = dd1;
  A.k2 = dk2;
  A.d2 = dd2;
  A.cell_ptr = dptr;
  A.cell_idx = didx;
  A.min_x = f2->min_x;
  A.min_y = f2->min_y;
  A.wi = wi;
  A.hi = hi;
  A.n1 = n1;
  const dim3 g((n1 + 3) / 4);
  hipLaunchKernelGGL(k_area_list<0>, g, dim3(256), 0, e->st, A, dcnt, (const int *)nullptr, (int2 *)nullptr);
  hipLaunchKernelGGL(k_orb_scan, dim3(1), dim3(1024), 0, e->st, dcnt, n1, doff);
  if (hipMemcpyAsync(hoff.data(), doff, sizeof(int) * (n1 + 1), hipMemcpyDeviceToHost, e->st) != hipSuccess ||
      hipStreamSynchronize(e->st) != hipSuccess)
    return SQLM_ERR_HIP;
  const int total = hoff[n1];
  int2 *dpairs = e->get<int2>(e->pairs, std::max(total, 1));
  if (!dpairs) return SQLM_ERR_OOM;
  hipLaunchKernelGGL(k_area_list<1>, g, dim3(256), 0, e->st, A, (int *)nullptr, (const int *)doff, dpairs);
  hp.resize(std::max(total, 1));
  if (total && hipMemcpyAsync(hp.data(), dpairs, sizeof(int2) * total, hipMemcpyDeviceToHost, e->st) != hipSuccess)
    return SQLM_ERR_HIP;
  if (hipStreamSynchronize(e->st) != hipSuccess) return SQLM_ERR_HIP;
  return SQLM_OK;
}

static float4 area_query(float x, float y, float r, int lv) {
  float4 q;
  q.x = x;
  q.y = y;
  q.z = r;
  std::memcpy(&q.w, &lv, 4);
  return q;
}

int orb_search_for_init(OrbEngine *e, const sqlm_keypoint *k1, const uint8_t *d1, int n1, const sqlm_keypoint *k2,
                        const uint8_t *d2, int n2, const sqlm_frame_bounds *f2, float *prev, int32_t *m12, int window,
                        float nnratio, int check_ori, int *n_matches) {
  if (n1 < 0 || n2 < 0 || !f2 || (n1 && (!k1 || !d1 || !prev || !m12)) || (n2 && (!k2 || !d2)))
    return SQLM_ERR_INVALID_ARG;
  for (int i = 0; i < n1; ++i) m12[i] = -1;
  if (n_matches) *n_matches = 0;
  if (n1 == 0) return SQLM_OK;
  // GetFeaturesInArea(prev.x, prev.y, windowSize, level1, level1) for level1 == 0 (ORBmatcher.cc:594-612)
  std::vector<float4> hq(n1);
  for (int i = 0; i < n1; ++i)
    hq[i] = area_query(prev[2 * i], prev[2 * i + 1], (float)window,
                       k1[i].octave > 0 ? kAreaSkip : area_levels(k1[i].octave, k1[i].octave));
  std::vector<int> hoff;
  std::vector<int2> hp;
  if (int rc = area_search(e, k2, d2, n2, f2, hq, d1, hoff, hp)) return rc;
  // acceptance loop (ORBmatcher.cc:594-682): order-dependent, over the GPU lists
  std::vector<int> vMatchedDistance(n2, INT_MAX), vnMatches21(n2, -1), rot_i, rot_bin;
  int hist[kHistoLength] = {0};
  const float factor = kHistoLength / 360.0f;
  int nmatches = 0;
  for (int i1 = 0; i1 < n1; i1++) {
    if (k1[i1].octave > 0 || hoff[i1 + 1] == hoff[i1]) continue;
    int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
    for (int q = hoff[i1]; q < hoff[i1 + 1]; ++q) {
      const int i2 = hp[q].x, dist = hp[q].y;
      if (vMatchedDistance[i2] <= dist) continue;
      if (dist < bestDist) {
        bestDist2 = bestDist;
        bestDist = dist;
        bestIdx2 = i2;
      } else if (dist < bestDist2) {
        bestDist2 = dist;
      }
    }
    if (bestDist <= kThLow && bestDist < (float)bestDist2 * nnratio) {
      if (vnMatches21[bestIdx2] >= 0) {
        m12[vnMatches21[bestIdx2]] = -1;
        nmatches--;
      }
      m12[i1] = bestIdx2;
      vnMatches21[bestIdx2] = i1;
      vMatchedDistance[bestIdx2] = bestDist;
      nmatches++;
      if (check_ori) {
        float rot = k1[i1].angle - k2[bestIdx2].angle;
        if (rot < 0.0) rot += 360.0f;
        int bin = (int)std::round(rot * factor);
        if (bin == kHistoLength) bin = 0;
        rot_i.push_back(i1);
        rot_bin.push_back(bin);
        hist[bin]++;
      }
    }
  }
  if (check_ori) {  // ComputeThreeMaxima (ORBmatcher.cc:2048-2090)
    int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
    for (int i = 0; i < kHistoLength; i++) {
      const int s = hist[i];
      if (s > max1) {
        max3 = max2; max2 = max1; max1 = s;
        ind3 = ind2; ind2 = ind1; ind1 = i;
      } else if (s > max2) {
        max3 = max2; max2 = s;
        ind3 = ind2; ind2 = i;
      } else if (s > max3) {
        max3 = s;
        ind3 = i;
      }
    }
    if (max2 < 0.1f * (float)max1) {
      ind2 = -1;
      ind3 = -1;
    } else if (max3 < 0.1f * (float)max1) {
      ind3 = -1;
    }
    for (size_t q = 0; q < rot_i.size(); ++q) {
      const int b = rot_bin[q];
      if (b == ind1 || b == ind2 || b == ind3) continue;
      if (m12[rot_i[q]] >= 0) {
        m12[rot_i[q]] = -1;
        nmatches--;
      }
    }
  }
  for (int i1 = 0; i1 < n1; i1++)
    if (m12[i1] >= 0) {
      prev[2 * i1] = k2[m12[i1]].x;
      prev[2 * i1 + 1] = k2[m12[i1]].y;
    }
  if (n_matches) *n_matches = nmatches;
  return SQLM_OK;
}

static bool frame_ok(const sqlm_orb_frame *F) {
  return F && F->n >= 0 && F->n_levels > 0 && F->scale_factors && F->slot_mp && F->slot_obs &&
         (F->n == 0 || (F->kps && F->desc));
}

// ComputeThreeMaxima (ORBmatcher.cc:2048-2090) over bin sizes.
static void three_maxima(const int *hist, int &ind1, int &ind2, int &ind3) {
  int max1 = 0, max2 = 0, max3 = 0;
  ind1 = ind2 = ind3 = -1;
  for (int i = 0; i < kHistoLength; i++) {
    const int s = hist[i];
    if (s > max1) {
      max3 = max2; max2 = max1; max1 = s;
      ind3 = ind2; ind2 = ind1; ind1 = i;
    } else if (s > max2) {
      max3 = max2; max2 = s;
      ind3 = ind2; ind2 = i;
    } else if (s > max3) {
      max3 = s;
      ind3 = i;
    }
  }
  if (max2 < 0.1f * (float)max1) {
    ind2 = -1;
    ind3 = -1;
  } else if (max3 < 0.1f * (float)max1) {
    ind3 = -1;
  }
}

int orb_search_by_projection_local(OrbEngine *e, sqlm_orb_frame *F, const sqlm_track_point *mps,
                                   const uint8_t *mp_desc, int n_mp, float th, float nnratio, int *n_matches) {
  if (!frame_ok(F) || n_mp < 0 || (n_mp && (!mps || !mp_desc))) return SQLM_ERR_INVALID_ARG;
  if (n_matches) *n_matches = 0;
  const bool bFactor = th != 1.0;
  // ORBmatcher.cc:78-101: the window of every point still to be projected
  std::vector<float4> hq(n_mp);
  std::vector<float> rwin(n_mp);
  for (int i = 0; i < n_mp; ++i) {
    const sqlm_track_point &p = mps[i];
    if (!p.in_view || p.bad || p.level < 0 || p.level >= F->n_levels) {
      if (p.in_view && !p.bad) return SQLM_ERR_INVALID_ARG;  // mnTrackScaleLevel outside mvScaleFactors
      hq[i] = area_query(0.f, 0.f, 0.f, kAreaSkip);
      continue;
    }
    float r = p.view_cos > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos (:183-190)
    if (bFactor) r *= th;
    rwin[i] = r * F->scale_factors[p.level];
    hq[i] = area_query(p.proj_x, p.proj_y, rwin[i], area_levels(p.level - 1, p.level));
  }
  std::vector<int> hoff;
  std::vector<int2> hp;
  if (int rc = area_search(e, F->kps, F->desc, F->n, &F->bounds, hq, mp_desc, hoff, hp)) return rc;
  int nmatches = 0;
  for (int i = 0; i < n_mp; ++i) {  // :118-175, in point order over the GPU lists
    if (hoff[i + 1] == hoff[i]) continue;
    int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
    for (int q = hoff[i]; q < hoff[i + 1]; ++q) {
      const int idx = hp[q].x, dist = hp[q].y;
      if (F->slot_mp[idx] >= 0 && F->slot_obs[idx]) continue;
      if (F->uright && F->uright[idx] > 0) {
        const float er = fabsf(mps[i].proj_xr - F->uright[idx]);
        if (er > rwin[i]) continue;
      }
      if (dist < bestDist) {
        bestDist2 = bestDist;
        bestDist = dist;
        bestLevel2 = bestLevel;
        bestLevel = F->kps[idx].octave;
        bestIdx = idx;
      } else if (dist < bestDist2) {
        bestLevel2 = F->kps[idx].octave;
        bestDist2 = dist;
      }
    }
    if (bestDist <= kThHigh) {
      if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;
      F->slot_mp[bestIdx] = mps[i].id;
      F->slot_obs[bestIdx] = mps[i].has_obs;
      nmatches++;
    }
  }
  if (n_matches) *n_matches = nmatches;
  return SQLM_OK;
}

// cv::Mat 3x3 (optionally transposed) * 3x1 (+ 3x1) on CV_32F as OpenCV's
// small-matrix gemm evaluates it: float dot left to right, then alpha * t +
// beta * c in double (one float addition for alpha = beta = 1).
static void mat3_mul_add(const float *T, bool transpose, const float *x, const float *c, double sign, float *out) {
  for (int i = 0; i < 3; ++i) {
    const float a0 = transpose ? T[i] : T[i * 4], a1 = transpose ? T[4 + i] : T[i * 4 + 1],
                a2 = transpose ? T[8 + i] : T[i * 4 + 2];
    const float t0 = a0 * x[0] + a1 * x[1] + a2 * x[2];
    out[i] = c ? (float)((double)t0 * sign + (double)c[i]) : (float)((double)t0 * sign);
  }
}

int orb_search_by_projection_last(OrbEngine *e, sqlm_orb_frame *F, const float *Tcw, const float *Tlw,
                                  const sqlm_last_point *lp, const uint8_t *ldesc, int n_last, float th, int mono,
                                  int check_ori, int *n_matches) {
  if (!frame_ok(F) || !Tcw || !Tlw || n_last < 0 || (n_last && (!lp || !ldesc))) return SQLM_ERR_INVALID_ARG;
  if (n_matches) *n_matches = 0;
  const float tcw[3] = {Tcw[3], Tcw[7], Tcw[11]}, tlw[3] = {Tlw[3], Tlw[7], Tlw[11]};
  float twc[3], tlc[3];
  mat3_mul_add(Tcw, true, tcw, nullptr, -1.0, twc);  // twc = -Rcw.t()*tcw (ORBmatcher.cc:1730)
  mat3_mul_add(Tlw, false, twc, tlw, 1.0, tlc);      // tlc = Rlw*twc+tlw (:1735)
  const bool bForward = tlc[2] > F->mb && !mono, bBackward = -tlc[2] > F->mb && !mono;
  // :1744-1790: projection and window of every slot (host, float as the reference)
  std::vector<float4> hq(n_last);
  std::vector<float> hu(n_last), hinvz(n_last), hrad(n_last);
  for (int i = 0; i < n_last; i++) {
    hq[i] = area_query(0.f, 0.f, 0.f, kAreaSkip);
    const sqlm_last_point &p = lp[i];
    if (p.id < 0 || p.outlier) continue;
    if (p.octave < 0 || p.octave >= F->n_levels) return SQLM_ERR_INVALID_ARG;
    const float x3Dw[3] = {p.x, p.y, p.z};
    float x3Dc[3];
    mat3_mul_add(Tcw, false, x3Dw, tcw, 1.0, x3Dc);
    const float xc = x3Dc[0], yc = x3Dc[1];
    const float invzc = (float)(1.0 / (double)x3Dc[2]);
    if (invzc < 0) continue;
    const float u = F->fx * xc * invzc + F->cx, v = F->fy * yc * invzc + F->cy;
    if (u < F->bounds.min_x || u > F->bounds.max_x) continue;
    if (v < F->bounds.min_y || v > F->bounds.max_y) continue;
    const int o = p.octave;
    const float radius = th * F->scale_factors[o];
    const int lv = bForward ? area_levels(o, -1) : bBackward ? area_levels(0, o) : area_levels(o - 1, o + 1);
    hq[i] = area_query(u, v, radius, lv);
    hu[i] = u;
    hinvz[i] = invzc;
    hrad[i] = radius;
  }
  std::vector<int> hoff;
  std::vector<int2> hp;
  if (int rc = area_search(e, F->kps, F->desc, F->n, &F->bounds, hq, ldesc, hoff, hp)) return rc;
  int nmatches = 0, hist[kHistoLength] = {0};
  std::vector<int> rot_bin, rot_idx;
  const float factor = kHistoLength / 360.0f;
  for (int i = 0; i < n_last; i++) {  // :1806-1858
    if (hoff[i + 1] == hoff[i]) continue;
    int bestDist = 256, bestIdx2 = -1;
    for (int q = hoff[i]; q < hoff[i + 1]; ++q) {
      const int i2 = hp[q].x, dist = hp[q].y;
      if (F->slot_mp[i2] >= 0 && F->slot_obs[i2]) continue;
      if (F->uright && F->uright[i2] > 0) {
        const float ur = hu[i] - F->bf * hinvz[i];
        const float er = fabsf(ur - F->uright[i2]);
        if (er > hrad[i]) continue;
      }
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx2 = i2;
      }
    }
    if (bestDist <= kThHigh) {
      F->slot_mp[bestIdx2] = lp[i].id;
      F->slot_obs[bestIdx2] = lp[i].has_obs;
      nmatches++;
      if (check_ori) {
        float rot = lp[i].angle - F->kps[bestIdx2].angle;
        if (rot < 0.0) rot += 360.0f;
        int bin = (int)std::round(rot * factor);
        if (bin == kHistoLength) bin = 0;
        rot_bin.push_back(bin);
        rot_idx.push_back(bestIdx2);
        hist[bin]++;
      }
    }
  }
  if (check_ori) {  // :1862-1880: every entry of a rejected bin is cleared, bin by bin
    int ind1, ind2, ind3;
    three_maxima(hist, ind1, ind2, ind3);
    for (int b = 0; b < kHistoLength; b++) {
      if (b == ind1 || b == ind2 || b == ind3) continue;
      for (size_t q = 0; q < rot_bin.size(); ++q)
        if (rot_bin[q] == b) {
          F->slot_mp[rot_idx[q]] = -1;
          F->slot_obs[rot_idx[q]] = 0;
          nmatches--;
        }
    }
  }
  if (n_matches) *n_matches = nmatches;
  return SQLM_OK;
}

// ---- keyframe projection searches (ORBmatcher.cc:423, :1109, :1296, :1902) ----
// [R | t] rows and Ow = -R^T t, as pKF->GetRotation() / GetTranslation() /
// GetCameraCenter() hold them.
struct ProjPose {
  float T[12];
  float Ow[3];
  void finish() {
    const float t[3] = {T[3], T[7], T[11]};
    mat3_mul_add(T, true, t, nullptr, -1.0, Ow);
  }
  explicit ProjPose(const float *Tcw) {
    std::memcpy(T, Tcw, sizeof(T));
    finish();
  }
  // Scw -> s = sqrt(row0 . row0) (Mat::dot in double), [R | t] = [sR | t] / s
  // (a float scale by (float)(1 / s)) (ORBmatcher.cc:434-441)
  ProjPose(const float *S, bool) {
    const double d = (double)S[0] * S[0] + (double)S[1] * S[1] + (double)S[2] * S[2];
    const float scw = (float)std::sqrt(d);
    const float inv = (float)(1.0 / (double)scw);
    for (int i = 0; i < 12; ++i) T[i] = S[i] * inv;
    finish();
  }
};

// cv::norm (double sum of squares) and Mat::dot (double) of 3x1 CV_32F
static float norm3(const float *v) {
  double s = 0;
  for (int i = 0; i < 3; ++i) s += (double)v[i] * v[i];
  return (float)std::sqrt(s);
}
static double dot3(const float *a, const float *b) {
  double s = 0;
  for (int i = 0; i < 3; ++i) s += (double)a[i] * b[i];
  return s;
}

// MapPoint::PredictScale (MapPoint.cc:610-650)
static int predict_scale(float max_dist, float dist, float log_scale, int n_levels) {
  const float ratio = max_dist / dist;
  int nScale = (int)std::ceil(std::log(ratio) / log_scale);
  if (nScale < 0)
    nScale = 0;
  else if (nScale >= n_levels)
    nScale = n_levels - 1;
  return nScale;
}

// The keyframe-side projection (ORBmatcher.cc:447-489, :1132-1180, :1327-1372):
// z >= 0, IsInImage, distance invariance band, viewing angle, predicted level.
static bool project_kf(const sqlm_orb_frame *F, const ProjPose &P, const sqlm_map_point &p, float &u, float &v,
                       float &invz, int &level) {
  const float X[3] = {p.x, p.y, p.z}, t[3] = {P.T[3], P.T[7], P.T[11]};
  float Xc[3];
  mat3_mul_add(P.T, false, X, t, 1.0, Xc);
  if (Xc[2] < 0.0f) return false;
  invz = 1 / Xc[2];
  const float x = Xc[0] * invz, y = Xc[1] * invz;
  u = F->fx * x + F->cx;
  v = F->fy * y + F->cy;
  if (!(u >= F->bounds.min_x && u < F->bounds.max_x && v >= F->bounds.min_y && v < F->bounds.max_y)) return false;
  const float maxDistance = 1.2f * p.max_dist, minDistance = 0.8f * p.min_dist;
  const float PO[3] = {X[0] - P.Ow[0], X[1] - P.Ow[1], X[2] - P.Ow[2]};
  const float dist = norm3(PO);
  if (dist < minDistance || dist > maxDistance) return false;
  const float Pn[3] = {p.nx, p.ny, p.nz};
  if (dot3(PO, Pn) < 0.5 * dist) return false;
  level = predict_scale(p.max_dist, dist, std::log(F->scale_factors[1]), F->n_levels);
  return true;
}

static bool kf_frame_ok(const sqlm_orb_frame *F) {
  return F && F->n >= 0 && F->n_levels >= 2 && F->scale_factors && (F->n == 0 || (F->kps && F->desc));
}

int orb_search_by_projection_sim3(OrbEngine *e, sqlm_orb_frame *F, const float *Scw, const sqlm_map_point *mps,
                                  const uint8_t *mp_desc, int n, int th, int *n_matches) {
  if (!kf_frame_ok(F) || !F->slot_mp || !Scw || n < 0 || (n && (!mps || !mp_desc))) return SQLM_ERR_INVALID_ARG;
  if (n_matches) *n_matches = 0;
  const ProjPose P(Scw, true);
  std::vector<float4> hq(n);
  for (int i = 0; i < n; ++i) {
    hq[i] = area_query(0.f, 0.f, 0.f, kAreaSkip);
    float u, v, invz;
    int pl;
    if (mps[i].skip || !project_kf(F, P, mps[i], u, v, invz, pl)) continue;
    // KeyFrame::GetFeaturesInArea (KeyFrame.cc:809-853) + the level test (ORBmatcher.cc:518-520)
    hq[i] = area_query(u, v, th * F->scale_factors[pl], area_levels(pl - 1, pl));
  }
  std::vector<int> hoff;
  std::vector<int2> hp;
  if (int rc = area_search(e, F->kps, F->desc, F->n, &F->bounds, hq, mp_desc, hoff, hp)) return rc;
  int nmatches = 0;
  for (int i = 0; i < n; ++i) {  // :505-541
    int bestDist = 256, bestIdx = -1;
    for (int q = hoff[i]; q < hoff[i + 1]; ++q) {
      const int idx = hp[q].x, dist = hp[q].y;
      if (F->slot_mp[idx] >= 0) continue;
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx = idx;
      }
    }
    if (bestDist <= kThLow) {
      F->slot_mp[bestIdx] = mps[i].id;
      nmatches++;
    }
  }
  if (n_matches) *n_matches = nmatches;
  return SQLM_OK;
}

int orb_fuse(OrbEngine *e, const sqlm_orb_frame *F, const float *T, int sim3, const sqlm_map_point *mps,
             const uint8_t *mp_desc, int n, float th, int32_t *fuse_idx, int *n_fused) {
  if (!kf_frame_ok(F) || !T || n < 0 || (n && (!mps || !mp_desc || !fuse_idx))) return SQLM_ERR_INVALID_ARG;
  if (n_fused) *n_fused = 0;
  const ProjPose P = sim3 ? ProjPose(T, true) : ProjPose(T);
  std::vector<float4> hq(n);
  std::vector<float> hu(n), hv(n), hur(n);
  for (int i = 0; i < n; ++i) {
    fuse_idx[i] = -1;
    hq[i] = area_query(0.f, 0.f, 0.f, kAreaSkip);
    float u, v, invz;
    int pl;
    if (mps[i].skip || !project_kf(F, P, mps[i], u, v, invz, pl)) continue;
    hu[i] = u;
    hv[i] = v;
    hur[i] = u - F->bf * invz;
    hq[i] = area_query(u, v, th * F->scale_factors[pl], area_levels(pl - 1, pl));
  }
  std::vector<int> hoff;
  std::vector<int2> hp;
  if (int rc = area_search(e, F->kps, F->desc, F->n, &F->bounds, hq, mp_desc, hoff, hp)) return rc;
  int nFused = 0;
  for (int i = 0; i < n; ++i) {
    int bestDist = sim3 ? INT_MAX : 256, bestIdx = -1;
    for (int q = hoff[i]; q < hoff[i + 1]; ++q) {
      const int idx = hp[q].x, dist = hp[q].y;
      const sqlm_keypoint &kp = F->kps[idx];
      if (!sim3) {  // :1209-1237: reprojection gate, stereo (3 dof) or monocular (2 dof)
        const float s2 = F->scale_factors[kp.octave] * F->scale_factors[kp.octave];
        const float inv_s2 = 1.0f / s2;
        if (F->uright && F->uright[idx] >= 0) {
          const float ex = hu[i] - kp.x, ey = hv[i] - kp.y, er = hur[i] - F->uright[idx];
          const float e2 = ex * ex + ey * ey + er * er;
          if (e2 * inv_s2 > 7.8) continue;
        } else {
          const float ex = hu[i] - kp.x, ey = hv[i] - kp.y;
          const float e2 = ex * ex + ey * ey;
          if (e2 * inv_s2 > 5.99) continue;
        }
      }
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx = idx;
      }
    }
    if (bestDist <= kThLow) {
      fuse_idx[i] = bestIdx;
      nFused++;
    }
  }
  if (n_fused) *n_fused = nFused;
  return SQLM_OK;
}

int orb_search_by_projection_kf(OrbEngine *e, sqlm_orb_frame *F, const float *Tcw, const sqlm_map_point *mps,
                                const uint8_t *mp_desc, const float *kf_angle, int n, float th, int orb_dist,
                                int check_ori, int *n_matches) {
  if (!kf_frame_ok(F) || !F->slot_mp || !Tcw || n < 0 || (n && (!mps || !mp_desc || !kf_angle)))
    return SQLM_ERR_INVALID_ARG;
  if (n_matches) *n_matches = 0;
  const ProjPose P(Tcw);
  const float t[3] = {P.T[3], P.T[7], P.T[11]};
  const float log_scale = std::log(F->scale_factors[1]);
  std::vector<float4> hq(n);
  for (int i = 0; i < n; ++i) {  // :1932-1968
    hq[i] = area_query(0.f, 0.f, 0.f, kAreaSkip);
    const sqlm_map_point &p = mps[i];
    if (p.skip) continue;
    const float X[3] = {p.x, p.y, p.z};
    float Xc[3];
    mat3_mul_add(P.T, false, X, t, 1.0, Xc);
    const float xc = Xc[0], yc = Xc[1];
    const float invzc = (float)(1.0 / (double)Xc[2]);
    const float u = F->fx * xc * invzc + F->cx, v = F->fy * yc * invzc + F->cy;
    if (u < F->bounds.min_x || u > F->bounds.max_x) continue;
    if (v < F->bounds.min_y || v > F->bounds.max_y) continue;
    const float PO[3] = {X[0] - P.Ow[0], X[1] - P.Ow[1], X[2] - P.Ow[2]};
    const float dist3D = norm3(PO);
    const float maxDistance = 1.2f * p.max_dist, minDistance = 0.8f * p.min_dist;
    if (dist3D < minDistance || dist3D > maxDistance) continue;
    const int pl = predict_scale(p.max_dist, dist3D, log_scale, F->n_levels);
    hq[i] = area_query(u, v, th * F->scale_factors[pl], area_levels(pl - 1, pl + 1));
  }
  std::vector<int> hoff;
  std::vector<int2> hp;
  if (int rc = area_search(e, F->kps, F->desc, F->n, &F->bounds, hq, mp_desc, hoff, hp)) return rc;
  int nmatches = 0, hist[kHistoLength] = {0};
  std::vector<int> rot_bin, rot_idx;
  const float factor = kHistoLength / 360.0f;
  for (int i = 0; i < n; ++i) {  // :1975-2013
    int bestDist = 256, bestIdx2 = -1;
    for (int q = hoff[i]; q < hoff[i + 1]; ++q) {
      const int i2 = hp[q].x, dist = hp[q].y;
      if (F->slot_mp[i2] >= 0) continue;
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx2 = i2;
      }
    }
    if (bestDist <= orb_dist) {
      F->slot_mp[bestIdx2] = mps[i].id;
      nmatches++;
      if (check_ori) {
        float rot = kf_angle[i] - F->kps[bestIdx2].angle;
        if (rot < 0.0) rot += 360.0f;
        int bin = (int)std::round(rot * factor);
        if (bin == kHistoLength) bin = 0;
        rot_bin.push_back(bin);
        rot_idx.push_back(bestIdx2);
        hist[bin]++;
      }
    }
  }
  if (check_ori) {  // :2017-2039
    int ind1, ind2, ind3;
    three_maxima(hist, ind1, ind2, ind3);
    for (int b = 0; b < kHistoLength; b++) {
      if (b == ind1 || b == ind2 || b == ind3) continue;
      for (size_t q = 0; q < rot_bin.size(); ++q)
        if (rot_bin[q] == b) {
          F->slot_mp[rot_idx[q]] = -1;
          nmatches--;
        }
    }
  }
  if (n_matches) *n_matches = nmatches;
  return SQLM_OK;
}

// ---- BoW searches (ORBmatcher.cc:246, :731, :887) ----
// One query per side-1 feature of every common FeatureVector node, in the
// reference's visiting order (common nodes ascending — the lower_bound merge
// of :280-382 — then the node's features in index order); its candidates are
// the node's side-2 run. The GPU fills every (query, candidate) distance; the
// order-dependent acceptance replays the visit on the host.
struct BowPlan {
  std::vector<int4> q;    // (side-1 feature, run begin, run end, distance offset)
  std::vector<int> cand;  // side-2 features, node-sorted
  std::vector<int> dist;
};

static bool bow_ok(const sqlm_bow_frame *K) {
  return K && K->n >= 0 && (K->n == 0 || (K->kps && K->desc && K->node && K->mp));
}

static std::vector<int> node_sorted(const sqlm_bow_frame *K) {
  std::vector<int> v;
  v.reserve(K->n);
  for (int i = 0; i < K->n; ++i)
    if (K->node[i] >= 0) v.push_back(i);
  std::stable_sort(v.begin(), v.end(), [K](int a, int b) { return K->node[a] < K->node[b]; });
  return v;
}

static int bow_plan(OrbEngine *e, const sqlm_bow_frame *K1, const sqlm_bow_frame *K2, BowPlan &B) {
  const std::vector<int> v1 = node_sorted(K1);
  B.cand = node_sorted(K2);
  const std::vector<int> &v2 = B.cand;
  B.q.clear();
  int total = 0;
  size_t a = 0, b = 0;
  while (a < v1.size() && b < v2.size()) {
    const int na = K1->node[v1[a]], nb = K2->node[v2[b]];
    if (na == nb) {
      size_t ea = a, eb = b;
      while (ea < v1.size() && K1->node[v1[ea]] == na) ea++;
      while (eb < v2.size() && K2->node[v2[eb]] == nb) eb++;
      for (size_t i = a; i < ea; ++i) {
        B.q.push_back(make_int4(v1[i], (int)b, (int)eb, total));
        total += (int)(eb - b);
      }
      a = ea;
      b = eb;
    } else if (na < nb) {
      while (a < v1.size() && K1->node[v1[a]] < nb) a++;
    } else {
      while (b < v2.size() && K2->node[v2[b]] < na) b++;
    }
  }
  B.dist.assign(std::max(total, 1), 0);
  const int nq = (int)B.q.size();
  if (nq == 0 || total == 0) return SQLM_OK;
  int4 *dq = e->get<int4>(e->q, nq);
  uint32_t *dd1 = e->get<uint32_t>(e->qd, (size_t)8 * K1->n);
  uint32_t *dd2 = e->get<uint32_t>(e->td, (size_t)8 * K2->n);
  int *dc = e->get<int>(e->gidx, B.cand.size()), *dd = e->get<int>(e->pairs, total);
  if (!dq || !dd1 || !dd2 || !dc || !dd) return SQLM_ERR_OOM;
  if (hipMemcpyAsync(dq, B.q.data(), sizeof(int4) * nq, hipMemcpyHostToDevice, e->st) != hipSuccess ||
      hipMemcpyAsync(dd1, K1->desc, (size_t)32 * K1->n, hipMemcpyHostToDevice, e->st) != hipSuccess ||
      hipMemcpyAsync(dd2, K2->desc, (size_t)32 * K2->n, hipMemcpyHostToDevice, e->st) != hipSuccess ||
      hipMemcpyAsync(dc, B.cand.data(), sizeof(int) * B.cand.size(), hipMemcpyHostToDevice, e->st) != hipSuccess)
    return SQLM_ERR_HIP;
  hipLaunchKernelGGL(k_cand_dist, dim3((nq + 3) / 4), dim3(256), 0, e->st, dq, nq, dd1, dd2, dc, dd);
  if (hipMemcpyAsync(B.dist.data(), dd, sizeof(int) * total, hipMemcpyDeviceToHost, e->st) != hipSuccess ||
      hipStreamSynchronize(e->st) != hipSuccess)
    return SQLM_ERR_HIP;
  return SQLM_OK;
}

struct RotHist {
  int hist[kHistoLength] = {0};
  std::vector<int> bin, idx;
  void push(float a1, float a2, int i) {
    const float factor = kHistoLength / 360.0f;
    float rot = a1 - a2;
    if (rot < 0.0) rot += 360.0f;
    int b = (int)std::round(rot * factor);
    if (b == kHistoLength) b = 0;
    bin.push_back(b);
    idx.push_back(i);
    hist[b]++;
  }
  // every entry of a rejected bin, bin by bin
  template <class F>
  void reject(int &nmatches, F clear) {
    int ind1, ind2, ind3;
    three_maxima(hist, ind1, ind2, ind3);
    for (int b = 0; b < kHistoLength; b++) {
      if (b == ind1 || b == ind2 || b == ind3) continue;
      for (size_t q = 0; q < bin.size(); ++q)
        if (bin[q] == b) {
          clear(idx[q]);
          nmatches--;
        }
    }
  }
};

int orb_search_by_bow_kf_frame(OrbEngine *e, const sqlm_bow_frame *KF, const sqlm_bow_frame *F, float nnratio,
                               int check_ori, int32_t *matches, int *n_matches) {
  if (!bow_ok(KF) || !bow_ok(F) || (F->n && !matches)) return SQLM_ERR_INVALID_ARG;
  for (int i = 0; i < F->n; ++i) matches[i] = -1;
  if (n_matches) *n_matches = 0;
  BowPlan B;
  if (int rc = bow_plan(e, KF, F, B)) return rc;
  int nmatches = 0;
  RotHist R;
  for (const int4 &Q : B.q) {  // :296-362
    const int realIdxKF = Q.x;
    if (KF->mp[realIdxKF] < 0 || (KF->mp_bad && KF->mp_bad[realIdxKF])) continue;
    int bestDist1 = 256, bestIdxF = -1, bestDist2 = 256;
    for (int j = Q.y; j < Q.z; ++j) {
      const int realIdxF = B.cand[j];
      if (matches[realIdxF] >= 0) continue;
      const int dist = B.dist[Q.w + j - Q.y];
      if (dist < bestDist1) {
        bestDist2 = bestDist1;
        bestDist1 = dist;
        bestIdxF = realIdxF;
      } else if (dist < bestDist2) {
        bestDist2 = dist;
      }
    }
    if (bestDist1 <= kThLow && (float)bestDist1 < nnratio * (float)bestDist2) {
      matches[bestIdxF] = KF->mp[realIdxKF];
      if (check_ori) R.push(KF->kps[realIdxKF].angle, F->kps[bestIdxF].angle, bestIdxF);
      nmatches++;
    }
  }
  if (check_ori) R.reject(nmatches, [&](int i) { matches[i] = -1; });
  if (n_matches) *n_matches = nmatches;
  return SQLM_OK;
}

int orb_search_by_bow_kf_kf(OrbEngine *e, const sqlm_bow_frame *K1, const sqlm_bow_frame *K2, float nnratio,
                            int check_ori, int32_t *matches12, int *n_matches) {
  if (!bow_ok(K1) || !bow_ok(K2) || (K1->n && !matches12)) return SQLM_ERR_INVALID_ARG;
  for (int i = 0; i < K1->n; ++i) matches12[i] = -1;
  if (n_matches) *n_matches = 0;
  BowPlan B;
  if (int rc = bow_plan(e, K1, K2, B)) return rc;
  std::vector<uint8_t> matched2(K2->n, 0);
  int nmatches = 0;
  RotHist R;
  for (const int4 &Q : B.q) {  // :775-845
    const int idx1 = Q.x;
    if (K1->mp[idx1] < 0 || (K1->mp_bad && K1->mp_bad[idx1])) continue;
    int bestDist1 = 256, bestIdx2 = -1, bestDist2 = 256;
    for (int j = Q.y; j < Q.z; ++j) {
      const int idx2 = B.cand[j];
      if (matched2[idx2] || K2->mp[idx2] < 0 || (K2->mp_bad && K2->mp_bad[idx2])) continue;
      const int dist = B.dist[Q.w + j - Q.y];
      if (dist < bestDist1) {
        bestDist2 = bestDist1;
        bestDist1 = dist;
        bestIdx2 = idx2;
      } else if (dist < bestDist2) {
        bestDist2 = dist;
      }
    }
    if (bestDist1 < kThLow && (float)bestDist1 < nnratio * (float)bestDist2) {
      matches12[idx1] = K2->mp[bestIdx2];
      matched2[bestIdx2] = 1;
      if (check_ori) R.push(K1->kps[idx1].angle, K2->kps[bestIdx2].angle, idx1);
      nmatches++;
    }
  }
  if (check_ori) R.reject(nmatches, [&](int i) { matches12[i] = -1; });
  if (n_matches) *n_matches = nmatches;
  return SQLM_OK;
}

int orb_search_for_triangulation(OrbEngine *e, const sqlm_bow_frame *K1, const sqlm_bow_frame *K2, const float *C1,
                                 const float *T2w, const float *cam2, const float *sf2, int n_levels2, const float *F12,
                                 int only_stereo, int check_ori, int32_t *m12, int *n_matches) {
  if (!bow_ok(K1) || !bow_ok(K2) || !C1 || !T2w || !cam2 || !sf2 || n_levels2 < 1 || !F12 || (K1->n && !m12))
    return SQLM_ERR_INVALID_ARG;
  for (int i = 0; i < K2->n; ++i)
    if (K2->kps[i].octave < 0 || K2->kps[i].octave >= n_levels2) return SQLM_ERR_INVALID_ARG;
  for (int i = 0; i < K1->n; ++i) m12[i] = -1;
  if (n_matches) *n_matches = 0;
  // epipole of pKF1's centre in pKF2 (:903-913)
  const float t2[3] = {T2w[3], T2w[7], T2w[11]};
  float C2[3];
  mat3_mul_add(T2w, false, C1, t2, 1.0, C2);
  const float invz = 1.0f / C2[2];
  const float ex = cam2[0] * C2[0] * invz + cam2[2], ey = cam2[1] * C2[1] * invz + cam2[3];
  BowPlan B;
  if (int rc = bow_plan(e, K1, K2, B)) return rc;
  std::vector<uint8_t> matched2(K2->n, 0);
  int nmatches = 0;
  RotHist R;
  for (const int4 &Q : B.q) {  // :936-1030
    const int idx1 = Q.x;
    if (K1->mp[idx1] >= 0) continue;
    const bool bStereo1 = K1->uright && K1->uright[idx1] >= 0;
    if (only_stereo && !bStereo1) continue;
    const sqlm_keypoint &kp1 = K1->kps[idx1];
    int bestDist = kThLow, bestIdx2 = -1;
    for (int j = Q.y; j < Q.z; ++j) {
      const int idx2 = B.cand[j];
      if (matched2[idx2] || K2->mp[idx2] >= 0) continue;
      const bool bStereo2 = K2->uright && K2->uright[idx2] >= 0;
      if (only_stereo && !bStereo2) continue;
      const int dist = B.dist[Q.w + j - Q.y];
      if (dist > kThLow || dist > bestDist) continue;
      const sqlm_keypoint &kp2 = K2->kps[idx2];
      if (!bStereo1 && !bStereo2) {
        const float distex = ex - kp2.x, distey = ey - kp2.y;
        if (distex * distex + distey * distey < 100 * sf2[kp2.octave]) continue;
      }
      // CheckDistEpipolarLine (:203-229)
      const float a = kp1.x * F12[0] + kp1.y * F12[3] + F12[6];
      const float b = kp1.x * F12[1] + kp1.y * F12[4] + F12[7];
      const float c = kp1.x * F12[2] + kp1.y * F12[5] + F12[8];
      const float num = a * kp2.x + b * kp2.y + c;
      const float den = a * a + b * b;
      if (den == 0) continue;
      const float dsqr = num * num / den;
      if (dsqr < 3.84 * (sf2[kp2.octave] * sf2[kp2.octave])) {
        bestIdx2 = idx2;
        bestDist = dist;
      }
    }
    if (bestIdx2 >= 0) {
      m12[idx1] = bestIdx2;
      matched2[bestIdx2] = 1;
      nmatches++;
      if (check_ori) R.push(kp1.angle, K2->kps[bestIdx2].angle, idx1);
    }
  }
  if (check_ori)
    R.reject(nmatches, [&](int i) {
      matched2[m12[i]] = 0;
      m12[i] = -1;
    });
  if (n_matches) *n_matches = nmatches;
  return SQLM_OK;
}

// ---- SearchBySim3 (ORBmatcher.cc:1448-1608): two independent directions,
// then the mutual check — no order dependence, every window on the GPU ----
static int sim3_direction(OrbEngine *e, const sqlm_orb_frame *cam, const sqlm_orb_frame *dst, const float *Tsw,
                          const float *sR, const float *t, const sqlm_map_point *mp, const uint8_t *md, int n,
                          const std::vector<uint8_t> &already, float th, std::vector<int> &vnMatch) {
  float sRT[12];
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c) sRT[r * 4 + c] = sR[r * 3 + c];
    sRT[r * 4 + 3] = 0.f;
  }
  const float ts[3] = {Tsw[3], Tsw[7], Tsw[11]};
  const float log_scale = std::log(dst->scale_factors[1]);
  std::vector<float4> hq(n);
  for (int i = 0; i < n; i++) {  // :1499-1540 / :1545-1586
    hq[i] = area_query(0.f, 0.f, 0.f, kAreaSkip);
    const sqlm_map_point &p = mp[i];
    if (p.id < 0 || already[i] || p.skip) continue;
    const float X[3] = {p.x, p.y, p.z};
    float Xs[3], Xd[3];
    mat3_mul_add(Tsw, false, X, ts, 1.0, Xs);
    mat3_mul_add(sRT, false, Xs, t, 1.0, Xd);
    if (Xd[2] < 0.0) continue;
    const float invz = (float)(1.0 / (double)Xd[2]);
    const float x = Xd[0] * invz, y = Xd[1] * invz;
    const float u = cam->fx * x + cam->cx, v = cam->fy * y + cam->cy;
    if (!(u >= dst->bounds.min_x && u < dst->bounds.max_x && v >= dst->bounds.min_y && v < dst->bounds.max_y))
      continue;
    const float maxDistance = 1.2f * p.max_dist, minDistance = 0.8f * p.min_dist;
    const float dist3D = norm3(Xd);
    if (dist3D < minDistance || dist3D > maxDistance) continue;
    const int pl = predict_scale(p.max_dist, dist3D, log_scale, dst->n_levels);
    hq[i] = area_query(u, v, th * dst->scale_factors[pl], area_levels(pl - 1, pl));
  }
  std::vector<int> hoff;
  std::vector<int2> hp;
  if (int rc = area_search(e, dst->kps, dst->desc, dst->n, &dst->bounds, hq, md, hoff, hp)) return rc;
  vnMatch.assign(n, -1);
  for (int i = 0; i < n; ++i) {
    int bestDist = INT_MAX, bestIdx = -1;
    for (int q = hoff[i]; q < hoff[i + 1]; ++q)
      if (hp[q].y < bestDist) {
        bestDist = hp[q].y;
        bestIdx = hp[q].x;
      }
    if (bestDist <= kThHigh) vnMatch[i] = bestIdx;
  }
  return SQLM_OK;
}

int orb_search_by_sim3(OrbEngine *e, const sqlm_orb_frame *K1, const sqlm_orb_frame *K2, const float *T1w,
                       const float *T2w, const sqlm_map_point *mp1, const uint8_t *md1, const sqlm_map_point *mp2,
                       const uint8_t *md2, float s12, const float *R12, const float *t12, float th, int32_t *matches12,
                       int *n_found) {
  if (!kf_frame_ok(K1) || !kf_frame_ok(K2) || !T1w || !T2w || !R12 || !t12 ||
      (K1->n && (!mp1 || !md1 || !matches12)) || (K2->n && (!mp2 || !md2)))
    return SQLM_ERR_INVALID_ARG;
  if (n_found) *n_found = 0;
  const int N1 = K1->n, N2 = K2->n;
  // sR12 = s12 R12, sR21 = (1 / s12) R12^T, t21 = -sR21 t12 (:1466-1469)
  float sR12[9], sR21[9], t21[3], sR21T[12];
  const float inv_s = (float)(1.0 / (double)s12);
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      sR12[r * 3 + c] = R12[r * 3 + c] * s12;
      sR21[r * 3 + c] = R12[c * 3 + r] * inv_s;
      sR21T[r * 4 + c] = sR21[r * 3 + c];
    }
  for (int r = 0; r < 3; ++r) sR21T[r * 4 + 3] = 0.f;
  mat3_mul_add(sR21T, false, t12, nullptr, -1.0, t21);
  // vbAlreadyMatched1 / 2 (:1480-1494): GetIndexInKeyFrame(pKF2) = pKF2's slot of the same point
  std::vector<uint8_t> am1(N1, 0), am2(N2, 0);
  {
    std::vector<int32_t> ids;
    for (int i = 0; i < N1; i++)
      if (matches12[i] >= 0) {
        am1[i] = 1;
        ids.push_back(matches12[i]);
      }
    std::sort(ids.begin(), ids.end());
    for (int j = 0; j < N2; ++j)
      if (std::binary_search(ids.begin(), ids.end(), mp2[j].id)) am2[j] = 1;
  }
  std::vector<int> vnMatch1, vnMatch2;
  if (int rc = sim3_direction(e, K1, K2, T1w, sR21, t21, mp1, md1, N1, am1, th, vnMatch1)) return rc;
  if (int rc = sim3_direction(e, K1, K1, T2w, sR12, t12, mp2, md2, N2, am2, th, vnMatch2)) return rc;
  int nFound = 0;
  for (int i1 = 0; i1 < N1; i1++) {  // :1592-1606
    const int idx2 = vnMatch1[i1];
    if (idx2 >= 0 && vnMatch2[idx2] == i1) {
      matches12[i1] = mp2[idx2].id;
      nFound++;
    }
  }
  if (n_found) *n_found = nFound;
  return SQLM_OK;
}

}  // namespace sqlm
