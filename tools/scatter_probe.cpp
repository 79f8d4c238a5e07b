// scatter_probe — host-side timing of the setup's observation scatter
// (sqlm_api.cpp prepare(): edges -> landmark slot order) on synthetic data of
// config-4 shape: 5M edges in landmark runs of 2..18, 500k landmarks whose
// slots are a shuffled order (the span sort). Variants: edge order (writes
// scattered), slot order (reads scattered) with software prefetch 0 / 8 / 16
// slots ahead, with and without MADV_HUGEPAGE on the inputs.
// Build: g++ -O2 -std=c++17 -pthread tools/scatter_probe.cpp -o tools/scatter_probe
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <random>
#include <thread>
#include <vector>

template <class T>
T *big(size_t n, bool huge) {
  void *p = nullptr;
  const size_t bytes = ((n * sizeof(T)) + (2u << 20) - 1) & ~size_t((2u << 20) - 1);
  if (posix_memalign(&p, 2u << 20, bytes)) std::abort();
  if (huge) madvise(p, bytes, MADV_HUGEPAGE);
  std::memset(p, 0, bytes);
  return static_cast<T *>(p);
}

template <class F>
void par(int nth, F &&f) {
  std::vector<std::thread> th;
  for (int t = 1; t < nth; ++t) th.emplace_back(f, t);
  f(0);
  for (auto &x : th) x.join();
}

int main(int argc, char **argv) {
  const int nth = argc > 1 ? std::atoi(argv[1]) : 8;
  const int nL = 500000;
  std::mt19937_64 rng(4);
  std::vector<int> len(nL);
  int64_t nE = 0;
  for (int l = 0; l < nL; ++l) nE += len[l] = 2 + (int)(rng() % 17);
  for (int huge = 0; huge < 2; ++huge) {
    int *pt = big<int>(nE, huge), *pose = big<int>(nE, huge);
    double *uv = big<double>(2 * nE, huge), *info = big<double>(nE, huge), *delta = big<double>(nE, huge);
    std::vector<int> efirst(nL), pts(nL), slot(nL), lm_begin(nL + 1, 0);
    int64_t e = 0;
    for (int l = 0; l < nL; ++l) {
      efirst[l] = (int)e;
      for (int i = 0; i < len[l]; ++i, ++e) {
        pt[e] = l;
        pose[e] = (int)(rng() % 5000);
        uv[2 * e] = 1.0;
        uv[2 * e + 1] = 2.0;
        info[e] = 1.0;
        delta[e] = 0.5;
      }
    }
    std::iota(pts.begin(), pts.end(), 0);
    std::shuffle(pts.begin(), pts.end(), rng);
    for (int s = 0; s < nL; ++s) {
      slot[pts[s]] = s;
      lm_begin[s + 1] = lm_begin[s] + len[pts[s]];
    }
    int *o_lm = big<int>(nE, huge), *o_cam = big<int>(nE, huge);
    float *o_q = big<float>(4 * nE, huge);
    int64_t *dev_edge = big<int64_t>(nE, huge);
    auto put = [&](int64_t e, int o, int sl) {
      dev_edge[o] = e;
      o_lm[o] = sl;
      o_cam[o] = pose[e];
      o_q[4 * (size_t)o] = (float)uv[2 * e];
      o_q[4 * (size_t)o + 1] = (float)uv[2 * e + 1];
      o_q[4 * (size_t)o + 2] = (float)info[e];
      o_q[4 * (size_t)o + 3] = (float)delta[e];
    };
    auto time = [&](const char *what, auto &&body) {
      double best = 1e30;
      for (int r = 0; r < 5; ++r) {
        const auto t0 = std::chrono::steady_clock::now();
        par(nth, body);
        best = std::min(best, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
      }
      std::printf("{\"huge\": %d, \"threads\": %d, \"variant\": \"%s\", \"best_ms\": %.2f}\n", huge, nth, what, best);
    };
    time("edge order", [&](int t) {
      for (int64_t e = nE * t / nth; e < nE * (t + 1) / nth; ++e) {
        const int l = pt[e], sl = slot[l];
        put(e, lm_begin[sl] + (int)(e - efirst[l]), sl);
      }
    });
    auto by_slot = [&](int pf) {
      return [&, pf](int t) {
        const int s1 = (int)((int64_t)nL * (t + 1) / nth);
        for (int sl = (int)((int64_t)nL * t / nth); sl < s1; ++sl) {
          if (pf > 0 && sl + 2 * pf < s1) __builtin_prefetch(&efirst[pts[sl + 2 * pf]]);
          if (pf > 0 && sl + pf < s1) {
            const int64_t ep = efirst[pts[sl + pf]];
            __builtin_prefetch(&uv[2 * ep]);
            __builtin_prefetch(&info[ep]);
            __builtin_prefetch(&delta[ep]);
            __builtin_prefetch(&pose[ep]);
          }
          const int b = lm_begin[sl], k = lm_begin[sl + 1] - b;
          const int64_t e0 = efirst[pts[sl]];
          for (int i = 0; i < k; ++i) put(e0 + i, b + i, sl);
        }
      };
    };
    time("slot order pf0", by_slot(0));
    time("slot order pf8", by_slot(8));
    time("slot order pf16", by_slot(16));
    for (void *p : {(void *)pt, (void *)pose, (void *)uv, (void *)info, (void *)delta, (void *)o_lm, (void *)o_cam,
                    (void *)o_q, (void *)dev_edge})
      std::free(p);
  }
  return 0;
}
