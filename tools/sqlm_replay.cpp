// sqlm_replay — replay captured Optimizer-seam calls (include/sqrtlm_capture.h)
// on the GPU and compare with the write-back recorded in the capture.
//
//   sqlm_replay [--device N] capture.sqcap [more.sqcap ...]
//
// Prints one JSON line per file: the schedule's per-pass iterations / trials /
// chi2, the replay time, and, when the capture holds the reference's results,
// max relative pose / point differences (float write-back), outlier-tag
// mismatches and chi2 agreement. Exit status 0 iff every file replayed and,
// where results exist, poses and points agree within --tol (default 1e-6)
// and the outlier tags are identical.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "sqrtlm.h"
#include "sqrtlm_capture.h"

namespace {

double max_rel(const float *a, const float *b, size_t n) {
  double d = 0.0, m = 1.0;
  for (size_t i = 0; i < n; ++i) {
    d = std::fmax(d, std::fabs((double)a[i] - (double)b[i]));
    m = std::fmax(m, std::fabs((double)b[i]));
  }
  return d / m;
}

}  // namespace

int main(int argc, char **argv) {
  int device = -1;
  double tol = 1e-6;
  std::vector<const char *> files;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--device") && i + 1 < argc) device = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--tol") && i + 1 < argc) tol = std::atof(argv[++i]);
    else files.push_back(argv[i]);
  }
  if (files.empty()) {
    std::fprintf(stderr, "usage: sqlm_replay [--device N] [--tol T] capture.sqcap ...\n");
    return 2;
  }
  sqlm_ctx *ctx = nullptr;
  int s = sqlm_ctx_create(device, &ctx);
  if (s) {
    std::fprintf(stderr, "sqlm_ctx_create: %s\n", sqlm_status_string(s));
    return 1;
  }
  int bad = 0;
  for (const char *path : files) {
    sqlm_capture *c = nullptr;
    s = sqlm_capture_read(path, &c);
    if (s) {
      std::printf("{\"file\": \"%s\", \"error\": \"%s\"}\n", path, sqlm_status_string(s));
      ++bad;
      continue;
    }
    std::vector<float> Tcw(16 * (size_t)c->n_pose), pt(3 * (size_t)c->n_pt);
    std::vector<uint8_t> outl(c->n_obs);
    std::vector<double> chi(c->n_obs);
    sqlm_replay_out out{};
    out.Tcw = Tcw.data();
    out.pt = pt.data();
    out.outlier = outl.data();
    out.chi2 = chi.data();
    const auto t0 = std::chrono::steady_clock::now();
    s = sqlm_capture_replay(ctx, c, nullptr, &out);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (s) {
      std::printf("{\"file\": \"%s\", \"error\": \"%s\"}\n", path, sqlm_status_string(s));
      ++bad;
      sqlm_capture_free(c);
      continue;
    }
    std::printf("{\"file\": \"%s\", \"kind\": \"%s\", \"n_pose\": %d, \"n_pt\": %d, \"n_obs\": %lld, \"n_lid\": %lld, "
                "\"ms\": %.3f, \"passes\": [",
                path, c->kind == SQLM_CAP_LBA ? "lba" : "gba", c->n_pose, c->n_pt, (long long)c->n_obs,
                (long long)c->n_lid, ms);
    const int np = c->kind == SQLM_CAP_LBA ? 3 : 1;
    for (int k = 0; k < np; ++k)
      std::printf("%s{\"iterations\": %d, \"trials\": %d, \"chi2_begin\": %.9g, \"chi2_end\": %.9g}", k ? ", " : "",
                  out.stats[k].iterations, out.stats[k].trials, out.stats[k].chi2_begin, out.stats[k].chi2_end);
    std::printf("]");
    if (c->has_result) {
      const double dp = c->res_Tcw ? max_rel(Tcw.data(), c->res_Tcw, Tcw.size()) : 0.0;
      const double dx = c->res_pt ? max_rel(pt.data(), c->res_pt, pt.size()) : 0.0;
      long long mism = 0;
      if (c->res_outlier)
        for (int64_t e = 0; e < c->n_obs; ++e) mism += outl[e] != c->res_outlier[e];
      double dchi = 0.0;
      if (c->res_chi2)
        for (int64_t e = 0; e < c->n_obs; ++e)
          dchi = std::fmax(dchi, std::fabs(chi[e] - c->res_chi2[e]) / std::fmax(1e-9, std::fabs(c->res_chi2[e])));
      const bool ok = dp < tol && dx < tol && mism == 0;
      std::printf(", \"pose_rel\": %.3e, \"point_rel\": %.3e, \"outlier_mismatch\": %lld, \"chi2_rel\": %.3e, "
                  "\"parity\": %s",
                  dp, dx, mism, dchi, ok ? "true" : "false");
      bad += !ok;
    }
    std::printf("}\n");
    sqlm_capture_free(c);
  }
  sqlm_ctx_destroy(ctx);
  return bad ? 1 : 0;
}
