// sqlm_capture.cpp — capture file I/O and GPU replay of a captured seam call
// (include/sqrtlm_capture.h). Host code only; the replay
// drives the same public entry points an adapter would.
#include "../../include/sqrtlm_capture.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <new>
#include <vector>

namespace {

constexpr char kMagic[8] = {'S', 'Q', 'L', 'M', 'C', 'A', 'P', '1'};
constexpr uint32_t kVersion = 1;

constexpr uint32_t cc(char a, char b, char c, char d) {
  return (uint32_t)(uint8_t)a | ((uint32_t)(uint8_t)b << 8) | ((uint32_t)(uint8_t)c << 16) |
         ((uint32_t)(uint8_t)d << 24);
}

// section tags
constexpr uint32_t kDims = cc('D', 'I', 'M', 'S');  // int64 {n_pose, n_pt, n_obs, n_lid}
constexpr uint32_t kMeta = cc('M', 'E', 'T', 'A');  // int32 {gba_iterations, gba_robust, has_result, 0}
constexpr uint32_t kTcw = cc('T', 'C', 'W', '_'), kPFix = cc('P', 'F', 'I', 'X'), kIntr = cc('I', 'N', 'T', 'R');
constexpr uint32_t kBf = cc('B', 'F', '_', '_'), kKfId = cc('K', 'F', 'I', 'D');
constexpr uint32_t kPt = cc('P', 'N', 'T', '_'), kMpId = cc('M', 'P', 'I', 'D');
constexpr uint32_t kObsP = cc('O', 'B', 'S', 'P'), kObsL = cc('O', 'B', 'S', 'L'), kObsU = cc('O', 'B', 'S', 'U');
constexpr uint32_t kObsR = cc('O', 'B', 'S', 'R'), kObsI = cc('O', 'B', 'S', 'I'), kObsD = cc('O', 'B', 'S', 'D');
constexpr uint32_t kLidP = cc('L', 'I', 'D', 'P'), kLidC = cc('L', 'I', 'D', 'C'), kLidW = cc('L', 'I', 'D', 'W');
constexpr uint32_t kLidN = cc('L', 'I', 'D', 'N'), kLidI = cc('L', 'I', 'D', 'I');
constexpr uint32_t kRTcw = cc('R', 'T', 'C', 'W'), kRPt = cc('R', 'P', 'N', 'T'), kROut = cc('R', 'O', 'U', 'T');
constexpr uint32_t kRChi = cc('R', 'C', 'H', 'I');

struct Writer {
  FILE *f;
  bool ok = true;
  void raw(const void *p, size_t n) {
    if (ok && n && std::fwrite(p, 1, n, f) != n) ok = false;
  }
  void section(uint32_t tag, uint32_t elem, uint64_t count, const void *p) {
    if (!p) return;
    raw(&tag, 4);
    raw(&elem, 4);
    raw(&count, 8);
    raw(p, (size_t)elem * count);
  }
};

struct Section {
  uint32_t elem = 0;
  uint64_t count = 0;
  std::vector<uint8_t> data;
};

// copy a section into a malloc'd array of `count` elements of `elem` bytes;
// NULL if absent, -1 on a size mismatch
template <typename T>
int take(std::map<uint32_t, Section> &s, uint32_t tag, uint64_t count, T **out) {
  *out = nullptr;
  auto it = s.find(tag);
  if (it == s.end()) return 0;
  if (it->second.elem != sizeof(T) || it->second.count != count) return -1;
  if (count == 0) return 0;
  *out = static_cast<T *>(std::malloc(sizeof(T) * count));
  if (!*out) return -1;
  std::memcpy(*out, it->second.data.data(), sizeof(T) * count);
  return 0;
}

inline bool stopped(const volatile uint8_t *s) { return s && *s; }

}  // namespace

extern "C" {

int sqlm_capture_write(const char *path, const sqlm_capture *c) {
  if (!path || !c || c->n_pose < 0 || c->n_pt < 0 || c->n_obs < 0 || c->n_lid < 0) return SQLM_ERR_INVALID_ARG;
  if ((c->n_pose && (!c->Tcw || !c->pose_fixed || !c->intr)) || (c->n_pt && !c->pt) ||
      (c->n_obs && (!c->obs_pose || !c->obs_pt || !c->obs_uv || !c->obs_inv_sigma2)) ||
      (c->n_lid && (!c->lid_pose || !c->lid_pc || !c->lid_pw || !c->lid_n || !c->lid_info)))
    return SQLM_ERR_INVALID_ARG;
  FILE *f = std::fopen(path, "wb");
  if (!f) return SQLM_ERR_INVALID_ARG;
  Writer w{f};
  w.raw(kMagic, 8);
  w.raw(&kVersion, 4);
  w.raw(&c->kind, 4);
  const int64_t dims[4] = {c->n_pose, c->n_pt, c->n_obs, c->n_lid};
  const int32_t meta[4] = {c->gba_iterations, c->gba_robust, c->has_result, 0};
  w.section(kDims, 8, 4, dims);
  w.section(kMeta, 4, 4, meta);
  const uint64_t P = c->n_pose, N = c->n_pt, E = c->n_obs, L = c->n_lid;
  if (P) {
    w.section(kTcw, 4, 16 * P, c->Tcw);
    w.section(kPFix, 1, P, c->pose_fixed);
    w.section(kIntr, 4, 4 * P, c->intr);
    w.section(kBf, 4, P, c->bf);
    w.section(kKfId, 8, P, c->kf_id);
  }
  if (N) {
    w.section(kPt, 4, 3 * N, c->pt);
    w.section(kMpId, 8, N, c->mp_id);
  }
  if (E) {
    w.section(kObsP, 4, E, c->obs_pose);
    w.section(kObsL, 4, E, c->obs_pt);
    w.section(kObsU, 4, 2 * E, c->obs_uv);
    w.section(kObsR, 4, E, c->obs_ur);
    w.section(kObsI, 4, E, c->obs_inv_sigma2);
    w.section(kObsD, 4, E, c->obs_delta);
  }
  if (L) {
    w.section(kLidP, 4, L, c->lid_pose);
    w.section(kLidC, 8, 3 * L, c->lid_pc);
    w.section(kLidW, 8, 3 * L, c->lid_pw);
    w.section(kLidN, 8, 3 * L, c->lid_n);
    w.section(kLidI, 8, L, c->lid_info);
  }
  if (c->has_result) {
    if (P) w.section(kRTcw, 4, 16 * P, c->res_Tcw);
    if (N) w.section(kRPt, 4, 3 * N, c->res_pt);
    if (E) {
      w.section(kROut, 1, E, c->res_outlier);
      w.section(kRChi, 8, E, c->res_chi2);
    }
  }
  const bool ok = w.ok;
  if (std::fclose(f) != 0 || !ok) return SQLM_ERR_INVALID_ARG;
  return SQLM_OK;
}

void sqlm_capture_free(sqlm_capture *c) {
  if (!c) return;
  void *arrays[] = {c->Tcw, c->pose_fixed, c->intr, c->bf, c->kf_id, c->pt, c->mp_id, c->obs_pose, c->obs_pt,
                    c->obs_uv, c->obs_ur, c->obs_inv_sigma2, c->obs_delta, c->lid_pose, c->lid_pc, c->lid_pw,
                    c->lid_n, c->lid_info, c->res_Tcw, c->res_pt, c->res_outlier, c->res_chi2};
  for (void *p : arrays) std::free(p);
  std::free(c);
}

int sqlm_capture_read(const char *path, sqlm_capture **out) {
  if (!path || !out) return SQLM_ERR_INVALID_ARG;
  *out = nullptr;
  FILE *f = std::fopen(path, "rb");
  if (!f) return SQLM_ERR_INVALID_ARG;
  // bytes in the file: a section header may not claim more payload than is left
  int64_t file_size = -1;
  if (std::fseek(f, 0, SEEK_END) == 0) file_size = (int64_t)std::ftell(f);
  if (file_size < 0 || std::fseek(f, 0, SEEK_SET) != 0) {
    std::fclose(f);
    return SQLM_ERR_INVALID_ARG;
  }
  char magic[8];
  uint32_t version = 0, kind = 0;
  std::map<uint32_t, Section> secs;
  bool ok = std::fread(magic, 1, 8, f) == 8 && std::memcmp(magic, kMagic, 8) == 0 &&
            std::fread(&version, 4, 1, f) == 1 && std::fread(&kind, 4, 1, f) == 1 && version >= 1;
  while (ok) {
    uint32_t tag, elem;
    uint64_t count;
    if (std::fread(&tag, 4, 1, f) != 1) break;  // clean EOF between sections
    if (std::fread(&elem, 4, 1, f) != 1 || std::fread(&count, 8, 1, f) != 1 || elem == 0 || elem > 64 ||
        count > (uint64_t)1 << 40) {
      ok = false;
      break;
    }
    const int64_t pos = (int64_t)std::ftell(f);
    if (pos < 0 || (uint64_t)elem * count > (uint64_t)(file_size - pos)) {  // truncated / corrupt header
      ok = false;
      break;
    }
    Section s;
    s.elem = elem;
    s.count = count;
    try {
      s.data.resize((size_t)elem * count);
    } catch (const std::bad_alloc &) {
      std::fclose(f);
      return SQLM_ERR_OOM;
    }
    if (!s.data.empty() && std::fread(s.data.data(), 1, s.data.size(), f) != s.data.size()) {
      ok = false;
      break;
    }
    secs[tag] = std::move(s);  // unknown tags are kept and ignored
  }
  std::fclose(f);
  auto dims_it = secs.find(kDims), meta_it = secs.find(kMeta);
  if (!ok || dims_it == secs.end() || dims_it->second.count != 4 || dims_it->second.elem != 8 ||
      meta_it == secs.end() || meta_it->second.count != 4 || meta_it->second.elem != 4)
    return SQLM_ERR_INVALID_ARG;
  int64_t dims[4];
  int32_t meta[4];
  std::memcpy(dims, dims_it->second.data.data(), sizeof(dims));
  std::memcpy(meta, meta_it->second.data.data(), sizeof(meta));
  if (dims[0] < 0 || dims[1] < 0 || dims[2] < 0 || dims[3] < 0 || dims[0] > INT32_MAX || dims[1] > INT32_MAX)
    return SQLM_ERR_INVALID_ARG;
  sqlm_capture *c = static_cast<sqlm_capture *>(std::calloc(1, sizeof(sqlm_capture)));
  if (!c) return SQLM_ERR_OOM;
  c->kind = kind;
  c->n_pose = (int32_t)dims[0];
  c->n_pt = (int32_t)dims[1];
  c->n_obs = dims[2];
  c->n_lid = dims[3];
  c->gba_iterations = meta[0];
  c->gba_robust = (uint8_t)meta[1];
  c->has_result = (uint8_t)meta[2];
  const uint64_t P = c->n_pose, N = c->n_pt, E = c->n_obs, L = c->n_lid;
  int bad = 0;
  bad |= take(secs, kTcw, 16 * P, &c->Tcw) | take(secs, kPFix, P, &c->pose_fixed) |
         take(secs, kIntr, 4 * P, &c->intr) | take(secs, kBf, P, &c->bf) | take(secs, kKfId, P, &c->kf_id);
  bad |= take(secs, kPt, 3 * N, &c->pt) | take(secs, kMpId, N, &c->mp_id);
  bad |= take(secs, kObsP, E, &c->obs_pose) | take(secs, kObsL, E, &c->obs_pt) | take(secs, kObsU, 2 * E, &c->obs_uv) |
         take(secs, kObsR, E, &c->obs_ur) | take(secs, kObsI, E, &c->obs_inv_sigma2) |
         take(secs, kObsD, E, &c->obs_delta);
  bad |= take(secs, kLidP, L, &c->lid_pose) | take(secs, kLidC, 3 * L, &c->lid_pc) |
         take(secs, kLidW, 3 * L, &c->lid_pw) | take(secs, kLidN, 3 * L, &c->lid_n) |
         take(secs, kLidI, L, &c->lid_info);
  bad |= take(secs, kRTcw, 16 * P, &c->res_Tcw) | take(secs, kRPt, 3 * N, &c->res_pt) |
         take(secs, kROut, E, &c->res_outlier) | take(secs, kRChi, E, &c->res_chi2);
  // required arrays, index ranges
  if (!bad && ((P && (!c->Tcw || !c->pose_fixed || !c->intr)) || (N && !c->pt) ||
               (E && (!c->obs_pose || !c->obs_pt || !c->obs_uv || !c->obs_inv_sigma2)) ||
               (L && (!c->lid_pose || !c->lid_pc || !c->lid_pw || !c->lid_n || !c->lid_info))))
    bad = 1;
  for (uint64_t e = 0; !bad && e < E; ++e)
    if (c->obs_pose[e] < 0 || c->obs_pose[e] >= c->n_pose || c->obs_pt[e] < 0 || c->obs_pt[e] >= c->n_pt) bad = 1;
  for (uint64_t e = 0; !bad && e < L; ++e)
    if (c->lid_pose[e] < 0 || c->lid_pose[e] >= c->n_pose) bad = 1;
  if (bad) {
    sqlm_capture_free(c);
    return SQLM_ERR_INVALID_ARG;
  }
  *out = c;
  return SQLM_OK;
}

int sqlm_capture_replay(sqlm_ctx *ctx, const sqlm_capture *c, const volatile uint8_t *stop, sqlm_replay_out *out) {
  if (!ctx || !c || (c->kind != SQLM_CAP_LBA && c->kind != SQLM_CAP_GBA)) return SQLM_ERR_INVALID_ARG;
  if (c->n_pose <= 0) return SQLM_ERR_INVALID_ARG;
  const bool lba = c->kind == SQLM_CAP_LBA;
  // Converter::toSE3Quat per keyframe, float -> double widening elsewhere
  std::vector<double> q(4 * (size_t)c->n_pose), t(3 * (size_t)c->n_pose), intr(4 * (size_t)c->n_pose);
  for (int p = 0; p < c->n_pose; ++p) {
    sqlm_pose_from_Tcw_f32(c->Tcw + 16 * (size_t)p, &q[4 * p], &t[3 * p]);
    for (int k = 0; k < 4; ++k) intr[4 * p + k] = c->intr[4 * p + k];
  }
  // Edges: LBA keeps mono observations only (the stereo branch of
  // g2oOptimizer.cc:914-916 adds nothing); a point left without edges is not
  // a vertex of the problem (GBA removes it, :285-289; in LBA it has no
  // Hessian and does not move), so it is compacted away and written back unchanged.
  std::vector<int64_t> edge_of;  // problem edge -> capture observation
  std::vector<uint8_t> stereo;
  for (int64_t e = 0; e < c->n_obs; ++e) {
    const bool st = c->obs_ur && c->obs_ur[e] >= 0.f;
    if (lba && st) continue;
    edge_of.push_back(e);
    stereo.push_back(st);
  }
  std::vector<int32_t> pt_map(c->n_pt, -1), pt_src;
  for (int64_t e : edge_of) pt_map[c->obs_pt[e]] = 0;
  // problem points keep the capture's point order (vertex id order)
  for (int32_t i = 0; i < c->n_pt; ++i)
    if (pt_map[i] >= 0) {
      pt_map[i] = (int32_t)pt_src.size();
      pt_src.push_back(i);
    }
  const int64_t E = (int64_t)edge_of.size();
  const int NL = (int)pt_src.size();
  std::vector<double> pt(3 * (size_t)NL), uv(2 * (size_t)E), info(E), delta(E, 0.0), ur;
  std::vector<int32_t> op(E), ol(E);
  for (int i = 0; i < NL; ++i)
    for (int k = 0; k < 3; ++k) pt[3 * i + k] = c->pt[3 * (size_t)pt_src[i] + k];
  bool any_stereo = false;
  for (int64_t k = 0; k < E; ++k) {
    const int64_t e = edge_of[k];
    op[k] = c->obs_pose[e];
    ol[k] = pt_map[c->obs_pt[e]];
    uv[2 * k] = c->obs_uv[2 * e];
    uv[2 * k + 1] = c->obs_uv[2 * e + 1];
    info[k] = c->obs_inv_sigma2[e];
    if (c->obs_delta && (lba || c->gba_robust)) delta[k] = c->obs_delta[e];
    any_stereo |= stereo[k] != 0;
  }
  int s = sqlm_set_problem(ctx, c->n_pose, q.data(), t.data(), c->pose_fixed, intr.data(), NL, pt.data(), E, op.data(),
                           ol.data(), uv.data(), info.data(), delta.data(), nullptr);
  if (s) return s;
  if (any_stereo) {
    if (!c->bf) return SQLM_ERR_INVALID_ARG;
    ur.assign(E, -1.0);
    for (int64_t k = 0; k < E; ++k)
      if (stereo[k]) ur[k] = c->obs_ur[edge_of[k]];
    std::vector<double> bf(c->n_pose);
    for (int p = 0; p < c->n_pose; ++p) bf[p] = c->bf[p];
    s = sqlm_set_stereo(ctx, ur.data(), bf.data());
    if (s) return s;
  }
  sqlm_replay_out tmp;
  if (!out) out = &tmp;
  std::memset(out->stats, 0, sizeof(out->stats));
  out->ran = 0;
  std::vector<uint8_t> outl(E, 0);
  if (lba) {
    if (c->n_lid) {
      s = sqlm_set_lidar(ctx, c->n_lid, c->lid_pose, c->lid_pc, c->lid_pw, c->lid_n, c->lid_info);
      if (s) return s;
    }
    s = sqlm_local_ba(ctx, stop, outl.data(), out->stats, &out->ran);
  } else {
    if (c->n_lid) return SQLM_ERR_INVALID_ARG;  // the reference's GBA has no LiDAR edges
    int n = 0;
    out->ran = !stopped(stop);
    s = sqlm_global_ba(ctx, c->gba_iterations, stop, &out->stats[0], &n);
  }
  if (s) return s;
  // write-back: Converter::toCvMat for poses, float points
  if (out->Tcw) {
    s = sqlm_get_poses(ctx, q.data(), t.data());
    if (s) return s;
    for (int p = 0; p < c->n_pose; ++p) sqlm_pose_to_Tcw_f32(&q[4 * p], &t[3 * p], out->Tcw + 16 * (size_t)p);
  }
  if (out->pt) {
    s = sqlm_get_points(ctx, pt.data());
    if (s) return s;
    for (int32_t i = 0; i < c->n_pt; ++i)
      for (int k = 0; k < 3; ++k)
        out->pt[3 * (size_t)i + k] = pt_map[i] >= 0 ? (float)pt[3 * (size_t)pt_map[i] + k] : c->pt[3 * (size_t)i + k];
  }
  if (out->outlier || out->chi2) {
    std::vector<double> chi(E);
    s = sqlm_get_edge_chi2(ctx, chi.data());
    if (s) return s;
    if (out->outlier) std::memset(out->outlier, 0, (size_t)c->n_obs);
    if (out->chi2)
      for (int64_t e = 0; e < c->n_obs; ++e) out->chi2[e] = 0.0;
    for (int64_t k = 0; k < E; ++k) {
      if (out->outlier) out->outlier[edge_of[k]] = lba ? outl[k] : 0;
      if (out->chi2) out->chi2[edge_of[k]] = chi[k];
    }
  }
  return SQLM_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- KITTI trajectory

namespace {
// c = a b for row-major 4x4 float matrices, k summed in order in float
void mul4(const float *a, const float *b, float *c) {
  float t[16];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      float s = 0.f;
      for (int k = 0; k < 4; ++k) s += a[4 * i + k] * b[4 * k + j];
      t[4 * i + j] = s;
    }
  std::memcpy(c, t, sizeof(t));
}
}  // namespace

int sqlm_save_trajectory_kitti(const char *path, int n_frames, const float *Tcr, const int32_t *frame_ref, int n_kf,
                               const float *Tcw, const float *Tcp, const int32_t *parent, const uint8_t *bad,
                               int origin_kf) {
  if (!path || n_frames < 0 || n_kf <= 0 || origin_kf < 0 || origin_kf >= n_kf || !Tcw || !parent ||
      (n_frames && (!Tcr || !frame_ref)) || (bad && !Tcp))
    return SQLM_ERR_INVALID_ARG;
  for (int f = 0; f < n_frames; ++f)
    if (frame_ref[f] < 0 || frame_ref[f] >= n_kf) return SQLM_ERR_INVALID_ARG;
  // Two = origin keyframe's Twc (KeyFrame::SetPose: Rwc = Rcw^T, Ow = -Rwc tcw)
  const float *T0 = Tcw + 16 * (size_t)origin_kf;
  float Two[16] = {0};
  for (int i = 0; i < 3; ++i) {
    float o = 0.f;
    for (int k = 0; k < 3; ++k) {
      Two[4 * i + k] = T0[4 * k + i];
      o += -T0[4 * k + i] * T0[4 * k + 3];
    }
    Two[4 * i + 3] = o;
  }
  Two[15] = 1.f;
  FILE *fp = std::fopen(path, "w");
  if (!fp) return SQLM_ERR_INVALID_ARG;
  int st = SQLM_OK;
  for (int f = 0; f < n_frames && st == SQLM_OK; ++f) {
    float Trw[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    int k = frame_ref[f], hops = 0;
    while (bad && bad[k]) {  // Trw = Trw * pKF->mTcp; pKF = pKF->GetParent()
      mul4(Trw, Tcp + 16 * (size_t)k, Trw);
      k = parent[k];
      if (k < 0 || k >= n_kf || ++hops > n_kf) { st = SQLM_ERR_INVALID_ARG; break; }
    }
    if (st) break;
    mul4(Trw, Tcw + 16 * (size_t)k, Trw);
    mul4(Trw, Two, Trw);
    float T[16];
    mul4(Tcr + 16 * (size_t)f, Trw, T);
    // Rwc = R^T, twc = -Rwc t (cv::Mat float products)
    float Rwc[9], twc[3];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Rwc[3 * i + j] = T[4 * j + i];
    for (int i = 0; i < 3; ++i) {
      float s = 0.f;
      for (int j = 0; j < 3; ++j) s += -Rwc[3 * i + j] * T[4 * j + 3];
      twc[i] = s;
    }
    std::fprintf(fp, "%.9f %.9f %.9f %.9f %.9f %.9f %.9f %.9f %.9f %.9f %.9f %.9f\n", Rwc[0], Rwc[1], Rwc[2], twc[0],
                 Rwc[3], Rwc[4], Rwc[5], twc[1], Rwc[6], Rwc[7], Rwc[8], twc[2]);
  }
  if (std::fclose(fp) != 0 && st == SQLM_OK) st = SQLM_ERR_INVALID_ARG;
  return st;
}
