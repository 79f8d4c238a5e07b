// sqlm_api.cpp — C ABI (include/sqrtlm.h) and host LM driver.
//
// The host side owns only control: it mirrors g2o's Levenberg–Marquardt loop
// decision for decision (optimization_algorithm_levenberg.cpp:61-164,
// sparse_optimizer.cpp:354-419) and keeps every array in HBM; one small
// device->host copy of the reduced scalars per LM trial is the only sync.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cmath>
#include <cstring>
#include <functional>
#include <limits>
#include <mutex>
#include <new>
#include <queue>
#include <thread>
#include <sys/mman.h>
#include <unistd.h>
#include <vector>

#include "../../include/sqrtlm.h"
#include "../../include/sqrtlm_orb.h"
#include "se3_dev.h"
#include "sqlm_comm.h"
#include "sqlm_internal.h"

using namespace sqlm;

namespace {

struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
  size_t map = 0;  // page-locked buffers: mapped length of a registered huge-page mapping (0: hipHostMalloc)
};

// Large host arrays on transparent huge pages. The setup's scatter and
// planning passes read 5M-edge arrays at random landmark runs and write the
// page-locked upload buffers; with 4 KiB pages nearly every run costs TLB
// misses. MADV_HUGEPAGE is set before the first touch (the box's THP mode is
// "madvise"); arrays under one huge page use malloc. (SQLM_HOST_HUGE=0: A/B.)
#ifndef SQLM_HOST_HUGE
#define SQLM_HOST_HUGE 1
#endif
constexpr size_t kHugePage = size_t(2) << 20;
inline size_t huge_len(size_t bytes) { return (bytes + kHugePage - 1) & ~(kHugePage - 1); }
// an anonymous mapping of huge_len(bytes), aligned to a huge page, advised; nullptr on failure
inline void *huge_map(size_t bytes) {
  const size_t len = huge_len(bytes);
  void *raw = mmap(nullptr, len + kHugePage, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (raw == MAP_FAILED) return nullptr;
  const uintptr_t r = (uintptr_t)raw, a = (r + kHugePage - 1) & ~(uintptr_t)(kHugePage - 1);
  if (a > r) munmap(raw, a - r);
  if (r + kHugePage > a) munmap((void *)(a + len), r + kHugePage - a);
  (void)madvise((void *)a, len, MADV_HUGEPAGE);
  return (void *)a;
}
template <class T>
struct HugeAlloc {
  using value_type = T;
  HugeAlloc() = default;
  template <class U>
  HugeAlloc(const HugeAlloc<U> &) {}
  static bool huge(size_t n) { return SQLM_HOST_HUGE && n * sizeof(T) >= kHugePage; }
  T *allocate(size_t n) {
    void *p = huge(n) ? huge_map(n * sizeof(T)) : std::malloc(std::max<size_t>(n, 1) * sizeof(T));
    if (!p) throw std::bad_alloc();
    return static_cast<T *>(p);
  }
  void deallocate(T *p, size_t n) {
    if (huge(n)) munmap(p, huge_len(n * sizeof(T)));
    else std::free(p);
  }
  template <class U>
  bool operator==(const HugeAlloc<U> &) const { return true; }
  template <class U>
  bool operator!=(const HugeAlloc<U> &) const { return false; }
};
template <class T>
using HVec = std::vector<T, HugeAlloc<T>>;

struct Timer {
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  double ms() const {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
};

const char *kTimerNames[SQLM_NKERNEL_TIMERS] = {"k_linearize", "k_camera_pass", "k_damp", "k_rcs_tile",
                                                "k_solve", "k_pose_update", "k_landmark_update", "reduce+sync",
                                                "k_rcs_reduce"};

}  // namespace

// Landmark tiles for the RCS assembly: runs of consecutive slots whose free
// cameras fit a window of <= kTileMaxCams cameras (sorted), plus the reduction
// lists that sum each S block / g row from its tiles in tile order.
struct TilePlan {
  std::vector<int> lm_ptr{0}, cam_ptr{0}, cams, ld, red_ptr, gred_ptr;
  std::vector<int2> urange, gred_idx;
  std::vector<int64_t> red_off;   // absolute offset (doubles) of each contribution's 6x6 block in part
  std::vector<int64_t> gred_off;  // ... and of each g contribution's 6 doubles in gpart
  std::vector<int> long_s, long_g;  // S blocks / cameras with more than kRedLong contributions
  std::vector<int64_t> part_ptr{0}, gpart_ptr{0};
  int max_cp = 0;
  bool dups = false;
  std::vector<int> order;  // tile ids grouped by nt class (ascending id within a class)
  int cls_off[kTileNtMax + 2] = {}, cls_cnt[kTileNtMax + 1] = {};
  // back to the empty plan, keeping every vector's memory (a context reuses
  // its plan across calls: no reallocation, no first-touch page faults)
  void reset() {
    lm_ptr.assign(1, 0);
    cam_ptr.assign(1, 0);
    part_ptr.assign(1, 0);
    gpart_ptr.assign(1, 0);
    for (auto *v : {&cams, &ld, &red_ptr, &gred_ptr, &long_s, &long_g, &order}) v->clear();
    urange.clear();
    gred_idx.clear();
    red_off.clear();
    gred_off.clear();
    max_cp = 0;
    dups = false;
    std::fill(cls_off, cls_off + kTileNtMax + 2, 0);
    std::fill(cls_cnt, cls_cnt + kTileNtMax + 1, 0);
  }
};



// Intermediate state of build_tiles between the tiles (passes 1-2) and the
// reduction lists, which need the S pattern (built from the tiles' camera
// pairs in between).
struct TileBuild {
  struct Red { int key, tile, code, j; };  // key: camera i until the pattern exists, then the S block
  struct TileOut { std::vector<int> cams; std::vector<Red> red; };
  std::vector<int> tstart;
  std::vector<TileOut> out;
};

struct sqlm_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  // ---- host copy of the graph (caller order) ----
  bool has_problem = false;
  bool prepared = false;  // the last prepare() completed (CR plan, buffers valid)
  int n_pose = 0, n_pt = 0;
  int64_t n_obs = 0, n_lid = 0;
  std::vector<double> pose_q, pose_t, intr, pt;
  std::vector<uint8_t> pose_fixed;
  HVec<int32_t> obs_pose, obs_pt;
  HVec<double> obs_uv, obs_info, obs_delta, obs_err;
  HVec<uint8_t> obs_level;
  bool has_stereo = false;           // some edge is an EdgeStereoSE3ProjectXYZ
  std::vector<double> obs_ur, pose_bf, obs_err3;
  std::vector<int32_t> lid_pose;
  std::vector<double> lid_pc, lid_pw, lid_n, lid_info, lid_err;
  std::vector<uint8_t> lid_level;
  // ---- structure of the current optimize() call ----
  DevProblem d;
  std::vector<Bucket> buckets;
  std::vector<int> bucket_part_off;
  UpdLaunch upd;  // every bucket's landmark update in one launch (nb = 0: per bucket)
  int n_lm_parts = 0;
  std::vector<int> slot_pt;          // device slot -> point id
  HVec<int64_t> dev_edge;            // device obs -> edge id
  std::vector<int64_t> dev_lid_edge; // device lidar -> lidar edge id
  std::vector<int> h_btot;           // setup: landmark-slot bucket totals
  int max_row_blocks = 0;
  int n_active_edges = 0;
  CRPlan cr;
  int n_cu = 0;
  std::vector<int> cam_pos;          // hidx -> band position or -(1 + border index)
  bool use_tiles = false;
  int tile_max_cp = 0, tile_max_k = 0;
  // the last optimize()'s per-edge errors are still on the device only
  // (fetched when an edge chi2 is asked for, or before the next prepare())
  bool err_pending = false;
  bool err_zero = false;  // obs_err is still to be sized and zeroed (a new problem: no error computed yet)
  // host plan scratch kept across calls (capacity reused: prepare() allocates
  // and first-touches none of its large arrays after the first call)
  TilePlan tp;
  TileBuild tb;
  std::vector<std::vector<int>> scat_base;  // per-thread counting-sort bases (slots)
  std::vector<int> h_kcount, h_span_lo, h_span_hi, h_pt_slot, h_key;
  std::vector<int> h_efirst, h_elast;  // first / last active edge of every landmark (contiguity test)
  std::vector<uint8_t> h_pose_act, h_pt_act;
  // ---- device memory ----
  std::vector<DevBuf> bufs;
  std::vector<DevBuf> pins;  // page-locked host staging of the large uploads (async DMA)
  double *h_scalars = nullptr;  // pinned
  CRSync crs;                   // completion words of the one-launch back substitution
  // the trial scalars' mailbox (mapped, coherent page-locked memory written by
  // k_reduce): the host polls its sequence number instead of a copy + stream
  // synchronize; timing runs and sharded runs copy
  double *mbox = nullptr, *mbox_dev = nullptr;
  unsigned long long mbox_seq = 0;
  // SQLM_HOST_TRACE=1: host-side time points of every trial (diagnostic)
  bool htrace = false;
  std::chrono::steady_clock::time_point ht_prev{};
  double ht_acc[10] = {};
  int ht_n = 0;
  // ---- comm ----
  Comm comm;
  // ---- essential graph (sqlm_eg.hip) ----
  // sharded runs: every rank's nonzero S block-row range [lo, hi), the BSR
  // row pointer (host), and on rank 0 the gather table into xstage
  std::vector<int> sh_lo, sh_hi, s_row_host;
  GatherTab gather;
  bool need_maxdiag = false;
  EGSolver *eg = nullptr;
  OrbEngine *orb = nullptr;
  // ---- timing ----
  hipEvent_t ev[2 * SQLM_NKERNEL_TIMERS] = {};
  // side stream: the camera pass runs concurrently with the landmark QR
  // (independent inputs and outputs); fork / join through two events
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // speculative linearization: every trial's k_landmark_update also linearizes
  // at the trial state (into the *_nx buffers) and the camera pass for that
  // state runs on the side stream; an accepted trial swaps them in, so the next
  // iteration starts without a linearization pass (g2o linearizes at exactly
  // that state: same device code, same bits). SQLM_NO_SPEC=1 turns it off.
  bool spec = false;
  bool no_pose_fuse = false;       // SQLM_NO_POSE_FUSE=1 (per prepare): the pose update as its own launch
  bool lin_valid = false;          // the current buffers hold the linearization at the current state
  bool spec_outstanding = false;   // a speculative camera pass may still run on the side stream
  bool cam_inline = false;         // small problem: the speculative camera pass on the context stream
  hipEvent_t ev_spec_fork = nullptr, ev_spec_join = nullptr;
  TileStreams tiles;  // RCS tile classes run on stream + these two
  hipEvent_t ev_cam[2][2] = {};    // timing of the speculative camera passes (ping-pong)
  bool cam_pending[2] = {false, false};
  int cam_par = 0;
  int lin_timers = 2;               // timers the last linearize() recorded
  bool timing = false;
  double kernel_ms_acc[SQLM_NKERNEL_TIMERS] = {};
  int kernel_ms_n = 0;
};

#define HIP_OK(x)                          \
  do {                                     \
    if ((x) != hipSuccess) return SQLM_ERR_HIP; \
  } while (0)

namespace {

template <class T>
int ensure(sqlm_ctx *c, int idx, size_t n, T **out) {
  if ((int)c->bufs.size() <= idx) c->bufs.resize(idx + 1);
  DevBuf &b = c->bufs[idx];
  size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
  bytes = (bytes + 255) & ~size_t(255);
  if (b.cap < bytes) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
    if (hipMalloc(&b.p, bytes) != hipSuccess) return SQLM_ERR_OOM;
    b.cap = bytes;
  }
  *out = static_cast<T *>(b.p);
  return SQLM_OK;
}

template <class T>
int upload(sqlm_ctx *c, int idx, const std::vector<T> &v, T **out) {
  int s = ensure(c, idx, v.size(), out);
  if (s) return s;
  if (!v.empty()) HIP_OK(hipMemcpyAsync(*out, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, c->stream));
  return SQLM_OK;
}

// A page-locked host array from the context's arena (grown, never shrunk):
// the large observation arrays are built in place and copied to the device
// asynchronously while the host goes on with the setup.
template <class T>
struct PinVec {
  T *p = nullptr;
  size_t n = 0;
  T &operator[](size_t i) const { return p[i]; }
  T *data() const { return p; }
  size_t size() const { return n; }
  T *begin() const { return p; }
  T *end() const { return p + n; }
};

inline void free_pinned(DevBuf &b) {
  if (b.p && b.map) {
    (void)hipHostUnregister(b.p);
    munmap(b.p, b.map);
  } else if (b.p) {
    (void)hipHostFree(b.p);
  }
  b.p = nullptr;
  b.cap = b.map = 0;
}

template <class T>
int pinned(sqlm_ctx *c, int idx, size_t n, PinVec<T> &out) {
  if ((int)c->pins.size() <= idx) c->pins.resize(idx + 1);
  DevBuf &b = c->pins[idx];
  const size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
  if (b.cap < bytes) {
    free_pinned(b);
    // large arrays: a huge-page mapping, touched, then page-locked for the DMA
    if (SQLM_HOST_HUGE && bytes >= kHugePage) {
      if (void *p = huge_map(bytes)) {
        std::memset(p, 0, huge_len(bytes));
        if (hipHostRegister(p, huge_len(bytes), hipHostRegisterDefault) == hipSuccess) {
          b.p = p;
          b.cap = bytes;
          b.map = huge_len(bytes);
        } else {
          munmap(p, huge_len(bytes));
        }
      }
    }
    if (!b.p) {
      if (hipHostMalloc(&b.p, bytes, hipHostMallocDefault) != hipSuccess) return SQLM_ERR_OOM;
      b.cap = bytes;
    }
  }
  out.p = static_cast<T *>(b.p);
  out.n = n;
  return SQLM_OK;
}

template <class T>
int upload(sqlm_ctx *c, int idx, const PinVec<T> &v, T **out) {
  int s = ensure(c, idx, v.size(), out);
  if (s) return s;
  if (v.size()) HIP_OK(hipMemcpyAsync(*out, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, c->stream));
  return SQLM_OK;
}

enum PinId { P_OBSLM, P_OBSCAM, P_OBSCAMH, P_OBSUV, P_OBSINFO, P_OBSDELTA, P_OBSUR, P_RQT, P_RX, P_RERR, P_RERR3, P_RLERR, P_OBSQ,
             P_X, P_OBSLOC, P_ARENA };

enum BufId {
  B_QT0, B_QT1, B_RT0, B_RT1, B_INTR, B_PHIDX, B_HIDXP, B_X0, B_X1, B_LMBEG, B_LMR, B_LMB, B_LMM, B_LMV,
  B_OBSLM, B_OBSCAM, B_OBSCAMH, B_OBSUV, B_OBSINFO, B_OBSDELTA, B_OBSS, B_OBSP, B_OBSJP, B_OBSERR, B_CAMPTR, B_CAMOBS, B_CAMSLOT, B_CAMUV, B_SROWIDX,
  B_HPP, B_BP, B_LIDPTR, B_LIDDATA, B_LIDPOSE, B_LIDERR, B_SROW, B_SCOL, B_S, B_G, B_DX, B_DENSE, B_PART,
  B_SCAL, B_MAXD, B_FLAGS, B_CRD, B_CRE, B_CRA, B_CRC, B_CRG, B_CRX, B_LMRP, B_TLM, B_TCAMP, B_TCAMS, B_TORDER,
  B_TPART, B_OBSLOC, B_PART2, B_GPART, B_REDP, B_REDI, B_GREDP, B_GREDI, B_TGPART, B_TLD, B_URANGE,
  B_OBSUR, B_OBSERR3, B_POSEBF, B_CAMUR, B_HDIAG, B_XSTAGE, B_DENSEL, B_DENSELI, B_DENSER, B_DENSEX,
  B_LMR_NX, B_LMB_NX, B_OBSS_NX, B_HPP_NX, B_BP_NX, B_CAMPOS, B_ARWS, B_ARWG, B_ARWZ, B_BDA, B_BDL, B_BDLI,
  B_BDR, B_BDX, B_LONGS, B_LONGG, B_UPDRNG, B_CRL, B_CAMKEY0, B_CAMKEY1, B_CAMVAL, B_SORTTMP, B_OBSQ, B_CAMQ,
  B_CRDONE, B_ARENA
};

// The small host arrays of a setup go to the device in one copy: their bytes
// are gathered into one block (256-byte aligned pieces) and their device
// pointers point into one arena buffer. A local-BA setup is otherwise ~35
// hipMemcpyAsync calls of a few KB at 3-10 us of host time each.
constexpr size_t kSmallUpload = 64 << 10;
template <class T>
struct is_pinvec : std::false_type {};
template <class T>
struct is_pinvec<PinVec<T>> : std::true_type {};
struct SmallUploads {
  std::vector<uint8_t> host;
  std::vector<std::pair<size_t, void **>> dst;
  template <class T>
  void add(const std::vector<T> &v, T **out) {
    const size_t off = host.size(), bytes = v.size() * sizeof(T);
    host.resize(off + ((std::max<size_t>(bytes, 1) + 255) & ~size_t(255)));
    if (bytes) std::memcpy(host.data() + off, v.data(), bytes);
    dst.push_back({off, reinterpret_cast<void **>(out)});
    *out = nullptr;  // set when the arena is copied: a kernel launched before that reads null, not stale memory
  }
};

// Persistent host worker pool for the setup passes (a prepare() runs ~20
// parallel passes; starting and joining 15 threads each time cost ~0.4 ms per
// pass). One caller at a time: a context that finds it busy (another context
// preparing on another thread) falls back to threads of its own.
class HostPool {
 public:
  // never destroyed: a process (or a forked child, whose copy has no worker
  // threads) exits without joining threads that may not exist
  static HostPool &get() {
    static HostPool *p = new HostPool();
    return *p;
  }
  // fn(t) for t = 1 .. nth-1 on the workers while the caller runs fn(0).
  // In a child forked after the pool started (multiprocessing's default start
  // method) the workers do not exist: false, the caller starts plain threads.
  bool try_run(int nth, const std::function<void(int)> &fn) {
    if (getpid() != pid_) return false;
    std::unique_lock<std::mutex> busy(use_, std::try_to_lock);
    if (!busy.owns_lock()) return false;
    {
      std::lock_guard<std::mutex> lk(m_);
      while ((int)th_.size() < nth - 1) {
        const int id = (int)th_.size() + 1;
        th_.emplace_back([this, id] { worker(id); });
      }
      job_ = &fn;
      active_ = nth;
      pending_ = nth - 1;
      ++gen_;
    }
    cv_.notify_all();
    fn(0);
    std::unique_lock<std::mutex> lk(m_);
    done_.wait(lk, [this] { return pending_ == 0; });
    job_ = nullptr;
    return true;
  }
 private:
  HostPool() : pid_(getpid()) {}
  void worker(int id) {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lk(m_);
    for (;;) {
      cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      if (id >= active_) continue;
      const std::function<void(int)> *f = job_;
      lk.unlock();
      (*f)(id);
      lk.lock();
      if (--pending_ == 0) done_.notify_one();
    }
  }
  std::mutex use_, m_;
  std::condition_variable cv_, done_;
  std::vector<std::thread> th_;
  const std::function<void(int)> *job_ = nullptr;
  uint64_t gen_ = 0;
  int active_ = 0, pending_ = 0;
  bool stop_ = false;
  const pid_t pid_;
};

// fn(t) for t = 0 .. nth-1 on nth host threads (t = 0 on the caller's)
template <class F>
void run_threads(int nth, F &&fn) {
  if (nth <= 1) {
    fn(0);
    return;
  }
  const std::function<void(int)> f = [&fn](int t) { fn(t); };
  if (HostPool::get().try_run(nth, f)) return;
  std::vector<std::thread> th;
  for (int t = 1; t < nth; ++t) th.emplace_back(fn, t);
  fn(0);
  for (auto &t : th) t.join();
}

// Host threads for a setup pass over `work` items: one per 128k items (thread
// start-up costs more than small passes save; a local-BA window uses one).
inline int host_threads(int64_t work) {
  const int64_t want = std::max<int64_t>(1, work / 131072);
  return (int)std::max<int64_t>(1, std::min<int64_t>({16, want, (int64_t)std::thread::hardware_concurrency()}));
}

// v <- src[0 .. n) on host threads (the caller's arrays are copied in: ABI)
template <class T, class A>
void par_assign(std::vector<T, A> &v, const T *src, size_t n) {
  v.resize(n);  // same size as the last call: no fill
  const int nth = host_threads((int64_t)n);
  run_threads(nth, [&](int t) {
    const size_t a = n * t / nth, b = n * (t + 1) / nth;
    if (b > a) {
      if (src) std::memcpy(v.data() + a, src + a, (b - a) * sizeof(T));
      else std::memset(static_cast<void *>(v.data() + a), 0, (b - a) * sizeof(T));
    }
  });
}

// v <- n copies of x on host threads
template <class T>
void fill_par(std::vector<T> &v, size_t n, T x) {
  v.resize(n);
  const int nth = host_threads((int64_t)n);
  run_threads(nth, [&](int t) { std::fill(v.begin() + n * t / nth, v.begin() + n * (t + 1) / nth, x); });
}

void build_tiles(int nP, int nL, const std::vector<int> &lm_begin, const int *obs_camh, int lm_cap, TilePlan &tp,
                 TileBuild &tb, int *obs_local) {
  const int64_t nE = lm_begin[nL];
  const bool ptime = std::getenv("SQLM_PREP_TIMING") != nullptr;
  auto pt0 = std::chrono::steady_clock::now();
  auto sub = [&](const char *what) {  // sub-phases of "tiles" (SQLM_PREP_TIMING=1)
    if (!ptime) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "  tiles %-14s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(now - pt0).count());
    pt0 = now;
  };
  tp.reset();
  tp.urange.assign(nL, int2{-1, -1});
  // pass 1 (greedy): tile boundaries -- a tile closes before the landmark that
  // would push its window past kTileMaxCams cameras or lm_cap. The slots are
  // cut into a number of chunks that depends on the problem only (one per
  // 128k observations, at most 16; a tile never crosses a chunk start), so the
  // tile plan -- and with it the fixed summation order of S -- is the same on
  // every host; the chunks are then dealt to however many threads there are.
  std::vector<int> &tstart = tb.tstart;
  tstart.clear();
  {
    const int nchunk = (int)std::max<int64_t>(1, std::min<int64_t>(16, nE / 131072));
    const int nth = std::min(nchunk, host_threads(nE));
    std::vector<std::vector<int>> cuts(nchunk);
    std::vector<uint8_t> dup(nchunk, 0);
    run_threads(nth, [&](int th) {
      std::vector<int> stamp(nP, -1), lmst(nP, -1);
      for (int ch = th; ch < nchunk; ch += nth) {
        const int s0 = (int)((int64_t)nL * ch / nchunk), s1 = (int)((int64_t)nL * (ch + 1) / nchunk);
        std::vector<int> &cv = cuts[ch];
        int t = 0, ncur = 0, cur_lm = 0;
        std::fill(stamp.begin(), stamp.end(), -1);
        for (int sl = s0; sl < s1; ++sl) {
          int nnew = 0;
          for (int o = lm_begin[sl]; o < lm_begin[sl + 1]; ++o) {
            const int h = obs_camh[o];
            if (h < 0) continue;
            if (lmst[h] == sl) { dup[ch] = 1; continue; }
            lmst[h] = sl;
            if (stamp[h] != t) ++nnew;
          }
          if (cur_lm == 0 || ncur + nnew > kTileMaxCams || cur_lm >= lm_cap) {
            cv.push_back(sl);
            ++t;
            ncur = 0;
            cur_lm = 0;
          }
          for (int o = lm_begin[sl]; o < lm_begin[sl + 1]; ++o) {
            const int h = obs_camh[o];
            if (h >= 0 && stamp[h] != t) { stamp[h] = t; ++ncur; }
          }
          ++cur_lm;
        }
      }
    });
    for (int ch = 0; ch < nchunk; ++ch) {
      tstart.insert(tstart.end(), cuts[ch].begin(), cuts[ch].end());
      if (dup[ch]) tp.dups = true;
    }
    if (tstart.empty() || tstart[0] != 0) tstart.insert(tstart.begin(), 0);
    if (nL > 0) tstart.push_back(nL);
    else tstart.assign(1, 0);
  }
  sub("pass 1");
  const int nt = (int)tstart.size() - 1;
  // pass 2 (tiles on host threads): window cameras, local camera of every
  // observation, landmark spans, and the S blocks each tile contributes to
    std::vector<TileBuild::TileOut> &out = tb.out;
  out.assign(nt, TileBuild::TileOut{});
  const int nth = host_threads(nE);
  run_threads(nth, [&](int th) {
    std::vector<int> lidx(nP, -1), lcams;
    std::vector<uint8_t> pst;
    std::vector<uint64_t> rowm;
    for (int t = th; t < nt; t += nth) {
      // the window's cameras: first sight marks (lidx = -2), then sorted (<= 24 of them)
      std::vector<int> &cur = out[t].cams;
      for (int o = lm_begin[tstart[t]]; o < lm_begin[tstart[t + 1]]; ++o) {
        const int h = obs_camh[o];
        if (h >= 0 && lidx[h] == -1) { lidx[h] = -2; cur.push_back(h); }
      }
      std::sort(cur.begin(), cur.end());
      const int cp = (int)cur.size();
      for (int u = 0; u < cp; ++u) lidx[cur[u]] = u;
      // co-observed camera pairs (u <= v): as one bit row per camera when the
      // window fits 64 (a landmark ORs its camera set into the rows of its
      // cameras: linear in its track, not quadratic), else as a byte matrix
      const bool bits = cp <= 64;
      if (bits) rowm.assign(cp, 0);
      else pst.assign((size_t)cp * cp, 0);
      for (int sl = tstart[t]; sl < tstart[t + 1]; ++sl) {
        lcams.clear();
        int lo = cp, hi = -1;
        uint64_t set = 0;
        for (int o = lm_begin[sl]; o < lm_begin[sl + 1]; ++o) {
          const int h = obs_camh[o];
          const int u = h >= 0 ? lidx[h] : -1;
          obs_local[o] = u;
          if (u >= 0) {
            lcams.push_back(u);
            lo = std::min(lo, u);
            hi = std::max(hi, u);
            if (bits) set |= uint64_t(1) << u;
          }
        }
        if (hi < 0) continue;
        tp.urange[sl] = int2{lo, hi};
        if (bits) {
          for (const int u : lcams) rowm[u] |= set;
          continue;
        }
        const size_t m = lcams.size();  // (a repeated camera only marks its pairs twice)
        for (size_t a = 0; a < m; ++a)
          for (size_t b = a; b < m; ++b) {
            const int u = std::min(lcams[a], lcams[b]), v = std::max(lcams[a], lcams[b]);
            pst[(size_t)u * cp + v] = 1;
          }
      }
      for (int u = 0; u < cp; ++u)
        for (int v = u; v < cp; ++v)
          if (bits ? (rowm[u] >> v & 1) : pst[(size_t)u * cp + v])
            out[t].red.push_back({cur[u], t, tile_blk(u, v, cp), cur[v]});
      for (int u = 0; u < cp; ++u) lidx[cur[u]] = -1;
    }
  });
  sub("pass 2");
}

// S pattern (upper, diagonal first) of the free cameras from the tiles'
// camera pairs: every pair of cameras that co-observe a landmark is marked in
// the tile that holds the landmark; plus every diagonal.
void pattern_from_tiles(int nP, const TileBuild &tb, std::vector<int> &s_row, std::vector<int> &s_col) {
  const int nt = (int)tb.out.size();
  const int nth = host_threads((int64_t)nt * 256);
  std::vector<std::vector<int>> cnt(nth, std::vector<int>(nP, 0));
  run_threads(nth, [&](int th) {
    for (int t = th; t < nt; t += nth)
      for (const auto &r : tb.out[t].red)
        if (r.j != r.key) ++cnt[th][r.key];
  });
  std::vector<int> ptr(nP + 1, 0);
  for (int i = 0; i < nP; ++i) {
    int b = ptr[i] + 1;  // the diagonal first
    for (int th = 0; th < nth; ++th) { const int k = cnt[th][i]; cnt[th][i] = b; b += k; }
    ptr[i + 1] = b;
  }
  std::vector<int> raw(ptr[nP]);
  for (int i = 0; i < nP; ++i) raw[ptr[i]] = i;
  run_threads(nth, [&](int th) {
    for (int t = th; t < nt; t += nth)
      for (const auto &r : tb.out[t].red)
        if (r.j != r.key) raw[cnt[th][r.key]++] = r.j;
  });
  std::vector<int> len(nP);
  // (sorting is heavier per entry than a copy: more threads than a pass would take)
  run_threads(host_threads(8 * (int64_t)ptr[nP]), [&](int th) {
    const int n = host_threads(8 * (int64_t)ptr[nP]);
    for (int i = (int)((int64_t)nP * th / n); i < (int)((int64_t)nP * (th + 1) / n); ++i) {
      int *b = raw.data() + ptr[i] + 1, *e = raw.data() + ptr[i + 1];
      std::sort(b, e);
      len[i] = 1 + (int)(std::unique(b, e) - b);
    }
  });
  s_row.assign(nP + 1, 0);
  for (int i = 0; i < nP; ++i) s_row[i + 1] = s_row[i] + len[i];
  s_col.resize(s_row[nP]);
  for (int i = 0; i < nP; ++i) std::copy(raw.begin() + ptr[i], raw.begin() + ptr[i] + len[i], s_col.begin() + s_row[i]);
}

// The reduction lists of the tiles (needs the final S pattern).
void build_tiles_finish(int nP, const std::vector<int> &s_row, const std::vector<int> &s_col, TilePlan &tp,
                        TileBuild &tb) {
  const bool ptime = std::getenv("SQLM_PREP_TIMING") != nullptr;
  auto pt0 = std::chrono::steady_clock::now();
  auto sub = [&](const char *what) {
    if (!ptime) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "  tiles %-14s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(now - pt0).count());
    pt0 = now;
  };
  using Red = TileBuild::Red;
  std::vector<TileBuild::TileOut> &out = tb.out;
  const std::vector<int> &tstart = tb.tstart;
  const int nt = (int)out.size();
  run_threads(host_threads((int64_t)nt * 256), [&](int th) {  // S block of every tile pair
    const int n = host_threads((int64_t)nt * 256);
    for (int t = th; t < nt; t += n)
      for (Red &r : out[t].red) {
        const int *b0 = s_col.data() + s_row[r.key], *b1 = s_col.data() + s_row[r.key + 1];
        r.key = (int)(std::lower_bound(b0, b1, r.j) - s_col.data());
      }
  });
  sub("keys");
  // pass 3 (tile order): offsets, camera lists, the reduction lists (the
  // lists concatenated on host threads at per-tile offsets)
  std::vector<Red> red, gred;
  {
    std::vector<size_t> roff(nt + 1, 0), goff(nt + 1, 0);
    for (int t = 0; t < nt; ++t) {
      roff[t + 1] = roff[t] + out[t].red.size();
      goff[t + 1] = goff[t] + out[t].cams.size();
    }
    red.resize(roff[nt]);
    gred.resize(goff[nt]);
    const int nr = host_threads((int64_t)roff[nt]);
    run_threads(nr, [&](int th) {
      for (int t = (int)((int64_t)nt * th / nr); t < (int)((int64_t)nt * (th + 1) / nr); ++t) {
        std::copy(out[t].red.begin(), out[t].red.end(), red.begin() + roff[t]);
        for (size_t u = 0; u < out[t].cams.size(); ++u) gred[goff[t] + u] = Red{out[t].cams[u], t, (int)u, 0};
      }
    });
  }
  for (int t = 0; t < nt; ++t) {
    const std::vector<int> &cur = out[t].cams;
    const int cp = (int)cur.size();
    const int ld = (6 * cp + 15) / 16 * 16;
    tp.ld.push_back(ld);
    tp.part_ptr.push_back(tp.part_ptr.back() + 36 * (int64_t)(cp * (cp + 1) / 2));
    tp.gpart_ptr.push_back(tp.gpart_ptr.back() + ld);
    tp.cams.insert(tp.cams.end(), cur.begin(), cur.end());
    tp.cam_ptr.push_back(tp.cam_ptr.back() + cp);
    tp.lm_ptr.push_back(tstart[t + 1]);
    tp.max_cp = std::max(tp.max_cp, cp);
  }
  {  // launch classes by accumulator width
    std::vector<int> cls(nt);
    bool any4 = false;
    for (int t = 0; t < nt; ++t) any4 |= (6 * (int)out[t].cams.size() + 15) / 16 == 4;
    for (int t = 0; t < nt; ++t) {
      // classes 3 (only when no tile needs 4: small windows, e.g. local BA), 4,
      // 6, 8, 9 — a tile goes to the narrowest one that holds it; the odd widths
      // hold a few dozen tiles each, too few for a launch of their own
      const int w = (6 * (int)out[t].cams.size() + 15) / 16;
      cls[t] = w <= 3 && !any4 ? 3 : w <= 4 ? 4 : w <= 6 ? 6 : w <= 8 ? 8 : kTileNtMax;
      tp.cls_cnt[cls[t]]++;
    }
    tp.cls_off[0] = 0;
    for (int k = 0; k <= kTileNtMax; ++k) tp.cls_off[k + 1] = tp.cls_off[k] + tp.cls_cnt[k];
    tp.order.assign(std::max(nt, 1), 0);
    std::vector<int> f(tp.cls_off, tp.cls_off + kTileNtMax + 1);
    for (int t = 0; t < nt; ++t) tp.order[f[cls[t]]++] = t;
  }
  if (std::getenv("SQLM_PREP_TIMING")) {  // window widths of the tiles (cameras), for the NT classes
    int hist[kTileHardCams + 2] = {0};
    for (int t = 0; t < nt; ++t) hist[std::min((int)out[t].cams.size(), kTileHardCams + 1)]++;
    std::fprintf(stderr, "sqlm tiles: %d, cameras per window:", nt);
    for (int c = 0; c <= kTileHardCams + 1; ++c)
      if (hist[c]) std::fprintf(stderr, " %d:%d", c, hist[c]);
    std::fprintf(stderr, "\n");
  }
  sub("pass 3");
  auto csr = [](const std::vector<Red> &v, int nkeys, std::vector<int> &ptr, std::vector<int2> &idx) {
    ptr.assign(nkeys + 1, 0);
    for (auto &r : v) ptr[r.key + 1]++;
    for (int k = 0; k < nkeys; ++k) ptr[k + 1] += ptr[k];
    idx.resize(v.size());
    std::vector<int> f(ptr.begin(), ptr.end() - 1);
    for (auto &r : v) idx[f[r.key]++] = int2{r.tile, r.code};
  };
  std::vector<int2> red_idx;
  csr(red, s_row[nP], tp.red_ptr, red_idx);
  tp.red_off.resize(red_idx.size());
  {
    const int64_t n = (int64_t)red_idx.size();
    const int nc = host_threads(n);
    run_threads(nc, [&](int t) {
      for (int64_t k = n * t / nc; k < n * (t + 1) / nc; ++k)
        tp.red_off[k] = tp.part_ptr[red_idx[k].x] + 36 * (int64_t)red_idx[k].y;
    });
  }
  csr(gred, nP, tp.gred_ptr, tp.gred_idx);
  tp.gred_off.resize(tp.gred_idx.size());
  for (size_t k = 0; k < tp.gred_idx.size(); ++k)
    tp.gred_off[k] = tp.gpart_ptr[tp.gred_idx[k].x] + 6 * (int64_t)tp.gred_idx[k].y;
  for (int s = 0; s < s_row[nP]; ++s)
    if (tp.red_ptr[s + 1] - tp.red_ptr[s] > kRedLong) tp.long_s.push_back(s);
  for (int i = 0; i < nP; ++i)
    if (tp.gred_ptr[i + 1] - tp.gred_ptr[i] > kRedLong) tp.long_g.push_back(i);
  sub("reduction csr");
}

// Reduced-camera-system solver plan from the upper block pattern of S (hidx
// order; SimplicialLDLT + AMD in the reference, linear_solver_eigen.h:60-75).
// Blocks within kBandMaxCams of the diagonal form the band, solved by cyclic
// reduction over superblocks of B = bandwidth + 1 cameras. Blocks farther off
// (loop closures) are covered by a greedy maximum-degree vertex cover; those
// cameras become the dense border, eliminated last (launch_arrow_solve). The
// cyclic reduction carries the band-border coupling only in the superblocks
// that can hold it: per level, the odd superblocks whose right-hand side is
// nonzero form Z = Linv G, the even ones next to them take the update.
// Returns false when S should go to the dense solver (border too large).
// Superblock width of a band-only S. Any B > bandwidth keeps S
// block-tridiagonal; a wider superblock means fewer cyclic-reduction levels and
// a longer factor chain per level. On small systems (a few superblocks) every
// level is latency -- a factor launch whose diagonal chain grows with n / 16,
// an update and a back-substitution launch -- so the estimate below (us per
// launch, measured: tools/cr_bench and the local-BA solve trace,
// profiles/r03/solve_trace_lba.txt) picks the cheapest B, ties to the
// narrowest. Larger systems keep B = bandwidth + 1 (their first levels are
// throughput-bound). SQLM_CR_B_MIN=1: always the narrowest (A/B only).
int cr_superblock_width(int bmin, int nband) {
  const bool keep = std::getenv("SQLM_CR_B_MIN") != nullptr;  // read per plan: tests switch it
  if (const char *fb = std::getenv("SQLM_CR_B")) {  // a fixed width (A/B of the estimate only)
    const int b = std::atoi(fb);
    if (b >= bmin && 6 * b <= kCRMaxN) return std::min(b, std::max(nband, 1));
  }
  auto cost = [&](int B) {
    const int nt = (6 * B + 15) / 16, p = (nband + B - 1) / B;
    int L = 0;
    while ((1 << L) < p) ++L;
    return (L + 1) * (2.0 + 2.6 * nt) + L * 5.5 + (L + 1) * 5.0;
  };
  if (keep || bmin <= 0 || (nband + bmin - 1) / bmin > 16) return bmin;
  int best = bmin;
  for (int B = bmin + 1; 6 * B <= kCRMaxN && B <= nband; ++B)
    if (cost(B) < cost(best) - 1e-9) best = B;
  return best;
}

bool plan_rcs(int nP, const std::vector<int> &s_row, const std::vector<int> &s_col, CRPlan &pl,
              std::vector<int> &cam_pos) {
  pl = CRPlan{};
  cam_pos.resize(nP);
  for (int i = 0; i < nP; ++i) cam_pos[i] = i;
  if (nP == 0) return false;
  std::vector<int> lptr(nP + 1, 0), ladj;
  std::vector<std::pair<int, int>> longe;
  for (int i = 0; i < nP; ++i)
    for (int k = s_row[i]; k < s_row[i + 1]; ++k)
      if (s_col[k] - i > kBandMaxCams) longe.emplace_back(i, s_col[k]);
  std::vector<uint8_t> border(nP, 0);
  int nbc = 0;
  if (!longe.empty()) {
    for (auto &e : longe) { ++lptr[e.first + 1]; ++lptr[e.second + 1]; }
    for (int i = 0; i < nP; ++i) lptr[i + 1] += lptr[i];
    ladj.resize(lptr[nP]);
    std::vector<int> fill(lptr.begin(), lptr.end() - 1), deg(nP, 0);
    for (auto &e : longe) { ladj[fill[e.first]++] = e.second; ladj[fill[e.second]++] = e.first; }
    std::priority_queue<std::pair<int, int>> pq;  // (remaining long blocks, camera): ties -> higher index
    for (int i = 0; i < nP; ++i) {
      deg[i] = lptr[i + 1] - lptr[i];
      if (deg[i]) pq.emplace(deg[i], i);
    }
    while (!pq.empty()) {
      const auto [dg, v] = pq.top();
      pq.pop();
      if (border[v] || dg != deg[v] || dg == 0) continue;
      border[v] = 1;
      ++nbc;
      for (int k = lptr[v]; k < lptr[v + 1]; ++k) {
        const int u = ladj[k];
        if (!border[u] && deg[u] > 0) pq.emplace(--deg[u], u);
      }
      deg[v] = 0;
    }
  }
  const int nband = nP - nbc;
  if (nbc > 0) {
    if (nband == 0 || 3 * nbc > nP) return false;
    int pos = 0, b = 0;
    for (int i = 0; i < nP; ++i) cam_pos[i] = border[i] ? -1 - b++ : pos++;
  }
  int bw = 0;
  for (int i = 0; i < nP; ++i)
    for (int k = s_row[i]; k < s_row[i + 1]; ++k)
      if (cam_pos[i] >= 0 && cam_pos[s_col[k]] >= 0) bw = std::max(bw, cam_pos[s_col[k]] - cam_pos[i]);
  int B = std::min(bw + 1, std::max(nband, 1));
  if (nbc == 0) B = cr_superblock_width(B, nband);
  const int n = (6 * B + 15) / 16 * 16;
  if (n > kCRMaxN) return false;
  pl.enabled = true;
  pl.B = B;
  pl.p = (nband + B - 1) / B;
  pl.n = n;
  pl.nband = nband;
  if (nbc == 0) return true;
  pl.nbc = nbc;
  pl.R = (6 * nbc + 15) / 16 * 16;
  pl.Rp = (pl.R + kCRMaxN - 1) / kCRMaxN * kCRMaxN;
  // superblocks holding band-border blocks, then the per-level lists
  std::vector<uint8_t> act(pl.p, 0);
  for (int i = 0; i < nP; ++i)
    for (int k = s_row[i]; k < s_row[i + 1]; ++k) {
      const int a = cam_pos[i], c2 = cam_pos[s_col[k]];
      if ((a < 0) != (c2 < 0)) act[(a >= 0 ? a : c2) / B] = 1;
    }
  std::vector<int> &S = pl.sched, elim;
  pl.init_off = 0;
  for (int I = 0; I < pl.p; ++I)
    if (act[I]) S.push_back(I);
  pl.init_cnt = (int)S.size();
  for (int h = 1; h < pl.p; h *= 2) {
    const int fo = (int)S.size();
    for (int I = h; I < pl.p; I += 2 * h)
      if (act[I]) { S.push_back(I); elim.push_back(I); }
    const int uo = (int)S.size();
    for (int J = 0; J < pl.p; J += 2 * h) {
      const bool r = J + h < pl.p && act[J + h], l = J >= h && act[J - h];
      if (!r && !l) continue;
      S.push_back(J | (act[J] ? kUpdHad : 0) | (r ? kUpdRight : 0) | (l ? kUpdLeft : 0));
      act[J] = 1;
    }
    pl.lvl.insert(pl.lvl.end(), {fo, uo - fo, uo, (int)S.size() - uo});
  }
  pl.top_active = act[0] != 0;
  if (pl.top_active) elim.push_back(0);
  pl.elim_off = (int)S.size();
  pl.elim_cnt = (int)elim.size();
  S.insert(S.end(), elim.begin(), elim.end());
  return true;
}

// Lanes per landmark segment in the per-landmark kernels: up to kObsPerLane
// observations per lane, at least 2 lanes.
inline int seg_width(int k) {
  int w = 2;
  while (kObsPerLane * w < k && w < 64) w <<= 1;
  return w;
}

inline bool stopped(const volatile uint8_t *s) { return s && *s; }

// initializeOptimization(level) + BlockSolver::buildStructure: active set,
// index mapping (free poses by id, then points), landmark-sorted buckets,
// camera CSR and the upper block pattern of the reduced camera system.
int fetch_errors(sqlm_ctx *c);

// setup passes (A/B builds: =0 keeps the previous form)
#ifndef SQLM_ACTIVE_FAST
#define SQLM_ACTIVE_FAST 1
#endif
#ifndef SQLM_SCATTER_BY_SLOT
#define SQLM_SCATTER_BY_SLOT 1
#endif
#ifndef SQLM_SCATTER_PF
#define SQLM_SCATTER_PF 8
#endif

int prepare(sqlm_ctx *c, int level) {
  DevProblem &d = c->d;
  // edges outside this call's level keep their last error (g2o semantics):
  // bring the previous call's errors home before the device copies change
  if (int s = fetch_errors(c)) return s;
  c->prepared = false;
  // the page-locked staging arrays are rewritten (or regrown) below: no DMA of
  // an earlier call, finished or abandoned on an error path, may still read them
  HIP_OK(hipStreamSynchronize(c->stream));
  // SQLM_PREP_TIMING=1: host phase times of this setup on stderr
  const bool ptime = std::getenv("SQLM_PREP_TIMING") != nullptr;
  auto pt0 = std::chrono::steady_clock::now();
  auto phase = [&](const char *what) {
    if (!ptime) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "prepare %-12s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(now - pt0).count());
    pt0 = now;
  };
  std::vector<uint8_t> &pose_act = c->h_pose_act, &pt_act = c->h_pt_act;
  std::vector<int> &kcount = c->h_kcount, &span_lo = c->h_span_lo, &span_hi = c->h_span_hi;
  std::vector<int> &efirst = c->h_efirst, &elast = c->h_elast;
  pose_act.assign(c->n_pose, 0);
  fill_par(pt_act, (size_t)c->n_pt, (uint8_t)0);
  fill_par(kcount, (size_t)c->n_pt, 0);
  fill_par(span_lo, (size_t)c->n_pt, std::numeric_limits<int>::max());
  fill_par(span_hi, (size_t)c->n_pt, -1);
  fill_par(efirst, (size_t)c->n_pt, std::numeric_limits<int>::max());
  fill_par(elast, (size_t)c->n_pt, -1);
  phase("  fills");
  int64_t n_ae = 0;
  // active set, track lengths and camera spans in one pass on host threads.
  // Fast pass: the chunks start at landmark changes, and a landmark's edges
  // are one run (g2o adds a point's edges together, g2oOptimizer.cc:213-281),
  // so a run's results are stored plainly; one atomic exchange per run on
  // pt_act finds a landmark met twice, and then the pass is redone with
  // relaxed atomics for every field.
  for (int pass = SQLM_ACTIVE_FAST ? 0 : 1; pass < 2; ++pass) {
    if (pass == 1 && SQLM_ACTIVE_FAST) {
      fill_par(pt_act, (size_t)c->n_pt, (uint8_t)0);
      fill_par(kcount, (size_t)c->n_pt, 0);
      fill_par(span_lo, (size_t)c->n_pt, std::numeric_limits<int>::max());
      fill_par(span_hi, (size_t)c->n_pt, -1);
      fill_par(efirst, (size_t)c->n_pt, std::numeric_limits<int>::max());
      fill_par(elast, (size_t)c->n_pt, -1);
    }
    const bool fast = pass == 0;
    const int nth = host_threads(c->n_obs);
    std::vector<int64_t> cnt(nth, 0), cut(nth + 1, c->n_obs);
    std::vector<uint8_t> dup(nth, 0);
    for (int t = 0; t < nth; ++t) {  // chunk starts moved forward to a change of landmark
      int64_t e = c->n_obs * t / nth;
      if (fast && t > 0)
        while (e < c->n_obs && e > 0 && c->obs_pt[e] == c->obs_pt[e - 1]) ++e;
      cut[t] = std::max(e, t > 0 ? cut[t - 1] : (int64_t)0);
    }
    run_threads(nth, [&](int t) {
      const int64_t e0 = cut[t], e1 = cut[t + 1];
      int64_t n = 0;
      bool seen_twice = false;
      // runs of one landmark (the reference adds a point's edges together,
      // g2oOptimizer.cc:213-281) are folded locally: one set of atomics per run
      int rl = -1, rk = 0, rlo = 0, rhi = 0, rf = 0, rla = 0;
      auto flush = [&] {
        if (rl < 0) return;
        if (fast && nth > 1) {  // the landmark's only run (checked): plain stores
          seen_twice |= __atomic_exchange_n(&pt_act[rl], (uint8_t)1, __ATOMIC_RELAXED) != 0;
          kcount[rl] = rk;
          span_lo[rl] = rlo;
          span_hi[rl] = rhi;
          efirst[rl] = rf;
          elast[rl] = rla;
          return;
        }
        if (nth == 1) {  // one thread (a local-BA window): plain updates (the min / max atomics are CAS loops)
          pt_act[rl] = 1;
          kcount[rl] += rk;
          span_lo[rl] = std::min(span_lo[rl], rlo);
          span_hi[rl] = std::max(span_hi[rl], rhi);
          efirst[rl] = std::min(efirst[rl], rf);
          elast[rl] = std::max(elast[rl], rla);
          return;
        }
        __atomic_store_n(&pt_act[rl], (uint8_t)1, __ATOMIC_RELAXED);
        __atomic_fetch_add(&kcount[rl], rk, __ATOMIC_RELAXED);
        __atomic_fetch_min(&span_lo[rl], rlo, __ATOMIC_RELAXED);
        __atomic_fetch_max(&span_hi[rl], rhi, __ATOMIC_RELAXED);
        __atomic_fetch_min(&efirst[rl], rf, __ATOMIC_RELAXED);
        __atomic_fetch_max(&elast[rl], rla, __ATOMIC_RELAXED);
      };
      for (int64_t e = e0; e < e1; ++e) {
        if (c->obs_level[e] != level) continue;
        const int l = c->obs_pt[e], pp = c->obs_pose[e];
        if (!__atomic_load_n(&pose_act[pp], __ATOMIC_RELAXED)) __atomic_store_n(&pose_act[pp], (uint8_t)1, __ATOMIC_RELAXED);
        if (l != rl) {
          flush();
          rl = l;
          rk = 0;
          rlo = rhi = pp;
          rf = (int)e;
        }
        ++rk;
        rla = (int)e;
        rlo = std::min(rlo, pp);
        rhi = std::max(rhi, pp);
        ++n;
      }
      flush();
      cnt[t] = n;
      dup[t] = seen_twice;
    });
    if (std::find(dup.begin(), dup.end(), 1) != dup.end()) continue;  // a landmark in two runs: the atomic pass
    for (int64_t v : cnt) n_ae += v;
    break;
  }
  phase("  active pass");
  std::vector<int64_t> lid_act;
  const bool sharded = c->comm.enabled();
  for (int64_t e = 0; e < c->n_lid; ++e) {
    if (sharded && c->comm.rank != 0) break;  // unary pose edges live on rank 0
    if (c->lid_level[e] != level || c->pose_fixed[c->lid_pose[e]]) continue;
    lid_act.push_back(e);
    pose_act[c->lid_pose[e]] = 1;
  }
  // sharded: every rank must index the same free cameras (union of shards)
  if (sharded &&
      comm_allreduce_host(c->comm, pose_act.data(), c->n_pose, SQLM_DT_U8, SQLM_OP_MAX, c->stream))
    return SQLM_ERR_COMM;
  c->n_active_edges = (int)(n_ae + (int64_t)lid_act.size());
  std::vector<int> phidx(c->n_pose, -1), hidxp;
  for (int p = 0; p < c->n_pose; ++p)
    if (pose_act[p] && !c->pose_fixed[p]) { phidx[p] = (int)hidxp.size(); hidxp.push_back(p); }
  const int nP = (int)hidxp.size();
  if (nP > kMaxFreePoses) return SQLM_ERR_UNSUPPORTED;
  phase("  lidar+poses");
  // landmark slots: bucket by segment width; inside a bucket by camera span
  // (first, last observing pose, then id), so a batch of consecutive slots in
  // the RCS tiles shares nearly one span (dense MFMA panels)
  std::vector<int> pts;
  // (segment width, first pose) buckets by a counting sort, then last pose
  // inside a bucket; ties keep id order (the order a stable sort would give)
  {
    auto wl = [](int k) { int w = seg_width(k), b = 0; while ((2 << b) < w) ++b; return b; };  // log2(W) - 1
    const int64_t nb = 7 * (int64_t)c->n_pose + 1;
    std::vector<int> bcnt(nb + 1, 0);
    std::vector<int> &key = c->h_key;
    key.resize(c->n_pt);
    // the counting sort on host threads: chunk t (ids in order) histograms its
    // keys, bucket-major / chunk-minor bases keep id order inside a bucket
    const int nk = host_threads(c->n_pt);
    std::vector<std::vector<int>> hist(nk);
    run_threads(nk, [&](int t) {
      std::vector<int> &h = hist[t];
      h.assign(nb, 0);
      for (int l = (int)((int64_t)c->n_pt * t / nk); l < (int)((int64_t)c->n_pt * (t + 1) / nk); ++l) {
        key[l] = pt_act[l] ? (int)(wl(kcount[l]) * (int64_t)c->n_pose + span_lo[l]) : -1;
        if (key[l] >= 0) ++h[key[l]];
      }
    });
    // bucket totals over the chunks, the bucket bases, then every chunk's base
    // inside each bucket (bucket ranges on host threads; one serial pass over
    // nb instead of nb x chunks)
    {
      std::vector<int> &btot = c->h_btot;
      btot.resize(nb);
      run_threads(nk, [&](int t) {
        for (int64_t b = nb * t / nk; b < nb * (t + 1) / nk; ++b) {
          int k = 0;
          for (int u = 0; u < nk; ++u) k += hist[u][b];
          btot[b] = k;
        }
      });
      int64_t run = 0;
      for (int64_t b = 0; b < nb; ++b) {
        bcnt[b] = (int)run;
        run += btot[b];
      }
      bcnt[nb] = (int)run;
      run_threads(nk, [&](int t) {
        for (int64_t b = nb * t / nk; b < nb * (t + 1) / nk; ++b) {
          int r = bcnt[b];
          for (int u = 0; u < nk; ++u) { const int k = hist[u][b]; hist[u][b] = r; r += k; }
        }
      });
    }
    pts.resize(bcnt[nb]);
    run_threads(nk, [&](int t) {
      std::vector<int> &f = hist[t];
      for (int l = (int)((int64_t)c->n_pt * t / nk); l < (int)((int64_t)c->n_pt * (t + 1) / nk); ++l)
        if (key[l] >= 0) pts[f[key[l]]++] = l;
    });
    // buckets hold a few dozen points: a stable insertion sort, buckets on host threads
    const int nth = host_threads(c->n_pt * 8);
    run_threads(nth, [&](int t) {
      for (int64_t b = nb * t / nth; b < nb * (t + 1) / nth; ++b) {
        int *v = pts.data() + bcnt[b];
        const int m = bcnt[b + 1] - bcnt[b];
        if (m > 64) {
          std::stable_sort(v, v + m, [&](int a, int bb) { return span_hi[a] < span_hi[bb]; });
          continue;
        }
        for (int i = 1; i < m; ++i) {
          const int x = v[i], key = span_hi[x];
          int j = i - 1;
          while (j >= 0 && span_hi[v[j]] > key) { v[j + 1] = v[j]; --j; }
          v[j + 1] = x;
        }
      }
    });
  }
  const int nL = (int)pts.size();
  phase("active+sort");
  if (nP + nL == 0) return SQLM_ERR_STATE;  // "0 vertices to optimize"
  std::vector<int> &pt_slot = c->h_pt_slot;
  fill_par(pt_slot, (size_t)c->n_pt, -1);
  const int nks = host_threads(nL);
  run_threads(nks, [&](int t) {
    for (int s = (int)((int64_t)nL * t / nks); s < (int)((int64_t)nL * (t + 1) / nks); ++s) pt_slot[pts[s]] = s;
  });
  c->slot_pt = pts;
  phase("  pt_slot");
  c->buckets.clear();
  c->upd = UpdLaunch{};
  c->bucket_part_off.clear();
  c->n_lm_parts = 0;
  // the slots ascend in segment width (the sort's major key): each bucket ends
  // at the first slot of a wider segment
  for (int s = 0; s < nL;) {
    const int W = seg_width(kcount[pts[s]]);
    const int e = (int)(std::partition_point(pts.begin() + s, pts.end(), [&](int l) { return seg_width(kcount[l]) <= W; }) -
                        pts.begin());
    // The per-landmark kernels run a bucket with half the lanes its slot-order
    // width names (up to 2 kObsPerLane observations per lane from W = 4 up):
    // longer per-lane Givens chains, fewer idle lanes and butterfly rounds.
    // The slot order -- which the RCS tiles inherit -- stays bucketed at
    // kObsPerLane (config 4: landmark update 0.177 -> 0.160 ms, 775 -> 787
    // it/s, profiles/r05/ab_upd_half_lanes_cr_upd2w.log; the order itself at 4
    // per lane made the tiles 0.05 ms slower, ab_obs_per_lane_rejected.log).
    // (a quarter of the lanes from W = 8 up: 0.160 -> 0.182 ms, ab_uq.log)
    // (one lane per landmark for the shortest tracks: config 4 the same, local
    // BA 7.37k -> 7.22k it/s, ab_upd_one_lane_rejected.log)
    Bucket b{W >= 4 ? W / 2 : W, s, e};
    c->buckets.push_back(b);
    c->bucket_part_off.push_back(c->n_lm_parts);
    c->n_lm_parts += linearize_blocks(b);
    s = e;
  }
  if (c->n_lm_parts > 16384) return SQLM_ERR_UNSUPPORTED;
  phase("  buckets");
  // observations in slot order (edge-id order inside a landmark): offsets by a
  // two-pass prefix over slot chunks
  std::vector<int> lm_begin(nL + 1, 0);
  {
    std::vector<int64_t> part(nks + 1, 0);
    run_threads(nks, [&](int t) {
      int64_t acc = 0;
      for (int s = (int)((int64_t)nL * t / nks); s < (int)((int64_t)nL * (t + 1) / nks); ++s) acc += kcount[pts[s]];
      part[t + 1] = acc;
    });
    for (int t = 0; t < nks; ++t) part[t + 1] += part[t];
    if (part[nks] > (int64_t)std::numeric_limits<int>::max()) return SQLM_ERR_UNSUPPORTED;
    run_threads(nks, [&](int t) {
      int acc = (int)part[t];
      for (int s = (int)((int64_t)nL * t / nks); s < (int)((int64_t)nL * (t + 1) / nks); ++s) {
        acc += kcount[pts[s]];
        lm_begin[s + 1] = acc;
      }
    });
  }
  const int64_t nE = lm_begin[nL];
  if (nE > (int64_t)std::numeric_limits<int>::max()) return SQLM_ERR_UNSUPPORTED;
  phase("  lm_begin");
  c->dev_edge.resize(nE);  // every entry is written by the scatter below
  PinVec<int> obs_lm, obs_cam, obs_camh;
  PinVec<double> obs_uv, obs_info, obs_delta, obs_ur;
  PinVec<float> obs_q;  // u v info delta as float32, exact when obs_f32 (below)
  {
    int e = 0;
    if ((e = pinned(c, P_OBSLM, nE, obs_lm)) || (e = pinned(c, P_OBSCAM, nE, obs_cam)) ||
        (e = pinned(c, P_OBSCAMH, nE, obs_camh)) || (e = pinned(c, P_OBSQ, 4 * nE, obs_q)) ||
        (e = pinned(c, P_OBSUR, c->has_stereo ? nE : 0, obs_ur)))
      return e;
  }
  phase("  pinned");
  // Stable scatter of the observations into slot order on a few host threads
  // (edge-id order inside a landmark). When every landmark's active edges are
  // one contiguous run of edge ids -- g2o's graphs add a point's edges together
  // (g2oOptimizer.cc:213-281, 868-912) -- an edge's position is its slot's
  // base plus its offset in the run: one streaming pass. Otherwise chunk t of the edge range
  // counts its edges per slot, the per-(chunk, slot) bases follow by a prefix
  // over chunks, then every chunk scatters its edges.
  const int nth = host_threads(c->n_obs);
  auto par = [&](auto &&fn) { run_threads(nth, fn); };
  std::vector<uint8_t> inexact(nth, 0);
  auto put = [&](int64_t e, int o, int sl, bool &bad) {
    c->dev_edge[o] = e;
    obs_lm[o] = sl;
    obs_cam[o] = c->obs_pose[e];
    obs_camh[o] = phidx[c->obs_pose[e]];
    const double u = c->obs_uv[2 * e], v = c->obs_uv[2 * e + 1], w = c->obs_info[e], dl = c->obs_delta[e];
    const float fu = (float)u, fv = (float)v, fw = (float)w, fd = (float)dl;
    obs_q[4 * (size_t)o] = fu;
    obs_q[4 * (size_t)o + 1] = fv;
    obs_q[4 * (size_t)o + 2] = fw;
    obs_q[4 * (size_t)o + 3] = fd;
    bad |= (double)fu != u || (double)fv != v || (double)fw != w || (double)fd != dl;
    if (c->has_stereo) obs_ur[o] = c->obs_ur[e];
  };
  bool contig = c->n_obs <= (int64_t)std::numeric_limits<int>::max();
  if (contig) {
    std::vector<uint8_t> split(nth, 0);
    par([&](int t) {
      for (int sl = (int)((int64_t)nL * t / nth); sl < (int)((int64_t)nL * (t + 1) / nth); ++sl) {
        const int l = pts[sl];
        if (elast[l] - efirst[l] + 1 != kcount[l]) { split[t] = 1; break; }
      }
    });
    contig = std::find(split.begin(), split.end(), 1) == split.end();
  }
  phase("  contig check");
  if (contig && SQLM_SCATTER_BY_SLOT) {
    // slot order: the outputs are written front to back (whole cache lines)
    // and each landmark's inputs are one run of edge ids
    par([&](int t) {
      bool bad = false;
      const int s1 = (int)((int64_t)nL * (t + 1) / nth);
      for (int sl = (int)((int64_t)nL * t / nth); sl < s1; ++sl) {
        // the inputs of the landmarks kPf slots ahead (their edge runs sit at
        // random places of the edge arrays), and the run starts 2 kPf ahead
        if (SQLM_SCATTER_PF > 0 && sl + 2 * SQLM_SCATTER_PF < s1) __builtin_prefetch(&efirst[pts[sl + 2 * SQLM_SCATTER_PF]]);
        if (SQLM_SCATTER_PF > 0 && sl + SQLM_SCATTER_PF < s1) {
          const int64_t ep = efirst[pts[sl + SQLM_SCATTER_PF]];
          __builtin_prefetch(&c->obs_uv[2 * ep]);
          __builtin_prefetch(&c->obs_info[ep]);
          __builtin_prefetch(&c->obs_delta[ep]);
          __builtin_prefetch(&c->obs_pose[ep]);
        }
        const int b = lm_begin[sl], k = lm_begin[sl + 1] - b;
        const int64_t e0 = efirst[pts[sl]];
        for (int i = 0; i < k; ++i) put(e0 + i, b + i, sl, bad);
      }
      inexact[t] = bad;
    });
  } else if (contig) {  // edge order (streaming reads): edge e of landmark l goes to its slot's base + (e - first edge)
    par([&](int t) {
      bool bad = false;
      for (int64_t e = c->n_obs * t / nth; e < c->n_obs * (t + 1) / nth; ++e) {
        if (c->obs_level[e] != level) continue;
        const int l = c->obs_pt[e], sl = pt_slot[l];
        put(e, lm_begin[sl] + (int)(e - efirst[l]), sl, bad);
      }
      inexact[t] = bad;
    });
  } else {
    auto ebeg = [&](int t) { return c->n_obs * t / nth; };
    std::vector<std::vector<int>> &base = c->scat_base;
    if ((int)base.size() < nth) base.resize(nth);
    par([&](int t) {
      std::vector<int> &cnt = base[t];
      cnt.assign(nL, 0);
      for (int64_t e = ebeg(t); e < ebeg(t + 1); ++e)
        if (c->obs_level[e] == level) ++cnt[pt_slot[c->obs_pt[e]]];
    });
    par([&](int t) {  // per-slot prefix over the chunks, slots split across threads
      const int s0 = (int)((int64_t)nL * t / nth), s1 = (int)((int64_t)nL * (t + 1) / nth);
      for (int sl = s0; sl < s1; ++sl) {
        int b = lm_begin[sl];
        for (int u = 0; u < nth; ++u) { const int k = base[u][sl]; base[u][sl] = b; b += k; }
      }
    });
    par([&](int t) {
      std::vector<int> &fill = base[t];
      bool bad = false;
      for (int64_t e = ebeg(t); e < ebeg(t + 1); ++e) {
        if (c->obs_level[e] != level) continue;
        const int sl = pt_slot[c->obs_pt[e]];
        put(e, fill[sl]++, sl, bad);
      }
      inexact[t] = bad;
    });
  }
  phase("  scatter");
  // inputs that are not all float32 values: the double arrays, from the same slot order
  const bool obs_f32 = std::find(inexact.begin(), inexact.end(), 1) == inexact.end();
  if (!obs_f32) {
    int e = 0;
    if ((e = pinned(c, P_OBSUV, 2 * nE, obs_uv)) || (e = pinned(c, P_OBSINFO, nE, obs_info)) ||
        (e = pinned(c, P_OBSDELTA, nE, obs_delta)))
      return e;
    par([&](int t) {
      for (int64_t o = nE * t / nth; o < nE * (t + 1) / nth; ++o) {
        const int64_t ed = c->dev_edge[o];
        obs_uv[2 * o] = c->obs_uv[2 * ed];
        obs_uv[2 * o + 1] = c->obs_uv[2 * ed + 1];
        obs_info[o] = c->obs_info[ed];
        obs_delta[o] = c->obs_delta[ed];
      }
    });
  }
  // camera CSR (device obs in slot order): on the device (launch_cam_csr,
  // after the observation upload); on the host, the same chunked counting
  // sort, only for a sharded run, whose S pattern union walks it
  std::vector<int> cam_ptr(nP + 1, 0), cam_obs;
  int64_t n_cam_obs = 0;
  if (sharded) {
    auto obeg = [&](int t) { return nE * t / nth; };
    std::vector<std::vector<int>> base(nth);
    par([&](int t) {
      base[t].assign(nP, 0);
      for (int64_t o = obeg(t); o < obeg(t + 1); ++o)
        if (obs_camh[o] >= 0) ++base[t][obs_camh[o]];
    });
    for (int i = 0; i < nP; ++i)
      for (int u = 0; u < nth; ++u) cam_ptr[i + 1] += base[u][i];
    for (int i = 0; i < nP; ++i) cam_ptr[i + 1] += cam_ptr[i];
    for (int i = 0; i < nP; ++i) {
      int b = cam_ptr[i];
      for (int u = 0; u < nth; ++u) { const int k = base[u][i]; base[u][i] = b; b += k; }
    }
    cam_obs.resize(cam_ptr[nP]);
    par([&](int t) {
      std::vector<int> &fill = base[t];
      for (int64_t o = obeg(t); o < obeg(t + 1); ++o)
        if (obs_camh[o] >= 0) cam_obs[fill[obs_camh[o]]++] = (int)o;
    });
    n_cam_obs = (int64_t)cam_obs.size();
  } else {
    std::vector<int64_t> cnt(nth, 0);
    par([&](int t) {
      int64_t k = 0;
      for (int64_t o = nE * t / nth; o < nE * (t + 1) / nth; ++o) k += obs_camh[o] >= 0;
      cnt[t] = k;
    });
    for (int64_t k : cnt) n_cam_obs += k;
  }
  phase("  camh count");
  {  // the observation arrays go to the device now, overlapped with the rest of the setup
    int e = 0;
    if ((e = upload(c, B_OBSLM, obs_lm, &d.obs_lm)) || (e = upload(c, B_OBSCAM, obs_cam, &d.obs_cam)) ||
        (e = upload(c, B_OBSCAMH, obs_camh, &d.obs_camh)))
      return e;
    d.obs_f32 = obs_f32 ? 1 : 0;
    if (obs_f32) {
      if ((e = upload(c, B_OBSQ, obs_q, &d.obs_q))) return e;
      d.obs_uv = d.obs_info = d.obs_delta = nullptr;
    } else {
      if ((e = upload(c, B_OBSUV, obs_uv, &d.obs_uv)) || (e = upload(c, B_OBSINFO, obs_info, &d.obs_info)) ||
          (e = upload(c, B_OBSDELTA, obs_delta, &d.obs_delta)))
        return e;
      d.obs_q = nullptr;
    }
    if (c->has_stereo && (e = upload(c, B_OBSUR, obs_ur, &d.obs_ur))) return e;
    (void)hipStreamQuery(c->stream);  // submit now: the runtime would otherwise batch them until the next sync
  }
  phase("obs+camcsr");
  if (ptime && std::getenv("SQLM_PREP_SYNC")) {  // diagnostic: the early uploads alone
    (void)hipStreamSynchronize(c->stream);
    phase("obs upload");
  }
  // pose id window of every per-landmark block tile (k_landmark_update)
  std::vector<int2> upd_rng;
  {  // block slot ranges in bucket order, then their pose windows on host threads
    std::vector<int2> blk_slots;
    for (Bucket &b : c->buckets) {
      b.rng_off = (int)blk_slots.size();
      const int spb = kBlock / b.W;
      for (int s0 = b.slot_begin; s0 < b.slot_end; s0 += spb) blk_slots.push_back(int2{s0, std::min(s0 + spb, b.slot_end)});
    }
    const size_t nb = blk_slots.size();
    upd_rng.resize(nb);
    par([&](int t) {
      for (size_t k = nb * t / nth; k < nb * (t + 1) / nth; ++k) {
        int lo = std::numeric_limits<int>::max(), hi = -1;
        for (int o = lm_begin[blk_slots[k].x]; o < lm_begin[blk_slots[k].y]; ++o) {
          lo = std::min(lo, obs_cam[o]);
          hi = std::max(hi, obs_cam[o]);
        }
        upd_rng[k] = hi < 0 ? int2{1, 0} : int2{lo, hi};
      }
    });
    for (Bucket &b : c->buckets) {
      const size_t k1 = b.rng_off + (b.slot_end - b.slot_begin + kBlock / b.W - 1) / (kBlock / b.W);
      b.wide = false;
      for (size_t k = b.rng_off; k < k1 && k < nb; ++k) b.wide |= upd_rng[k].y - upd_rng[k].x + 1 > kUpdWin;
    }
    if (upd_launch_plan(c->buckets, c->bucket_part_off, c->upd)) c->upd = UpdLaunch{};  // per-bucket launches
  }
  // RCS tiles (passes 1-2: windows, local cameras, camera pairs), then the
  // reduced-camera-system pattern (upper, diagonal first) from the tiles'
  // camera pairs, then the tiles' reduction lists over that pattern
  TilePlan &tp = c->tp;
  // landmarks per tile: up to kTileMaxLm, fewer on small problems so that the
  // tiles still cover every CU twice (a local-BA window of 5k landmarks would
  // otherwise run ~40 long tiles on 256 CUs)
  // (nL / 160, / 80, / 40 measured slower, profiles/r03/ab_lba_tile_lmcap.log)
  const int lm_cap = std::max(16, std::min(kTileMaxLm, (nL / 512 + 3) & ~3));
  TileBuild &tb = c->tb;
  // every observation's camera in its tile's window, written straight into the
  // page-locked upload buffer
  PinVec<int> obs_loc;
  if (int e = pinned(c, P_OBSLOC, (size_t)nE, obs_loc)) return e;
  build_tiles(nP, nL, lm_begin, obs_camh.data(), lm_cap, tp, tb, obs_loc.data());
  phase("tiles");
  std::vector<int> s_row(nP + 1, 0), s_col;
  if (!sharded) {
    pattern_from_tiles(nP, tb, s_row, s_col);
    phase("  S rows");
  } else {
    std::vector<std::vector<int>> rows(nP);
    {  // rows are independent: a few host threads, each with its own marks
      const int nth = host_threads(nE);
      auto work = [&](int t0) {
        std::vector<int> mark(nP, -1), row;
        for (int i = t0; i < nP; i += nth) {
          row.clear();
          row.push_back(i);
          mark[i] = i;
          for (int t = cam_ptr[i]; t < cam_ptr[i + 1]; ++t) {
            const int s = obs_lm[cam_obs[t]];
            for (int o = lm_begin[s]; o < lm_begin[s + 1]; ++o) {
              const int j = obs_camh[o];
              if (j > i && mark[j] != i) { mark[j] = i; row.push_back(j); }
            }
          }
          std::sort(row.begin() + 1, row.end());
          rows[i] = row;
        }
      };
      run_threads(nth, work);
    }
    {  // every rank needs the same pattern: the union of the shards' patterns.
      // Blocks within kNearCams of the diagonal as one flag per (row, offset),
      // OR-ed by an all-reduce (max); the few far blocks (loop closures) as
      // (row, column) pairs all-gathered through a summed, zero-padded buffer
      constexpr int kNearCams = 64;
      std::vector<uint8_t> near((size_t)nP * kNearCams, 0);
      std::vector<int> far;
      for (int i = 0; i < nP; ++i)
        for (size_t k = 1; k < rows[i].size(); ++k) {
          const int off = rows[i][k] - i;
          if (off < kNearCams) near[(size_t)i * kNearCams + off] = 1;
          else { far.push_back(i); far.push_back(rows[i][k]); }
        }
      if (comm_allreduce_host(c->comm, near.data(), (int64_t)near.size(), SQLM_DT_U8, SQLM_OP_MAX, c->stream))
        return SQLM_ERR_COMM;
      const int R = c->comm.nranks, me = c->comm.rank;
      std::vector<int> cnt(R, 0);
      cnt[me] = (int)far.size();
      if (comm_allreduce_host(c->comm, cnt.data(), R, SQLM_DT_I32, SQLM_OP_SUM, c->stream)) return SQLM_ERR_COMM;
      int64_t tot = 0, mine = 0;
      for (int r = 0; r < R; ++r) { if (r < me) mine += cnt[r]; tot += cnt[r]; }
      std::vector<int> all((size_t)tot, 0);
      std::copy(far.begin(), far.end(), all.begin() + mine);
      if (tot && comm_allreduce_host(c->comm, all.data(), tot, SQLM_DT_I32, SQLM_OP_SUM, c->stream))
        return SQLM_ERR_COMM;
      for (int i = 0; i < nP; ++i) {
        rows[i].assign(1, i);
        for (int off = 1; off < kNearCams && i + off < nP; ++off)
          if (near[(size_t)i * kNearCams + off]) rows[i].push_back(i + off);
      }
      for (int64_t k = 0; k < tot; k += 2) rows[all[k]].push_back(all[k + 1]);
      for (int i = 0; i < nP; ++i) {
        std::sort(rows[i].begin() + 1, rows[i].end());
        rows[i].erase(std::unique(rows[i].begin() + 1, rows[i].end()), rows[i].end());
      }
    }
    for (int i = 0; i < nP; ++i) s_row[i + 1] = s_row[i] + (int)rows[i].size();
    s_col.resize(s_row[nP]);
    for (int i = 0; i < nP; ++i) std::copy(rows[i].begin(), rows[i].end(), s_col.begin() + s_row[i]);
  }
  {
    int mx = 0;
    for (int i = 0; i < nP; ++i) mx = std::max(mx, s_row[i + 1] - s_row[i]);
    c->max_row_blocks = mx;
    // band (+ border) superblock plan; the dense Cholesky otherwise
    if (!plan_rcs(nP, s_row, s_col, c->cr, c->cam_pos)) c->cr = CRPlan{};
  }
  phase("S pattern");
  build_tiles_finish(nP, s_row, s_col, tp, tb);
  phase("tile lists");
  if (ptime) {  // plan shape: tile count, longest reduction lists, solver layout
    int rmax = 0, gmax = 0;
    for (size_t s = 0; s + 1 < tp.red_ptr.size(); ++s) rmax = std::max(rmax, tp.red_ptr[s + 1] - tp.red_ptr[s]);
    for (size_t s = 0; s + 1 < tp.gred_ptr.size(); ++s) gmax = std::max(gmax, tp.gred_ptr[s + 1] - tp.gred_ptr[s]);
    std::fprintf(stderr,
                 "prepare plan: nP %d nL %d nnzb %d tiles %zu max_cp %d red %zu (max/block %d, long %zu) gred max %d "
                 "(long %zu) | CR %d B %d p %d n %d border %d R %d init %d elim %d\n",
                 nP, nL, s_row[nP], tp.lm_ptr.size() - 1, tp.max_cp, tp.red_off.size(), rmax, tp.long_s.size(), gmax,
                 tp.long_g.size(),
                 (int)c->cr.enabled, c->cr.B, c->cr.p, c->cr.n, c->cr.nbc, c->cr.R, c->cr.init_cnt, c->cr.elim_cnt);
  }
  c->use_tiles = nP > 0 && tp.max_cp <= kTileHardCams;
  c->tile_max_cp = tp.max_cp;
  c->tile_max_k = 0;
  if (!c->use_tiles && c->max_row_blocks > 128) return SQLM_ERR_UNSUPPORTED;
  // lidar edges grouped by free camera
  std::vector<int> lid_ptr(nP + 1, 0), lid_pose;
  std::vector<double> lid_data;
  {
    std::vector<std::vector<int64_t>> per(nP);
    for (int64_t e : lid_act) per[phidx[c->lid_pose[e]]].push_back(e);
    c->dev_lid_edge.clear();
    for (int i = 0; i < nP; ++i) {
      lid_ptr[i + 1] = lid_ptr[i] + (int)per[i].size();
      for (int64_t e : per[i]) {
        c->dev_lid_edge.push_back(e);
        lid_pose.push_back(c->lid_pose[e]);
        for (int k = 0; k < 3; ++k) lid_data.push_back(c->lid_pc[3 * e + k]);
        for (int k = 0; k < 3; ++k) lid_data.push_back(c->lid_pw[3 * e + k]);
        for (int k = 0; k < 3; ++k) lid_data.push_back(c->lid_n[3 * e + k]);
        lid_data.push_back(c->lid_info[e]);
        lid_data.push_back(0.0);
        lid_data.push_back(0.0);
      }
    }
  }
  phase("lidar");
  // ---------------- upload ----------------
  d.n_pose = c->n_pose;
  d.sharded = c->comm.enabled() ? 1 : 0;
  d.rank = c->comm.rank;
  d.nP = nP;
  d.nL = nL;
  d.nE = nE;
  d.nLid = (int64_t)lid_act.size();
  d.nnzb = s_row[nP];
  // single-GPU tiled path: k_rcs_reduce writes the CR superblocks directly
  d.cr_direct = (c->cr.enabled && c->use_tiles && !c->comm.enabled()) ? 1 : 0;
  d.cr_B = c->cr.B;
  d.cr_n = c->cr.n;
  d.cr_p = c->cr.p;
  d.cr_nband = c->cr.nband;
  d.arw_R = c->cr.R;
  d.arw_Rp = c->cr.Rp;
  std::vector<double> qt(8 * (size_t)c->n_pose, 0.0);
  for (int p = 0; p < c->n_pose; ++p) {
    for (int k = 0; k < 4; ++k) qt[8 * p + k] = c->pose_q[4 * p + k];
    for (int k = 0; k < 3; ++k) qt[8 * p + 4 + k] = c->pose_t[3 * p + k];
  }
  // the landmark states in slot order go through a page-locked buffer filled
  // on host threads, like obs_local (a pageable copy is staged by the runtime
  // on the calling thread: ~3 ms for these two arrays, 36 MB)
  PinVec<double> X;
  {
    if (int e = pinned(c, P_X, 4 * (size_t)nL, X)) return e;
    par([&](int t) {
      for (int sl = (int)((int64_t)nL * t / nth); sl < (int)((int64_t)nL * (t + 1) / nth); ++sl) {
        const double *src = c->pt.data() + 3 * (size_t)pts[sl];
        double *dst = X.data() + 4 * (size_t)sl;
        dst[0] = src[0];
        dst[1] = src[1];
        dst[2] = src[2];
        dst[3] = 0.0;
      }
    });
  }
  int st = 0;
  SmallUploads small;
  auto up = [&](int id, auto &vec, auto **ptr) -> int {  // std::vector: small ones into the arena
    using V = std::decay_t<decltype(vec)>;
    if constexpr (!is_pinvec<V>::value) {
      if (vec.size() * sizeof(typename V::value_type) <= kSmallUpload) {
        small.add(vec, ptr);
        return SQLM_OK;
      }
    }
    return upload(c, id, vec, ptr);
  };
  // UP: small arrays' device pointers are set when the arena is copied (before
  // the first kernel that reads them); UPD: a direct copy, pointer set now
#define UP(id, vec, ptr) \
  if ((st = up(id, vec, &ptr))) return st;
#define UPD(id, vec, ptr) \
  if ((st = upload(c, id, vec, &ptr))) return st;
#define AL(id, n, ptr) \
  if ((st = ensure(c, id, n, &ptr))) return st;
  UP(B_QT0, qt, d.pose_qt[0]);
  UP(B_QT1, qt, d.pose_qt[1]);
  AL(B_RT0, 16 * (size_t)c->n_pose, d.pose_rt[0]);
  AL(B_RT1, 16 * (size_t)c->n_pose, d.pose_rt[1]);
  UP(B_INTR, c->intr, d.intr);
  UP(B_PHIDX, phidx, d.pose_hidx);
  UP(B_HIDXP, hidxp, d.hidx_pose);
  UP(B_X0, X, d.X[0]);
  AL(B_X1, 4 * (size_t)nL, d.X[1]);
  if (nL) HIP_OK(hipMemcpyAsync(d.X[1], d.X[0], 4 * (size_t)nL * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
  UP(B_LMBEG, lm_begin, d.lm_begin);
  AL(B_LMR, 8 * (size_t)nL, d.lm_R);
  AL(B_LMB, 4 * (size_t)nL, d.lm_b);
  AL(B_LMM, 8 * (size_t)nL, d.lm_M);
  AL(B_LMV, 4 * (size_t)nL, d.lm_v);
  d.n_tiles = c->use_tiles ? (int)tp.lm_ptr.size() - 1 : 0;
  std::copy(tp.cls_off, tp.cls_off + kTileNtMax + 2, d.tile_cls_off);
  std::copy(tp.cls_cnt, tp.cls_cnt + kTileNtMax + 1, d.tile_cls_cnt);
  d.tile_dups = tp.dups ? 1 : 0;
  {
    const char *tw = std::getenv("SQLM_TILE_PROD");  // read per setup: tests switch it
    d.tile_prod = tw && std::atoi(tw) == 0 ? 0 : 1;
  }
  {
    int mk = 0;
    for (int sl = 0; sl < nL; ++sl) mk = std::max(mk, lm_begin[sl + 1] - lm_begin[sl]);
    d.tile_maxk = mk;
  }
  d.n_long_s = d.n_long_g = 0;
  if (c->use_tiles) {
    UP(B_TLM, tp.lm_ptr, d.tile_lm_ptr);
    UP(B_TCAMP, tp.cam_ptr, d.tile_cam_ptr);
    UP(B_TORDER, tp.order, d.tile_order);
    UP(B_TCAMS, tp.cams, d.tile_cams);
    UP(B_TPART, tp.part_ptr, d.tile_part_ptr);
    UP(B_TGPART, tp.gpart_ptr, d.tile_gpart_ptr);
    UP(B_TLD, tp.ld, d.tile_ld);
    UP(B_URANGE, tp.urange, d.lm_urange);
    UP(B_OBSLOC, obs_loc, d.obs_local);
    AL(B_PART2, (size_t)tp.part_ptr.back(), d.part);
    AL(B_GPART, (size_t)tp.gpart_ptr.back(), d.gpart);
    UP(B_REDP, tp.red_ptr, d.red_ptr);
    UP(B_REDI, tp.red_off, d.red_off);
    UP(B_GREDP, tp.gred_ptr, d.gred_ptr);
    UP(B_GREDI, tp.gred_off, d.gred_off);
    UP(B_LONGS, tp.long_s, d.long_s);
    UP(B_LONGG, tp.long_g, d.long_g);
    d.n_long_s = (int)tp.long_s.size();
    d.n_long_g = (int)tp.long_g.size();
  }
  UP(B_UPDRNG, upd_rng, d.upd_rng);

  AL(B_OBSS, (size_t)nE, d.obs_s);
  if (c->use_tiles) {
    d.obs_P = nullptr;  // consumers recompute the H_lp blocks from obs_s
  } else {
    AL(B_OBSP, 18 * (size_t)nE, d.obs_P);
  }
  AL(B_OBSERR, 2 * (size_t)nE, d.obs_err);
  if (sharded) {
    UPD(B_CAMPTR, cam_ptr, d.cam_obs_ptr);  // (k_cam_gather below reads them)
    UPD(B_CAMOBS, cam_obs, d.cam_obs);
  } else {  // the stable counting sort on the device (same result as the host's)
    unsigned *k0 = nullptr, *k1 = nullptr;
    int *v0 = nullptr;
    unsigned char *tmp = nullptr;
    const size_t sort_bytes = cam_csr_temp_bytes(nE, nP);
    AL(B_CAMKEY0, (size_t)nE, k0);
    AL(B_CAMKEY1, (size_t)nE, k1);
    AL(B_CAMVAL, (size_t)nE, v0);
    AL(B_SORTTMP, sort_bytes, tmp);
    AL(B_CAMOBS, (size_t)nE, d.cam_obs);
    AL(B_CAMPTR, (size_t)nP + 1, d.cam_obs_ptr);
    if (launch_cam_csr(d.obs_camh, nE, nP, k0, k1, v0, d.cam_obs, d.cam_obs_ptr, tmp, sort_bytes, c->stream))
      return SQLM_ERR_HIP;
  }
  d.has_stereo = c->has_stereo ? 1 : 0;
  if (c->has_stereo) {
    UP(B_POSEBF, c->pose_bf, d.pose_bf);
    AL(B_OBSERR3, (size_t)nE, d.obs_err3);
    AL(B_CAMUR, (size_t)n_cam_obs, d.cam_ur);
  } else {
    d.obs_ur = d.obs_err3 = d.pose_bf = d.cam_ur = nullptr;
  }
  // camera-ordered copies of the camera pass inputs (one coalesced stream +
  // the X gather), gathered on the device from the slot-ordered arrays
  AL(B_CAMSLOT, (size_t)n_cam_obs, d.cam_slot);
  if (d.obs_f32) {
    AL(B_CAMQ, 4 * (size_t)n_cam_obs, d.cam_q);
    d.cam_uv = nullptr;
  } else {
    AL(B_CAMUV, 4 * (size_t)n_cam_obs, d.cam_uv);
    d.cam_q = nullptr;
  }
  launch_cam_gather(d, n_cam_obs, c->stream);
  AL(B_HPP, 36 * (size_t)nP, d.Hpp);
  AL(B_BP, 8 * (size_t)nP, d.bp);
  {
    const bool no_spec = getenv("SQLM_NO_SPEC") && atoi(getenv("SQLM_NO_SPEC")) != 0;
    c->no_pose_fuse = getenv("SQLM_NO_POSE_FUSE") != nullptr;
    c->spec = c->use_tiles && d.obs_P == nullptr && !no_spec;
    // the side stream's fork / join (two event records, two waits: ~20 us of
    // host API time per trial) pays only when the pass is long enough to hide
    // (profiles/r03/ab_lba_cam_inline.log)
    c->cam_inline = d.nE < (1 << 18);
    if (sharded) c->cam_inline = false;
  }
  c->lin_valid = false;
  d.pc_lm = kPartChiCurLm;
  d.pc_lid = kPartChiCurLid;
  d.px_lm = kPartChiCurLm2;
  d.px_lid = kPartChiCurLid2;
  if (c->spec) {
    AL(B_LMR_NX, 8 * (size_t)nL, d.lm_R_nx);
    AL(B_LMB_NX, 4 * (size_t)nL, d.lm_b_nx);
    AL(B_OBSS_NX, (size_t)nE, d.obs_s_nx);
    AL(B_HPP_NX, 36 * (size_t)nP, d.Hpp_nx);
    AL(B_BP_NX, 8 * (size_t)nP, d.bp_nx);
  } else {
    d.lm_R_nx = d.lm_b_nx = d.obs_s_nx = d.Hpp_nx = d.bp_nx = nullptr;
  }
  UP(B_LIDPTR, lid_ptr, d.lid_cam_ptr);
  UP(B_LIDDATA, lid_data, d.lid_data);
  UP(B_LIDPOSE, lid_pose, d.lid_pose);
  AL(B_LIDERR, (size_t)d.nLid, d.lid_err);
  UP(B_SROW, s_row, d.s_row_ptr);
  UP(B_SCOL, s_col, d.s_col);
  {
    std::vector<int> srow(s_col.size());
    for (int i = 0; i < nP; ++i)
      for (int k = s_row[i]; k < s_row[i + 1]; ++k) srow[k] = i;
    UP(B_SROWIDX, srow, d.s_row);
  }
  AL(B_S, 36 * (size_t)d.nnzb, d.S);
  AL(B_G, 6 * (size_t)nP, d.g);
  AL(B_DX, 6 * (size_t)nP + 1, d.dx);
  d.cam_pos = nullptr;
  if (c->cr.enabled) {
    const size_t nb = (size_t)c->cr.p * c->cr.n * c->cr.n;
    AL(B_CRD, nb, d.cr_D);
    AL(B_CRL, nb, d.cr_L);
    AL(B_CRE, nb, d.cr_E);
    AL(B_CRA, nb, d.cr_A);
    AL(B_CRC, nb, d.cr_C);
    AL(B_CRG, (size_t)c->cr.p * c->cr.n, d.cr_g);
    AL(B_CRX, (size_t)c->cr.p * c->cr.n, d.cr_x);
    {  // completion words of the one-launch back substitution, from epoch 0
      int *dn = nullptr;
      AL(B_CRDONE, (size_t)c->cr.p, dn);
      HIP_OK(hipMemsetAsync(dn, 0, (size_t)c->cr.p * sizeof(int), c->stream));
      c->crs = CRSync{dn, c->cr.p, 0};
    }
    if (c->cr.R) {  // band + border layout
      const size_t fr = (size_t)c->cr.p * c->cr.n * c->cr.R, rp = (size_t)c->cr.Rp;
      UP(B_CAMPOS, c->cam_pos, d.cam_pos);
      int *sd = nullptr;
      UPD(B_ARWS, c->cr.sched, sd);
      c->cr.sched_dev = sd;
      AL(B_ARWG, fr, d.arw_G);
      AL(B_ARWZ, fr, d.arw_Z);
      AL(B_BDA, rp * rp, d.bd_A);
      AL(B_BDL, rp * rp, d.bd_L);
      AL(B_BDLI, rp * kCRMaxN, d.bd_Linv);
      AL(B_BDR, rp, d.bd_r);
      AL(B_BDX, rp, d.bd_x);
    }
  } else {  // blocked MFMA Cholesky of the dense S (sqlm_rcs_solve.hip)
    const int np_ = (6 * nP + kCRMaxN - 1) / kCRMaxN * kCRMaxN;
    {  // two np_ x np_ matrices: refuse what the device cannot hold instead of failing mid-solve
      size_t fr = 0, tot = 0;
      if (hipMemGetInfo(&fr, &tot) == hipSuccess && 2.0 * 8.0 * np_ * (double)np_ > 0.9 * (double)fr)
        return SQLM_ERR_OOM;
    }
    d.dense_n = np_;
    AL(B_DENSE, (size_t)np_ * np_, d.dense);
    AL(B_DENSEL, (size_t)np_ * np_, d.dense_L);
    AL(B_DENSELI, (size_t)np_ * kCRMaxN, d.dense_Linv);
    AL(B_DENSER, (size_t)np_, d.dense_r);
    AL(B_DENSEX, (size_t)np_, d.dense_x);
  }
  AL(B_PART, (size_t)kMaxPartials, d.partials);
  AL(B_SCAL, (size_t)kNScalars, d.scalars);
  AL(B_MAXD, 1, d.maxdiag);
  AL(B_FLAGS, 4, d.flags);
  HIP_OK(hipMemsetAsync(d.flags, 0, 4 * sizeof(int), c->stream));  // flags[1]: sticky device error of the solves
  d.hdiag = nullptr;
  d.xstage = nullptr;
  if (c->comm.enabled()) {
    AL(B_HDIAG, 6 * (size_t)nP, d.hdiag);
    c->s_row_host = s_row;
    // every rank's nonzero S rows: the free cameras its own edges (and, on
    // rank 0, the LiDAR edges) touch; rank 0 stages the others' rows
    int lo = nP, hi = 0;
    for (int64_t o = 0; o < nE; ++o)
      if (obs_camh[o] >= 0) { lo = std::min(lo, obs_camh[o]); hi = std::max(hi, obs_camh[o] + 1); }
    for (int i = 0; i < nP; ++i)
      if (lid_ptr[i + 1] > lid_ptr[i]) { lo = std::min(lo, i); hi = std::max(hi, i + 1); }
    if (lo >= hi) lo = hi = 0;
    const int R = c->comm.nranks, me = c->comm.rank;
    if (R > kMaxRanks) return SQLM_ERR_UNSUPPORTED;
    std::vector<int> rng(2 * R, 0);
    rng[2 * me] = lo;
    rng[2 * me + 1] = hi;
    if (comm_allreduce_host(c->comm, rng.data(), 2 * R, SQLM_DT_I32, SQLM_OP_SUM, c->stream)) return SQLM_ERR_COMM;
    c->sh_lo.assign(R, 0);
    c->sh_hi.assign(R, 0);
    for (int r = 0; r < R; ++r) { c->sh_lo[r] = rng[2 * r]; c->sh_hi[r] = rng[2 * r + 1]; }
    GatherTab &t = c->gather;
    t.n = 0;
    int64_t off = 0;
    for (int r = 1; r < R; ++r) {
      const int a = c->sh_lo[r], b = c->sh_hi[r];
      t.s_lo[t.n] = 36 * (int64_t)s_row[a];
      t.s_hi[t.n] = 36 * (int64_t)s_row[b];
      t.s_src[t.n] = off;
      off += t.s_hi[t.n] - t.s_lo[t.n];
      t.g_lo[t.n] = 6 * (int64_t)a;
      t.g_hi[t.n] = 6 * (int64_t)b;
      t.g_src[t.n] = off;
      off += t.g_hi[t.n] - t.g_lo[t.n];
      ++t.n;
    }
    if (me == 0) AL(B_XSTAGE, (size_t)std::max<int64_t>(off, 1), d.xstage);
  }
  if (!small.host.empty()) {  // the arena: one page-locked block, one copy
    uint8_t *dev = nullptr;
    AL(B_ARENA, small.host.size(), dev);
    PinVec<uint8_t> stg;
    if ((st = pinned(c, P_ARENA, small.host.size(), stg))) return st;
    std::memcpy(stg.data(), small.host.data(), small.host.size());
    HIP_OK(hipMemcpyAsync(dev, stg.data(), small.host.size(), hipMemcpyHostToDevice, c->stream));
    for (const auto &[off, p] : small.dst) *p = dev + off;
  }
#undef UP
#undef UPD
#undef AL
  HIP_OK(hipMemsetAsync(d.partials, 0, sizeof(double) * kMaxPartials, c->stream));
  HIP_OK(hipMemsetAsync(d.maxdiag, 0, sizeof(unsigned long long), c->stream));
  HIP_OK(hipMemsetAsync(d.obs_err, 0, sizeof(double) * 2 * std::max<int64_t>(nE, 1), c->stream));
  if (d.obs_err3) HIP_OK(hipMemsetAsync(d.obs_err3, 0, sizeof(double) * std::max<int64_t>(nE, 1), c->stream));
  launch_pose_prep(d, 0, c->stream);
  phase("upload");
  if (ptime) {  // how long the queued copies and setup kernels still run after the host is done
    (void)hipStreamSynchronize(c->stream);
    phase("gpu drain");
  }
  c->prepared = true;
  return SQLM_OK;
}

// The per-edge errors of the last optimize() (computeActiveErrors' _error of
// every active edge) into the caller-order host arrays: ~90 MB on config 4,
// fetched only when a caller needs an edge chi2 (LBA outlier tags,
// sqlm_get_edge_chi2) or before the next prepare() replaces them on the
// device -- a GBA call that never asks does not pay for the copy.
void ensure_host_errors(sqlm_ctx *c) {
  if (!c->err_zero) return;
  c->err_zero = false;
  par_assign(c->obs_err, (const double *)nullptr, 2 * (size_t)c->n_obs);
}

int fetch_errors(sqlm_ctx *c) {
  if (!c->err_pending) return SQLM_OK;
  c->err_pending = false;
  if (hipSetDevice(c->device) != hipSuccess) return SQLM_ERR_HIP;
  ensure_host_errors(c);
  DevProblem &d = c->d;
  PinVec<double> err, err3, lerr;
  std::vector<double> fallback[3];
  auto stage = [&](int id, size_t n, PinVec<double> &v, int k) {
    if (pinned(c, id, n, v) == SQLM_OK) return;
    fallback[k].resize(std::max<size_t>(n, 1));
    v.p = fallback[k].data();
    v.n = n;
  };
  stage(P_RERR, 2 * (size_t)d.nE, err, 0);
  stage(P_RERR3, d.obs_err3 ? (size_t)d.nE : 0, err3, 1);
  stage(P_RLERR, (size_t)d.nLid, lerr, 2);
  if (err3.size())
    HIP_OK(hipMemcpyAsync(err3.data(), d.obs_err3, err3.size() * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  if (d.nE) HIP_OK(hipMemcpyAsync(err.data(), d.obs_err, err.size() * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  if (d.nLid)
    HIP_OK(hipMemcpyAsync(lerr.data(), d.lid_err, lerr.size() * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIP_OK(hipStreamSynchronize(c->stream));
  const int nth = host_threads(d.nE);
  run_threads(nth, [&](int t) {
    for (int64_t o = d.nE * t / nth; o < d.nE * (t + 1) / nth; ++o) {
      c->obs_err[2 * c->dev_edge[o]] = err[2 * o];
      c->obs_err[2 * c->dev_edge[o] + 1] = err[2 * o + 1];
      if (err3.size()) c->obs_err3[c->dev_edge[o]] = err3[o];
    }
  });
  for (int64_t t = 0; t < d.nLid; ++t) c->lid_err[c->dev_lid_edge[t]] = lerr[t];
  return SQLM_OK;
}

int finish(sqlm_ctx *c) {
  DevProblem &d = c->d;
  // device -> page-locked staging (one DMA each; pageable vectors if the
  // page-locked arena cannot grow), then the scatter back to caller order on
  // host threads; the edge errors stay on the device until asked for
  PinVec<double> qt, X;
  std::vector<double> fallback[2];
  auto stage = [&](int id, size_t n, PinVec<double> &v, int k) {
    if (pinned(c, id, n, v) == SQLM_OK) return;
    fallback[k].resize(std::max<size_t>(n, 1));
    v.p = fallback[k].data();
    v.n = n;
  };
  stage(P_RQT, 8 * (size_t)c->n_pose, qt, 0);
  stage(P_RX, 4 * (size_t)d.nL, X, 1);
  HIP_OK(hipMemcpyAsync(qt.data(), d.pose_qt[0], qt.size() * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  if (d.nL) HIP_OK(hipMemcpyAsync(X.data(), d.X[0], X.size() * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIP_OK(hipStreamSynchronize(c->stream));
  for (int p = 0; p < c->n_pose; ++p) {
    for (int k = 0; k < 4; ++k) c->pose_q[4 * p + k] = qt[8 * p + k];
    for (int k = 0; k < 3; ++k) c->pose_t[3 * p + k] = qt[8 * p + 4 + k];
  }
  const int nth = host_threads(d.nL * 8);
  run_threads(nth, [&](int t) {
    for (int s = (int)((int64_t)d.nL * t / nth); s < (int)((int64_t)d.nL * (t + 1) / nth); ++s)
      for (int k = 0; k < 3; ++k) c->pt[3 * c->slot_pt[s] + k] = X[4 * s + k];
  });
  c->err_pending = d.nE > 0 || d.nLid > 0;
  return SQLM_OK;
}

inline void tmark(sqlm_ctx *c, int i, bool end) {
  if (c->timing) (void)hipEventRecord(c->ev[2 * i + (end ? 1 : 0)], c->stream);
}

// Add the elapsed times of timer pairs [i0, i1) (events already complete).
void acc_events(sqlm_ctx *c, int i0, int i1) {
  if (!c->timing) return;
  for (int i = i0; i < i1; ++i) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, c->ev[2 * i], c->ev[2 * i + 1]) == hipSuccess) c->kernel_ms_acc[i] += ms;
  }
}

// computeActiveErrors + buildSystem for the current state.
int linearize(sqlm_ctx *c) {
  DevProblem &d = c->d;
  c->lin_timers = 1;
  if (c->spec && c->lin_valid) {  // the accepted trial already linearized at this state
    tmark(c, 0, false);
    tmark(c, 0, true);
    return SQLM_OK;
  }
  c->lin_timers = 2;  // + the camera pass on the side stream
  // the camera pass (H_pp, b_p, LiDAR) reads only the state, like the landmark
  // QR: fork it onto the side stream and join before anything consumes H_pp
  HIP_OK(hipEventRecord(c->ev_fork, c->stream));
  HIP_OK(hipStreamWaitEvent(c->side, c->ev_fork, 0));
  if (c->timing) HIP_OK(hipEventRecord(c->ev[2], c->side));
  launch_camera_pass(d, c->side);
  if (c->timing) HIP_OK(hipEventRecord(c->ev[3], c->side));
  HIP_OK(hipEventRecord(c->ev_join, c->side));
  tmark(c, 0, false);  // maxdiag was zeroed by the last k_reduce (or prepare)
  for (size_t b = 0; b < c->buckets.size(); ++b) launch_linearize(d, c->buckets[b], c->bucket_part_off[b], c->stream);
  tmark(c, 0, true);
  HIP_OK(hipStreamWaitEvent(c->stream, c->ev_join, 0));
  if (c->comm.enabled() && c->need_maxdiag) {  // lambda_0 needs the summed pose diagonals
    launch_pose_diag(d, c->stream);
    if (comm_allreduce_dev(c->comm, d.hdiag, 6 * (int64_t)d.nP, SQLM_DT_F64, SQLM_OP_SUM, c->stream))
      return SQLM_ERR_COMM;
    launch_pose_maxdiag(d, c->stream);
  }
  return SQLM_OK;
}

struct TrialOut {
  double chi_cur, chi_new, scale, maxdiag;
  bool ok;
  bool dev_err;  // a solve kernel gave up a bounded wait (flags[1]): the result is not trusted
};

// Wait for k_reduce's mailbox entry `seq`. The stream is polled now and then:
// an error ends the wait, and so does a drained stream without the entry
// (the copy path then takes over). Returns the scalars or null.
const double *mbox_wait(sqlm_ctx *c, unsigned long long seq, int &err) {
  err = SQLM_OK;
  const unsigned long long *slot = reinterpret_cast<const unsigned long long *>(c->mbox + kMboxSeq);
  Timer t;
  for (unsigned it = 1;; ++it) {
    if (__atomic_load_n(slot, __ATOMIC_ACQUIRE) == seq) return c->mbox;
    if ((it & 1023) == 0) {
      // bounded: a stream that never drains (an error the query does not report) ends the wait
      const hipError_t q = hipStreamQuery(c->stream);
      if (q == hipSuccess) return __atomic_load_n(slot, __ATOMIC_ACQUIRE) == seq ? c->mbox : nullptr;
      if (q != hipErrorNotReady || t.ms() > 60000.0) {
        err = SQLM_ERR_HIP;
        return nullptr;
      }
    }
    __builtin_ia32_pause();
  }
}

// The speculative camera pass (H_pp / b_p at the trial state) on stream st,
// with its HIP-event timing in the timing run.
int spec_camera_pass(sqlm_ctx *c, hipStream_t st) {
  const int p = c->cam_par;
  if (c->timing && c->cam_pending[p]) {  // the pass two trials back is long complete
    float ms = 0.f;
    if (hipEventSynchronize(c->ev_cam[p][1]) == hipSuccess &&
        hipEventElapsedTime(&ms, c->ev_cam[p][0], c->ev_cam[p][1]) == hipSuccess)
      c->kernel_ms_acc[1] += ms;
    c->cam_pending[p] = false;
  }
  if (c->timing) HIP_OK(hipEventRecord(c->ev_cam[p][0], st));
  launch_camera_pass(c->d, st, true);
  if (c->timing) { HIP_OK(hipEventRecord(c->ev_cam[p][1], st)); c->cam_pending[p] = true; }
  c->cam_par ^= 1;
  return SQLM_OK;
}

// The speculative camera pass behind the work enqueued so far: inline on the
// context stream (small problems), else forked to the side stream and joined
// before the next trial's RCS reduce.
int spec_camera_launch(sqlm_ctx *c) {
  if (!c->cam_inline) {
    HIP_OK(hipEventRecord(c->ev_spec_fork, c->stream));
    HIP_OK(hipStreamWaitEvent(c->side, c->ev_spec_fork, 0));
  }
  if (int s = spec_camera_pass(c, c->cam_inline ? c->stream : c->side)) return s;
  if (!c->cam_inline) {
    HIP_OK(hipEventRecord(c->ev_spec_join, c->side));
    c->spec_outstanding = true;
  }
  return SQLM_OK;
}

// cam_after: the speculative camera pass goes right behind k_reduce (it runs
// while the host waits for the scalars and decides)
int reduce_and_fetch(sqlm_ctx *c, TrialOut &o, bool cam_after = false) {
  DevProblem &d = c->d;
  const bool mb = c->mbox && !c->timing && !c->comm.enabled();
  const unsigned long long seq = mb ? ++c->mbox_seq : 0;
  launch_reduce(d, c->n_lm_parts, c->n_lm_parts, (c->n_pose + 255) / 256, (int)((d.nLid + 255) / 256), c->stream,
                mb ? c->mbox_dev : nullptr, seq);
  if (cam_after) {
    if (int e = spec_camera_launch(c)) return e;
  }
  int s = comm_allreduce_scalars(c->comm, d.scalars, c->need_maxdiag, c->stream);
  if (s) return s;
  const double *h = nullptr;
  if (mb) {
    h = mbox_wait(c, seq, s);
    if (s) return s;
  }
  if (!h) {
    HIP_OK(hipMemcpyAsync(c->h_scalars, d.scalars, sizeof(double) * kNScalars, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    h = c->h_scalars;
  }
  o.chi_cur = h[kChiCur];
  o.chi_new = h[kChiNew];
  o.scale = h[kScale];
  o.maxdiag = h[kMaxDiag];
  o.ok = h[kSolveOk] > 0.5;
  o.dev_err = h[kDevErr] != 0.0;
  return SQLM_OK;
}

// host trace point i of the current trial: time since the previous point
inline void hmark(sqlm_ctx *c, int i) {
  if (!c->htrace) return;
  const auto now = std::chrono::steady_clock::now();
  if (i > 0 || c->ht_n > 0) c->ht_acc[i] += std::chrono::duration<double, std::micro>(now - c->ht_prev).count();
  c->ht_prev = now;
}

// setLambda + BlockSolver::solve + update + restoreDiagonal + computeActiveErrors,
// enqueued up to (not including) the trial scalars' reduction. cam_after: the
// speculative camera pass is still to go behind k_reduce.
int trial_launch(sqlm_ctx *c, double lambda, bool &cam_after) {
  DevProblem &d = c->d;
  hmark(c, 0);  // since the previous trial's scalars arrived: the host's decision
  tmark(c, 2, false);
  launch_damp(d, lambda, c->stream);
  tmark(c, 2, true);
  tmark(c, 3, false);
  if (c->use_tiles) launch_rcs_tiles(d, lambda, c->tile_max_cp, c->tile_max_k, c->stream, &c->tiles);
  else launch_rcs(d, lambda, c->max_row_blocks, c->stream);
  tmark(c, 3, true);
  hmark(c, 1);  // damp + tile launches
  tmark(c, 8, false);
  if (c->spec_outstanding) {  // H_pp / b_p (if swapped in) and the trial state buffers it reads
    HIP_OK(hipStreamWaitEvent(c->stream, c->ev_spec_join, 0));
    c->spec_outstanding = false;
  }
  if (c->use_tiles) {
    // cr_direct: the reduce assembles the CR superblocks itself; the RCS tile
    // kernel cleared them (no memset launches) unless there were no tiles
    if (d.cr_direct && d.n_tiles == 0) {
      const size_t blkbytes = (size_t)c->cr.p * c->cr.n * c->cr.n * sizeof(double);
      HIP_OK(hipMemsetAsync(d.cr_D, 0, blkbytes, c->stream));
      HIP_OK(hipMemsetAsync(d.cr_E, 0, blkbytes, c->stream));
    }
    if (d.cr_direct && c->cr.R) launch_arrow_clear(d, c->cr, c->stream);
    launch_rcs_reduce(d, lambda, c->stream);
  }
  tmark(c, 8, true);
  hmark(c, 2);  // RCS reduce
  int s = 0;
  const bool sharded = c->comm.enabled(), root = !sharded || c->comm.rank == 0;
  if (sharded) {  // gather every rank's S / g rows on rank 0
    std::vector<P2POp> ops;
    if (root) {
      const GatherTab &t = c->gather;
      for (int k = 0; k < t.n; ++k) {
        ops.push_back(P2POp{k + 1, false, d.xstage + t.s_src[k], t.s_hi[k] - t.s_lo[k], SQLM_DT_F64});
        ops.push_back(P2POp{k + 1, false, d.xstage + t.g_src[k], t.g_hi[k] - t.g_lo[k], SQLM_DT_F64});
      }
    } else {
      const int me = c->comm.rank, a = c->sh_lo[me], b = c->sh_hi[me];
      const int64_t s0 = 36 * (int64_t)c->s_row_host[a], s1 = 36 * (int64_t)c->s_row_host[b];
      ops.push_back(P2POp{0, true, d.S + s0, s1 - s0, SQLM_DT_F64});
      ops.push_back(P2POp{0, true, d.g + 6 * (int64_t)a, 6 * (int64_t)(b - a), SQLM_DT_F64});
    }
    if (comm_group_p2p(c->comm, ops, c->stream)) return SQLM_ERR_COMM;
    if (root) launch_gather_add(d, c->gather, c->stream);
  }
  tmark(c, 4, false);
  // unsharded CR: the pose update reads dx off the CR solution (no gather launch)
  const bool pose_from_cr = !sharded && c->cr.enabled;
  if (root) {
    s = c->cr.enabled ? launch_cr_solve(d, c->cr, c->stream, !pose_from_cr, &c->crs)
                      : launch_dense_solve(d, c->stream);
    if (s) return s == -2 ? SQLM_ERR_HIP : SQLM_ERR_UNSUPPORTED;
  }
  if (sharded) {  // dx and the solve flag from rank 0
    if (root) launch_flag_pack(d, false, c->stream);
    if (comm_bcast_dev(c->comm, d.dx, 6 * (int64_t)d.nP + 1, SQLM_DT_F64, 0, c->stream)) return SQLM_ERR_COMM;
    if (!root) launch_flag_pack(d, true, c->stream);
  }
  tmark(c, 4, true);
  hmark(c, 3);  // solve launches
  // the pose update folded into the first landmark-update launch (one launch
  // less per trial; SQLM_NO_POSE_FUSE=1 keeps it separate, A/B and tests)
  const bool no_fuse = c->no_pose_fuse;
  // (small problems only: the fused variant runs at lower occupancy, which the
  // latency-bound config-4 update pays for more than one launch saves)
  // (the fused variant is instantiated for the speculative schedule only)
  const bool fuse = pose_from_cr && c->spec && c->cam_inline && !no_fuse && !c->buckets.empty() && !c->buckets[0].wide;
  tmark(c, 5, false);
  if (!fuse) launch_pose_update(d, lambda, c->stream, pose_from_cr);
  tmark(c, 5, true);
  tmark(c, 6, false);
  // (the buckets on three streams, like the tile classes, measured slower:
  // 686 -> 647 it/s, the CR solve after them 0.54 -> 0.61 ms; profiles/r03/ab_upd_streams.log)
  // every bucket in one launch (the fused first bucket of a small problem
  // keeps its own launch: the fused form of the merged kernel measured slower)
  if (!fuse && c->upd.nb > 0) {
    launch_landmark_update_all(d, c->upd, lambda, c->stream, c->spec);
  } else {
    for (size_t b = 0; b < c->buckets.size(); ++b)
      launch_landmark_update(d, c->buckets[b], lambda, c->bucket_part_off[b], c->stream, c->spec, fuse && b == 0);
  }
  launch_lidar_chi2(d, c->stream);
  tmark(c, 6, true);
  hmark(c, 4);  // pose + landmark updates
  // camera pass at the trial state: on the side stream, overlapped with the
  // host's decision and the next trial; small problems (cam_inline) keep it on
  // the context stream behind k_reduce instead -- the fork / join costs the
  // host more than the overlap saves there
  // (config 4 with the fork after k_reduce too, so that the host's scalars
  // come ~4 us sooner: within noise, profiles/r05/ab_stream_order_rejected.log)
  cam_after = c->spec && c->cam_inline && !c->timing;
  if (c->spec && !cam_after) return spec_camera_launch(c);
  return SQLM_OK;
}

int trial(sqlm_ctx *c, double lambda, TrialOut &o) {
  bool cam_after = false;
  int s = trial_launch(c, lambda, cam_after);
  if (s) return s;
  tmark(c, 7, false);
  hmark(c, 5);  // speculative camera pass
  s = reduce_and_fetch(c, o, cam_after);
  tmark(c, 7, true);
  hmark(c, 6);  // reduce launch + wait for the scalars
  if (c->htrace) ++c->ht_n;
  acc_events(c, 2, SQLM_NKERNEL_TIMERS);
  return s;
}

void swap_state(sqlm_ctx *c) {
  DevProblem &d = c->d;
  std::swap(d.pose_qt[0], d.pose_qt[1]);
  std::swap(d.pose_rt[0], d.pose_rt[1]);
  std::swap(d.X[0], d.X[1]);
  c->lin_valid = c->spec;
  if (c->spec) {  // the speculative linearization at the accepted state becomes current
    std::swap(d.lm_R, d.lm_R_nx);
    std::swap(d.lm_b, d.lm_b_nx);
    std::swap(d.obs_s, d.obs_s_nx);
    std::swap(d.Hpp, d.Hpp_nx);
    std::swap(d.bp, d.bp_nx);
    std::swap(d.pc_lm, d.px_lm);
    std::swap(d.pc_lid, d.px_lid);
  }
}

// Timing of speculative camera passes not yet added (end of an LM run).
void flush_cam_timers(sqlm_ctx *c) {
  for (int p = 0; p < 2; ++p) {
    if (!c->cam_pending[p]) continue;
    float ms = 0.f;
    if (hipEventSynchronize(c->ev_cam[p][1]) == hipSuccess &&
        hipEventElapsedTime(&ms, c->ev_cam[p][0], c->ev_cam[p][1]) == hipSuccess)
      c->kernel_ms_acc[1] += ms;
    c->cam_pending[p] = false;
  }
}

// Host loop: every trial's scalars come back before the next trial is
// enqueued, and the host applies lm_decide. (A device-side loop -- k_reduce
// deciding, trials enqueued two ahead -- measured slower on MI355X: every
// per-trial kernel then starts with a dependent load of the control block,
// which costs more than the host turnaround it hides, config 4 703 -> 649-675
// it/s, config 2 5.58-5.61k -> 5.40k it/s, profiles/r04/ab_dlm_fuse_r4.log;
// removed in round 5.)
int lm_host(sqlm_ctx *c, LMCtl &L, const volatile uint8_t *stop) {
  while (!L.done) {
    if (L.qmax == 0 && L.its > 0) {  // the next iteration (sparse_optimizer.cpp:376-414)
      if (stopped(stop)) break;
      c->need_maxdiag = false;
      if (int s = linearize(c)) return s;
    }
    TrialOut o{};
    if (int s = trial(c, L.lambda, o)) return s;
    if (o.dev_err) return SQLM_ERR_HIP;  // a solve gave up a bounded wait (the step was rejected on the device too)
    if (L.qmax == 0) acc_events(c, 0, c->lin_timers);
    if (lm_decide(L, o.chi_cur, o.chi_new, o.scale, o.ok, stopped(stop))) swap_state(c);
    if (L.qmax == 0) c->kernel_ms_n++;  // an iteration ended
  }
  return SQLM_OK;
}

// The Levenberg–Marquardt loop of g2o (levenberg.cpp:61-164 inside
// sparse_optimizer.cpp:376-414). `bench` keeps iterating after Terminate so a
// fixed number of iterations can be timed.
int run_lm(sqlm_ctx *c, int iterations, double user_lambda, const volatile uint8_t *stop, sqlm_stats *st,
           int *n_iter, bool bench) {
  sqlm_stats local;
  if (!st) st = &local;
  std::memset(st, 0, sizeof(*st));
  st->n_active_edges = c->n_active_edges;
  c->lin_valid = false;  // iteration 0 linearizes in full (lambda_0 needs max diag H)
  Timer tt;
  LMCtl L;
  std::memset(&L, 0, sizeof(LMCtl));
  L.iterations = iterations;
  L.bench = bench ? 1 : 0;
  L.done = iterations <= 0 || stopped(stop);
  if (!L.done) {
    Timer tl;
    c->need_maxdiag = true;
    int s = linearize(c);
    if (s) return s;
    TrialOut o0{};
    s = reduce_and_fetch(c, o0);
    c->need_maxdiag = false;
    if (s) return s;
    L.currentChi = L.iniChi = o0.chi_cur;  // computeActiveErrors at iteration 0 (levenberg.cpp:66-97)
    st->chi2_begin = o0.chi_cur;
    L.lambda = user_lambda > 0 ? user_lambda : 1e-5 * o0.maxdiag;  // computeLambdaInit
    L.ni = 2;
    st->ms_linearize += tl.ms();
    Timer tr;
    s = lm_host(c, L, stop);
    if (s) return s;
    st->ms_trials += tr.ms();
  }
  if (c->spec_outstanding) {  // nothing of a speculative pass outlives the run
    HIP_OK(hipStreamWaitEvent(c->stream, c->ev_spec_join, 0));
    c->spec_outstanding = false;
  }
  flush_cam_timers(c);
  if (c->htrace && c->ht_n > 0) {
    static const char *nm[7] = {"decide", "tiles", "reduce", "solve", "updates", "campass", "wait"};
    std::fprintf(stderr, "host trace (%d trials, us/trial):", c->ht_n);
    for (int i = 0; i < 7; ++i) std::fprintf(stderr, " %s %.1f", nm[i], c->ht_acc[i] / c->ht_n);
    std::fprintf(stderr, "\n");
    std::memset(c->ht_acc, 0, sizeof(c->ht_acc));
    c->ht_n = 0;
  }
  st->iterations = L.its;
  st->trials = L.trials;
  st->result = L.result;
  st->chi2_end = L.chi2_end;
  st->lambda_end = L.lambda_end;
  st->trace_len = std::min(L.its, SQLM_TRACE_MAX);
  for (int k = 0; k < st->trace_len; ++k) {
    st->trace_chi2[k] = L.trace_chi2[k];
    st->trace_lambda[k] = L.trace_lambda[k];
    st->trace_trials[k] = L.trace_trials[k];
  }
  st->ms_total = tt.ms();
  if (n_iter) *n_iter = L.its;
  return SQLM_OK;
}

int optimize_impl(sqlm_ctx *c, int level, int iterations, double user_lambda, const volatile uint8_t *stop,
                  sqlm_stats *st, int *n_iter) {
  if (!c->has_problem) return SQLM_ERR_STATE;
  Timer ts;
  int s = prepare(c, level);
  if (s == SQLM_ERR_STATE) {  // nothing to optimize: optimize() returns -1
    if (st) std::memset(st, 0, sizeof(*st));
    if (n_iter) *n_iter = -1;
    return SQLM_OK;
  }
  if (s) return s;
  const double setup = ts.ms();
  s = run_lm(c, iterations, user_lambda, stop, st, n_iter, false);
  if (s) return s;
  s = finish(c);
  if (s) return s;
  if (st) st->ms_setup = setup;
  return SQLM_OK;
}

void depth_positive_host(const sqlm_ctx *c, std::vector<uint8_t> &out) {
  out.resize(c->n_obs);
  for (int64_t e = 0; e < c->n_obs; ++e) {
    const int p = c->obs_pose[e];
    double o[3];
    q_rotate(&c->pose_q[4 * p], &c->pt[3 * c->obs_pt[e]], o);
    out[e] = (o[2] + c->pose_t[3 * p + 2]) > 0.0;
  }
}

inline double edge_chi2(const sqlm_ctx *c, int64_t e) {
  const double e0 = c->obs_err[2 * e], e1 = c->obs_err[2 * e + 1], w = c->obs_info[e];
  if (c->has_stereo && c->obs_ur[e] >= 0.0) {  // BaseEdge::chi2 of the 3-D stereo error
    const double e2 = c->obs_err3[e];
    return e0 * (w * e0) + e1 * (w * e1) + e2 * (w * e2);
  }
  return e0 * (w * e0) + e1 * (w * e1);
}

// LBA outlier threshold: chi2(0.95), 2 DoF for mono edges (g2oOptimizer.cc:956,
// 1123). The reference's LBA adds no stereo edges (:914-916); 7.815 (3 DoF) is
// the ORB-SLAM2 value for them.
inline double tag_threshold(const sqlm_ctx *c, int64_t e) {
  return (c->has_stereo && c->obs_ur[e] >= 0.0) ? 7.815 : 5.991;
}

}  // namespace

// ====================================================================== ABI

extern "C" {

const char *sqlm_version(void) { return "sqrtlm-mi355x 0.1.0 (gfx950)"; }

const char *sqlm_status_string(int s) {
  switch (s) {
    case SQLM_OK: return "ok";
    case SQLM_ERR_INVALID_ARG: return "invalid argument";
    case SQLM_ERR_HIP: return "HIP runtime error";
    case SQLM_ERR_NOT_SPD: return "system not positive definite";
    case SQLM_ERR_OOM: return "out of device memory";
    case SQLM_ERR_ABORTED: return "aborted by stop flag";
    case SQLM_ERR_NO_DEVICE: return "no HIP device";
    case SQLM_ERR_STATE: return "call order / state error";
    case SQLM_ERR_UNSUPPORTED: return "problem shape not supported by this build";
    case SQLM_ERR_COMM: return "RCCL communicator error";
    default: return "unknown";
  }
}

int sqlm_ctx_create(int device_id, sqlm_ctx **out) {
  if (!out) return SQLM_ERR_INVALID_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return SQLM_ERR_NO_DEVICE;
  int dev = device_id;
  if (dev < 0 && hipGetDevice(&dev) != hipSuccess) return SQLM_ERR_HIP;
  if (dev >= n) return SQLM_ERR_INVALID_ARG;
  if (hipSetDevice(dev) != hipSuccess) return SQLM_ERR_HIP;
  sqlm_ctx *c = new (std::nothrow) sqlm_ctx();
  if (!c) return SQLM_ERR_OOM;
  c->device = dev;
  if (hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c->n_cu <= 0)
    c->n_cu = 256;
  c->htrace = std::getenv("SQLM_HOST_TRACE") != nullptr;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) { delete c; return SQLM_ERR_HIP; }
  if (hipHostMalloc((void **)&c->h_scalars, sizeof(double) * kNScalars) != hipSuccess) {
    (void)hipStreamDestroy(c->stream);
    delete c;
    return SQLM_ERR_HIP;
  }
  // the mailbox is an optimisation: without it the trial scalars are copied
  if (hipHostMalloc((void **)&c->mbox, sizeof(double) * kNScalars, hipHostMallocMapped | hipHostMallocCoherent) ==
      hipSuccess) {
    std::memset(c->mbox, 0, sizeof(double) * kNScalars);
    if (hipHostGetDevicePointer((void **)&c->mbox_dev, c->mbox, 0) != hipSuccess) {
      (void)hipHostFree(c->mbox);
      c->mbox = c->mbox_dev = nullptr;
    }
  } else {
    c->mbox = nullptr;
  }
  // timing-only events: no system-scope fence, which would flush caches and
  // leave a ~10 us bubble between the kernels they separate
  for (auto &e : c->ev) (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
  for (auto &pr : c->ev_cam)
    for (auto &e : pr) (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
  // The side stream (the speculative camera pass of large problems, beside the
  // next trial's RCS tiles) at the lowest priority: the tiles keep the CUs and
  // the pass fills their tails (config 4 727.7-728.7 -> 729.6-734.6 it/s,
  // interleaved, profiles/r04/ab_side_prio.log).
  auto side_stream = [](hipStream_t *s) {
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess)
      return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
    return hipStreamCreateWithPriority(s, hipStreamNonBlocking, least);
  };
  // the two extra RCS-tile class streams at normal priority (lowest / highest
  // measured within noise, profiles/r04/ab_tile_prio.log)
  auto tile_stream = [](hipStream_t *s, int) { return hipStreamCreateWithFlags(s, hipStreamNonBlocking); };
  if (side_stream(&c->side) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_spec_fork, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_spec_join, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess ||
      tile_stream(&c->tiles.s[0], 0) != hipSuccess || tile_stream(&c->tiles.s[1], 1) != hipSuccess ||
      hipEventCreateWithFlags(&c->tiles.fork, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess ||
      hipEventCreateWithFlags(&c->tiles.join[0], hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess ||
      hipEventCreateWithFlags(&c->tiles.join[1], hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess) {
    sqlm_ctx_destroy(c);
    return SQLM_ERR_HIP;
  }
  *out = c;
  return SQLM_OK;
}

int sqlm_ctx_destroy(sqlm_ctx *c) {
  if (!c) return SQLM_ERR_INVALID_ARG;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  comm_destroy(c->comm);
  if (c->eg) eg_destroy(c->eg);
  if (c->orb) orb_destroy(c->orb);
  for (auto &b : c->bufs)
    if (b.p) (void)hipFree(b.p);
  for (auto &b : c->pins) free_pinned(b);
  for (auto &e : c->ev)
    if (e) (void)hipEventDestroy(e);
  if (c->h_scalars) (void)hipHostFree(c->h_scalars);
  if (c->mbox) (void)hipHostFree(c->mbox);
  if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
  if (c->ev_join) (void)hipEventDestroy(c->ev_join);
  if (c->ev_spec_fork) (void)hipEventDestroy(c->ev_spec_fork);
  if (c->ev_spec_join) (void)hipEventDestroy(c->ev_spec_join);
  for (hipStream_t &x : c->tiles.s)
    if (x) (void)hipStreamDestroy(x);
  for (hipEvent_t x : {c->tiles.fork, c->tiles.join[0], c->tiles.join[1]})
    if (x) (void)hipEventDestroy(x);
  for (auto &pr : c->ev_cam)
    for (auto &e : pr)
      if (e) (void)hipEventDestroy(e);
  if (c->side) (void)hipStreamDestroy(c->side);
  (void)hipStreamDestroy(c->stream);
  delete c;
  return SQLM_OK;
}

int sqlm_set_problem(sqlm_ctx *c, int n_pose, const double *pose_q, const double *pose_t,
                     const uint8_t *pose_fixed, const double *intr, int n_pt, const double *pt, int64_t n_obs,
                     const int32_t *obs_pose, const int32_t *obs_pt, const double *obs_uv, const double *obs_info,
                     const double *obs_delta, const uint8_t *obs_level) {
  if (!c || n_pose < 0 || n_pt < 0 || n_obs < 0) return SQLM_ERR_INVALID_ARG;
  if ((n_pose && (!pose_q || !pose_t || !pose_fixed || !intr)) || (n_pt && !pt) ||
      (n_obs && (!obs_pose || !obs_pt || !obs_uv || !obs_info)))
    return SQLM_ERR_INVALID_ARG;
  {
    const int nth = host_threads(n_obs);
    std::vector<uint8_t> bad(nth, 0);
    run_threads(nth, [&](int t) {
      for (int64_t e = n_obs * t / nth; e < n_obs * (t + 1) / nth; ++e)
        if (obs_pose[e] < 0 || obs_pose[e] >= n_pose || obs_pt[e] < 0 || obs_pt[e] >= n_pt) { bad[t] = 1; break; }
    });
    for (uint8_t b : bad)
      if (b) return SQLM_ERR_INVALID_ARG;
  }
  c->n_pose = n_pose;
  c->n_pt = n_pt;
  c->n_obs = n_obs;
  c->pose_q.assign(pose_q, pose_q + 4 * (size_t)n_pose);
  c->pose_t.assign(pose_t, pose_t + 3 * (size_t)n_pose);
  c->pose_fixed.assign(pose_fixed, pose_fixed + n_pose);
  c->intr.assign(intr, intr + 4 * (size_t)n_pose);
  par_assign(c->pt, pt, 3 * (size_t)n_pt);
  par_assign(c->obs_pose, obs_pose, (size_t)n_obs);
  par_assign(c->obs_pt, obs_pt, (size_t)n_obs);
  par_assign(c->obs_uv, obs_uv, 2 * (size_t)n_obs);
  par_assign(c->obs_info, obs_info, (size_t)n_obs);
  par_assign(c->obs_delta, obs_delta, (size_t)n_obs);  // null: no robust kernel (zeros)
  par_assign(c->obs_level, obs_level, (size_t)n_obs);  // null: level 0
  c->err_pending = false;  // sized and zeroed when first read (ensure_host_errors)
  c->err_zero = true;
  c->has_stereo = false;
  c->obs_ur.clear(); c->pose_bf.clear(); c->obs_err3.clear();
  c->n_lid = 0;
  c->lid_pose.clear(); c->lid_pc.clear(); c->lid_pw.clear(); c->lid_n.clear(); c->lid_info.clear();
  c->lid_level.clear(); c->lid_err.clear();
  c->has_problem = true;
  c->prepared = false;  // the CR layout of the previous problem no longer applies
  return SQLM_OK;
}

int sqlm_set_stereo(sqlm_ctx *c, const double *obs_ur, const double *pose_bf) {
  if (!c || !c->has_problem) return SQLM_ERR_STATE;
  c->prepared = false;  // a setter changes what prepare() plans
  if (int s = fetch_errors(c)) return s;  // the last call's errors, in the layout they were computed in
  c->has_stereo = false;
  c->obs_ur.clear(); c->pose_bf.clear(); c->obs_err3.clear();
  if (!obs_ur) return SQLM_OK;  // back to all-mono
  if (!pose_bf && c->n_pose) return SQLM_ERR_INVALID_ARG;
  bool any = false;
  for (int64_t e = 0; e < c->n_obs; ++e) {
    if (!std::isfinite(obs_ur[e])) return SQLM_ERR_INVALID_ARG;
    any |= obs_ur[e] >= 0.0;
  }
  if (!any) return SQLM_OK;
  c->obs_ur.assign(obs_ur, obs_ur + c->n_obs);
  c->pose_bf.assign(pose_bf, pose_bf + c->n_pose);
  c->obs_err3.assign(c->n_obs, 0.0);
  c->has_stereo = true;
  return SQLM_OK;
}

int sqlm_set_lidar(sqlm_ctx *c, int64_t n, const int32_t *pose, const double *p_cam, const double *p_world,
                   const double *normal, const double *info) {
  if (!c || !c->has_problem || n < 0) return SQLM_ERR_INVALID_ARG;
  c->prepared = false;  // a setter changes what prepare() plans
  if (n && (!pose || !p_cam || !p_world || !normal || !info)) return SQLM_ERR_INVALID_ARG;
  for (int64_t e = 0; e < n; ++e)
    if (pose[e] < 0 || pose[e] >= c->n_pose) return SQLM_ERR_INVALID_ARG;
  if (int s = fetch_errors(c)) return s;  // the last call's errors, in the layout they were computed in
  c->n_lid = n;
  c->lid_pose.assign(pose, pose + n);
  c->lid_pc.assign(p_cam, p_cam + 3 * n);
  c->lid_pw.assign(p_world, p_world + 3 * n);
  c->lid_n.assign(normal, normal + 3 * n);
  c->lid_info.assign(info, info + n);
  c->lid_level.assign(n, 0);
  c->lid_err.assign(n, 0.0);
  return SQLM_OK;
}

int sqlm_set_edge_level(sqlm_ctx *c, const uint8_t *level) {
  if (!c || !c->has_problem || (!level && c->n_obs)) return SQLM_ERR_INVALID_ARG;
  c->prepared = false;  // a setter changes what prepare() plans
  c->obs_level.assign(level, level + c->n_obs);
  return SQLM_OK;
}

int sqlm_set_lidar_level(sqlm_ctx *c, const uint8_t *level) {
  if (!c || !c->has_problem || (!level && c->n_lid)) return SQLM_ERR_INVALID_ARG;
  c->prepared = false;  // a setter changes what prepare() plans
  c->lid_level.assign(level, level + c->n_lid);
  return SQLM_OK;
}

int sqlm_set_robust(sqlm_ctx *c, const double *delta) {
  if (!c || !c->has_problem) return SQLM_ERR_INVALID_ARG;
  c->prepared = false;  // a setter changes what prepare() plans
  if (delta) c->obs_delta.assign(delta, delta + c->n_obs);
  else c->obs_delta.assign(c->n_obs, 0.0);
  return SQLM_OK;
}

int sqlm_optimize(sqlm_ctx *c, int level, int iterations, double user_lambda, const volatile uint8_t *stop,
                  sqlm_stats *st, int *n_iter) {
  if (!c || iterations < 0) return SQLM_ERR_INVALID_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return SQLM_ERR_HIP;
  return optimize_impl(c, level, iterations, user_lambda, stop, st, n_iter);
}

int sqlm_local_ba(sqlm_ctx *c, const volatile uint8_t *stop, uint8_t *outlier, sqlm_stats st[3], int *ran) {
  if (!c || !c->has_problem) return SQLM_ERR_STATE;
  if (hipSetDevice(c->device) != hipSuccess) return SQLM_ERR_HIP;
  sqlm_stats tmp[3];
  if (!st) st = tmp;
  std::memset(st, 0, 3 * sizeof(sqlm_stats));
  if (ran) *ran = 0;
  if (stopped(stop)) return SQLM_OK;  // g2oOptimizer.cc:923-928
  for (auto &l : c->lid_level) l = 255;  // LiDAR edges only exist in pass 3
  int n = 0, s = optimize_impl(c, 0, 5, 0.0, stop, &st[0], &n);
  if (s) return s;
  if ((s = fetch_errors(c))) return s;
  ensure_host_errors(c);
  if (!stopped(stop)) {  // :952-975
    std::vector<uint8_t> dp;
    depth_positive_host(c, dp);
    for (int64_t e = 0; e < c->n_obs; ++e) {
      if (edge_chi2(c, e) > tag_threshold(c, e) || !dp[e]) c->obs_level[e] = 1;
      c->obs_delta[e] = 0.0;
    }
    s = optimize_impl(c, 0, 10, 0.0, stop, &st[1], &n);
    if (s) return s;
  }
  for (auto &l : c->lid_level) l = 0;  // :1113-1114
  s = optimize_impl(c, 0, 20, 0.0, stop, &st[2], &n);
  if (s) return s;
  if (outlier) {  // :1119-1136
    std::vector<uint8_t> dp;
    depth_positive_host(c, dp);
    if ((s = fetch_errors(c))) return s;
    ensure_host_errors(c);
    for (int64_t e = 0; e < c->n_obs; ++e) outlier[e] = (edge_chi2(c, e) > tag_threshold(c, e) || !dp[e]);
  }
  if (ran) *ran = 1;
  return SQLM_OK;
}

int sqlm_eg_set_problem(sqlm_ctx *c, int n_kf, const double *Siw, const uint8_t *fixed, int fix_scale, int64_t n_edge,
                        const int32_t *ei, const int32_t *ej, const double *Sji, const double *info) {
  if (!c) return SQLM_ERR_INVALID_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return SQLM_ERR_HIP;
  if (!c->eg && !(c->eg = eg_create(c->stream))) return SQLM_ERR_OOM;
  return eg_set_problem(c->eg, n_kf, Siw, fixed, fix_scale, n_edge, ei, ej, Sji, info);
}

int sqlm_eg_optimize(sqlm_ctx *c, int iterations, double user_lambda, const volatile uint8_t *stop, sqlm_stats *st,
                     int *n_iter) {
  if (!c || !c->eg) return SQLM_ERR_STATE;
  if (hipSetDevice(c->device) != hipSuccess) return SQLM_ERR_HIP;
  return eg_optimize(c->eg, iterations, user_lambda, stop, st, n_iter);
}

int sqlm_eg_get_poses(sqlm_ctx *c, double *Siw) {
  if (!c || !c->eg) return SQLM_ERR_STATE;
  return eg_get_poses(c->eg, Siw);
}

int sqlm_eg_get_edge_chi2(sqlm_ctx *c, double *chi2) {
  if (!c || !c->eg) return SQLM_ERR_STATE;
  return eg_get_edge_chi2(c->eg, chi2);
}

int sqlm_eg_get_jacobians(sqlm_ctx *c, double *J) {
  if (!c || !c->eg) return SQLM_ERR_STATE;
  if (hipSetDevice(c->device) != hipSuccess) return SQLM_ERR_HIP;
  return eg_get_jacobians(c->eg, J);
}

int sqlm_global_ba(sqlm_ctx *c, int iterations, const volatile uint8_t *stop, sqlm_stats *st, int *n_iter) {
  return sqlm_optimize(c, 0, iterations, 0.0, stop, st, n_iter);
}

int sqlm_get_poses(sqlm_ctx *c, double *q, double *t) {
  if (!c || !c->has_problem) return SQLM_ERR_STATE;
  if (q) std::memcpy(q, c->pose_q.data(), sizeof(double) * c->pose_q.size());
  if (t) std::memcpy(t, c->pose_t.data(), sizeof(double) * c->pose_t.size());
  return SQLM_OK;
}

int sqlm_get_points(sqlm_ctx *c, double *pt) {
  if (!c || !c->has_problem) return SQLM_ERR_STATE;
  if (pt) std::memcpy(pt, c->pt.data(), sizeof(double) * c->pt.size());
  return SQLM_OK;
}

int sqlm_get_edge_chi2(sqlm_ctx *c, double *chi2) {
  if (!c || !c->has_problem) return SQLM_ERR_STATE;
  if (!chi2 && c->n_obs) return SQLM_ERR_INVALID_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return SQLM_ERR_HIP;
  if (int s = fetch_errors(c)) return s;
  ensure_host_errors(c);
  for (int64_t e = 0; e < c->n_obs; ++e) chi2[e] = edge_chi2(c, e);
  return SQLM_OK;
}

int sqlm_get_edge_depth_positive(sqlm_ctx *c, uint8_t *pos) {
  if (!c || !c->has_problem) return SQLM_ERR_STATE;
  if (!pos && c->n_obs) return SQLM_ERR_INVALID_ARG;
  std::vector<uint8_t> dp;
  depth_positive_host(c, dp);
  if (c->n_obs) std::memcpy(pos, dp.data(), c->n_obs);
  return SQLM_OK;
}

int sqlm_get_rcs_layout(sqlm_ctx *c, int out[8]) {
  if (!c || !out) return SQLM_ERR_INVALID_ARG;
  if (!c->has_problem || !c->prepared) return SQLM_ERR_STATE;
  const CRPlan &pl = c->cr;
  const int nP = c->d.nP;
  out[0] = nP == 0 ? 0 : !pl.enabled ? 3 : pl.R ? 2 : 1;
  out[1] = pl.B;
  out[2] = pl.p;
  out[3] = pl.n;
  out[4] = pl.nbc;
  out[5] = pl.R;
  out[6] = nP;
  out[7] = pl.init_cnt;
  return SQLM_OK;
}

int sqlm_get_exec_info(sqlm_ctx *c, int out[8]) {
  if (!c || !out) return SQLM_ERR_INVALID_ARG;
  if (!c->has_problem || !c->prepared) return SQLM_ERR_STATE;
  const CRPlan &pl = c->cr;
  for (int k = 0; k < 8; ++k) out[k] = 0;
  out[0] = c->d.obs_f32 ? 1 : 0;
  out[1] = c->d.nP == 0 ? 0 : !pl.enabled ? 4 : pl.R ? 3 : 1;
  return SQLM_OK;
}

int sqlm_get_edge_level(sqlm_ctx *c, uint8_t *level) {
  if (!c || !c->has_problem) return SQLM_ERR_STATE;
  if (!level && c->n_obs) return SQLM_ERR_INVALID_ARG;
  if (c->n_obs) std::memcpy(level, c->obs_level.data(), c->n_obs);
  return SQLM_OK;
}

void sqlm_pose_from_Tcw_f32(const float T[16], double q[4], double t[3]) {
  double R[9];
  for (int r = 0; r < 3; ++r)
    for (int k = 0; k < 3; ++k) R[r * 3 + k] = (double)T[r * 4 + k];
  q_from_mat(R, q);
  q_normalize_rot(q);
  for (int r = 0; r < 3; ++r) t[r] = (double)T[r * 4 + 3];
}

void sqlm_pose_to_Tcw_f32(const double q[4], const double t[3], float T[16]) {
  double R[9];
  q_to_mat(q, R);
  for (int r = 0; r < 3; ++r) {
    for (int k = 0; k < 3; ++k) T[r * 4 + k] = (float)R[r * 3 + k];
    T[r * 4 + 3] = (float)t[r];
  }
  T[12] = 0.f; T[13] = 0.f; T[14] = 0.f; T[15] = 1.f;
}

int sqlm_ctx_set_host_comm(sqlm_ctx *c, int rank, int nranks, sqlm_allreduce_fn fn, void *user) {
  if (!c || nranks < 1 || rank < 0 || rank >= nranks || (nranks > 1 && !fn)) return SQLM_ERR_INVALID_ARG;
  return comm_init_host(c->comm, rank, nranks, fn, user);
}

int sqlm_ctx_set_host_p2p(sqlm_ctx *c, sqlm_p2p_fn fn, void *user) {
  if (!c || !fn) return SQLM_ERR_INVALID_ARG;
  c->comm.host_p2p = fn;
  c->comm.host_p2p_user = user;
  return SQLM_OK;
}

int sqlm_comm_id_size(void) { return comm_id_size(); }
int sqlm_comm_get_unique_id(char *id) { return comm_get_unique_id(id); }
int sqlm_ctx_set_comm(sqlm_ctx *c, const char *id, int rank, int nranks) {
  if (!c || !id || rank < 0 || nranks < 1 || rank >= nranks) return SQLM_ERR_INVALID_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return SQLM_ERR_HIP;
  return comm_init(c->comm, id, rank, nranks);
}

int sqlm_ctx_comm_info(const sqlm_ctx *c, int *transport, int *rank, int *nranks) {
  if (!c || !transport || !rank || !nranks) return SQLM_ERR_INVALID_ARG;
  return comm_info(c->comm, transport, rank, nranks);
}

int sqlm_ctx_set_comm_selfloop(sqlm_ctx *c, const char *id) {
  if (!c || !id) return SQLM_ERR_INVALID_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return SQLM_ERR_HIP;
  return comm_init_selfloop(c->comm, id) ? SQLM_ERR_COMM : SQLM_OK;
}

int sqlm_comm_selftest(int device, const char *id, int64_t n, double *max_err) {
  if (!id || n <= 0 || !max_err) return SQLM_ERR_INVALID_ARG;
  if (hipSetDevice(device) != hipSuccess) return SQLM_ERR_HIP;
  Comm cm;
  if (comm_init_selfloop(cm, id)) return SQLM_ERR_COMM;
  hipStream_t st = nullptr;
  double *a = nullptr, *b = nullptr;
  int32_t *ia = nullptr;
  uint8_t *ua = nullptr;
  int r = SQLM_OK;
  std::vector<double> ha(n), hb(n);
  std::vector<int32_t> hi(n);
  std::vector<uint8_t> hu(n);
  for (int64_t i = 0; i < n; ++i) {
    ha[i] = 0.5 * (double)i - 3.25;
    hi[i] = (int32_t)(7 * i - 11);
    hu[i] = (uint8_t)(i * 13);
  }
  double err = 0.0;
  auto upd = [&](double v) { err = std::max(err, std::fabs(v)); };
  if (hipStreamCreate(&st) != hipSuccess || hipMalloc(&a, n * 8) != hipSuccess || hipMalloc(&b, n * 8) != hipSuccess ||
      hipMalloc(&ia, n * 4) != hipSuccess || hipMalloc(&ua, n) != hipSuccess) {
    r = SQLM_ERR_HIP;
  } else if (hipMemcpyAsync(a, ha.data(), n * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
             hipMemsetAsync(b, 0, n * 8, st) != hipSuccess ||
             hipMemcpyAsync(ia, hi.data(), n * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
             hipMemcpyAsync(ua, hu.data(), n, hipMemcpyHostToDevice, st) != hipSuccess) {
    r = SQLM_ERR_HIP;
  } else {
    // grouped send to self + receive from self (the rank-0 gather's RCCL group)
    std::vector<P2POp> ops{P2POp{0, true, a, n, SQLM_DT_F64}, P2POp{0, false, b, n, SQLM_DT_F64}};
    if (comm_group_p2p(cm, ops, st)) r = SQLM_ERR_COMM;
    if (!r && comm_bcast_dev(cm, b, n, SQLM_DT_F64, 0, st)) r = SQLM_ERR_COMM;
    if (!r && comm_allreduce_dev(cm, a, n, SQLM_DT_F64, SQLM_OP_SUM, st)) r = SQLM_ERR_COMM;
    if (!r && comm_allreduce_dev(cm, a, n, SQLM_DT_F64, SQLM_OP_MAX, st)) r = SQLM_ERR_COMM;
    if (!r && comm_allreduce_dev(cm, ia, n, SQLM_DT_I32, SQLM_OP_SUM, st)) r = SQLM_ERR_COMM;
    if (!r && comm_allreduce_dev(cm, ua, n, SQLM_DT_U8, SQLM_OP_MAX, st)) r = SQLM_ERR_COMM;
    double hs = 2.5;  // host-buffer all-reduce (setup-time exchanges)
    if (!r && comm_allreduce_host(cm, &hs, 1, SQLM_DT_F64, SQLM_OP_SUM, st)) r = SQLM_ERR_COMM;
    if (!r) upd(hs - 2.5);
    std::vector<double> ra(n), rb(n);
    std::vector<int32_t> ri(n);
    std::vector<uint8_t> ru(n);
    if (!r && (hipMemcpyAsync(ra.data(), a, n * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
               hipMemcpyAsync(rb.data(), b, n * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
               hipMemcpyAsync(ri.data(), ia, n * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
               hipMemcpyAsync(ru.data(), ua, n, hipMemcpyDeviceToHost, st) != hipSuccess ||
               hipStreamSynchronize(st) != hipSuccess))
      r = SQLM_ERR_HIP;
    if (!r)
      for (int64_t i = 0; i < n; ++i) {
        upd(ra[i] - ha[i]);
        upd(rb[i] - ha[i]);
        upd((double)(ri[i] - hi[i]));
        upd((double)ru[i] - (double)hu[i]);
      }
  }
  if (st) (void)hipStreamSynchronize(st);
  (void)hipFree(a);
  (void)hipFree(b);
  (void)hipFree(ia);
  (void)hipFree(ua);
  if (st) (void)hipStreamDestroy(st);
  comm_destroy(cm);
  *max_err = err;
  return r;
}

int sqlm_bench_iterations(sqlm_ctx *c, int warmup, int n, double *ms_per_iter, double *kernel_ms, sqlm_stats *st) {
  if (!c || !c->has_problem || n <= 0 || warmup < 0) return SQLM_ERR_INVALID_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return SQLM_ERR_HIP;
  // warmup from the initial state, then reset and time n iterations
  const auto q0 = c->pose_q, t0 = c->pose_t, p0 = c->pt;
  int s = prepare(c, 0);
  if (s) return s;
  if (warmup > 0) {
    s = run_lm(c, warmup, 0.0, nullptr, nullptr, nullptr, true);
    if (s) return s;
    c->pose_q = q0; c->pose_t = t0; c->pt = p0;
    s = prepare(c, 0);
    if (s) return s;
  }
  HIP_OK(hipStreamSynchronize(c->stream));
  s = comm_barrier(c->comm, c->stream);
  if (s) return s;
  c->timing = kernel_ms != nullptr;
  std::fill(c->kernel_ms_acc, c->kernel_ms_acc + SQLM_NKERNEL_TIMERS, 0.0);
  c->kernel_ms_n = 0;
  Timer t;
  s = run_lm(c, n, 0.0, nullptr, st, nullptr, true);
  HIP_OK(hipStreamSynchronize(c->stream));
  const double ms = t.ms();
  c->timing = false;
  if (s) return s;
  if (ms_per_iter) *ms_per_iter = ms / n;
  if (kernel_ms) {
    for (int i = 0; i < SQLM_NKERNEL_TIMERS; ++i)
      kernel_ms[i] = c->kernel_ms_n ? c->kernel_ms_acc[i] / c->kernel_ms_n : 0.0;
  }
  return finish(c);
}

#ifdef SQLM_TILE_PROF
// Diagnostic build only: 64 tiles x 8 phase cycle sums of k_rcs_tile.
int sqlm_debug_tile_profile(long long *out) { return sqlm::tile_profile_read(out); }
#endif

const char *sqlm_kernel_timer_name(int i) {
  return (i >= 0 && i < SQLM_NKERNEL_TIMERS) ? kTimerNames[i] : "";
}

// ---- ORB front end (include/sqrtlm_orb.h) ----
static int orb_engine(sqlm_ctx *c) {
  if (!c) return SQLM_ERR_INVALID_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return SQLM_ERR_HIP;
  if (!c->orb && !(c->orb = orb_create(c->stream))) return SQLM_ERR_OOM;
  return SQLM_OK;
}

int sqlm_orb_extract(sqlm_ctx *c, const sqlm_orb_params *p, const uint8_t *image, int w, int h, int stride,
                     sqlm_keypoint *kps, uint8_t *desc, int cap, int *n_out) {
  if (int r = orb_engine(c)) return r;
  return orb_extract(c->orb, p, image, w, h, stride, kps, desc, cap, n_out);
}

int sqlm_orb_get_level(sqlm_ctx *c, int level, uint8_t *out, int cap, int *lw, int *lh) {
  if (!c || !c->orb) return SQLM_ERR_STATE;
  if (hipSetDevice(c->device) != hipSuccess) return SQLM_ERR_HIP;
  return orb_get_level(c->orb, level, out, cap, lw, lh);
}

int sqlm_orb_match_bf(sqlm_ctx *c, const uint8_t *query, int nq, const uint8_t *train, int nt, int32_t *best_idx,
                      int32_t *best_dist, int32_t *second_dist) {
  if (int r = orb_engine(c)) return r;
  return orb_match_bf(c->orb, query, nq, train, nt, best_idx, best_dist, second_dist);
}

int sqlm_orb_search_for_init(sqlm_ctx *c, const sqlm_keypoint *k1, const uint8_t *d1, int n1, const sqlm_keypoint *k2,
                             const uint8_t *d2, int n2, const sqlm_frame_bounds *f2, float *prev, int32_t *m12,
                             int window, float nnratio, int check_ori, int *n_matches) {
  if (int r = orb_engine(c)) return r;
  return orb_search_for_init(c->orb, k1, d1, n1, k2, d2, n2, f2, prev, m12, window, nnratio, check_ori, n_matches);
}

int sqlm_orb_search_by_projection_local(sqlm_ctx *c, sqlm_orb_frame *F, const sqlm_track_point *mps,
                                        const uint8_t *mp_desc, int n_mp, float th, float nnratio, int *n_matches) {
  if (int r = orb_engine(c)) return r;
  return orb_search_by_projection_local(c->orb, F, mps, mp_desc, n_mp, th, nnratio, n_matches);
}

int sqlm_orb_search_by_projection_last(sqlm_ctx *c, sqlm_orb_frame *F, const float *Tcw, const float *Tlw,
                                       const sqlm_last_point *lp, const uint8_t *ldesc, int n_last, float th,
                                       int mono, int check_ori, int *n_matches) {
  if (int r = orb_engine(c)) return r;
  return orb_search_by_projection_last(c->orb, F, Tcw, Tlw, lp, ldesc, n_last, th, mono, check_ori, n_matches);
}

int sqlm_orb_search_by_projection_sim3(sqlm_ctx *c, sqlm_orb_frame *F, const float *Scw, const sqlm_map_point *mps,
                                       const uint8_t *mp_desc, int n, int th, int *n_matches) {
  if (int r = orb_engine(c)) return r;
  return orb_search_by_projection_sim3(c->orb, F, Scw, mps, mp_desc, n, th, n_matches);
}

int sqlm_orb_fuse(sqlm_ctx *c, const sqlm_orb_frame *F, const float *T, int sim3, const sqlm_map_point *mps,
                  const uint8_t *mp_desc, int n, float th, int32_t *fuse_idx, int *n_fused) {
  if (int r = orb_engine(c)) return r;
  return orb_fuse(c->orb, F, T, sim3, mps, mp_desc, n, th, fuse_idx, n_fused);
}

int sqlm_orb_search_by_projection_kf(sqlm_ctx *c, sqlm_orb_frame *F, const float *Tcw, const sqlm_map_point *mps,
                                     const uint8_t *mp_desc, const float *kf_angle, int n, float th, int orb_dist,
                                     int check_ori, int *n_matches) {
  if (int r = orb_engine(c)) return r;
  return orb_search_by_projection_kf(c->orb, F, Tcw, mps, mp_desc, kf_angle, n, th, orb_dist, check_ori, n_matches);
}

int sqlm_orb_search_by_sim3(sqlm_ctx *c, const sqlm_orb_frame *K1, const sqlm_orb_frame *K2, const float *T1w,
                            const float *T2w, const sqlm_map_point *mp1, const uint8_t *md1, const sqlm_map_point *mp2,
                            const uint8_t *md2, float s12, const float *R12, const float *t12, float th,
                            int32_t *matches12, int *n_found) {
  if (int r = orb_engine(c)) return r;
  return orb_search_by_sim3(c->orb, K1, K2, T1w, T2w, mp1, md1, mp2, md2, s12, R12, t12, th, matches12, n_found);
}

int sqlm_orb_search_by_bow_kf_frame(sqlm_ctx *c, const sqlm_bow_frame *KF, const sqlm_bow_frame *F, float nnratio,
                                    int check_ori, int32_t *matches, int *n_matches) {
  if (int r = orb_engine(c)) return r;
  return orb_search_by_bow_kf_frame(c->orb, KF, F, nnratio, check_ori, matches, n_matches);
}

int sqlm_orb_search_by_bow_kf_kf(sqlm_ctx *c, const sqlm_bow_frame *K1, const sqlm_bow_frame *K2, float nnratio,
                                 int check_ori, int32_t *matches12, int *n_matches) {
  if (int r = orb_engine(c)) return r;
  return orb_search_by_bow_kf_kf(c->orb, K1, K2, nnratio, check_ori, matches12, n_matches);
}

int sqlm_orb_search_for_triangulation(sqlm_ctx *c, const sqlm_bow_frame *K1, const sqlm_bow_frame *K2,
                                      const float *C1, const float *T2w, const float *cam2,
                                      const float *scale_factors2, int n_levels2, const float *F12, int only_stereo,
                                      int check_ori, int32_t *m12, int *n_matches) {
  if (int r = orb_engine(c)) return r;
  return orb_search_for_triangulation(c->orb, K1, K2, C1, T2w, cam2, scale_factors2, n_levels2, F12, only_stereo,
                                      check_ori, m12, n_matches);
}

int sqlm_orb_bench_extract(sqlm_ctx *c, const sqlm_orb_params *p, const uint8_t *image, int w, int h, int stride,
                           int reps, double *ms_per_frame, double *stage_ms) {
  if (int r = orb_engine(c)) return r;
  return orb_bench_extract(c->orb, p, image, w, h, stride, reps, ms_per_frame, stage_ms);
}

}  // extern "C"
