// sqlm_comm.h — exchange layer for landmark-sharded bundle adjustment.
//
// Each rank holds all poses and a disjoint shard of landmarks (and their
// observations). The exchange steps are:
//   setup (per optimize() call): union of the active pose set, max of the
//     S block bandwidth  -> every rank builds the same camera index and the
//     same banded S pattern;
//   per LM iteration: sum of H_pp / b_p;
//   per trial: sum of S and g, of the trial scalars (chi2, computeScale), max
//     of the landmark diagonal.
// Everything else is local. Two transports share this interface: RCCL over
// xGMI (production, one process per GPU), and a host callback (the caller's
// own collective, e.g. torch.distributed gloo) used to test the sharded
// algorithm with several ranks on one GPU.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <vector>

#include "sqlm_internal.h"
#include "../../include/sqrtlm.h"

namespace sqlm {

struct Comm {
  ncclComm_t comm = nullptr;
  sqlm_allreduce_fn host_fn = nullptr;
  void *host_user = nullptr;
  int rank = 0, nranks = 1;
  std::vector<char> stage;  // host staging for the callback transport
  bool enabled() const { return nranks > 1 && (comm != nullptr || host_fn != nullptr); }
};

inline int comm_id_size() { return (int)sizeof(ncclUniqueId); }

inline int comm_get_unique_id(char *out) {
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return -9;
  std::memcpy(out, &id, sizeof(id));
  return 0;
}

inline void comm_destroy(Comm &c) {
  if (c.comm) ncclCommDestroy(c.comm);
  c.comm = nullptr;
  c.host_fn = nullptr;
  c.host_user = nullptr;
  c.rank = 0;
  c.nranks = 1;
}

inline int comm_init(Comm &c, const char *idbytes, int rank, int nranks) {
  comm_destroy(c);
  c.rank = rank;
  c.nranks = nranks;
  if (nranks <= 1) return 0;
  ncclUniqueId id;
  std::memcpy(&id, idbytes, sizeof(id));
  if (ncclCommInitRank(&c.comm, nranks, id, rank) != ncclSuccess) {
    c.comm = nullptr;
    return -9;
  }
  return 0;
}

inline int comm_init_host(Comm &c, int rank, int nranks, sqlm_allreduce_fn fn, void *user) {
  comm_destroy(c);
  c.rank = rank;
  c.nranks = nranks;
  c.host_fn = fn;
  c.host_user = user;
  return 0;
}

inline size_t dt_size(int dt) { return dt == SQLM_DT_F64 ? 8 : dt == SQLM_DT_I32 ? 4 : 1; }

inline ncclDataType_t dt_nccl(int dt) {
  return dt == SQLM_DT_F64 ? ncclDouble : dt == SQLM_DT_I32 ? ncclInt32 : ncclUint8;
}

// In-place all-reduce of a DEVICE buffer, ordered on `st`.
inline int comm_allreduce_dev(Comm &c, void *dptr, int64_t count, int dt, int op, hipStream_t st) {
  if (!c.enabled() || count == 0) return 0;
  if (c.comm) {
    return ncclAllReduce(dptr, dptr, (size_t)count, dt_nccl(dt), op == SQLM_OP_MAX ? ncclMax : ncclSum, c.comm,
                         st) == ncclSuccess
               ? 0
               : -9;
  }
  const size_t bytes = (size_t)count * dt_size(dt);
  if (c.stage.size() < bytes) c.stage.resize(bytes);
  if (hipMemcpyAsync(c.stage.data(), dptr, bytes, hipMemcpyDeviceToHost, st) != hipSuccess) return -2;
  if (hipStreamSynchronize(st) != hipSuccess) return -2;
  if (c.host_fn(c.host_user, c.stage.data(), count, dt, op) != 0) return -9;
  if (hipMemcpyAsync(dptr, c.stage.data(), bytes, hipMemcpyHostToDevice, st) != hipSuccess) return -2;
  if (hipStreamSynchronize(st) != hipSuccess) return -2;
  return 0;
}

// In-place all-reduce of a HOST buffer (setup-time exchanges).
inline int comm_allreduce_host(Comm &c, void *hptr, int64_t count, int dt, int op, hipStream_t st) {
  if (!c.enabled() || count == 0) return 0;
  if (c.host_fn) return c.host_fn(c.host_user, hptr, count, dt, op) == 0 ? 0 : -9;
  const size_t bytes = (size_t)count * dt_size(dt);
  void *tmp = nullptr;
  if (hipMallocAsync(&tmp, bytes, st) != hipSuccess) return -2;
  int r = 0;
  if (hipMemcpyAsync(tmp, hptr, bytes, hipMemcpyHostToDevice, st) != hipSuccess) r = -2;
  if (!r) r = comm_allreduce_dev(c, tmp, count, dt, op, st);
  if (!r && hipMemcpyAsync(hptr, tmp, bytes, hipMemcpyDeviceToHost, st) != hipSuccess) r = -2;
  (void)hipFreeAsync(tmp, st);
  if (hipStreamSynchronize(st) != hipSuccess && !r) r = -2;
  return r;
}

// Sum H_pp and b_p across shards (in place), once per LM iteration.
inline int comm_allreduce_hpp(Comm &c, const DevProblem &d, hipStream_t st) {
  if (!c.enabled() || d.nP == 0) return 0;
  if (comm_allreduce_dev(c, d.Hpp, (int64_t)36 * d.nP, SQLM_DT_F64, SQLM_OP_SUM, st)) return -9;
  return comm_allreduce_dev(c, d.bp, (int64_t)8 * d.nP, SQLM_DT_F64, SQLM_OP_SUM, st);
}

// Sum the reduced camera system S (BSR upper, identical banded pattern on
// every rank) and its right-hand side g; every rank then runs the same
// deterministic solve, so dx agrees without a broadcast.
inline int comm_allreduce_rcs(Comm &c, const DevProblem &d, hipStream_t st) {
  if (!c.enabled() || d.nP == 0) return 0;
  if (comm_allreduce_dev(c, d.S, (int64_t)36 * d.nnzb, SQLM_DT_F64, SQLM_OP_SUM, st)) return -9;
  return comm_allreduce_dev(c, d.g, (int64_t)6 * d.nP, SQLM_DT_F64, SQLM_OP_SUM, st);
}

// scalars: [chi_cur, chi_new, scale] summed, [maxdiag] max.
inline int comm_allreduce_scalars(Comm &c, double *scalars, hipStream_t st) {
  if (!c.enabled()) return 0;
  if (comm_allreduce_dev(c, scalars, 3, SQLM_DT_F64, SQLM_OP_SUM, st)) return -9;
  return comm_allreduce_dev(c, scalars + kMaxDiag, 1, SQLM_DT_F64, SQLM_OP_MAX, st);
}

inline int comm_barrier(Comm &c, hipStream_t st) {
  if (!c.enabled()) return 0;
  double v = 0.0;  // a 1-element all-reduce: every rank has arrived
  return comm_allreduce_host(c, &v, 1, SQLM_DT_F64, SQLM_OP_SUM, st);
}

}  // namespace sqlm
