// sqlm_comm.h — RCCL (xGMI) layer for landmark-sharded bundle adjustment.
//
// Each rank holds all poses and a disjoint shard of landmarks (and their
// observations). The only exchange steps of an LM trial are sums of the
// per-shard reduced-camera-system contributions (S, g), of the per-shard
// camera Hessian blocks (H_pp, b_p, once per iteration) and of the scalar
// reductions (chi2, computeScale, max diagonal). Everything else is local.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>

#include "sqlm_internal.h"

namespace sqlm {

struct Comm {
  ncclComm_t comm = nullptr;
  int rank = 0, nranks = 1;
  bool enabled() const { return comm != nullptr && nranks > 1; }
};

inline int comm_id_size() { return (int)sizeof(ncclUniqueId); }

inline int comm_get_unique_id(char *out) {
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return -9;
  std::memcpy(out, &id, sizeof(id));
  return 0;
}

inline int comm_init(Comm &c, const char *idbytes, int rank, int nranks) {
  if (c.comm) {
    ncclCommDestroy(c.comm);
    c.comm = nullptr;
  }
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

inline void comm_destroy(Comm &c) {
  if (c.comm) ncclCommDestroy(c.comm);
  c.comm = nullptr;
}

// Sum H_pp and b_p across shards (in place), once per LM iteration.
inline int comm_allreduce_hpp(const Comm &c, const DevProblem &d, hipStream_t st) {
  if (!c.enabled() || d.nP == 0) return 0;
  if (ncclAllReduce(d.Hpp, d.Hpp, (size_t)36 * d.nP, ncclDouble, ncclSum, c.comm, st) != ncclSuccess) return -9;
  if (ncclAllReduce(d.bp, d.bp, (size_t)8 * d.nP, ncclDouble, ncclSum, c.comm, st) != ncclSuccess) return -9;
  return 0;
}

// Sum the reduced camera system S (BSR upper, identical pattern on every rank)
// and its right-hand side g. One fused buffer would save a launch; kept as two
// calls so the pattern can later be split for reduce-scatter + replicated
// factorisation of a partitioned solver.
inline int comm_allreduce_rcs(const Comm &c, const DevProblem &d, double /*lambda*/, hipStream_t st) {
  if (!c.enabled() || d.nP == 0) return 0;
  if (ncclAllReduce(d.S, d.S, (size_t)36 * d.nnzb, ncclDouble, ncclSum, c.comm, st) != ncclSuccess) return -9;
  if (ncclAllReduce(d.g, d.g, (size_t)6 * d.nP, ncclDouble, ncclSum, c.comm, st) != ncclSuccess) return -9;
  return 0;
}

// scalars: [chi_cur, chi_new, scale] summed, [maxdiag] max.
inline int comm_allreduce_scalars(const Comm &c, double *scalars, hipStream_t st) {
  if (!c.enabled()) return 0;
  if (ncclAllReduce(scalars, scalars, 3, ncclDouble, ncclSum, c.comm, st) != ncclSuccess) return -9;
  if (ncclAllReduce(scalars + kMaxDiag, scalars + kMaxDiag, 1, ncclDouble, ncclMax, c.comm, st) != ncclSuccess)
    return -9;
  return 0;
}

inline int comm_barrier(const Comm &c, hipStream_t st) {
  if (!c.enabled()) return 0;
  // a 1-element all-reduce on the stream, then wait: every rank has arrived
  double *tmp = nullptr;
  if (hipMallocAsync((void **)&tmp, sizeof(double), st) != hipSuccess) return -2;
  (void)hipMemsetAsync(tmp, 0, sizeof(double), st);
  int r = ncclAllReduce(tmp, tmp, 1, ncclDouble, ncclSum, c.comm, st) == ncclSuccess ? 0 : -9;
  (void)hipFreeAsync(tmp, st);
  if (hipStreamSynchronize(st) != hipSuccess) return -2;
  return r;
}

}  // namespace sqlm
