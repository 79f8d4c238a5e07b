// sqlm_comm.h — exchange layer for landmark-sharded bundle adjustment.
//
// Each rank holds all poses and a disjoint shard of landmarks (and their
// observations). The exchange steps are:
//   setup (per optimize() call): union of the active pose set, max of the
//     S block bandwidth  -> every rank builds the same camera index and the
//     same banded S pattern; every rank's nonzero S row range;
//   iteration 0: sum of the pose Hessian diagonals (lambda_0 = tau max diag);
//   per trial: gather of every rank's S / g row range to rank 0 (point-to-
//     point, all links of rank 0 in parallel), the solve on rank 0, broadcast
//     of dx (+ the solve flag); sum of the trial scalars (chi2, computeScale);
//     max of the landmark diagonal at iteration 0.
// Rank r's landmarks only touch the cameras they observe, a contiguous window
// of the trajectory, so its S rows are ~1/N of S: the gather moves each S
// entry once (an all-reduce would move it twice, zeros included).
// Everything else is local. Two transports share this interface: RCCL over
// xGMI (production, one process per GPU), and host callbacks (the caller's
// own collectives, e.g. torch.distributed gloo) used to test the sharded
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
  sqlm_p2p_fn host_p2p = nullptr;  // send / recv / broadcast for the host transport
  void *host_p2p_user = nullptr;
  int rank = 0, nranks = 1;
  bool selfloop = false;    // a one-rank RCCL communicator that still takes the sharded path (tests)
  std::vector<char> stage;  // host staging for the callback transport
  bool enabled() const { return (nranks > 1 || selfloop) && (comm != nullptr || host_fn != nullptr); }
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
  c.host_p2p = nullptr;
  c.host_p2p_user = nullptr;
  c.rank = 0;
  c.nranks = 1;
  c.selfloop = false;
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

// A one-rank RCCL communicator on which every exchange of the sharded path
// runs for real (all-reduces and broadcasts of one rank, the rank-0 gather
// with no peers): the RCCL transport exercised on a one-GPU box.
inline int comm_init_selfloop(Comm &c, const char *idbytes) {
  comm_destroy(c);
  ncclUniqueId id;
  std::memcpy(&id, idbytes, sizeof(id));
  if (ncclCommInitRank(&c.comm, 1, id, 0) != ncclSuccess) {
    c.comm = nullptr;
    return -9;
  }
  c.selfloop = true;
  return 0;
}

// transport, rank and rank count as the communicator reports them
inline int comm_info(const Comm &c, int *transport, int *rank, int *nranks) {
  if (c.comm) {
    int n = 0, r = 0;
    if (ncclCommCount(c.comm, &n) != ncclSuccess || ncclCommUserRank(c.comm, &r) != ncclSuccess) return SQLM_ERR_COMM;
    *transport = c.selfloop ? SQLM_COMM_RCCL_SELFLOOP : SQLM_COMM_RCCL;
    *rank = r;
    *nranks = n;
    return SQLM_OK;
  }
  *transport = c.host_fn ? SQLM_COMM_HOST : SQLM_COMM_NONE;
  *rank = c.rank;
  *nranks = c.nranks;
  return SQLM_OK;
}

inline int comm_init_host(Comm &c, int rank, int nranks, sqlm_allreduce_fn fn, void *user) {
  const sqlm_p2p_fn p2p = c.host_p2p;  // survives a re-init of the collective
  void *p2p_user = c.host_p2p_user;
  comm_destroy(c);
  c.host_p2p = p2p;
  c.host_p2p_user = p2p_user;
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

// scalars: [chi_cur, chi_new, scale] summed; [maxdiag] max (iteration 0 only).
inline int comm_allreduce_scalars(Comm &c, double *scalars, bool with_max, hipStream_t st) {
  if (!c.enabled()) return 0;
  if (comm_allreduce_dev(c, scalars, 3, SQLM_DT_F64, SQLM_OP_SUM, st)) return -9;
  return with_max ? comm_allreduce_dev(c, scalars + kMaxDiag, 1, SQLM_DT_F64, SQLM_OP_MAX, st) : 0;
}

// One point-to-point transfer of a DEVICE buffer.
struct P2POp {
  int peer;
  bool send;
  void *dptr;
  int64_t count;
  int dt;
};

// A group of sends / receives, ordered on `st`. RCCL: one ncclGroup (the
// transfers of rank 0 from all peers proceed in parallel over its links).
// Host transport: in list order through the p2p callback (each peer pairs its
// operations with rank 0 in the same order, so blocking transports cannot
// deadlock).
inline int comm_group_p2p(Comm &c, const std::vector<P2POp> &ops, hipStream_t st) {
  if (!c.enabled() || ops.empty()) return 0;
  if (c.comm) {
    if (ncclGroupStart() != ncclSuccess) return -9;
    int r = 0;
    for (const P2POp &o : ops) {
      if (o.count <= 0) continue;
      const ncclResult_t e = o.send ? ncclSend(o.dptr, (size_t)o.count, dt_nccl(o.dt), o.peer, c.comm, st)
                                    : ncclRecv(o.dptr, (size_t)o.count, dt_nccl(o.dt), o.peer, c.comm, st);
      if (e != ncclSuccess) r = -9;
    }
    if (ncclGroupEnd() != ncclSuccess) r = -9;
    return r;
  }
  if (!c.host_p2p) return -9;
  if (hipStreamSynchronize(st) != hipSuccess) return -2;
  for (const P2POp &o : ops) {
    if (o.count <= 0) continue;
    const size_t bytes = (size_t)o.count * dt_size(o.dt);
    if (c.stage.size() < bytes) c.stage.resize(bytes);
    if (o.send) {
      if (hipMemcpy(c.stage.data(), o.dptr, bytes, hipMemcpyDeviceToHost) != hipSuccess) return -2;
      if (c.host_p2p(c.host_p2p_user, c.stage.data(), o.count, o.dt, o.peer, SQLM_P2P_SEND) != 0) return -9;
    } else {
      if (c.host_p2p(c.host_p2p_user, c.stage.data(), o.count, o.dt, o.peer, SQLM_P2P_RECV) != 0) return -9;
      if (hipMemcpy(o.dptr, c.stage.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) return -2;
    }
  }
  return 0;
}

// In-place broadcast of a DEVICE buffer from `root`, ordered on `st`.
inline int comm_bcast_dev(Comm &c, void *dptr, int64_t count, int dt, int root, hipStream_t st) {
  if (!c.enabled() || count == 0) return 0;
  if (c.comm)
    return ncclBroadcast(dptr, dptr, (size_t)count, dt_nccl(dt), root, c.comm, st) == ncclSuccess ? 0 : -9;
  if (!c.host_p2p) return -9;
  const size_t bytes = (size_t)count * dt_size(dt);
  if (c.stage.size() < bytes) c.stage.resize(bytes);
  if (hipStreamSynchronize(st) != hipSuccess) return -2;
  if (c.rank == root && hipMemcpy(c.stage.data(), dptr, bytes, hipMemcpyDeviceToHost) != hipSuccess) return -2;
  if (c.host_p2p(c.host_p2p_user, c.stage.data(), count, dt, root, SQLM_P2P_BCAST) != 0) return -9;
  if (c.rank != root && hipMemcpy(dptr, c.stage.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) return -2;
  return 0;
}

inline int comm_barrier(Comm &c, hipStream_t st) {
  if (!c.enabled()) return 0;
  double v = 0.0;  // a 1-element all-reduce: every rank has arrived
  return comm_allreduce_host(c, &v, 1, SQLM_DT_F64, SQLM_OP_SUM, st);
}

}  // namespace sqlm
