"""Host-side mirror of the reference's BA entry points, over the C ABI.

``Optimizer`` reproduces the static façade of include/backend/Optimizer.h:42-71
for the bundle-adjustment calls; each method takes the graph the reference's
``g2oOptimizer`` would have assembled (a :class:`BAProblem`) and runs the same
schedule on the MI355X through libsqrtlm.so:

* ``LocalBundleAdjustment``  -> g2oOptimizer.cc:704-1191 (3 passes, outlier tags)
* ``GlobalBundleAdjustemnt`` -> g2oOptimizer.cc:80-89 (the reference's spelling)
* ``BundleAdjustment``       -> g2oOptimizer.cc:110-362

Results are written back into the problem (poses, points) like the
reference's ``SetPose`` / ``SetWorldPos`` write-back (g2oOptimizer.cc:1167-1189).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import check, lib, ptr
from .problem import HUBER_STEREO, HUBER_MONO_GBA, BAProblem


class Context:
    """One ``sqlm_ctx``: a HIP stream + device memory on one GPU. Create one per
    calling thread (the reference runs LBA, loop closing and GBA concurrently)."""

    def __init__(self, device: int = -1):
        self._h = C.c_void_p()
        check(lib().sqlm_ctx_create(int(device), C.byref(self._h)), "sqlm_ctx_create")
        self.problem: BAProblem | None = None

    def close(self) -> None:
        if self._h:
            lib().sqlm_ctx_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ------------------------------------------------------------- graph
    def set_problem(self, p: BAProblem) -> None:
        check(lib().sqlm_set_problem(
            self._h, p.n_pose, ptr(p.pose_q), ptr(p.pose_t), ptr(p.pose_fixed), ptr(p.intr), p.n_pt, ptr(p.pt),
            C.c_int64(p.n_obs), ptr(p.obs_pose), ptr(p.obs_pt), ptr(p.obs_uv), ptr(p.obs_info), ptr(p.obs_delta),
            ptr(p.obs_level)), "sqlm_set_problem")
        if p.n_lid:
            check(lib().sqlm_set_lidar(self._h, C.c_int64(p.n_lid), ptr(p.lid_pose), ptr(p.lid_pc), ptr(p.lid_pw),
                                       ptr(p.lid_n), ptr(p.lid_info)), "sqlm_set_lidar")
        if p.obs_ur is not None:
            check(lib().sqlm_set_stereo(self._h, ptr(p.obs_ur), ptr(p.pose_bf)), "sqlm_set_stereo")
        self.problem = p

    def set_edge_level(self, level: np.ndarray) -> None:
        level = np.ascontiguousarray(level, np.uint8)
        check(lib().sqlm_set_edge_level(self._h, ptr(level)), "sqlm_set_edge_level")

    def set_robust(self, delta: np.ndarray | None) -> None:
        d = None if delta is None else np.ascontiguousarray(delta, np.float64)
        check(lib().sqlm_set_robust(self._h, ptr(d)), "sqlm_set_robust")

    def set_lidar_level(self, level: np.ndarray) -> None:
        level = np.ascontiguousarray(level, np.uint8)
        check(lib().sqlm_set_lidar_level(self._h, ptr(level)), "sqlm_set_lidar_level")

    # ------------------------------------------------------------- solve
    def optimize(self, level: int = 0, iterations: int = 10, user_lambda: float = 0.0, stop=None):
        st = _lib.Stats()
        n = C.c_int(0)
        check(lib().sqlm_optimize(self._h, int(level), int(iterations), C.c_double(user_lambda), ptr(stop),
                                  C.byref(st), C.byref(n)), "sqlm_optimize")
        return n.value, st.as_dict()

    def local_ba(self, stop=None):
        st = (_lib.Stats * 3)()
        ran = C.c_int(0)
        outl = np.zeros(self.problem.n_obs if self.problem else 0, np.uint8)
        check(lib().sqlm_local_ba(self._h, ptr(stop), ptr(outl), st, C.byref(ran)), "sqlm_local_ba")
        return ran.value, outl, [s.as_dict() for s in st]

    def global_ba(self, iterations: int, stop=None):
        st = _lib.Stats()
        n = C.c_int(0)
        check(lib().sqlm_global_ba(self._h, int(iterations), ptr(stop), C.byref(st), C.byref(n)), "sqlm_global_ba")
        return n.value, st.as_dict()

    def rcs_layout(self) -> dict:
        """The reduced-camera-system layout of the last optimize() (sqlm_get_rcs_layout)."""
        out = (C.c_int * 8)()
        check(lib().sqlm_get_rcs_layout(self._h, out), "sqlm_get_rcs_layout")
        kind = {0: "none", 1: "band", 2: "band+border", 3: "dense"}[out[0]]
        return dict(kind=kind, B=out[1], p=out[2], n=out[3], border_cams=out[4], R=out[5], n_free=out[6],
                    coupled_superblocks=out[7])

    def exec_info(self) -> dict:
        """Device paths of the last optimize() (sqlm_get_exec_info)."""
        out = (C.c_int * 8)()
        check(lib().sqlm_get_exec_info(self._h, out), "sqlm_get_exec_info")
        solve = {0: "none", 1: "cr_levels", 3: "band+border", 4: "dense"}[out[1]]
        return dict(obs_f32=bool(out[0]), solve=solve)

    def bench(self, warmup: int, n: int, timers: bool = True):
        """(ms per LM iteration, per-phase ms from HIP events or {} without
        timers, stats). timers=False runs without the phase events."""
        ms = C.c_double(0)
        kms = np.zeros(_lib.NKERNEL_TIMERS)
        st = _lib.Stats()
        check(lib().sqlm_bench_iterations(self._h, int(warmup), int(n), C.byref(ms), ptr(kms) if timers else None,
                                          C.byref(st)), "sqlm_bench_iterations")
        if not timers:
            return ms.value, {}, st.as_dict()
        names = [lib().sqlm_kernel_timer_name(i).decode() for i in range(_lib.NKERNEL_TIMERS)]
        return ms.value, dict(zip(names, kms.tolist())), st.as_dict()

    def set_comm(self, unique_id: bytes, rank: int, nranks: int) -> None:
        buf = C.create_string_buffer(unique_id, len(unique_id))
        check(lib().sqlm_ctx_set_comm(self._h, buf, int(rank), int(nranks)), "sqlm_ctx_set_comm")

    def comm_info(self) -> dict:
        """The transport the exchange runs on and the rank / rank count as
        the communicator reports them (RCCL: ncclCommUserRank / ncclCommCount)."""
        tr, r, n = C.c_int(), C.c_int(), C.c_int()
        check(lib().sqlm_ctx_comm_info(self._h, C.byref(tr), C.byref(r), C.byref(n)), "sqlm_ctx_comm_info")
        names = {0: "none", 1: "rccl", 2: "rccl-selfloop", 3: "host"}
        return {"transport": names.get(tr.value, str(tr.value)), "rank": r.value, "nranks": n.value}

    def set_comm_selfloop(self, unique_id: bytes) -> None:
        """A one-rank RCCL communicator: the sharded code path with every
        exchange through real RCCL on one GPU (sqlm_ctx_set_comm_selfloop)."""
        buf = C.create_string_buffer(unique_id, len(unique_id))
        check(lib().sqlm_ctx_set_comm_selfloop(self._h, buf), "sqlm_ctx_set_comm_selfloop")

    def set_host_comm(self, rank: int, nranks: int, allreduce, p2p) -> None:
        """Shard over host collectives: ``allreduce(arr, op)`` must reduce the
        numpy array ``arr`` in place across ranks (op "sum" or "max");
        ``p2p(arr, peer, op)`` sends ``arr`` to / receives it from ``peer``
        (op "send" / "recv") or broadcasts it in place from root ``peer``
        (op "bcast"), e.g. with torch.distributed gloo. Runs several ranks on
        one GPU (tests)."""
        ops = {0: "send", 1: "recv", 2: "bcast"}

        def _p2p(_user, buf, count, dtype, peer, op):
            try:
                dt = _lib.DTYPES[dtype]
                arr = np.ctypeslib.as_array((C.c_char * (int(count) * np.dtype(dt).itemsize)).from_address(buf))
                p2p(arr.view(dt), int(peer), ops[int(op)])
                return 0
            except Exception:  # noqa: BLE001 — never unwind through the C ABI
                import traceback
                traceback.print_exc()
                return -1
        self._host_p2p = _lib.P2P_FN(_p2p)
        check(lib().sqlm_ctx_set_host_p2p(self._h, self._host_p2p, None), "sqlm_ctx_set_host_p2p")

        def _cb(_user, buf, count, dtype, op):
            try:
                dt = _lib.DTYPES[dtype]
                arr = np.ctypeslib.as_array((C.c_char * (int(count) * np.dtype(dt).itemsize)).from_address(buf))
                allreduce(arr.view(dt), "max" if op == 1 else "sum")
                return 0
            except Exception:  # noqa: BLE001 — never unwind through the C ABI
                import traceback
                traceback.print_exc()
                return -1
        self._host_cb = _lib.ALLREDUCE_FN(_cb)  # keep alive while the context lives
        check(lib().sqlm_ctx_set_host_comm(self._h, int(rank), int(nranks), self._host_cb, None),
              "sqlm_ctx_set_host_comm")

    # ------------------------------------------------------------- results
    def poses(self):
        n = self.problem.n_pose
        q, t = np.zeros((n, 4)), np.zeros((n, 3))
        check(lib().sqlm_get_poses(self._h, ptr(q), ptr(t)), "sqlm_get_poses")
        return q, t

    def points(self):
        X = np.zeros((self.problem.n_pt, 3))
        check(lib().sqlm_get_points(self._h, ptr(X)), "sqlm_get_points")
        return X

    def edge_chi2(self):
        out = np.zeros(self.problem.n_obs)
        check(lib().sqlm_get_edge_chi2(self._h, ptr(out)), "sqlm_get_edge_chi2")
        return out

    def depth_positive(self):
        out = np.zeros(self.problem.n_obs, np.uint8)
        check(lib().sqlm_get_edge_depth_positive(self._h, ptr(out)), "sqlm_get_edge_depth_positive")
        return out

    def edge_level(self):
        out = np.zeros(self.problem.n_obs, np.uint8)
        check(lib().sqlm_get_edge_level(self._h, ptr(out)), "sqlm_get_edge_level")
        return out

    # ------------------------------------------------------------- essential graph
    def eg_set_problem(self, pg) -> None:
        """A synth.PoseGraph (Sim3 vertices, EdgeSim3 edges) -> sqlm_eg_set_problem."""
        info = None if pg.info is None else np.ascontiguousarray(pg.info.reshape(-1, 49), np.float64)
        check(lib().sqlm_eg_set_problem(self._h, pg.n_kf, ptr(pg.Siw), ptr(pg.fixed), int(pg.fix_scale),
                                        C.c_int64(pg.n_edge), ptr(pg.ei), ptr(pg.ej), ptr(pg.Sji), ptr(info)),
              "sqlm_eg_set_problem")
        self.pose_graph = pg

    def eg_optimize(self, iterations: int = 20, user_lambda: float = 1e-16, stop=None):
        st = _lib.Stats()
        n = C.c_int(0)
        check(lib().sqlm_eg_optimize(self._h, int(iterations), C.c_double(user_lambda), ptr(stop), C.byref(st),
                                     C.byref(n)), "sqlm_eg_optimize")
        return n.value, st.as_dict()

    def eg_poses(self):
        S = np.zeros((self.pose_graph.n_kf, 8))
        check(lib().sqlm_eg_get_poses(self._h, ptr(S)), "sqlm_eg_get_poses")
        return S

    def eg_edge_chi2(self):
        out = np.zeros(self.pose_graph.n_edge)
        check(lib().sqlm_eg_get_edge_chi2(self._h, ptr(out)), "sqlm_eg_get_edge_chi2")
        return out

    def eg_jacobians(self):
        """(n_edge, 2, 7, 7): d e / d S_i and d e / d S_j at the current estimates
        (sqlm_eg_get_jacobians, the optimizer's numeric Jacobians)."""
        out = np.zeros((self.pose_graph.n_edge, 2, 7, 7))
        check(lib().sqlm_eg_get_jacobians(self._h, ptr(out)), "sqlm_eg_get_jacobians")
        return out


def comm_unique_id() -> bytes:
    n = lib().sqlm_comm_id_size()
    buf = C.create_string_buffer(n)
    check(lib().sqlm_comm_get_unique_id(buf), "sqlm_comm_get_unique_id")
    return buf.raw


def comm_selftest(device: int = 0, count: int = 1 << 16) -> float:
    """sqlm_comm_selftest: the RCCL exchange primitives on a one-rank
    communicator; returns the largest deviation from the expected buffers."""
    err = C.c_double(-1.0)
    buf = C.create_string_buffer(comm_unique_id(), lib().sqlm_comm_id_size())
    check(lib().sqlm_comm_selftest(int(device), buf, C.c_int64(count), C.byref(err)), "sqlm_comm_selftest")
    return err.value


def pose_from_Tcw_f32(T):
    """Converter::toSE3Quat (src/utils/Converter.cc:55-68)."""
    q, t = np.zeros(4), np.zeros(3)
    lib().sqlm_pose_from_Tcw_f32(ptr(np.ascontiguousarray(T, np.float32).reshape(16)), ptr(q), ptr(t))
    return q, t


def pose_to_Tcw_f32(q, t):
    """Converter::toCvMat(SE3Quat) (src/utils/Converter.cc:73-79,98-109)."""
    T = np.zeros(16, np.float32)
    lib().sqlm_pose_to_Tcw_f32(ptr(np.ascontiguousarray(q, np.float64)), ptr(np.ascontiguousarray(t, np.float64)),
                               ptr(T))
    return T.reshape(4, 4)


@dataclass
class LBAResult:
    ran: bool
    outlier: np.ndarray
    stats: list


class Optimizer:
    """Static façade mirroring include/backend/Optimizer.h:42-71 (BA calls)."""

    _ctx: Context | None = None

    @classmethod
    def _context(cls, ctx):
        if ctx is not None:
            return ctx
        if cls._ctx is None:
            cls._ctx = Context()
        return cls._ctx

    @staticmethod
    def _write_back(ctx: Context, prob: BAProblem) -> None:
        q, t = ctx.poses()
        prob.pose_q[:] = q
        prob.pose_t[:] = t
        prob.pt[:] = ctx.points()

    @classmethod
    def LocalBundleAdjustment(cls, prob: BAProblem, stop_flag=None, ctx: Context | None = None) -> LBAResult:
        """Local BA on an assembled local window (g2oOptimizer.cc:704-1191).
        ``prob.obs_delta`` carries the pass-1 Huber deltas ((float)sqrt(5.991));
        LiDAR flat edges in ``prob`` join in pass 3. Outlier tags returned are
        the edges the reference erases (chi2 > 5.991 or depth <= 0)."""
        c = cls._context(ctx)
        c.set_problem(prob)
        ran, outl, st = c.local_ba(stop_flag)
        if ran:
            cls._write_back(c, prob)
        return LBAResult(bool(ran), outl, st)

    @classmethod
    def BundleAdjustment(cls, prob: BAProblem, nIterations: int = 5, stop_flag=None, nLoopKF: int = 0,
                         bRobust: bool = True, ctx: Context | None = None):
        """g2oOptimizer::BundleAdjustment (g2oOptimizer.cc:110-362): KF 0 fixed
        (caller sets pose_fixed), Huber (float)sqrt(5.99) if bRobust."""
        c = cls._context(ctx)
        stereo = prob.obs_ur >= 0 if prob.obs_ur is not None else np.zeros(prob.n_obs, bool)
        prob.obs_delta[:] = np.where(stereo, HUBER_STEREO, HUBER_MONO_GBA) if bRobust else 0.0
        c.set_problem(prob)
        n, st = c.global_ba(nIterations, stop_flag)
        cls._write_back(c, prob)
        return n, st

    @classmethod
    def GlobalBundleAdjustemnt(cls, prob: BAProblem, nIterations: int = 5, stop_flag=None, nLoopKF: int = 0,
                               bRobust: bool = True, ctx: Context | None = None):
        """g2oOptimizer::GlobalBundleAdjustemnt (g2oOptimizer.cc:80-89)."""
        return cls.BundleAdjustment(prob, nIterations, stop_flag, nLoopKF, bRobust, ctx)

    @classmethod
    def OptimizeEssentialGraph(cls, pg, ctx: Context | None = None, stop_flag=None):
        """g2oOptimizer::OptimizeEssentialGraph (g2oOptimizer.cc:1212-1534) on an
        assembled pose graph: setUserLambdaInit(1e-16), optimize(20); the
        corrected Sim3 estimates are written back into ``pg.Siw``."""
        c = cls._context(ctx)
        c.eg_set_problem(pg)
        n, st = c.eg_optimize(20, 1e-16, stop_flag)
        pg.Siw[:] = c.eg_poses()
        return n, st
