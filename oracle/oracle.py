"""TEST INFRASTRUCTURE — ctypes binding of the CPU oracle (oracle/g2o_ref.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker / CPU baseline. PARITY UNPINNED: see
oracle/oracle.h.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_LIB_OMP_PATH = os.path.join(_HERE, "_build", "liboracle_omp.so")  # all-cores variant (ORC_OMP)
_LIB_GLIBC_PATH = os.path.join(_HERE, "_build", "liboracle_glibc.so")  # EG on glibc's libm (ORC_GLIBC_LIBM)
TRACE_MAX = 256


class OrcGraph(C.Structure):
    _fields_ = [
        ("n_pose", C.c_int), ("pose_q", C.c_void_p), ("pose_t", C.c_void_p), ("pose_fixed", C.c_void_p),
        ("intr", C.c_void_p), ("n_pt", C.c_int), ("pt", C.c_void_p), ("n_obs", C.c_int64),
        ("obs_pose", C.c_void_p), ("obs_pt", C.c_void_p), ("obs_uv", C.c_void_p), ("obs_info", C.c_void_p),
        ("obs_delta", C.c_void_p), ("obs_level", C.c_void_p), ("obs_err", C.c_void_p), ("n_lid", C.c_int64),
        ("lid_pose", C.c_void_p), ("lid_pc", C.c_void_p), ("lid_pw", C.c_void_p), ("lid_n", C.c_void_p),
        ("lid_info", C.c_void_p), ("lid_level", C.c_void_p), ("lid_err", C.c_void_p),
        ("obs_ur", C.c_void_p), ("pose_bf", C.c_void_p), ("obs_err3", C.c_void_p),
    ]


class OrcStats(C.Structure):
    _fields_ = [
        ("iterations", C.c_int), ("trials", C.c_int), ("result", C.c_int), ("n_active_edges", C.c_int),
        ("chi2_begin", C.c_double), ("chi2_end", C.c_double), ("lambda_end", C.c_double),
        ("trace_len", C.c_int), ("trace_chi2", C.c_double * TRACE_MAX),
        ("trace_lambda", C.c_double * TRACE_MAX), ("trace_trials", C.c_int * TRACE_MAX),
    ]

    def as_dict(self) -> dict:
        n = self.trace_len
        return dict(iterations=self.iterations, trials=self.trials, result=self.result,
                    n_active_edges=self.n_active_edges, chi2_begin=self.chi2_begin,
                    chi2_end=self.chi2_end, lambda_end=self.lambda_end,
                    trace_chi2=list(self.trace_chi2[:n]), trace_lambda=list(self.trace_lambda[:n]),
                    trace_trials=list(self.trace_trials[:n]))


_libs = {}


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib(omp: bool = False, glibc: bool = False) -> C.CDLL:
    """The serial oracle, or (omp=True) the same restatement built with g2o's
    OpenMP loops on every core (OMP_NUM_THREADS), bit-identical results, or
    (glibc=True) the serial build whose Sim3 code calls the platform libm
    instead of include/sqlm_libm.h."""
    key = "glibc" if glibc else omp
    if key not in _libs:
        path = _LIB_GLIBC_PATH if glibc else _LIB_OMP_PATH if omp else _LIB_PATH
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.orc_optimize.restype = C.c_int
        L.orc_local_ba.restype = C.c_int
        L.orc_global_ba.restype = C.c_int
        L.orc_lidar_error.restype = C.c_double
        _libs[key] = L
    return _libs[key]


def omp_threads() -> int:
    """OpenMP threads of the all-cores build's loops (OMP_NUM_THREADS or the
    runtime's default) -- the `cores` of its labelled baseline."""
    return int(lib(True).orc_omp_threads())


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


class OracleGraph:
    """Owns numpy copies of a BAProblem and the orc_graph view over them."""

    def __init__(self, prob, omp: bool = False):
        self._omp = omp
        self.pose_q = prob.pose_q.copy()
        self.pose_t = prob.pose_t.copy()
        self.pose_fixed = prob.pose_fixed.copy()
        self.intr = prob.intr.copy()
        self.pt = prob.pt.copy()
        self.obs_pose = prob.obs_pose.copy()
        self.obs_pt = prob.obs_pt.copy()
        self.obs_uv = prob.obs_uv.copy()
        self.obs_info = prob.obs_info.copy()
        self.obs_delta = prob.obs_delta.copy()
        self.obs_level = prob.obs_level.copy()
        self.obs_err = np.zeros((prob.n_obs, 2))
        self.lid_pose = prob.lid_pose.copy()
        self.lid_pc = prob.lid_pc.copy()
        self.lid_pw = prob.lid_pw.copy()
        self.lid_n = prob.lid_n.copy()
        self.lid_info = prob.lid_info.copy()
        self.lid_level = np.zeros(prob.n_lid, np.uint8)
        self.lid_err = np.zeros(prob.n_lid)
        self.obs_ur = prob.obs_ur.copy() if prob.obs_ur is not None else None
        self.pose_bf = prob.pose_bf.copy() if prob.pose_bf is not None else None
        self.obs_err3 = np.zeros(prob.n_obs) if prob.obs_ur is not None else None
        g = OrcGraph()
        g.n_pose, g.n_pt, g.n_obs, g.n_lid = prob.n_pose, prob.n_pt, prob.n_obs, prob.n_lid
        for name in ("pose_q", "pose_t", "pose_fixed", "intr", "pt", "obs_pose", "obs_pt", "obs_uv",
                     "obs_info", "obs_delta", "obs_level", "obs_err", "lid_pose", "lid_pc", "lid_pw",
                     "lid_n", "lid_info", "lid_level", "lid_err", "obs_ur", "pose_bf", "obs_err3"):
            setattr(g, name, _p(getattr(self, name)))
        self.g = g

    def optimize(self, level=0, iterations=10, user_lambda=0.0, stop=None):
        st = OrcStats()
        n = lib(self._omp).orc_optimize(C.byref(self.g), level, iterations, C.c_double(user_lambda),
                               _p(stop), C.byref(st))
        return n, st.as_dict()

    def local_ba(self, stop=None):
        st = (OrcStats * 3)()
        outl = np.zeros(self.obs_pose.shape[0], np.uint8)
        ran = lib(self._omp).orc_local_ba(C.byref(self.g), _p(stop), _p(outl), st)
        return ran, outl, [s.as_dict() for s in st]

    def global_ba(self, iterations=10, stop=None):
        st = OrcStats()
        n = lib(self._omp).orc_global_ba(C.byref(self.g), iterations, _p(stop), C.byref(st))
        return n, st.as_dict()

    def edge_chi2(self):
        out = np.zeros(self.obs_pose.shape[0])
        lib(self._omp).orc_edge_chi2(C.byref(self.g), _p(out))
        return out

    def depth_positive(self):
        out = np.zeros(self.obs_pose.shape[0], np.uint8)
        lib(self._omp).orc_depth_positive(C.byref(self.g), _p(out))
        return out

    def compute_errors(self):
        lib(self._omp).orc_compute_mono_errors(C.byref(self.g))
        return self.obs_err


def se3_exp(upd):
    q, t = np.zeros(4), np.zeros(3)
    lib().orc_se3_exp(_p(np.ascontiguousarray(upd, np.float64)), _p(q), _p(t))
    return q, t


def se3_oplus(q, t, d):
    q = np.array(q, np.float64); t = np.array(t, np.float64)
    lib().orc_se3_oplus(_p(q), _p(t), _p(np.ascontiguousarray(d, np.float64)))
    return q, t


def mono_jacobians(q, t, intr, X):
    Jl, Jp = np.zeros(6), np.zeros(12)
    f = lambda a: _p(np.ascontiguousarray(a, np.float64))
    lib().orc_mono_jacobians(f(q), f(t), f(intr), f(X), _p(Jl), _p(Jp))
    return Jl.reshape(2, 3), Jp.reshape(2, 6)


def quat_rotate(q, v):
    o = np.zeros(3)
    f = lambda a: _p(np.ascontiguousarray(a, np.float64))
    lib().orc_quat_rotate(f(q), f(v), _p(o))
    return o


def stereo_project(q, t, intr, bf, X):
    out = np.zeros(3)
    f = lambda a: _p(np.ascontiguousarray(a, np.float64))
    lib().orc_stereo_project(f(q), f(t), f(intr), C.c_double(bf), f(X), _p(out))
    return out


def stereo_jacobians(q, t, intr, bf, X):
    Jl, Jp = np.zeros(9), np.zeros(18)
    f = lambda a: _p(np.ascontiguousarray(a, np.float64))
    lib().orc_stereo_jacobians(f(q), f(t), f(intr), C.c_double(bf), f(X), _p(Jl), _p(Jp))
    return Jl.reshape(3, 3), Jp.reshape(3, 6)


def lidar_error(q, t, pc, pw, n):
    f = lambda a: _p(np.ascontiguousarray(a, np.float64))
    return lib().orc_lidar_error(f(q), f(t), f(pc), f(pw), f(n))


def lidar_jacobian(q, t, pc, pw, n):
    J = np.zeros(6)
    f = lambda a: _p(np.ascontiguousarray(a, np.float64))
    lib().orc_lidar_jacobian(f(q), f(t), f(pc), f(pw), f(n), _p(J))
    return J


def se3_from_Tcw_f32(T):
    q, t = np.zeros(4), np.zeros(3)
    lib().orc_se3_from_Tcw_f32(_p(np.ascontiguousarray(T, np.float32)), _p(q), _p(t))
    return q, t


def se3_to_Tcw_f32(q, t):
    T = np.zeros(16, np.float32)
    f = lambda a: _p(np.ascontiguousarray(a, np.float64))
    lib().orc_se3_to_Tcw_f32(f(q), f(t), _p(T))
    return T.reshape(4, 4)


# ---------------------------------------------------------------- essential graph (eg_ref.c)

class OrcEgGraph(C.Structure):
    _fields_ = [("n_kf", C.c_int), ("Siw", C.c_void_p), ("fixed", C.c_void_p), ("fix_scale", C.c_int),
                ("n_edge", C.c_int64), ("ei", C.c_void_p), ("ej", C.c_void_p), ("Sji", C.c_void_p),
                ("info", C.c_void_p), ("err", C.c_void_p)]


class OracleEG:
    """Owns numpy copies of a synth.PoseGraph and the orc_eg_graph view."""

    def __init__(self, pg, glibc: bool = False):
        self._glibc = glibc
        self.Siw = pg.Siw.copy()
        self.fixed = pg.fixed.copy()
        self.ei, self.ej, self.Sji = pg.ei.copy(), pg.ej.copy(), pg.Sji.copy()
        self.info = None if pg.info is None else np.ascontiguousarray(pg.info.reshape(-1, 49))
        self.err = np.zeros((pg.n_edge, 7))
        g = OrcEgGraph()
        g.n_kf, g.n_edge, g.fix_scale = pg.n_kf, pg.n_edge, pg.fix_scale
        for name in ("Siw", "fixed", "ei", "ej", "Sji", "info", "err"):
            setattr(g, name, _p(getattr(self, name)))
        self.g = g

    def optimize(self, iterations=20, user_lambda=1e-16, stop=None):
        st = OrcStats()
        L = lib(glibc=self._glibc)
        L.orc_eg_optimize.restype = C.c_int
        n = L.orc_eg_optimize(C.byref(self.g), iterations, C.c_double(user_lambda), _p(stop), C.byref(st))
        return n, st.as_dict()

    def edge_chi2(self):
        if self.info is None:
            return np.einsum("ei,ei->e", self.err, self.err)
        I = self.info.reshape(-1, 7, 7)
        return np.einsum("ei,eij,ej->e", self.err, I, self.err)


def _f(a):
    return _p(np.ascontiguousarray(a, np.float64))


def sim3_from_update(u):
    S = np.zeros(8)
    lib().orc_sim3_from_update(_f(u), _p(S))
    return S


def libm(fn: str, x):
    """include/sqlm_libm.h (the bits the GPU's Sim3 code computes) on an array."""
    x = np.ascontiguousarray(x, np.float64).reshape(-1)
    y = np.zeros_like(x)
    code = {"exp": 0, "log": 1, "sin": 2, "cos": 3, "acos": 4}[fn]
    lib().orc_libm(code, _p(x), _p(y), x.size)
    return y


def sim3_log(S):
    o = np.zeros(7)
    lib().orc_sim3_log(_f(S), _p(o))
    return o


def sim3_mul(a, b):
    o = np.zeros(8)
    lib().orc_sim3_mul(_f(a), _f(b), _p(o))
    return o


def sim3_inverse(a):
    o = np.zeros(8)
    lib().orc_sim3_inverse(_f(a), _p(o))
    return o


def eg_edge_error(Si, Sj, Cm):
    e = np.zeros(7)
    lib().orc_eg_edge_error(_f(Si), _f(Sj), _f(Cm), _p(e))
    return e


def eg_edge_jacobians(Si, Sj, Cm, fix_scale=0, free_i=1, free_j=1):
    Ji, Jj = np.zeros(49), np.zeros(49)
    lib().orc_eg_edge_jacobians(_f(Si), _f(Sj), _f(Cm), int(fix_scale), int(free_i), int(free_j), _p(Ji), _p(Jj))
    return Ji.reshape(7, 7), Jj.reshape(7, 7)
