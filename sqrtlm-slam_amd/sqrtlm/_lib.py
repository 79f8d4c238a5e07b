"""ctypes binding of libsqrtlm.so (include/sqrtlm.h).

The library is the product: there is no CPU fallback. Importing works without
a GPU (the CPU test suite checks the exports), but creating a context on a
machine without a HIP device fails loudly with SQLM_ERR_NO_DEVICE.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# SQLM_LIB_PATH selects a diagnostic build of the same library (libsqrtlm_prof.so)
LIB_PATH = os.environ.get("SQLM_LIB_PATH", os.path.join(_HERE, "libsqrtlm.so"))
TRACE_MAX = 256
NKERNEL_TIMERS = 9

SQLM_OK = 0
STATUS = {0: "ok", -1: "invalid argument", -2: "HIP runtime error", -3: "not SPD", -4: "out of device memory",
          -5: "aborted", -6: "no HIP device", -7: "state error", -8: "unsupported problem shape", -9: "RCCL error"}

# every symbol include/sqrtlm.h declares
EXPORTS = [
    "sqlm_version", "sqlm_status_string", "sqlm_ctx_create", "sqlm_ctx_destroy", "sqlm_set_problem",
    "sqlm_set_lidar", "sqlm_set_edge_level", "sqlm_set_robust", "sqlm_set_lidar_level", "sqlm_optimize",
    "sqlm_local_ba", "sqlm_global_ba", "sqlm_get_poses", "sqlm_get_points", "sqlm_get_edge_chi2",
    "sqlm_get_edge_depth_positive", "sqlm_get_edge_level", "sqlm_pose_from_Tcw_f32", "sqlm_pose_to_Tcw_f32",
    "sqlm_comm_id_size", "sqlm_comm_get_unique_id", "sqlm_ctx_set_comm", "sqlm_ctx_set_host_comm",
    "sqlm_ctx_set_host_p2p", "sqlm_ctx_set_comm_selfloop", "sqlm_comm_selftest", "sqlm_ctx_comm_info",
    "sqlm_bench_iterations",
    "sqlm_kernel_timer_name", "sqlm_set_stereo",
    "sqlm_eg_set_problem", "sqlm_eg_optimize", "sqlm_eg_get_poses", "sqlm_eg_get_edge_chi2",
    "sqlm_eg_get_jacobians",
    "sqlm_get_rcs_layout", "sqlm_get_exec_info",
]
# every symbol include/sqrtlm_capture.h declares
CAPTURE_EXPORTS = ["sqlm_capture_write", "sqlm_capture_read", "sqlm_capture_free", "sqlm_capture_replay",
                   "sqlm_save_trajectory_kitti"]
# every symbol include/sqrtlm_orb.h declares
ORB_EXPORTS = ["sqlm_orb_extract", "sqlm_orb_get_level", "sqlm_orb_match_bf", "sqlm_orb_search_for_init",
               "sqlm_orb_search_by_projection_local", "sqlm_orb_search_by_projection_last",
               "sqlm_orb_search_by_projection_sim3", "sqlm_orb_fuse", "sqlm_orb_search_by_projection_kf",
               "sqlm_orb_search_by_sim3", "sqlm_orb_search_by_bow_kf_frame", "sqlm_orb_search_by_bow_kf_kf", "sqlm_orb_search_for_triangulation",
               "sqlm_orb_bench_extract"]


class SqlmError(RuntimeError):
    def __init__(self, status: int, what: str):
        super().__init__(f"{what}: {STATUS.get(status, status)} ({status})")
        self.status = status


class Stats(C.Structure):
    _fields_ = [
        ("iterations", C.c_int), ("trials", C.c_int), ("result", C.c_int), ("n_active_edges", C.c_int),
        ("chi2_begin", C.c_double), ("chi2_end", C.c_double), ("lambda_end", C.c_double),
        ("trace_len", C.c_int), ("trace_chi2", C.c_double * TRACE_MAX),
        ("trace_lambda", C.c_double * TRACE_MAX), ("trace_trials", C.c_int * TRACE_MAX),
        ("ms_total", C.c_double), ("ms_setup", C.c_double), ("ms_linearize", C.c_double),
        ("ms_trials", C.c_double),
    ]

    def as_dict(self) -> dict:
        n = self.trace_len
        return dict(iterations=self.iterations, trials=self.trials, result=self.result,
                    n_active_edges=self.n_active_edges, chi2_begin=self.chi2_begin, chi2_end=self.chi2_end,
                    lambda_end=self.lambda_end, trace_chi2=list(self.trace_chi2[:n]),
                    trace_lambda=list(self.trace_lambda[:n]), trace_trials=list(self.trace_trials[:n]),
                    ms_total=self.ms_total, ms_setup=self.ms_setup, ms_linearize=self.ms_linearize,
                    ms_trials=self.ms_trials)


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: build it with __graft_entry__.build() "
                              "(make -C sqrtlm-slam_amd/csrc); there is no CPU fallback")
        L = C.CDLL(LIB_PATH)
        L.sqlm_version.restype = C.c_char_p
        L.sqlm_status_string.restype = C.c_char_p
        L.sqlm_kernel_timer_name.restype = C.c_char_p
        _lib = L
    return _lib


def check(status: int, what: str) -> None:
    if status != SQLM_OK:
        raise SqlmError(status, what)


# int (*sqlm_allreduce_fn)(void *user, void *buf, int64_t count, int dtype, int op)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_int)
# int (*sqlm_p2p_fn)(void *user, void *buf, int64_t count, int dtype, int peer, int op)
P2P_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_int)
DTYPES = {0: np.float64, 1: np.uint8, 2: np.int32}


def ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)
