"""BA problem capture / replay at the Optimizer seam.

Thin ctypes view of include/sqrtlm_capture.h: files are written and parsed by
the native library (the same code the C++ adapter links), and
``replay(ctx, cap)`` runs a captured LocalBundleAdjustment / BundleAdjustment
call on the GPU with the reference's conversions (Converter.cc:55-109).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from ._lib import Stats, check, lib, ptr
from .optimizer import Context

LBA = 1
GBA = 2


class _Cap(C.Structure):
    _fields_ = [
        ("kind", C.c_uint32), ("gba_iterations", C.c_int32), ("gba_robust", C.c_uint8),
        ("n_pose", C.c_int32), ("Tcw", C.c_void_p), ("pose_fixed", C.c_void_p), ("intr", C.c_void_p),
        ("bf", C.c_void_p), ("kf_id", C.c_void_p),
        ("n_pt", C.c_int32), ("pt", C.c_void_p), ("mp_id", C.c_void_p),
        ("n_obs", C.c_int64), ("obs_pose", C.c_void_p), ("obs_pt", C.c_void_p), ("obs_uv", C.c_void_p),
        ("obs_ur", C.c_void_p), ("obs_inv_sigma2", C.c_void_p), ("obs_delta", C.c_void_p),
        ("n_lid", C.c_int64), ("lid_pose", C.c_void_p), ("lid_pc", C.c_void_p), ("lid_pw", C.c_void_p),
        ("lid_n", C.c_void_p), ("lid_info", C.c_void_p),
        ("has_result", C.c_uint8), ("res_Tcw", C.c_void_p), ("res_pt", C.c_void_p), ("res_outlier", C.c_void_p),
        ("res_chi2", C.c_void_p),
    ]


class _ReplayOut(C.Structure):
    _fields_ = [("Tcw", C.c_void_p), ("pt", C.c_void_p), ("outlier", C.c_void_p), ("chi2", C.c_void_p),
                ("stats", Stats * 3), ("ran", C.c_int)]


# (field, dtype, per-element shape, count attribute); optional arrays may be None
_ARRAYS = [
    ("Tcw", np.float32, (4, 4), "n_pose"), ("pose_fixed", np.uint8, (), "n_pose"),
    ("intr", np.float32, (4,), "n_pose"), ("bf", np.float32, (), "n_pose"), ("kf_id", np.uint64, (), "n_pose"),
    ("pt", np.float32, (3,), "n_pt"), ("mp_id", np.uint64, (), "n_pt"),
    ("obs_pose", np.int32, (), "n_obs"), ("obs_pt", np.int32, (), "n_obs"), ("obs_uv", np.float32, (2,), "n_obs"),
    ("obs_ur", np.float32, (), "n_obs"), ("obs_inv_sigma2", np.float32, (), "n_obs"),
    ("obs_delta", np.float32, (), "n_obs"),
    ("lid_pose", np.int32, (), "n_lid"), ("lid_pc", np.float64, (3,), "n_lid"), ("lid_pw", np.float64, (3,), "n_lid"),
    ("lid_n", np.float64, (3,), "n_lid"), ("lid_info", np.float64, (), "n_lid"),
    ("res_Tcw", np.float32, (4, 4), "n_pose"), ("res_pt", np.float32, (3,), "n_pt"),
    ("res_outlier", np.uint8, (), "n_obs"), ("res_chi2", np.float64, (), "n_obs"),
]


_REQUIRED = {"Tcw", "pose_fixed", "intr", "pt", "obs_pose", "obs_pt", "obs_uv", "obs_inv_sigma2"}


@dataclass
class Capture:
    """One captured seam call, in the reference's float32 input form."""
    kind: int
    Tcw: np.ndarray
    pose_fixed: np.ndarray
    intr: np.ndarray
    pt: np.ndarray
    obs_pose: np.ndarray
    obs_pt: np.ndarray
    obs_uv: np.ndarray
    obs_inv_sigma2: np.ndarray
    gba_iterations: int = 0
    gba_robust: int = 0
    bf: np.ndarray | None = None
    kf_id: np.ndarray | None = None
    mp_id: np.ndarray | None = None
    obs_ur: np.ndarray | None = None
    obs_delta: np.ndarray | None = None
    lid_pose: np.ndarray | None = None
    lid_pc: np.ndarray | None = None
    lid_pw: np.ndarray | None = None
    lid_n: np.ndarray | None = None
    lid_info: np.ndarray | None = None
    res_Tcw: np.ndarray | None = None
    res_pt: np.ndarray | None = None
    res_outlier: np.ndarray | None = None
    res_chi2: np.ndarray | None = None
    keep: list = field(default_factory=list, repr=False)

    @property
    def n_pose(self) -> int:
        return self.Tcw.shape[0]

    @property
    def n_pt(self) -> int:
        return self.pt.shape[0]

    @property
    def n_obs(self) -> int:
        return self.obs_pose.shape[0]

    @property
    def n_lid(self) -> int:
        return 0 if self.lid_pose is None else self.lid_pose.shape[0]

    @property
    def has_result(self) -> bool:
        return self.res_Tcw is not None

    def _struct(self) -> _Cap:
        c = _Cap()
        c.kind, c.gba_iterations, c.gba_robust = self.kind, self.gba_iterations, self.gba_robust
        c.n_pose, c.n_pt, c.n_obs, c.n_lid = self.n_pose, self.n_pt, self.n_obs, self.n_lid
        c.has_result = 1 if self.has_result else 0
        self.keep = []
        for name, dt, shape, _n in _ARRAYS:
            a = getattr(self, name)
            if a is not None:
                a = np.ascontiguousarray(a, dt)
                self.keep.append(a)
                setattr(c, name, a.ctypes.data_as(C.c_void_p))
        return c


def write(path: str, cap: Capture) -> None:
    st = cap._struct()
    check(lib().sqlm_capture_write(str(path).encode(), C.byref(st)), "sqlm_capture_write")


def read(path: str) -> Capture:
    L = lib()
    p = C.POINTER(_Cap)()
    check(L.sqlm_capture_read(str(path).encode(), C.byref(p)), "sqlm_capture_read")
    try:
        c = p.contents
        out = {}
        for name, dt, shape, n in _ARRAYS:
            addr = getattr(c, name)
            cnt = getattr(c, n)
            if not addr:  # optional section absent, or a required one of length 0
                out[name] = np.zeros((0,) + shape, dt) if name in _REQUIRED else None
                continue
            size = cnt * int(np.prod(shape, dtype=np.int64)) if shape else cnt
            buf = (C.c_char * (size * np.dtype(dt).itemsize)).from_address(addr)
            out[name] = np.frombuffer(bytes(buf), dt).reshape((cnt,) + shape).copy()
        return Capture(kind=c.kind, gba_iterations=c.gba_iterations, gba_robust=c.gba_robust, **out)
    finally:
        L.sqlm_capture_free(p)


def replay(ctx: Context, cap: Capture, stop=None) -> dict:
    """Run the captured call on ctx's GPU; returns the write-back in the
    reference's float form plus the per-pass stats."""
    st = cap._struct()
    o = _ReplayOut()
    Tcw = np.zeros((cap.n_pose, 4, 4), np.float32)
    pt = np.zeros((cap.n_pt, 3), np.float32)
    outl = np.zeros(cap.n_obs, np.uint8)
    chi = np.zeros(cap.n_obs)
    o.Tcw, o.pt, o.outlier, o.chi2 = ptr(Tcw), ptr(pt), ptr(outl), ptr(chi)
    check(lib().sqlm_capture_replay(ctx._h, C.byref(st), ptr(stop), C.byref(o)), "sqlm_capture_replay")
    return dict(Tcw=Tcw, pt=pt, outlier=outl, chi2=chi, ran=o.ran, stats=[s.as_dict() for s in o.stats])


def save_trajectory_kitti(path: str, Tcr, frame_ref, Tcw, Tcp, parent, bad=None, origin_kf: int = 0) -> None:
    """System::SaveTrajectoryKITTI (src/System.cc:503-560) through
    sqlm_save_trajectory_kitti: Tcr (F,4,4) frame poses relative to their
    reference keyframe frame_ref (F,), keyframe poses Tcw (K,4,4), Tcp (K,4,4)
    relative to the parent keyframe parent (K,), bad (K,) flags; float32."""
    f32 = lambda a: np.ascontiguousarray(a, np.float32).reshape(-1)  # noqa: E731
    i32 = lambda a: np.ascontiguousarray(a, np.int32)  # noqa: E731
    Tcr, Tcw, Tcp = f32(Tcr), f32(Tcw), f32(Tcp)
    fr, par = i32(frame_ref), i32(parent)
    b = None if bad is None else np.ascontiguousarray(bad, np.uint8)
    check(lib().sqlm_save_trajectory_kitti(str(path).encode(), int(fr.size), ptr(Tcr), ptr(fr), int(par.size),
                                           ptr(Tcw), ptr(Tcp), ptr(par), ptr(b) if b is not None else None,
                                           int(origin_kf)), "sqlm_save_trajectory_kitti")
