"""BA problem container: the plain arrays the reference's graph builder hands
to g2o, in the layout the C-ABI (include/sqrtlm.h) takes.

Mirrors what ``g2oOptimizer::LocalBundleAdjustment`` / ``BundleAdjustment``
assemble (src/backend/g2oOptimizer.cc:805-912, :142-296):

* poses   -> ``VertexSE3Expmap`` (q = x,y,z,w ; t), ``setFixed`` flag and the
  per-keyframe intrinsics the edges copy (``e->fx = pKF->fx`` ...);
* points  -> ``VertexSBAPointXYZ`` (always marginalised);
* obs     -> ``EdgeSE3ProjectXYZ`` in insertion order (pose, point, uv,
  ``invSigma2`` information, Huber delta or 0 for "no kernel", level);
* lidar   -> ``EdgeLidarFlatPoint`` unary pose edges (g2oOptimizer.cc:1062-1070);
* stereo  -> an observation with ``obs_ur >= 0`` is an ``EdgeStereoSE3ProjectXYZ``
  (u, v, u_right; ``bf`` of its keyframe), the GBA stereo branch
  (g2oOptimizer.cc:247-281); ``obs_ur = None`` means every edge is mono.
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field

import numpy as np

# (float)sqrt(5.991) and (float)sqrt(5.99): the Huber thresholds the reference
# stores in a float before setDelta (g2oOptimizer.cc:850,902 / :163,236).
HUBER_MONO_LBA = float(np.float32(np.sqrt(5.991)))
HUBER_MONO_GBA = float(np.float32(np.sqrt(5.99)))
HUBER_STEREO = float(np.float32(np.sqrt(7.815)))  # thHuber3D (g2oOptimizer.cc:164)
CHI2_MONO = 5.991


@dataclass
class BAProblem:
    pose_q: np.ndarray          # (P,4) float64 x y z w
    pose_t: np.ndarray          # (P,3) float64
    pose_fixed: np.ndarray      # (P,)  uint8
    intr: np.ndarray            # (P,4) float64 fx fy cx cy
    pt: np.ndarray              # (L,3) float64
    obs_pose: np.ndarray        # (E,)  int32
    obs_pt: np.ndarray          # (E,)  int32
    obs_uv: np.ndarray          # (E,2) float64
    obs_info: np.ndarray        # (E,)  float64
    obs_delta: np.ndarray       # (E,)  float64, 0 = no robust kernel
    obs_level: np.ndarray       # (E,)  uint8
    lid_pose: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))
    lid_pc: np.ndarray = field(default_factory=lambda: np.zeros((0, 3)))
    lid_pw: np.ndarray = field(default_factory=lambda: np.zeros((0, 3)))
    lid_n: np.ndarray = field(default_factory=lambda: np.zeros((0, 3)))
    lid_info: np.ndarray = field(default_factory=lambda: np.zeros(0))
    obs_ur: np.ndarray | None = None    # (E,) float64, < 0 = mono edge
    pose_bf: np.ndarray | None = None   # (P,) float64 mbf (stereo edges)
    meta: dict = field(default_factory=dict)

    def __post_init__(self):
        self.pose_q = np.ascontiguousarray(self.pose_q, np.float64).reshape(-1, 4)
        self.pose_t = np.ascontiguousarray(self.pose_t, np.float64).reshape(-1, 3)
        self.pose_fixed = np.ascontiguousarray(self.pose_fixed, np.uint8).reshape(-1)
        self.intr = np.ascontiguousarray(self.intr, np.float64).reshape(-1, 4)
        self.pt = np.ascontiguousarray(self.pt, np.float64).reshape(-1, 3)
        self.obs_pose = np.ascontiguousarray(self.obs_pose, np.int32).reshape(-1)
        self.obs_pt = np.ascontiguousarray(self.obs_pt, np.int32).reshape(-1)
        self.obs_uv = np.ascontiguousarray(self.obs_uv, np.float64).reshape(-1, 2)
        self.obs_info = np.ascontiguousarray(self.obs_info, np.float64).reshape(-1)
        self.obs_delta = np.ascontiguousarray(self.obs_delta, np.float64).reshape(-1)
        self.obs_level = np.ascontiguousarray(self.obs_level, np.uint8).reshape(-1)
        self.lid_pose = np.ascontiguousarray(self.lid_pose, np.int32).reshape(-1)
        self.lid_pc = np.ascontiguousarray(self.lid_pc, np.float64).reshape(-1, 3)
        self.lid_pw = np.ascontiguousarray(self.lid_pw, np.float64).reshape(-1, 3)
        self.lid_n = np.ascontiguousarray(self.lid_n, np.float64).reshape(-1, 3)
        self.lid_info = np.ascontiguousarray(self.lid_info, np.float64).reshape(-1)
        if self.obs_ur is not None:
            self.obs_ur = np.ascontiguousarray(self.obs_ur, np.float64).reshape(-1)
            if self.pose_bf is None:
                raise ValueError("stereo observations need pose_bf")
        if self.pose_bf is not None:
            self.pose_bf = np.ascontiguousarray(self.pose_bf, np.float64).reshape(-1)
        self.validate()

    @property
    def n_pose(self) -> int:
        return self.pose_q.shape[0]

    @property
    def n_pt(self) -> int:
        return self.pt.shape[0]

    @property
    def n_obs(self) -> int:
        return self.obs_pose.shape[0]

    @property
    def n_lid(self) -> int:
        return self.lid_pose.shape[0]

    def validate(self) -> None:
        P, L, E, K = self.n_pose, self.n_pt, self.n_obs, self.n_lid
        if not (self.pose_t.shape[0] == P and self.pose_fixed.shape[0] == P and self.intr.shape[0] == P):
            raise ValueError("pose arrays disagree in length")
        for name in ("obs_pt", "obs_uv", "obs_info", "obs_delta", "obs_level"):
            if getattr(self, name).shape[0] != E:
                raise ValueError(f"{name} has wrong length")
        if E and (self.obs_pose.min() < 0 or self.obs_pose.max() >= P):
            raise ValueError("obs_pose out of range")
        if E and (self.obs_pt.min() < 0 or self.obs_pt.max() >= L):
            raise ValueError("obs_pt out of range")
        for name in ("lid_pc", "lid_pw", "lid_n", "lid_info"):
            if getattr(self, name).shape[0] != K:
                raise ValueError(f"{name} has wrong length")
        if K and (self.lid_pose.min() < 0 or self.lid_pose.max() >= P):
            raise ValueError("lid_pose out of range")
        if self.obs_ur is not None and self.obs_ur.shape[0] != E:
            raise ValueError("obs_ur has wrong length")
        if self.pose_bf is not None and self.pose_bf.shape[0] != P:
            raise ValueError("pose_bf has wrong length")

    @property
    def has_stereo(self) -> bool:
        return self.obs_ur is not None and bool(np.any(self.obs_ur >= 0))

    def copy(self) -> "BAProblem":
        return copy.deepcopy(self)
