"""Landmark sharding for multi-GPU global BA.

Every rank holds all poses and one contiguous range of landmarks with their
observations. Landmarks are in trajectory order (sorted by first observing
keyframe, as `synth.config4` and the reference's point ids produce them), so a
contiguous range touches a contiguous band of cameras. Ranges are balanced by
observation count, the unit of the linearisation / RCS work. LiDAR unary pose
edges go to rank 0 only (the library ignores them elsewhere as well).
"""
from __future__ import annotations

import numpy as np

from .problem import BAProblem


def landmark_ranges(prob: BAProblem, world: int) -> list[tuple[int, int]]:
    """[lo, hi) landmark ranges, one per rank, balanced by observations."""
    if world <= 1:
        return [(0, prob.n_pt)]
    counts = np.bincount(prob.obs_pt, minlength=prob.n_pt)
    cum = np.cumsum(counts)
    targets = np.linspace(0, cum[-1], world + 1)[1:-1]
    cuts = [0] + [int(np.searchsorted(cum, t)) + 1 for t in targets] + [prob.n_pt]
    cuts = np.maximum.accumulate(np.minimum(cuts, prob.n_pt))
    return [(int(cuts[r]), int(cuts[r + 1])) for r in range(world)]


def shard(prob: BAProblem, rank: int, world: int) -> BAProblem:
    """The sub-problem rank `rank` optimises: all poses, its landmark range
    (re-indexed from 0), the observations of those landmarks in their original
    relative order."""
    if world <= 1:
        return prob
    lo, hi = landmark_ranges(prob, world)[rank]
    sel = (prob.obs_pt >= lo) & (prob.obs_pt < hi)
    lid = {}
    if rank == 0 and prob.n_lid:
        lid = dict(lid_pose=prob.lid_pose, lid_pc=prob.lid_pc, lid_pw=prob.lid_pw, lid_n=prob.lid_n,
                   lid_info=prob.lid_info)
    stereo = {}
    if prob.obs_ur is not None:
        stereo = dict(obs_ur=prob.obs_ur[sel], pose_bf=prob.pose_bf)
    return BAProblem(pose_q=prob.pose_q, pose_t=prob.pose_t, pose_fixed=prob.pose_fixed, intr=prob.intr,
                     pt=prob.pt[lo:hi], obs_pose=prob.obs_pose[sel], obs_pt=prob.obs_pt[sel] - lo,
                     obs_uv=prob.obs_uv[sel], obs_info=prob.obs_info[sel], obs_delta=prob.obs_delta[sel],
                     obs_level=prob.obs_level[sel], **lid, **stereo)
