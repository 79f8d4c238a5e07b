"""The LoopClosing::CorrectLoop sequence on one synthetic map (stand-in for
BASELINE configs 3 and 5, whose KITTI data is not available): local BA
windows as LocalMapping runs them, the essential graph of the loop closure,
the map correction, then the loop-closed global BA.

Reference call sites: LocalBundleAdjustment (LocalMapping.cc:131, selection
g2oOptimizer.cc:709-781); OptimizeEssentialGraph (LoopClosing.cc:863,
g2oOptimizer.cc:1212-1534, point correction :1500-1530); the detached GBA
(LoopClosing.cc:877, :987-991 -> GlobalBundleAdjustemnt, bRobust = false).

Every stage hands the SAME inputs to the HIP path and to the oracle (the map
advances with the oracle's result), so each stage is a parity check of its own.
"""
from __future__ import annotations

import numpy as np

from sqrtlm import synth
from sqrtlm.problem import HUBER_MONO_GBA, HUBER_MONO_LBA, BAProblem


def sub_problem(prob: BAProblem, kfs: np.ndarray, fixed: np.ndarray, pts: np.ndarray, obs: np.ndarray,
                delta: float) -> tuple[BAProblem, np.ndarray, np.ndarray]:
    """The poses `kfs` (fixed flags `fixed`), points `pts` and observations
    `obs` of `prob` as a problem of their own (ids ascending, as g2o orders
    vertices); returns it with the maps back to `prob`'s pose / point ids."""
    pmap = -np.ones(prob.n_pose, np.int64)
    pmap[kfs] = np.arange(kfs.size)
    lmap = -np.ones(prob.n_pt, np.int64)
    lmap[pts] = np.arange(pts.size)
    sub = BAProblem(
        pose_q=prob.pose_q[kfs].copy(), pose_t=prob.pose_t[kfs].copy(), pose_fixed=fixed.astype(np.uint8),
        intr=prob.intr[kfs].copy(), pt=prob.pt[pts].copy(), obs_pose=pmap[prob.obs_pose[obs]].astype(np.int32),
        obs_pt=lmap[prob.obs_pt[obs]].astype(np.int32), obs_uv=prob.obs_uv[obs].copy(),
        obs_info=prob.obs_info[obs].copy(), obs_delta=np.full(obs.size, delta),
        obs_level=np.zeros(obs.size, np.uint8))
    if prob.obs_ur is not None and (prob.obs_ur[obs] >= 0).any():  # stereo edges travel along
        sub.obs_ur = prob.obs_ur[obs].copy()
        sub.pose_bf = prob.pose_bf[kfs].copy()
    return sub, kfs, pts


def lba_window(prob: BAProblem, alive: np.ndarray, k: int, n_cov: int = 8):
    """LocalBundleAdjustment's graph for keyframe k: k and its covisible
    keyframes (here the n_cov previous ones, which share its landmarks) are
    optimised, the other keyframes observing their points are fixed (KF 0
    always), Huber (float)sqrt(5.991) on every edge (g2oOptimizer.cc:709-912).
    Stereo observations get no edge: the reference's LBA stereo branch is
    empty (g2oOptimizer.cc:914-916), so a window holds the mono edges only
    (a vertex left without edges is not in g2o's active set)."""
    edge = alive if prob.obs_ur is None else alive & (prob.obs_ur < 0)
    local = np.arange(max(0, k - n_cov), k + 1)
    on_local = edge & np.isin(prob.obs_pose, local)
    pts = np.unique(prob.obs_pt[on_local])
    obs = np.nonzero(edge & np.isin(prob.obs_pt, pts))[0]
    kfs = np.unique(prob.obs_pose[obs])
    fixed = (~np.isin(kfs, local)) | (kfs == 0)
    return sub_problem(prob, kfs, fixed, pts, obs, HUBER_MONO_LBA) + (obs,)


def add_window_lidar(sub: BAProblem, prob: BAProblem, kfs: np.ndarray, k: int, n: int = 200) -> BAProblem:
    """Pass 3 of LocalBundleAdjustment (g2oOptimizer.cc:1034-1070): n
    EdgeLidarFlatPoint pairs on the window's current keyframe k, planes taken
    at its ground-truth pose (synth.add_lidar_flat)."""
    sub.meta = dict(gt_q=prob.meta["gt_q"][kfs], gt_t=prob.meta["gt_t"][kfs])
    return synth.add_lidar_flat(sub, int(np.searchsorted(kfs, k)), n, seed=k)


def write_back(prob: BAProblem, kfs, pts, q, t, X) -> None:
    prob.pose_q[kfs] = q
    prob.pose_t[kfs] = t
    prob.pt[pts] = X


def loop_pairs(prob: BAProblem, loop: int):
    """(first-pass keyframe, revisiting keyframe) pairs of the map's loop
    closures: the revisit segments of synth.make_problem(revisits=...), or the
    last `loop` keyframes revisiting the first ones."""
    K = prob.n_pose
    rv = prob.meta.get("revisits")
    if not rv:
        a = np.arange(loop)
        return a, K - loop + a
    first = np.ones(K, bool)
    for s0, ln, _ in rv:
        first[s0:s0 + ln] = False
    fp = np.nonzero(first)[0]  # place -> first-pass keyframe
    la, lb = [], []
    for s0, ln, p0 in rv:
        la.append(fp[p0 + np.arange(ln)])
        lb.append(s0 + np.arange(ln))
    return np.concatenate(la), np.concatenate(lb)


def essential_graph(prob: BAProblem, alive: np.ndarray, loop: int, window: int = 6, min_shared: int = 15):
    """OptimizeEssentialGraph's graph on the map's keyframes: Sim3 vertices at
    the current poses (scale 1, bFixScale: stereo), the spanning tree (i-1, i),
    covisibility edges to the previous `window` keyframes sharing >= min_shared
    landmarks, and every third loop pair of each closure (loop_pairs) measured
    from the true relative poses (what the loop detection's Sim3 gives), loop
    keyframe 0 fixed. Regular edges are measured from the current (non-corrected)
    poses."""
    K = prob.n_pose
    Siw = np.concatenate([prob.pose_q, prob.pose_t, np.ones((K, 1))], axis=1)
    obs_p, obs_l = prob.obs_pose[alive], prob.obs_pt[alive]
    order = np.argsort(obs_p, kind="stable")
    bounds = np.searchsorted(obs_p[order], np.arange(K + 1))
    sets = [np.unique(obs_l[order[bounds[i]:bounds[i + 1]]]) for i in range(K)]
    ei, ej = [], []
    for i in range(1, K):
        for j in range(max(0, i - window), i):
            if j == i - 1 or np.intersect1d(sets[i], sets[j], assume_unique=True).size >= min_shared:
                ei.append(j)
                ej.append(i)
    ei, ej = np.asarray(ei, np.int32), np.asarray(ej, np.int32)
    Sji = synth._sim3_compose(Siw[ej], synth._sim3_inv(Siw[ei]))
    gq, gt = prob.meta["gt_q"], prob.meta["gt_t"]
    Sgt = np.concatenate([gq, gt, np.ones((K, 1))], axis=1)
    la, lb = loop_pairs(prob, loop)
    la, lb = la[::3].astype(np.int32), lb[::3].astype(np.int32)
    Sji_loop = synth._sim3_compose(Sgt[lb], synth._sim3_inv(Sgt[la]))
    fixed = np.zeros(K, np.uint8)
    fixed[0] = 1
    return synth.PoseGraph(Siw=Siw, fixed=fixed, fix_scale=1, ei=np.concatenate([ei, la]),
                           ej=np.concatenate([ej, lb]), Sji=np.concatenate([Sji, Sji_loop]))


def correct_map(prob: BAProblem, alive: np.ndarray, Siw_old: np.ndarray, Siw_new: np.ndarray) -> None:
    """The map after OptimizeEssentialGraph (g2oOptimizer.cc:1480-1530): every
    keyframe takes its corrected pose, every point is moved with its reference
    keyframe (here: its first observer), X' = S_new^-1 S_old X."""
    prob.pose_q[:] = Siw_new[:, :4]
    prob.pose_t[:] = Siw_new[:, 4:7] / Siw_new[:, 7:8]
    ref = np.full(prob.n_pt, prob.n_pose, np.int64)
    np.minimum.at(ref, prob.obs_pt[alive], prob.obs_pose[alive])
    has = ref < prob.n_pose
    r = ref[has]
    Ro, Rn = synth.quat_to_mat(Siw_old[r, :4]), synth.quat_to_mat(Siw_new[r, :4])
    Xc = Siw_old[r, 7:8] * np.einsum("nij,nj->ni", Ro, prob.pt[has]) + Siw_old[r, 4:7]
    prob.pt[has] = np.einsum("nji,nj->ni", Rn, (Xc - Siw_new[r, 4:7]) / Siw_new[r, 7:8])


def gba_problem(prob: BAProblem, alive: np.ndarray) -> BAProblem:
    """GlobalBundleAdjustemnt after the loop (bRobust = false): every keyframe
    (KF 0 fixed) and every point still observed, mono and stereo edges
    (g2oOptimizer.cc:213-281)."""
    obs = np.nonzero(alive)[0]
    pts = np.unique(prob.obs_pt[obs])
    kfs = np.arange(prob.n_pose)
    sub, _, _ = sub_problem(prob, kfs, kfs == 0, pts, obs, 0.0)
    sub.obs_delta[:] = 0.0
    return sub, pts


def make_map(scale: float = 0.05, loop: int = 20, seed: int = 4) -> BAProblem:
    """A loop-closed map (config4_loop geometry), robust kernels as LBA uses them."""
    return synth.config4_loop(seed=seed, scale=scale, loop=loop)


def make_kitti00_map(seed: int = 4) -> BAProblem:
    """The KITTI-00-scale stand-in (synth.kitti00_map): 1.5k KFs, 1e5 points,
    ~1.1e6 observations (half stereo), a 40-KF re-entry and a 100-KF final revisit."""
    return synth.kitti00_map(seed=seed)


__all__ = ["lba_window", "add_window_lidar", "write_back", "loop_pairs", "essential_graph", "correct_map",
           "gba_problem", "make_map", "make_kitti00_map", "HUBER_MONO_GBA"]
