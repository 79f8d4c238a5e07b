"""TEST INFRASTRUCTURE — build capture files from synthetic problems and fill
their ``res_*`` sections with the CPU oracle (the checker), applying exactly
the conversions ``sqlm_capture_replay`` applies (Converter.cc:55-109 via the
oracle's restatement; LBA keeps mono edges only; points without edges are
not vertices)."""
from __future__ import annotations

import numpy as np

from sqrtlm import capture as cap_mod
from sqrtlm.problem import BAProblem


def problem_to_capture(prob: BAProblem, kind: int, oracle, *, gba_iterations: int = 10,
                       gba_robust: int = 0) -> cap_mod.Capture:
    """The float32 seam inputs a reference run would have captured for `prob`."""
    Tcw = np.stack([oracle.se3_to_Tcw_f32(prob.pose_q[p], prob.pose_t[p]) for p in range(prob.n_pose)])
    c = cap_mod.Capture(
        kind=kind, Tcw=Tcw.astype(np.float32), pose_fixed=prob.pose_fixed.copy(),
        intr=prob.intr.astype(np.float32), pt=prob.pt.astype(np.float32), obs_pose=prob.obs_pose.copy(),
        obs_pt=prob.obs_pt.copy(), obs_uv=prob.obs_uv.astype(np.float32),
        obs_inv_sigma2=prob.obs_info.astype(np.float32), obs_delta=prob.obs_delta.astype(np.float32),
        gba_iterations=gba_iterations, gba_robust=gba_robust,
        kf_id=np.arange(prob.n_pose, dtype=np.uint64), mp_id=np.arange(prob.n_pt, dtype=np.uint64) + 1000)
    if prob.obs_ur is not None:
        c.obs_ur = prob.obs_ur.astype(np.float32)
        c.bf = prob.pose_bf.astype(np.float32)
    if prob.n_lid:
        c.lid_pose, c.lid_pc, c.lid_pw = prob.lid_pose.copy(), prob.lid_pc.copy(), prob.lid_pw.copy()
        c.lid_n, c.lid_info = prob.lid_n.copy(), prob.lid_info.copy()
    return c


def capture_to_problem(c: cap_mod.Capture, oracle):
    """(problem, edge_of, pt_src): the graph sqlm_capture_replay builds."""
    lba = c.kind == cap_mod.LBA
    stereo = (c.obs_ur >= 0) if c.obs_ur is not None else np.zeros(c.n_obs, bool)
    keep = ~stereo if lba else np.ones(c.n_obs, bool)
    edge_of = np.nonzero(keep)[0]
    used = np.zeros(c.n_pt, bool)
    used[c.obs_pt[edge_of]] = True
    pt_src = np.nonzero(used)[0]
    pt_map = -np.ones(c.n_pt, np.int64)
    pt_map[pt_src] = np.arange(pt_src.size)
    q = np.zeros((c.n_pose, 4)); t = np.zeros((c.n_pose, 3))
    for p in range(c.n_pose):
        q[p], t[p] = oracle.se3_from_Tcw_f32(c.Tcw[p].reshape(-1))
    delta = np.zeros(edge_of.size)
    if c.obs_delta is not None and (lba or c.gba_robust):
        delta = c.obs_delta[edge_of].astype(np.float64)
    kw = {}
    if not lba and stereo.any():
        kw = dict(obs_ur=np.where(stereo[edge_of], c.obs_ur[edge_of].astype(np.float64), -1.0),
                  pose_bf=c.bf.astype(np.float64))
    if lba and c.n_lid:
        kw.update(lid_pose=c.lid_pose, lid_pc=c.lid_pc, lid_pw=c.lid_pw, lid_n=c.lid_n, lid_info=c.lid_info)
    prob = BAProblem(pose_q=q, pose_t=t, pose_fixed=c.pose_fixed, intr=c.intr.astype(np.float64),
                     pt=c.pt[pt_src].astype(np.float64), obs_pose=c.obs_pose[edge_of],
                     obs_pt=pt_map[c.obs_pt[edge_of]], obs_uv=c.obs_uv[edge_of].astype(np.float64),
                     obs_info=c.obs_inv_sigma2[edge_of].astype(np.float64), obs_delta=delta,
                     obs_level=np.zeros(edge_of.size, np.uint8), **kw)
    return prob, edge_of, pt_src


def oracle_results(c: cap_mod.Capture, oracle) -> cap_mod.Capture:
    """Fill res_* with the oracle's run of the captured call (what a reference
    capture would hold from the g2o backend)."""
    prob, edge_of, pt_src = capture_to_problem(c, oracle)
    g = oracle.OracleGraph(prob)
    outl = np.zeros(c.n_obs, np.uint8)
    if c.kind == cap_mod.LBA:
        _, o, _ = g.local_ba()
        outl[edge_of] = o
    else:
        g.global_ba(c.gba_iterations)
    chi = np.zeros(c.n_obs)
    chi[edge_of] = g.edge_chi2()
    c.res_Tcw = np.stack([oracle.se3_to_Tcw_f32(g.pose_q[p], g.pose_t[p]) for p in range(c.n_pose)]).astype(np.float32)
    pt = c.pt.copy()
    pt[pt_src] = g.pt.astype(np.float32)
    c.res_pt = pt
    c.res_outlier = outl
    c.res_chi2 = chi
    return c
