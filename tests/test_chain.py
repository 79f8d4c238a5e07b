"""CorrectLoop chain (BASELINE configs 3 / 5 stand-in): LBA windows ->
essential graph -> map correction -> loop-closed GBA on one map
(tests/chain_util.py). The CPU test runs the oracle alone and checks the
workload does what the reference's loop closure is for; the GPU test hands
every stage's inputs to both paths and compares each stage like the
single-call parity tests (poses / points / Sim3 within 1e-6, equal decisions).
"""
import numpy as np
import pytest

import chain_util as CU

LBA_KFS = (60, 120, 180)


def _rel(a, b):
    return np.abs(a - b).max() / max(1.0, np.abs(b).max())


def _loop_error(prob, loop):
    """Position error of the revisiting keyframes vs ground truth (camera centres)."""
    from sqrtlm import synth
    K = prob.n_pose
    idx = np.arange(K - loop, K)

    def centres(q, t):
        R = synth.quat_to_mat(q)
        return -np.einsum("nji,nj->ni", R, t)
    c = centres(prob.pose_q[idx], prob.pose_t[idx])
    g = centres(prob.meta["gt_q"][idx], prob.meta["gt_t"][idx])
    return float(np.abs(c - g).max())


def _run_chain(oracle, gpu_ctx=None, loop=20):
    prob = CU.make_map(loop=loop)
    alive = np.ones(prob.n_obs, bool)
    out = {"lba": [], "eg": None, "gba": None}
    for k in LBA_KFS:  # LocalMapping: a local BA per new keyframe (LocalMapping.cc:131)
        sub, kfs, pts, obs = CU.lba_window(prob, alive, k)
        ref = oracle.OracleGraph(sub)
        ran, outl, st = ref.local_ba()
        rec = {"ref": (ran, outl.copy(), st, ref.pose_q.copy(), ref.pose_t.copy(), ref.pt.copy())}
        if gpu_ctx is not None:
            gpu_ctx.set_problem(sub)
            ran_g, outl_g, st_g = gpu_ctx.local_ba()
            q, t = gpu_ctx.poses()
            rec["gpu"] = (ran_g, outl_g.copy(), st_g, q, t, gpu_ctx.points())
        out["lba"].append(rec)
        CU.write_back(prob, kfs, pts, ref.pose_q, ref.pose_t, ref.pt)
        alive[obs[outl.astype(bool)]] = False  # EraseMapPointMatch / EraseObservation (:1150-1161)
    err_before = _loop_error(prob, loop)
    pg = CU.essential_graph(prob, alive, loop)  # LoopClosing.cc:863
    ref_e = oracle.OracleEG(pg)
    ne, se = ref_e.optimize(20, 1e-16)
    out["eg"] = {"ref": (ne, se, ref_e.Siw.copy())}
    if gpu_ctx is not None:
        gpu_ctx.eg_set_problem(pg)
        ng, sg = gpu_ctx.eg_optimize(20, 1e-16)
        out["eg"]["gpu"] = (ng, sg, gpu_ctx.eg_poses().copy())
    CU.correct_map(prob, alive, pg.Siw, ref_e.Siw)
    err_eg = _loop_error(prob, loop)
    gba, pts = CU.gba_problem(prob, alive)  # LoopClosing.cc:877, :987-991
    ref_g = oracle.OracleGraph(gba)
    n, st = ref_g.global_ba(10)
    out["gba"] = {"ref": (n, st, ref_g.pose_q.copy(), ref_g.pose_t.copy(), ref_g.pt.copy())}
    if gpu_ctx is not None:
        gpu_ctx.set_problem(gba)
        n_g, st_g = gpu_ctx.global_ba(10)
        q, t = gpu_ctx.poses()
        out["gba"]["gpu"] = (n_g, st_g, q, t, gpu_ctx.points(), gpu_ctx.rcs_layout())
    gba.pose_q[:], gba.pose_t[:] = ref_g.pose_q, ref_g.pose_t
    out["err"] = (err_before, err_eg, _loop_error(gba, loop) if "gt_q" in gba.meta else None)
    out["gba_problem"] = gba
    return out


def test_chain_oracle_closes_the_loop(oracle):
    """The workload itself (oracle only): every LBA window runs its three
    passes, the essential graph converges and moves the revisiting keyframes
    towards their true places, and the GBA lowers chi2 on the corrected map."""
    out = _run_chain(oracle)
    for rec in out["lba"]:
        ran, outl, st = rec["ref"][:3]
        assert ran == 1 and st[0]["iterations"] > 0
    ne, se, _ = out["eg"]["ref"]
    assert ne > 0 and se["chi2_end"] < se["chi2_begin"]
    n, st = out["gba"]["ref"][:2]
    assert n == 10 and st["trace_chi2"][-1] < st["chi2_begin"]


@pytest.mark.gpu
def test_chain_gpu_matches_oracle_every_stage(gpu_ctx, oracle):
    out = _run_chain(oracle, gpu_ctx)
    tol = 1e-6
    for rec in out["lba"]:
        ran, outl, st, q, t, X = rec["ref"]
        ran_g, outl_g, st_g, q_g, t_g, X_g = rec["gpu"]
        assert ran_g == ran and np.array_equal(outl_g, outl)
        for a, b in zip(st_g, st):
            assert a["iterations"] == b["iterations"] and a["trace_trials"] == b["trace_trials"]
            np.testing.assert_allclose(a["trace_chi2"], b["trace_chi2"], rtol=tol)
        assert np.abs(q_g - q).max() < tol and _rel(t_g, t) < tol and _rel(X_g, X) < tol
    ne, se, S = out["eg"]["ref"]
    ng, sg, S_g = out["eg"]["gpu"]
    assert abs(sg["chi2_end"] - se["chi2_end"]) <= 1e-6 * max(se["chi2_end"], 1e-12)
    assert _rel(S_g, S) < tol
    n, st, q, t, X = out["gba"]["ref"]
    n_g, st_g, q_g, t_g, X_g, lay = out["gba"]["gpu"]
    assert lay["kind"] == "band+border", lay
    assert n_g == n and st_g["trace_trials"] == st["trace_trials"]
    np.testing.assert_allclose(st_g["trace_chi2"], st["trace_chi2"], rtol=tol)
    assert np.abs(q_g - q).max() < tol and _rel(t_g, t) < tol and _rel(X_g, X) < tol


def test_kitti00_map_shape():
    """The KITTI-00-scale stand-in of tests/test_chain_kitti.py (GPU test):
    its size, the two loop closures (revisit keyframes co-observe landmarks
    with the first-pass keyframes at their places), the stereo share, and the
    odometry-drift initial error (neighbours consistent, the revisit far end
    drifted)."""
    from sqrtlm import synth
    prob = CU.make_kitti00_map()
    assert prob.n_pose == 1500 and 90_000 < prob.n_pt <= 100_000 and prob.n_obs > 1_000_000
    assert 0.4 < float((prob.obs_ur >= 0).mean()) < 0.6
    la, lb = CU.loop_pairs(prob, 0)
    assert la.size == lb.size == 140 and set(lb[:40].tolist()) == set(range(700, 740))
    # fused points: a revisit keyframe shares landmarks with its first-pass twin
    obs_p, obs_l = prob.obs_pose, prob.obs_pt
    shared = [np.intersect1d(obs_l[obs_p == a], obs_l[obs_p == b]).size for a, b in zip(la[::20], lb[::20])]
    assert min(shared) > 50, shared

    def centres(q, t):
        return -np.einsum("nji,nj->ni", synth.quat_to_mat(q), t)
    err = np.linalg.norm(centres(prob.pose_q, prob.pose_t) - centres(prob.meta["gt_q"], prob.meta["gt_t"]), axis=1)
    step = np.linalg.norm(np.diff(centres(prob.pose_q, prob.pose_t), axis=0)
                          - np.diff(centres(prob.meta["gt_q"], prob.meta["gt_t"]), axis=0), axis=1)
    assert err[0] == 0.0 and err[1400:].mean() > 0.1 and np.median(step) < 0.05
