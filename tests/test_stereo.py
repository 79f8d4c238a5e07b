"""EdgeStereoSE3ProjectXYZ in the CPU oracle.

Pins the restatement of types_six_dof_expmap.h:112-145 / .cpp:150-234 the same
way the mono edge is pinned (parity with the reference itself is unpinned,
see oracle/oracle.h): analytic Jacobians against central differences, the
float ``invz`` / float ``bf*invz`` projection, one LM step against
independently assembled dense normal equations, and noise-free convergence.
"""
import numpy as np

from sqrtlm import synth


def _rand_pose(rng):
    w = rng.normal(size=3) * 0.3
    R = synth._so3_exp(w[None])[0]
    return synth.quat_from_mat(R)[0], rng.normal(size=3)


def _proj_f64(q, t, intr, bf, X):
    """Double-precision stereo projection (what the analytic Jacobian differentiates)."""
    c = synth.quat_to_mat(q)[0] @ X + t
    u = c[0] / c[2] * intr[0] + intr[2]
    return np.array([u, c[1] / c[2] * intr[1] + intr[3], u - bf / c[2]])


def test_stereo_projection_float_quirk(oracle):
    rng = np.random.default_rng(11)
    intr = np.array(synth.KITTI_INTR)
    bf = synth.KITTI_BF
    for _ in range(50):
        q, t = _rand_pose(rng)
        X = rng.normal(size=3) * 4
        r = oracle.quat_rotate(q, X)
        c = np.array([r[0] + t[0], r[1] + t[1], r[2] + t[2]])  # SE3Quat::map, same rounding
        if c[2] <= 0.1:
            continue
        p = oracle.stereo_project(q, t, intr, bf, X)
        invz = np.float32(1.0 / c[2])  # const float invz = 1.0f/z
        u = c[0] * np.float64(invz) * intr[0] + intr[2]
        v = c[1] * np.float64(invz) * intr[1] + intr[3]
        bz = np.float32(np.float32(bf) * invz)  # float * float
        assert p[0] == u and p[1] == v and p[2] == u - np.float64(bz)


def test_stereo_jacobians_match_central_differences(oracle):
    rng = np.random.default_rng(12)
    intr = np.array(synth.KITTI_INTR)
    bf = synth.KITTI_BF
    for _ in range(20):
        q, t = _rand_pose(rng)
        R = synth.quat_to_mat(q)[0]
        Xc = np.array([rng.uniform(-3, 3), rng.uniform(-1, 1), rng.uniform(5, 30)])
        X = R.T @ (Xc - t)
        Jl, Jp = oracle.stereo_jacobians(q, t, intr, bf, X)
        # rows 0/1 are the mono Jacobian
        Ml, Mp = oracle.mono_jacobians(q, t, intr, X)
        np.testing.assert_allclose(Jl[:2], Ml, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(Jp[:2], Mp, rtol=1e-12, atol=1e-9)
        err = lambda qq, tt, XX: -_proj_f64(qq, tt, intr, bf, XX)
        h = 1e-6
        for c in range(3):
            dX = np.zeros(3); dX[c] = h
            num = (err(q, t, X + dX) - err(q, t, X - dX)) / (2 * h)
            np.testing.assert_allclose(Jl[:, c], num, rtol=1e-5, atol=1e-4)
        for c in range(6):
            d = np.zeros(6); d[c] = h
            qa, ta = oracle.se3_oplus(q, t, d)
            qb, tb = oracle.se3_oplus(q, t, -d)
            num = (err(qa, ta, X) - err(qb, tb, X)) / (2 * h)
            np.testing.assert_allclose(Jp[:, c], num, rtol=1e-5, atol=1e-3)


def _dense_normal_equations(prob, oracle):
    P, L = prob.n_pose, prob.n_pt
    free = np.nonzero(prob.pose_fixed == 0)[0]
    pidx = -np.ones(P, int); pidx[free] = np.arange(free.size)
    n = 6 * free.size + 3 * L
    H = np.zeros((n, n)); b = np.zeros(n)
    for e in range(prob.n_obs):
        p, l = prob.obs_pose[e], prob.obs_pt[e]
        st = prob.obs_ur[e] >= 0
        if st:
            Jl, Jp = oracle.stereo_jacobians(prob.pose_q[p], prob.pose_t[p], prob.intr[p], prob.pose_bf[p], prob.pt[l])
            proj = oracle.stereo_project(prob.pose_q[p], prob.pose_t[p], prob.intr[p], prob.pose_bf[p], prob.pt[l])
            r = np.array([prob.obs_uv[e, 0], prob.obs_uv[e, 1], prob.obs_ur[e]]) - proj
        else:
            Jl, Jp = oracle.mono_jacobians(prob.pose_q[p], prob.pose_t[p], prob.intr[p], prob.pt[l])
            c = synth.quat_to_mat(prob.pose_q[p])[0] @ prob.pt[l] + prob.pose_t[p]
            fx, fy, cx, cy = prob.intr[p]
            r = prob.obs_uv[e] - np.array([c[0] / c[2] * fx + cx, c[1] / c[2] * fy + cy])
        J = np.zeros((Jl.shape[0], n))
        lo = 6 * free.size + 3 * l
        J[:, lo:lo + 3] = Jl
        if pidx[p] >= 0:
            J[:, 6 * pidx[p]:6 * pidx[p] + 6] = Jp
        H += prob.obs_info[e] * J.T @ J
        b -= prob.obs_info[e] * J.T @ r
    return H, b, free


def test_stereo_lm_step_equals_dense_normal_equations(oracle):
    prob = synth.make_problem(6, 40, pair_window=3, n_fixed=1, seed=3, robust=False, outlier_frac=0.0)
    synth.add_stereo(prob, 0.6, seed=3)
    assert prob.has_stereo and np.any(prob.obs_ur < 0)
    H, b, free = _dense_normal_equations(prob, oracle)
    lam = 1e-5 * np.max(np.abs(np.diag(H)))
    dx = np.linalg.solve(H + lam * np.eye(H.shape[0]), b)
    g = oracle.OracleGraph(prob)
    n, st = g.optimize(0, 1)
    assert st["trace_trials"][0] == 1
    X1 = prob.pt + dx[6 * free.size:].reshape(-1, 3)
    np.testing.assert_allclose(g.pt, X1, rtol=0, atol=1e-9 * max(1, np.abs(X1).max()))
    for k, p in enumerate(free):
        q1, t1 = oracle.se3_oplus(prob.pose_q[p], prob.pose_t[p], dx[6 * k:6 * k + 6])
        np.testing.assert_allclose(g.pose_t[p], t1, atol=1e-9)
        np.testing.assert_allclose(g.pose_q[p], q1, atol=1e-12)


def test_noise_free_stereo_problem_converges(oracle):
    prob = synth.make_problem(10, 300, k_min=3, k_max=6, n_fixed=2, seed=5, noise=False, robust=False)
    synth.add_stereo(prob, 0.5, seed=5, noise=False)
    g = oracle.OracleGraph(prob)
    n, st = g.global_ba(30)
    # floor: float32 keypoints / u_right and the float invz of the stereo projection
    assert st["chi2_begin"] > 1e3 and st["chi2_end"] / prob.n_obs < 1e-6


def test_all_mono_ur_matches_mono_problem(oracle):
    """obs_ur < 0 everywhere gives exactly the mono result."""
    a = synth.make_problem(8, 120, k_min=2, k_max=5, n_fixed=1, seed=9)
    b = a.copy()
    b.obs_ur = -np.ones(b.n_obs)
    b.pose_bf = np.full(b.n_pose, synth.KITTI_BF)
    ga, gb = oracle.OracleGraph(a), oracle.OracleGraph(b)
    _, sa = ga.global_ba(5)
    _, sb = gb.global_ba(5)
    assert sa["trace_chi2"] == sb["trace_chi2"]
    assert np.array_equal(ga.pose_q, gb.pose_q) and np.array_equal(ga.pt, gb.pt)
