"""Essential-graph oracle: Sim3 algebra of
Thirdparty/g2o/g2o/types/sim3.h, EdgeSim3 numeric Jacobians and the LM loop,
pinned by independent checks (parity with the reference itself is unpinned,
oracle/oracle.h): exp/log inverse pairs on both branches, group identities,
numeric Jacobians against wider central differences, one LM step against
numpy-assembled dense normal equations, noise-free convergence."""
import numpy as np
import pytest

from sqrtlm import synth

pytestmark = []


@pytest.mark.parametrize("scale", [0.0, 0.3])
@pytest.mark.parametrize("rot", [1e-7, 0.4])
def test_sim3_exp_log_roundtrip(oracle, scale, rot):
    rng = np.random.default_rng(int(scale * 10 + rot * 100))
    for _ in range(10):
        u = np.concatenate([rng.normal(size=3) * rot, rng.normal(size=3), [rng.normal() * scale]])
        S = oracle.sim3_from_update(u)
        np.testing.assert_allclose(oracle.sim3_log(S), u, rtol=1e-9, atol=1e-12)


def test_sim3_group_identities(oracle):
    rng = np.random.default_rng(3)
    a = oracle.sim3_from_update(rng.normal(size=7) * 0.3)
    b = oracle.sim3_from_update(rng.normal(size=7) * 0.3)
    c = oracle.sim3_from_update(rng.normal(size=7) * 0.3)
    I = oracle.sim3_mul(a, oracle.sim3_inverse(a))
    np.testing.assert_allclose(oracle.sim3_log(I), np.zeros(7), atol=1e-12)
    ab_c = oracle.sim3_mul(oracle.sim3_mul(a, b), c)
    a_bc = oracle.sim3_mul(a, oracle.sim3_mul(b, c))
    np.testing.assert_allclose(ab_c, a_bc, rtol=1e-12, atol=1e-12)


def test_eg_numeric_jacobians_vs_wide_differences(oracle):
    rng = np.random.default_rng(5)
    for fix_scale in (0, 1):
        Si = oracle.sim3_from_update(rng.normal(size=7) * 0.5)
        Sj = oracle.sim3_from_update(rng.normal(size=7) * 0.5)
        Cm = oracle.sim3_mul(oracle.sim3_from_update(rng.normal(size=7) * 0.01), oracle.sim3_mul(Sj, oracle.sim3_inverse(Si)))
        Ji, Jj = oracle.eg_edge_jacobians(Si, Sj, Cm, fix_scale)
        h = 1e-5
        for side, J in ((0, Ji), (1, Jj)):
            for d in range(7):
                u = np.zeros(7); u[d] = h
                if fix_scale:
                    u[6] = 0.0
                P = oracle.sim3_mul(oracle.sim3_from_update(u), Si if side == 0 else Sj)
                M = oracle.sim3_mul(oracle.sim3_from_update(-u), Si if side == 0 else Sj)
                ep = oracle.eg_edge_error(P, Sj, Cm) if side == 0 else oracle.eg_edge_error(Si, P, Cm)
                em = oracle.eg_edge_error(M, Sj, Cm) if side == 0 else oracle.eg_edge_error(Si, M, Cm)
                np.testing.assert_allclose(J[:, d], (ep - em) / (2 * h), rtol=1e-4, atol=1e-5)
            if fix_scale:
                assert np.all(J[:, 6] == 0.0)


def test_eg_lm_step_equals_dense_normal_equations(oracle):
    pg = synth.make_pose_graph(12, window=3, n_loops=1, seed=2)
    K = pg.n_kf
    free = np.nonzero(pg.fixed == 0)[0]
    hid = -np.ones(K, int); hid[free] = np.arange(free.size)
    n = 7 * free.size
    H = np.zeros((n, n)); b = np.zeros(n)
    for e in range(pg.n_edge):
        i, j = pg.ei[e], pg.ej[e]
        err = oracle.eg_edge_error(pg.Siw[i], pg.Siw[j], pg.Sji[e])
        Ji, Jj = oracle.eg_edge_jacobians(pg.Siw[i], pg.Siw[j], pg.Sji[e], 0, hid[i] >= 0, hid[j] >= 0)
        J = np.zeros((7, n))
        if hid[i] >= 0:
            J[:, 7 * hid[i]:7 * hid[i] + 7] = Ji
        if hid[j] >= 0:
            J[:, 7 * hid[j]:7 * hid[j] + 7] = Jj
        H += J.T @ J
        b -= J.T @ err
    lam = 1e-16
    dx = np.linalg.solve(H + lam * np.eye(n), b)
    g = oracle.OracleEG(pg)
    _, st = g.optimize(1, lam)
    assert st["trace_trials"][0] == 1
    for k, p in enumerate(free):
        S1 = oracle.sim3_mul(oracle.sim3_from_update(dx[7 * k:7 * k + 7]), pg.Siw[p])
        np.testing.assert_allclose(g.Siw[p], S1, rtol=1e-7, atol=1e-8)


@pytest.mark.parametrize("fix_scale", [False, True])
def test_eg_noise_free_converges(oracle, fix_scale):
    pg = synth.make_pose_graph(60, window=3, n_loops=2, seed=7, noise=False, fix_scale=fix_scale)
    g = oracle.OracleEG(pg)
    n, st = g.optimize(20, 1e-16)
    assert st["chi2_begin"] > 1e-2 and st["chi2_end"] < 1e-16 * max(1.0, st["chi2_begin"]) + 1e-18
    gt = pg.meta["gt"]
    # poses relative to the fixed KF 0 recover the ground truth
    for p in range(pg.n_kf):
        np.testing.assert_allclose(g.Siw[p, 4:], gt[p, 4:], rtol=1e-6, atol=1e-6)


def test_shared_libm_within_one_ulp_of_glibc(oracle):
    """include/sqlm_libm.h (the sin / cos / exp / log / acos both the oracle's
    and the GPU's Sim3 code use, so their numeric Jacobians agree bit for bit)
    stays within 1 ulp of the platform libm on the arguments Sim3 exp / log
    meet and well beyond them."""
    rng = np.random.default_rng(3)
    cases = {
        "exp": np.concatenate([rng.uniform(-5, 5, 20000), rng.uniform(-1e-6, 1e-6, 500), rng.uniform(-700, 700, 2000),
                               [0.0, -0.0, 1e-300, 0.5 * np.log(2), 1.5 * np.log(2)]]),
        "log": np.concatenate([rng.uniform(0.5, 2, 20000), np.exp(rng.uniform(-700, 700, 2000)),
                               [1.0, 2.0, 1e-310, 1 - 1e-16, 1 + 2e-16]]),
        "sin": np.concatenate([rng.uniform(-4, 4, 20000), rng.uniform(-1e-9, 1e-9, 500), rng.uniform(-1e4, 1e4, 2000),
                               [0.0, np.pi, np.pi / 4, 3 * np.pi / 4]]),
        "cos": np.concatenate([rng.uniform(-4, 4, 20000), rng.uniform(-1e-9, 1e-9, 500), rng.uniform(-1e4, 1e4, 2000),
                               [0.0, np.pi, np.pi / 4, 3 * np.pi / 4]]),
        "acos": np.concatenate([rng.uniform(-1, 1, 20000), [1.0, -1.0, 0.0, 0.5, -0.5, 1 - 1e-16, 1e-17]]),
    }
    ref = {"exp": np.exp, "log": np.log, "sin": np.sin, "cos": np.cos, "acos": np.arccos}
    for fn, x in cases.items():
        y, r = oracle.libm(fn, x), ref[fn](x)
        ulp = np.abs(y.view(np.int64) - r.view(np.int64))
        assert ulp.max() <= 1, (fn, x[ulp.argmax()], y[ulp.argmax()], r[ulp.argmax()])


def test_shared_libm_trig_range_limit(oracle):
    """sqlm_sin / sqlm_cos reduce with fdlibm's medium-range algorithm only:
    within 1 ulp of glibc up to 2^20 pi/2, NaN beyond (a rotation that large is
    a wild trial step: its chi2 is NaN and the step is rejected)."""
    lim = np.ldexp(np.pi / 2, 20)
    x = np.array([np.ldexp(np.pi / 2, 19), lim * (1 - 1e-15), -lim * (1 - 1e-15), 1.3e6, -1.6e6, 12345.678])
    for fn, ref in (("sin", np.sin), ("cos", np.cos)):
        y, r = oracle.libm(fn, x), ref(x)
        ulp = np.abs(y.view(np.int64) - r.view(np.int64))
        assert ulp.max() <= 1, (fn, x[ulp.argmax()])
        big = np.array([lim * (1 + 1e-6), 2.0 ** 31, -1e9, 1e300])
        assert np.all(np.isnan(oracle.libm(fn, big))), fn


def test_glibc_build_uses_platform_libm(oracle):
    """liboracle_glibc.so really computes with glibc (orc_libm there = np's)."""
    import ctypes as C
    x = np.linspace(-3.0, 3.0, 4097)
    y = np.zeros_like(x)
    oracle.lib(glibc=True).orc_libm(2, x.ctypes.data_as(C.c_void_p), y.ctypes.data_as(C.c_void_p), x.size)
    np.testing.assert_array_equal(y, np.sin(x))


@pytest.mark.parametrize("fix_scale", [True, False])
def test_shared_libm_oracle_matches_glibc_oracle_first_iteration(oracle, fix_scale):
    """The essential-graph oracle on include/sqlm_libm.h (the GPU's libm)
    against the same restatement on glibc (the reference's libm) on the
    1,500-keyframe bench graph: the first LM iteration (lambda 1e-16, a
    Gauss-Newton step) within the north-star 1e-6, chi2 within 1e-8 -- the
    shared-libm change cannot hide a divergence from the reference's
    arithmetic (tests/test_eg_gpu.py pins the GPU to this build too).
    Free scale (monocular Sim3) is the exception the reference itself makes:
    there ONE input moved by one ulp moves the first step by 4e-4 (measured:
    the 7-DoF system of this graph is far worse conditioned), so the two libms
    are held to 10x that own spread instead (measured 8.9e-4 vs 4.3e-4); the
    fixed-scale bench graph differs by 1.0e-7."""
    pg = synth.make_pose_graph(1500, window=8, n_loops=20, seed=5, fix_scale=fix_scale)
    a, b = oracle.OracleEG(pg), oracle.OracleEG(pg, glibc=True)
    na, sa = a.optimize(1, 1e-16)
    nb, sb = b.optimize(1, 1e-16)
    assert na == nb and sa["trace_trials"] == sb["trace_trials"]

    def rel(x, y):
        return np.abs(x - y).max() / max(1.0, np.abs(y).max())

    if fix_scale:
        assert rel(a.Siw, b.Siw) < 1e-6, rel(a.Siw, b.Siw)
        assert abs(sa["chi2_end"] - sb["chi2_end"]) <= 1e-8 * sb["chi2_begin"]
    else:
        spread = 0.0
        for r, c in ((0, 4), (5, 0), (100, 2)):
            p2 = pg.copy()
            p2.Sji[r, c] = np.nextafter(p2.Sji[r, c], 1e9)
            g = oracle.OracleEG(p2)
            g.optimize(1, 1e-16)
            spread = max(spread, rel(g.Siw, a.Siw))
        assert rel(a.Siw, b.Siw) < 10.0 * spread, (rel(a.Siw, b.Siw), spread)
