"""Essential graph on the HIP path vs the CPU oracle
on identical seeded pose graphs.

What is compared, and why (measured):
  * one LM iteration: the whole pipeline (numeric Jacobians, assembly, dense
    Cholesky, Sim3 update) — estimates within 1e-8 relative;
  * to convergence, noise-free graphs: the same optimum within 1e-9;
  * to convergence with measurement noise: final chi2 within 1e-6 relative and
    estimates within max(1e-6, 10x the oracle's own sensitivity to a 1-ulp
    change of one measurement), measured in the test. The LM stops on
    accept/reject decisions made on chi2 differences at the numeric-Jacobian
    noise floor (central differences over 1e-9), so the last iteration can
    differ and the optimum is flat in some directions: iteration counts are
    not compared.
Problems use bFixScale = true (stereo / RGB-D, the KITTI case). With a free
scale, g2o's Sim3(update) (sim3.h:98-104, theta < 1e-5 <= |sigma|) computes
B = ((sigma^2/2 - sigma + 1) s) / sigma^3, which makes the update erratic; the
restatement reproduces it, so only the first step is compared there.
"""
import numpy as np
import pytest

from sqrtlm import synth

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return np.abs(a - b).max() / max(1.0, np.abs(b).max())


def _oracle_sensitivity(oracle, pg, iters, ref_siw):
    """Relative change of the ORACLE's own result when one edge measurement
    moves by 1 ulp: the rounding-noise floor of the reference path on this
    graph (central-difference Jacobians over delta = 1e-9 amplify last-ulp
    differences of sin / cos / exp, which the GPU's and glibc's libms have)."""
    p2 = pg.copy()
    p2.Sji[0, 4] = np.nextafter(p2.Sji[0, 4], 1e9)  # a translation component
    g = oracle.OracleEG(p2)
    g.optimize(iters, 1e-16)
    return _rel(g.Siw, ref_siw)


def _tol(oracle, pg, iters, ref_siw, cap):
    """max(1e-6, 10x the oracle's own 1-ulp sensitivity), never above `cap`
    (the fixed tolerance these tests used before): a graph whose rounding
    sensitivity reaches the cap fails instead of widening the check."""
    sens = _oracle_sensitivity(oracle, pg, iters, ref_siw)
    assert 10.0 * sens < cap, f"fixture too ill-conditioned: 1-ulp sensitivity {sens:.3e}"
    return max(1e-6, 10.0 * sens)


def _both(gpu_ctx, oracle, pg, iters):
    ref = oracle.OracleEG(pg)
    nr, sr = ref.optimize(iters, 1e-16)
    gpu_ctx.eg_set_problem(pg)
    ng, sg = gpu_ctx.eg_optimize(iters, 1e-16)
    return ref, sr, sg


@pytest.mark.parametrize("seed", [1, 2])
def test_eg_first_iteration_matches(gpu_ctx, oracle, seed):
    pg = synth.make_pose_graph(300, window=4, n_loops=3, seed=seed, fix_scale=True, rot_noise=3e-4,
                               trans_noise=5e-4)
    ref, sr, sg = _both(gpu_ctx, oracle, pg, 1)
    assert sg["trace_trials"] == sr["trace_trials"]
    assert abs(sg["chi2_end"] - sr["chi2_end"]) <= 1e-8 * sr["chi2_begin"]
    assert _rel(gpu_ctx.eg_poses(), ref.Siw) < 1e-8
    np.testing.assert_allclose(gpu_ctx.eg_edge_chi2(), ref.edge_chi2(), rtol=1e-6, atol=1e-12)


def test_eg_free_scale_first_iteration(gpu_ctx, oracle):
    pg = synth.make_pose_graph(60, window=4, n_loops=3, seed=3, noise=False, fix_scale=False)
    ref, sr, sg = _both(gpu_ctx, oracle, pg, 1)
    assert _rel(gpu_ctx.eg_poses(), ref.Siw) < _tol(oracle, pg, 1, ref.Siw, cap=1e-5)


@pytest.mark.parametrize("seed", [1, 2])
def test_eg_noise_free_same_optimum(gpu_ctx, oracle, seed):
    pg = synth.make_pose_graph(400, window=4, n_loops=3, seed=seed, noise=False, fix_scale=True)
    ref, sr, sg = _both(gpu_ctx, oracle, pg, 20)
    assert sg["chi2_end"] < 1e-18 and sr["chi2_end"] < 1e-18
    assert _rel(gpu_ctx.eg_poses(), ref.Siw) < 1e-9
    np.testing.assert_allclose(gpu_ctx.eg_poses()[:, 4:], pg.meta["gt"][:, 4:], atol=1e-6)


@pytest.mark.parametrize("seed", [1, 3])
def test_eg_noisy_same_optimum(gpu_ctx, oracle, seed):
    pg = synth.make_pose_graph(150, window=4, n_loops=3, seed=seed, fix_scale=True, rot_noise=3e-4,
                               trans_noise=5e-4)
    ref, sr, sg = _both(gpu_ctx, oracle, pg, 20)
    assert abs(sg["chi2_end"] - sr["chi2_end"]) <= 1e-6 * sr["chi2_end"]
    assert _rel(gpu_ctx.eg_poses(), ref.Siw) < _tol(oracle, pg, 20, ref.Siw, cap=1e-4)


def test_eg_facade_writes_back(gpu_ctx, oracle):
    from sqrtlm.optimizer import Optimizer
    pg = synth.make_pose_graph(60, seed=14, noise=False, fix_scale=True)
    ref = oracle.OracleEG(pg)
    ref.optimize(20, 1e-16)
    n, st = Optimizer.OptimizeEssentialGraph(pg, ctx=gpu_ctx)
    assert n > 0 and _rel(pg.Siw, ref.Siw) < 1e-9


@pytest.mark.parametrize("dense", [False, True])
def test_eg_layouts_match(gpu_ctx, oracle, monkeypatch, dense):
    """Block-arrow layout (band + loop-vertex border, the default) and the fully
    dense layout (SQLM_EG_DENSE=1) solve the same system: both match the oracle
    on graphs with many loop edges (a border of ~12 vertices) — the first step
    within 1e-8, the noise-free optimum within 1e-9, the noisy optimum like
    test_eg_noisy_same_optimum."""
    if dense:
        monkeypatch.setenv("SQLM_EG_DENSE", "1")
    kw = dict(window=6, n_loops=12, seed=7, fix_scale=True)
    pg = synth.make_pose_graph(500, rot_noise=3e-4, trans_noise=5e-4, **kw)
    ref, sr, sg = _both(gpu_ctx, oracle, pg, 1)
    assert abs(sg["chi2_end"] - sr["chi2_end"]) <= 1e-8 * sr["chi2_begin"]
    assert _rel(gpu_ctx.eg_poses(), ref.Siw) < 1e-8
    # 20 noisy iterations: the accept / reject decisions sit at the numeric-
    # Jacobian noise floor (module docstring), and this 500-keyframe graph is
    # still creeping down at iteration 20, so the end chi2 is compared at 1e-5
    ref, sr, sg = _both(gpu_ctx, oracle, pg, 20)
    assert abs(sg["chi2_end"] - sr["chi2_end"]) <= 1e-5 * sr["chi2_end"]
    assert _rel(gpu_ctx.eg_poses(), ref.Siw) < _tol(oracle, pg, 20, ref.Siw, cap=1e-4)
    pg = synth.make_pose_graph(500, noise=False, **kw)
    ref, sr, sg = _both(gpu_ctx, oracle, pg, 20)
    assert sg["chi2_end"] < 1e-18 and sr["chi2_end"] < 1e-18
    assert _rel(gpu_ctx.eg_poses(), ref.Siw) < 1e-9


def _eg_solve_once(gpu_ctx, pg, iters, env, monkeypatch):
    for k in ("SQLM_EG_CR", "SQLM_EG_DENSE"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    gpu_ctx.eg_set_problem(pg)
    n, st = gpu_ctx.eg_optimize(iters, 1e-16)
    return st, gpu_ctx.eg_poses().copy()


@pytest.mark.parametrize("n_kf,n_loops", [(12, 0), (300, 0), (500, 12), (1500, 20)])
def test_eg_cyclic_reduction_matches(gpu_ctx, oracle, monkeypatch, n_kf, n_loops):
    """Block-arrow band by cyclic reduction with the border columns as extra
    right-hand sides (the default) against the arrow Cholesky (SQLM_EG_CR=0)
    and the oracle: one band block (12 KF), no border (0 loops), borders of
    ~12 and ~20 vertices. First step within 1e-9 of the Cholesky (a different
    elimination order of the same SPD system) and within the north-star 1e-6
    of the oracle; chi2 within 1e-8."""
    pg = synth.make_pose_graph(n_kf, window=6, n_loops=n_loops, seed=9, fix_scale=True, rot_noise=3e-4,
                               trans_noise=5e-4)
    ref = oracle.OracleEG(pg)
    nr, sr = ref.optimize(1, 1e-16)
    s_cr, p_cr = _eg_solve_once(gpu_ctx, pg, 1, {}, monkeypatch)
    s_ch, p_ch = _eg_solve_once(gpu_ctx, pg, 1, {"SQLM_EG_CR": "0"}, monkeypatch)
    assert s_cr["trace_trials"] == sr["trace_trials"]
    assert abs(s_cr["chi2_end"] - sr["chi2_end"]) <= 1e-8 * sr["chi2_begin"]
    assert _rel(p_cr, p_ch) < 1e-9
    assert _rel(p_cr, ref.Siw) < 1e-6


def test_eg_cyclic_reduction_converges(gpu_ctx, oracle, monkeypatch):
    """20 iterations on a noise-free graph with loop edges: the same optimum as
    the oracle within 1e-9 (the CR path end to end, trials included)."""
    pg = synth.make_pose_graph(500, window=6, n_loops=12, seed=7, noise=False, fix_scale=True)
    ref = oracle.OracleEG(pg)
    ref.optimize(20, 1e-16)
    st, poses = _eg_solve_once(gpu_ctx, pg, 20, {}, monkeypatch)
    assert st["chi2_end"] < 1e-18
    assert _rel(poses, ref.Siw) < 1e-9


def test_eg_bench_size_first_iteration(gpu_ctx, oracle, monkeypatch):
    """The bench graph itself (1500 keyframes, 20 loop edges, block-arrow
    layout with a border): the first LM iteration (lambda 1e-16, i.e. a
    Gauss-Newton step on a 10.5k-unknown system with accumulated drift) matches
    the oracle within the north-star 1e-6 (measured 6.3e-7: the numeric
    Jacobians go through the GPU's and glibc's sin / cos / exp, whose last-ulp
    differences this nearly Gauss-Newton step amplifies), chi2 within 1e-8;
    the arrow and the dense GPU layouts agree within 1e-9 (measured 8e-11)."""
    pg = synth.make_pose_graph(1500, window=8, n_loops=20, seed=5, fix_scale=True)
    ref, sr, sg = _both(gpu_ctx, oracle, pg, 1)
    assert sg["trace_trials"] == sr["trace_trials"]
    assert abs(sg["chi2_end"] - sr["chi2_end"]) <= 1e-8 * sr["chi2_begin"]
    arrow = gpu_ctx.eg_poses().copy()
    monkeypatch.setenv("SQLM_EG_DENSE", "1")
    gpu_ctx.eg_set_problem(pg)
    gpu_ctx.eg_optimize(1, 1e-16)
    dense = gpu_ctx.eg_poses().copy()
    assert _rel(arrow, ref.Siw) < 1e-6 and _rel(dense, ref.Siw) < 1e-6
    assert _rel(arrow, dense) < 1e-9
    # and against the oracle built on glibc's sin / cos / exp / log / acos (the
    # reference's own libm; the oracle above shares the GPU's include/sqlm_libm.h)
    ref_glibc = oracle.OracleEG(pg, glibc=True)
    _, sgl = ref_glibc.optimize(1, 1e-16)
    assert sgl["trace_trials"] == sg["trace_trials"]
    assert _rel(arrow, ref_glibc.Siw) < 1e-6 and _rel(dense, ref_glibc.Siw) < 1e-6
    assert abs(sg["chi2_end"] - sgl["chi2_end"]) <= 1e-8 * sgl["chi2_begin"]


def _oracle_jacobians(oracle, pg):
    out = np.zeros((pg.n_edge, 2, 7, 7))
    for e in range(pg.n_edge):
        i, j = pg.ei[e], pg.ej[e]
        Ji, Jj = oracle.eg_edge_jacobians(pg.Siw[i], pg.Siw[j], pg.Sji[e], pg.fix_scale,
                                          int(pg.fixed[i] == 0), int(pg.fixed[j] == 0))
        out[e, 0], out[e, 1] = Ji, Jj
    return out


@pytest.mark.parametrize("fix_scale", [True, False])
def test_eg_numeric_jacobians_bitwise(gpu_ctx, oracle, fix_scale):
    """The GPU's 7x7 numeric Jacobians (the arithmetic of k_eg_linearize:
    central differences over delta = 1e-9 through oplus, base_binary_edge.hpp:
    131-205) equal the oracle's BIT FOR BIT on the 1500-keyframe bench graph:
    both sides evaluate Sim3 exp / log with include/sqlm_libm.h's sin / cos /
    exp / log / acos and IEEE + - * / sqrt without contraction."""
    pg = synth.make_pose_graph(1500, window=8, n_loops=20, seed=5, fix_scale=fix_scale)
    gpu_ctx.eg_set_problem(pg)
    Jg = gpu_ctx.eg_jacobians()
    Jo = _oracle_jacobians(oracle, pg)
    assert np.abs(Jo).max() > 0.1
    np.testing.assert_array_equal(Jg, Jo)


def test_eg_bench_size_full_schedule(gpu_ctx, oracle):
    """The bench graph through the whole optimize(20) (lambda 1e-16, the
    reference's schedule, LoopClosing.cc:863 -> g2oOptimizer.cc:1212-1534).

    1e-6 after 20 iterations is NOT a property the reference itself has on
    this graph, so it is not what is asserted: the oracle run twice, with ONE
    measurement moved by one ulp, ends up to 3e-3 apart (translations of far
    keyframes moving metres) after 2-20 iterations (measured
    below). The normal equations of this graph have a condition number of
    5.5e13 (Lanczos on the oracle's H: eigenvalues 4e-8 .. 2.2e6; rotations
    couple to world-frame translations of up to 1.5 km), so a Gauss-Newton
    step (lambda 1e-16) resolves its near-null directions only to ~kappa * eps
    = 5e-3, whichever the summation order: the second iteration's chi2 already
    moves by percents between two correct implementations. With the Jacobians bitwise
    equal (test above), what still differs is the order of the sums in H and
    in the factorization; the GPU must stay within 10x of the reference's own
    one-ulp spread (and under a 1e-2 cap), reach the same chi2 within 10x of
    the reference's own spread, and take the same first step to 1e-6."""
    pg = synth.make_pose_graph(1500, window=8, n_loops=20, seed=5, fix_scale=True)
    ref = oracle.OracleEG(pg)
    nr, sr = ref.optimize(20, 1e-16)
    gpu_ctx.eg_set_problem(pg)
    ng, sg = gpu_ctx.eg_optimize(20, 1e-16)
    assert sg["trace_trials"][0] == sr["trace_trials"][0] and min(ng, nr) >= 10
    np.testing.assert_allclose(sg["trace_chi2"][0], sr["trace_chi2"][0], rtol=1e-6)
    spread, chi_spread = 0.0, 0.0
    for r, c in ((0, 4), (5, 0)):
        p2 = pg.copy()
        p2.Sji[r, c] = np.nextafter(p2.Sji[r, c], 1e9)
        g = oracle.OracleEG(p2)
        _, s2 = g.optimize(20, 1e-16)
        spread = max(spread, _rel(g.Siw, ref.Siw))
        chi_spread = max(chi_spread, abs(s2["chi2_end"] - sr["chi2_end"]) / sr["chi2_end"])
    assert spread > 1e-5  # the reference's own rounding sensitivity on this graph
    d = _rel(gpu_ctx.eg_poses(), ref.Siw)
    print(f"eg 20 iterations: gpu {ng} it, oracle {nr} it | gpu-oracle {d:.2e}, oracle 1-ulp spread {spread:.2e} | "
          f"chi2 gpu {sg['chi2_end']:.9g} oracle {sr['chi2_end']:.9g} (1-ulp spread {chi_spread:.2e})")
    assert d < min(1e-2, 10.0 * spread)
    assert abs(sg["chi2_end"] - sr["chi2_end"]) / sr["chi2_end"] < max(1e-6, 10.0 * chi_spread)
