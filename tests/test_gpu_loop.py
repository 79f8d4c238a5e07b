"""Loop-closed global BA on the GPU vs the oracle.

The reference runs GBA only after a loop closure (LoopClosing.cc:877,
:987-991), so its reduced camera system always couples the revisited
keyframes far off the band. g2o solves that with SimplicialLDLT + AMD
(linear_solver_eigen.h:60-75); the HIP path eliminates the loop-coupled
cameras last as a dense border (band by cyclic reduction, border Schur
complement by MFMA Cholesky). Same tolerance as the other parity tests:
identical LM decisions, estimates within 1e-6.
"""
import numpy as np
import pytest

from sqrtlm import synth

pytestmark = pytest.mark.gpu

TOL = 1e-6


def _rel(a, b):
    return np.abs(a - b).max() / max(1.0, np.abs(b).max())


def _check(ctx, ref, sg, sr, tol=TOL):
    assert sg["iterations"] == sr["iterations"]
    assert sg["trace_trials"] == sr["trace_trials"]
    np.testing.assert_allclose(sg["trace_chi2"], sr["trace_chi2"], rtol=tol)
    np.testing.assert_allclose(sg["trace_lambda"], sr["trace_lambda"], rtol=tol)
    q, t = ctx.poses()
    X = ctx.points()
    assert np.abs(q - ref.pose_q).max() < tol
    assert _rel(t, ref.pose_t) < tol
    assert _rel(X, ref.pt) < tol


@pytest.mark.parametrize("scale,loop", [(0.02, 8), (0.05, 20), (0.1, 30)])
def test_loop_gba_band_border(gpu_ctx, oracle, scale, loop):
    prob = synth.config4_loop(scale=scale, loop=loop)
    ref = oracle.OracleGraph(prob)
    nr, sr = ref.global_ba(10)
    gpu_ctx.set_problem(prob)
    ng, sg = gpu_ctx.global_ba(10)
    lay = gpu_ctx.rcs_layout()
    assert lay["kind"] == "band+border", lay
    assert 0 < lay["border_cams"] <= 2 * loop
    assert ng == nr
    _check(gpu_ctx, ref, sg, sr)


def test_loop_robust_window(gpu_ctx, oracle):
    """A robust (Huber) window whose border is a handful of cameras: rejected
    trials and re-linearization through the border path."""
    prob = synth.make_problem(60, 3000, k_min=2, k_max=10, seed=11, robust=True, loop=12, n_fixed=2)
    ref = oracle.OracleGraph(prob)
    nr, sr = ref.optimize(0, 15)
    gpu_ctx.set_problem(prob)
    ng, sg = gpu_ctx.optimize(0, 15)
    assert gpu_ctx.rcs_layout()["kind"] == "band+border"
    assert ng == nr
    _check(gpu_ctx, ref, sg, sr)


@pytest.mark.timeout(900)
def test_config4_loop_full_size(gpu_ctx, oracle):
    """Loop-closed config 4 at BASELINE size (5k poses, 500k landmarks, ~5.04M
    observations, the last 30 keyframes revisiting the first ones) through
    the whole GBA schedule, optimize(10) (g2oOptimizer.cc:300-301)."""
    prob = synth.config4_loop(seed=4)
    ref = oracle.OracleGraph(prob)
    nr, sr = ref.global_ba(10)
    gpu_ctx.set_problem(prob)
    ng, sg = gpu_ctx.global_ba(10)
    lay = gpu_ctx.rcs_layout()
    assert lay["kind"] == "band+border" and lay["border_cams"] <= 60, lay
    assert ng == nr == 10
    _check(gpu_ctx, ref, sg, sr)
