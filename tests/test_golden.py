"""The oracle reproduces the committed golden fixtures exactly (regression pin)."""
import numpy as np
import pytest

import golden_util as G


@pytest.mark.parametrize("name", G.names())
def test_oracle_reproduces_golden(oracle, name):
    kind, prob, exp = G.load(name)
    g = oracle.OracleGraph(prob)
    if kind == "local_ba":
        ran, outl, st = g.local_ba()
        assert ran == 1
        np.testing.assert_array_equal(outl, exp["outlier"])
        np.testing.assert_array_equal(g.obs_level, exp["edge_level_out"])
        for i, s in enumerate(st):
            assert s["iterations"] == int(exp[f"pass{i}_iters"])
            np.testing.assert_array_equal(s["trace_chi2"], exp[f"pass{i}_trace_chi2"])
    else:
        n, s = g.global_ba(10)
        assert n == int(exp["pass0_iters"])
        np.testing.assert_array_equal(s["trace_chi2"], exp["pass0_trace_chi2"])
    np.testing.assert_array_equal(g.pose_q, exp["out_pose_q"])
    np.testing.assert_array_equal(g.pose_t, exp["out_pose_t"])
    np.testing.assert_array_equal(g.pt, exp["out_pt"])


def test_golden_inputs_are_sane():
    for name in G.names():
        kind, prob, exp = G.load(name)
        assert prob.n_obs > 0 and np.all(np.isfinite(prob.obs_uv))
        assert kind in ("local_ba", "global_ba")
