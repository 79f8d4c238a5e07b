"""The CR solve's factor + elimination kernels, schedule against schedule.

k_cr_aug (the default) factors each odd superblock as an augmented blocked
Cholesky; `split` workgroups share a superblock's E / g columns and each
repeats the factorization. The split is a pure scheduling choice: with
SQLM_CR_SPLIT=1 (the fewest workgroups the columns fit in) and =15 (one column
per workgroup) the results must be bit-identical to the default.

SQLM_CR_LEGACY=1 runs the round-2 kernels (panel Cholesky, explicit Linv,
separate top kernel): a different elimination arithmetic of the same SPD
systems, so it is compared within rounding (1e-9 relative), iteration count and
trial trace equal. The settings are read once per process, hence one child
process per schedule.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[2], sys.argv[2] + '/sqrtlm-slam_amd']
from sqrtlm import synth
from sqrtlm.optimizer import Context
prob = synth.config4(scale=0.05, seed=11)
ctx = Context(0)
ctx.set_problem(prob)
n, st = ctx.global_ba(6)
q, t = ctx.poses()
np.savez(sys.argv[1], q=q, t=t, X=ctx.points(), chi2=np.asarray(st["trace_chi2"]), n=n,
         trials=np.asarray(st["trace_trials"]))
ctx.close()
"""


def _run(tmp_path, tag, env_extra):
    out = str(tmp_path / f"{tag}.npz")
    env = dict(os.environ)
    for k in ("SQLM_CR_UNFUSED", "SQLM_CR_FUSE_MIN", "SQLM_CR_LEGACY", "SQLM_CR_SPLIT"):
        env.pop(k, None)
    env.update(env_extra)
    subprocess.run([sys.executable, "-c", CHILD, out, ROOT], env=env, check=True, timeout=100)
    return np.load(out)


def _rel(a, b):
    return np.abs(a - b).max() / max(1.0, np.abs(b).max())


def test_split_bit_identical(tmp_path):
    base = _run(tmp_path, "default", {})
    for tag, env in (("min", {"SQLM_CR_SPLIT": "1"}), ("max", {"SQLM_CR_SPLIT": "15"})):
        r = _run(tmp_path, tag, env)
        assert int(r["n"]) == int(base["n"]) > 0
        for k in ("q", "t", "X", "chi2"):
            assert np.array_equal(r[k], base[k]), (tag, k)


def test_legacy_factor_agrees(tmp_path):
    base = _run(tmp_path, "default", {})
    leg = _run(tmp_path, "legacy", {"SQLM_CR_LEGACY": "1"})
    assert int(leg["n"]) == int(base["n"]) > 0
    assert np.array_equal(leg["trials"], base["trials"])
    np.testing.assert_allclose(leg["chi2"], base["chi2"], rtol=1e-9)
    for k in ("q", "t", "X"):
        assert _rel(leg[k], base[k]) < 1e-9, k
