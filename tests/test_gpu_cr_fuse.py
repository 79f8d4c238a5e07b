"""The CR solve's fused factor + elimination (k_cr_factor_elim) against the
separate launches (k_cr_factor + k_cr_elim_gemm), at every level.

The default runs every level fused: one workgroup per odd superblock on levels
with >= 128 of them (full-size config 4), `split` workgroups per superblock
below (each factors it redundantly and forms a share of the strips).
SQLM_CR_FUSE_MIN=1 forces one workgroup per superblock on every level of a
14-superblock system, including the last odd block, which has no right
neighbour; SQLM_CR_UNFUSED=1 runs the separate launches. All three schedules
run the same MFMA K order, so the results must be bit-identical.
The threshold is read once per process, hence one child process per schedule.
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
np.savez(sys.argv[1], q=q, t=t, X=ctx.points(), chi2=np.asarray(st["trace_chi2"]), n=n)
ctx.close()
"""


def _run(tmp_path, tag, env_extra):
    out = str(tmp_path / f"{tag}.npz")
    env = dict(os.environ)
    env.pop("SQLM_CR_UNFUSED", None)
    env.pop("SQLM_CR_FUSE_MIN", None)
    env.update(env_extra)
    subprocess.run([sys.executable, "-c", CHILD, out, ROOT], env=env, check=True, timeout=100)
    return np.load(out)


def test_fused_every_level_bit_identical(tmp_path):
    a = _run(tmp_path, "fused", {"SQLM_CR_FUSE_MIN": "1"})
    b = _run(tmp_path, "unfused", {"SQLM_CR_UNFUSED": "1"})
    c = _run(tmp_path, "split", {})
    assert int(a["n"]) == int(b["n"]) == int(c["n"]) > 0
    for k in ("q", "t", "X", "chi2"):
        assert np.array_equal(a[k], b[k]), k
        assert np.array_equal(c[k], b[k]), k
