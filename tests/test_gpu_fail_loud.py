"""The solver's bounded waits fail loudly (linear_solver_eigen.h:105-111: a
failed factorization is reported, never used; levenberg.cpp:126-127).

Every in-workgroup wait of the cyclic-reduction factor (aug::spin / spin_to)
is bounded; one that gives up marks the solve failed (flags[0] = 0) and sets
the device error word (flags[1]), which k_reduce copies into the trial's
scalars and the host turns into SQLM_ERR_HIP. libsqrtlm_tmo.so is the same
library built with -DSQLM_SPIN_FORCE_TIMEOUT: every wait reports a timeout
after it has completed, so that path runs on an otherwise correct solve. The
optimize() call must return SQLM_ERR_HIP (never a result computed from a
factor that a wait gave up on), while the product library solves the same
problem to the oracle's result.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from sqrtlm import synth

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TMO = os.path.join(ROOT, "sqrtlm-slam_amd", "sqrtlm", "libsqrtlm_tmo.so")

CHILD = r"""
import json, sys
sys.path.insert(0, sys.argv[1])
from sqrtlm import synth
from sqrtlm._lib import SqlmError
from sqrtlm.optimizer import Context
prob = synth.make_problem(28, 1400, pair_window=4, n_fixed=3, seed=128, robust=True)
out = {}
with Context(0) as ctx:
    ctx.set_problem(prob)
    try:
        n, st = ctx.optimize(0, 10)
        out = {"status": 0, "iterations": n}
    except SqlmError as e:
        out = {"status": e.status}
    out["layout"] = ctx.rcs_layout()["kind"]
print("RESULT " + json.dumps(out))
"""


def test_forced_wait_timeout_returns_hip_error(gpu_ctx, oracle):
    assert os.path.exists(TMO), "libsqrtlm_tmo.so missing: __graft_entry__.build() makes it"
    env = dict(os.environ, SQLM_LIB_PATH=TMO)
    r = subprocess.run([sys.executable, "-c", CHILD, os.path.join(ROOT, "sqrtlm-slam_amd")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")][-1]
    res = json.loads(line[len("RESULT "):])
    assert res["layout"] == "band"  # the cyclic-reduction path ran
    assert res["status"] == -2, res  # SQLM_ERR_HIP
    # the product library: same problem, solved
    prob = synth.make_problem(28, 1400, pair_window=4, n_fixed=3, seed=128, robust=True)
    ref = oracle.OracleGraph(prob)
    nr, _ = ref.optimize(0, 10)
    gpu_ctx.set_problem(prob)
    ng, _ = gpu_ctx.optimize(0, 10)
    assert ng == nr
    q, t = gpu_ctx.poses()
    assert np.abs(q - ref.pose_q).max() < 1e-6
