"""The RCCL transport of sqlm_comm.h on real hardware with one GPU.

RCCL refuses two ranks on one device, so the multi-rank algorithm is tested
through the host transport (test_gpu_sharded.py). These tests run the RCCL
code itself on a one-rank communicator:
- the exchange primitives (grouped ncclSend / ncclRecv to self, ncclBroadcast,
  ncclAllReduce sum / max over f64, i32, u8, and the host-buffer all-reduce);
- a whole global BA on the sharded code path (S pattern all-reduce, row-range
  exchange, rank-0 gather, dx broadcast, scalar all-reduces) over RCCL, which
  must give the same result as the unsharded path (g2oOptimizer.cc:80-362
  semantics are unchanged by the transport)."""
import numpy as np
import pytest

from sqrtlm import synth
from sqrtlm.optimizer import Context, comm_selftest, comm_unique_id

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("count", [1, 1000, 1 << 20])
def test_rccl_primitives_one_rank(count):
    assert comm_selftest(0, count) == 0.0


@pytest.mark.parametrize("gen", ["band", "loop"])
def test_rccl_selfloop_global_ba_matches_unsharded(gen):
    prob = synth.config4_loop(seed=4, scale=0.02) if gen == "loop" else synth.config4(seed=4, scale=0.02)
    out = []
    for selfloop in (False, True):
        with Context(0) as ctx:
            if selfloop:
                ctx.set_comm_selfloop(comm_unique_id())
            ctx.set_problem(prob)
            n, st = ctx.global_ba(10)
            q, t = ctx.poses()
            out.append((n, st, q, t, ctx.points()))
    (n0, s0, q0, t0, X0), (n1, s1, q1, t1, X1) = out
    assert n1 == n0 and s1["trace_trials"] == s0["trace_trials"]
    # the sharded path scatters the BSR S into the solver layout instead of
    # reducing straight into it: the same sums, so the same bits
    np.testing.assert_array_equal(q1, q0)
    np.testing.assert_array_equal(t1, t0)
    np.testing.assert_array_equal(X1, X0)
