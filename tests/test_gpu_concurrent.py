"""Concurrent callers on one GPU (SURVEY.md §8b threading).

The reference runs LocalMapping (LocalBundleAdjustment, LocalMapping.cc:131),
LoopClosing (OptimizeEssentialGraph, LoopClosing.cc:863) and the detached GBA
thread (LoopClosing.cc:877, :987-991) at the same time (System.cc:144,153).
The ABI promises one context per calling thread (include/sqrtlm.h): three host
threads, each with its own sqlm_ctx (own HIP streams and buffers), run local
BA (config 2), the essential graph and a loop-closed global BA concurrently;
each result must equal, bit for bit, the same call made alone, and match the
oracle like the single-caller tests.
"""
import threading

import numpy as np
import pytest

from sqrtlm import synth

pytestmark = pytest.mark.gpu

TOL = 1e-6


def _rel(a, b):
    return np.abs(a - b).max() / max(1.0, np.abs(b).max())


def _lba(ctx, prob):
    ctx.set_problem(prob)
    ran, outl, st = ctx.local_ba()
    q, t = ctx.poses()
    return dict(ran=ran, outl=outl, st=st, q=q, t=t, X=ctx.points())


def _eg(ctx, pg):
    ctx.eg_set_problem(pg)
    n, st = ctx.eg_optimize(20, 1e-16)
    return dict(n=n, st=st, S=ctx.eg_poses().copy())


def _gba(ctx, prob):
    ctx.set_problem(prob)
    n, st = ctx.global_ba(10)
    q, t = ctx.poses()
    return dict(n=n, st=st, q=q, t=t, X=ctx.points())


def test_lba_eg_gba_threads(oracle):
    from sqrtlm.optimizer import Context
    lba_p = synth.config2(seed=2)
    eg_p = synth.make_pose_graph(300, window=4, n_loops=3, seed=1, fix_scale=True, noise=False)
    gba_p = synth.config4_loop(scale=0.05, loop=20)
    jobs = [(_lba, lba_p), (_eg, eg_p), (_gba, gba_p)]
    ctxs = [Context(0) for _ in jobs]
    try:
        alone = [fn(c, p) for c, (fn, p) in zip(ctxs, jobs)]
        out = [None] * len(jobs)
        errs = []

        def run(i):
            try:
                for _ in range(2):  # twice, so the calls overlap in more than one phase
                    out[i] = jobs[i][0](ctxs[i], jobs[i][1])
            except Exception as e:  # noqa: BLE001
                errs.append(e)

        th = [threading.Thread(target=run, args=(i,)) for i in range(len(jobs))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errs, errs
    finally:
        for c in ctxs:
            c.close()
    # concurrent == alone, bit for bit
    a, b = alone[0], out[0]
    assert a["ran"] == b["ran"] and np.array_equal(a["outl"], b["outl"])
    for k in ("q", "t", "X"):
        np.testing.assert_array_equal(a[k], b[k])
    np.testing.assert_array_equal(alone[1]["S"], out[1]["S"])
    for k in ("q", "t", "X"):
        np.testing.assert_array_equal(alone[2][k], out[2][k])
    assert [s["trace_chi2"] for s in a["st"]] == [s["trace_chi2"] for s in b["st"]]
    assert alone[2]["st"]["trace_chi2"] == out[2]["st"]["trace_chi2"]
    # and each matches its oracle
    ref = oracle.OracleGraph(lba_p)
    ran_r, outl_r, _ = ref.local_ba()
    assert ran_r == b["ran"] and np.array_equal(outl_r, b["outl"])
    assert np.abs(b["q"] - ref.pose_q).max() < TOL and _rel(b["X"], ref.pt) < TOL
    ref_e = oracle.OracleEG(eg_p)
    ref_e.optimize(20, 1e-16)
    assert _rel(out[1]["S"], ref_e.Siw) < 1e-9
    ref_g = oracle.OracleGraph(gba_p)
    nr, sr = ref_g.global_ba(10)
    assert out[2]["n"] == nr and out[2]["st"]["trace_trials"] == sr["trace_trials"]
    assert np.abs(out[2]["q"] - ref_g.pose_q).max() < TOL and _rel(out[2]["X"], ref_g.pt) < TOL
