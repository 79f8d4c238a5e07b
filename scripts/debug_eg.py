"""EG GPU vs oracle, step by step on small graphs (diagnostic)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sqrtlm-slam_amd"), ROOT]
import numpy as np
from oracle import oracle as O
from sqrtlm import synth
from sqrtlm.optimizer import Context

ctx = Context(0)
pg = synth.make_pose_graph(6, window=3, n_loops=1, seed=1, noise=False)
ctx.eg_set_problem(pg); ctx.eg_optimize(1, 1e-16); S1 = ctx.eg_poses()
pg2 = pg.copy(); pg2.Siw[:] = S1
print("--- restart from GPU iteration-1 state", file=sys.stderr)
ctx.eg_set_problem(pg2); n, st = ctx.eg_optimize(1, 1e-16 / 3)
ref = O.OracleEG(pg2); ref.optimize(1, 1e-16 / 3)
print("restart: gpu chi", st["chi2_begin"], "->", st["chi2_end"], "trials", st["trace_trials"], "dS", np.abs(ctx.eg_poses() - ref.Siw).max())
print("--- continued", file=sys.stderr)
ctx.eg_set_problem(pg); ctx.eg_optimize(2, 1e-16)
for K, win, loops, noise in [(6, 3, 1, False)]:
    pg = synth.make_pose_graph(K, window=win, n_loops=loops, seed=1, noise=noise)
    for iters in (1, 2, 5):
        ref = O.OracleEG(pg)
        nr, sr = ref.optimize(iters, 1e-16)
        ctx.eg_set_problem(pg)
        ng, sg = ctx.eg_optimize(iters, 1e-16)
        S = ctx.eg_poses()
        print(f"K={K} it={iters} n {ng}/{nr} trials {sg['trace_trials']}/{sr['trace_trials']} "
              f"chi2 {sg['chi2_begin']:.6g}->{sg['chi2_end']:.6g} / {sr['chi2_begin']:.6g}->{sr['chi2_end']:.6g} "
              f"dS {np.abs(S - ref.Siw).max():.3e}")
    if K == 3:
        print("S0", pg.Siw, "\nref", ref.Siw, "\ngpu", S)
