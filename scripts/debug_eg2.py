"""EG GPU vs oracle outcome statistics across seeds (diagnostic)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sqrtlm-slam_amd"), ROOT]
import numpy as np
from oracle import oracle as O
from sqrtlm import synth
from sqrtlm.optimizer import Context

ctx = Context(0)
def rel(a, b): return np.abs(a - b).max() / max(1.0, np.abs(b).max())
for noise, K, fs, rn in [(True, 150, True, 3e-4), (True, 150, True, 2e-2), (True, 400, True, 3e-4), (False, 400, True, 0)]:
    for seed in range(1, 5):
        pg = synth.make_pose_graph(K, window=4, n_loops=3, seed=seed, noise=noise, fix_scale=fs, rot_noise=rn,
                                   trans_noise=5e-4 if rn < 1e-3 else 5e-2)
        ref = O.OracleEG(pg); nr, sr = ref.optimize(1, 1e-16)
        ctx.eg_set_problem(pg); ng, sg = ctx.eg_optimize(1, 1e-16)
        d1 = rel(ctx.eg_poses(), ref.Siw)
        ref = O.OracleEG(pg); nr, sr = ref.optimize(20, 1e-16)
        ctx.eg_set_problem(pg); ng, sg = ctx.eg_optimize(20, 1e-16)
        print(f"noise={noise} rn={rn} K={K} fs={fs} seed={seed} it1 dS {d1:.2e} | 20it: n {ng}/{nr} chi {sg['chi2_end']:.6g}/{sr['chi2_end']:.6g} dS {rel(ctx.eg_poses(), ref.Siw):.2e} trials {sum(sg['trace_trials'])}/{sum(sr['trace_trials'])}")
