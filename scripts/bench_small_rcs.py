"""ms per LM iteration and solve time of small local-BA windows (2..8
superblocks); run it under two environments to A/B a solve or launch setting
(the tag printed is $SQLM_AB_TAG)."""
import os, sys
sys.path[:0] = ['sqrtlm-slam_amd', '.']
from sqrtlm import synth
from sqrtlm.optimizer import Context
tag = os.environ.get("SQLM_AB_TAG", "default")
with Context(0) as ctx:
    for n_pose, pw in ((9, 4), (16, 4), (23, 4), (28, 4), (43, 4), (43, 15)):
        prob = synth.make_problem(n_pose, 50 * n_pose, pair_window=pw, n_fixed=3, seed=100 + n_pose, robust=True)
        ctx.set_problem(prob)
        ctx.optimize(0, 1)
        lay = ctx.rcs_layout()
        best = min(ctx.bench(3, 40, False)[0] for _ in range(3))
        _, k, _ = ctx.bench(3, 40, True)
        print(f"{tag} n_pose={n_pose} p={lay['p']} B={lay['B']} n={lay['n']} "
              f"ms/it={best:.4f} solve_ms={k.get('k_solve', 0):.4f}", flush=True)
