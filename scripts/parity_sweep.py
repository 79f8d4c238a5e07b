"""A long run of tests/test_gpu_sweep.py's shape generator: N seeded problem
shapes, HIP path vs the CPU oracle, one JSON line per case with the largest
deviations (poses, points, chi2 trace) and whether iteration / trial counts
agree; the last line sums it up. usage: python scripts/parity_sweep.py [N] [seed]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sqrtlm-slam_amd"), os.path.join(ROOT, "tests")]
from oracle import oracle as O  # noqa: E402  (the checker)
from sqrtlm.optimizer import Context  # noqa: E402
from test_gpu_sweep import _shapes, make  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 7
worst = {"pose": 0.0, "point": 0.0, "chi2": 0.0}
bad = 0
t0 = time.time()
with Context(0) as ctx:
    for i, kind, n_kf, n_lm, kw in _shapes(n, seed):
        prob = make(n_kf, n_lm, kw)
        ref = O.OracleGraph(prob)
        nr, sr = ref.optimize(0, 8)
        ctx.set_problem(prob)
        ng, sg = ctx.optimize(0, 8)
        q, t = ctx.poses()
        X = ctx.points()
        dq = float(np.abs(q - ref.pose_q).max())
        dt = float(np.abs(t - ref.pose_t).max() / max(1.0, np.abs(ref.pose_t).max()))
        dx = float(np.abs(X - ref.pt).max() / max(1.0, np.abs(ref.pt).max()))
        dc = float(np.max(np.abs(np.asarray(sg["trace_chi2"]) - np.asarray(sr["trace_chi2"])) /
                          np.maximum(1e-300, np.abs(np.asarray(sr["trace_chi2"])))))
        same = ng == nr and sg["iterations"] == sr["iterations"] and sg["trace_trials"] == sr["trace_trials"]
        ok = same and max(dq, dt, dx, dc) < 1e-6
        bad += not ok
        worst["pose"] = max(worst["pose"], dq, dt)
        worst["point"] = max(worst["point"], dx)
        worst["chi2"] = max(worst["chi2"], dc)
        print(json.dumps({"case": i, "kind": kind, "n_kf": n_kf, "n_lm": n_lm, "n_obs": int(prob.n_obs),
                          "counts_equal": same, "d_pose": max(dq, dt), "d_point": dx, "d_chi2_trace": dc, "ok": ok}),
              flush=True)
print(json.dumps({"cases": n, "seed": seed, "failed": bad, "worst": worst, "seconds": round(time.time() - t0, 1)}))
sys.exit(1 if bad else 0)
