"""Replay vs direct library LBA vs oracle on the LBA capture fixture (diagnostic)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sqrtlm-slam_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np
from oracle import oracle as O
from sqrtlm import capture
from sqrtlm.optimizer import Context
from capture_util import capture_to_problem

name = sys.argv[1] if len(sys.argv) > 1 else "lba_capture.sqcap"
c = capture.read(os.path.join(ROOT, "tests", "golden", name))
prob, edge_of, pt_src = capture_to_problem(c, O)
ctx = Context(0)
out = capture.replay(ctx, c)
print("replay stats", [(s["iterations"], s["trace_trials"]) for s in out["stats"]])
ref = O.OracleGraph(prob)
if c.kind == capture.LBA:
    _, ro, rs = ref.local_ba()
    print("oracle stats", [(s["iterations"], s["trace_trials"]) for s in rs])
    ctx.set_problem(prob)
    _, go, gs = ctx.local_ba()
    print("direct stats", [(s["iterations"], s["trace_trials"]) for s in gs])
    print("outliers replay/direct/oracle", out["outlier"].sum(), go.sum(), ro.sum())
    for a, b in zip(gs, rs):
        print("chi2 traces", np.max(np.abs(np.array(a["trace_chi2"]) - b["trace_chi2"]) / np.abs(b["trace_chi2"])) if a["trace_chi2"] and len(a["trace_chi2"]) == len(b["trace_chi2"]) else (a["trace_chi2"], b["trace_chi2"]))
ctx.set_problem(prob)
if c.kind == capture.GBA:
    ctx.global_ba(c.gba_iterations); ref.global_ba(c.gba_iterations)
else:
    ctx.local_ba()
q, t = ctx.poses()
print("direct vs oracle pose t", np.abs(t - ref.pose_t).max(), "q", np.abs(q - ref.pose_q).max(), "X", np.abs(ctx.points() - ref.pt).max())
Tcw = np.stack([O.se3_to_Tcw_f32(ref.pose_q[p], ref.pose_t[p]) for p in range(c.n_pose)])
print("oracle rerun vs fixture Tcw", np.abs(Tcw - c.res_Tcw).max(), "replay vs fixture", np.abs(out["Tcw"] - c.res_Tcw).max())
