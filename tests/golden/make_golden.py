"""Generates the committed golden fixtures (inputs + oracle outputs).

The reference ships no fixtures for this path and cannot be
compiled or run here (§8c), so these vectors come from the repo's oracle
(oracle/g2o_ref.c, a restatement of the g2o path) on the repo's seeded
generator. They pin regressions of the oracle and are the shared expected
outputs of the CPU and GPU parity tests. PARITY UNPINNED against the
reference itself. Re-generate with:  python tests/golden/make_golden.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "sqrtlm-slam_amd"), ROOT]

import numpy as np  # noqa: E402

from oracle import oracle as O  # noqa: E402
from sqrtlm import synth  # noqa: E402

FIELDS = ("pose_q", "pose_t", "pose_fixed", "intr", "pt", "obs_pose", "obs_pt", "obs_uv", "obs_info",
          "obs_delta", "obs_level", "lid_pose", "lid_pc", "lid_pw", "lid_n", "lid_info")


def cases():
    lba = synth.make_problem(16, 600, pair_window=5, n_fixed=4, seed=21, robust=True)
    lba_lidar = synth.add_lidar_flat(synth.make_problem(16, 600, pair_window=5, n_fixed=4, seed=22, robust=True),
                                     pose=15, n=200, seed=22)
    gba = synth.config4(scale=0.006, seed=23)
    return {"lba_small": ("local_ba", lba), "lba_lidar": ("local_ba", lba_lidar), "gba_small": ("global_ba", gba)}


def run(kind, prob):
    g = O.OracleGraph(prob)
    out = {}
    if kind == "local_ba":
        ran, outl, st = g.local_ba()
        out["outlier"] = outl
        out["edge_level_out"] = g.obs_level.copy()
        for i, s in enumerate(st):
            out[f"pass{i}_iters"] = np.array(s["iterations"])
            out[f"pass{i}_trace_chi2"] = np.array(s["trace_chi2"])
            out[f"pass{i}_trace_trials"] = np.array(s["trace_trials"])
    else:
        n, s = g.global_ba(10)
        out["pass0_iters"] = np.array(n)
        out["pass0_trace_chi2"] = np.array(s["trace_chi2"])
        out["pass0_trace_trials"] = np.array(s["trace_trials"])
    out["out_pose_q"], out["out_pose_t"], out["out_pt"] = g.pose_q, g.pose_t, g.pt
    out["out_edge_chi2"] = g.edge_chi2()
    return out


if __name__ == "__main__":
    O.build()
    for name, (kind, prob) in cases().items():
        arrays = {f"in_{f}": getattr(prob, f) for f in FIELDS}
        arrays.update(run(kind, prob))
        arrays["kind"] = np.array(kind)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrays)
        print(name, prob.n_pose, prob.n_pt, prob.n_obs, prob.n_lid)
