"""Shared loader for tests/golden/*.npz fixtures (inputs + expected outputs)."""
import glob
import os

import numpy as np

from sqrtlm.problem import BAProblem

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIELDS = ("pose_q", "pose_t", "pose_fixed", "intr", "pt", "obs_pose", "obs_pt", "obs_uv", "obs_info",
          "obs_delta", "obs_level", "lid_pose", "lid_pc", "lid_pw", "lid_n", "lid_info")


def names():
    return sorted(os.path.splitext(os.path.basename(p))[0] for p in glob.glob(os.path.join(GOLDEN, "*.npz")))


def load(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    prob = BAProblem(**{f: z["in_" + f] for f in FIELDS})
    exp = {k: z[k] for k in z.files if not k.startswith("in_")}
    return str(z["kind"]), prob, exp
