"""Generates the committed capture fixtures.

Each file is a seam capture in the reference's float32 input form
(include/sqrtlm_capture.h) whose res_* sections hold the CPU oracle's run of
the captured call, with the same conversions the replay applies. No capture
from the reference itself exists here (it cannot be built or run, §8c), so
these pin the format and the replay path; PARITY UNPINNED against the
reference. Re-generate with:  python tests/golden/make_captures.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "sqrtlm-slam_amd"), ROOT, os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

from capture_util import oracle_results, problem_to_capture  # noqa: E402
from oracle import oracle as O  # noqa: E402
from sqrtlm import capture, synth  # noqa: E402
from sqrtlm.problem import HUBER_MONO_GBA, HUBER_STEREO  # noqa: E402


def cases():
    # LocalBundleAdjustment: a 16-KF window, LiDAR pairs on the current KF, and
    # stereo observations that the reference's LBA does not turn into edges
    lba = synth.make_problem(16, 500, pair_window=5, n_fixed=4, seed=31, robust=True)
    synth.add_lidar_flat(lba, pose=15, n=150, seed=31)
    synth.add_stereo(lba, 0.3, seed=31)
    # keep >= 2 mono edges per point: a point left with one edge after the
    # stereo observations are dropped has a rank-2 block (depth fixed only by
    # the damping), which would make the fixture ill-conditioned
    mono = lba.obs_ur < 0
    for l in np.nonzero(np.bincount(lba.obs_pt[mono], minlength=lba.n_pt) < 2)[0]:
        lba.obs_ur[lba.obs_pt == l] = -1.0
    # GBA with stereo edges, bRobust: Huber sqrt(5.991)/sqrt(7.815) per edge type
    gba = synth.make_problem(24, 900, k_min=2, k_max=8, n_fixed=1, seed=32, robust=True,
                             huber_delta=HUBER_MONO_GBA)
    synth.add_stereo(gba, 0.5, seed=32, robust_delta=HUBER_STEREO)
    return {
        "lba_capture.sqcap": problem_to_capture(lba, capture.LBA, O),
        "gba_stereo_capture.sqcap": problem_to_capture(gba, capture.GBA, O, gba_iterations=10, gba_robust=1),
    }


def main():
    O.build()
    for name, c in cases().items():
        oracle_results(c, O)
        path = os.path.join(HERE, name)
        capture.write(path, c)
        back = capture.read(path)
        assert np.array_equal(back.res_Tcw, c.res_Tcw)
        print(name, os.path.getsize(path), "bytes", c.n_pose, "poses", c.n_pt, "points", c.n_obs, "obs",
              int(c.res_outlier.sum()), "outliers")


if __name__ == "__main__":
    main()
