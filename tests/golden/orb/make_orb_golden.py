"""Freeze the ORB oracle's output (tests/golden/orb/orb_golden.npz): one synthetic
640x300 image pair, extractor keypoints / descriptors (800 features) and the
SearchForInitialization matches. The oracle is pinned by tests/test_orb_oracle.py;
this file guards it against silent drift. Run: python tests/golden/orb/make_orb_golden.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path[:0] = [os.path.join(ROOT, "sqrtlm-slam_amd"), ROOT]

from oracle import orb as OB  # noqa: E402
from sqrtlm import synth  # noqa: E402

seed, shift = 21, (6.0, -2.0)
a, b = synth.make_image_pair(640, 300, seed=seed, shift=shift)
p = OB.params(800)
k1, d1 = OB.extract(p, a)
k2, d2 = OB.extract(p, b)
prev = np.ascontiguousarray(np.stack([k1["x"], k1["y"]], 1), np.float32)
n, m12, _ = OB.search_for_init(k1, d1, k2, d2, (0.0, 640.0, 0.0, 300.0), prev, 100, 0.9, True)
out = dict(seed=seed, shift=np.array(shift), img1=a, d1=d1, d2=d2, n_matches=n, m12=m12)
for f in OB.KP_DTYPE.names:
    out["k1_" + f] = k1[f]
np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "orb_golden.npz"), **out)
print(f"{len(k1)} / {len(k2)} keypoints, {n} matches")
