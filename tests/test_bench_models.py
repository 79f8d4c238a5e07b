"""bench.py's cost models (CPU): the block-arrow split of the essential graph
mirrors sqlm_eg.hip's rule, and the FLOP / byte counts behind the roofline
fields are the formulas DESIGN.md states."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from sqrtlm import synth  # noqa: E402


def test_eg_arrow_layout_no_loops_is_all_band():
    pg = synth.make_pose_graph(200, window=6, n_loops=0, seed=1, fix_scale=True)
    band, border = bench.eg_arrow_layout(pg)
    assert border == 0 and band == int((pg.fixed == 0).sum())


def test_eg_arrow_layout_covers_every_long_edge():
    pg = synth.make_pose_graph(600, window=6, n_loops=12, seed=7, fix_scale=True)
    band, border = bench.eg_arrow_layout(pg)
    assert 0 < border <= 12 and band + border == int((pg.fixed == 0).sum())


def test_eg_solve_flops_band_only():
    pg = synth.make_pose_graph(224, window=4, n_loops=0, seed=2, fix_scale=True)
    band, border = bench.eg_arrow_layout(pg)
    p = -(-7 * band // 112)
    expect = p * (7.0 / 3.0) * 112 ** 3 + p * 4.0 * 112 ** 2
    assert border == 0 and np.isclose(bench.eg_solve_flops(pg), expect)


def test_update_bytes_model():
    """56 B per observation (ids 8, float4 inputs 16, s 8 read; error 16, s' 8
    written) and 196 B per landmark; the generator's inputs are float32 values,
    so the library takes the float4 path (DevProblem::obs_f32) on them."""
    prob = synth.config4(scale=0.002, seed=4)
    assert bench.algorithmic_bytes_update(prob) == prob.n_obs * 56 + prob.n_pt * 196
    for a in (prob.obs_uv, prob.obs_info):
        a = np.asarray(a, dtype=np.float64)
        assert np.array_equal(a.astype(np.float32).astype(np.float64), a)
