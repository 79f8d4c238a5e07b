"""Multi-rank host logic of the landmark-sharded global BA, world size 2 over
gloo on CPU. The GPU counterpart, which runs the library's
sharded solve on two ranks and compares it with one rank, is
test_gpu_sharded.py."""
import numpy as np
import pytest

from dist_util import gloo_allreduce, gloo_p2p, run_ranks
from sqrtlm import synth
from sqrtlm.shard import landmark_ranges, shard


def _sse(p):
    R = synth.quat_to_mat(p.pose_q)
    Xc = np.einsum("nij,nj->ni", R[p.obs_pose], p.pt[p.obs_pt]) + p.pose_t[p.obs_pose]
    fx, fy, cx, cy = (p.intr[p.obs_pose, k] for k in range(4))
    e = p.obs_uv - np.stack([Xc[:, 0] / Xc[:, 2] * fx + cx, Xc[:, 1] / Xc[:, 2] * fy + cy], axis=1)
    return float(np.sum(p.obs_info * np.sum(e * e, axis=1)))


def _rank_work(rank, world, scale):
    prob = synth.config4(seed=4, scale=scale)
    loc = shard(prob, rank, world)
    # the exchanges prepare() performs, through the same host collective
    act = np.zeros(prob.n_pose, np.uint8)
    act[np.unique(loc.obs_pose)] = 1
    gloo_allreduce(act, "max")
    cnt = np.array([loc.n_obs, loc.n_pt], np.int64).astype(np.float64)
    gloo_allreduce(cnt, "sum")
    chi = np.array([_sse(loc)])
    gloo_allreduce(chi, "sum")
    bw = np.array([int(np.max(np.bincount(loc.obs_pt, minlength=loc.n_pt)))], np.int32)  # longest track
    gloo_allreduce(bw, "max")
    return dict(act=act, cnt=cnt, chi=float(chi[0]), bw=int(bw[0]), n_obs=loc.n_obs,
                lid=loc.n_lid, first_pose=int(loc.obs_pose.min()), last_pose=int(loc.obs_pose.max()))


def test_ranges_cover_and_balance():
    prob = synth.config4(seed=4, scale=0.01)
    for world in (1, 2, 3, 8):
        rng = landmark_ranges(prob, world)
        assert rng[0][0] == 0 and rng[-1][1] == prob.n_pt
        assert all(a[1] == b[0] for a, b in zip(rng, rng[1:]))
        obs = [int(np.sum((prob.obs_pt >= lo) & (prob.obs_pt < hi))) for lo, hi in rng]
        assert sum(obs) == prob.n_obs
        assert max(obs) - min(obs) <= 2 * 18 + 1  # one landmark's track of slack per cut


@pytest.mark.parametrize("world", [2, 8])
def test_rank_exchanges_match_single_process(world):
    """The setup exchanges of prepare() at world size 2 and 8 (the driver's
    8-GPU node): camera set, counts, chi2 and the longest track agree with
    the single process; the shards cover the trajectory end to end."""
    prob = synth.config4(seed=4, scale=0.01)
    res = run_ranks(_rank_work, world, 0.01)
    full_act = np.zeros(prob.n_pose, np.uint8)
    full_act[np.unique(prob.obs_pose)] = 1
    for r in res:
        np.testing.assert_array_equal(r["act"], full_act)         # global camera set
        assert r["cnt"][0] == prob.n_obs and r["cnt"][1] == prob.n_pt
        assert r["chi"] == pytest.approx(_sse(prob), rel=1e-12)   # chi2 sums across shards
        assert r["bw"] == int(np.max(np.bincount(prob.obs_pt)))
    assert sum(r["n_obs"] for r in res) == prob.n_obs
    # contiguous landmark ranges in trajectory order touch overlapping camera bands
    assert res[0]["first_pose"] == 0 and res[-1]["last_pose"] == prob.n_pose - 1
    for a, b in zip(res, res[1:]):
        assert a["first_pose"] <= b["first_pose"] <= a["last_pose"] + 1


def test_lidar_edges_only_on_rank0():
    prob = synth.add_lidar_flat(synth.config4(seed=4, scale=0.01), pose=5, n=20, seed=1)
    assert shard(prob, 0, 2).n_lid == prob.n_lid
    assert shard(prob, 1, 2).n_lid == 0


def _gather_work(rank, world, n_rows, seed):
    """The per-trial exchange of sqlm_api.cpp trial() with the host transport:
    every rank > 0 sends its nonzero row range of S (here a dense [n_rows, 4]
    stand-in) to rank 0, which adds the ranges in rank order, then broadcasts
    the result (dx stand-in). Ranges are agreed by an all-reduce."""
    rng = np.random.default_rng(seed + rank)
    lo = rank * n_rows // world - (3 if rank else 0)
    hi = min(n_rows, (rank + 1) * n_rows // world + 3)
    S = np.zeros((n_rows, 4))
    S[lo:hi] = rng.normal(size=(hi - lo, 4))
    rngs = np.zeros(2 * world, np.int32)
    rngs[2 * rank], rngs[2 * rank + 1] = lo, hi
    gloo_allreduce(rngs, "sum")
    if rank == 0:
        tot = S.copy()
        for r in range(1, world):
            a, b = rngs[2 * r], rngs[2 * r + 1]
            buf = np.zeros((b - a, 4))
            gloo_p2p(buf, r, "recv")
            tot[a:b] += buf
        x = tot.sum(axis=1)
    else:
        gloo_p2p(np.ascontiguousarray(S[lo:hi]), 0, "send")
        x = np.zeros(n_rows)
    gloo_p2p(x, 0, "bcast")
    full = S.copy()
    gloo_allreduce(full, "sum")
    return dict(x=x, ref=full.sum(axis=1))


@pytest.mark.parametrize("world", [2, 3, 8])
def test_gather_to_root_and_broadcast(world):
    res = run_ranks(_gather_work, world, 50, 7)
    for r in res:
        np.testing.assert_allclose(r["x"], r["ref"], rtol=1e-12, atol=1e-12)
        np.testing.assert_array_equal(r["x"], res[0]["x"])


def test_balance_at_eight_ranks_full_size():
    """shard.py at the driver's N = 8 on config 4's full-size landmark layout:
    observation counts within one track of each other, every rank's camera
    window a contiguous 1/8 of the trajectory plus the overlap of the tracks
    cut at its ends (<= 17 cameras on each side)."""
    prob = synth.config4(seed=4, scale=0.2)
    rng = landmark_ranges(prob, 8)
    obs = []
    for lo, hi in rng:
        sel = (prob.obs_pt >= lo) & (prob.obs_pt < hi)
        obs.append(int(sel.sum()))
        cams = np.unique(prob.obs_pose[sel])
        assert cams[-1] - cams[0] + 1 == cams.size  # contiguous window
        assert cams.size <= prob.n_pose / 8 + 2 * 18
    assert max(obs) - min(obs) <= 2 * 18 + 1
