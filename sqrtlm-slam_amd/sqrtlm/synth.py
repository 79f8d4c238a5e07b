"""Synthetic KITTI-like bundle-adjustment problems.

Portable and seeded: a counter-based SplitMix64 stream with Box–Muller normals,
so the same seed gives the same problem on any host. Inputs are rounded to
float32 exactly where the reference's are (keypoints ``cv::KeyPoint.pt``,
``cv::Mat CV_32F`` poses and points, ``mvInvLevelSigma2``), then widened to
double as ``Converter::toSE3Quat`` / ``toVector3d`` do (src/utils/Converter.cc:55-68,166-174).

* intrinsics: KITTI-00 ``cfg/KITTI00-02.yaml:8-19`` (fx=fy=718.856, 1241x376);
* trajectory: forward along camera +z at 1 m per keyframe, yaw 0.02 sin(i/10);
* landmarks: back-projected from a pixel of the first observing keyframe at
  depth U[5,40] m, observed by the following keyframes where they project;
* octave ~ Geometric(0.5) clipped to [0,7], information ``invSigma2`` built in
  float like ``ORBextractor`` (src/frontend/ORBextractor.cc:485-505), pixel
  noise N(0, sigma2[octave]); a fraction of observations displaced 10-50 px;
* initial guess: free poses perturbed N(0,(0.3 deg)^2) in rotation and
  N(0,(0.05 m)^2) in translation, points N(0,(0.1 m)^2).
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field

import numpy as np

from .problem import HUBER_MONO_GBA, HUBER_MONO_LBA, BAProblem

KITTI_INTR = (718.856, 718.856, 607.1928, 185.2157)
KITTI_WH = (1241, 376)
_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


class SplitMix64:
    """Counter-based SplitMix64: draw i = mix(seed + (i+1)*golden)."""

    def __init__(self, seed: int):
        self.seed = np.uint64(seed & 0xFFFFFFFFFFFFFFFF)
        self.ctr = 0

    def u64(self, n: int) -> np.ndarray:
        with np.errstate(over="ignore"):
            i = np.arange(self.ctr + 1, self.ctr + n + 1, dtype=np.uint64)
            self.ctr += n
            z = self.seed + i * _GOLDEN
            z = (z ^ (z >> np.uint64(30))) * _M1
            z = (z ^ (z >> np.uint64(27))) * _M2
            return z ^ (z >> np.uint64(31))

    def uniform(self, n: int) -> np.ndarray:
        return (self.u64(n) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)

    def normal(self, n: int) -> np.ndarray:
        u1 = 1.0 - self.uniform(n)  # (0,1]
        u2 = self.uniform(n)
        return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)

    def integers(self, lo: int, hi: int, n: int) -> np.ndarray:
        """Uniform integers in [lo, hi]."""
        return lo + np.minimum((self.uniform(n) * (hi - lo + 1)).astype(np.int64), hi - lo)


def orb_inv_level_sigma2(n_levels: int = 8, scale: float = 1.2) -> np.ndarray:
    """mvInvLevelSigma2 computed in float as ORBextractor.cc:485-505."""
    s = [np.float32(1.0)]
    for _ in range(1, n_levels):
        s.append(np.float32(s[-1] * np.float32(scale)))
    sig2 = [np.float32(v * v) for v in s]
    return np.array([np.float32(1.0) / v for v in sig2], np.float32)


def _rot_y(a: np.ndarray) -> np.ndarray:
    c, s = np.cos(a), np.sin(a)
    R = np.zeros(a.shape + (3, 3))
    R[..., 0, 0] = c; R[..., 0, 2] = s; R[..., 1, 1] = 1.0; R[..., 2, 0] = -s; R[..., 2, 2] = c
    return R


def _so3_exp(w: np.ndarray) -> np.ndarray:
    th = np.linalg.norm(w, axis=-1)[..., None, None]
    K = np.zeros(w.shape[:-1] + (3, 3))
    K[..., 0, 1] = -w[..., 2]; K[..., 0, 2] = w[..., 1]
    K[..., 1, 0] = w[..., 2]; K[..., 1, 2] = -w[..., 0]
    K[..., 2, 0] = -w[..., 1]; K[..., 2, 1] = w[..., 0]
    th_safe = np.where(th < 1e-12, 1.0, th)
    a = np.where(th < 1e-12, 1.0, np.sin(th_safe) / th_safe)
    b = np.where(th < 1e-12, 0.5, (1 - np.cos(th_safe)) / th_safe ** 2)
    return np.eye(3) + a * K + b * (K @ K)


def quat_from_mat(R: np.ndarray) -> np.ndarray:
    """Eigen Quaterniond(Matrix3d) + SE3Quat::normalizeRotation, vectorised.
    Returns (N,4) x,y,z,w."""
    R = np.asarray(R, np.float64).reshape(-1, 3, 3)
    q = np.zeros((R.shape[0], 4))
    tr = (R[:, 0, 0] + R[:, 1, 1]) + R[:, 2, 2]
    pos = tr > 0
    if pos.any():
        Rp = R[pos]
        t = np.sqrt(tr[pos] + 1.0)
        w = 0.5 * t
        t = 0.5 / t
        q[pos, 3] = w
        q[pos, 0] = (Rp[:, 2, 1] - Rp[:, 1, 2]) * t
        q[pos, 1] = (Rp[:, 0, 2] - Rp[:, 2, 0]) * t
        q[pos, 2] = (Rp[:, 1, 0] - Rp[:, 0, 1]) * t
    for n in np.nonzero(~pos)[0]:
        m = R[n]
        i = 0
        if m[1, 1] > m[0, 0]:
            i = 1
        if m[2, 2] > m[i, i]:
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        t = np.sqrt(m[i, i] - m[j, j] - m[k, k] + 1.0)
        q[n, i] = 0.5 * t
        t = 0.5 / t
        q[n, 3] = (m[k, j] - m[j, k]) * t
        q[n, j] = (m[j, i] + m[i, j]) * t
        q[n, k] = (m[k, i] + m[i, k]) * t
    q[q[:, 3] < 0] *= -1.0
    nrm = np.sqrt((q[:, 0] ** 2 + q[:, 2] ** 2) + (q[:, 1] ** 2 + q[:, 3] ** 2))
    return q / nrm[:, None]


def quat_to_mat(q: np.ndarray) -> np.ndarray:
    q = np.asarray(q, np.float64).reshape(-1, 4)
    x, y, z, w = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    tx, ty, tz = 2 * x, 2 * y, 2 * z
    R = np.empty((q.shape[0], 3, 3))
    R[:, 0, 0] = 1 - (ty * y + tz * z); R[:, 0, 1] = ty * x - tz * w; R[:, 0, 2] = tz * x + ty * w
    R[:, 1, 0] = ty * x + tz * w; R[:, 1, 1] = 1 - (tx * x + tz * z); R[:, 1, 2] = tz * y - tx * w
    R[:, 2, 0] = tz * x - ty * w; R[:, 2, 1] = tz * y + tx * w; R[:, 2, 2] = 1 - (tx * x + ty * y)
    return R


def pose_through_f32(R: np.ndarray, t: np.ndarray):
    """Round a pose through a CV_32F Tcw and back (Converter::toSE3Quat)."""
    Rf = np.asarray(R, np.float32).astype(np.float64)
    tf = np.asarray(t, np.float32).astype(np.float64)
    return quat_from_mat(Rf), tf.reshape(-1, 3)


def make_problem(n_kf: int, n_lm: int, *, k_min: int = 2, k_max: int = 18, pair_window: int = 0,
                 n_fixed: int = 1, seed: int = 0, outlier_frac: float = 0.02, robust: bool = True,
                 huber_delta: float | None = None, noise: bool = True, perturb: bool = True,
                 loop: int = 0, loop_cams: int = 24, perturb_center: bool = False,
                 revisits: tuple = (), drift: tuple | None = None) -> BAProblem:
    """Generate a synthetic BA problem.

    pair_window > 0 selects the local-BA layout of config 2: every landmark has
    exactly two observers, the second within ``pair_window`` keyframes of the
    first. Otherwise k ~ U{k_min..k_max} consecutive keyframes (config 4).

    loop > 0 closes the trajectory: the keyframes drive a circle of
    circumference n_kf - loop metres (1 m per keyframe) and the last ``loop``
    keyframes revisit the places of the first ``loop`` ones, 0.5 m to the side.
    Every landmark is also observed by the keyframes of the other pass at the
    places of its track (its "twins", up to ``loop_cams`` observers in all), as
    a loop-closed map is after LoopClosing::CorrectLoop fuses the matched
    points (src/backend/LoopClosing.cc:863-877): the reduced camera system then
    couples keyframes 0.. with n_kf - loop.. far off its band.

    revisits = ((start_kf, length, place0), ...) generalises ``loop`` to several
    loop closures: keyframes start_kf .. start_kf+length-1 re-drive the places
    place0 .. of keyframes driven earlier (0.5 m to alternating sides), the
    other keyframes drive new places around the circle; twins as for ``loop``.
    A revisit must go to places already driven before it starts.

    drift = (deg, m) replaces the independent initial errors by the error of a
    visual-odometry map: a world-frame rigid motion G_i per keyframe, a random
    walk of N(0, deg^2) rotation and N(0, m^2) translation steps from KF 0 (exact),
    applied to the keyframe (T_wc' = G_i T_wc) and to each point with its first
    observer, plus small independent noise (deg / 2, m, points 0.02 m):
    neighbouring keyframes stay consistent, the far end of a loop has drifted.

    perturb_center: the initial pose error is a rotation about the camera
    centre plus a displacement of the centre (a drifted keyframe), instead of a
    perturbation of T_cw = [R | t] itself, whose rotation part swings the
    centre by |c| x angle (metres at kilometres from the origin)."""
    rng = SplitMix64(seed)
    fx, fy, cx, cy = KITTI_INTR
    W, H = KITTI_WH
    idx = np.arange(n_kf)
    rv_place = None
    if revisits:
        place = np.full(n_kf, -1, np.int64)
        side = np.zeros(n_kf)
        for r, (s0, ln, p0) in enumerate(revisits):
            place[s0:s0 + ln] = p0 + np.arange(ln)
            side[s0:s0 + ln] = 0.5 if r % 2 == 0 else -0.5
        first = place < 0
        place[first] = np.arange(int(first.sum()))
        Lc = int(first.sum())
        for s0, ln, p0 in revisits:
            if p0 + ln > int(first[:s0].sum()):
                raise ValueError("a revisit must go to places driven before it")
        th = 2.0 * np.pi * place / Lc
        rad = Lc / (2.0 * np.pi)
        yaw = th + 0.02 * np.sin(idx / 10.0)
        c = np.stack([rad * (1.0 - np.cos(th)) + side * np.cos(th), np.zeros(n_kf),
                      rad * np.sin(th) - side * np.sin(th)], axis=1)
        fp_of_place = np.empty(Lc, np.int64)
        fp_of_place[place[first]] = idx[first]
        rv_place = -np.ones(Lc, np.int64)  # the (first) revisiting keyframe of each place
        for k in idx[~first][::-1]:
            rv_place[place[k]] = k
        twin_of = np.where(first, rv_place[place], fp_of_place[place])
    elif loop > 0:
        Lc = n_kf - loop
        place = np.where(idx < Lc, idx, idx - Lc)
        th = 2.0 * np.pi * place / Lc
        rad = Lc / (2.0 * np.pi)
        yaw = th + 0.02 * np.sin(idx / 10.0)
        side = np.where(idx < Lc, 0.0, 0.5)
        c = np.stack([rad * (1.0 - np.cos(th)) + side * np.cos(th), np.zeros(n_kf),
                      rad * np.sin(th) - side * np.sin(th)], axis=1)
    else:
        yaw = 0.02 * np.sin(idx / 10.0)
        c = np.stack([np.zeros(n_kf), np.zeros(n_kf), idx * 1.0], axis=1)
    R_wc = _rot_y(yaw)
    R_cw = np.transpose(R_wc, (0, 2, 1))
    t_cw = -np.einsum("nij,nj->ni", R_cw, c)

    # landmark spans
    if pair_window > 0:
        k = np.full(n_lm, 2, np.int64)
        a = rng.integers(0, n_kf - 1 - 1, n_lm)
        off = rng.integers(1, pair_window, n_lm)
        b = np.minimum(a + off, n_kf - 1)
        span = b - a + 1
    else:
        k = rng.integers(k_min, k_max, n_lm)
        k = np.minimum(k, n_kf)
        a = (rng.uniform(n_lm) * (n_kf - k + 1)).astype(np.int64)
        a = np.minimum(a, n_kf - k)
        span = k
    dmin = np.maximum(5.0, span + 3.0)
    d = dmin + rng.uniform(n_lm) * (40.0 - dmin)
    s = (d - (span - 1)) / d
    xb = np.array([(0 - cx) / fx, (W - cx) / fx]) * 0.9
    yb = np.array([(0 - cy) / fy, (H - cy) / fy]) * 0.9
    xi = (xb[0] + rng.uniform(n_lm) * (xb[1] - xb[0])) * s
    yi = (yb[0] + rng.uniform(n_lm) * (yb[1] - yb[0])) * s
    pc = np.stack([xi * d, yi * d, d], axis=1)
    X = np.einsum("nij,nj->ni", R_wc[a], pc) + c[a]

    # observations
    if pair_window > 0:
        lm = np.repeat(np.arange(n_lm), 2)
        kf = np.stack([a, b], axis=1).reshape(-1)
    else:
        lm = np.repeat(np.arange(n_lm), k)
        starts = np.repeat(a, k)
        first = np.repeat(np.cumsum(k) - k, k)
        kf = starts + (np.arange(lm.size) - first)
    if loop > 0 or rv_place is not None:
        # twins: the other pass's keyframe at the place of each track keyframe,
        # in track order, while the landmark has fewer than loop_cams observers
        if rv_place is not None:
            tw = twin_of[kf]
        else:
            Lc = n_kf - loop
            tw = np.where(kf < loop, kf + Lc, np.where(kf >= Lc, kf - Lc, -1))
        cand = tw >= 0
        cnt = np.bincount(lm[cand], minlength=n_lm)
        rank_in_lm = np.cumsum(cand) - 1 - (np.cumsum(cnt) - cnt)[lm]  # lm is grouped, ascending
        room = loop_cams - k[lm]
        sel = cand & (rank_in_lm < room)
        lm = np.concatenate([lm, lm[sel]])
        kf = np.concatenate([kf, tw[sel]])
    Xc =np.einsum("nij,nj->ni", R_cw[kf], X[lm]) + t_cw[kf]
    u = fx * Xc[:, 0] / Xc[:, 2] + cx
    v = fy * Xc[:, 1] / Xc[:, 2] + cy
    vis = (Xc[:, 2] > 0.5) & (u >= 0) & (u < W) & (v >= 0) & (v < H)
    # keep landmarks with >= 2 visible observations
    cnt = np.bincount(lm[vis], minlength=n_lm)
    keep_lm = cnt >= 2
    keep = vis & keep_lm[lm]
    lm, kf, u, v = lm[keep], kf[keep], u[keep], v[keep]
    remap = -np.ones(n_lm, np.int64)
    remap[keep_lm] = np.arange(int(keep_lm.sum()))
    lm = remap[lm]
    X = X[keep_lm]
    # sort landmarks by first observing keyframe (stable)
    first_kf = np.full(X.shape[0], n_kf, np.int64)
    np.minimum.at(first_kf, lm, kf)
    order = np.argsort(first_kf, kind="stable")
    inv = np.empty_like(order)
    inv[order] = np.arange(order.size)
    X = X[order]
    lm = inv[lm]
    o2 = np.lexsort((kf, lm))
    lm, kf, u, v = lm[o2], kf[o2], u[o2], v[o2]
    E = lm.size

    # octaves, information, noise, outliers
    uo = 1.0 - rng.uniform(E)
    octave = np.minimum(np.floor(-np.log2(uo)).astype(np.int64), 7)
    inv_s2 = orb_inv_level_sigma2()
    info = inv_s2[octave].astype(np.float64)
    sigma = np.sqrt((np.float32(1.0) / inv_s2[octave]).astype(np.float64))
    if noise:
        u = u + sigma * rng.normal(E)
        v = v + sigma * rng.normal(E)
        n_out = int(round(outlier_frac * E))
        if n_out:
            sel = np.unique(rng.integers(0, E - 1, n_out))
            mag = 10.0 + rng.uniform(sel.size) * 40.0
            ang = 2 * np.pi * rng.uniform(sel.size)
            u[sel] += mag * np.cos(ang)
            v[sel] += mag * np.sin(ang)
    uv = np.stack([u, v], axis=1).astype(np.float32).astype(np.float64)

    fixed = np.zeros(n_kf, np.uint8)
    fixed[:max(1, n_fixed)] = 1
    gt_q, gt_t = pose_through_f32(R_cw, t_cw)
    gt_X = X.astype(np.float32).astype(np.float64)
    R0, t0 = R_cw.copy(), t_cw.copy()
    X0 = X.copy()
    if perturb and drift is not None:
        free = np.nonzero(fixed == 0)[0]
        sr, st_ = np.deg2rad(drift[0]), drift[1]
        w = np.cumsum(rng.normal(3 * n_kf).reshape(-1, 3) * sr, axis=0)
        tau = np.cumsum(rng.normal(3 * n_kf).reshape(-1, 3) * st_, axis=0)
        w -= w[0]
        tau -= tau[0]
        Gr = _so3_exp(w)
        Gr[fixed != 0] = np.eye(3)
        tau[fixed != 0] = 0.0
        c0 = np.einsum("nij,nj->ni", Gr, c) + tau
        R0 = np.transpose(np.einsum("nij,njk->nik", Gr, R_wc), (0, 2, 1))
        dth = rng.normal(3 * free.size).reshape(-1, 3) * (0.5 * sr)
        R0[free] = _so3_exp(dth) @ R0[free]
        c0[free] += rng.normal(3 * free.size).reshape(-1, 3) * st_
        t0 = -np.einsum("nij,nj->ni", R0, c0)
        fo = np.full(X.shape[0], n_kf, np.int64)  # first observer of each point
        np.minimum.at(fo, lm, kf)
        X0 = np.einsum("nij,nj->ni", Gr[fo], X) + tau[fo] + rng.normal(3 * X.shape[0]).reshape(-1, 3) * 0.02
    elif perturb:
        free = np.nonzero(fixed == 0)[0]
        dth = rng.normal(3 * free.size).reshape(-1, 3) * np.deg2rad(0.3)
        dt = rng.normal(3 * free.size).reshape(-1, 3) * 0.05
        R0[free] = _so3_exp(dth) @ R0[free]
        if perturb_center:
            t0[free] = -np.einsum("nij,nj->ni", R0[free], c[free] + dt)
        else:
            t0[free] = t0[free] + dt
        X0 = X0 + rng.normal(3 * X0.shape[0]).reshape(-1, 3) * 0.1
    q0, t0 = pose_through_f32(R0, t0)
    X0 = X0.astype(np.float32).astype(np.float64)

    if huber_delta is None:
        huber_delta = HUBER_MONO_LBA if pair_window > 0 else HUBER_MONO_GBA
    delta = np.full(E, huber_delta if robust else 0.0)
    prob = BAProblem(
        pose_q=q0, pose_t=t0, pose_fixed=fixed, intr=np.tile(np.array(KITTI_INTR), (n_kf, 1)),
        pt=X0, obs_pose=kf.astype(np.int32), obs_pt=lm.astype(np.int32), obs_uv=uv, obs_info=info,
        obs_delta=delta, obs_level=np.zeros(E, np.uint8),
        meta=dict(gt_q=gt_q, gt_t=gt_t, gt_pt=gt_X, octave=octave, seed=seed),
    )
    return prob


def config2(seed: int = 2, **kw) -> BAProblem:
    """BASELINE config 2: synthetic local BA, 50 KF (10 fixed) x 5k landmarks x
    200 obs/KF, k = 2, Huber (float)sqrt(5.991)."""
    kw.setdefault("n_fixed", 10)
    return make_problem(50, 5000, pair_window=5, seed=seed, robust=True, **kw)


def config4(seed: int = 4, scale: float = 1.0, **kw) -> BAProblem:
    """BASELINE config 4: synthetic global BA, 5k poses x 500k landmarks,
    k ~ U{2..18} consecutive keyframes, KF0 fixed, no robust kernel
    (LoopClosing.cc:987-991 passes bRobust=false). ``scale`` shrinks both
    counts proportionally for parity-sized cases."""
    n_kf = max(20, int(round(5000 * scale)))
    n_lm = max(100, int(round(500000 * scale)))
    kw.setdefault("robust", False)
    return make_problem(n_kf, n_lm, k_min=2, k_max=18, n_fixed=1, seed=seed, **kw)


def config4_loop(seed: int = 4, scale: float = 1.0, loop: int = 30, **kw) -> BAProblem:
    """Config 4 on a loop-closed map, the shape the reference's GBA always has
    (it only runs after a loop closure: LoopClosing.cc:877, :987-991): a
    circular trajectory whose last ``loop`` keyframes revisit the first ones,
    every landmark at those places also observed from the other pass (a few
    thousand landmarks co-observed by KF 0..~47 and KF n-loop..n-1). Same
    counts, track lengths and GBA schedule as config 4 otherwise; the initial
    error is a drift of every keyframe about its own centre (on a 790 m
    circle a perturbation of T_cw itself would move centres by metres and put
    points behind cameras)."""
    n_kf = max(20, int(round(5000 * scale)))
    n_lm = max(100, int(round(500000 * scale)))
    kw.setdefault("robust", False)
    kw.setdefault("perturb_center", True)
    return make_problem(n_kf, n_lm, k_min=2, k_max=18, n_fixed=1, seed=seed, loop=min(loop, n_kf // 4), **kw)


KITTI00_REVISITS = ((700, 40, 200), (1400, 100, 0))


def kitti00_map(seed: int = 4, n_kf: int = 1500, n_lm: int = 100000, revisits=KITTI00_REVISITS,
                stereo_frac: float = 0.5) -> BAProblem:
    """Stand-in for the KITTI-00 map that configs 3 / 5 run on (the sequence
    itself is not available): 1.5k keyframes, 1e5 landmarks over k ~ U{2..18}
    consecutive keyframes (~1e6 observations), two loop closures — a 40-KF
    re-entry into a stretch driven 500 KFs earlier and the final 100-KF revisit
    of the start — with the matched points fused into both passes, odometry
    drift (0.005 deg and 0.005 m per keyframe, random walk), and half of the
    observations stereo (KITTI is a stereo rig; cfg/KITTI00-02.yaml Camera.bf)."""
    prob = make_problem(n_kf, n_lm, k_min=2, k_max=18, n_fixed=1, seed=seed, robust=True, revisits=revisits,
                        drift=(0.005, 0.005))
    prob.meta["revisits"] = tuple(revisits)
    return add_stereo(prob, stereo_frac, seed=seed)


def add_lidar_flat(prob: BAProblem, pose: int, n: int, *, seed: int = 0, noise: float = 0.01,
                   weight: float = 50.0) -> BAProblem:
    """Attach ``n`` EdgeLidarFlatPoint unary edges to ``pose`` (the current KF of
    local-BA pass 3, g2oOptimizer.cc:1034-1070): a current-frame point p_c with
    its plane normal n_c and a map point p_w on the same plane, so that
    e = (T_cw p_w - p_c) . n_c is zero at the ground-truth pose up to ``noise``.
    Information = flat_optimized_weight (cfg/lidar_slam.yaml:58)."""
    rng = SplitMix64(seed ^ 0x5EED)
    gq, gt = prob.meta["gt_q"][pose], prob.meta["gt_t"][pose]
    R = quat_to_mat(gq)[0]
    nrm = rng.normal(3 * n).reshape(-1, 3)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    pc = np.stack([rng.uniform(n) * 20 - 10, rng.uniform(n) * 4 - 2, 2 + rng.uniform(n) * 30], axis=1)
    tang = rng.normal(3 * n).reshape(-1, 3) * 0.3
    tang -= np.sum(tang * nrm, axis=1, keepdims=True) * nrm
    on_plane = pc + tang + noise * rng.normal(n)[:, None] * nrm
    pw = (on_plane - gt) @ R  # R^T (p - t)
    prob.lid_pose = np.full(n, pose, np.int32)
    prob.lid_pc = pc.astype(np.float32).astype(np.float64)
    prob.lid_pw = pw.astype(np.float32).astype(np.float64)
    prob.lid_n = nrm.astype(np.float32).astype(np.float64)
    prob.lid_info = np.full(n, weight)
    prob.validate()
    return prob


KITTI_BF = 386.1448  # Camera.bf, cfg/KITTI00-02.yaml


def add_stereo(prob: BAProblem, frac: float = 0.5, *, bf: float = KITTI_BF, seed: int = 0,
               robust_delta: float | None = None, noise: bool = True) -> BAProblem:
    """Turn a fraction of the observations into EdgeStereoSE3ProjectXYZ edges
    (GBA stereo branch, g2oOptimizer.cc:247-281): u_right = u - bf / z at the
    ground truth plus the observation's pixel noise, rounded through float32
    like ``mvuRight``; every keyframe gets ``mbf = bf``. ``robust_delta``
    replaces the Huber delta of the stereo edges (the reference uses
    thHuber3D = sqrt(7.815) when bRobust)."""
    rng = SplitMix64(seed ^ 0x57E0)
    E = prob.n_obs
    sel = rng.uniform(E) < frac
    gq, gt, gX = prob.meta["gt_q"], prob.meta["gt_t"], prob.meta["gt_pt"]
    R = quat_to_mat(gq[prob.obs_pose])
    Xc = np.einsum("eij,ej->ei", R, gX[prob.obs_pt]) + gt[prob.obs_pose]
    z = Xc[:, 2]
    oct_ = prob.meta.get("octave")
    sigma = np.ones(E) if oct_ is None else np.sqrt(1.0 / orb_inv_level_sigma2()[oct_].astype(np.float64))
    ur = prob.obs_uv[:, 0] - bf / z + (sigma * rng.normal(E) if noise else 0.0)
    ur = np.where(sel & (z > 0), ur, -1.0).astype(np.float32).astype(np.float64)
    prob.obs_ur = ur
    prob.pose_bf = np.full(prob.n_pose, float(np.float32(bf)))
    if robust_delta is not None:
        prob.obs_delta = np.where(ur >= 0, robust_delta, prob.obs_delta)
    prob.validate()
    return prob


# ---------------------------------------------------------------- essential graph

@dataclass
class PoseGraph:
    """Essential graph of g2oOptimizer::OptimizeEssentialGraph (g2oOptimizer.cc:1212-1534):
    Sim3 S_iw per keyframe [qx qy qz qw tx ty tz s], EdgeSim3 (i = vertex 0,
    j = vertex 1, measurement S_ji), identity information unless ``info``."""
    Siw: np.ndarray                 # (K,8)
    fixed: np.ndarray               # (K,) uint8, the loop keyframe
    fix_scale: int
    ei: np.ndarray                  # (E,) int32
    ej: np.ndarray                  # (E,) int32
    Sji: np.ndarray                 # (E,8)
    info: np.ndarray | None = None  # (E,7,7)
    meta: dict = field(default_factory=dict)

    def __post_init__(self):
        self.Siw = np.ascontiguousarray(self.Siw, np.float64).reshape(-1, 8)
        self.fixed = np.ascontiguousarray(self.fixed, np.uint8).reshape(-1)
        self.ei = np.ascontiguousarray(self.ei, np.int32).reshape(-1)
        self.ej = np.ascontiguousarray(self.ej, np.int32).reshape(-1)
        self.Sji = np.ascontiguousarray(self.Sji, np.float64).reshape(-1, 8)
        if self.info is not None:
            self.info = np.ascontiguousarray(self.info, np.float64).reshape(-1, 7, 7)
        K, E = self.Siw.shape[0], self.ei.shape[0]
        if self.fixed.shape[0] != K or self.ej.shape[0] != E or self.Sji.shape[0] != E:
            raise ValueError("pose graph arrays disagree in length")
        if E and (min(self.ei.min(), self.ej.min()) < 0 or max(self.ei.max(), self.ej.max()) >= K):
            raise ValueError("edge vertex out of range")

    @property
    def n_kf(self) -> int:
        return self.Siw.shape[0]

    @property
    def n_edge(self) -> int:
        return self.ei.shape[0]

    def copy(self) -> "PoseGraph":
        return copy.deepcopy(self)


def _sim3_np(R, t, s):
    q = quat_from_mat(R)
    return np.concatenate([q, t, np.atleast_1d(s)[:, None] if np.ndim(s) else np.full((q.shape[0], 1), s)], axis=1)


def _sim3_compose(a, b):
    """a*b for arrays of [q t s] (numpy restatement for data generation only)."""
    Ra, Rb = quat_to_mat(a[:, :4]), quat_to_mat(b[:, :4])
    R = Ra @ Rb
    t = a[:, 7:8] * np.einsum("nij,nj->ni", Ra, b[:, 4:7]) + a[:, 4:7]
    return np.concatenate([quat_from_mat(R), t, (a[:, 7] * b[:, 7])[:, None]], axis=1)


def _sim3_inv(a):
    R = quat_to_mat(a[:, :4])
    Rt = np.transpose(R, (0, 2, 1))
    t = np.einsum("nij,nj->ni", Rt, -a[:, 4:7] / a[:, 7:8])
    return np.concatenate([quat_from_mat(Rt), t, (1.0 / a[:, 7])[:, None]], axis=1)


def make_pose_graph(n_kf: int = 200, *, window: int = 4, n_loops: int = 3, seed: int = 0, noise: bool = True,
                    drift: float = 0.01, fix_scale: bool = False, rot_noise: float = 2e-3,
                    trans_noise: float = 5e-3, scale_noise: float = 1e-3) -> PoseGraph:
    """A loop-closing essential graph on the generator's trajectory: spanning
    tree i -> i-1, covisibility edges to the previous ``window`` keyframes,
    and ``n_loops`` long edges closing the trajectory onto its start. Edge
    measurements are ground-truth relative Sim3 (plus noise of the given
    standard deviations: rotation rad, translation m, log-scale); the initial
    estimates carry an accumulated rotation / translation / scale drift, as
    the uncorrected side of a loop does. Keyframe 0 (the loop keyframe) is fixed."""
    rng = SplitMix64(seed ^ 0xE55E)
    i = np.arange(n_kf)
    yaw = 0.02 * np.sin(i / 10.0)
    R_cw = np.transpose(_rot_y(yaw), (0, 2, 1))
    C = np.stack([np.sin(i / 40.0) * 20.0, np.zeros(n_kf), i * 1.0], axis=1)  # camera centres
    t_cw = -np.einsum("nij,nj->ni", R_cw, C)
    gt = _sim3_np(R_cw, t_cw, 1.0)
    pairs = [(k, k - 1) for k in range(1, n_kf)]
    pairs += [(k, k - d) for k in range(n_kf) for d in range(2, window + 1) if k - d >= 0]
    loop_src = np.linspace(n_kf - 1, n_kf - 1 - 3 * max(n_loops - 1, 0), n_loops).astype(int)
    pairs += [(int(a), int(b)) for a, b in zip(loop_src, np.arange(n_loops) * 2)]
    ei = np.array([p[0] for p in pairs], np.int32)
    ej = np.array([p[1] for p in pairs], np.int32)
    Sji = _sim3_compose(gt[ej], _sim3_inv(gt[ei]))
    if noise:
        E = ei.size
        w = rng.normal(3 * E).reshape(-1, 3) * rot_noise
        dR = _so3_exp(w)
        Sji = _sim3_compose(np.concatenate([quat_from_mat(dR), rng.normal(3 * E).reshape(-1, 3) * trans_noise,
                                            np.exp(rng.normal(E) * (0.0 if fix_scale else scale_noise))[:, None]],
                                           axis=1), Sji)
    # drifted initial estimates: accumulated along the trajectory, KF 0 exact
    acc = np.cumsum(rng.normal(3 * n_kf).reshape(-1, 3) * drift, axis=0)
    acc[0] = 0.0
    dS = np.concatenate([quat_from_mat(_so3_exp(acc * 0.2)), acc * 2.0,
                         np.exp(np.cumsum(rng.normal(n_kf) * drift * (0 if fix_scale else 1)))[:, None]], axis=1)
    dS[0] = [0, 0, 0, 1, 0, 0, 0, 1]
    S0 = _sim3_compose(gt, dS)
    fixed = np.zeros(n_kf, np.uint8)
    fixed[0] = 1
    return PoseGraph(Siw=S0, fixed=fixed, fix_scale=int(fix_scale), ei=ei, ej=ej, Sji=Sji,
                     meta=dict(gt=gt, seed=seed))


# ---- synthetic grey images for the ORB front end ----------

def make_scene(w: int, h: int, *, seed: int = 0, n_rect: int = 0, n_disk: int = 0) -> np.ndarray:
    """A textured 8-bit scene (float, unclipped): gradient background, random
    filled rectangles and disks of random grey levels (corners for FAST), and a
    fine random texture. Sized w x h; n_rect / n_disk default to the area."""
    rng = np.random.default_rng(seed)
    n_rect = n_rect or max(40, w * h // 2500)
    n_disk = n_disk or max(20, w * h // 5000)
    yy, xx = np.mgrid[0:h, 0:w]
    img = 60.0 + 80.0 * (xx / w) + 40.0 * np.sin(yy / 37.0)
    for _ in range(n_rect):
        rw, rh = rng.integers(6, 60, 2)
        x0, y0 = rng.integers(-20, w), rng.integers(-20, h)
        img[max(y0, 0):max(y0 + rh, 0), max(x0, 0):max(x0 + rw, 0)] = rng.uniform(0, 255)
    for _ in range(n_disk):
        r = rng.uniform(3, 25)
        cx, cy = rng.uniform(0, w), rng.uniform(0, h)
        x0, x1 = int(max(cx - r, 0)), int(min(cx + r + 1, w))
        y0, y1 = int(max(cy - r, 0)), int(min(cy + r + 1, h))
        if x1 <= x0 or y1 <= y0:
            continue
        m = (xx[y0:y1, x0:x1] - cx) ** 2 + (yy[y0:y1, x0:x1] - cy) ** 2 <= r * r
        img[y0:y1, x0:x1][m] = rng.uniform(0, 255)
    img += rng.normal(0, 6.0, img.shape)
    return img


def make_image_pair(w: int = 1241, h: int = 376, *, seed: int = 0, shift=(7.0, 3.0), noise: float = 2.0):
    """Two frames of one scene (KITTI-00 size by default): frame 2 is the scene
    translated by `shift` pixels (integer part by cropping, so FAST corners
    move exactly) with independent sensor noise. Returns (img1, img2) uint8."""
    rng = np.random.default_rng(seed + 1)
    pad = 16
    scene = make_scene(w + 2 * pad, h + 2 * pad, seed=seed)
    sx, sy = int(round(shift[0])), int(round(shift[1]))
    a = scene[pad:pad + h, pad:pad + w] + rng.normal(0, noise, (h, w))
    b = scene[pad - sy:pad - sy + h, pad - sx:pad - sx + w] + rng.normal(0, noise, (h, w))
    return (np.clip(np.rint(a), 0, 255).astype(np.uint8), np.clip(np.rint(b), 0, 255).astype(np.uint8))
