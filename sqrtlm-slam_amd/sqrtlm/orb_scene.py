"""Tracking scenes for ORBmatcher's projection searches, built from two
extracted synthetic frames (synth.make_image_pair): frame 1 plays LastFrame /
the keyframes the local map comes from, frame 2 is CurrentFrame.

- local map points (SearchByProjection(F, vpMapPoints, th), ORBmatcher.cc:67):
  frame-1 keypoints predicted at their true shifted place plus noise, the
  tracking flags (mbTrackInView, isBad, mTrackViewCos, mnTrackScaleLevel)
  mixed so every branch is taken, duplicates so points compete for slots;
- last-frame slots (SearchByProjection(CurrentFrame, LastFrame, th, bMono),
  :1717): frame-1 keypoints back-projected at random depths with LastFrame at
  the origin, CurrentFrame rotated so they reproject about the image shift.

Stereo cases give CurrentFrame an mvuRight from random depths; some slots of
CurrentFrame start occupied (with and without observations).
"""
from __future__ import annotations

import numpy as np

FX = FY = 500.0
MB = 0.5  # stereo baseline (m)

TRACK_POINT_DTYPE = np.dtype([("id", "<i4"), ("proj_x", "<f4"), ("proj_y", "<f4"), ("proj_xr", "<f4"),
                              ("view_cos", "<f4"), ("level", "<i4"), ("in_view", "u1"), ("bad", "u1"),
                              ("has_obs", "u1"), ("pad", "u1")])
LAST_POINT_DTYPE = np.dtype([("id", "<i4"), ("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("octave", "<i4"),
                             ("angle", "<f4"), ("outlier", "u1"), ("has_obs", "u1"), ("pad", "u1", (2,))])


def scale_factors(n=8, f=1.2):
    sf = [np.float32(1.0)]
    for _ in range(1, n):
        sf.append(np.float32(sf[-1] * np.float32(f)))
    return np.array(sf, np.float32)


def camera(w, h):
    """(fx, fy, cx, cy, mbf, mb)."""
    return (FX, FY, w / 2.0, h / 2.0, MB * FX, MB)


def current_slots(k2, seed, stereo):
    """CurrentFrame's mvuRight (or None) and initial mvpMapPoints / slot_obs."""
    rng = np.random.default_rng(seed + 100)
    n = len(k2)
    uright = None
    if stereo:
        z = rng.uniform(4.0, 30.0, n).astype(np.float32)
        uright = (k2["x"] - np.float32(MB * FX) / z).astype(np.float32)
        uright[rng.random(n) < 0.3] = -1.0
    slot_mp = np.full(n, -1, np.int32)
    slot_obs = np.zeros(n, np.uint8)
    occ = rng.random(n)
    slot_mp[occ < 0.12] = 900000 + np.nonzero(occ < 0.12)[0]
    slot_obs[occ < 0.08] = 1  # occupied with observations; 0.08..0.12 occupied by a point without any
    return uright, slot_mp, slot_obs


def local_points(k1, d1, shift, seed, stereo):
    """(TRACK_POINT_DTYPE [m], descriptors [m, 32]) for SearchLocalPoints."""
    rng = np.random.default_rng(seed)
    n = len(k1)
    dup = rng.choice(n, n // 5, replace=False)  # a fifth of the points appear twice (fresh ids)
    src = np.concatenate([np.arange(n), dup])
    m = len(src)
    mp = np.zeros(m, TRACK_POINT_DTYPE)
    mp["id"] = np.arange(m)
    mp["proj_x"] = (k1["x"][src] + np.float32(shift[0]) + rng.normal(0, 1.0, m)).astype(np.float32)
    mp["proj_y"] = (k1["y"][src] + np.float32(shift[1]) + rng.normal(0, 1.0, m)).astype(np.float32)
    disp = rng.uniform(5.0, 60.0, m).astype(np.float32)
    mp["proj_xr"] = (mp["proj_x"] - disp) if stereo else np.float32(-1.0)
    mp["view_cos"] = rng.choice(np.array([0.9985, 0.9979, 0.99, 1.0], np.float32), m)
    lvl = k1["octave"][src] + rng.choice([-1, 0, 0, 0, 1], m)
    mp["level"] = np.clip(lvl, 0, 7)
    mp["in_view"] = rng.random(m) < 0.9
    mp["bad"] = rng.random(m) < 0.05
    mp["has_obs"] = rng.random(m) < 0.95
    return mp, np.ascontiguousarray(d1[src])


def _rot(ax, ay):
    cx, sx, cy, sy = np.cos(ax), np.sin(ax), np.cos(ay), np.sin(ay)
    Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    return Ry @ Rx


def last_frame(k1, d1, shift, w, h, seed, tz=0.0):
    """(Tcw, Tlw, LAST_POINT_DTYPE [n], descriptors): LastFrame at the origin,
    CurrentFrame rotated by the image shift and moved tz along its optical axis."""
    rng = np.random.default_rng(seed + 7)
    n = len(k1)
    fx, fy, cx, cy, _, _ = camera(w, h)
    z = rng.uniform(4.0, 40.0, n)
    X = np.stack([(k1["x"] - cx) / fx * z, (k1["y"] - cy) / fy * z, z], 1)
    lp = np.zeros(n, LAST_POINT_DTYPE)
    lp["id"] = np.where(rng.random(n) < 0.85, np.arange(n) + 5000, -1)
    lp["x"], lp["y"], lp["z"] = X[:, 0], X[:, 1], X[:, 2]
    lp["octave"] = k1["octave"]
    lp["angle"] = k1["angle"]
    lp["outlier"] = rng.random(n) < 0.05
    lp["has_obs"] = rng.random(n) < 0.8  # the rest: temporal stereo points (no observations)
    # points behind CurrentFrame and outside its image are part of the scene
    far = rng.random(n) < 0.03
    lp["z"][far] = -lp["z"][far]
    R = _rot(-shift[1] / fy, shift[0] / fx)  # u' ~ u + shift
    Tcw = np.zeros((3, 4), np.float32)
    Tcw[:, :3] = R
    Tcw[2, 3] = -tz
    Tlw = np.zeros((3, 4), np.float32)
    Tlw[:, :3] = np.eye(3)
    return Tcw, Tlw, lp, np.ascontiguousarray(d1)


MAP_POINT_DTYPE = np.dtype([("id", "<i4"), ("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("nx", "<f4"), ("ny", "<f4"),
                            ("nz", "<f4"), ("min_dist", "<f4"), ("max_dist", "<f4"), ("skip", "u1"),
                            ("pad", "u1", (3,))])


def keyframe_pose(shift, w, h, t=(0.0, 0.0, 0.0)):
    """3x4 Tcw of a keyframe that sees frame-1 content about `shift` pixels on."""
    R = _rot(-shift[1] / FY, shift[0] / FX)
    T = np.zeros((3, 4), np.float32)
    T[:, :3] = R
    T[:, 3] = t
    return T


def sim3_of(T, s):
    """Scw = [sR | s t] of a 3x4 Tcw."""
    return (np.asarray(T, np.float64) * s).astype(np.float32)


def map_points(k1, d1, w, h, seed, n_levels=8):
    """(MAP_POINT_DTYPE [n], descriptors): frame-1 keypoints back-projected at
    random depths from the origin, normals along the viewing ray (noisy),
    mfMaxDistance = dist * scale[octave], mfMinDistance = max / scale[n-1]
    (MapPoint ctor, MapPoint.cc:95-106); a few skipped (bad / already found)."""
    rng = np.random.default_rng(seed + 31)
    n = len(k1)
    fx, fy, cx, cy, _, _ = camera(w, h)
    z = rng.uniform(3.0, 40.0, n)
    X = np.stack([(k1["x"] - cx) / fx * z, (k1["y"] - cy) / fy * z, z], 1)
    dist = np.linalg.norm(X, axis=1)
    nrm = X / dist[:, None] + rng.normal(0, 0.2, (n, 3))
    nrm /= np.linalg.norm(nrm, axis=1)[:, None]
    sf = scale_factors(n_levels)
    mp = np.zeros(n, MAP_POINT_DTYPE)
    mp["id"] = np.arange(n) + 7000
    mp["x"], mp["y"], mp["z"] = X[:, 0], X[:, 1], X[:, 2]
    mp["nx"], mp["ny"], mp["nz"] = nrm[:, 0], nrm[:, 1], nrm[:, 2]
    mx = (dist * sf[np.clip(k1["octave"], 0, n_levels - 1)]).astype(np.float32)
    mp["max_dist"] = mx
    mp["min_dist"] = (mx / sf[-1]).astype(np.float32)
    mp["skip"] = rng.random(n) < 0.05
    return mp, np.ascontiguousarray(d1)


def bow_nodes(desc, seed, absent=0.08):
    """A stand-in DBoW2 FeatureVector: the node of a feature from its first
    descriptor byte (similar descriptors share nodes), some features absent."""
    rng = np.random.default_rng(seed + 57)
    node = (desc[:, 0].astype(np.int32) >> 3) * 37 + 1000
    node[rng.random(len(desc)) < absent] = -1
    return node


def bow_points(n, seed, frac=0.7, bad=0.05, base=0):
    """GetMapPointMatches ids (-1: NULL) and isBad() flags."""
    rng = np.random.default_rng(seed + 91)
    mp = np.where(rng.random(n) < frac, np.arange(n) + base, -1).astype(np.int32)
    return mp, (rng.random(n) < bad).astype(np.uint8)


def fundamental_12(T1w, T2w, cam1, cam2):
    """F12 (ComputeF12, LocalMapping.cc): K1^-T [t12]x R12 K2^-1 from 3x4 poses (float32)."""
    def K(c):
        return np.array([[c[0], 0, c[2]], [0, c[1], c[3]], [0, 0, 1.0]])
    R1, t1 = np.asarray(T1w[:, :3], np.float64), np.asarray(T1w[:, 3], np.float64)
    R2, t2 = np.asarray(T2w[:, :3], np.float64), np.asarray(T2w[:, 3], np.float64)
    R12 = R1 @ R2.T
    t12 = -R1 @ R2.T @ t2 + t1
    tx = np.array([[0, -t12[2], t12[1]], [t12[2], 0, -t12[0]], [-t12[1], t12[0], 0]])
    return (np.linalg.inv(K(cam1)).T @ tx @ R12 @ np.linalg.inv(K(cam2))).astype(np.float32)


def keyframe_points(k, d, T, w, h, seed, n_levels=8):
    """map_points for a keyframe with pose T (3x4 Tcw): its keypoints
    back-projected at random depths into the world."""
    mp, desc = map_points(k, d, w, h, seed, n_levels)
    R, t = np.asarray(T[:, :3], np.float64), np.asarray(T[:, 3], np.float64)
    Xc = np.stack([mp["x"], mp["y"], mp["z"]], 1).astype(np.float64)
    Xw = (Xc - t) @ R  # R^T (Xc - t)
    nw = np.stack([mp["nx"], mp["ny"], mp["nz"]], 1).astype(np.float64) @ R
    mp["x"], mp["y"], mp["z"] = Xw[:, 0], Xw[:, 1], Xw[:, 2]
    mp["nx"], mp["ny"], mp["nz"] = nw[:, 0], nw[:, 1], nw[:, 2]
    return mp, desc


def sim3_scene(k1, d1, k2, d2, shift, w, h, seed):
    """Two keyframes for SearchBySim3: T1w = I, T2w from the image shift plus a
    small translation, both map-point slot sets (a quarter NULL), S12 = their
    relative pose, and vpMatches12 with a few matches already in."""
    rng = np.random.default_rng(seed + 13)
    T1 = keyframe_pose((0.0, 0.0), w, h)
    T2 = keyframe_pose(shift, w, h, (0.05, 0.0, 0.02))
    mp1, md1 = map_points(k1, d1, w, h, seed)
    mp2, md2 = keyframe_points(k2, d2, T2, w, h, seed + 1)
    mp2["id"] = np.arange(len(mp2)) + 20000
    mp1["id"][rng.random(len(mp1)) < 0.25] = -1
    mp2["id"][rng.random(len(mp2)) < 0.25] = -1
    R2, t2 = T2[:, :3].astype(np.float64), T2[:, 3].astype(np.float64)
    R12 = R2.T.astype(np.float32)
    t12 = (-R2.T @ t2).astype(np.float32)
    m12 = np.full(len(k1), -1, np.int32)
    pick = rng.choice(len(k1), 20, replace=False)
    m12[pick] = rng.choice(mp2["id"][mp2["id"] >= 0], 20, replace=False)
    return T1, T2, mp1, md1, mp2, md2, R12, t12, m12
