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
