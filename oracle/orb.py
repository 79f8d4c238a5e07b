"""TEST INFRASTRUCTURE — ctypes binding of the ORB oracle (oracle/orb_ref.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this
module, as the checker. Parity statement: oracle/orb_ref.h.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .oracle import _p, build, lib  # noqa: F401 (build re-exported)

# cv::KeyPoint fields the reference uses (orc_kp / sqlm_keypoint layout)
KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                     ("octave", "<i4")])


class OrbParams(C.Structure):
    _fields_ = [("nfeatures", C.c_int), ("scale_factor", C.c_float), ("nlevels", C.c_int),
                ("ini_th_fast", C.c_int), ("min_th_fast", C.c_int)]


def params(nfeatures=2000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7) -> OrbParams:
    """cfg/KITTI00-02.yaml ORBextractor block (nFeatures 2000, scaleFactor 1.2, nLevels 8, 20 / 7)."""
    return OrbParams(nfeatures, scale_factor, nlevels, ini_th, min_th)


def levels(p, w, h):
    L = p.nlevels
    lw, lh, nf = (np.zeros(L, np.int32) for _ in range(3))
    sc = np.zeros(L, np.float32)
    r = lib().orc_orb_levels(C.byref(p), w, h, _p(lw), _p(lh), _p(nf), _p(sc))
    if r:
        raise ValueError(f"orc_orb_levels: {r}")
    return lw, lh, nf, sc


def resize(src, dw, dh):
    src = np.ascontiguousarray(src, np.uint8)
    out = np.zeros((dh, dw), np.uint8)
    lib().orc_orb_resize(_p(src), src.shape[1], src.shape[0], src.shape[1], _p(out), dw, dh, dw)
    return out


def blur(src):
    src = np.ascontiguousarray(src, np.uint8)
    out = np.zeros_like(src)
    lib().orc_orb_blur(_p(src), src.shape[1], src.shape[0], src.shape[1], _p(out), src.shape[1])
    return out


def gauss_kernel():
    k = np.zeros(7, np.int32)
    lib().orc_orb_gauss_kernel(_p(k))
    return k


def fast(img, th, cap=100000):
    img = np.ascontiguousarray(img, np.uint8)
    out = np.zeros(cap, KP_DTYPE)
    n = lib().orc_orb_fast(_p(img), img.shape[1], img.shape[1], img.shape[0], th, _p(out), cap)
    return out[:min(n, cap)]


def level_candidates(p, img, cap=400000):
    img = np.ascontiguousarray(img, np.uint8)
    out = np.zeros(cap, KP_DTYPE)
    n = lib().orc_orb_level_candidates(C.byref(p), _p(img), img.shape[1], img.shape[0], img.shape[1], _p(out), cap)
    return out[:min(n, cap)]


def distribute(keys, minX, maxX, minY, maxY, N):
    keys = np.ascontiguousarray(keys, KP_DTYPE)
    out = np.zeros(max(len(keys), 1), KP_DTYPE)
    n = lib().orc_orb_distribute(_p(keys), len(keys), minX, maxX, minY, maxY, N, _p(out))
    return out[:n]


def ic_angle(img, x, y):
    img = np.ascontiguousarray(img, np.uint8)
    f = lib().orc_orb_ic_angle
    f.restype = C.c_float
    return f(_p(img), img.shape[1], C.c_float(x), C.c_float(y))


def fast_atan2(y, x):
    f = lib().orc_fast_atan2
    f.restype = C.c_float
    return f(C.c_float(y), C.c_float(x))


def describe(img, kp):
    img = np.ascontiguousarray(img, np.uint8)
    k = np.ascontiguousarray(np.asarray(kp, KP_DTYPE).reshape(1))
    d = np.zeros(32, np.uint8)
    lib().orc_orb_describe(_p(img), img.shape[1], _p(k), _p(d))
    return d


def extract(p, img, cap=100000, with_levels=False):
    """ORBextractor::operator(): (keypoints KP_DTYPE, descriptors uint8 [n][32][, pyramid levels])."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    kps = np.zeros(cap, KP_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    lev = None
    if with_levels:
        lw, lh, _, _ = levels(p, w, h)
        lev = np.zeros(int(np.sum(lw.astype(np.int64) * lh)), np.uint8)
    n = lib().orc_orb_extract(C.byref(p), _p(img), w, h, w, _p(kps), _p(desc), cap, _p(lev))
    if n < 0:
        raise ValueError("orc_orb_extract failed")
    n = min(n, cap)
    if with_levels:
        lw, lh, _, _ = levels(p, w, h)
        offs = np.concatenate([[0], np.cumsum(lw.astype(np.int64) * lh)])
        pyr = [lev[offs[i]:offs[i + 1]].reshape(lh[i], lw[i]) for i in range(len(lw))]
        return kps[:n], desc[:n], pyr
    return kps[:n], desc[:n]


def hamming(a, b):
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    return lib().orc_hamming(_p(a), _p(b))


class FrameGrid(C.Structure):
    _fields_ = [("min_x", C.c_float), ("max_x", C.c_float), ("min_y", C.c_float), ("max_y", C.c_float)]


def search_for_init(k1, d1, k2, d2, grid, prev, window=100, nnratio=0.9, check_ori=True):
    """ORBmatcher(nnratio, check_ori).SearchForInitialization(F1, F2, prev, m12, window)
    -> (nmatches, m12, updated prev)."""
    k1 = np.ascontiguousarray(k1, KP_DTYPE)
    k2 = np.ascontiguousarray(k2, KP_DTYPE)
    d1 = np.ascontiguousarray(d1, np.uint8)
    d2 = np.ascontiguousarray(d2, np.uint8)
    prev = np.ascontiguousarray(prev, np.float32).copy()
    m12 = np.zeros(len(k1), np.int32)
    g = FrameGrid(*grid)
    n = lib().orc_search_for_init(_p(k1), _p(d1), len(k1), _p(k2), _p(d2), len(k2), C.byref(g), _p(prev), _p(m12),
                                  int(window), C.c_float(nnratio), int(bool(check_ori)))
    return n, m12, prev


# Projection searches (orb_ref.h orc_frame / orc_track_point / orc_last_point)
TRACK_POINT_DTYPE = np.dtype([("id", "<i4"), ("proj_x", "<f4"), ("proj_y", "<f4"), ("proj_xr", "<f4"),
                              ("view_cos", "<f4"), ("level", "<i4"), ("in_view", "u1"), ("bad", "u1"),
                              ("has_obs", "u1"), ("pad", "u1")])
LAST_POINT_DTYPE = np.dtype([("id", "<i4"), ("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("octave", "<i4"),
                             ("angle", "<f4"), ("outlier", "u1"), ("has_obs", "u1"), ("pad", "u1", (2,))])


class _Frame(C.Structure):
    _fields_ = [("kps", C.c_void_p), ("desc", C.c_void_p), ("uright", C.c_void_p), ("n", C.c_int),
                ("bounds", FrameGrid), ("scale_factors", C.c_void_p), ("n_levels", C.c_int),
                ("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float), ("bf", C.c_float),
                ("mb", C.c_float), ("slot_mp", C.c_void_p), ("slot_obs", C.c_void_p)]


def _frame(kps, desc, bounds, scale, cam, uright, slot_mp, slot_obs):
    """(struct, arrays kept alive, slot_mp copy, slot_obs copy)."""
    kps = np.ascontiguousarray(kps, KP_DTYPE)
    desc = np.ascontiguousarray(desc, np.uint8)
    scale = np.ascontiguousarray(scale, np.float32)
    uright = None if uright is None else np.ascontiguousarray(uright, np.float32)
    slot_mp = np.array(slot_mp, np.int32)
    slot_obs = np.array(slot_obs, np.uint8)
    f = _Frame()
    f.kps, f.desc, f.n = kps.ctypes.data, desc.ctypes.data, len(kps)
    f.uright = None if uright is None else uright.ctypes.data
    f.bounds = FrameGrid(*[float(v) for v in bounds])
    f.scale_factors, f.n_levels = scale.ctypes.data, len(scale)
    f.fx, f.fy, f.cx, f.cy, f.bf, f.mb = (float(v) for v in cam)
    f.slot_mp, f.slot_obs = slot_mp.ctypes.data, slot_obs.ctypes.data
    return f, (kps, desc, scale, uright), slot_mp, slot_obs


def features_in_area(kps, bounds, x, y, r, min_level=-1, max_level=-1):
    """Frame::GetFeaturesInArea (Frame.cc:1463-1552) -> keypoint indices."""
    n = len(kps)
    f, keep, _, _ = _frame(kps, np.zeros((n, 32), np.uint8), bounds, [1.0], (0,) * 6, None,
                           np.full(n, -1), np.zeros(n))
    out = np.zeros(max(n, 1), np.int32)
    m = lib().orc_features_in_area(C.byref(f), C.c_float(x), C.c_float(y), C.c_float(r), int(min_level),
                                   int(max_level), _p(out))
    return out[:m]


def search_by_projection_local(kps, desc, bounds, scale, uright, slot_mp, slot_obs, mps, mp_desc, th=1.0,
                               nnratio=0.6):
    """ORBmatcher(nnratio).SearchByProjection(F, vpMapPoints, th) -> (n, slot_mp, slot_obs)."""
    f, keep, sm, so = _frame(kps, desc, bounds, scale, (0,) * 6, uright, slot_mp, slot_obs)
    mps = np.ascontiguousarray(mps, TRACK_POINT_DTYPE)
    mp_desc = np.ascontiguousarray(mp_desc, np.uint8)
    n = lib().orc_search_by_projection_local(C.byref(f), _p(mps), _p(mp_desc), len(mps), C.c_float(th),
                                             C.c_float(nnratio))
    return n, sm, so


def search_by_projection_last(kps, desc, bounds, scale, cam, uright, slot_mp, slot_obs, Tcw, Tlw, lp, ldesc, th,
                              mono, check_ori=True):
    """ORBmatcher(., check_ori).SearchByProjection(CurrentFrame, LastFrame, th, bMono)
    -> (n, slot_mp, slot_obs). cam = (fx, fy, cx, cy, mbf, mb)."""
    f, keep, sm, so = _frame(kps, desc, bounds, scale, cam, uright, slot_mp, slot_obs)
    Tcw = np.ascontiguousarray(np.asarray(Tcw, np.float32)[:3, :4])
    Tlw = np.ascontiguousarray(np.asarray(Tlw, np.float32)[:3, :4])
    lp = np.ascontiguousarray(lp, LAST_POINT_DTYPE)
    ldesc = np.ascontiguousarray(ldesc, np.uint8)
    n = lib().orc_search_by_projection_last(C.byref(f), _p(Tcw), _p(Tlw), _p(lp), _p(ldesc), len(lp),
                                            C.c_float(th), int(bool(mono)), int(bool(check_ori)))
    return n, sm, so


MAP_POINT_DTYPE = np.dtype([("id", "<i4"), ("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("nx", "<f4"), ("ny", "<f4"),
                            ("nz", "<f4"), ("min_dist", "<f4"), ("max_dist", "<f4"), ("skip", "u1"),
                            ("pad", "u1", (3,))])


def search_by_projection_sim3(kps, desc, bounds, scale, cam, slot_mp, Scw, mps, mp_desc, th):
    """SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) -> (n, vpMatched)."""
    n = len(kps)
    f, keep, sm, _ = _frame(kps, desc, bounds, scale, cam, None, slot_mp, np.zeros(n))
    S = np.ascontiguousarray(np.asarray(Scw, np.float32)[:3, :4])
    mps = np.ascontiguousarray(mps, MAP_POINT_DTYPE)
    r = lib().orc_search_by_projection_sim3(C.byref(f), _p(S), _p(mps), _p(np.ascontiguousarray(mp_desc, np.uint8)),
                                            len(mps), int(th))
    return r, sm


def fuse(kps, desc, bounds, scale, cam, uright, T, sim3, mps, mp_desc, th):
    """Fuse(pKF, vpMapPoints, th) (sim3 False, T = Tcw) / Fuse(pKF, Scw, ...) -> (nFused, fuse_idx)."""
    n = len(kps)
    f, keep, _, _ = _frame(kps, desc, bounds, scale, cam, uright, np.full(n, -1), np.zeros(n))
    T = np.ascontiguousarray(np.asarray(T, np.float32)[:3, :4])
    mps = np.ascontiguousarray(mps, MAP_POINT_DTYPE)
    out = np.zeros(max(len(mps), 1), np.int32)
    r = lib().orc_fuse(C.byref(f), _p(T), int(bool(sim3)), _p(mps), _p(np.ascontiguousarray(mp_desc, np.uint8)),
                       len(mps), C.c_float(th), _p(out))
    return r, out[:len(mps)]


def search_by_projection_kf(kps, desc, bounds, scale, cam, slot_mp, Tcw, mps, mp_desc, kf_angle, th, orb_dist,
                            check_ori=True):
    """SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) -> (n, mvpMapPoints)."""
    n = len(kps)
    f, keep, sm, _ = _frame(kps, desc, bounds, scale, cam, None, slot_mp, np.zeros(n))
    T = np.ascontiguousarray(np.asarray(Tcw, np.float32)[:3, :4])
    mps = np.ascontiguousarray(mps, MAP_POINT_DTYPE)
    ang = np.ascontiguousarray(kf_angle, np.float32)
    r = lib().orc_search_by_projection_kf(C.byref(f), _p(T), _p(mps), _p(np.ascontiguousarray(mp_desc, np.uint8)),
                                          _p(ang), len(mps), C.c_float(th), int(orb_dist), int(bool(check_ori)))
    return r, sm


class _BowFrame(C.Structure):
    _fields_ = [("kps", C.c_void_p), ("desc", C.c_void_p), ("node", C.c_void_p), ("mp", C.c_void_p),
                ("mp_bad", C.c_void_p), ("uright", C.c_void_p), ("n", C.c_int)]


def _bow(kps, desc, node, mp, mp_bad=None, uright=None):
    arrs = [np.ascontiguousarray(kps, KP_DTYPE), np.ascontiguousarray(desc, np.uint8),
            np.ascontiguousarray(node, np.int32), np.ascontiguousarray(mp, np.int32),
            None if mp_bad is None else np.ascontiguousarray(mp_bad, np.uint8),
            None if uright is None else np.ascontiguousarray(uright, np.float32)]
    b = _BowFrame()
    b.kps, b.desc, b.node, b.mp = (a.ctypes.data for a in arrs[:4])
    b.mp_bad = None if arrs[4] is None else arrs[4].ctypes.data
    b.uright = None if arrs[5] is None else arrs[5].ctypes.data
    b.n = len(arrs[0])
    return b, arrs


def search_by_bow_kf_frame(kf, f, nnratio=0.7, check_ori=True):
    """SearchByBoW(pKF, F, vpMapPointMatches); kf / f = (kps, desc, node, mp[, mp_bad[, uright]])."""
    a, ka = _bow(*kf)
    b, kb = _bow(*f)
    out = np.zeros(max(b.n, 1), np.int32)
    r = lib().orc_search_by_bow_kf_frame(C.byref(a), C.byref(b), C.c_float(nnratio), int(bool(check_ori)), _p(out))
    return r, out[:b.n]


def search_by_bow_kf_kf(k1, k2, nnratio=0.75, check_ori=True):
    """SearchByBoW(pKF1, pKF2, vpMatches12)."""
    a, ka = _bow(*k1)
    b, kb = _bow(*k2)
    out = np.zeros(max(a.n, 1), np.int32)
    r = lib().orc_search_by_bow_kf_kf(C.byref(a), C.byref(b), C.c_float(nnratio), int(bool(check_ori)), _p(out))
    return r, out[:a.n]


def search_for_triangulation(k1, k2, C1, T2w, cam2, scale2, F12, only_stereo, check_ori=False):
    """SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, bOnlyStereo) -> (n, m12)."""
    a, ka = _bow(*k1)
    b, kb = _bow(*k2)
    C1 = np.ascontiguousarray(C1, np.float32)
    T = np.ascontiguousarray(np.asarray(T2w, np.float32)[:3, :4])
    cam2 = np.ascontiguousarray(cam2, np.float32)
    s2 = np.ascontiguousarray(scale2, np.float32)
    F = np.ascontiguousarray(F12, np.float32)
    out = np.zeros(max(a.n, 1), np.int32)
    r = lib().orc_search_for_triangulation(C.byref(a), C.byref(b), _p(C1), _p(T), _p(cam2), _p(s2), _p(F),
                                           int(bool(only_stereo)), int(bool(check_ori)), _p(out))
    return r, out[:a.n]


def search_by_sim3(k1, d1, k2, d2, bounds, scale, cam, T1w, T2w, mp1, md1, mp2, md2, s12, R12, t12, th, matches12):
    """SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th) -> (nFound, vpMatches12)."""
    n1, n2 = len(k1), len(k2)
    f1, keep1, _, _ = _frame(k1, d1, bounds, scale, cam, None, np.full(n1, -1), np.zeros(n1))
    f2, keep2, _, _ = _frame(k2, d2, bounds, scale, cam, None, np.full(n2, -1), np.zeros(n2))
    arr = [np.ascontiguousarray(np.asarray(T, np.float32)[:3, :4]) for T in (T1w, T2w)]
    mp1 = np.ascontiguousarray(mp1, MAP_POINT_DTYPE)
    mp2 = np.ascontiguousarray(mp2, MAP_POINT_DTYPE)
    md1 = np.ascontiguousarray(md1, np.uint8)
    md2 = np.ascontiguousarray(md2, np.uint8)
    R = np.ascontiguousarray(R12, np.float32)
    t = np.ascontiguousarray(t12, np.float32)
    m = np.array(matches12, np.int32)
    r = lib().orc_search_by_sim3(C.byref(f1), C.byref(f2), _p(arr[0]), _p(arr[1]), _p(mp1), _p(md1), _p(mp2),
                                 _p(md2), C.c_float(s12), _p(R), _p(t), C.c_float(th), _p(m))
    return r, m
