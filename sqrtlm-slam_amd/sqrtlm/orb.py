"""Host-side mirror of the reference's ORB front end over the C ABI
(include/sqrtlm_orb.h): ``ORBextractor`` (include/frontend/ORBextractor.h,
src/frontend/ORBextractor.cc) and the Hamming part of ``ORBmatcher``
(src/frontend/ORBmatcher.cc). Same names, argument meaning and defaults as the
reference; the work runs on the GPU (libsqrtlm.so), there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, lib, ptr
from .optimizer import Context

# cv::KeyPoint fields the reference uses (sqlm_keypoint)
KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                     ("octave", "<i4")])



# MapPoint tracking fields of one local map point (sqlm_track_point)
TRACK_POINT_DTYPE = np.dtype([("id", "<i4"), ("proj_x", "<f4"), ("proj_y", "<f4"), ("proj_xr", "<f4"),
                              ("view_cos", "<f4"), ("level", "<i4"), ("in_view", "u1"), ("bad", "u1"),
                              ("has_obs", "u1"), ("pad", "u1")])
# one LastFrame keypoint slot (sqlm_last_point)
LAST_POINT_DTYPE = np.dtype([("id", "<i4"), ("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("octave", "<i4"),
                             ("angle", "<f4"), ("outlier", "u1"), ("has_obs", "u1"), ("pad", "u1", (2,))])


# a map point as the keyframe searches read it (sqlm_map_point)
MAP_POINT_DTYPE = np.dtype([("id", "<i4"), ("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("nx", "<f4"), ("ny", "<f4"),
                            ("nz", "<f4"), ("min_dist", "<f4"), ("max_dist", "<f4"), ("skip", "u1"),
                            ("pad", "u1", (3,))])


class OrbParams(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32)]


class FrameBounds(C.Structure):
    _fields_ = [("min_x", C.c_float), ("max_x", C.c_float), ("min_y", C.c_float), ("max_y", C.c_float)]


class _OrbFrame(C.Structure):
    _fields_ = [("kps", C.c_void_p), ("desc", C.c_void_p), ("uright", C.c_void_p), ("n", C.c_int32),
                ("bounds", FrameBounds), ("scale_factors", C.c_void_p), ("n_levels", C.c_int32),
                ("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float), ("bf", C.c_float),
                ("mb", C.c_float), ("slot_mp", C.c_void_p), ("slot_obs", C.c_void_p)]


class Frame:
    """The Frame fields ORBmatcher's projection searches read and write
    (include/data_structure/Frame.h): mvKeysUn, mDescriptors, mvuRight (None:
    monocular), the grid bounds (mnMinX, mnMaxX, mnMinY, mnMaxY),
    mvScaleFactors, fx fy cx cy, mbf, mb, mTcw, and the keypoint slots
    mvpMapPoints as map-point ids (-1 = NULL) with slot_obs = that point's
    Observations() > 0; the searches update the last two in place."""

    def __init__(self, mvKeysUn, mDescriptors, bounds, mvScaleFactors, fx, fy, cx, cy, mbf=0.0, mb=0.0,
                 mvuRight=None, mTcw=None, mvpMapPoints=None, slot_obs=None):
        self.mvKeysUn = np.ascontiguousarray(mvKeysUn, KP_DTYPE)
        n = len(self.mvKeysUn)
        self.N = n
        self.mDescriptors = np.ascontiguousarray(mDescriptors, np.uint8).reshape(n, 32)
        self.bounds = tuple(float(v) for v in bounds)
        self.mvScaleFactors = np.ascontiguousarray(mvScaleFactors, np.float32)
        self.fx, self.fy, self.cx, self.cy, self.mbf, self.mb = (float(v) for v in (fx, fy, cx, cy, mbf, mb))
        self.mvuRight = None if mvuRight is None else np.ascontiguousarray(mvuRight, np.float32)
        if self.mvuRight is not None and self.mvuRight.shape != (n,):
            raise ValueError("mvuRight must hold one entry per keypoint")
        self.mTcw = None if mTcw is None else np.ascontiguousarray(np.asarray(mTcw, np.float32)[:3, :4])
        self.mvpMapPoints = np.full(n, -1, np.int32) if mvpMapPoints is None else np.ascontiguousarray(
            mvpMapPoints, np.int32)
        self.slot_obs = (self.mvpMapPoints >= 0).astype(np.uint8) if slot_obs is None else np.ascontiguousarray(
            slot_obs, np.uint8)
        if self.mvpMapPoints.shape != (n,) or self.slot_obs.shape != (n,):
            raise ValueError("mvpMapPoints / slot_obs must hold one entry per keypoint")

    def _struct(self) -> _OrbFrame:
        f = _OrbFrame()
        f.kps, f.desc = self.mvKeysUn.ctypes.data, self.mDescriptors.ctypes.data
        f.uright = None if self.mvuRight is None else self.mvuRight.ctypes.data
        f.n = self.N
        f.bounds = FrameBounds(*self.bounds)
        f.scale_factors, f.n_levels = self.mvScaleFactors.ctypes.data, len(self.mvScaleFactors)
        f.fx, f.fy, f.cx, f.cy, f.bf, f.mb = self.fx, self.fy, self.cx, self.cy, self.mbf, self.mb
        f.slot_mp, f.slot_obs = self.mvpMapPoints.ctypes.data, self.slot_obs.ctypes.data
        return f


class LastFrameSlots:
    """LastFrame as SearchByProjection(CurrentFrame, LastFrame, ...) reads it:
    mTcw and, per keypoint slot, LAST_POINT_DTYPE (mvpMapPoints id, world
    position, mvKeys octave, mvKeysUn angle, mvbOutlier, Observations() > 0)
    with the points' descriptors [N, 32]."""

    def __init__(self, mTcw, slots, descriptors):
        self.mTcw = np.ascontiguousarray(np.asarray(mTcw, np.float32)[:3, :4])
        self.slots = np.ascontiguousarray(slots, LAST_POINT_DTYPE)
        self.descriptors = np.ascontiguousarray(descriptors, np.uint8).reshape(len(self.slots), 32)


class KeyFrameSlots:
    """pKF as SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist)
    reads it: its map-point slots MAP_POINT_DTYPE [N] (skip set for NULL, bad
    and already-found slots), their descriptors and mvKeysUn[i].angle."""

    def __init__(self, slots, descriptors, angles):
        self.slots = np.ascontiguousarray(slots, MAP_POINT_DTYPE)
        self.descriptors = np.ascontiguousarray(descriptors, np.uint8).reshape(len(self.slots), 32)
        self.angles = np.ascontiguousarray(angles, np.float32)


class _BowFrame(C.Structure):
    _fields_ = [("kps", C.c_void_p), ("desc", C.c_void_p), ("node", C.c_void_p), ("mp", C.c_void_p),
                ("mp_bad", C.c_void_p), ("uright", C.c_void_p), ("n", C.c_int32)]


def _f32_mat3_mul(R, x):
    """cv::Mat 3x3 * 3x1 on CV_32F: float products summed left to right."""
    f32 = np.float32
    return [f32(f32(R[i][0]) * f32(x[0]) + f32(R[i][1]) * f32(x[1]) + f32(R[i][2]) * f32(x[2])) for i in range(3)]


class BowFrame:
    """A KeyFrame (keyframe=True) or Frame as the BoW searches read it:
    mvKeysUn, mDescriptors, the DBoW2 FeatureVector as one node id per feature
    (-1: not in mFeatVec), GetMapPointMatches() ids (-1: NULL) with isBad(),
    mvuRight, and for SearchForTriangulation the pose Tcw (3x4), fx fy cx cy and
    mvScaleFactors."""

    def __init__(self, mvKeysUn, mDescriptors, node, mapPoints=None, mapPointBad=None, mvuRight=None,
                 keyframe=True, Tcw=None, cam=None, mvScaleFactors=None):
        self.mvKeysUn = np.ascontiguousarray(mvKeysUn, KP_DTYPE)
        n = self.N = len(self.mvKeysUn)
        self.mDescriptors = np.ascontiguousarray(mDescriptors, np.uint8).reshape(n, 32)
        self.node = np.ascontiguousarray(node, np.int32)
        self.mp = np.full(n, -1, np.int32) if mapPoints is None else np.ascontiguousarray(mapPoints, np.int32)
        self.mp_bad = None if mapPointBad is None else np.ascontiguousarray(mapPointBad, np.uint8)
        self.mvuRight = None if mvuRight is None else np.ascontiguousarray(mvuRight, np.float32)
        for a in (self.node, self.mp, self.mp_bad, self.mvuRight):
            if a is not None and a.shape != (n,):
                raise ValueError("per-feature arrays must hold one entry per keypoint")
        self.keyframe = bool(keyframe)
        self.Tcw = None if Tcw is None else np.ascontiguousarray(np.asarray(Tcw, np.float32)[:3, :4])
        self.cam = None if cam is None else np.ascontiguousarray(cam, np.float32)[:4]
        self.mvScaleFactors = None if mvScaleFactors is None else np.ascontiguousarray(mvScaleFactors, np.float32)

    def GetCameraCenter(self):
        """Ow = -R^T t (KeyFrame::SetPose), float as cv::Mat computes it."""
        t = self.Tcw[:, 3]
        return np.array([-v for v in _f32_mat3_mul(self.Tcw[:, :3].T, t)], np.float32)

    def _struct(self) -> _BowFrame:
        b = _BowFrame()
        b.kps, b.desc, b.node, b.mp = (a.ctypes.data for a in (self.mvKeysUn, self.mDescriptors, self.node, self.mp))
        b.mp_bad = None if self.mp_bad is None else self.mp_bad.ctypes.data
        b.uright = None if self.mvuRight is None else self.mvuRight.ctypes.data
        b.n = self.N
        return b


class ORBextractor:
    """ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)
    (ORBextractor.cc:474-560). ``extractor(image)`` is operator()
    (:1284-1399): returns (keypoints KP_DTYPE[n], descriptors uint8[n, 32])."""

    def __init__(self, nfeatures: int = 2000, scaleFactor: float = 1.2, nlevels: int = 8, iniThFAST: int = 20,
                 minThFAST: int = 7, ctx: Context | None = None):
        self.params = OrbParams(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)
        self._own = ctx is None
        self.ctx = ctx if ctx is not None else Context(-1)
        sf = [np.float32(1.0)]
        for _ in range(1, nlevels):
            sf.append(np.float32(sf[-1] * np.float32(scaleFactor)))
        self.mvScaleFactor = np.array(sf, np.float32)
        self.mvLevelSigma2 = (self.mvScaleFactor * self.mvScaleFactor).astype(np.float32)
        self.mvInvScaleFactor = (np.float32(1.0) / self.mvScaleFactor).astype(np.float32)
        self.mvInvLevelSigma2 = (np.float32(1.0) / self.mvLevelSigma2).astype(np.float32)

    def __call__(self, image: np.ndarray):
        img = np.ascontiguousarray(image, np.uint8)
        if img.ndim != 2:
            raise ValueError("ORBextractor expects a CV_8UC1 image")
        h, w = img.shape
        cap = max(64, 2 * int(self.params.nfeatures))
        while True:
            kps = np.zeros(cap, KP_DTYPE)
            desc = np.zeros((cap, 32), np.uint8)
            n = C.c_int(0)
            check(lib().sqlm_orb_extract(self.ctx._h, C.byref(self.params), ptr(img), w, h, w, ptr(kps), ptr(desc),
                                         cap, C.byref(n)), "sqlm_orb_extract")
            if n.value <= cap:
                return kps[:n.value], desc[:n.value]
            cap = n.value

    def GetLevels(self) -> int:
        return int(self.params.nlevels)

    def GetScaleFactor(self) -> float:
        return float(self.params.scale_factor)

    def GetScaleFactors(self):
        return self.mvScaleFactor

    def GetInverseScaleFactors(self):
        return self.mvInvScaleFactor

    def GetScaleSigmaSquares(self):
        return self.mvLevelSigma2

    def GetInverseScaleSigmaSquares(self):
        return self.mvInvLevelSigma2

    def image_pyramid(self):
        """mvImagePyramid of the last call (level images without the border)."""
        out = []
        for lvl in range(self.params.nlevels):
            lw, lh = C.c_int(0), C.c_int(0)
            # first call: size query (returns INVALID_ARG for the missing buffer, sizes are set)
            lib().sqlm_orb_get_level(self.ctx._h, lvl, None, 0, C.byref(lw), C.byref(lh))
            buf = np.zeros((lh.value, lw.value), np.uint8)
            check(lib().sqlm_orb_get_level(self.ctx._h, lvl, ptr(buf), buf.size, C.byref(lw), C.byref(lh)),
                  "sqlm_orb_get_level")
            out.append(buf)
        return out

    def bench(self, image: np.ndarray, reps: int = 50):
        """(ms per frame, stage ms [pyramid, fast, compact, blur, describe, host quadtree])."""
        img = np.ascontiguousarray(image, np.uint8)
        ms = C.c_double(0)
        st = (C.c_double * 6)()
        check(lib().sqlm_orb_bench_extract(self.ctx._h, C.byref(self.params), ptr(img), img.shape[1], img.shape[0],
                                           img.shape[1], int(reps), C.byref(ms), st), "sqlm_orb_bench_extract")
        return ms.value, list(st)

    def close(self):
        if self._own:
            self.ctx.close()


class ORBmatcher:
    """ORBmatcher(nnratio=0.6, checkOri=true) (ORBmatcher.cc:50-51)."""

    TH_HIGH = 100
    TH_LOW = 50
    HISTO_LENGTH = 30

    def __init__(self, nnratio: float = 0.6, checkOri: bool = True, ctx: Context | None = None):
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)
        self.ctx = ctx if ctx is not None else Context(-1)

    def match_bf(self, query: np.ndarray, train: np.ndarray):
        """Brute force over all train descriptors: (best_idx, best_dist, second_dist) per query."""
        q = np.ascontiguousarray(query, np.uint8).reshape(-1, 32)
        t = np.ascontiguousarray(train, np.uint8).reshape(-1, 32)
        bi, bd, bd2 = (np.zeros(len(q), np.int32) for _ in range(3))
        check(lib().sqlm_orb_match_bf(self.ctx._h, ptr(q), len(q), ptr(t), len(t), ptr(bi), ptr(bd), ptr(bd2)),
              "sqlm_orb_match_bf")
        return bi, bd, bd2

    def DescriptorDistance(self, a: np.ndarray, b: np.ndarray) -> int:
        """ORBmatcher::DescriptorDistance (ORBmatcher.cc:2096-2116), on the GPU."""
        _, d, _ = self.match_bf(np.asarray(a, np.uint8).reshape(1, 32), np.asarray(b, np.uint8).reshape(1, 32))
        return int(d[0])

    def SearchForInitialization(self, k1, d1, k2, d2, bounds2, vbPrevMatched, windowSize: int = 10):
        """SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize)
        (ORBmatcher.cc:573-718). k1/d1, k2/d2: mvKeysUn / mDescriptors of F1 and
        F2; bounds2 = (mnMinX, mnMaxX, mnMinY, mnMaxY) of F2; vbPrevMatched
        float32 [n1, 2] is updated in place. Returns (nmatches, vnMatches12)."""
        k1 = np.ascontiguousarray(k1, KP_DTYPE)
        k2 = np.ascontiguousarray(k2, KP_DTYPE)
        d1 = np.ascontiguousarray(d1, np.uint8)
        d2 = np.ascontiguousarray(d2, np.uint8)
        if vbPrevMatched.dtype != np.float32 or not vbPrevMatched.flags.c_contiguous:
            raise ValueError("vbPrevMatched must be a C-contiguous float32 [n1, 2] array (updated in place)")
        m12 = np.zeros(len(k1), np.int32)
        n = C.c_int(0)
        fb = FrameBounds(*[float(v) for v in bounds2])
        check(lib().sqlm_orb_search_for_init(self.ctx._h, ptr(k1), ptr(d1), len(k1), ptr(k2), ptr(d2), len(k2),
                                             C.byref(fb), ptr(vbPrevMatched), ptr(m12), int(windowSize),
                                             C.c_float(self.mfNNratio), int(self.mbCheckOrientation), C.byref(n)),
              "sqlm_orb_search_for_init")
        return n.value, m12

    def SearchByProjection(self, F: Frame, second, *args):
        """The projection searches on the GPU candidate windows (F.mvpMapPoints
        / F.slot_obs updated in place; returns nmatches):

        - ``SearchByProjection(F, vpMapPoints, descriptors, th=1.0)``
          (ORBmatcher.cc:67-181): vpMapPoints TRACK_POINT_DTYPE [n] as
          Tracking::SearchLocalPoints leaves them, descriptors [n, 32];
        - ``SearchByProjection(CurrentFrame, LastFrame, th, bMono)``
          (ORBmatcher.cc:1717-1883): LastFrame a LastFrameSlots, CurrentFrame.mTcw set;
        - ``SearchByProjection(pKF, Scw, vpPoints, descriptors, th)``
          (ORBmatcher.cc:423-571): vpMatched = pKF.mvpMapPoints, vpPoints
          MAP_POINT_DTYPE (skip = isBad() or already in vpMatched);
        - ``SearchByProjection(CurrentFrame, pKF, th, ORBdist)``
          (ORBmatcher.cc:1902-2046): pKF a KeyFrameSlots, CurrentFrame.mTcw set."""
        n = C.c_int(0)
        fs = F._struct()
        if isinstance(second, LastFrameSlots):
            if len(args) != 2:
                raise TypeError("SearchByProjection(CurrentFrame, LastFrame, th, bMono)")
            th, bMono = args
            if F.mTcw is None:
                raise ValueError("CurrentFrame.mTcw is not set")
            L = second
            check(lib().sqlm_orb_search_by_projection_last(
                self.ctx._h, C.byref(fs), ptr(F.mTcw), ptr(L.mTcw), ptr(L.slots), ptr(L.descriptors), len(L.slots),
                C.c_float(th), int(bool(bMono)), int(self.mbCheckOrientation), C.byref(n)),
                "sqlm_orb_search_by_projection_last")
            return n.value
        if isinstance(second, KeyFrameSlots):
            if len(args) != 2:
                raise TypeError("SearchByProjection(CurrentFrame, pKF, th, ORBdist)")
            if F.mTcw is None:
                raise ValueError("CurrentFrame.mTcw is not set")
            th, orb_dist = args
            K = second
            check(lib().sqlm_orb_search_by_projection_kf(
                self.ctx._h, C.byref(fs), ptr(F.mTcw), ptr(K.slots), ptr(K.descriptors), ptr(K.angles), len(K.slots),
                C.c_float(th), int(orb_dist), int(self.mbCheckOrientation), C.byref(n)),
                "sqlm_orb_search_by_projection_kf")
            return n.value
        if isinstance(second, np.ndarray) and second.dtype.kind == "f" and second.shape in ((3, 4), (4, 4)):
            if len(args) != 3:
                raise TypeError("SearchByProjection(pKF, Scw, vpPoints, descriptors, th)")
            Scw = np.ascontiguousarray(second[:3, :4], np.float32)
            pts = np.ascontiguousarray(args[0], MAP_POINT_DTYPE)
            desc = np.ascontiguousarray(args[1], np.uint8).reshape(len(pts), 32)
            check(lib().sqlm_orb_search_by_projection_sim3(self.ctx._h, C.byref(fs), ptr(Scw), ptr(pts), ptr(desc),
                                                           len(pts), int(args[2]), C.byref(n)),
                  "sqlm_orb_search_by_projection_sim3")
            return n.value
        if len(args) not in (1, 2):
            raise TypeError("SearchByProjection(F, vpMapPoints, descriptors, th=1.0)")
        third, th = args[0], (args[1] if len(args) == 2 else 1.0)
        mps = np.ascontiguousarray(second, TRACK_POINT_DTYPE)
        desc = np.ascontiguousarray(third, np.uint8).reshape(len(mps), 32)
        check(lib().sqlm_orb_search_by_projection_local(self.ctx._h, C.byref(fs), ptr(mps), ptr(desc), len(mps),
                                                        C.c_float(th), C.c_float(self.mfNNratio), C.byref(n)),
              "sqlm_orb_search_by_projection_local")
        return n.value

    def Fuse(self, pKF: Frame, *args):
        """Fuse(pKF, vpMapPoints, descriptors, th=3.0) (ORBmatcher.cc:1109-1294,
        pKF.mTcw set) or Fuse(pKF, Scw, vpPoints, descriptors, th)
        (:1296-1446). Points MAP_POINT_DTYPE (skip = isBad() or already in
        pKF). Returns (nFused, fuse_idx): the keypoint each point fuses into
        (-1: none); MapPoint::Replace / AddObservation are the caller's."""
        if args and isinstance(args[0], np.ndarray) and args[0].dtype.kind == "f" and args[0].shape in ((3, 4),
                                                                                                       (4, 4)):
            T, sim3, rest = np.ascontiguousarray(args[0][:3, :4], np.float32), 1, args[1:]
            if len(rest) != 3:
                raise TypeError("Fuse(pKF, Scw, vpPoints, descriptors, th)")
        else:
            if pKF.mTcw is None:
                raise ValueError("pKF.mTcw is not set")
            T, sim3, rest = pKF.mTcw, 0, args
            if len(rest) == 2:
                rest = (*rest, 3.0)
            if len(rest) != 3:
                raise TypeError("Fuse(pKF, vpMapPoints, descriptors, th=3.0)")
        pts = np.ascontiguousarray(rest[0], MAP_POINT_DTYPE)
        desc = np.ascontiguousarray(rest[1], np.uint8).reshape(len(pts), 32)
        idx = np.zeros(len(pts), np.int32)
        n = C.c_int(0)
        fs = pKF._struct()
        check(lib().sqlm_orb_fuse(self.ctx._h, C.byref(fs), ptr(T), int(sim3), ptr(pts), ptr(desc), len(pts),
                                  C.c_float(rest[2]), ptr(idx), C.byref(n)), "sqlm_orb_fuse")
        return n.value, idx

    def SearchByBoW(self, pKF: BowFrame, second: BowFrame):
        """SearchByBoW(pKF, F) (ORBmatcher.cc:246-403; second.keyframe False):
        (nmatches, vpMapPointMatches [F.N] ids); SearchByBoW(pKF1, pKF2)
        (:731-869): (nmatches, vpMatches12 [pKF1.N] ids of pKF2's points)."""
        n = C.c_int(0)
        a, b = pKF._struct(), second._struct()
        if second.keyframe:
            out = np.zeros(pKF.N, np.int32)
            check(lib().sqlm_orb_search_by_bow_kf_kf(self.ctx._h, C.byref(a), C.byref(b), C.c_float(self.mfNNratio),
                                                     int(self.mbCheckOrientation), ptr(out), C.byref(n)),
                  "sqlm_orb_search_by_bow_kf_kf")
        else:
            out = np.zeros(second.N, np.int32)
            check(lib().sqlm_orb_search_by_bow_kf_frame(self.ctx._h, C.byref(a), C.byref(b),
                                                        C.c_float(self.mfNNratio), int(self.mbCheckOrientation),
                                                        ptr(out), C.byref(n)), "sqlm_orb_search_by_bow_kf_frame")
        return n.value, out

    def SearchForTriangulation(self, pKF1: BowFrame, pKF2: BowFrame, F12, bOnlyStereo: bool):
        """SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, bOnlyStereo)
        (ORBmatcher.cc:887-1096) -> (nmatches, vMatchedPairs as [(i1, i2)])."""
        if pKF1.Tcw is None or pKF2.Tcw is None or pKF2.cam is None or pKF2.mvScaleFactors is None:
            raise ValueError("pKF1.Tcw, pKF2.Tcw, pKF2.cam and pKF2.mvScaleFactors are required")
        F = np.ascontiguousarray(F12, np.float32).reshape(3, 3)
        C1 = pKF1.GetCameraCenter()
        m12 = np.zeros(pKF1.N, np.int32)
        n = C.c_int(0)
        a, b = pKF1._struct(), pKF2._struct()
        check(lib().sqlm_orb_search_for_triangulation(
            self.ctx._h, C.byref(a), C.byref(b), ptr(C1), ptr(pKF2.Tcw), ptr(pKF2.cam), ptr(pKF2.mvScaleFactors),
            len(pKF2.mvScaleFactors), ptr(F), int(bool(bOnlyStereo)), int(self.mbCheckOrientation), ptr(m12),
            C.byref(n)), "sqlm_orb_search_for_triangulation")
        i1 = np.nonzero(m12 >= 0)[0]
        return n.value, [(int(i), int(m12[i])) for i in i1]

    def SearchBySim3(self, pKF1: Frame, pKF2: Frame, mapPoints1, descriptors1, mapPoints2, descriptors2,
                     vpMatches12, s12: float, R12, t12, th: float):
        """SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th)
        (ORBmatcher.cc:1448-1608). pKF1 / pKF2 Frames with mTcw; mapPoints1 /
        mapPoints2 their slots MAP_POINT_DTYPE [N] (id -1: NULL, skip: isBad());
        vpMatches12 int32 [pKF1.N] ids, updated in place. Returns nFound."""
        if pKF1.mTcw is None or pKF2.mTcw is None:
            raise ValueError("pKF1.mTcw and pKF2.mTcw are required")
        m1 = np.ascontiguousarray(mapPoints1, MAP_POINT_DTYPE)
        m2 = np.ascontiguousarray(mapPoints2, MAP_POINT_DTYPE)
        if len(m1) != pKF1.N or len(m2) != pKF2.N:
            raise ValueError("one map-point slot per keypoint")
        d1 = np.ascontiguousarray(descriptors1, np.uint8).reshape(len(m1), 32)
        d2 = np.ascontiguousarray(descriptors2, np.uint8).reshape(len(m2), 32)
        if vpMatches12.dtype != np.int32 or not vpMatches12.flags.c_contiguous or vpMatches12.shape != (pKF1.N,):
            raise ValueError("vpMatches12 must be a C-contiguous int32 [pKF1.N] array (updated in place)")
        R = np.ascontiguousarray(R12, np.float32).reshape(3, 3)
        t = np.ascontiguousarray(t12, np.float32).reshape(3)
        n = C.c_int(0)
        a, b = pKF1._struct(), pKF2._struct()
        check(lib().sqlm_orb_search_by_sim3(self.ctx._h, C.byref(a), C.byref(b), ptr(pKF1.mTcw), ptr(pKF2.mTcw),
                                            ptr(m1), ptr(d1), ptr(m2), ptr(d2), C.c_float(s12), ptr(R), ptr(t),
                                            C.c_float(th), ptr(vpMatches12), C.byref(n)), "sqlm_orb_search_by_sim3")
        return n.value
