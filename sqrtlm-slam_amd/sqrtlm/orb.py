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



class OrbParams(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32)]


class FrameBounds(C.Structure):
    _fields_ = [("min_x", C.c_float), ("max_x", C.c_float), ("min_y", C.c_float), ("max_y", C.c_float)]


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
