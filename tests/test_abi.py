"""C-ABI library: loads, exports every symbol include/sqrtlm.h declares, and its
host-only entry points behave (no GPU needed)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from sqrtlm import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_header_and_binding_agree():
    hdr = open(os.path.join(ROOT, "include", "sqrtlm.h")).read()
    declared = set(re.findall(r"\b(sqlm_[A-Za-z0-9_]+)\s*\(", hdr))
    assert declared == set(_lib.EXPORTS), declared ^ set(_lib.EXPORTS)


def test_capture_header_and_binding_agree():
    hdr = open(os.path.join(ROOT, "include", "sqrtlm_capture.h")).read()
    declared = set(re.findall(r"\b(sqlm_[A-Za-z0-9_]+)\s*\(", hdr))
    assert declared == set(_lib.CAPTURE_EXPORTS), declared ^ set(_lib.CAPTURE_EXPORTS)


def test_orb_header_and_binding_agree():
    hdr = open(os.path.join(ROOT, "include", "sqrtlm_orb.h")).read()
    declared = set(re.findall(r"\b(sqlm_[A-Za-z0-9_]+)\s*\(", hdr))
    assert declared == set(_lib.ORB_EXPORTS), declared ^ set(_lib.ORB_EXPORTS)


def test_library_exports_every_symbol():
    L = _lib.lib()
    for s in _lib.EXPORTS + _lib.CAPTURE_EXPORTS + _lib.ORB_EXPORTS:
        assert hasattr(L, s), s
    assert b"gfx950" in L.sqlm_version()
    assert L.sqlm_status_string(-8) == b"problem shape not supported by this build"


def test_ctx_create_without_device_fails_loudly():
    import subprocess, sys
    code = ("import sys; sys.path[:0]=[%r]; from sqrtlm import _lib; import ctypes as C; "
            "h=C.c_void_p(); print(_lib.lib().sqlm_ctx_create(0, C.byref(h)))") % os.path.join(ROOT, "sqrtlm-slam_amd")
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    if out.returncode == 0 and out.stdout.strip():
        assert int(out.stdout.strip().splitlines()[-1]) in (-6, -2)  # NO_DEVICE (or HIP init error)


def test_null_and_invalid_arguments():
    L = _lib.lib()
    assert L.sqlm_ctx_create(0, None) == -1
    assert L.sqlm_ctx_destroy(None) == -1
    assert L.sqlm_set_problem(None, 0, None, None, None, None, 0, None, C.c_int64(0), None, None, None, None, None,
                              None) == -1
    assert L.sqlm_optimize(None, 0, 1, C.c_double(0), None, None, None) == -1


def test_converter_matches_oracle(oracle):
    from sqrtlm.optimizer import pose_from_Tcw_f32, pose_to_Tcw_f32
    from sqrtlm import synth
    rng = np.random.default_rng(3)
    for _ in range(20):
        w = rng.normal(size=3)
        R = synth._so3_exp(w[None])[0]
        T = np.eye(4, dtype=np.float32)
        T[:3, :3] = R
        T[:3, 3] = rng.normal(size=3) * 10
        q1, t1 = pose_from_Tcw_f32(T)
        q2, t2 = oracle.se3_from_Tcw_f32(T)
        np.testing.assert_allclose(q1, q2, atol=1e-15)
        np.testing.assert_array_equal(t1, t2)
        np.testing.assert_array_equal(pose_to_Tcw_f32(q1, t1), oracle.se3_to_Tcw_f32(q2, t2))
