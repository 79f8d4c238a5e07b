"""Capture / replay at the Optimizer seam and the stereo
edge on the HIP path (row f4).

CPU: the native writer/reader round-trips every section, rejects corrupt
files, skips unknown sections; the committed fixtures reproduce from the
oracle bit for bit. GPU: sqlm_capture_replay of each fixture matches the
oracle's recorded write-back (poses / points within 1e-6 relative as float
write-back, identical LBA outlier tags, chi2 within 1e-6 relative), and the
stereo GBA matches the oracle directly.
"""
import os
import struct

import numpy as np
import pytest

from sqrtlm import capture, synth
from sqrtlm.problem import HUBER_MONO_GBA, HUBER_STEREO

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURES = ["lba_capture.sqcap", "gba_stereo_capture.sqcap"]
TOL = 1e-6


def _fixture(name):
    return capture.read(os.path.join(HERE, "golden", name))


def _eq(a, b):
    if a is None or b is None:
        return a is None and b is None
    return a.dtype == b.dtype and a.shape == b.shape and np.array_equal(a, b)


def test_roundtrip_every_section(tmp_path, oracle):
    from capture_util import problem_to_capture
    prob = synth.add_stereo(synth.add_lidar_flat(synth.make_problem(6, 50, pair_window=3, seed=1), 5, 10), 0.5)
    c = problem_to_capture(prob, capture.LBA, oracle)
    c.res_Tcw = c.Tcw + 1
    c.res_pt = c.pt * 2
    c.res_outlier = (np.arange(c.n_obs) % 3 == 0).astype(np.uint8)
    c.res_chi2 = np.linspace(0, 1, c.n_obs)
    p = tmp_path / "a.sqcap"
    capture.write(p, c)
    b = capture.read(p)
    assert (b.kind, b.gba_iterations, b.gba_robust) == (c.kind, c.gba_iterations, c.gba_robust)
    for name, dt, _, _ in capture._ARRAYS:
        x, y = getattr(c, name), getattr(b, name)
        assert _eq(None if x is None else np.asarray(x, dt), y), name


def test_optional_sections_absent(tmp_path):
    c = capture.Capture(kind=capture.GBA, Tcw=np.tile(np.eye(4, dtype=np.float32), (2, 1, 1)),
                        pose_fixed=np.array([1, 0], np.uint8), intr=np.ones((2, 4), np.float32),
                        pt=np.ones((1, 3), np.float32), obs_pose=np.array([0, 1], np.int32),
                        obs_pt=np.zeros(2, np.int32), obs_uv=np.zeros((2, 2), np.float32),
                        obs_inv_sigma2=np.ones(2, np.float32), gba_iterations=7)
    p = tmp_path / "b.sqcap"
    capture.write(p, c)
    b = capture.read(p)
    assert b.gba_iterations == 7 and not b.has_result
    assert b.obs_ur is None and b.bf is None and b.lid_pose is None and b.obs_delta is None


def test_reader_rejects_corrupt_and_skips_unknown(tmp_path):
    from sqrtlm._lib import SqlmError
    src = open(os.path.join(HERE, "golden", FIXTURES[0]), "rb").read()
    bad = tmp_path / "bad.sqcap"
    for blob in (b"NOTACAPT" + src[8:], src[: len(src) // 2], src[:20]):
        bad.write_bytes(blob)
        with pytest.raises(SqlmError):
            capture.read(bad)
    # an out-of-range observation index
    c = _fixture(FIXTURES[0])
    c.obs_pt = c.obs_pt.copy()
    c.obs_pt[3] = c.n_pt + 5
    capture.write(bad, c)
    with pytest.raises(SqlmError):
        capture.read(bad)
    # a section header claiming far more payload than the file holds (up to
    # 64 TiB by its own limits): rejected before anything is allocated
    huge = tmp_path / "huge.sqcap"
    huge.write_bytes(src[:16] + struct.pack("<IIQ", 0x4B4E5558, 64, (1 << 40) - 1) + b"\x00" * 64)
    with pytest.raises(SqlmError):
        capture.read(huge)
    # unknown trailing section: ignored
    ext = tmp_path / "ext.sqcap"
    ext.write_bytes(src + struct.pack("<IIQ", 0x4B4E5558, 4, 2) + b"\x00" * 8)
    b = capture.read(ext)
    assert np.array_equal(b.res_Tcw, _fixture(FIXTURES[0]).res_Tcw)


@pytest.mark.parametrize("name", FIXTURES)
def test_fixture_reproduces_from_oracle(name, oracle):
    from capture_util import oracle_results
    c = _fixture(name)
    ref = (c.res_Tcw.copy(), c.res_pt.copy(), c.res_outlier.copy(), c.res_chi2.copy())
    oracle_results(c, oracle)
    assert np.array_equal(c.res_Tcw, ref[0]) and np.array_equal(c.res_pt, ref[1])
    assert np.array_equal(c.res_outlier, ref[2]) and np.array_equal(c.res_chi2, ref[3])


def _rel(a, b):
    return np.abs(a.astype(np.float64) - b.astype(np.float64)).max() / max(1.0, np.abs(b).max())


@pytest.mark.gpu
@pytest.mark.parametrize("name", FIXTURES)
def test_replay_matches_recorded_writeback(gpu_ctx, name):
    c = _fixture(name)
    out = capture.replay(gpu_ctx, c)
    assert out["ran"] == 1
    assert _rel(out["Tcw"], c.res_Tcw) < TOL
    assert _rel(out["pt"], c.res_pt) < TOL
    assert np.array_equal(out["outlier"], c.res_outlier)
    np.testing.assert_allclose(out["chi2"], c.res_chi2, rtol=TOL, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("robust", [False, True])
def test_stereo_gba_matches_oracle(gpu_ctx, oracle, robust):
    prob = synth.make_problem(20, 700, k_min=2, k_max=10, n_fixed=1, seed=41, robust=robust,
                              huber_delta=HUBER_MONO_GBA)
    synth.add_stereo(prob, 0.5, seed=41, robust_delta=HUBER_STEREO if robust else None)
    ref = oracle.OracleGraph(prob)
    nr, sr = ref.global_ba(10)
    gpu_ctx.set_problem(prob)
    ng, sg = gpu_ctx.global_ba(10)
    assert ng == nr
    assert sg["iterations"] == sr["iterations"] and sg["trace_trials"] == sr["trace_trials"]
    np.testing.assert_allclose(sg["trace_chi2"], sr["trace_chi2"], rtol=TOL)
    q, t = gpu_ctx.poses()
    assert np.abs(q - ref.pose_q).max() < TOL
    assert _rel(t, ref.pose_t) < TOL and _rel(gpu_ctx.points(), ref.pt) < TOL
    np.testing.assert_allclose(gpu_ctx.edge_chi2(), ref.edge_chi2(), rtol=TOL, atol=1e-9)


@pytest.mark.gpu
def test_stereo_local_ba_tags(gpu_ctx, oracle):
    """Library LBA with stereo edges set (3-DoF tag threshold 7.815)."""
    prob = synth.make_problem(14, 400, pair_window=4, n_fixed=3, seed=42, robust=True)
    synth.add_stereo(prob, 0.4, seed=42, robust_delta=HUBER_STEREO)
    ref = oracle.OracleGraph(prob)
    _, outl_r, sr = ref.local_ba()
    gpu_ctx.set_problem(prob)
    _, outl_g, sg = gpu_ctx.local_ba()
    assert np.array_equal(outl_g, outl_r)
    for a, b in zip(sg, sr):
        assert a["iterations"] == b["iterations"] and a["trace_trials"] == b["trace_trials"]
    q, t = gpu_ctx.poses()
    assert np.abs(q - ref.pose_q).max() < TOL and _rel(gpu_ctx.points(), ref.pt) < TOL


@pytest.mark.gpu
def test_replay_cli_reports_parity():
    import json
    import subprocess
    root = os.path.dirname(HERE)
    exe = os.path.join(root, "tools", "sqlm_replay")
    assert os.path.exists(exe), "build tools/ first (__graft_entry__.build())"
    files = [os.path.join(HERE, "golden", f) for f in FIXTURES]
    r = subprocess.run([exe] + files, capture_output=True, text=True, timeout=300)
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert r.returncode == 0, r.stdout + r.stderr
    assert len(lines) == 2 and all(x["parity"] for x in lines)
    assert lines[0]["kind"] == "lba" and lines[0]["n_lid"] > 0 and len(lines[0]["passes"]) == 3
    assert lines[1]["kind"] == "gba" and lines[1]["passes"][0]["iterations"] == 10
