"""KITTI trajectory writer (System::SaveTrajectoryKITTI,
src/System.cc:503-560) through the C ABI, on the host (no GPU).

The reference multiplies CV_32F cv::Mat poses; the expected lines here come
from a float32 numpy restatement with the same product order (k summed in
order, each step rounded to float). OpenCV's own gemm accumulation is not
available here: parity unpinned at the last float ulp, pinned by the
semantics checks (bad reference keyframes walk to their parent through Tcp;
the first keyframe is the origin)."""
import numpy as np

from sqrtlm import capture, synth


def _mul(a, b):
    c = np.zeros((4, 4), np.float32)
    for i in range(4):
        for j in range(4):
            s = np.float32(0)
            for k in range(4):
                s = np.float32(s + np.float32(a[i, k] * b[k, j]))
            c[i, j] = s
    return c


def _expected(Tcr, ref, Tcw, Tcp, parent, bad, origin):
    T0 = Tcw[origin]
    Two = np.zeros((4, 4), np.float32)
    for i in range(3):
        o = np.float32(0)
        for k in range(3):
            Two[i, k] = T0[k, i]
            o = np.float32(o + np.float32(-T0[k, i] * T0[k, 3]))
        Two[i, 3] = o
    Two[3, 3] = 1
    lines = []
    for f in range(len(ref)):
        Trw = np.eye(4, dtype=np.float32)
        k = ref[f]
        while bad[k]:
            Trw = _mul(Trw, Tcp[k])
            k = parent[k]
        Trw = _mul(_mul(Trw, Tcw[k]), Two)
        T = _mul(Tcr[f], Trw)
        R = T[:3, :3].T
        t = np.zeros(3, np.float32)
        for i in range(3):
            s = np.float32(0)
            for j in range(3):
                s = np.float32(s + np.float32(-R[i, j] * T[j, 3]))
            t[i] = s
        vals = [R[0, 0], R[0, 1], R[0, 2], t[0], R[1, 0], R[1, 1], R[1, 2], t[1], R[2, 0], R[2, 1], R[2, 2], t[2]]
        lines.append(" ".join("%.9f" % float(v) for v in vals))
    return lines


def _poses(n, seed):
    p = synth.make_problem(n, 50, k_min=2, k_max=4, seed=seed)
    R = synth.quat_to_mat(p.pose_q)
    T = np.zeros((n, 4, 4), np.float32)
    T[:, :3, :3] = R
    T[:, :3, 3] = p.pose_t
    T[:, 3, 3] = 1
    return T


def test_kitti_writer_matches_float_restatement(tmp_path):
    K, F = 12, 40
    Tcw = _poses(K, 3)
    rng = np.random.default_rng(5)
    parent = np.arange(K) - 1
    bad = np.zeros(K, np.uint8)
    bad[[3, 4, 9]] = 1  # 4 -> 3 -> 2: a chain of bad keyframes
    Tcp = np.stack([_mul(Tcw[k], np.linalg.inv(Tcw[max(k - 1, 0)]).astype(np.float32)) for k in range(K)])
    ref = rng.integers(0, K, F).astype(np.int32)
    Tcr = np.stack([_mul(_poses(2, 100 + f)[1], np.linalg.inv(_poses(2, 100 + f)[0]).astype(np.float32))
                    for f in range(F)])
    out = tmp_path / "traj.txt"
    capture.save_trajectory_kitti(out, Tcr, ref, Tcw, Tcp, parent, bad, origin_kf=0)
    got = out.read_text().splitlines()
    assert got == _expected(Tcr, ref, Tcw, Tcp, parent, bad, 0)
    assert all(len(line.split()) == 12 for line in got)


def test_kitti_writer_semantics(tmp_path):
    """Frames sitting on their keyframes (Tcr = I) print Twc of the keyframe in
    the origin keyframe's frame: the first keyframe at the identity."""
    K = 6
    Tcw = _poses(K, 7)
    out = tmp_path / "t.txt"
    I = np.tile(np.eye(4, dtype=np.float32), (K, 1, 1))
    capture.save_trajectory_kitti(out, I, np.arange(K), Tcw, I, np.arange(K) - 1, None, origin_kf=0)
    rows = np.loadtxt(out).reshape(K, 3, 4)
    np.testing.assert_allclose(rows[0], np.eye(4)[:3], atol=1e-6)
    for k in range(K):
        Twc_rel = np.linalg.inv(Tcw[k].astype(np.float64) @ np.linalg.inv(Tcw[0].astype(np.float64)))
        np.testing.assert_allclose(rows[k], Twc_rel[:3], atol=1e-4)
