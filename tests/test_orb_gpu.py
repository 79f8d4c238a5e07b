"""ORB front end on the HIP path vs the CPU restatement
(oracle/orb_ref.c) on identical synthetic images: bit-exact pyramid levels,
keypoints (position, angle, response, octave, size) and descriptors; bit-exact
brute-force Hamming matches and SearchForInitialization match indices."""
import numpy as np
import pytest

from sqrtlm import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def orb_oracle(oracle):
    from oracle import orb as OB
    return OB


@pytest.fixture(scope="module")
def extractor(gpu_ctx):
    from sqrtlm.orb import ORBextractor
    return ORBextractor(2000, 1.2, 8, 20, 7, ctx=gpu_ctx)


def _cmp_kps(kg, kr):
    assert len(kg) == len(kr)
    for f in ("x", "y", "size", "angle", "response", "octave"):
        np.testing.assert_array_equal(kg[f], kr[f], err_msg=f)


@pytest.mark.parametrize("seed,w,h", [(3, 1241, 376), (5, 640, 480), (9, 753, 301), (13, 480, 400)])
def test_extract_bit_exact(extractor, orb_oracle, seed, w, h):
    img, _ = synth.make_image_pair(w, h, seed=seed)
    kg, dg = extractor(img)
    kr, dr, pyr = orb_oracle.extract(orb_oracle.params(), img, with_levels=True)
    for lvl, ref in enumerate(pyr):
        np.testing.assert_array_equal(extractor.image_pyramid()[lvl], ref, err_msg=f"level {lvl}")
    _cmp_kps(kg, kr)
    np.testing.assert_array_equal(dg, dr)
    assert len(kg) > 500


def test_extract_other_params(gpu_ctx, orb_oracle):
    from sqrtlm.orb import ORBextractor
    img, _ = synth.make_image_pair(900, 500, seed=11)
    ex = ORBextractor(1000, 1.3, 5, 30, 10, ctx=gpu_ctx)
    kg, dg = ex(img)
    kr, dr = orb_oracle.extract(orb_oracle.params(1000, 1.3, 5, 30, 10), img)
    _cmp_kps(kg, kr)
    np.testing.assert_array_equal(dg, dr)


def test_extract_flat_and_low_texture(extractor, orb_oracle):
    flat = np.full((376, 1241), 128, np.uint8)
    kg, dg = extractor(flat)
    assert len(kg) == 0 and dg.shape == (0, 32)
    rng = np.random.default_rng(1)  # weak texture: cells fall back to minThFAST
    weak = np.clip(128 + rng.normal(0, 4, (376, 1241)), 0, 255).astype(np.uint8)
    kg, dg = extractor(weak)
    kr, dr = orb_oracle.extract(orb_oracle.params(), weak)
    _cmp_kps(kg, kr)
    np.testing.assert_array_equal(dg, dr)


def test_extract_rejects_too_small(extractor):
    from sqrtlm._lib import SqlmError
    with pytest.raises(SqlmError):
        extractor(np.zeros((120, 160), np.uint8))  # level 7 narrower than one 30-px cell
    with pytest.raises(SqlmError):
        extractor(np.zeros((900, 300), np.uint8))  # portrait: no initial quadtree node


def test_match_bf(gpu_ctx, orb_oracle):
    from sqrtlm.orb import ORBmatcher
    rng = np.random.default_rng(4)
    q = rng.integers(0, 256, (700, 32), dtype=np.uint8)
    t = rng.integers(0, 256, (1500, 32), dtype=np.uint8)
    t[100] = q[5]
    t[900] = q[5]  # tie: the first index wins
    bi, bd, bd2 = ORBmatcher(ctx=gpu_ctx).match_bf(q, t)
    D = np.unpackbits(q[:, None, :] ^ t[None, :, :], axis=2).sum(axis=2)
    np.testing.assert_array_equal(bd, D.min(axis=1))
    np.testing.assert_array_equal(bi, D.argmin(axis=1))
    s = np.sort(D, axis=1)
    np.testing.assert_array_equal(bd2, s[:, 1])
    assert bi[5] == 100 and bd[5] == 0 and bd2[5] == 0
    for i in (0, 7, 42):
        assert bd[i] == orb_oracle.hamming(q[i], t[bi[i]])


def test_match_bf_edge_sizes(gpu_ctx):
    from sqrtlm.orb import ORBmatcher
    m = ORBmatcher(ctx=gpu_ctx)
    q = np.arange(64, dtype=np.uint8).reshape(2, 32)
    bi, bd, bd2 = m.match_bf(q, q[:1])
    assert list(bi) == [0, 0] and bd[0] == 0 and bd2[0] == 2 ** 31 - 1
    bi, bd, bd2 = m.match_bf(q[:0], q)
    assert len(bi) == 0


@pytest.mark.parametrize("seed,shift,check_ori", [(3, (7.0, 3.0), True), (6, (-12.0, 5.0), True),
                                                  (8, (2.0, -1.0), False)])
def test_search_for_initialization(gpu_ctx, extractor, orb_oracle, seed, shift, check_ori):
    from sqrtlm.orb import ORBmatcher
    a, b = synth.make_image_pair(1241, 376, seed=seed, shift=shift)
    k1, d1 = extractor(a)
    k2, d2 = extractor(b)
    bounds = (0.0, 1241.0, 0.0, 376.0)
    prev = np.ascontiguousarray(np.stack([k1["x"], k1["y"]], 1), np.float32)
    nr, mr, pr = orb_oracle.search_for_init(k1, d1, k2, d2, bounds, prev, 100, 0.9, check_ori)
    pg = prev.copy()
    ng, mg = ORBmatcher(0.9, check_ori, ctx=gpu_ctx).SearchForInitialization(k1, d1, k2, d2, bounds, pg, 100)
    assert ng == nr and ng > 50
    np.testing.assert_array_equal(mg, mr)
    np.testing.assert_array_equal(pg, pr)
    ok = mg >= 0
    assert np.median(k2["x"][mg[ok]] - k1["x"][ok]) == shift[0]


# ---- projection searches (ORBmatcher.cc:67, :1717) vs the oracle, bit-exact slots ----
@pytest.fixture(scope="module")
def kitti_pair(extractor):
    a, b = synth.make_image_pair(1241, 376, seed=17, shift=(9.0, 2.0))
    k1, d1 = extractor(a)
    k2, d2 = extractor(b)
    return k1, d1, k2, d2, (0.0, 1241.0, 0.0, 376.0)


def _gpu_frame(k2, d2, bounds, ur, sm, so, Tcw=None, w=1241, h=376):
    from sqrtlm import orb_scene as S
    from sqrtlm.orb import Frame
    fx, fy, cx, cy, bf, mb = S.camera(w, h)
    return Frame(k2, d2, bounds, S.scale_factors(), fx, fy, cx, cy, bf, mb, mvuRight=ur, mTcw=Tcw,
                 mvpMapPoints=sm.copy(), slot_obs=so.copy())


@pytest.mark.parametrize("stereo,th,nnratio", [(False, 1.0, 0.8), (True, 1.0, 0.8), (True, 5.0, 0.9),
                                               (False, 10.0, 0.6)])
def test_search_by_projection_local(gpu_ctx, orb_oracle, kitti_pair, stereo, th, nnratio):
    from sqrtlm import orb_scene as S
    from sqrtlm.orb import ORBmatcher
    k1, d1, k2, d2, bounds = kitti_pair
    mps, md = S.local_points(k1, d1, (9.0, 2.0), seed=3, stereo=stereo)
    ur, sm, so = S.current_slots(k2, 3, stereo)
    n_r, m_r, o_r = orb_oracle.search_by_projection_local(k2, d2, bounds, S.scale_factors(), ur, sm, so, mps, md, th,
                                                          nnratio)
    F = _gpu_frame(k2, d2, bounds, ur, sm, so)
    n_g = ORBmatcher(nnratio, ctx=gpu_ctx).SearchByProjection(F, mps, md, th)
    assert n_g == n_r and n_r > 100
    np.testing.assert_array_equal(F.mvpMapPoints, m_r)
    np.testing.assert_array_equal(F.slot_obs, o_r)


@pytest.mark.parametrize("stereo,mono,tz,th,check_ori", [(False, True, 0.0, 7.0, True), (True, False, 1.0, 7.0, True),
                                                         (True, False, -1.0, 15.0, True),
                                                         (True, False, 0.0, 15.0, False)])
def test_search_by_projection_last(gpu_ctx, orb_oracle, kitti_pair, stereo, mono, tz, th, check_ori):
    from sqrtlm import orb_scene as S
    from sqrtlm.orb import LastFrameSlots, ORBmatcher
    k1, d1, k2, d2, bounds = kitti_pair
    Tcw, Tlw, lp, ld = S.last_frame(k1, d1, (9.0, 2.0), 1241, 376, seed=4, tz=tz)
    ur, sm, so = S.current_slots(k2, 4, stereo)
    n_r, m_r, o_r = orb_oracle.search_by_projection_last(k2, d2, bounds, S.scale_factors(), S.camera(1241, 376), ur,
                                                         sm, so, Tcw, Tlw, lp, ld, th, mono, check_ori)
    F = _gpu_frame(k2, d2, bounds, ur, sm, so, Tcw=Tcw)
    n_g = ORBmatcher(0.9, check_ori, ctx=gpu_ctx).SearchByProjection(F, LastFrameSlots(Tlw, lp, ld), th, mono)
    assert n_g == n_r and n_r > 100
    np.testing.assert_array_equal(F.mvpMapPoints, m_r)
    np.testing.assert_array_equal(F.slot_obs, o_r)


def test_search_by_projection_edge_cases(gpu_ctx, orb_oracle, kitti_pair):
    from sqrtlm import orb_scene as S
    from sqrtlm._lib import SqlmError
    from sqrtlm.orb import LastFrameSlots, ORBmatcher
    k1, d1, k2, d2, bounds = kitti_pair
    m = ORBmatcher(0.8, ctx=gpu_ctx)
    ur, sm, so = S.current_slots(k2, 1, False)
    F = _gpu_frame(k2, d2, bounds, ur, sm, so, Tcw=np.eye(4)[:3])
    mps, md = S.local_points(k1, d1, (9.0, 2.0), seed=1, stereo=False)
    assert m.SearchByProjection(F, mps[:0], md[:0]) == 0  # no map points
    off = mps.copy()
    off["in_view"] = 0
    assert m.SearchByProjection(F, off, md) == 0  # nothing to project
    np.testing.assert_array_equal(F.mvpMapPoints, sm)
    far = mps.copy()
    far["proj_x"] += 5000.0  # every window outside the grid
    assert m.SearchByProjection(F, far, md) == 0
    bad = mps[:4].copy()
    bad["level"] = 8  # mnTrackScaleLevel beyond mvScaleFactors
    with pytest.raises(SqlmError):
        m.SearchByProjection(F, bad, md[:4])
    E = _gpu_frame(k2[:0], d2[:0], bounds, None, sm[:0], so[:0], Tcw=np.eye(4)[:3])  # frame without keypoints
    assert m.SearchByProjection(E, mps, md) == 0
    Tcw, Tlw, lp, ld = S.last_frame(k1, d1, (9.0, 2.0), 1241, 376, seed=2)
    assert m.SearchByProjection(E, LastFrameSlots(Tlw, lp, ld), 7.0, True) == 0
    n_r, m_r, _ = orb_oracle.search_by_projection_last(k2, d2, bounds, S.scale_factors(), S.camera(1241, 376), None,
                                                       sm, so, np.eye(4)[:3], Tlw, lp, ld, 7.0, True)
    F2 = _gpu_frame(k2, d2, bounds, None, sm, so, Tcw=np.eye(4)[:3])  # identity motion: the old positions
    assert m.SearchByProjection(F2, LastFrameSlots(Tlw, lp, ld), 7.0, True) == n_r
    np.testing.assert_array_equal(F2.mvpMapPoints, m_r)


# ---- keyframe projection searches (ORBmatcher.cc:423, :1109, :1296, :1902) ----
@pytest.mark.parametrize("s,th", [(1.0, 10), (1.3, 10), (0.8, 4)])
def test_search_by_projection_sim3(gpu_ctx, orb_oracle, kitti_pair, s, th):
    from sqrtlm import orb_scene as S
    from sqrtlm.orb import ORBmatcher
    k1, d1, k2, d2, bounds = kitti_pair
    cam = S.camera(1241, 376)
    mps, md = S.map_points(k1, d1, 1241, 376, seed=3)
    Scw = S.sim3_of(S.keyframe_pose((9.0, 2.0), 1241, 376, (0.02, 0.0, 0.1)), s)
    _, sm, so = S.current_slots(k2, 3, False)
    n_r, m_r = orb_oracle.search_by_projection_sim3(k2, d2, bounds, S.scale_factors(), cam, sm, Scw, mps, md, th)
    F = _gpu_frame(k2, d2, bounds, None, sm, so)
    n_g = ORBmatcher(0.75, ctx=gpu_ctx).SearchByProjection(F, Scw, mps, md, th)
    assert n_g == n_r and n_r > 100
    np.testing.assert_array_equal(F.mvpMapPoints, m_r)


@pytest.mark.parametrize("sim3,stereo,th", [(False, False, 3.0), (False, True, 5.0), (True, False, 4.0)])
def test_fuse(gpu_ctx, orb_oracle, kitti_pair, sim3, stereo, th):
    from sqrtlm import orb_scene as S
    from sqrtlm.orb import ORBmatcher
    k1, d1, k2, d2, bounds = kitti_pair
    cam = S.camera(1241, 376)
    mps, md = S.map_points(k1, d1, 1241, 376, seed=4)
    T = S.keyframe_pose((9.0, 2.0), 1241, 376, (0.0, 0.01, 0.05))
    ur, sm, so = S.current_slots(k2, 4, stereo)
    Tq = S.sim3_of(T, 1.2) if sim3 else T
    n_r, idx_r = orb_oracle.fuse(k2, d2, bounds, S.scale_factors(), cam, ur, Tq, sim3, mps, md, th)
    F = _gpu_frame(k2, d2, bounds, ur, sm, so, Tcw=T)
    m = ORBmatcher(0.6, ctx=gpu_ctx)
    n_g, idx_g = m.Fuse(F, Tq, mps, md, th) if sim3 else m.Fuse(F, mps, md, th)
    assert n_g == n_r and n_r > 50
    np.testing.assert_array_equal(idx_g, idx_r)


@pytest.mark.parametrize("th,orb_dist,check_ori", [(10.0, 100, True), (3.0, 64, False)])
def test_search_by_projection_kf(gpu_ctx, orb_oracle, kitti_pair, th, orb_dist, check_ori):
    from sqrtlm import orb_scene as S
    from sqrtlm.orb import KeyFrameSlots, ORBmatcher
    k1, d1, k2, d2, bounds = kitti_pair
    cam = S.camera(1241, 376)
    mps, md = S.map_points(k1, d1, 1241, 376, seed=5)
    Tcw = S.keyframe_pose((9.0, 2.0), 1241, 376, (0.01, 0.0, -0.1))
    _, sm, so = S.current_slots(k2, 5, False)
    n_r, m_r = orb_oracle.search_by_projection_kf(k2, d2, bounds, S.scale_factors(), cam, sm, Tcw, mps, md,
                                                  k1["angle"], th, orb_dist, check_ori)
    F = _gpu_frame(k2, d2, bounds, None, sm, so, Tcw=Tcw)
    n_g = ORBmatcher(0.75, check_ori, ctx=gpu_ctx).SearchByProjection(F, KeyFrameSlots(mps, md, k1["angle"]), th,
                                                                      orb_dist)
    assert n_g == n_r and n_r > 100
    np.testing.assert_array_equal(F.mvpMapPoints, m_r)


# ---- BoW searches (ORBmatcher.cc:246, :731, :887) ----
@pytest.mark.parametrize("check_ori", [True, False])
def test_search_by_bow(gpu_ctx, orb_oracle, kitti_pair, check_ori):
    from sqrtlm import orb_scene as S
    from sqrtlm.orb import BowFrame, ORBmatcher
    k1, d1, k2, d2, bounds = kitti_pair
    n1, n2 = S.bow_nodes(d1, 1), S.bow_nodes(d2, 2)
    mp1, bad1 = S.bow_points(len(k1), 1)
    mp2, bad2 = S.bow_points(len(k2), 2, base=10000)
    a = (k1, d1, n1, mp1, bad1)
    n_r, out_r = orb_oracle.search_by_bow_kf_frame(a, (k2, d2, n2, mp2), 0.7, check_ori)
    KF = BowFrame(k1, d1, n1, mp1, bad1)
    n_g, out_g = ORBmatcher(0.7, check_ori, ctx=gpu_ctx).SearchByBoW(KF, BowFrame(k2, d2, n2, keyframe=False))
    assert n_g == n_r and n_r > 100
    np.testing.assert_array_equal(out_g, out_r)
    n_r, out_r = orb_oracle.search_by_bow_kf_kf(a, (k2, d2, n2, mp2, bad2), 0.75, check_ori)
    n_g, out_g = ORBmatcher(0.75, check_ori, ctx=gpu_ctx).SearchByBoW(KF, BowFrame(k2, d2, n2, mp2, bad2))
    assert n_g == n_r and n_r > 100
    np.testing.assert_array_equal(out_g, out_r)


@pytest.mark.parametrize("stereo,only_stereo,check_ori", [(False, False, False), (True, False, True),
                                                          (True, True, False)])
def test_search_for_triangulation(gpu_ctx, orb_oracle, kitti_pair, stereo, only_stereo, check_ori):
    from sqrtlm import orb_scene as S
    from sqrtlm.orb import BowFrame, ORBmatcher
    k1, d1, k2, d2, bounds = kitti_pair
    cam = S.camera(1241, 376)
    T1 = S.keyframe_pose((0.0, 0.0), 1241, 376)
    T2 = S.keyframe_pose((9.0, 2.0), 1241, 376, (0.3, 0.0, 0.05))
    F12 = S.fundamental_12(T1, T2, cam, cam)
    n1, n2 = S.bow_nodes(d1, 5), S.bow_nodes(d2, 6)
    mp1, _ = S.bow_points(len(k1), 5, frac=0.3)
    mp2, _ = S.bow_points(len(k2), 6, frac=0.3)
    ur1, _, _ = S.current_slots(k1, 5, stereo)
    ur2, _, _ = S.current_slots(k2, 6, stereo)
    sf = S.scale_factors()
    K1 = BowFrame(k1, d1, n1, mp1, None, ur1, Tcw=T1, cam=cam[:4], mvScaleFactors=sf)
    K2 = BowFrame(k2, d2, n2, mp2, None, ur2, Tcw=T2, cam=cam[:4], mvScaleFactors=sf)
    n_r, m_r = orb_oracle.search_for_triangulation((k1, d1, n1, mp1, None, ur1), (k2, d2, n2, mp2, None, ur2),
                                                   K1.GetCameraCenter(), T2, cam[:4], sf, F12, only_stereo, check_ori)
    n_g, pairs = ORBmatcher(0.6, check_ori, ctx=gpu_ctx).SearchForTriangulation(K1, K2, F12, only_stereo)
    assert n_g == n_r and n_r > 10
    assert pairs == [(int(i), int(m_r[i])) for i in np.nonzero(m_r >= 0)[0]]


def test_bow_edge_cases(gpu_ctx, kitti_pair):
    from sqrtlm.orb import BowFrame, ORBmatcher
    k1, d1, k2, d2, bounds = kitti_pair
    m = ORBmatcher(0.7, True, ctx=gpu_ctx)
    none = np.full(len(k1), -1, np.int32)
    n, out = m.SearchByBoW(BowFrame(k1, d1, none, np.arange(len(k1))), BowFrame(k2, d2, np.zeros(len(k2)),
                                                                                keyframe=False))
    assert n == 0 and (out == -1).all()  # no feature in the vocabulary: no common node
    n, out = m.SearchByBoW(BowFrame(k1[:0], d1[:0], none[:0]), BowFrame(k2, d2, np.zeros(len(k2))))
    assert n == 0 and len(out) == 0


@pytest.mark.parametrize("s12,th", [(1.0, 7.5), (1.03, 10.0)])
def test_search_by_sim3(gpu_ctx, orb_oracle, kitti_pair, s12, th):
    from sqrtlm import orb_scene as S
    from sqrtlm.orb import Frame, ORBmatcher
    k1, d1, k2, d2, bounds = kitti_pair
    cam = S.camera(1241, 376)
    T1, T2, mp1, md1, mp2, md2, R12, t12, m12 = S.sim3_scene(k1, d1, k2, d2, (9.0, 2.0), 1241, 376, 7)
    sf = S.scale_factors()
    n_r, m_r = orb_oracle.search_by_sim3(k1, d1, k2, d2, bounds, sf, cam, T1, T2, mp1, md1, mp2, md2, s12, R12, t12,
                                         th, m12)
    K1 = Frame(k1, d1, bounds, sf, *cam[:4], mTcw=T1)
    K2 = Frame(k2, d2, bounds, sf, *cam[:4], mTcw=T2)
    m = m12.copy()
    n_g = ORBmatcher(0.75, ctx=gpu_ctx).SearchBySim3(K1, K2, mp1, md1, mp2, md2, m, s12, R12, t12, th)
    assert n_g == n_r and n_r > 100
    np.testing.assert_array_equal(m, m_r)
