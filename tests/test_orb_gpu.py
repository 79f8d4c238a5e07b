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
