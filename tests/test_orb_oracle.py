"""Pins of the ORB oracle (oracle/orb_ref.c) by independent restatements.

OpenCV is absent here and the reference ships no ORB fixtures, so the
OpenCV-implemented stages (resize, GaussianBlur, FAST) are parity UNPINNED
against the reference binary (oracle/orb_ref.h); they are pinned below by
their defining properties (FAST: the 9-of-16 arc definition and the score as
the largest threshold that keeps the corner; resize / blur: within one grey
level of the exact bilinear / Gaussian filter). The stages the reference
implements itself (IC_Angle, steered BRIEF, Hamming distance, quadtree,
SearchForInitialization) are checked against direct numpy / Python
transliterations of the reference source, and the whole extractor output is
frozen in tests/golden/orb/orb_golden.npz."""
import math
import os

import numpy as np
import pytest

from sqrtlm import synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "orb", "orb_golden.npz")
CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3), (-2, -2),
          (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


@pytest.fixture(scope="module")
def OB(oracle):
    from oracle import orb
    return orb


def test_level_geometry(OB):
    lw, lh, nf, sc = OB.levels(OB.params(), 1241, 376)
    assert list(lw) == [1241, 1034, 862, 718, 598, 499, 416, 346]
    assert list(lh) == [376, 313, 261, 218, 181, 151, 126, 105]
    assert nf.sum() == 2000 and list(nf[:3]) == [434, 362, 302]
    np.testing.assert_allclose(sc, 1.2 ** np.arange(8), rtol=1e-6)


def test_gauss_kernel(OB):
    k = OB.gauss_kernel()  # getGaussianKernel(7, 2) x 256: 18 34 49 55 49 34 18
    assert list(k) == [18, 34, 49, 55, 49, 34, 18]


def test_hamming_matches_popcount(OB):
    rng = np.random.default_rng(0)
    for _ in range(50):
        a, b = rng.integers(0, 256, (2, 32), dtype=np.uint8)
        assert OB.hamming(a, b) == int(np.unpackbits(a ^ b).sum())


def _brute_fast(img, th):
    """9-contiguous-of-16 definition; score = max over arcs of min |d| - 1."""
    h, w = img.shape
    I = img.astype(int)
    score = np.zeros((h, w), int)
    for y in range(3, h - 3):
        for x in range(3, w - 3):
            v = I[y, x]
            d = np.array([v - I[y + dy, x + dx] for dx, dy in CIRCLE])
            best = -1
            for s in range(16):
                arc = d[[(s + k) % 16 for k in range(9)]]
                best = max(best, arc.min() - 1, (-arc).min() - 1)
            if best >= th:
                score[y, x] = best
    return score


def test_fast_against_definition(OB):
    img, _ = synth.make_image_pair(90, 70, seed=2)
    for th in (7, 20):
        kps = OB.fast(img, th)
        score = _brute_fast(img, th)
        exp = []
        h, w = img.shape
        for y in range(3, h - 3):
            for x in range(3, w - 3):
                s = score[y, x]
                if s and all(s > score[y + dy, x + dx] for dy in (-1, 0, 1) for dx in (-1, 0, 1) if dy or dx):
                    exp.append((x, y, s))
        got = [(int(k["x"]), int(k["y"]), int(k["response"])) for k in kps]
        assert got == exp and len(got) > 5


def test_resize_close_to_bilinear(OB):
    img, _ = synth.make_image_pair(300, 200, seed=3)
    out = OB.resize(img, 250, 167)
    sx, sy = 300 / 250, 200 / 167
    fx = (np.arange(250) + 0.5) * sx - 0.5
    fy = (np.arange(167) + 0.5) * sy - 0.5
    x0 = np.clip(np.floor(fx).astype(int), 0, 298)
    y0 = np.clip(np.floor(fy).astype(int), 0, 198)
    ax = np.clip(fx - x0, 0, 1)[None, :]
    ay = np.clip(fy - y0, 0, 1)[:, None]
    I = img.astype(float)
    ref = ((1 - ay) * ((1 - ax) * I[y0][:, x0] + ax * I[y0][:, x0 + 1]) +
           ay * ((1 - ax) * I[y0 + 1][:, x0] + ax * I[y0 + 1][:, x0 + 1]))
    assert np.abs(out.astype(float) - ref).max() <= 1.0


def test_blur_close_to_gaussian(OB):
    img, _ = synth.make_image_pair(120, 90, seed=4)
    out = OB.blur(img)
    x = np.arange(7) - 3.0
    g = np.exp(-x * x / 8.0)
    g /= g.sum()
    P = np.pad(img.astype(float), 3, mode="reflect")  # numpy "reflect" = BORDER_REFLECT_101
    R = sum(g[i] * P[:, i:i + 120] for i in range(7))
    ref = sum(g[i] * R[i:i + 90, :] for i in range(7))
    assert np.abs(out.astype(float) - ref).max() <= 2.5  # the x256 integer taps sum to 257
    # exactly the integer-tap filter, rounded to nearest (ties either way)
    ik = OB.gauss_kernel().astype(np.int64)
    Pi = np.pad(img.astype(np.int64), 3, mode="reflect")
    Ri = sum(ik[i] * Pi[:, i:i + 120] for i in range(7))
    N = sum(ik[i] * Ri[i:i + 90, :] for i in range(7))
    assert np.abs(out.astype(float) - np.minimum(N / 65536.0, 255.0)).max() <= 0.5


def _umax():
    import math
    umax = [0] * 16
    vmax = math.floor(15 * math.sqrt(2) / 2 + 1)
    vmin = math.ceil(15 * math.sqrt(2) / 2)
    for v in range(vmax + 1):
        umax[v] = int(np.rint(math.sqrt(225 - v * v)))
    v0 = 0
    for v in range(15, vmin - 1, -1):
        while umax[v0] == umax[v0 + 1]:
            v0 += 1
        umax[v] = v0
        v0 += 1
    return umax


def test_ic_angle_is_intensity_centroid(OB):
    img, _ = synth.make_image_pair(200, 120, seed=5)
    umax = _umax()
    I = img.astype(np.int64)
    for (x, y) in [(40, 40), (100, 60), (150, 80), (77, 33)]:
        m10 = m01 = 0
        for v in range(-15, 16):
            d = umax[abs(v)]
            for u in range(-d, d + 1):
                m10 += u * I[y + v, x + u]
                m01 += v * I[y + v, x + u]
        ang = OB.ic_angle(img, x, y)
        exact = np.degrees(np.arctan2(m01, m10)) % 360.0
        diff = abs((ang - exact + 180.0) % 360.0 - 180.0)
        assert diff < 0.02  # fastAtan2 polynomial accuracy


def test_fast_atan2_quadrants(OB):
    for y, x in [(1, 1), (1, -1), (-1, -1), (-1, 1), (0, 1), (1, 0), (3, 7), (-7, 3)]:
        ref = np.degrees(np.arctan2(y, x)) % 360.0
        assert abs((OB.fast_atan2(y, x) - ref + 180) % 360 - 180) < 0.02


def _pattern():
    import re
    txt = open(os.path.join(os.path.dirname(GOLDEN), "..", "..", "..", "oracle", "orb_pattern.h")).read()
    body = txt[txt.index("{") + 1:txt.index("};")]
    vals = [int(v) for v in re.findall(r"-?\d+", body)]
    assert len(vals) == 1024
    return vals


def test_descriptor_matches_steered_brief(OB):
    pattern = _pattern()
    img, _ = synth.make_image_pair(160, 120, seed=6)
    I = img.astype(int)
    for (x, y, ang) in [(50, 50, 0.0), (80, 60, 37.5), (100, 70, 211.25), (60, 40, 359.0)]:
        kp = np.zeros(1, OB.KP_DTYPE)
        kp["x"], kp["y"], kp["angle"] = x, y, ang
        d = OB.describe(img, kp)
        angle = np.float32(np.float32(ang) * np.float32(np.pi / 180.0))
        a, b = np.float32(np.cos(np.float64(angle))), np.float32(np.sin(np.float64(angle)))
        bits = []
        for i in range(256):
            x0, y0, x1, y1 = (np.float32(v) for v in pattern[4 * i:4 * i + 4])
            t0 = I[y + int(np.rint(x0 * b + y0 * a)), x + int(np.rint(x0 * a - y0 * b))]
            t1 = I[y + int(np.rint(x1 * b + y1 * a)), x + int(np.rint(x1 * a - y1 * b))]
            bits.append(int(t0 < t1))
        exp = np.packbits(np.array(bits, np.uint8).reshape(32, 8), axis=1, bitorder="little").ravel()
        np.testing.assert_array_equal(d, exp)


def test_distribute_invariants(OB):
    rng = np.random.default_rng(7)
    n = 3000
    keys = np.zeros(n, OB.KP_DTYPE)
    keys["x"] = rng.integers(0, 1209, n)
    keys["y"] = rng.integers(0, 344, n)
    keys["response"] = rng.integers(7, 120, n)
    for N in (50, 434, 2000):
        out = OB.distribute(keys, 16, 1225, 16, 360, N)
        assert N <= len(out) <= N + 3 * 64 or len(out) == n
        src = set(zip(keys["x"].tolist(), keys["y"].tolist(), keys["response"].tolist()))
        assert all((k["x"], k["y"], k["response"]) in src for k in out)
    out = OB.distribute(keys[:1], 16, 1225, 16, 360, 10)
    assert len(out) == 1
    assert len(OB.distribute(keys[:0], 16, 1225, 16, 360, 10)) == 0


def _py_search_for_init(k1, d1, k2, d2, grid, prev, window, nnratio, check_ori):
    """Direct transliteration of ORBmatcher::SearchForInitialization
    (ORBmatcher.cc:573-718) with Frame::GetFeaturesInArea / PosInGrid."""
    import math
    f32 = np.float32
    minx, maxx, miny, maxy = (f32(v) for v in grid)
    wi, hi = f32(64) / (maxx - minx), f32(48) / (maxy - miny)
    cells = [[[] for _ in range(48)] for _ in range(64)]
    for i in range(len(k2)):
        px = math.floor(float((f32(k2["x"][i]) - minx) * wi) + 0.5)
        py = math.floor(float((f32(k2["y"][i]) - miny) * hi) + 0.5)
        if 0 <= px < 64 and 0 <= py < 48:
            cells[px][py].append(i)
    D = np.unpackbits(d1[:, None, :] ^ d2[None, :, :], axis=2).sum(axis=2)
    m12 = [-1] * len(k1)
    vmd = [2 ** 31 - 1] * len(k2)
    m21 = [-1] * len(k2)
    hist = [[] for _ in range(30)]
    n = 0
    r = f32(window)
    for i1 in range(len(k1)):
        if k1["octave"][i1] > 0:
            continue
        x, y = f32(prev[i1, 0]), f32(prev[i1, 1])
        x0 = max(0, math.floor((x - minx - r) * wi))
        x1 = min(63, math.ceil((x - minx + r) * wi))
        y0 = max(0, math.floor((y - miny - r) * hi))
        y1 = min(47, math.ceil((y - miny + r) * hi))
        if x0 >= 64 or x1 < 0 or y0 >= 48 or y1 < 0:
            continue
        cand = [j for ix in range(x0, x1 + 1) for iy in range(y0, y1 + 1) for j in cells[ix][iy]
                if k2["octave"][j] == 0 and abs(f32(k2["x"][j]) - x) < r and abs(f32(k2["y"][j]) - y) < r]
        if not cand:
            continue
        b1 = b2 = 2 ** 31 - 1
        bi = -1
        for j in cand:
            dist = int(D[i1, j])
            if vmd[j] <= dist:
                continue
            if dist < b1:
                b2, b1, bi = b1, dist, j
            elif dist < b2:
                b2 = dist
        if b1 <= 50 and b1 < f32(b2) * f32(nnratio):
            if m21[bi] >= 0:
                m12[m21[bi]] = -1
                n -= 1
            m12[i1], m21[bi], vmd[bi] = bi, i1, b1
            n += 1
            if check_ori:
                rot = f32(k1["angle"][i1]) - f32(k2["angle"][bi])
                if rot < 0:
                    rot = f32(rot + f32(360))
                v = float(rot * (f32(30) / f32(360)))
                b = int(math.floor(v + 0.5))
                hist[0 if b == 30 else b].append(i1)
    if check_ori:
        sizes = [len(h) for h in hist]
        m1 = m2 = m3 = 0
        i1_ = i2_ = i3_ = -1
        for i, s in enumerate(sizes):
            if s > m1:
                m3, m2, m1, i3_, i2_, i1_ = m2, m1, s, i2_, i1_, i
            elif s > m2:
                m3, m2, i3_, i2_ = m2, s, i2_, i
            elif s > m3:
                m3, i3_ = s, i
        if f32(m2) < f32(0.1) * f32(m1):
            i2_ = i3_ = -1
        elif f32(m3) < f32(0.1) * f32(m1):
            i3_ = -1
        for i in range(30):
            if i in (i1_, i2_, i3_):
                continue
            for idx in hist[i]:
                if m12[idx] >= 0:
                    m12[idx] = -1
                    n -= 1
    return n, np.array(m12, np.int32)


@pytest.mark.parametrize("check_ori", [True, False])
def test_search_for_init_matches_transliteration(OB, check_ori):
    a, b = synth.make_image_pair(640, 300, seed=12, shift=(5.0, 2.0))
    p = OB.params(800)
    k1, d1 = OB.extract(p, a)
    k2, d2 = OB.extract(p, b)
    prev = np.ascontiguousarray(np.stack([k1["x"], k1["y"]], 1), np.float32)
    grid = (0.0, 640.0, 0.0, 300.0)
    n, m12, pr = OB.search_for_init(k1, d1, k2, d2, grid, prev, 100, 0.9, check_ori)
    n_py, m_py = _py_search_for_init(k1, d1, k2, d2, grid, prev, 100, 0.9, check_ori)
    assert n == n_py and n > 20
    np.testing.assert_array_equal(m12, m_py)
    ok = m12 >= 0
    np.testing.assert_array_equal(pr[ok, 0], k2["x"][m12[ok]])


def test_golden_extract_and_match(OB):
    g = np.load(GOLDEN)
    a, b = synth.make_image_pair(640, 300, seed=int(g["seed"]), shift=tuple(g["shift"]))
    p = OB.params(800)
    k1, d1 = OB.extract(p, a)
    k2, d2 = OB.extract(p, b)
    np.testing.assert_array_equal(np.asarray(a), g["img1"])
    for f in OB.KP_DTYPE.names:
        np.testing.assert_array_equal(k1[f], g["k1_" + f])
    np.testing.assert_array_equal(d1, g["d1"])
    np.testing.assert_array_equal(d2, g["d2"])
    prev = np.ascontiguousarray(np.stack([k1["x"], k1["y"]], 1), np.float32)
    n, m12, _ = OB.search_for_init(k1, d1, k2, d2, (0.0, 640.0, 0.0, 300.0), prev, 100, 0.9, True)
    assert n == int(g["n_matches"])
    np.testing.assert_array_equal(m12, g["m12"])


# ---- projection searches: the C oracle vs a second, pure-Python transliteration ----
def _py_grid(kps, bounds):
    import math
    f32 = np.float32
    minx, maxx, miny, maxy = (f32(v) for v in bounds)
    wi, hi = f32(64) / (maxx - minx), f32(48) / (maxy - miny)
    cells = [[[] for _ in range(48)] for _ in range(64)]
    for i in range(len(kps)):
        px = math.floor(float((f32(kps["x"][i]) - minx) * wi) + 0.5)
        py = math.floor(float((f32(kps["y"][i]) - miny) * hi) + 0.5)
        if 0 <= px < 64 and 0 <= py < 48:
            cells[px][py].append(i)
    return cells, minx, miny, wi, hi


def _py_area(G, kps, x, y, r, minL, maxL):
    """Frame::GetFeaturesInArea (Frame.cc:1463-1552)."""
    import math
    cells, minx, miny, wi, hi = G
    x, y, r = np.float32(x), np.float32(y), np.float32(r)
    x0 = max(0, math.floor((x - minx - r) * wi))
    if x0 >= 64:
        return []
    x1 = min(63, math.ceil((x - minx + r) * wi))
    if x1 < 0:
        return []
    y0 = max(0, math.floor((y - miny - r) * hi))
    if y0 >= 48:
        return []
    y1 = min(47, math.ceil((y - miny + r) * hi))
    if y1 < 0:
        return []
    check = minL > 0 or maxL >= 0
    out = []
    for ix in range(x0, x1 + 1):
        for iy in range(y0, y1 + 1):
            for j in cells[ix][iy]:
                o = kps["octave"][j]
                if check and (o < minL or (maxL >= 0 and o > maxL)):
                    continue
                if abs(kps["x"][j] - x) < r and abs(kps["y"][j] - y) < r:
                    out.append(j)
    return out


def _py_sbp_local(kps, desc, bounds, scale, uright, slot_mp, slot_obs, mps, mp_desc, th, nnratio):
    """ORBmatcher::SearchByProjection(F, vpMapPoints, th) (ORBmatcher.cc:67-181)."""
    f32 = np.float32
    G = _py_grid(kps, bounds)
    sm, so = slot_mp.copy(), slot_obs.copy()
    D = np.unpackbits(mp_desc[:, None, :] ^ desc[None, :, :], axis=2).sum(axis=2)
    n = 0
    for i, p in enumerate(mps):
        if not p["in_view"] or p["bad"]:
            continue
        lvl = int(p["level"])
        r = f32(2.5) if float(p["view_cos"]) > 0.998 else f32(4.0)
        if f32(th) != 1.0:
            r = r * f32(th)
        rw = r * scale[lvl]
        cand = _py_area(G, kps, p["proj_x"], p["proj_y"], rw, lvl - 1, lvl)
        if not cand:
            continue
        b1, l1, b2, l2, bi = 256, -1, 256, -1, -1
        for j in cand:
            if sm[j] >= 0 and so[j]:
                continue
            if uright is not None and uright[j] > 0 and abs(p["proj_xr"] - uright[j]) > rw:
                continue
            d = int(D[i, j])
            if d < b1:
                b2, l2, b1, l1, bi = b1, l1, d, int(kps["octave"][j]), j
            elif d < b2:
                l2, b2 = int(kps["octave"][j]), d
        if b1 <= 100:
            if l1 == l2 and f32(b1) > f32(nnratio) * f32(b2):
                continue
            sm[bi], so[bi] = p["id"], p["has_obs"]
            n += 1
    return n, sm, so


def _py_sbp_last(kps, desc, bounds, scale, cam, uright, slot_mp, slot_obs, Tcw, Tlw, lp, ldesc, th, mono, check_ori):
    """ORBmatcher::SearchByProjection(CurrentFrame, LastFrame, th, bMono) (ORBmatcher.cc:1717-1883)."""
    import math
    f32 = np.float32
    fx, fy, cx, cy, bf, mb = (f32(v) for v in cam)
    G = _py_grid(kps, bounds)
    sm, so = slot_mp.copy(), slot_obs.copy()
    D = np.unpackbits(ldesc[:, None, :] ^ desc[None, :, :], axis=2).sum(axis=2)

    def mul_add(A, x, c, sign):
        out = []
        for i in range(3):
            t0 = f32(A[i][0]) * f32(x[0]) + f32(A[i][1]) * f32(x[1]) + f32(A[i][2]) * f32(x[2])
            out.append(f32(float(t0) * sign + (float(c[i]) if c is not None else 0.0)))
        return out
    Tcw, Tlw = np.asarray(Tcw, f32), np.asarray(Tlw, f32)
    tcw, tlw = Tcw[:, 3], Tlw[:, 3]
    twc = mul_add(Tcw[:, :3].T, tcw, None, -1.0)
    tlc = mul_add(Tlw[:, :3], twc, tlw, 1.0)
    fwd = tlc[2] > mb and not mono
    bwd = -tlc[2] > mb and not mono
    n = 0
    hist = [[] for _ in range(30)]
    for i, p in enumerate(lp):
        if p["id"] < 0 or p["outlier"]:
            continue
        xc, yc, zc = mul_add(Tcw[:, :3], (p["x"], p["y"], p["z"]), tcw, 1.0)
        invz = f32(1.0 / float(zc))
        if invz < 0:
            continue
        u = fx * xc * invz + cx
        v = fy * yc * invz + cy
        if u < f32(bounds[0]) or u > f32(bounds[1]) or v < f32(bounds[2]) or v > f32(bounds[3]):
            continue
        o = int(p["octave"])
        rad = f32(th) * scale[o]
        lv = (o, -1) if fwd else (0, o) if bwd else (o - 1, o + 1)
        cand = _py_area(G, kps, u, v, rad, *lv)
        if not cand:
            continue
        b1, bi = 256, -1
        for j in cand:
            if sm[j] >= 0 and so[j]:
                continue
            if uright is not None and uright[j] > 0:
                ur = u - bf * invz
                if abs(ur - uright[j]) > rad:
                    continue
            d = int(D[i, j])
            if d < b1:
                b1, bi = d, j
        if b1 <= 100:
            sm[bi], so[bi] = p["id"], p["has_obs"]
            n += 1
            if check_ori:
                rot = f32(p["angle"]) - f32(kps["angle"][bi])
                if rot < 0:
                    rot = f32(rot + f32(360))
                b = int(math.floor(float(rot * (f32(30) / f32(360))) + 0.5))
                hist[0 if b == 30 else b].append(bi)
    if check_ori:
        sizes = [len(h) for h in hist]
        m1 = m2 = m3 = 0
        i1 = i2 = i3 = -1
        for i, s in enumerate(sizes):
            if s > m1:
                m3, m2, m1, i3, i2, i1 = m2, m1, s, i2, i1, i
            elif s > m2:
                m3, m2, i3, i2 = m2, s, i2, i
            elif s > m3:
                m3, i3 = s, i
        if f32(m2) < f32(0.1) * f32(m1):
            i2 = i3 = -1
        elif f32(m3) < f32(0.1) * f32(m1):
            i3 = -1
        for b in range(30):
            if b in (i1, i2, i3):
                continue
            for j in hist[b]:
                sm[j], so[j] = -1, 0
                n -= 1
    return n, sm, so


@pytest.fixture(scope="module")
def proj_scene(OB):
    from sqrtlm import orb_scene as S
    a, b = synth.make_image_pair(640, 300, seed=21, shift=(6.0, -2.0))
    p = OB.params(800)
    k1, d1 = OB.extract(p, a)
    k2, d2 = OB.extract(p, b)
    return S, k1, d1, k2, d2, (0.0, 640.0, 0.0, 300.0)


def test_features_in_area_matches_transliteration(OB, proj_scene):
    S, k1, d1, k2, d2, bounds = proj_scene
    G = _py_grid(k2, bounds)
    rng = np.random.default_rng(3)
    for _ in range(60):
        x, y = rng.uniform(-20, 660), rng.uniform(-20, 320)
        r = float(rng.choice([2.5, 4.0, 7.2, 30.0]))
        lv = [(-1, -1), (0, -1), (2, -1), (-1, 0), (0, 3), (1, 1), (3, 5)][rng.integers(7)]
        got = OB.features_in_area(k2, bounds, x, y, r, *lv)
        assert list(got) == _py_area(G, k2, x, y, r, *lv)
    assert len(OB.features_in_area(k2, bounds, 320, 150, 40)) > 0


@pytest.mark.parametrize("stereo,th", [(False, 1.0), (True, 1.0), (True, 3.0)])
def test_search_by_projection_local_matches_transliteration(OB, proj_scene, stereo, th):
    S, k1, d1, k2, d2, bounds = proj_scene
    mps, md = S.local_points(k1, d1, (6.0, -2.0), seed=5, stereo=stereo)
    ur, sm, so = S.current_slots(k2, 5, stereo)
    sf = S.scale_factors()
    n, m, o = OB.search_by_projection_local(k2, d2, bounds, sf, ur, sm, so, mps, md, th, 0.8)
    n_py, m_py, o_py = _py_sbp_local(k2, d2, bounds, sf, ur, sm, so, mps, md, th, 0.8)
    assert n == n_py and n > 30
    np.testing.assert_array_equal(m, m_py)
    np.testing.assert_array_equal(o, o_py)


@pytest.mark.parametrize("stereo,mono,tz,th,check_ori", [(False, True, 0.0, 7.0, True), (True, False, 1.0, 7.0, True),
                                                         (True, False, -1.0, 15.0, False),
                                                         (True, False, 0.0, 7.0, True)])
def test_search_by_projection_last_matches_transliteration(OB, proj_scene, stereo, mono, tz, th, check_ori):
    S, k1, d1, k2, d2, bounds = proj_scene
    Tcw, Tlw, lp, ld = S.last_frame(k1, d1, (6.0, -2.0), 640, 300, seed=9, tz=tz)
    ur, sm, so = S.current_slots(k2, 9, stereo)
    sf, cam = S.scale_factors(), S.camera(640, 300)
    n, m, o = OB.search_by_projection_last(k2, d2, bounds, sf, cam, ur, sm, so, Tcw, Tlw, lp, ld, th, mono, check_ori)
    n_py, m_py, o_py = _py_sbp_last(k2, d2, bounds, sf, cam, ur, sm, so, Tcw, Tlw, lp, ld, th, mono, check_ori)
    assert n == n_py and n > 20
    np.testing.assert_array_equal(m, m_py)
    np.testing.assert_array_equal(o, o_py)


# ---- keyframe projection and BoW searches vs pure-Python transliterations ----
def _f32_mul_add(A, x, c, sign=1.0):
    f32 = np.float32
    out = []
    for i in range(3):
        t0 = f32(A[i][0]) * f32(x[0]) + f32(A[i][1]) * f32(x[1]) + f32(A[i][2]) * f32(x[2])
        out.append(f32(float(t0) * sign + (float(c[i]) if c is not None else 0.0)))
    return out


def _py_pose(T, sim3):
    f32 = np.float32
    T = np.asarray(T, f32)[:3, :4]
    if sim3:
        s = f32(math.sqrt(sum(float(T[0, j]) * float(T[0, j]) for j in range(3))))
        inv = f32(1.0 / float(s))
        T = (T * inv).astype(f32)
    Ow = _f32_mul_add(T[:, :3].T, T[:, 3], None, -1.0)
    return T, Ow


def _py_norm_dot(PO, Pn):
    n = np.float32(math.sqrt(sum(float(v) * float(v) for v in PO)))
    d = sum(float(a) * float(b) for a, b in zip(PO, Pn))
    return n, d


def _py_predict(max_dist, dist, sf):
    f32 = np.float32
    ratio = f32(max_dist) / f32(dist)
    ls = f32(math.log(float(sf[1])))
    v = f32(f32(math.log(float(ratio))) / ls)
    s = math.ceil(float(v))
    return 0 if s < 0 else min(s, len(sf) - 1)


def _py_project_kf(T, Ow, p, cam, bounds, sf):
    f32 = np.float32
    X = (p["x"], p["y"], p["z"])
    Xc = _f32_mul_add(T[:, :3], X, T[:, 3])
    if Xc[2] < 0:
        return None
    invz = f32(1) / Xc[2]
    u = f32(cam[0]) * (Xc[0] * invz) + f32(cam[2])
    v = f32(cam[1]) * (Xc[1] * invz) + f32(cam[3])
    if not (u >= f32(bounds[0]) and u < f32(bounds[1]) and v >= f32(bounds[2]) and v < f32(bounds[3])):
        return None
    PO = [f32(X[i]) - Ow[i] for i in range(3)]
    dist, dot = _py_norm_dot(PO, (p["nx"], p["ny"], p["nz"]))
    if dist < f32(1.2) * p["max_dist"] and dist >= f32(0.8) * p["min_dist"] and not dot < 0.5 * float(dist):
        return u, v, invz, _py_predict(p["max_dist"], dist, sf)
    return None


def _py_sbp_sim3(kps, desc, bounds, sf, cam, slot_mp, Scw, mps, md, th):
    T, Ow = _py_pose(Scw, True)
    G = _py_grid(kps, bounds)
    D = np.unpackbits(md[:, None, :] ^ desc[None, :, :], axis=2).sum(axis=2)
    sm = slot_mp.copy()
    n = 0
    for i, p in enumerate(mps):
        if p["skip"]:
            continue
        r = _py_project_kf(T, Ow, p, cam, bounds, sf)
        if r is None:
            continue
        u, v, _, pl = r
        bd, bi = 256, -1
        for j in _py_area(G, kps, u, v, np.float32(th) * sf[pl], -1, -1):
            if sm[j] >= 0 or kps["octave"][j] < pl - 1 or kps["octave"][j] > pl:
                continue
            if D[i, j] < bd:
                bd, bi = int(D[i, j]), j
        if bd <= 50:
            sm[bi] = p["id"]
            n += 1
    return n, sm


def _py_fuse(kps, desc, bounds, sf, cam, uright, T, sim3, mps, md, th):
    f32 = np.float32
    T, Ow = _py_pose(T, sim3)
    G = _py_grid(kps, bounds)
    D = np.unpackbits(md[:, None, :] ^ desc[None, :, :], axis=2).sum(axis=2)
    out = np.full(len(mps), -1, np.int32)
    n = 0
    for i, p in enumerate(mps):
        if p["skip"]:
            continue
        r = _py_project_kf(T, Ow, p, cam, bounds, sf)
        if r is None:
            continue
        u, v, invz, pl = r
        ur = u - f32(cam[4]) * invz
        bd, bi = (2 ** 31 - 1) if sim3 else 256, -1
        for j in _py_area(G, kps, u, v, f32(th) * sf[pl], -1, -1):
            lv = int(kps["octave"][j])
            if lv < pl - 1 or lv > pl:
                continue
            if not sim3:
                inv = f32(1.0) / (sf[lv] * sf[lv])
                ex, ey = u - kps["x"][j], v - kps["y"][j]
                if uright is not None and uright[j] >= 0:
                    er = ur - uright[j]
                    if float((ex * ex + ey * ey + er * er) * inv) > 7.8:
                        continue
                elif float((ex * ex + ey * ey) * inv) > 5.99:
                    continue
            if D[i, j] < bd:
                bd, bi = int(D[i, j]), j
        if bd <= 50:
            out[i] = bi
            n += 1
    return n, out


def _py_hist_reject(hist_entries, clear):
    """ComputeThreeMaxima + removal; hist_entries: list of (bin, payload). Returns removed count."""
    f32 = np.float32
    sizes = [0] * 30
    for b, _ in hist_entries:
        sizes[b] += 1
    m1 = m2 = m3 = 0
    i1 = i2 = i3 = -1
    for i, s in enumerate(sizes):
        if s > m1:
            m3, m2, m1, i3, i2, i1 = m2, m1, s, i2, i1, i
        elif s > m2:
            m3, m2, i3, i2 = m2, s, i2, i
        elif s > m3:
            m3, i3 = s, i
    if f32(m2) < f32(0.1) * f32(m1):
        i2 = i3 = -1
    elif f32(m3) < f32(0.1) * f32(m1):
        i3 = -1
    removed = 0
    for b in range(30):
        if b in (i1, i2, i3):
            continue
        for bb, pay in hist_entries:
            if bb == b:
                clear(pay)
                removed += 1
    return removed


def _py_bin(a1, a2):
    f32 = np.float32
    rot = f32(a1) - f32(a2)
    if rot < 0:
        rot = f32(rot + f32(360))
    b = int(math.floor(float(rot * (f32(30) / f32(360))) + 0.5))
    return 0 if b == 30 else b


def _py_sbp_kf(kps, desc, bounds, sf, cam, slot_mp, Tcw, mps, md, ang, th, orb_dist, check_ori):
    f32 = np.float32
    T, Ow = _py_pose(Tcw, False)
    G = _py_grid(kps, bounds)
    D = np.unpackbits(md[:, None, :] ^ desc[None, :, :], axis=2).sum(axis=2)
    sm = slot_mp.copy()
    n = 0
    hist = []
    for i, p in enumerate(mps):
        if p["skip"]:
            continue
        X = (p["x"], p["y"], p["z"])
        Xc = _f32_mul_add(T[:, :3], X, T[:, 3])
        invz = f32(1.0 / float(Xc[2]))
        u = f32(cam[0]) * Xc[0] * invz + f32(cam[2])
        v = f32(cam[1]) * Xc[1] * invz + f32(cam[3])
        if u < f32(bounds[0]) or u > f32(bounds[1]) or v < f32(bounds[2]) or v > f32(bounds[3]):
            continue
        dist, _ = _py_norm_dot([f32(X[k]) - Ow[k] for k in range(3)], (0, 0, 0))
        if dist < f32(0.8) * p["min_dist"] or dist > f32(1.2) * p["max_dist"]:
            continue
        pl = _py_predict(p["max_dist"], dist, sf)
        bd, bi = 256, -1
        for j in _py_area(G, kps, u, v, f32(th) * sf[pl], pl - 1, pl + 1):
            if sm[j] >= 0:
                continue
            if D[i, j] < bd:
                bd, bi = int(D[i, j]), j
        if bd <= orb_dist:
            sm[bi] = p["id"]
            n += 1
            if check_ori:
                hist.append((_py_bin(ang[i], kps["angle"][bi]), bi))
    if check_ori:
        n -= _py_hist_reject(hist, lambda j: sm.__setitem__(j, -1))
    return n, sm


def _py_common_nodes(node1, node2):
    nodes = sorted(set(int(v) for v in node1 if v >= 0) & set(int(v) for v in node2 if v >= 0))
    for nd in nodes:
        yield [i for i in range(len(node1)) if node1[i] == nd], [j for j in range(len(node2)) if node2[j] == nd]


def _py_bow_kf_frame(kf, f, nnratio, check_ori):
    k1, d1, n1, mp1, bad1 = kf
    k2, d2, n2 = f[:3]
    D = np.unpackbits(d1[:, None, :] ^ d2[None, :, :], axis=2).sum(axis=2)
    out = np.full(len(k2), -1, np.int32)
    n, hist = 0, []
    for r1, r2 in _py_common_nodes(n1, n2):
        for i in r1:
            if mp1[i] < 0 or bad1[i]:
                continue
            b1, b2, bi = 256, 256, -1
            for j in r2:
                if out[j] >= 0:
                    continue
                d = int(D[i, j])
                if d < b1:
                    b2, b1, bi = b1, d, j
                elif d < b2:
                    b2 = d
            if b1 <= 50 and np.float32(b1) < np.float32(nnratio) * np.float32(b2):
                out[bi] = mp1[i]
                if check_ori:
                    hist.append((_py_bin(k1["angle"][i], k2["angle"][bi]), bi))
                n += 1
    if check_ori:
        n -= _py_hist_reject(hist, lambda j: out.__setitem__(j, -1))
    return n, out


def _py_bow_kf_kf(a, b, nnratio, check_ori):
    k1, d1, n1, mp1, bad1 = a
    k2, d2, n2, mp2, bad2 = b
    D = np.unpackbits(d1[:, None, :] ^ d2[None, :, :], axis=2).sum(axis=2)
    out = np.full(len(k1), -1, np.int32)
    matched = np.zeros(len(k2), bool)
    n, hist = 0, []
    for r1, r2 in _py_common_nodes(n1, n2):
        for i in r1:
            if mp1[i] < 0 or bad1[i]:
                continue
            b1, b2, bi = 256, 256, -1
            for j in r2:
                if matched[j] or mp2[j] < 0 or bad2[j]:
                    continue
                d = int(D[i, j])
                if d < b1:
                    b2, b1, bi = b1, d, j
                elif d < b2:
                    b2 = d
            if b1 < 50 and np.float32(b1) < np.float32(nnratio) * np.float32(b2):
                out[i] = mp2[bi]
                matched[bi] = True
                if check_ori:
                    hist.append((_py_bin(k1["angle"][i], k2["angle"][bi]), i))
                n += 1
    if check_ori:
        n -= _py_hist_reject(hist, lambda i: out.__setitem__(i, -1))
    return n, out


def _py_triangulation(a, b, C1, T2w, cam2, sf2, F12, only_stereo, check_ori):
    f32 = np.float32
    k1, d1, n1, mp1, _, ur1 = a
    k2, d2, n2, mp2, _, ur2 = b
    C2 = _f32_mul_add(T2w[:, :3], C1, T2w[:, 3])
    invz = f32(1.0) / C2[2]
    ex = f32(cam2[0]) * C2[0] * invz + f32(cam2[2])
    ey = f32(cam2[1]) * C2[1] * invz + f32(cam2[3])
    D = np.unpackbits(d1[:, None, :] ^ d2[None, :, :], axis=2).sum(axis=2)
    m12 = np.full(len(k1), -1, np.int32)
    matched = np.zeros(len(k2), bool)
    n, hist = 0, []
    F = np.asarray(F12, f32)
    for r1, r2 in _py_common_nodes(n1, n2):
        for i in r1:
            if mp1[i] >= 0:
                continue
            s1 = ur1 is not None and ur1[i] >= 0
            if only_stereo and not s1:
                continue
            x1, y1 = k1["x"][i], k1["y"][i]
            bd, bi = 50, -1
            for j in r2:
                if matched[j] or mp2[j] >= 0:
                    continue
                s2 = ur2 is not None and ur2[j] >= 0
                if only_stereo and not s2:
                    continue
                d = int(D[i, j])
                if d > 50 or d > bd:
                    continue
                x2, y2, o2 = k2["x"][j], k2["y"][j], int(k2["octave"][j])
                if not s1 and not s2:
                    dx, dy = ex - x2, ey - y2
                    if dx * dx + dy * dy < f32(100) * sf2[o2]:
                        continue
                la = x1 * F[0, 0] + y1 * F[1, 0] + F[2, 0]
                lb = x1 * F[0, 1] + y1 * F[1, 1] + F[2, 1]
                lc = x1 * F[0, 2] + y1 * F[1, 2] + F[2, 2]
                num = la * x2 + lb * y2 + lc
                den = la * la + lb * lb
                if den == 0:
                    continue
                if float(num * num / den) < 3.84 * float(sf2[o2] * sf2[o2]):
                    bi, bd = j, d
            if bi >= 0:
                m12[i] = bi
                matched[bi] = True
                n += 1
                if check_ori:
                    hist.append((_py_bin(k1["angle"][i], k2["angle"][bi]), i))

    def clear(i):
        matched[m12[i]] = False
        m12[i] = -1
    if check_ori:
        n -= _py_hist_reject(hist, clear)
    return n, m12


@pytest.fixture(scope="module")
def kf_scene(OB, proj_scene):
    S, k1, d1, k2, d2, bounds = proj_scene
    cam = S.camera(640, 300)
    mps, md = S.map_points(k1, d1, 640, 300, seed=2)
    return S, k1, d1, k2, d2, bounds, cam, mps, md


@pytest.mark.parametrize("s,th", [(1.0, 10), (1.3, 10), (0.8, 4)])
def test_search_by_projection_sim3_matches_transliteration(OB, kf_scene, s, th):
    S, k1, d1, k2, d2, bounds, cam, mps, md = kf_scene
    Scw = S.sim3_of(S.keyframe_pose((6.0, -2.0), 640, 300, (0.02, 0.0, 0.1)), s)
    _, sm, _ = S.current_slots(k2, 2, False)
    sf = S.scale_factors()
    n, m = OB.search_by_projection_sim3(k2, d2, bounds, sf, cam, sm, Scw, mps, md, th)
    n_py, m_py = _py_sbp_sim3(k2, d2, bounds, sf, cam, sm, Scw, mps, md, th)
    assert n == n_py and n > 20
    np.testing.assert_array_equal(m, m_py)


@pytest.mark.parametrize("sim3,stereo,th", [(False, False, 3.0), (False, True, 5.0), (True, False, 4.0)])
def test_fuse_matches_transliteration(OB, kf_scene, sim3, stereo, th):
    S, k1, d1, k2, d2, bounds, cam, mps, md = kf_scene
    T = S.keyframe_pose((6.0, -2.0), 640, 300, (0.0, 0.01, 0.05))
    if sim3:
        T = S.sim3_of(T, 1.2)
    ur, _, _ = S.current_slots(k2, 3, stereo)
    sf = S.scale_factors()
    n, idx = OB.fuse(k2, d2, bounds, sf, cam, ur, T, sim3, mps, md, th)
    n_py, idx_py = _py_fuse(k2, d2, bounds, sf, cam, ur, T, sim3, mps, md, th)
    assert n == n_py and n > 10
    np.testing.assert_array_equal(idx, idx_py)


@pytest.mark.parametrize("th,orb_dist,check_ori", [(10.0, 100, True), (3.0, 64, False)])
def test_search_by_projection_kf_matches_transliteration(OB, kf_scene, th, orb_dist, check_ori):
    S, k1, d1, k2, d2, bounds, cam, mps, md = kf_scene
    Tcw = S.keyframe_pose((6.0, -2.0), 640, 300, (0.01, 0.0, -0.1))
    _, sm, _ = S.current_slots(k2, 4, False)
    sf = S.scale_factors()
    n, m = OB.search_by_projection_kf(k2, d2, bounds, sf, cam, sm, Tcw, mps, md, k1["angle"], th, orb_dist,
                                      check_ori)
    n_py, m_py = _py_sbp_kf(k2, d2, bounds, sf, cam, sm, Tcw, mps, md, k1["angle"], th, orb_dist, check_ori)
    assert n == n_py and n > 20
    np.testing.assert_array_equal(m, m_py)


@pytest.mark.parametrize("check_ori", [True, False])
def test_search_by_bow_matches_transliteration(OB, proj_scene, check_ori):
    S, k1, d1, k2, d2, bounds = proj_scene
    n1, n2 = S.bow_nodes(d1, 1), S.bow_nodes(d2, 2)
    mp1, bad1 = S.bow_points(len(k1), 1)
    mp2, bad2 = S.bow_points(len(k2), 2, base=10000)
    a = (k1, d1, n1, mp1, bad1)
    n, out = OB.search_by_bow_kf_frame(a, (k2, d2, n2, mp2), 0.7, check_ori)
    n_py, out_py = _py_bow_kf_frame(a, (k2, d2, n2), 0.7, check_ori)
    assert n == n_py and n > 20
    np.testing.assert_array_equal(out, out_py)
    b = (k2, d2, n2, mp2, bad2)
    n, out = OB.search_by_bow_kf_kf(a, b, 0.75, check_ori)
    n_py, out_py = _py_bow_kf_kf(a, b, 0.75, check_ori)
    assert n == n_py and n > 20
    np.testing.assert_array_equal(out, out_py)


@pytest.mark.parametrize("stereo,only_stereo,check_ori", [(False, False, False), (True, False, True),
                                                          (True, True, False)])
def test_search_for_triangulation_matches_transliteration(OB, proj_scene, stereo, only_stereo, check_ori):
    S, k1, d1, k2, d2, bounds = proj_scene
    cam = S.camera(640, 300)
    T1 = S.keyframe_pose((0.0, 0.0), 640, 300)
    T2 = S.keyframe_pose((6.0, -2.0), 640, 300, (0.3, 0.0, 0.05))
    F12 = S.fundamental_12(T1, T2, cam, cam)
    n1, n2 = S.bow_nodes(d1, 5), S.bow_nodes(d2, 6)
    mp1, _ = S.bow_points(len(k1), 5, frac=0.3)
    mp2, _ = S.bow_points(len(k2), 6, frac=0.3)
    ur1, _, _ = S.current_slots(k1, 5, stereo)
    ur2, _, _ = S.current_slots(k2, 6, stereo)
    C1 = np.zeros(3, np.float32)
    a = (k1, d1, n1, mp1, None, ur1)
    b = (k2, d2, n2, mp2, None, ur2)
    sf = S.scale_factors()
    n, m12 = OB.search_for_triangulation(a, b, C1, T2, cam[:4], sf, F12, only_stereo, check_ori)
    n_py, m_py = _py_triangulation(a, b, C1, T2, cam[:4], sf, F12, only_stereo, check_ori)
    assert n == n_py and n > 5
    np.testing.assert_array_equal(m12, m_py)


def _py_sim3_dir(cam, kd, bounds, sf, Tsw, sR, t, mps, md, already, th):
    f32 = np.float32
    G = _py_grid(kd[0], bounds)
    D = np.unpackbits(md[:, None, :] ^ kd[1][None, :, :], axis=2).sum(axis=2)
    out = np.full(len(mps), -1, np.int32)
    for i, p in enumerate(mps):
        if p["id"] < 0 or already[i] or p["skip"]:
            continue
        Xs = _f32_mul_add(Tsw[:, :3], (p["x"], p["y"], p["z"]), Tsw[:, 3])
        Xd = _f32_mul_add(sR, Xs, t)
        if Xd[2] < 0:
            continue
        invz = f32(1.0 / float(Xd[2]))
        u = f32(cam[0]) * (Xd[0] * invz) + f32(cam[2])
        v = f32(cam[1]) * (Xd[1] * invz) + f32(cam[3])
        if not (u >= f32(bounds[0]) and u < f32(bounds[1]) and v >= f32(bounds[2]) and v < f32(bounds[3])):
            continue
        dist, _ = _py_norm_dot(Xd, (0, 0, 0))
        if dist < f32(0.8) * p["min_dist"] or dist > f32(1.2) * p["max_dist"]:
            continue
        pl = _py_predict(p["max_dist"], dist, sf)
        bd, bi = 2 ** 31 - 1, -1
        for j in _py_area(G, kd[0], u, v, f32(th) * sf[pl], -1, -1):
            o = kd[0]["octave"][j]
            if o < pl - 1 or o > pl:
                continue
            if D[i, j] < bd:
                bd, bi = int(D[i, j]), j
        if bd <= 100:
            out[i] = bi
    return out


def _py_search_by_sim3(k1, d1, k2, d2, bounds, sf, cam, T1, T2, mp1, md1, mp2, md2, s12, R12, t12, th, m12):
    f32 = np.float32
    R12 = np.asarray(R12, f32)
    sR12 = (R12 * f32(s12)).astype(f32)
    sR21 = (R12.T * f32(1.0 / float(f32(s12)))).astype(f32)
    t21 = _f32_mul_add(sR21, t12, None, -1.0)
    am1 = m12 >= 0
    ids = set(int(v) for v in m12 if v >= 0)
    am2 = np.array([int(v) in ids for v in mp2["id"]])
    v1 = _py_sim3_dir(cam, (k2, d2), bounds, sf, np.asarray(T1, f32), sR21, t21, mp1, md1, am1, th)
    v2 = _py_sim3_dir(cam, (k1, d1), bounds, sf, np.asarray(T2, f32), sR12, np.asarray(t12, f32), mp2, md2, am2, th)
    out = m12.copy()
    n = 0
    for i1 in range(len(k1)):
        j = v1[i1]
        if j >= 0 and v2[j] == i1:
            out[i1] = mp2["id"][j]
            n += 1
    return n, out


@pytest.mark.parametrize("s12,th", [(1.0, 7.5), (1.03, 10.0)])
def test_search_by_sim3_matches_transliteration(OB, proj_scene, s12, th):
    S, k1, d1, k2, d2, bounds = proj_scene
    cam = S.camera(640, 300)
    T1, T2, mp1, md1, mp2, md2, R12, t12, m12 = S.sim3_scene(k1, d1, k2, d2, (6.0, -2.0), 640, 300, 3)
    sf = S.scale_factors()
    n, m = OB.search_by_sim3(k1, d1, k2, d2, bounds, sf, cam, T1, T2, mp1, md1, mp2, md2, s12, R12, t12, th, m12)
    n_py, m_py = _py_search_by_sim3(k1, d1, k2, d2, bounds, sf, cam, T1, T2, mp1, md1, mp2, md2, s12, R12, t12, th,
                                    m12)
    assert n == n_py and n > 20
    np.testing.assert_array_equal(m, m_py)
