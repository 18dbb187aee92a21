"""Oracle known-answer tests (CPU).  The reference ships no tests or golden data; what
pins the oracle is (a) the RNG KATs derived from assets/raytracing.glsl:13-25,
(b) analytic cases for every intersection routine, (c) the rgba8 store/load rules, and (d) the
accuracy of the pinned transcendentals against libm in float64."""
import math

import numpy as np
import pytest

import pyoracle as O
from epq_raytracer_amd import _lib

FLT_MAX = float(np.float32(3.402823466e38))


def test_hash_kats_from_survey():
    # seed 1*719393 + 0 (frame 1, pixel 0) and seed 0
    assert O.hash_sequence(719393, 4) == [3032883327, 3675371623, 163780757, 779951943]
    assert O.hash_sequence(0, 4) == [1739749167, 1640446612, 2645431204, 4252402365]


def test_hash_matches_python_restatement():
    def h(s):
        s ^= 2747636419; s = (s * 2654435769) & 0xFFFFFFFF
        s ^= s >> 16; s = (s * 2654435769) & 0xFFFFFFFF
        s ^= s >> 16; s = (s * 2654435769) & 0xFFFFFFFF
        return s
    for seed in (0, 1, 12345, 0xFFFFFFFF, 719393 * 7 + 99):
        seq, s = [], seed
        for _ in range(16):
            s = h(s); seq.append(s)
        assert O.hash_sequence(seed, 16) == seq


def test_scale01_values():
    # u01 = float(s) / float(4294967295.0) = float_rne(s) * 2^-32
    assert O.scale01(0) == 0.0
    assert O.scale01(0xFFFFFFFF) == 1.0          # float(2^32-1) rounds to 2^32
    assert O.scale01(3032883327) == pytest.approx(0.706148148, abs=1e-8)
    for s in (1, 3675371623, 163780757, 779951943, 2**31):
        assert O.scale01(s) == float(np.float32(s)) / 2.0**32


def test_u01_endpoint_test_on_hash_bits():
    """adjust_dir's fast path (csrc/hrt_kernels.hip, HRT_FUZZ_INT) decides u01(h) not in {0, 1} as the
    integer compare (h - 1) mod 2^32 < 0xFFFFFF7F: u01(h) is 0 iff h == 0 and 1 iff float_rne(h) == 2^32,
    i.e. h >= 2^32 - 128.  Checked here on both ends of the range and a random sample (the device
    self-check hrt_debug_math_check_rng covers all 2^32 states)."""
    rng = np.random.default_rng(5)
    hs = np.concatenate([np.arange(0, 1 << 20, dtype=np.uint64),
                         np.arange((1 << 32) - (1 << 20), 1 << 32, dtype=np.uint64),
                         rng.integers(0, 1 << 32, 1 << 20, dtype=np.uint64)]).astype(np.uint32)
    u = hs.astype(np.float32) * np.float32(2.0 ** -32)
    fast_float = (u != 0.0) & (u != 1.0)
    fast_int = (hs - np.uint32(1)) < np.uint32(0xFFFFFF7F)
    np.testing.assert_array_equal(fast_int, fast_float)
    assert O.scale01(0xFFFFFF7F) < 1.0 and O.scale01(0xFFFFFF80) == 1.0


def test_spec_log_accuracy_and_specials():
    rng = np.random.default_rng(1)
    xs = np.concatenate([rng.random(4000), rng.random(500) * 1e-40, [1.0, 2.0**-32, 0.5, 1e-45, 3.0, 1e30]])
    for x in xs.astype(np.float32):
        y = O.spec_log(float(x))
        r = math.log(float(x))
        assert abs(y - r) <= 1.0 * abs(float(np.spacing(np.float32(r)))) + 1e-45
    assert O.spec_log(0.0) == -math.inf
    assert O.spec_log(1.0) == 0.0
    assert math.isnan(O.spec_log(-1.0))
    assert O.spec_log(math.inf) == math.inf


def test_spec_sincos_accuracy():
    rng = np.random.default_rng(2)
    for x in (rng.random(4000) * 2 * math.pi).astype(np.float32):
        assert abs(O.spec_sin(float(x)) - math.sin(float(x))) < 2e-7
        assert abs(O.spec_cos(float(x)) - math.cos(float(x))) < 2e-7
    assert O.spec_sin(0.0) == 0.0 and O.spec_cos(0.0) == 1.0
    assert math.isnan(O.spec_sin(math.inf)) and math.isnan(O.spec_cos(math.nan))


def test_normal_dist_consumes_two_hashes_and_u2_zero_gives_inf():
    v, s = O.normal_dist(0)
    assert O.hash_sequence(0, 2)[-1] == s  # two hashes drawn
    p, s2 = O.point_on_sphere(0)
    assert abs(float(np.linalg.norm(p.astype(np.float64))) - 1.0) < 1e-6
    assert O.hash_sequence(0, 6)[-1] == s2  # six hashes drawn (x, y, z)


def test_unorm8_rules():
    assert O.unorm8(0.0) == 0 and O.unorm8(-3.0) == 0 and O.unorm8(math.nan) == 0
    assert O.unorm8(1.0) == 255 and O.unorm8(7.5) == 255 and O.unorm8(math.inf) == 255
    assert O.unorm8(0.5) == 128                       # rint(127.5) -> 128 (ties to even)
    assert O.unorm8(float(np.float32(1.5 / 255))) == 2  # 1.5 -> 2 (even)
    assert O.unorm8(float(np.float32(2.5 / 255))) == 2  # 2.5 -> 2 (even)
    for k in range(256):
        assert O.unorm8(float(np.float32(k) / np.float32(255))) == k  # load/store round trip


def _tri(a, b, c):
    a, b, c = (np.asarray(v, np.float32) for v in (a, b, c))
    t = np.zeros((), dtype=_lib.TRIANGLE_DTYPE)
    e1, e2 = b - a, c - a
    n = np.float32([e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]])
    t["a"][:3], t["edge_one"][:3], t["edge_two"][:3], t["normal"][:3] = a, e1, e2, n
    return t


def test_intersecting_tri_kats():
    t = _tri([0, 0, 0], [1, 0, 0], [0, 1, 0])       # normal +z
    np.testing.assert_array_equal(O.intersecting_tri(t, [0.25, 0.25, 1], [0, 0, -1]), [0, 0, 1, 1])
    # back face: culled with (0,0,0,FLT_MAX) (raytracing.glsl:217-219)
    np.testing.assert_array_equal(O.intersecting_tri(t, [0.25, 0.25, -1], [0, 0, 1]), [0, 0, 0, FLT_MAX])
    # outside the triangle / behind the origin: vec4(FLT_MAX)
    np.testing.assert_array_equal(O.intersecting_tri(t, [2, 2, 1], [0, 0, -1]), [FLT_MAX] * 4)
    np.testing.assert_array_equal(O.intersecting_tri(t, [0.25, 0.25, -1], [0, 0, -1]), [FLT_MAX] * 4)
    # on an edge (u == 0) and on a vertex: accepted (tests are strict '< 0')
    assert O.intersecting_tri(t, [0.0, 0.5, 2], [0, 0, -1])[3] == 2.0
    assert O.intersecting_tri(t, [0.0, 0.0, 2], [0, 0, -1])[3] == 2.0
    # grazing ray in the plane: dot(d, n) == 0 -> culled
    np.testing.assert_array_equal(O.intersecting_tri(t, [-1, 0.25, 0], [1, 0, 0]), [0, 0, 0, FLT_MAX])
    # the normal is normalised on a hit, the record's normal is not
    big = _tri([0, 0, 0], [4, 0, 0], [0, 4, 0])
    np.testing.assert_array_equal(O.intersecting_tri(big, [1, 1, 3], [0, 0, -1]), [0, 0, 1, 3])


def test_intersecting_aabb_quirks():
    # the reference's slab test returns true as soon as any running bound is positive
    # (raytracing.glsl:199,203,207): a box off to the side but ahead in x "passes"
    assert O.intersecting_aabb([1, 5, 0], [2, 6, 1], [0, 0, 0], [1, 0, 0])
    # a box entirely behind the origin is culled
    assert not O.intersecting_aabb([1, 1, 1], [2, 2, 2], [0, 0, 0], [-1, -1, -1])
    # a box containing the origin passes
    assert O.intersecting_aabb([-1, -1, -1], [1, 1, 1], [0, 0, 0], [0.6, 0.0, 0.8])
    # sign of a zero direction component matters: 1/-0 = -inf selects the min corner
    # ((1-3) * -inf = +inf > 0 -> pass), 1/+0 = +inf gives -inf bounds (-> culled)
    assert O.intersecting_aabb([1, 1, 1], [2, 2, 2], [3, 3, 3], [-0.0, 1.0, 1.0])
    assert not O.intersecting_aabb([1, 1, 1], [2, 2, 2], [3, 3, 3], [0.0, 1.0, 1.0])


def _octant_pass(mn, mx, o, d):
    """The kernels' primary-ray AABB shortcut (hrt_kernels.hip aabb_truth_table): the reference's
    quirked test evaluated at the direction's sign octant (+-1 per axis) instead of d itself."""
    sd = [(-1.0 if math.copysign(1.0, float(v)) < 0 else 1.0) for v in np.float32(d)]
    return O.intersecting_aabb(mn, mx, o, sd)


def test_aabb_octant_rule_matches_quirked_test():
    # valid while every bound - o is nonzero and not NaN and |d| <= 1.5 per component
    rng = np.random.default_rng(7)
    specials = np.float32([0.0, -0.0, 1e-30, -1e-30, 1e-45, -1e-45, 1.0, -1.0, 1.5, -1.5, 1e-7, -1e-7])
    n = 0
    for i in range(6000):
        o = rng.uniform(-20, 20, 3).astype(np.float32)
        a, b = rng.uniform(-20, 20, 3).astype(np.float32), rng.uniform(-20, 20, 3).astype(np.float32)
        if i % 7 == 0:  # bounds one ulp off the origin
            a = np.nextafter(o, np.float32(np.inf)).astype(np.float32)
        if i % 11 == 0:
            b = np.nextafter(o, np.float32(-np.inf)).astype(np.float32)
        mn, mx = np.minimum(a, b), np.maximum(a, b)
        d = rng.normal(size=3).astype(np.float32)
        d = (d / np.float32(np.sqrt(np.float32(d @ d)))).astype(np.float32)
        if i % 3 == 0:
            d[rng.integers(0, 3)] = specials[rng.integers(0, len(specials))]
        if i % 5 == 0:
            d = rng.choice(specials, 3)
        assert np.all(mn - o != 0) and np.all(mx - o != 0)
        assert O.intersecting_aabb(mn, mx, o, d) == _octant_pass(mn, mx, o, d), (mn, mx, o, d)
        n += 1
    assert n == 6000


def test_accumulate_semantics():
    new = np.full((2, 3, 4), 200, np.uint8)
    cur = np.full((2, 3, 4), 77, np.uint8)
    O.accumulate_rgba8(0, cur, new)
    assert (cur[..., :3] == 0).all() and (cur[..., 3] == 255).all()  # frame 0 clears (image_combiner.glsl:33-36)
    O.accumulate_rgba8(1, cur, new)                                    # (200/255 + 0*1)/2 -> 100
    assert (cur[..., :3] == 100).all()
    O.accumulate_rgba8(2, cur, new)                                    # (200 + 100*2)/3 -> 133.33 -> 133
    assert (cur[..., :3] == 133).all()
    f = np.zeros((1, 1, 4), np.float32)
    O.accumulate_rgba32f(1, f, np.float32([[[0.5, 1.0, 2.0, 1.0]]]))
    np.testing.assert_array_equal(f, np.float32([[[0.25, 0.5, 1.0, 1.0]]]))
