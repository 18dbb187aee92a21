"""The BUNDLE_BVH hierarchy as hrt_set_scene builds it (host C++, csrc/hrt_bvh.cpp), inspected on the
CPU through hrt_debug_bvh_build: the structural facts the kernel's exact cull relies on (DESIGN.md
"BVH cull").  The GPU parity tests check the frames; these check the invariants directly.

* every (mesh, triangle) entry of the reference's scan sits in exactly one of: a leaf, the
  irregular list (tested for every ray), or "never" (zero normal: raytracing.glsl:219 rejects it);
* leaf records carry the entry's scan key (1 + position in mesh order, then index order);
* the preorder / escape links visit every node once; child boxes nest in their parent's box and
  every leaf triangle's vertices lie in its leaf box; the normal cone bounds every normal below;
* grazing band: for random directions d, every regular triangle with d.n^ in
  (-kBandTau - 1e-5, 2e-5) is in the band list of d's cube-map cell, the cell computed in binary32
  exactly as the kernel's dir_cell does."""
import ctypes

import numpy as np
import pytest

from helpers import E, SceneCase, _lib

TAU_G = np.float32(3e-3)     # hrt_bvh.h kBandTau
DIR_RES_MAX = 256          # hrt_bvh.h kDirResMax (the scene's resolution comes back in counts[6])


def build(tris, meshes, leaf=4):
    lib = _lib.load()
    counts = (ctypes.c_uint32 * 7)()
    P = ctypes.c_void_p
    r = lib.hrt_debug_bvh_build(tris.ctypes.data, len(tris), meshes.ctypes.data, len(meshes), leaf, counts,
                                None, 0, None, 0, None, 0, None, 0, None, 0)
    nn, npr, nirr, nnever, built, nband, res = list(counts)
    if not built:
        return None
    nodes = np.zeros(max(nn, 1) * 16, np.float32)
    prims = np.zeros(max(npr, 1) * 16, np.float32)
    irr = np.zeros(max(nirr, 1) * 16, np.float32)
    boff = np.zeros(6 * res * res + 1, np.uint32)
    band = np.zeros(max(nband, 1), np.uint32)
    r = lib.hrt_debug_bvh_build(tris.ctypes.data, len(tris), meshes.ctypes.data, len(meshes), leaf, counts,
                                P(nodes.ctypes.data), nodes.size, P(prims.ctypes.data), prims.size,
                                P(irr.ctypes.data), irr.size, P(boff.ctypes.data), boff.size,
                                P(band.ctypes.data), band.size)
    assert r == 1
    return dict(nodes=nodes[:nn * 16].reshape(nn, 16), prims=prims[:npr * 16].reshape(npr, 16),
                irregular=irr[:nirr * 16].reshape(nirr, 16), never=nnever, band_off=boff, dir_res=res,
                band=band[:nband])


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def ubits(x):
    return int(np.array([x], np.float32).view(np.uint32)[0])


def scan_entries(tris, meshes):
    """(key, mesh, index) of every entry of the reference's scan, in scan order."""
    out, key = [], 1
    for m, mesh in enumerate(meshes):
        for k in range(int(mesh["len"])):
            out.append((key, m, int(mesh["first_index"]) + k))
            key += 1
    return out


def adversarial_soup(seed=11):
    rng = np.random.default_rng(seed)
    v = []
    for _ in range(150):  # slivers
        a = rng.uniform(-3, 3, 3)
        b = a + rng.uniform(-2, 2, 3)
        v += [a, b, a + (b - a) * rng.uniform() + rng.normal(size=3) * 1e-6]
    for _ in range(40):  # zero area
        a = rng.uniform(-3, 3, 3)
        v += [a, a, a + rng.uniform(-1, 1, 3)]
    for _ in range(200):  # ordinary
        a = rng.uniform(-5, 5, 3)
        v += [a, a + rng.uniform(-1, 1, 3), a + rng.uniform(-1, 1, 3)]
    v = np.array(v, np.float32)
    mesh = E.Mesh(v, np.arange(len(v), dtype=np.uint32))
    st = E.RayTracerSettings(num_samples=1, max_bounces=1, use_environment_lighting=True, mesh_data=[
        E.RayTracingMesh(mesh, E.LambertianMaterial([0.5, 0.5, 0.5])),
        E.RayTracingMesh(E.Mesh(v[::-1].copy(), np.arange(len(v), dtype=np.uint32)),
                         E.LambertianMaterial([0.5, 0.5, 0.5]))])
    return SceneCase(settings=st, camera=E.Camera([0, 0, -10], [0, 0, 1]), size=(8, 8))


CASES = {
    "island": lambda: SceneCase("island", (8, 8), 1, 1),
    "cave": lambda: SceneCase("cave", (8, 8), 1, 1),
    "box": lambda: SceneCase("box", (8, 8), 1, 1),
    "soup": adversarial_soup,
}


@pytest.fixture(scope="module", params=list(CASES))
def built(request):
    case = CASES[request.param]()
    return case, build(case.tris, case.meshes)


def test_every_entry_exactly_once_with_its_scan_key(built):
    case, b = built
    T = case.tris.view(np.float32).reshape(-1, 16)
    entries = scan_entries(case.tris, case.meshes)
    placed = {}
    for rec in list(b["prims"]) + list(b["irregular"]):
        key, m, idx = ubits(rec[3]), ubits(rec[7]), ubits(rec[11])
        assert (key, m, idx) not in placed
        placed[(key, m, idx)] = rec
        np.testing.assert_array_equal(bits(rec[[0, 1, 2, 4, 5, 6, 8, 9, 10, 12, 13, 14]]),
                                      bits(T[idx][[0, 1, 2, 4, 5, 6, 8, 9, 10, 12, 13, 14]]))
    never = [e for e in entries if e not in placed]
    assert len(never) == b["never"]
    for _, _, idx in never:  # only exactly-zero normals are dropped
        assert (T[idx][12:15] == 0).all()
    assert len(placed) + len(never) == len(entries)


def test_tree_structure_boxes_and_cones(built):
    case, b = built
    N = b["nodes"]
    if len(N) == 0:
        return
    Nu = N.view(np.uint32)
    n_nodes, n_prims = len(N), len(b["prims"])
    covered = np.zeros(n_prims, np.int32)

    def verts(rec):
        a = rec[0:3].astype(np.float64)
        return np.stack([a, a + rec[4:7].astype(np.float64), a + rec[8:11].astype(np.float64)])

    def walk(k):  # returns the index after k's subtree
        lo, hi = N[k, 0:3], N[k, 4:7]
        assert (lo <= hi).all()
        assert N[k, 3] >= 0 and N[k, 7] >= 0  # margin coefficients
        info = int(Nu[k, 14])
        count, first = info >> 27, info & 0x07FFFFFF
        axis, cphi, sphi = N[k, 8:11].astype(np.float64), float(N[k, 11]), float(N[k, 12])
        assert abs(cphi * cphi + sphi * sphi - 1) < 1e-5
        if count:
            for p in range(first, first + count):
                covered[p] += 1
                v = verts(b["prims"][p])
                assert (v >= lo - 0).all() and (v <= hi + 0).all(), (k, p)
                n = b["prims"][p][12:15].astype(np.float64)
                if cphi > 0:
                    assert axis @ (n / np.linalg.norm(n)) >= cphi - 1e-6
            end = k + 1
        else:
            left_end = walk(k + 1)
            assert int(Nu[k + 1, 15]) == left_end
            assert first == left_end  # inner node word 14: the right child
            for c in (k + 1, left_end):  # children nest in the parent box
                assert (N[c, 0:3] >= lo).all() and (N[c, 4:7] <= hi).all()
            end = walk(left_end)
        assert int(Nu[k, 15]) == end
        return end

    assert walk(0) == n_nodes
    assert (covered == 1).all()


def dir_cell(d, res):
    """The kernel's dir_cell in binary32 (hrt_kernels.hip)."""
    d = d.astype(np.float32)
    a = np.abs(d)
    fx = (a[:, 0] >= a[:, 1]) & (a[:, 0] >= a[:, 2])
    fy = ~fx & (a[:, 1] >= a[:, 2])
    face = np.where(fx, np.where(d[:, 0] < 0, 1, 0), np.where(fy, np.where(d[:, 1] < 0, 3, 2),
                                                              np.where(d[:, 2] < 0, 5, 4)))
    with np.errstate(divide="ignore", invalid="ignore"):
        u = np.where(fx, d[:, 1] / a[:, 0], np.where(fy, d[:, 2] / a[:, 1], d[:, 0] / a[:, 2])).astype(np.float32)
        v = np.where(fx, d[:, 2] / a[:, 0], np.where(fy, d[:, 0] / a[:, 1], d[:, 1] / a[:, 2])).astype(np.float32)
    s = np.float32(0.5 * res)
    iu = np.clip(((u + np.float32(1)) * s).astype(np.int64), 0, res - 1)
    iv = np.clip(((v + np.float32(1)) * s).astype(np.int64), 0, res - 1)
    return (face * res + iu) * res + iv


def test_band_lists_cover_every_grazing_triangle(built):
    case, b = built
    assert_band_coverage(b)


def assert_band_coverage(b, n_dirs=6000):
    prims = b["prims"]
    if len(prims) == 0:
        return
    n = prims[:, 12:15].astype(np.float64)
    nh = n / np.linalg.norm(n, axis=1, keepdims=True)
    rng = np.random.default_rng(3)
    d = rng.normal(size=(n_dirs, 3))
    # plus directions right at cube-face edges and corners, and exactly in some triangles' planes
    edge = np.array([[1, 1, 0.3], [1, -1, 0.2], [1, 1, 1], [-1, 1, -1], [0.5, 1, 1], [1, 0, 0], [0, 0, -1]], float)
    t = rng.integers(len(nh), size=300)
    inplane = np.cross(nh[t], rng.normal(size=(300, 3)))
    d = np.concatenate([d, edge, inplane])
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    cells = dir_cell(d, b["dir_res"])
    band_idx = b["band"]
    off = b["band_off"]
    lo, hi = -(float(TAU_G) + 1e-5), 2e-5
    for i in range(len(d)):
        dn = nh @ d[i].astype(np.float64)
        need = np.nonzero((dn > lo) & (dn < hi))[0]
        if len(need) == 0:
            continue
        c = cells[i]
        have = set(band_idx[off[c]:off[c + 1]].tolist())
        missing = [k for k in need if k not in have]
        assert not missing, f"direction {d[i]} cell {c}: band prims {missing[:5]} missing"


def test_band_lists_follow_the_scene_content():
    """hrt_bvh.cpp build_bands keeps the last two list sets per process, keyed on the prim records, tau_g
    and the cell count: a scene whose geometry changed (a rotated copy of island) gets its own lists,
    which cover its grazing triangles; the first scene again gets the first lists back."""
    case = SceneCase("island", (8, 8), 1, 1)
    a = build(case.tris, case.meshes, leaf=2)
    c, s_ = np.cos(0.4), np.sin(0.4)
    R = np.array([[c, 0, s_], [0, 1, 0], [-s_, 0, c]], np.float64)
    tris = case.tris.copy()
    for f in ("a", "edge_one", "edge_two", "normal"):
        tris[f][:, :3] = (tris[f][:, :3].astype(np.float64) @ R.T).astype(np.float32)
    b = build(tris, case.meshes, leaf=2)
    assert b["dir_res"] == a["dir_res"] and not np.array_equal(b["band"], a["band"])
    assert_band_coverage(b, n_dirs=1500)
    a2 = build(case.tris, case.meshes, leaf=2)
    assert np.array_equal(a2["band"], a["band"]) and np.array_equal(a2["band_off"], a["band_off"])


def test_release_caches_drops_the_band_lists():
    """hrt_release_caches: the process-wide band-list cache is released on request (its bytes
    reported, nothing the second time), and a later build of the same scene rebuilds the same lists."""
    lib = _lib.load()
    case = SceneCase("island", (8, 8), 1, 1)
    a = build(case.tris, case.meshes, leaf=2)
    freed = ctypes.c_uint64(0)
    assert lib.hrt_release_caches(ctypes.byref(freed)) == 0
    # at least this scene's lists and prim image (cached once per process, whichever test built them)
    assert freed.value >= (a["band"].size + a["band_off"].size) * 4
    assert lib.hrt_release_caches(ctypes.byref(freed)) == 0 and freed.value == 0
    assert lib.hrt_release_caches(None) == 0
    b = build(case.tris, case.meshes, leaf=2)
    assert np.array_equal(a["band"], b["band"]) and np.array_equal(a["band_off"], b["band_off"])


def test_band_entries_are_prim_indices(built):
    """Band entries are prim indices (hrt_bvh.h "Grazing-band entries"): in range, no duplicates in a
    cell's list (the kernels upload them as 16-bit words up to 65536 prims)."""
    case, b = built
    band, off = b["band"], b["band_off"]
    if len(band) == 0:
        return
    assert band.max() < len(b["prims"])
    assert off[-1] == len(band) and np.all(np.diff(off.astype(np.int64)) >= 0)
    for c in np.random.default_rng(5).integers(len(off) - 1, size=200):
        cell = band[off[c]:off[c + 1]]
        assert len(np.unique(cell)) == len(cell)


def test_not_built_above_the_mesh_limit():
    rng = np.random.default_rng(1)
    meshes = [E.RayTracingMesh(E.Mesh(rng.uniform(-1, 1, (3, 3)).astype(np.float32), np.arange(3, dtype=np.uint32)),
                               E.LambertianMaterial([0.5, 0.5, 0.5])) for _ in range(65)]
    st = E.RayTracerSettings(num_samples=1, max_bounces=1, use_environment_lighting=True, mesh_data=meshes)
    case = SceneCase(settings=st, camera=E.Camera([0, 0, -5], [0, 0, 1]), size=(4, 4))
    assert build(case.tris, case.meshes) is None


@pytest.mark.parametrize("leaf", [1, 2, 16])
def test_leaf_sizes(leaf):
    case = SceneCase("box", (8, 8), 1, 1)
    b = build(case.tris, case.meshes, leaf)
    counts = (b["nodes"].view(np.uint32)[:, 14] >> 27)
    assert counts.max() <= leaf and counts.sum() == len(b["prims"])


def wq_image(case, width, leaf=4):
    lib = _lib.load()
    cap = 70000 * 12
    img = np.zeros(cap, np.float32)
    got = lib.hrt_debug_bvh_wq_nodes(case.tris.ctypes.data, len(case.tris), case.meshes.ctypes.data,
                                     len(case.meshes), leaf, width, img.ctypes.data, img.size)
    assert got > 0
    return img[:got * 12].reshape(got, 12)


@pytest.mark.parametrize("scene", ["island", "cave", "box"])
def test_wq_node_image(scene):
    """BUNDLE_WQ's 48 B node image (hrt_bvh.h make_wq_nodes) with 2-member groups (the binary tree)
    against the full preorder nodes: the same boxes and margins in sibling-adjacent order (an inner
    node's children at fc, fc + 1, group word fc | 1 << 16), leaf info copied, escapes that continue a
    stackless walk after each subtree; the binary16 cone only ever widens (cos rounded down, sin^2 x 1.00001 up)
    and the axis is within 2^-12 per component (kernel: 5e-4)."""
    case = SceneCase(scene, (8, 8), 1, 1)
    b = build(case.tris, case.meshes, 4)
    if b is None:
        return
    nn = len(b["nodes"])
    img = wq_image(case, 2)
    assert len(img) == nn
    w = bits(img[:, 8:12])
    N = b["nodes"]
    Nu = N.view(np.uint32)
    # map preorder node -> image node by walking both trees together
    new_of = np.full(nn, -1, np.int64)
    esc_of = np.full(nn, -1, np.int64)
    new_of[0], esc_of[0] = 0, nn
    for k in range(nn):
        info = int(Nu[k, 14])
        if info >> 27:
            continue
        g = int(w[new_of[k], 3])
        assert g >> 16 == 1  # two members
        fc = g & 0xFFFF
        left, right = k + 1, info
        new_of[left], new_of[right] = fc, fc + 1
        esc_of[left], esc_of[right] = fc + 1, esc_of[k]
    assert sorted(new_of.tolist()) == list(range(nn))
    img_o = img[new_of]
    w_o = w[new_of]
    np.testing.assert_array_equal(bits(img_o[:, 0:8]), bits(N[:, 0:8]))
    leaf = (Nu[:, 14] >> 27) > 0
    np.testing.assert_array_equal(w_o[leaf, 3], Nu[leaf, 14])          # leaf info
    np.testing.assert_array_equal(w_o[:, 2] >> 16, esc_of)              # escapes
    half = lambda u: (u & 0xFFFF).astype(np.uint16).view(np.float16).astype(np.float64)
    ax, ay, az = half(w_o[:, 0]), half(w_o[:, 0] >> 16), half(w_o[:, 1])
    cq, sq = half(w_o[:, 1] >> 16), half(w_o[:, 2])
    axis = N[:, 8:11].astype(np.float64)
    assert np.abs(np.stack([ax, ay, az], 1) - axis).max() <= 2.0 ** -12
    assert (cq <= N[:, 11].astype(np.float64)).all() and (cq >= 0).all()
    sin = N[:, 12].astype(np.float64)
    assert (sin >= 0).all() and (sq >= sin * sin * 1.00001).all()  # S >= sin^2 x 1.00001, rounded up
    assert (sq <= sin * sin * 1.00001 * (1 + 2.0 ** -10) + 2.0 ** -24).all()  # and within 1 ulp (subnormals: 2^-24)
    assert np.linalg.norm(np.stack([ax, ay, az], 1) - axis, axis=1).max() <= 5e-4  # |d.(A16 - A)| <= |A16 - A|
    # a stackless walk over the image visits every node once, in preorder of the full tree
    order, cur = [], 0
    while cur != nn:
        order.append(cur)
        info = int(w[cur, 3])
        cur = (info & 0xFFFF) if not (info >> 27) else int(w[cur, 2] >> 16)
    assert order == new_of.tolist()


@pytest.mark.parametrize("width", [3, 4])
@pytest.mark.parametrize("scene", ["island", "cave", "box"])
def test_wq_group_image(scene, width):
    """The grouped image (HRT_OPT_BVH_WIDTH 3, 4): every record is a binary node's record (box, margins,
    cone words), a group of 2..width members sits side by side with each member's box inside its
    parent's, every binary leaf appears exactly once, the collapse keeps the group members in the
    binary tree's left-to-right order, and a stackless walk (escape links) visits every node once,
    depth first."""
    case = SceneCase(scene, (8, 8), 1, 1)
    b = build(case.tris, case.meshes, 4)
    if b is None:
        return
    img = wq_image(case, width)
    ref2 = wq_image(case, 2)
    n = len(img)
    w = bits(img[:, 8:12])
    # records are binary-node records (compare against the 2-wide image, whose rows are all nodes)
    rec = lambda im, k: np.concatenate([bits(im[k, 0:10]), bits(im[k, 10:11]) & 0xFFFF]).tobytes()  # minus escape
    rows2 = {rec(ref2, k) for k in range(len(ref2))}
    for k in range(n):
        assert rec(img, k) in rows2
    leaves = sorted(int(x) for x in w[:, 3] if x >> 27)
    Nu = b["nodes"].view(np.uint32)
    assert leaves == sorted(int(x) for x in Nu[:, 14] if x >> 27)
    widest, seen, stack = 2, {0}, [0]
    while stack:
        k = stack.pop()
        info = int(w[k, 3])
        if info >> 27:
            continue
        fc, cnt = info & 0xFFFF, (info >> 16) + 1
        assert 2 <= cnt <= width and fc + cnt <= n
        widest = max(widest, cnt)
        prims = [int(w[fc + j, 3]) & 0x07FFFFFF for j in range(cnt) if int(w[fc + j, 3]) >> 27]
        assert prims == sorted(prims)  # members in the binary tree's order (leaf prims are leaf-ordered)
        for j in range(cnt):
            c = fc + j
            assert c not in seen
            seen.add(c)
            assert (img[c, 0:3] >= img[k, 0:3]).all() and (img[c, 4:7] <= img[k, 4:7]).all()
            assert (img[c, [3, 7]] <= img[k, [3, 7]]).all()  # margins grow toward the root
            assert int(w[c, 2] >> 16) == (c + 1 if j + 1 < cnt else int(w[k, 2] >> 16) if k else n)
            stack.append(c)
    assert seen == set(range(n))
    if width > 2 and len(b["nodes"]) > 7:
        assert widest == width and n < len(b["nodes"])
    order, cur = [], 0
    while cur != n:
        order.append(cur)
        info = int(w[cur, 3])
        cur = (info & 0xFFFF) if not (info >> 27) else int(w[cur, 2] >> 16)
    assert sorted(order) == list(range(n))
