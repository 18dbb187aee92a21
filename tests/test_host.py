"""Host-side prep (CPU): the product's native host helpers (hrt_host_*, C++) against the oracle's
independent C restatement of src/raytrace_pipeline.rs:269-428, byte for byte; the OBJ reader
against an independent Python parser; the presets' constants against Rust f32 literal rounding."""
import os
from fractions import Fraction

import numpy as np
import pytest

import pyoracle as O
import epq_raytracer_amd as E
from epq_raytracer_amd import _lib

REF_ASSETS = "/root/reference/assets"
CAMERAS = [(name, *E.PRESETS[name]()) for name in E.PRESETS]


@pytest.mark.parametrize("size", [(1, 1), (2, 3), (64, 64), (1920, 1080), (37, 23), (1080, 720)])
@pytest.mark.parametrize("up", [(0.0, 1.0, 0.0), (0.1, 0.9, 0.2)])
def test_create_rays_matches_oracle(size, up):
    rays, n, jit = E.create_rays(size, 1.0, 2.0, up)
    ref, n2, jit2 = O.create_rays(size[0], size[1], 1.0, 2.0, up)
    assert n == n2 == size[0] * size[1]
    assert np.float32(jit) == np.float32(jit2)
    np.testing.assert_array_equal(rays["sample_centre"][:n].view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("size", [(1, 1), (37, 23), (1920, 1080)])
@pytest.mark.parametrize("up", [(0.0, 1.0, 0.0), (0.1, 0.9, 0.2)])
def test_ray_grid_reproduces_create_rays(size, up):
    """hrt_host_ray_grid's (first, px, py): (first + px*x) + py*y in binary32, each operation rounded
    as written (what the device's make_rays evaluates), gives create_rays' records bit for bit."""
    import ctypes
    lib = _lib.load()
    f3 = lambda v=(0.0, 0.0, 0.0): (ctypes.c_float * 3)(*v)
    first, px, py, upc, jit = f3(), f3(), f3(), f3(up), ctypes.c_float()
    n = lib.hrt_host_ray_grid(size[0], size[1], 1.0, 2.0, upc, first, px, py, ctypes.byref(jit))
    rays, n2, jit2 = E.create_rays(size, 1.0, 2.0, up)
    assert n == n2 and np.float32(jit.value) == np.float32(jit2)
    f, a, b = (np.array(list(v), np.float32) for v in (first, px, py))
    xs = np.arange(size[0], dtype=np.float32)[None, :, None]
    ys = np.arange(size[1], dtype=np.float32)[:, None, None]
    grid = (f + a * xs) + b * ys  # numpy float32: each op correctly rounded, no contraction
    np.testing.assert_array_equal(grid.reshape(-1, 3).view(np.uint32),
                                  rays["sample_centre"][:n, :3].view(np.uint32))


def test_create_rays_geometry():
    # up=(0,1,0): viewport_x = (0,0,-1), viewport_y = (0,-1,0): row 0 is the top
    rays, n, jit = E.create_rays((4, 2), 1.0, 2.0, (0, 1, 0))
    c = rays["sample_centre"][:n].reshape(2, 4, 4)
    assert np.all(c[..., 0] == 1.0)                      # focal plane x = 1
    assert c[0, 0, 1] > 0 > c[1, 0, 1]                   # y decreases down the image
    assert c[0, 0, 2] > 0 > c[0, 3, 2]                   # z decreases left to right
    assert jit == pytest.approx(0.5 * 4.0 / 4, rel=1e-6)  # max(|px|, |py|) / 2 with vw = 4


def test_zero_size_rays():
    rays, n, jit = E.create_rays((0, 5), 1.0, 2.0, (0, 1, 0))
    assert n == 0 and jit == 0.0


@pytest.mark.parametrize("name,cam,settings", CAMERAS)
def test_view_matrix_matches_oracle(name, cam, settings):
    m = E.view_matrix(cam.direction, cam.up)
    r = O.view_matrix(cam.direction, cam.up)
    np.testing.assert_array_equal(m.view(np.uint32), r.view(np.uint32))
    # mat3(M) * (1,0,0) is the normalised view direction
    d = np.asarray(cam.direction, np.float64)
    np.testing.assert_allclose(m[:3], d / np.linalg.norm(d), rtol=1e-6)


def test_view_matrix_random():
    rng = np.random.default_rng(7)
    for _ in range(200):
        d = rng.normal(size=3).astype(np.float32)
        m, r = E.view_matrix(d, (0, 1, 0)), O.view_matrix(d, (0, 1, 0))
        np.testing.assert_array_equal(m.view(np.uint32), r.view(np.uint32))


@pytest.mark.parametrize("name", ["Cube", "box", "island", "Cave"])
def test_transform_meshes_matches_oracle(name):
    meshes = E.load_asset(name)
    rt = [E.RayTracingMesh(m, E.LambertianMaterial([0.5, 0.25, 0.125])) for m in meshes]
    tris, recs = E.transform_meshes(rt)
    mats = [E.LambertianMaterial([0.5, 0.25, 0.125]).into() for _ in meshes]
    rtris, rrecs = O.transform_meshes([(m.positions, m.indices, mat) for m, mat in zip(meshes, mats)],
                                      _lib.TRIANGLE_DTYPE, _lib.MESH_DTYPE, _lib.MATERIAL_DTYPE)
    assert tris.tobytes() == rtris.tobytes()
    assert recs.tobytes() == rrecs.tobytes()
    assert int(recs["len"].sum()) == len(tris)
    assert list(recs["first_index"]) == list(np.cumsum([0] + list(recs["len"][:-1])))


def test_transform_meshes_rejects_bad_index():
    m = E.Mesh(np.zeros((3, 3), np.float32), np.array([0, 1, 3], np.uint32))
    with pytest.raises(_lib.HrtError):
        E.transform_meshes([E.RayTracingMesh(m, E.LambertianMaterial([1, 1, 1]))])


def test_null_mesh_record():
    # src/objects.rs:40-47: one degenerate triangle at the origin, uploaded with count 0
    tris, recs = E.transform_meshes([E.get_null_mesh()])
    assert len(tris) == 1 and recs[0]["len"] == 1
    assert np.all(tris[0]["normal"][:3] == 0)


def _parse_obj_py(path):
    """Independent restatement of load_obj semantics for the test (one mesh per `o`)."""
    V, objs = [], []
    for line in open(path):
        t = line.split()
        if not t:
            continue
        if t[0] == "v":
            V.append([np.float32(x) for x in t[1:4]])
        elif t[0] == "o":
            objs.append((" ".join(t[1:]), []))
        elif t[0] == "f":
            if not objs:
                objs.append(("", []))
            ids = [int(s.split("/")[0]) for s in t[1:]]
            ids = [i - 1 if i > 0 else len(V) + i for i in ids]
            for k in range(1, len(ids) - 1):
                objs[-1][1].extend([ids[0], ids[k], ids[k + 1]])
    V = np.array(V, np.float32)
    return [(n, V[np.array(f, np.int64)].reshape(-1, 3, 3)) for n, f in objs]


@pytest.mark.skipif(not os.path.isdir(REF_ASSETS), reason="reference checkout not mounted")
@pytest.mark.parametrize("name", ["Cube", "box", "island", "Cave"])
def test_obj_loader_and_bundled_asset(name):
    path = os.path.join(REF_ASSETS, f"{name}.obj")
    native = E.load_obj(path)
    py = _parse_obj_py(path)
    bundled = E.load_asset(name)
    assert [m.name for m in native] == [n for n, _ in py] == [m.name for m in bundled]
    for m, (_, tri), b in zip(native, py, bundled):
        got = m.positions[m.indices].reshape(-1, 3, 3)
        np.testing.assert_array_equal(got, tri)
        np.testing.assert_array_equal(b.positions[b.indices].reshape(-1, 3, 3), tri)


def test_obj_loader_polygons_negative_indices_and_errors(tmp_path):
    p = tmp_path / "t.obj"
    p.write_text("v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nf 1 2 3 4\no second\nv 0 0 1\nf -1 -4 -3\n")
    ms = E.load_obj(str(p))
    assert [m.name for m in ms] == ["", "second"]
    assert list(ms[0].indices) == [0, 1, 2, 0, 2, 3]   # fan triangulation keeps winding
    assert list(ms[1].indices) == [4, 1, 2]
    bad = tmp_path / "bad.obj"
    bad.write_text("v 0 0 0\nf 1 2 3\n")
    with pytest.raises(_lib.HrtError):
        E.load_obj(str(bad))
    with pytest.raises(_lib.HrtError):
        E.load_obj(str(tmp_path / "missing.obj"))


def test_obj_loader_long_lines(tmp_path):
    """lines longer than any fixed buffer (a 3,000-gon face, a 6,000-character object name)
    are read whole, not split into a parsed head and a silently dropped tail."""
    n = 3000
    ang = np.linspace(0, 2 * np.pi, n, endpoint=False)
    name = "o" * 6000
    lines = [f"o {name}"] + [f"v {np.cos(a):.6f} {np.sin(a):.6f} 0.25" for a in ang]
    lines.append("f " + " ".join(f"{i}/{i}/{i}" for i in range(1, n + 1)))
    p = tmp_path / "long.obj"
    p.write_text("\n".join(lines) + "\n")
    assert max(len(line) for line in lines) > 16384
    ms = E.load_obj(str(p))
    assert len(ms) == 1 and ms[0].name == name
    assert len(ms[0].indices) == 3 * (n - 2)
    assert list(ms[0].indices[-3:]) == [0, n - 2, n - 1]


def _rust_f32(s: str) -> np.float32:
    """Correctly rounded decimal -> binary32 (what rustc does for an f32 literal)."""
    q = Fraction(s)
    f = np.float32(float(q))
    cands = [np.nextafter(f, np.float32(-np.inf)), f, np.nextafter(f, np.float32(np.inf))]
    return min(cands, key=lambda c: (abs(Fraction(float(c)) - q), int(np.float32(c).view(np.uint32)) & 1))


LITERALS = ["0.5", "100.0", "2.5", "0.75", "0.2", "1.0", "0.1", "0.6", "25.0", "500.0", "250.0", "-0.35", "0.87",
            "0.7", "0.005", "5.0", "1.5", "-0.2", "0.40", "0.26", "0.16", "0.46", "0.14", "0.18", "0.21", "0.63", "0.82",
            "-5.0", "10.0", "-20.0", "-0.4", "2.0", "-100.0", "-2.5", "-1.0", "3.0", "0.55", "0.35", "0.45", "0.42",
            "0.95", "0.05"]


@pytest.mark.parametrize("lit", LITERALS)
def test_python_float_literals_round_like_rust(lit):
    assert np.float32(float(lit)) == _rust_f32(lit)


def test_box_wall_colours_are_f32_divisions():
    cam, st = E.load_box_scene()
    c = st.mesh_data[1].material.into()["colour"]
    assert c[0] == np.float32(166.0) / np.float32(255.0)


def test_presets_build_records():
    for name in E.PRESETS:
        cam, st = E.PRESETS[name]()
        tris, recs = E.transform_meshes(st.mesh_data if st.mesh_data else [E.get_null_mesh()])
        assert len(recs) == max(len(st.mesh_data), 1)
    cam, st = E.load_island_scene()
    assert [len(m.mesh.indices) // 3 for m in st.mesh_data] == [80, 992, 180, 358]
    cam, st = E.load_box_scene()
    assert st.mesh_data[-1].material.into()["settings"][3] == 1.0   # invisible light flag


def test_subdivide_preserves_surface_and_winding():
    """scene.subdivide (the triangle-count scaling workload): k*k triangles per input triangle,
    same total area, every piece's normal parallel to (and oriented like) its parent's."""
    import epq_raytracer_amd as E
    rng = np.random.default_rng(2)
    v = rng.uniform(-3, 3, (12, 3)).astype(np.float32)
    m = E.Mesh(v, np.arange(12, dtype=np.uint32))
    for k in (1, 2, 3, 5):
        s = E.subdivide(m, k)
        assert len(s.indices) == 3 * 4 * k * k
        p = s.positions[s.indices.reshape(-1, 3)].astype(np.float64)
        q = m.positions[m.indices.reshape(-1, 3)].astype(np.float64)
        ns = np.cross(p[:, 1] - p[:, 0], p[:, 2] - p[:, 0]).reshape(4, k * k, 3)
        nq = np.cross(q[:, 1] - q[:, 0], q[:, 2] - q[:, 0])
        np.testing.assert_allclose(np.linalg.norm(ns, axis=-1).sum(1), np.linalg.norm(nq, axis=-1), rtol=1e-4)
        cos = np.einsum("tkc,tc->tk", ns, nq) / (np.linalg.norm(ns, axis=-1) * np.linalg.norm(nq, axis=-1)[:, None])
        assert (cos > 0.9999).all()
