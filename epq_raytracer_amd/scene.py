"""Scene data model: the Python mirror of src/materials.rs, src/objects.rs and the external
``graphics::Mesh`` / ``load_obj`` / ``Camera`` the reference's scene presets are built from.

All values are binary32 exactly as the Rust f32 code computes them (e.g. ``166.0 / 255.0`` is
divided in f32, src/main.rs:145).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from . import _lib

F32 = np.float32


def _f3(v) -> np.ndarray:
    return np.asarray(v, dtype=np.float32).reshape(3)


# ---- materials (src/materials.rs) ------------------------------------------------------------

def _material(colour4, emission4, settings4) -> np.ndarray:
    m = np.zeros((), dtype=_lib.MATERIAL_DTYPE)
    m["colour"] = np.asarray(colour4, dtype=np.float32)
    m["emission"] = np.asarray(emission4, dtype=np.float32)
    m["settings"] = np.asarray(settings4, dtype=np.float32)
    return m


@dataclass
class CustomMaterial:
    """src/materials.rs:4-34 (Default: colour 0.5, no emission, smoothness/fuzz/spec_prob 0)."""
    colour: Sequence[float] = (0.5, 0.5, 0.5)
    emission_colour: Sequence[float] = (0.0, 0.0, 0.0)
    emission_strength: float = 0.0
    smoothness: float = 0.0
    fuzz: float = 0.0
    specular_probability: float = 0.0

    def into(self) -> np.ndarray:
        c, e = list(self.colour), list(self.emission_colour)
        return _material([c[0], c[1], c[2], 0.0], [e[0], e[1], e[2], self.emission_strength],
                         [self.specular_probability, self.smoothness, self.fuzz, 0.0])


@dataclass
class LambertianMaterial:
    """src/materials.rs:38-50: settings (1, 0, 0, 0)."""
    colour: Sequence[float]

    def into(self) -> np.ndarray:
        c = list(self.colour)
        return _material([c[0], c[1], c[2], 0.0], [0.0] * 4, [1.0, 0.0, 0.0, 0.0])


@dataclass
class MetalMaterial:
    """src/materials.rs:52-66: settings (1, smoothness, fuzz, 0)."""
    colour: Sequence[float]
    smoothness: float
    fuzz: float

    def into(self) -> np.ndarray:
        c = list(self.colour)
        return _material([c[0], c[1], c[2], 0.0], [0.0] * 4, [1.0, self.smoothness, self.fuzz, 0.0])


@dataclass
class LightMaterial:
    """src/materials.rs:68-80: colour 1, settings (1, 1, 0, 0)."""
    emission: Sequence[float]

    def into(self) -> np.ndarray:
        return _material([1.0] * 4, list(self.emission), [1.0, 1.0, 0.0, 0.0])


@dataclass
class InvisLightMaterial:
    """src/materials.rs:82-94: colour 1, settings (0, 1, 0, 1) -- the invisible-light flag."""
    emission: Sequence[float]

    def into(self) -> np.ndarray:
        return _material([1.0] * 4, list(self.emission), [0.0, 1.0, 0.0, 1.0])


def as_material(m) -> np.ndarray:
    if isinstance(m, np.ndarray) and m.dtype == _lib.MATERIAL_DTYPE:
        return m
    return m.into()


# ---- meshes, spheres (src/objects.rs) -------------------------------------------------------

@dataclass
class Mesh:
    """graphics::Mesh reduced to what the path tracer reads: positions and triangle indices."""
    positions: np.ndarray  # (N, 3) float32
    indices: np.ndarray    # (3T,) uint32, 0-based into positions
    name: str = ""

    def __post_init__(self):
        self.positions = np.ascontiguousarray(self.positions, dtype=np.float32).reshape(-1, 3)
        self.indices = np.ascontiguousarray(self.indices, dtype=np.uint32).reshape(-1)
        if self.indices.size % 3:
            raise ValueError("mesh index count must be a multiple of 3")


def subdivide(mesh: Mesh, k: int) -> Mesh:
    """Split every triangle (a, b, c) into k*k triangles on the same plane, same winding (a scaling
    workload: the same surface with k*k times the triangles; not a reference feature)."""
    if k <= 1:
        return mesh
    tri = mesh.positions[mesh.indices.reshape(-1, 3)].astype(np.float64)  # (T, 3, 3)
    a, ab, ac = tri[:, 0], tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0]
    grid = [(i, j) for i in range(k + 1) for j in range(k + 1 - i)]
    gid = {g: n for n, g in enumerate(grid)}
    pts = np.stack([a + ab * (i / k) + ac * (j / k) for i, j in grid], 1)  # (T, G, 3)
    local = []
    for i in range(k):
        for j in range(k - i):
            local.append((gid[(i, j)], gid[(i + 1, j)], gid[(i, j + 1)]))
            if i + j + 1 < k:
                local.append((gid[(i + 1, j)], gid[(i + 1, j + 1)], gid[(i, j + 1)]))
    local = np.array(local, np.uint32)
    base = (np.arange(len(tri), dtype=np.uint32) * len(grid))[:, None, None]
    return Mesh(pts.reshape(-1, 3).astype(np.float32), (base + local[None]).reshape(-1), mesh.name)


@dataclass
class Sphere:
    """src/objects.rs:8-22."""
    centre: Sequence[float]
    radius: float
    material: object

    def record(self) -> np.ndarray:
        r = np.zeros((), dtype=_lib.SPHERE_DTYPE)
        r["centre"] = _f3(self.centre)
        r["radius"] = F32(self.radius)
        r["material"] = as_material(self.material)
        return r


@dataclass
class RayTracingMesh:
    """src/objects.rs:35-38."""
    mesh: Mesh
    material: object


def get_null_sphere() -> Sphere:
    """src/objects.rs:24-30 (uploaded when the sphere list is empty; its count stays 0)."""
    return Sphere([0.0, 0.0, 0.0], 0.0, LambertianMaterial([1.0, 1.0, 1.0]))


def get_null_mesh() -> RayTracingMesh:
    """src/objects.rs:40-47."""
    return RayTracingMesh(Mesh(np.zeros((1, 3), np.float32), np.zeros(3, np.uint32)), LambertianMaterial([1.0] * 3))


# ---- camera (graphics::Camera, external) -----------------------------------------------------

@dataclass
class Camera:
    """The fields of graphics::Camera the path reads (src/raytrace_pipeline.rs:244,273-274).
    Assumptions: default up = (0,1,0); the direction is stored as given.
    ``do_move`` is a no-op (the reference camera is not made controllable, src/main.rs:27)."""
    position: Sequence[float] = (0.0, 0.0, 0.0)
    direction: Sequence[float] = (1.0, 0.0, 0.0)
    up: Sequence[float] = (0.0, 1.0, 0.0)

    def do_move(self, frame_time: float) -> None:  # src/raytracing_app.rs:169
        return None


# ---- OBJ loading (graphics::load_obj semantics, via the native reader) -------------------------

ASSET_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets")


def load_obj(path: str) -> List[Mesh]:
    """One Mesh per ``o`` record in file order, face winding preserved (native hrt_obj_load)."""
    lib = _lib.load()
    h = ctypes.c_void_p()
    _lib.check(lib.hrt_obj_load(path.encode(), ctypes.byref(h)), f"hrt_obj_load({path})")
    try:
        meshes = []
        for i in range(lib.hrt_obj_num_meshes(h)):
            name = ctypes.c_char_p()
            pos = ctypes.c_void_p()
            nv = ctypes.c_uint32()
            idx = ctypes.c_void_p()
            ni = ctypes.c_uint32()
            _lib.check(lib.hrt_obj_mesh(h, i, ctypes.byref(name), ctypes.byref(pos), ctypes.byref(nv),
                                        ctypes.byref(idx), ctypes.byref(ni)), "hrt_obj_mesh")
            P = np.ctypeslib.as_array((ctypes.c_float * (3 * nv.value)).from_address(pos.value)).reshape(-1, 3).copy()
            I = (np.ctypeslib.as_array((ctypes.c_uint32 * ni.value).from_address(idx.value)).copy()
                 if ni.value else np.zeros(0, np.uint32))
            meshes.append(Mesh(P, I, (name.value or b"").decode()))
        return meshes
    finally:
        lib.hrt_obj_free(h)


def save_mesh_asset(meshes: List[Mesh], path: str) -> None:
    """Store meshes as a compact .npz (positions shared per mesh, indices, names)."""
    arrays = {"names": np.array([m.name for m in meshes])}
    for i, m in enumerate(meshes):
        used = np.unique(m.indices)
        remap = np.zeros(max(int(m.positions.shape[0]), 1), np.uint32)
        remap[used] = np.arange(used.size, dtype=np.uint32)
        arrays[f"pos{i}"] = m.positions[used]
        arrays[f"idx{i}"] = remap[m.indices]
    np.savez_compressed(path, **arrays)


def load_asset(name: str) -> List[Mesh]:
    """Bundled scene geometry: ``<name>.npz`` in epq_raytracer_amd/assets (made by tools/import_assets.py
    from the reference's OBJ files with load_obj semantics), else ``<name>.obj`` by path."""
    npz = os.path.join(ASSET_DIR, f"{name}.npz")
    if os.path.exists(npz):
        with np.load(npz, allow_pickle=False) as z:
            names = [str(s) for s in z["names"]]
            return [Mesh(z[f"pos{i}"], z[f"idx{i}"], names[i]) for i in range(len(names))]
    if os.path.exists(name):
        return load_obj(name)
    raise FileNotFoundError(f"no bundled asset {name!r} in {ASSET_DIR}")
