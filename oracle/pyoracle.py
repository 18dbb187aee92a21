"""ctypes front-end of the CPU oracle (oracle/rt_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg -- never by the product.  Parity status: "parity unpinned" against the GLSL reference (which
cannot run here); pinned by the RNG known-answer vectors and analytic KATs.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_float, c_int, c_uint8, c_uint32, c_uint64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "build")


def _cpu_has_fma() -> bool:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("flags"):
                    return " fma " in f" {line.split(':', 1)[1].strip()} "
    except OSError:
        pass
    return False


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None
_variants = {}

# Parity-risk variants (rt_oracle.c header): driver-typical numerics, never the checker.
DRIVER_VARIANTS = ("math", "rsq", "contract", "all")


def load_driver_variant(name: str) -> ctypes.CDLL:
    """liborc_drv_<name>.so: the oracle with one driver-typical numerics choice (needs FMA hardware)."""
    if name not in DRIVER_VARIANTS:
        raise ValueError(name)
    if name not in _variants:
        path = os.path.join(BUILD, f"liborc_drv_{name}.so")
        if not os.path.exists(path):
            build()
        _variants[name] = _bind(ctypes.CDLL(path))
    return _variants[name]


def load(prefer_fma: bool | None = None) -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if prefer_fma is None and os.environ.get("ORC_VARIANT") in ("fma", "generic"):
        prefer_fma = os.environ["ORC_VARIANT"] == "fma"
    fma = _cpu_has_fma() if prefer_fma is None else prefer_fma
    path = os.path.join(BUILD, "liborc_fma.so" if fma else "liborc.so")
    path = os.environ.get("ORC_LIB", path)  # the sanitizer build (tests/test_sanitizers.py)
    if not os.path.exists(path):
        build()
    _lib = _bind(ctypes.CDLL(path))
    return _lib


def _bind(lib: ctypes.CDLL) -> ctypes.CDLL:
    P = c_void_p
    lib.orc_hash_step.restype = c_uint32
    lib.orc_hash_step.argtypes = [POINTER(c_uint32)]
    lib.orc_scale01.restype = c_float
    lib.orc_scale01.argtypes = [c_uint32]
    lib.orc_normal_dist.restype = c_float
    lib.orc_normal_dist.argtypes = [POINTER(c_uint32)]
    lib.orc_point_on_sphere.restype = None
    lib.orc_point_on_sphere.argtypes = [POINTER(c_uint32), P]
    for fn in ("spec_logf", "spec_sinf", "spec_cosf"):
        getattr(lib, fn).restype = c_float
        getattr(lib, fn).argtypes = [c_float]
    lib.orc_intersecting_aabb.restype = c_int
    lib.orc_intersecting_aabb.argtypes = [P, P, P, P]
    lib.orc_intersecting_tri.restype = None
    lib.orc_intersecting_tri.argtypes = [P, P, P, P]
    lib.orc_trace_rows.restype = None
    lib.orc_trace_rows.argtypes = [P, P, P, P, P, c_uint32, c_uint32, P, P, POINTER(c_uint64), POINTER(c_uint64),
                                   c_int]
    lib.orc_trace_pixel.restype = None
    lib.orc_trace_pixel.argtypes = [P, P, P, P, P, c_uint32, c_uint32, P, POINTER(c_uint64), POINTER(c_uint64)]
    lib.orc_accumulate_rgba8.restype = None
    lib.orc_accumulate_rgba8.argtypes = [c_uint32, P, P, ctypes.c_size_t]
    lib.orc_accumulate_rgba32f.restype = None
    lib.orc_accumulate_rgba32f.argtypes = [c_uint32, P, P, ctypes.c_size_t]
    lib.orc_unorm8.restype = c_uint8
    lib.orc_unorm8.argtypes = [c_float]
    lib.orc_view_matrix.restype = None
    lib.orc_view_matrix.argtypes = [P, P, P]
    lib.orc_create_rays.restype = c_uint32
    lib.orc_create_rays.argtypes = [c_uint32, c_uint32, c_float, c_float, P, P, POINTER(c_float)]
    lib.orc_transform_mesh.restype = None
    lib.orc_transform_mesh.argtypes = [P, P, c_uint32, P, P, P]
    lib.orc_trace_pixels.restype = None
    lib.orc_trace_pixels.argtypes = [P, P, P, P, P, P, c_uint32, P, POINTER(c_uint64), POINTER(c_uint64), c_int]
    lib.orc_num_threads.restype = c_int
    return lib


def _p(a):
    if a is None or a.size == 0:
        return c_void_p(0)
    assert a.flags["C_CONTIGUOUS"]
    return c_void_p(a.ctypes.data)


def _f32(v, n):
    return np.ascontiguousarray(np.asarray(v, dtype=np.float32).reshape(n))


# ---- RNG / numerics KAT helpers ----------------------------------------------------------------

def hash_sequence(seed: int, n: int):
    lib = load()
    s = c_uint32(seed)
    return [lib.orc_hash_step(ctypes.byref(s)) for _ in range(n)]


def scale01(u: int) -> float:
    return load().orc_scale01(u)


def normal_dist(seed: int):
    s = c_uint32(seed)
    v = load().orc_normal_dist(ctypes.byref(s))
    return v, s.value


def point_on_sphere(seed: int):
    s = c_uint32(seed)
    out = np.zeros(3, np.float32)
    load().orc_point_on_sphere(ctypes.byref(s), _p(out))
    return out, s.value


def spec_log(x):
    return load().spec_logf(x)


def spec_sin(x):
    return load().spec_sinf(x)


def spec_cos(x):
    return load().spec_cosf(x)


def unorm8(x: float) -> int:
    return load().orc_unorm8(x)


def intersecting_aabb(mn, mx, o, d) -> bool:
    keep = [_f32(v, 3) for v in (mn, mx, o, d)]  # arrays must outlive the call
    return bool(load().orc_intersecting_aabb(*[_p(a) for a in keep]))


def intersecting_tri(tri_record: np.ndarray, o, d) -> np.ndarray:
    out = np.zeros(4, np.float32)
    t = np.ascontiguousarray(tri_record).view(np.uint8)
    oo, dd = _f32(o, 3), _f32(d, 3)
    load().orc_intersecting_tri(_p(t), _p(oo), _p(dd), _p(out))
    return out


# ---- host prep ------------------------------------------------------------------------------

def view_matrix(direction, up) -> np.ndarray:
    out = np.zeros(16, np.float32)
    d, u = _f32(direction, 3), _f32(up, 3)
    load().orc_view_matrix(_p(d), _p(u), _p(out))
    return out


def create_rays(w: int, h: int, focal: float, vh: float, up):
    out = np.zeros((max(w * h, 1), 4), np.float32)
    jit = c_float()
    u = _f32(up, 3)
    n = load().orc_create_rays(w, h, focal, vh, _p(u), _p(out), ctypes.byref(jit))
    return out[:n], n, jit.value


def transform_meshes(meshes, tri_dtype, mesh_dtype, material_dtype):
    """meshes: list of (positions (N,3) f32, indices (3T,) u32, material record)."""
    lib = load()
    ntri = sum(len(m[1]) // 3 for m in meshes)
    tris = np.zeros(max(ntri, 1), dtype=tri_dtype)
    recs = np.zeros(len(meshes), dtype=mesh_dtype)
    first = 0
    for k, (pos, idx, mat) in enumerate(meshes):
        pos = np.ascontiguousarray(pos, np.float32)
        idx = np.ascontiguousarray(idx, np.uint32)
        n = len(idx) // 3
        mn = np.zeros(3, np.float32)
        mx = np.zeros(3, np.float32)
        sub = np.zeros(max(n, 1), dtype=tri_dtype)
        sub_b = sub.view(np.uint8)
        lib.orc_transform_mesh(_p(pos), _p(idx), len(idx), _p(sub_b), _p(mn), _p(mx))
        tris[first:first + n] = sub[:n]
        recs[k]["min_point"] = mn
        recs[k]["max_point"] = mx
        recs[k]["first_index"] = first
        recs[k]["len"] = n
        recs[k]["material"] = mat
        first += n
    return tris[:ntri], recs


# ---- trace / accumulate ------------------------------------------------------------------------

def trace(pc, rays, spheres, tris, meshes, rows=None, nthreads: int = 0, want_f32: bool = False, lib=None):
    """Trace the full frame (or global rows [y0, y1)).  pc: a 124-byte ctypes PushConstants.
    Returns (rgba8 (H, W, 4) uint8, rgba32f or None, segments, tri_tests); rows outside the range
    are left zero.  lib: a load_driver_variant() library instead of the pinned oracle."""
    lib = lib or load()
    W, H = pc.width, pc.height
    y0, y1 = (0, H) if rows is None else rows
    img8 = np.zeros((H, W, 4), np.uint8)
    img32 = np.zeros((H, W, 4), np.float32) if want_f32 else None
    seg, tt = c_uint64(), c_uint64()
    keep = [np.ascontiguousarray(rays).view(np.uint8), _bytes(spheres), _bytes(tris), _bytes(meshes)]
    lib.orc_trace_rows(ctypes.byref(pc), *[_p(a) for a in keep], y0, y1, _p(img8), _p(img32), ctypes.byref(seg),
                       ctypes.byref(tt), int(nthreads))
    return img8, img32, seg.value, tt.value


def trace_pixels(pc, rays, spheres, tris, meshes, xs, ys, nthreads: int = 0):
    """rgba8 (n, 4) of the listed pixels of one frame, plus the exact segment / triangle-test counts."""
    xy = np.ascontiguousarray(np.stack([np.asarray(xs, np.uint32), np.asarray(ys, np.uint32)], -1).reshape(-1))
    n = len(xy) // 2
    out = np.zeros((n, 4), np.uint8)
    seg, tt = c_uint64(), c_uint64()
    keep = [np.ascontiguousarray(rays).view(np.uint8), _bytes(spheres), _bytes(tris), _bytes(meshes)]
    load().orc_trace_pixels(ctypes.byref(pc), *[_p(a) for a in keep], _p(xy), n, _p(out), ctypes.byref(seg),
                            ctypes.byref(tt), int(nthreads))
    return out, seg.value, tt.value


def trace_pixel(pc, rays, spheres, tris, meshes, x: int, y: int):
    out = np.zeros(3, np.float32)
    seg, tt = c_uint64(), c_uint64()
    keep = [np.ascontiguousarray(rays).view(np.uint8), _bytes(spheres), _bytes(tris), _bytes(meshes)]
    load().orc_trace_pixel(ctypes.byref(pc), *[_p(a) for a in keep], x, y, _p(out), ctypes.byref(seg),
                           ctypes.byref(tt))
    return out, seg.value, tt.value


def accumulate_rgba8(frame: int, current: np.ndarray, new_image: np.ndarray) -> None:
    assert current.dtype == np.uint8 and new_image.dtype == np.uint8 and current.shape == new_image.shape
    nw = np.ascontiguousarray(new_image)
    load().orc_accumulate_rgba8(frame, _p(current), _p(nw), current.size // 4)


def accumulate_rgba32f(frame: int, current: np.ndarray, new_image: np.ndarray) -> None:
    assert current.dtype == np.float32 and current.shape == new_image.shape
    nw = np.ascontiguousarray(new_image)
    load().orc_accumulate_rgba32f(frame, _p(current), _p(nw), current.size // 4)


def num_threads() -> int:
    return load().orc_num_threads()


def _bytes(a):
    if a is None:
        return None
    a = np.ascontiguousarray(a)
    return a.view(np.uint8) if a.size else a
