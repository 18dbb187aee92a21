"""Host side of the path: the Python mirror of RayTracePipeline (src/raytrace_pipeline.rs) and
DiffusePipeline (src/diffuse.rs) on top of the C ABI.  Host prep arithmetic (ray centres, view
matrix, mesh flattening) runs in the native library (hrt_host_*), the dispatches on the GPU.

Mapping to the reference:
  RayTracerSettings        src/raytracing_app.rs:17-29
  RayTracePipeline.__init__ src/raytrace_pipeline.rs:51-97   (-> hrt_create + hrt_set_scene)
  RayTracePipeline.compute  src/raytrace_pipeline.rs:162-187 (-> hrt_trace, init = 0)
  RayTracePipeline.init     src/raytrace_pipeline.rs:190-213 (-> hrt_trace, init = 1)
  RayTracePipeline.push_constants  dispatch :216-266 (124-byte block :243-257)
  DiffusePipeline.next_frame       src/diffuse.rs:73-101 (-> hrt_accumulate)
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from .scene import Camera, RayTracingMesh, Sphere, as_material, get_null_mesh, get_null_sphere


@dataclass
class RayTracerSettings:
    """src/raytracing_app.rs:17-29."""
    num_samples: int
    max_bounces: int
    use_environment_lighting: bool
    sample_jitter: Optional[float] = None
    sphere_data: List[Sphere] = field(default_factory=list)
    mesh_data: List[RayTracingMesh] = field(default_factory=list)
    camera_focal_length: float = 1.0
    viewport_height: float = 2.0
    up: Sequence[float] = (0.0, 1.0, 0.0)


# ---- host prep (native) ---------------------------------------------------------------------

def create_rays(image_size, camera_focal_length, viewport_height, up):
    """create_ray_subbuffer, src/raytrace_pipeline.rs:289-338 -> (rays[W*H], num_rays, default_jitter)."""
    lib = _lib.load()
    w, h = int(image_size[0]), int(image_size[1])
    rays = np.zeros(max(w * h, 1), dtype=_lib.RAY_DTYPE)
    jit = ctypes.c_float()
    n = lib.hrt_host_create_rays(w, h, float(np.float32(camera_focal_length)), float(np.float32(viewport_height)),
                                 _lib.f3(up), _lib.ptr(rays), ctypes.byref(jit))
    return rays, int(n), float(jit.value)


def view_matrix(direction, up) -> np.ndarray:
    """get_view_matrix, src/raytrace_pipeline.rs:269-285 -> column-major mat4 as float32[16]."""
    lib = _lib.load()
    out = (ctypes.c_float * 16)()
    lib.hrt_host_view_matrix(_lib.f3(direction), _lib.f3(up), out)
    return np.frombuffer(out, dtype=np.float32).copy()


def transform_meshes(meshes: List[RayTracingMesh]):
    """transform_meshes, src/raytrace_pipeline.rs:377-428 -> (triangles, mesh records)."""
    lib = _lib.load()
    n = len(meshes)
    pos = [np.ascontiguousarray(m.mesh.positions, np.float32) for m in meshes]
    idx = [np.ascontiguousarray(m.mesh.indices, np.uint32) for m in meshes]
    mats = np.array([as_material(m.material) for m in meshes], dtype=_lib.MATERIAL_DTYPE)
    ntri = sum(int(i.size) // 3 for i in idx)
    tris = np.zeros(max(ntri, 1), dtype=_lib.TRIANGLE_DTYPE)
    recs = np.zeros(max(n, 1), dtype=_lib.MESH_DTYPE)
    pos_ptrs = (ctypes.c_void_p * n)(*[p.ctypes.data for p in pos])
    idx_ptrs = (ctypes.c_void_p * n)(*[i.ctypes.data if i.size else 0 for i in idx])
    nv = (ctypes.c_uint32 * n)(*[p.shape[0] for p in pos])
    ni = (ctypes.c_uint32 * n)(*[i.size for i in idx])
    st = lib.hrt_host_transform_meshes(n, pos_ptrs, nv, idx_ptrs, ni, _lib.ptr(mats), _lib.ptr(tris), ntri,
                                       _lib.ptr(recs))
    _lib.check(st, "hrt_host_transform_meshes")
    return tris[:ntri], recs[:n]


def sphere_records(spheres: List[Sphere]) -> np.ndarray:
    """create_sphere_subbuffer, src/raytrace_pipeline.rs:342-360."""
    if not spheres:
        return np.zeros(0, dtype=_lib.SPHERE_DTYPE)
    return np.array([s.record() for s in spheres], dtype=_lib.SPHERE_DTYPE)


# ---- the device context (one hrt_context = the trace image + the accumulated image) ------------

class HrtContext:
    """Owner of one hrt_context.  ``partition`` = (row_tile, part_index, part_count) selects the
    interleaved row tiles this context renders (multi-GPU).  ``debug=True`` binds
    libhip_raytrace_debug.so (diagnostics-only options)."""

    def __init__(self, image_size, device: int = -1, mode: int = _lib.MODE_RGBA8, partition=None,
                 debug: bool = False):
        self.lib = _lib.load(debug)
        info = _lib.CreateInfo()
        info.width, info.height = int(image_size[0]), int(image_size[1])
        info.device = int(device)
        info.mode = int(mode)
        if partition is not None:
            info.row_tile, info.part_index, info.part_count = (int(v) for v in partition)
        else:
            info.row_tile, info.part_index, info.part_count = 0, 0, 1
        h = ctypes.c_void_p()
        _lib.check(self.lib.hrt_create(ctypes.byref(info), ctypes.byref(h)), "hrt_create", None, self.lib)
        self.handle = h
        lay = _lib.Layout()
        _lib.check(self.lib.hrt_get_layout(self.handle, ctypes.byref(lay)), "hrt_get_layout", self.handle, self.lib)
        self.width, self.height = lay.width, lay.height
        self.local_rows, self.row_tile = lay.local_rows, lay.row_tile
        self.part_index, self.part_count, self.mode = lay.part_index, lay.part_count, lay.mode

    def close(self):
        if getattr(self, "handle", None):
            self.lib.hrt_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, st, where):
        _lib.check(st, where, self.handle, self.lib)

    def set_scene(self, rays, spheres, tris, meshes):
        """rays=None keeps the context's rays (hrt_generate_rays or an earlier set_scene)."""
        n_rays = 0 if rays is None else len(rays)
        self._check(self.lib.hrt_set_scene(self.handle, None if rays is None else _lib.ptr(rays), n_rays,
                                           _lib.ptr(spheres), len(spheres), _lib.ptr(tris), len(tris),
                                           _lib.ptr(meshes), len(meshes)),
                    "hrt_set_scene")

    def generate_rays(self, camera_focal_length: float, viewport_height: float, up) -> float:
        """Ray centres on the device (hrt_generate_rays); returns the default jitter."""
        u = (ctypes.c_float * 3)(*[float(np.float32(v)) for v in up])
        jit = ctypes.c_float()
        self._check(self.lib.hrt_generate_rays(self.handle, float(np.float32(camera_focal_length)),
                                               float(np.float32(viewport_height)), u, ctypes.byref(jit)),
                    "hrt_generate_rays")
        return jit.value

    def import_external(self, fd: int, size: int, offset: int, nbytes: int) -> int:
        """hrt_import_external_memory: device pointer (int) to [offset, offset + nbytes) of the fd."""
        ptr = ctypes.c_void_p()
        self._check(self.lib.hrt_import_external_memory(self.handle, int(fd), int(size), int(offset), int(nbytes),
                                                        ctypes.byref(ptr)), "hrt_import_external_memory")
        return int(ptr.value)

    def release_external(self, dev_ptr: int):
        self._check(self.lib.hrt_release_external_memory(self.handle, ctypes.c_void_p(dev_ptr)),
                    "hrt_release_external_memory")

    def read_rays(self) -> np.ndarray:
        out = np.empty(self.width * self.height, dtype=_lib.RAY_DTYPE)
        self._check(self.lib.hrt_read_rays(self.handle, _lib.ptr(out), len(out)), "hrt_read_rays")
        return out

    def trace(self, pc: _lib.PushConstants):
        self._check(self.lib.hrt_trace(self.handle, ctypes.byref(pc)), "hrt_trace")

    def accumulate(self, frame: int):
        self._check(self.lib.hrt_accumulate(self.handle, int(frame) & 0xFFFFFFFF), "hrt_accumulate")

    def compute_n(self, pc: _lib.PushConstants, n: int):
        """hrt_compute_n: n x (trace with rng_offset = pc.rng_offset + k, accumulate(that k))."""
        self._check(self.lib.hrt_compute_n(self.handle, ctypes.byref(pc), int(n)), "hrt_compute_n")

    def synchronize(self):
        self._check(self.lib.hrt_synchronize(self.handle), "hrt_synchronize")

    def set_option(self, key: int, value: int):
        self._check(self.lib.hrt_set_option(self.handle, key, value), "hrt_set_option")

    def stats(self) -> _lib.Stats:
        s = _lib.Stats()
        self._check(self.lib.hrt_get_stats(self.handle, ctypes.byref(s)), "hrt_get_stats")
        return s

    def diagnostics(self) -> dict:
        """Cull diagnostics (needs set_option(OPT_COUNTERS, 2) before the traces)."""
        out = np.zeros(len(_lib.DIAG_NAMES), np.uint64)
        self._check(self.lib.hrt_get_diagnostics(self.handle, _lib.ptr(out), len(out)), "hrt_get_diagnostics")
        return dict(zip(_lib.DIAG_NAMES, (int(v) for v in out)))

    def tile_profile(self) -> np.ndarray:
        """Per 8x8 tile of the last trace, (ceil(local_rows/8), ceil(W/8), 4): shader clocks, bounce
        iterations, bounce survivor tests, bounce clocks (needs OPT_COUNTERS=2)."""
        ty, tx = (self.local_rows + 7) // 8, (self.width + 7) // 8
        out = np.zeros(ty * tx * 4, np.uint64)
        self._check(self.lib.hrt_get_tile_profile(self.handle, _lib.ptr(out), len(out)), "hrt_get_tile_profile")
        return out.reshape(ty, tx, 4)

    def scene_info(self) -> dict:
        """What the last set_scene built for the BVH kernel (hrt_get_scene_info)."""
        out = np.zeros(len(_lib.SCENE_INFO_NAMES), np.uint32)
        self._check(self.lib.hrt_get_scene_info(self.handle, _lib.ptr(out), len(out)), "hrt_get_scene_info")
        return dict(zip(_lib.SCENE_INFO_NAMES, (int(v) for v in out)))

    def reset_stats(self):
        self._check(self.lib.hrt_reset_stats(self.handle), "hrt_reset_stats")

    def read(self, image_id: int, fmt: int = _lib.FMT_RGBA8) -> np.ndarray:
        """Local rows of an image: uint8 (local_rows, W, 4) or float32 (local_rows, W, 4) -- this
        context's own rows even when it is joined to a communicator (HRT_IMG_LOCAL: never the
        collective gather; read_frame is the gathered frame)."""
        dt = np.uint8 if fmt == _lib.FMT_RGBA8 else np.float32
        out = np.empty((self.local_rows, self.width, 4), dtype=dt)
        self._check(self.lib.hrt_read_image(self.handle, image_id | _lib.IMG_LOCAL, fmt, _lib.ptr(out), out.nbytes),
                    "hrt_read_image")
        return out

    def load_accumulator(self, img: np.ndarray):
        """Checkpoint / resume: restore the accumulated image from an earlier read(IMG_ACCUM) in the
        context's own format (hrt_load_accumulator)."""
        fmt = _lib.FMT_RGBA8 if self.mode == _lib.MODE_RGBA8 else _lib.FMT_RGBA32F
        img = np.ascontiguousarray(img)
        self._check(self.lib.hrt_load_accumulator(self.handle, fmt, _lib.ptr(img), img.nbytes), "hrt_load_accumulator")

    def read_into(self, image_id: int, fmt: int, dst_ptr: int, nbytes: int):
        """Copy into caller memory (host or device pointer, e.g. a torch tensor's data_ptr())."""
        self._check(self.lib.hrt_read_image(self.handle, image_id, fmt, ctypes.c_void_p(dst_ptr), nbytes),
                    "hrt_read_image")

    def check_guards(self):
        """libhip_raytrace_debug.so: (guarded device buffers, buffers whose guard bands were overwritten)."""
        n, bad = ctypes.c_uint32(), ctypes.c_uint32()
        self._check(self.lib.hrt_debug_check_guards(self.handle, ctypes.byref(n), ctypes.byref(bad)),
                    "hrt_debug_check_guards")
        return n.value, bad.value

    # ---- multi-GPU framebuffer gather (hrt_comm_*) ----

    @staticmethod
    def comm_unique_id() -> bytes:
        """A fresh RCCL unique id (rank 0 creates it and shares the bytes, e.g. by torch.distributed)."""
        lib = _lib.load()
        buf = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)()
        _lib.check(lib.hrt_comm_unique_id(buf), "hrt_comm_unique_id", None, lib)
        return bytes(buf)

    def comm_init(self, uid: bytes, rank: int, world: int):
        """Join the RCCL communicator of a world-way partition (collective over the ranks)."""
        buf = (ctypes.c_uint8 * _lib.COMM_ID_BYTES).from_buffer_copy(uid)
        self._check(self.lib.hrt_comm_init(self.handle, buf, int(rank), int(world)), "hrt_comm_init")

    @staticmethod
    def comm_init_all(ctxs):
        """One process driving every part: ctxs[i] is part i of len(ctxs)."""
        lib = ctxs[0].lib
        arr = (ctypes.c_void_p * len(ctxs))(*[c.handle.value for c in ctxs])
        _lib.check(lib.hrt_comm_init_all(arr, len(ctxs)), "hrt_comm_init_all", None, lib)

    def comm_info(self):
        """(rank, world, transport) of the context's communicator."""
        r, w, t = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        self._check(self.lib.hrt_comm_info(self.handle, ctypes.byref(r), ctypes.byref(w), ctypes.byref(t)),
                    "hrt_comm_info")
        return r.value, w.value, t.value

    def read_frame(self, image_id: int, fmt: int = _lib.FMT_RGBA8, root: bool = True):
        """The gathered full frame (height, W, 4) through hrt_read_image on a context with a
        communicator; ranks other than the root pass root=False and get None."""
        if not root:
            self._check(self.lib.hrt_read_image(self.handle, image_id, fmt, None, 0), "hrt_read_image")
            return None
        dt = np.uint8 if fmt == _lib.FMT_RGBA8 else np.float32
        out = np.empty((self.height, self.width, 4), dtype=dt)
        self._check(self.lib.hrt_read_image(self.handle, image_id, fmt, _lib.ptr(out), out.nbytes), "hrt_read_image")
        return out

    def global_rows(self) -> np.ndarray:
        """Global row index of each local row (rows >= height are padding)."""
        lr = np.arange(self.local_rows, dtype=np.int64)
        if self.part_count <= 1:
            return lr
        t = lr // self.row_tile
        return (t * self.part_count + self.part_index) * self.row_tile + lr % self.row_tile


class Image:
    """What RayTracePipeline::image / DiffusePipeline::image hand to the presenter."""

    def __init__(self, ctx: HrtContext, image_id: int):
        self.ctx, self.image_id = ctx, image_id

    def read(self, fmt: int = _lib.FMT_RGBA8) -> Optional[np.ndarray]:
        """What the presenter gets.  Without a communicator: the context's rows.  On a context joined to
        one (hrt_comm_init): the gathered FULL frame -- a collective every rank must call; ranks other
        than 0 get None.  On a group (hrt_comm_init_all): the full frame."""
        rank, _, transport = self.ctx.comm_info()
        if transport == _lib.COMM_NONE:
            return self.ctx.read(self.image_id, fmt)
        return self.ctx.read_frame(self.image_id, fmt, root=transport != _lib.COMM_RCCL or rank == 0)


# ---- pipelines ---------------------------------------------------------------------------------

class RayTracePipeline:
    """src/raytrace_pipeline.rs:31-266 on the HIP context."""

    def __init__(self, ctx: HrtContext, image_size, settings: RayTracerSettings):
        self.ctx = ctx
        self.image_size = (int(image_size[0]), int(image_size[1]))
        rays, num_rays, jitter = create_rays(self.image_size, settings.camera_focal_length, settings.viewport_height,
                                             settings.up)
        spheres = sphere_records(settings.sphere_data)
        tris, meshes = transform_meshes(settings.mesh_data if settings.mesh_data else [get_null_mesh()])
        n_meshes = len(settings.mesh_data)
        self.ray_count = num_rays
        self.sphere_count = len(settings.sphere_data)
        self.mesh_count = n_meshes
        self.num_samples = max(int(settings.num_samples), 1)       # :88
        self.max_bounces = max(int(settings.max_bounces), 0)       # :89
        self.use_environment_lighting = bool(settings.use_environment_lighting)
        self.sample_jitter = float(np.float32(settings.sample_jitter if settings.sample_jitter is not None else jitter))
        self.rays, self.tris, self.meshes, self.spheres = rays[:num_rays], tris, meshes[:n_meshes], spheres
        ctx.set_scene(rays[:num_rays], spheres, tris, meshes[:n_meshes])

    def image(self) -> Image:
        return Image(self.ctx, _lib.IMG_TRACE)

    def push_constants(self, camera: Camera, rng_offset: int, init: bool) -> _lib.PushConstants:
        """The 124-byte block of dispatch(), src/raytrace_pipeline.rs:243-257."""
        pc = _lib.PushConstants()
        pos = np.asarray(camera.position, np.float32)
        pc.cam_pos[:] = [float(pos[0]), float(pos[1]), float(pos[2]), 1.0]
        pc.cam_alignment_mat[:] = [float(v) for v in view_matrix(camera.direction, camera.up)]
        pc.num_rays = self.ray_count
        pc.num_spheres = self.sphere_count
        pc.num_meshes = self.mesh_count
        pc.num_samples = self.num_samples
        pc.jitter_size = self.sample_jitter
        pc.max_bounces = self.max_bounces
        pc.use_environment_light = int(self.use_environment_lighting)
        pc.rng_offset = int(rng_offset) & 0xFFFFFFFF
        pc.init = int(bool(init))
        pc.width, pc.height = self.image_size
        return pc

    def compute(self, camera: Camera, rng_offset: int) -> None:
        self.ctx.trace(self.push_constants(camera, rng_offset, False))

    def init(self) -> None:
        self.ctx.trace(self.push_constants(Camera(), 0, True))


class DiffusePipeline:
    """src/diffuse.rs:22-136: the progressive accumulator (image_combiner.glsl)."""

    def __init__(self, ctx: HrtContext, image_size):
        self.ctx = ctx
        self.image_size = (int(image_size[0]), int(image_size[1]))

    def image(self) -> Image:
        return Image(self.ctx, _lib.IMG_ACCUM)

    def next_frame(self, frame_num: int, next_image: Image) -> None:
        if next_image.ctx is not self.ctx or next_image.image_id != _lib.IMG_TRACE:
            raise ValueError("next_image must be the trace image of the same context")
        self.ctx.accumulate(frame_num)
