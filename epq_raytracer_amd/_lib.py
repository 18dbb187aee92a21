"""ctypes binding of libhip_raytrace.so (include/hip_raytrace.h, include/hrt_host.h).

The library is built in-tree by ``__graft_entry__.build()`` / ``make -C epq_raytracer_amd/csrc``.
There is no fallback: if the shared object is missing or a call fails, this module raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_float, c_int32, c_int64, c_size_t, c_uint32, c_uint64, c_void_p

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libhip_raytrace.so")
DEBUG_LIB_PATH = os.path.join(_HERE, "lib", "libhip_raytrace_debug.so")  # -DHRT_DEBUG_OPTIONS (tests, tools)

# ---- std430 records (assets/raytracing.glsl:51-153) as numpy dtypes + ctypes structs ----------

MATERIAL_DTYPE = np.dtype([("colour", "<f4", 4), ("emission", "<f4", 4), ("settings", "<f4", 4)])
RAY_DTYPE = np.dtype([("sample_centre", "<f4", 4)])
SPHERE_DTYPE = np.dtype([("centre", "<f4", 3), ("radius", "<f4"), ("material", MATERIAL_DTYPE)])
TRIANGLE_DTYPE = np.dtype([("a", "<f4", 4), ("edge_one", "<f4", 4), ("edge_two", "<f4", 4), ("normal", "<f4", 4)])
MESH_DTYPE = np.dtype([("min_point", "<f4", 3), ("first_index", "<u4"), ("max_point", "<f4", 3), ("len", "<u4"),
                       ("material", MATERIAL_DTYPE)])
assert MATERIAL_DTYPE.itemsize == 48 and RAY_DTYPE.itemsize == 16 and SPHERE_DTYPE.itemsize == 64
assert TRIANGLE_DTYPE.itemsize == 64 and MESH_DTYPE.itemsize == 80


class PushConstants(ctypes.Structure):
    """raytrace_shader::PushConstants (assets/raytracing.glsl:135-153), 124 bytes."""

    _fields_ = [
        ("cam_pos", c_float * 4),
        ("cam_alignment_mat", c_float * 16),
        ("num_rays", c_int32),
        ("num_spheres", c_int32),
        ("num_meshes", c_int32),
        ("num_samples", c_int32),
        ("jitter_size", c_float),
        ("max_bounces", c_int32),
        ("use_environment_light", c_uint32),
        ("rng_offset", c_uint32),
        ("init", c_uint32),
        ("width", c_uint32),
        ("height", c_uint32),
    ]


assert ctypes.sizeof(PushConstants) == 124


class CreateInfo(ctypes.Structure):
    _fields_ = [("width", c_uint32), ("height", c_uint32), ("device", c_int32), ("mode", c_uint32),
                ("row_tile", c_uint32), ("part_index", c_uint32), ("part_count", c_uint32)]


class Layout(ctypes.Structure):
    _fields_ = [("width", c_uint32), ("height", c_uint32), ("local_rows", c_uint32), ("row_tile", c_uint32),
                ("part_index", c_uint32), ("part_count", c_uint32), ("mode", c_uint32)]


class Stats(ctypes.Structure):
    _fields_ = [("segments", c_uint64), ("tri_tests", c_uint64), ("traces", c_uint64), ("accumulates", c_uint64),
                ("last_trace_ms", c_float), ("total_trace_ms", c_float), ("wave_steps", c_uint64),
                ("last_kernel", c_uint32), ("last_block", c_uint32), ("last_frames", c_uint32),
                ("reserved", c_uint32)]


ABI_VERSION = 6  # HRT_ABI_VERSION this binding's signatures describe
HRT_OK = 0
STATUS_NAMES = {0: "HRT_OK", 1: "HRT_ERR_INVALID_ARGUMENT", 2: "HRT_ERR_NO_DEVICE", 3: "HRT_ERR_OUT_OF_MEMORY",
                4: "HRT_ERR_NO_SCENE", 5: "HRT_ERR_HIP", 6: "HRT_ERR_IO", 7: "HRT_ERR_COMM"}
ERR_COMM = 7
MODE_RGBA8, MODE_RGBA32F = 0, 1
IMG_TRACE, IMG_ACCUM = 0, 1
IMG_LOCAL = 0x100  # flag: this context's local rows, never the collective gather
FMT_RGBA8, FMT_RGBA32F = 0, 1
OPT_KERNEL_VARIANT, OPT_COUNTERS, OPT_SECONDARY_BATCH, OPT_BVH_LEAF_SIZE = 1, 2, 3, 4
OPT_SPLIT, OPT_SPLIT_FACTOR, OPT_PRIORITY, OPT_GRID_CUS, OPT_COOP, OPT_WQ_NODE_CAP, OPT_PROBE = 5, 6, 7, 8, 9, 10, 11
OPT_FRAMES_PER_LAUNCH, OPT_OVERLAP, OPT_BUSY_SPLIT, OPT_BVH_WIDTH, OPT_WQ_NODE_RADIUS = 12, 13, 14, 15, 16
OPT_COMM_TIMEOUT_MS, OPT_DEFER_COMBINE = 17, 18
DEBUG_OPT_FAIL_ALLOC = 1001  # libhip_raytrace_debug.so only
DEBUG_OPT_WQ_TRI_CAP = 1002  # libhip_raytrace_debug.so only
DEBUG_OPT_GRAB_RUNS = 1003  # libhip_raytrace_debug.so only
DEBUG_OPT_TIMELINE = 1004  # builds with -DHRT_TIMELINE=1 only (tools/timeline.py)
DEBUG_OPT_STACK_LIMIT = 1005  # libhip_raytrace_debug.so only
COMM_ID_BYTES = 128
COMM_NONE, COMM_RCCL, COMM_RCCL_GROUP, COMM_DEVICE_COPY = 0, 1, 2, 3
# hrt_kernel (include/hip_raytrace.h)
KERNEL_AUTO, KERNEL_LITERAL, KERNEL_BRUTE, KERNEL_BRUTE_LDS, KERNEL_BUNDLE, KERNEL_BUNDLE_CULL = 0, 1, 2, 3, 4, 5
KERNEL_BUNDLE_BVH, KERNEL_BUNDLE_CULL_LDS, KERNEL_BUNDLE_BVH_LDS, KERNEL_BUNDLE_WQ = 6, 7, 8, 9
# kernel symbol (as rocprofv3 names it) of a resolved hrt_kernel + workgroup size
NODE_RADIUS_MARGIN_MILLI = 100  # auto HRT_OPT_WQ_NODE_RADIUS: per-node R above this bvh_margin_milli (hrt_bvh.h)


def wq_node_radius(scene_info: dict, option: int = 0) -> bool:
    """Whether BUNDLE_WQ runs its per-node-radius kernel (trace_bundle_wq_nr) for this scene."""
    return option == 2 or (option == 0 and scene_info.get("bvh_margin_milli", 0) > NODE_RADIUS_MARGIN_MILLI)


def kernel_symbol(kernel: int, block: int, diag: bool = False, node_r: bool = False) -> str:
    d = "true" if diag else "false"
    if kernel == 9 and node_r:
        return f"void hrt::trace_bundle_wq_nr<{d}>(hrt::TraceParams)"
    if kernel in (1, 2, 3):
        return "hrt::" + {1: "trace_literal", 2: "trace_brute", 3: "trace_brute_lds"}[kernel] + "(hrt::TraceParams)"
    if kernel == 7:
        return f"void hrt::trace_bundle_cull_lds<{block}, {d}>(hrt::TraceParams)"
    name = {4: "trace_bundle", 5: "trace_bundle_cull", 6: "trace_bundle_bvh", 8: "trace_bundle_bvh_lds",
            9: "trace_bundle_wq"}.get(kernel, "?")
    return f"void hrt::{name}<{d}>(hrt::TraceParams)"


KERNEL_NAMES = {0: "auto", 1: "literal", 2: "brute", 3: "brute_lds", 4: "bundle", 5: "bundle_cull", 6: "bundle_bvh",
                7: "bundle_cull_lds", 8: "bundle_bvh_lds", 9: "bundle_wq"}
DIAG_NAMES = ("primary_iters", "primary_considered", "primary_survivors", "bounce_iters", "bounce_considered",
              "bounce_survivors", "bounce_lanes", "bvh_visits", "bvh_prim_tests", "bvh_band_tests", "primary_cycles", "bounce_cycles",
              "shade_cycles", "bounce_stage2", "bounce_front", "bvh_trips",
              "bvh_leaf_trips", "band_scan_max", "band_scan_len", "sky_items", "sky_cycles",
              "primary_lanes", "loop_iters", "live_lanes", "wq_steps_16", "wq_steps_32", "wq_steps_48",
              "wq_steps_64", "wq_members")
SCENE_INFO_NAMES = ("bvh_nodes", "bvh_prims", "bvh_irregular", "bvh_never", "bvh_built", "bvh_band_entries",
                    "bvh_sah_milli", "bvh_margin_milli")

# Every symbol include/*.h declares (tests/test_abi.py checks the export table against this).
EXPORTED_SYMBOLS = (
    "hrt_abi_version", "hrt_build_id", "hrt_debug_build", "hrt_debug_check_guards", "hrt_create", "hrt_destroy", "hrt_set_scene", "hrt_trace", "hrt_accumulate", "hrt_compute_n",
    "hrt_read_image", "hrt_load_accumulator", "hrt_get_layout", "hrt_synchronize", "hrt_get_stats", "hrt_reset_stats", "hrt_set_option",
    "hrt_get_diagnostics", "hrt_get_tile_profile", "hrt_get_scene_info", "hrt_generate_rays", "hrt_read_rays",
    "hrt_import_external_memory", "hrt_release_external_memory", "hrt_debug_export_memory", "hrt_debug_unmap_memory", "hrt_debug_math_check", "hrt_debug_math_check_rng", "hrt_debug_band_flatten", "hrt_debug_wq_protocol",
    "hrt_debug_timeline", "hrt_debug_band_records", "hrt_debug_tile_costs",
    "hrt_stream", "hrt_release_caches", "hrt_last_error", "hrt_comm_unique_id", "hrt_comm_init", "hrt_comm_init_all", "hrt_comm_info",
    "hrt_host_create_rays", "hrt_host_ray_grid", "hrt_host_view_matrix", "hrt_host_transform_meshes",
    "hrt_debug_bvh_build", "hrt_debug_bvh_wq_nodes",
    "hrt_obj_load", "hrt_obj_num_meshes", "hrt_obj_mesh", "hrt_obj_free",
)


class HrtError(RuntimeError):
    """A non-OK hrt_status (the reference would have panicked in .unwrap())."""

    def __init__(self, status: int, where: str, detail: str = ""):
        self.status = status
        super().__init__(f"{where} failed: {STATUS_NAMES.get(status, status)}{': ' + detail if detail else ''}")


_libs = {}


def load(debug: bool = False) -> ctypes.CDLL:
    """Load libhip_raytrace.so, or with debug=True libhip_raytrace_debug.so (the same objects with the
    diagnostics-only options compiled in).  Raises if the library has not been built."""
    if debug in _libs:
        return _libs[debug]
    # HRT_LIB: A/B builds of the same ABI (tools/kbench.py experiments)
    path = DEBUG_LIB_PATH if debug else os.environ.get("HRT_LIB", LIB_PATH)
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                           " or `make -C epq_raytracer_amd/csrc` (no CPU fallback exists)")
    lib = ctypes.CDLL(path)
    lib.hrt_abi_version.restype = c_uint32
    lib.hrt_abi_version.argtypes = []
    if lib.hrt_abi_version() != ABI_VERSION:  # the signatures below would bind shifted arguments
        raise RuntimeError(f"{path} implements HRT_ABI_VERSION {lib.hrt_abi_version()}, this binding "
                           f"{ABI_VERSION}: rebuild it (make -C epq_raytracer_amd/csrc)")
    P = c_void_p
    sig = {
        "hrt_abi_version": (c_uint32, []),
        "hrt_debug_build": (c_uint32, []),
        "hrt_build_id": (c_char_p, []),
        "hrt_debug_check_guards": (c_int32, [P, POINTER(c_uint32), POINTER(c_uint32)]),
        "hrt_comm_unique_id": (c_int32, [P]),
        "hrt_comm_init": (c_int32, [P, P, c_uint32, c_uint32]),
        "hrt_comm_init_all": (c_int32, [P, c_uint32]),
        "hrt_comm_info": (c_int32, [P, POINTER(c_uint32), POINTER(c_uint32), POINTER(c_uint32)]),
        "hrt_create": (c_int32, [POINTER(CreateInfo), POINTER(c_void_p)]),
        "hrt_destroy": (None, [P]),
        "hrt_set_scene": (c_int32, [P, P, c_uint32, P, c_uint32, P, c_uint32, P, c_uint32]),
        "hrt_trace": (c_int32, [P, POINTER(PushConstants)]),
        "hrt_accumulate": (c_int32, [P, c_uint32]),
        "hrt_compute_n": (c_int32, [P, POINTER(PushConstants), c_uint32]),
        "hrt_read_image": (c_int32, [P, c_uint32, c_uint32, P, c_size_t]),
        "hrt_load_accumulator": (c_int32, [P, c_uint32, P, c_size_t]),
        "hrt_get_layout": (c_int32, [P, POINTER(Layout)]),
        "hrt_synchronize": (c_int32, [P]),
        "hrt_get_stats": (c_int32, [P, POINTER(Stats)]),
        "hrt_reset_stats": (c_int32, [P]),
        "hrt_get_diagnostics": (c_int32, [P, P, c_uint32]),
        "hrt_get_scene_info": (c_int32, [P, P, c_uint32]),
        "hrt_get_tile_profile": (c_int32, [P, P, c_uint32]),
        "hrt_generate_rays": (c_int32, [P, c_float, c_float, POINTER(c_float), POINTER(c_float)]),
        "hrt_read_rays": (c_int32, [P, P, c_uint32]),
        "hrt_import_external_memory": (c_int32, [P, c_int32, c_uint64, c_uint64, c_uint64, POINTER(c_void_p)]),
        "hrt_release_external_memory": (c_int32, [P, P]),
        "hrt_debug_export_memory": (c_int32, [c_int32, c_uint64, POINTER(c_int32), POINTER(c_void_p),
                                              POINTER(c_uint64)]),
        "hrt_debug_unmap_memory": (c_int32, [P, c_uint64]),
        "hrt_debug_math_check": (c_int32, [c_int32, c_uint32, c_uint32, P]),
        "hrt_debug_math_check_rng": (c_int32, [c_int32, P]),
        "hrt_debug_band_flatten": (c_int32, [c_int32, P, P, c_uint32, P, P]),
        "hrt_debug_wq_protocol": (c_int32, [c_int32, c_uint32, P, P, P, P, P, P, P, P, P]),
        "hrt_debug_timeline": (c_int32, [c_void_p, P, c_uint32, P]),
        "hrt_debug_band_records": (c_int32, [c_void_p, P, c_uint64, P, c_uint64, P, c_uint64, P]),
        "hrt_debug_tile_costs": (c_int32, [c_void_p, P, c_uint32]),
        "hrt_debug_bvh_build": (c_int32, [P, c_uint32, P, c_uint32, c_uint32, P, P, c_uint64, P, c_uint64, P,
                                          c_uint64, P, c_uint64, P, c_uint64]),
        "hrt_debug_bvh_wq_nodes": (c_int64, [P, c_uint32, P, c_uint32, c_uint32, c_uint32, P, c_uint64]),
        "hrt_host_ray_grid": (c_uint32, [c_uint32, c_uint32, c_float, c_float, POINTER(c_float), POINTER(c_float),
                                         POINTER(c_float), POINTER(c_float), POINTER(c_float)]),
        "hrt_set_option": (c_int32, [P, c_uint32, c_int64]),
        "hrt_stream": (c_void_p, [P]),
        "hrt_last_error": (c_char_p, [P]),
        "hrt_release_caches": (c_int32, [P]),
        "hrt_host_create_rays": (c_uint32, [c_uint32, c_uint32, c_float, c_float, POINTER(c_float), P,
                                            POINTER(c_float)]),
        "hrt_host_view_matrix": (None, [POINTER(c_float), POINTER(c_float), POINTER(c_float)]),
        "hrt_host_transform_meshes": (c_int32, [c_uint32, P, P, P, P, P, P, c_uint32, P]),
        "hrt_obj_load": (c_int32, [c_char_p, POINTER(c_void_p)]),
        "hrt_obj_num_meshes": (c_uint32, [P]),
        "hrt_obj_mesh": (c_int32, [P, c_uint32, POINTER(c_char_p), POINTER(c_void_p), POINTER(c_uint32),
                                   POINTER(c_void_p), POINTER(c_uint32)]),
        "hrt_obj_free": (None, [P]),
    }
    for name, (res, args) in sig.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            if path == LIB_PATH or path == DEBUG_LIB_PATH:
                raise  # the in-tree build must export the whole ABI (tests/test_abi.py)
            continue   # an older A/B build (HRT_LIB): calls of the missing entry point fail loudly
        fn.restype = res
        fn.argtypes = args
    _libs[debug] = lib
    return lib


def build_id() -> str:
    """hrt_build_id(): hash of the kernel sources + flags the loaded library was built from."""
    return load().hrt_build_id().decode()


def check(status: int, where: str, ctx=None, lib=None) -> None:
    if status != HRT_OK:
        detail = (lib or load()).hrt_last_error(ctx)
        raise HrtError(status, where, detail.decode() if detail else "")


def ptr(a: np.ndarray | None) -> c_void_p:
    if a is None or a.size == 0:
        return c_void_p(0)
    assert a.flags["C_CONTIGUOUS"]
    return c_void_p(a.ctypes.data)


def f3(v) -> ctypes.Array:
    return (c_float * 3)(*[float(np.float32(x)) for x in v])
