"""The C ABI (CPU): libhip_raytrace.so loads, exports exactly what include/*.h declares, the record
layouts are the std430 ones, and calls fail loudly (status + message) instead of falling back."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from epq_raytracer_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_functions():
    names = set()
    for h in ("hip_raytrace.h", "hrt_host.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(hrt_[a-z0-9_]+)\s*\(", src))
    return names


def test_every_declared_symbol_is_exported():
    declared = _declared_functions()
    assert declared == set(_lib.EXPORTED_SYMBOLS)
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    exported = {line.split()[-1] for line in out.stdout.splitlines() if " T " in line}
    missing = declared - exported
    assert not missing, missing


def test_library_loads_and_reports_abi():
    lib = _lib.load()
    assert lib.hrt_abi_version() == _lib.ABI_VERSION == 6
    assert lib.hrt_debug_build() == 0
    assert len(_lib.build_id()) == 16 and _lib.build_id() != "unknown"


def test_debug_library_is_the_same_abi():
    """libhip_raytrace_debug.so: the same exports, hrt_debug_build() == 1, the same device code."""
    dbg = _lib.load(debug=True)
    assert dbg.hrt_debug_build() == 1 and dbg.hrt_abi_version() == _lib.ABI_VERSION
    assert dbg.hrt_build_id().decode() == _lib.build_id()
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.DEBUG_LIB_PATH], capture_output=True, text=True,
                         check=True)
    exported = {line.split()[-1] for line in out.stdout.splitlines() if " T " in line}
    assert _declared_functions() <= exported


def test_rccl_is_not_a_load_time_dependency():
    """RCCL is dlopen'ed by the first hrt_comm_* call (single-GPU users never load it)."""
    out = subprocess.run(["readelf", "-d", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    assert "rccl" not in out.stdout


def test_code_object_targets_gfx950():
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in blob  # the fat binary carries a gfx950 code object
    for k in (b"trace_literal", b"trace_brute", b"trace_brute_lds", b"trace_bundle", b"trace_bundle_cull", b"trace_bundle_bvh", b"trace_bundle_cull_lds", b"trace_bundle_bvh_lds", b"camera_lists",
              b"trace_bundle_wq", b"trace_bundle_wq_nr"):
        assert k in blob, k


def test_node_radius_kernel_symbol():
    """bench.py names the kernel its PMC record must match: BUNDLE_WQ runs trace_bundle_wq_nr when the
    scene's margins are wide (HRT_SCENE_BVH_MARGIN_MILLI > 100) or HRT_OPT_WQ_NODE_RADIUS = 2."""
    assert not _lib.wq_node_radius({"bvh_margin_milli": 26})
    assert _lib.wq_node_radius({"bvh_margin_milli": 197})
    assert _lib.wq_node_radius({"bvh_margin_milli": 26}, option=2)
    assert not _lib.wq_node_radius({"bvh_margin_milli": 197}, option=1)
    assert _lib.kernel_symbol(9, 1024) == "void hrt::trace_bundle_wq<false>(hrt::TraceParams)"
    assert _lib.kernel_symbol(9, 1024, node_r=True) == "void hrt::trace_bundle_wq_nr<false>(hrt::TraceParams)"
    assert _lib.kernel_symbol(7, 512, node_r=True) == "void hrt::trace_bundle_cull_lds<512, false>(hrt::TraceParams)"
    assert "bvh_margin_milli" in _lib.SCENE_INFO_NAMES


def test_record_layouts_match_std430():
    assert _lib.MATERIAL_DTYPE.itemsize == 48
    assert _lib.SPHERE_DTYPE.fields["material"][1] == 16
    assert _lib.MESH_DTYPE.fields["first_index"][1] == 12
    assert _lib.MESH_DTYPE.fields["len"][1] == 28
    assert _lib.MESH_DTYPE.fields["material"][1] == 32
    assert ctypes.sizeof(_lib.PushConstants) == 124
    assert _lib.PushConstants.num_rays.offset == 80
    assert _lib.PushConstants.jitter_size.offset == 96
    assert _lib.PushConstants.use_environment_light.offset == 104
    assert _lib.PushConstants.height.offset == 120
    # the host structs (include/hip_raytrace.h static_asserts the same; INTEGRATION.md's Rust binding is
    # pinned to the header by tests/test_rust_binding.py)
    assert ctypes.sizeof(_lib.Stats) == 64
    assert _lib.Stats.last_frames.offset == 56 and _lib.Stats.wave_steps.offset == 40
    assert ctypes.sizeof(_lib.CreateInfo) == 28 and ctypes.sizeof(_lib.Layout) == 28


def test_create_fails_loudly():
    lib = _lib.load()
    info = _lib.CreateInfo(0, 0, -1, 0, 0, 0, 1)
    h = ctypes.c_void_p()
    st = lib.hrt_create(ctypes.byref(info), ctypes.byref(h))
    assert st == 1 and not h.value  # zero size -> HRT_ERR_INVALID_ARGUMENT, no context
    assert b"zero image size" in lib.hrt_last_error(None)
    info = _lib.CreateInfo(8, 8, -1, 7, 0, 0, 1)
    assert lib.hrt_create(ctypes.byref(info), ctypes.byref(h)) == 1  # unknown mode
    info = _lib.CreateInfo(8, 8, -1, 0, 0, 0, 2)
    assert lib.hrt_create(ctypes.byref(info), ctypes.byref(h)) == 1  # partition without row_tile


def test_no_cpu_fallback_without_device():
    lib = _lib.load()
    info = _lib.CreateInfo(8, 8, -1, 0, 0, 0, 1)
    h = ctypes.c_void_p()
    st = lib.hrt_create(ctypes.byref(info), ctypes.byref(h))
    if st == 0:
        lib.hrt_destroy(h)
        pytest.skip("a GPU is visible here")
    assert st == 2, _lib.STATUS_NAMES.get(st)  # HRT_ERR_NO_DEVICE: there is no CPU path
    with pytest.raises(_lib.HrtError):
        import epq_raytracer_amd as E
        E.HrtContext((8, 8))


def test_null_handles_are_rejected():
    lib = _lib.load()
    pc = _lib.PushConstants()
    assert lib.hrt_trace(None, ctypes.byref(pc)) == 1
    assert lib.hrt_accumulate(None, 1) == 1
    assert lib.hrt_synchronize(None) == 1
    buf = np.zeros(4, np.uint8)
    assert lib.hrt_read_image(None, 0, 0, _lib.ptr(buf), 4) == 1
