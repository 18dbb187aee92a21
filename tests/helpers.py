"""Shared test helpers: build the same scene records + push constants for the HIP path and the oracle."""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

import epq_raytracer_amd as E  # noqa: E402
from epq_raytracer_amd import _lib  # noqa: E402


class SceneCase:
    """Host-prepared records for a preset (or custom settings) at a given size / spp / bounces."""

    def __init__(self, name=None, size=(64, 64), num_samples=1, max_bounces=1, rng_offset=1, settings=None,
                 camera=None):
        if settings is None:
            camera, settings = E.preset(name)
        settings.num_samples, settings.max_bounces = num_samples, max_bounces
        self.name, self.size, self.camera, self.settings = name, tuple(size), camera, settings
        self.rays, self.n_rays, jit = E.create_rays(size, settings.camera_focal_length, settings.viewport_height,
                                                    settings.up)
        self.tris, meshes = E.transform_meshes(settings.mesh_data if settings.mesh_data else [E.get_null_mesh()])
        self.meshes = meshes[:len(settings.mesh_data)]
        self.spheres = E.sphere_records(settings.sphere_data)
        self.jitter = float(np.float32(settings.sample_jitter if settings.sample_jitter is not None else jit))
        self.rng_offset = rng_offset

    def push(self, rng_offset=None, init=False) -> _lib.PushConstants:
        pc = _lib.PushConstants()
        pos = np.asarray(self.camera.position, np.float32)
        pc.cam_pos[:] = [float(pos[0]), float(pos[1]), float(pos[2]), 1.0]
        pc.cam_alignment_mat[:] = [float(v) for v in E.view_matrix(self.camera.direction, self.camera.up)]
        pc.num_rays = self.n_rays
        pc.num_spheres = len(self.spheres)
        pc.num_meshes = len(self.meshes)
        pc.num_samples = max(int(self.settings.num_samples), 1)
        pc.jitter_size = self.jitter
        pc.max_bounces = max(int(self.settings.max_bounces), 0)
        pc.use_environment_light = int(bool(self.settings.use_environment_lighting))
        pc.rng_offset = self.rng_offset if rng_offset is None else rng_offset
        pc.init = int(init)
        pc.width, pc.height = self.size
        return pc

    def oracle(self, rng_offset=None, rows=None, want_f32=False, nthreads=0):
        import pyoracle
        return pyoracle.trace(self.push(rng_offset), self.rays, self.spheres, self.tris, self.meshes, rows=rows,
                              nthreads=nthreads, want_f32=want_f32)

    def context(self, mode=_lib.MODE_RGBA8, partition=None, variant=0, device=0, options=None,  # noqa: PLR0913
                debug=False):
        """options: {hrt_option: value} applied before set_scene (e.g. the BVH leaf size); debug binds
        libhip_raytrace_debug.so (diagnostics-only options, guard bands)."""
        ctx = E.HrtContext(self.size, device=device, mode=mode, partition=partition, debug=debug)
        ctx.set_option(_lib.OPT_KERNEL_VARIANT, variant)
        for k, v in (options or {}).items():
            ctx.set_option(k, v)
        ctx.set_scene(self.rays, self.spheres, self.tris, self.meshes)
        return ctx

    def gpu(self, rng_offset=None, mode=_lib.MODE_RGBA8, variant=0, fmt=None):
        ctx = self.context(mode=mode, variant=variant)
        ctx.trace(self.push(rng_offset))
        st = ctx.stats()
        img = ctx.read(_lib.IMG_TRACE, _lib.FMT_RGBA8 if fmt is None else fmt)
        ctx.close()
        return img, st.segments, st.tri_tests


def mismatch_report(a: np.ndarray, b: np.ndarray) -> str:
    diff = np.argwhere(np.any(a != b, axis=-1))
    if diff.size == 0:
        return "identical"
    y, x = diff[0]
    return f"{len(diff)} pixels differ; first at (x={x}, y={y}): {a[y, x]} vs {b[y, x]}"


GOLDEN_FULL = os.path.join(ROOT, "tests", "golden", "golden_full.json")


def golden_full(name: str) -> dict:
    """Whole-frame oracle digests at the BASELINE sizes (tests/golden/make_golden_full.py)."""
    import json
    with open(GOLDEN_FULL) as f:
        return json.load(f)["frames"][name]


def assert_frame_digest(img: np.ndarray, rec: dict, what: str) -> None:
    """img's SHA-256 equals the oracle's whole-frame digest; on a mismatch, name the rows that differ."""
    import hashlib
    if hashlib.sha256(np.ascontiguousarray(img).tobytes()).hexdigest() == rec["sha256_rgba8"]:
        return
    bad = [y for y in range(img.shape[0])
           if hashlib.sha256(np.ascontiguousarray(img[y]).tobytes()).hexdigest()[:16] != rec["row_sha256_16"][y]]
    raise AssertionError(f"{what}: the frame differs from the oracle's in {len(bad)} rows (first {bad[:10]})")
