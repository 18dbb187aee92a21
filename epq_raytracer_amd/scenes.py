"""Scene presets: src/main.rs:62-347 (spheres, box, cube, island) plus the build-defined Cave scene
(Cave.obj ships without a preset in the reference).

Each ``load_*_scene`` returns ``(camera, settings)`` -- the arguments the reference passes to
``RayTracingApp::new`` -- and ``make_app`` wraps them.
"""
from __future__ import annotations

import numpy as np

from .app import RayTracingApp
from .pipeline import RayTracerSettings
from .scene import (Camera, CustomMaterial, InvisLightMaterial, LambertianMaterial, LightMaterial, Mesh, MetalMaterial,
                    RayTracingMesh, Sphere, load_asset, subdivide)

F = np.float32


def _div(a, b):
    return float(F(a) / F(b))  # Rust f32 division


def load_spheres_scene():
    """src/main.rs:62-126."""
    spheres = [
        Sphere([0.0, -100.0, 0.0], 100.0, LambertianMaterial([0.5, 0.5, 0.5])),
        Sphere([2.5, 0.75, 0.0], 1.0, MetalMaterial([0.2, 0.2, 1.0], 1.0, 0.1)),
        Sphere([-2.5, 0.75, 0.0], 1.0, MetalMaterial([1.0, 0.2, 0.2], 1.0, 0.1)),
        Sphere([0.0, 1.0, 0.0], 1.0, MetalMaterial([0.2, 1.0, 0.2], 1.0, 0.1)),
        Sphere([500.0, 100.0, 500.0], 250.0, InvisLightMaterial([0.6, 0.6, 1.0, 25.0])),
    ]
    cam = Camera([2.0, 2.0, -5.0], [-0.35, -0.35, 0.87])
    return cam, RayTracerSettings(num_samples=25, max_bounces=50, use_environment_lighting=False, sample_jitter=None,
                                  sphere_data=spheres, mesh_data=[], camera_focal_length=1.0, viewport_height=2.0,
                                  up=cam.up)


def load_box_scene():
    """src/main.rs:130-233 (box.obj; meshes re-ordered as listed there)."""
    m = load_asset("box")
    wall = dict(smoothness=0.7, specular_probability=0.5)
    mesh_data = [
        RayTracingMesh(m[0], CustomMaterial(colour=[1.0, 1.0, 1.0], **wall)),                       # floor
        RayTracingMesh(m[4], CustomMaterial(colour=[_div(166.0, 255.0), _div(45.0, 255.0), _div(23.0, 255.0)],
                                            **wall)),                                                 # left wall
        RayTracingMesh(m[3], CustomMaterial(colour=[_div(19.0, 255.0), _div(133.0, 255.0), _div(34.0, 255.0)],
                                            **wall)),                                                 # right wall
        RayTracingMesh(m[1], CustomMaterial(colour=[1.0] * 3, **wall)),                              # back wall
        RayTracingMesh(m[5], CustomMaterial(colour=[1.0] * 3, **wall)),                              # ceiling
        RayTracingMesh(m[2], CustomMaterial(colour=[1.0] * 3, **wall)),                              # front wall
        RayTracingMesh(m[6], InvisLightMaterial([1.0, 1.0, 1.0, 5.0])),                              # light
    ]
    spheres = [Sphere([0.0, 0.5, 0.0], 0.5, MetalMaterial([1.0, 1.0, 1.0], 1.0, 0.0))]
    cam = Camera([1.5, 1.0, 0.0], [-1.0, 0.0, 0.0])
    return cam, RayTracerSettings(num_samples=5, max_bounces=50, use_environment_lighting=False, sample_jitter=0.005,
                                  sphere_data=spheres, mesh_data=mesh_data, camera_focal_length=1.0,
                                  viewport_height=2.0, up=cam.up)


def load_cube_scene():
    """src/main.rs:236-278 (Cube.obj)."""
    m = load_asset("Cube")
    mesh_data = [RayTracingMesh(m[0], MetalMaterial([0.7, 0.7, 0.7], 1.0, 0.0))]
    spheres = [Sphere([0.0, 0.0, 0.0], 1.0, MetalMaterial([1.0, 1.0, 1.0], 1.0, 0.0))]
    cam = Camera([5.0, 2.0, 0.0], [-1.0, -0.2, 0.0])
    return cam, RayTracerSettings(num_samples=10, max_bounces=50, use_environment_lighting=True, sample_jitter=None,
                                  sphere_data=spheres, mesh_data=mesh_data, camera_focal_length=1.0,
                                  viewport_height=2.0, up=cam.up)


def load_island_scene():
    """src/main.rs:282-347 (island.obj: Tree, Island, Leaves, Water; island.mtl defines nothing)."""
    m = load_asset("island")
    mesh_data = [
        RayTracingMesh(m[0], LambertianMaterial([0.40, 0.26, 0.16])),  # Tree
        RayTracingMesh(m[1], LambertianMaterial([0.46, 0.46, 0.46])),  # Island
        RayTracingMesh(m[2], LambertianMaterial([0.14, 0.46, 0.18])),  # leaves
        RayTracingMesh(m[3], LambertianMaterial([0.21, 0.63, 0.82])),  # glowing water
    ]
    cam = Camera([-5.0, 10.0, -20.0], [0.2, -0.4, 1.0])
    return cam, RayTracerSettings(num_samples=10, max_bounces=50, use_environment_lighting=True, sample_jitter=None,
                                  sphere_data=[], mesh_data=mesh_data, camera_focal_length=1.0, viewport_height=2.0,
                                  up=cam.up)


def load_cave_scene():
    """Build-defined (no reference preset): camera inside the cave looking at the crystals, the four
    crystals as visible lights, the cave shell Lambertian, the water metal; environment light on
    (the icosphere's normals face outward, so from inside the shell is back-face culled)."""
    m = load_asset("Cave")
    crystal = LightMaterial([0.55, 0.35, 1.0, 2.0])
    mesh_data = [
        RayTracingMesh(m[0], crystal),
        RayTracingMesh(m[1], crystal),
        RayTracingMesh(m[2], crystal),
        RayTracingMesh(m[3], crystal),
        RayTracingMesh(m[4], LambertianMaterial([0.45, 0.42, 0.40])),
        RayTracingMesh(m[5], MetalMaterial([0.2, 0.5, 0.7], 0.95, 0.05)),
    ]
    cam = Camera([5.0, 3.0, 10.0], [-20.0, -1.0, -15.0])
    return cam, RayTracerSettings(num_samples=10, max_bounces=50, use_environment_lighting=True, sample_jitter=None,
                                  sphere_data=[], mesh_data=mesh_data, camera_focal_length=1.0, viewport_height=2.0,
                                  up=cam.up)


PRESETS = {
    "spheres": load_spheres_scene,
    "box": load_box_scene,
    "cube": load_cube_scene,
    "island": load_island_scene,
    "cave": load_cave_scene,
}


def scaled_preset(name: str, k: int):
    """Preset `name` with every mesh triangle split into k*k (scene.subdivide): the triangle-count
    scaling workload for the kernel variants (e.g. "island@4" = 16x the island's triangles)."""
    cam, settings = PRESETS[name]()
    for rm in settings.mesh_data:
        rm.mesh = subdivide(rm.mesh, k)
    return cam, settings


def soup_scene(n: int, seed: int = 0x5EED):
    """SURVEY.md 8(d)'s roofline-sweep scene: n triangles with vertices uniform in [-10, 10]^3 (seed
    0x5EED), one Lambertian 0.5 mesh, environment light on, camera at (0, 0, -25) looking +z."""
    rng = np.random.default_rng(seed)
    v = rng.uniform(-10.0, 10.0, size=(n * 3, 3)).astype(np.float32)
    mesh = Mesh(v, np.arange(n * 3, dtype=np.uint32))
    cam = Camera([0.0, 0.0, -25.0], [0.0, 0.0, 1.0])
    return cam, RayTracerSettings(num_samples=1, max_bounces=8, use_environment_lighting=True,
                                  mesh_data=[RayTracingMesh(mesh, LambertianMaterial([0.5, 0.5, 0.5]))], up=cam.up)


def preset(name: str):
    """PRESETS[name]() or, for "<preset>@<k>", scaled_preset(preset, k); "soup<n>" = soup_scene(n)."""
    if "@" in name:
        base, k = name.split("@")
        return scaled_preset(base, int(k))
    if name.startswith("soup") and name[4:].isdigit():
        return soup_scene(int(name[4:]))
    return PRESETS[name]()


def make_app(name: str, num_samples=None, max_bounces=None, **kw) -> RayTracingApp:
    cam, settings = preset(name)
    if num_samples is not None:
        settings.num_samples = num_samples
    if max_bounces is not None:
        settings.max_bounces = max_bounces
    return RayTracingApp(cam, settings, **kw)
