"""epq_raytracer_amd -- MI355X-native (gfx950 HIP) drop-in for the compute path of
hindlet/EPQ_Raytracer: the path-trace dispatch (assets/raytracing.glsl) and the progressive
accumulator (assets/image_combiner.glsl), behind the C ABI of libhip_raytrace.so
(include/hip_raytrace.h).  See DESIGN.md.
"""
from . import _lib
from .app import RayTracingApp, compute_n_then_render, compute_then_render
from .pipeline import (DiffusePipeline, HrtContext, Image, RayTracePipeline, RayTracerSettings, create_rays,
                       sphere_records, transform_meshes, view_matrix)
from .scene import (Camera, CustomMaterial, InvisLightMaterial, LambertianMaterial, LightMaterial, Mesh,
                    MetalMaterial, RayTracingMesh, Sphere, get_null_mesh, get_null_sphere, load_asset, load_obj, subdivide)
from .scenes import PRESETS, load_box_scene, load_cave_scene, load_cube_scene, load_island_scene, \
    load_spheres_scene, make_app, preset, scaled_preset

__all__ = [
    "RayTracingApp", "compute_then_render", "compute_n_then_render", "DiffusePipeline", "HrtContext", "Image",
    "RayTracePipeline", "RayTracerSettings", "create_rays", "sphere_records", "transform_meshes", "view_matrix",
    "Camera", "CustomMaterial", "InvisLightMaterial", "LambertianMaterial", "LightMaterial", "Mesh", "MetalMaterial",
    "RayTracingMesh", "Sphere", "get_null_mesh", "get_null_sphere", "load_asset", "load_obj", "PRESETS",
    "load_box_scene", "load_cave_scene", "load_cube_scene", "load_island_scene", "load_spheres_scene", "make_app",
    "preset", "scaled_preset", "subdivide",
]
