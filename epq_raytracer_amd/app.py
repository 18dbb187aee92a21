"""RayTracingApp: frame sequencing of src/raytracing_app.rs without the window.

The reference's frame counter is both the accumulator weight and the RNG ``rng_offset``:
``open`` clears the trace image and the accumulator with frame 0 (:128-129) and leaves frame = 1,
so the first traced frame uses rng_offset = 1 (:139, :181, :193).  Presentation
(RenderPassOverFrame, src/texture_draw_pipeline.rs) is out of scope: ``render`` hooks receive the
accumulated Image and may read it back.
"""
from __future__ import annotations

from typing import Callable, Optional

from . import _lib
from .pipeline import DiffusePipeline, HrtContext, Image, RayTracePipeline, RayTracerSettings
from .scene import Camera


class RayTracingApp:
    """src/raytracing_app.rs:32-140 (public fields camera / pipeline; private frame / settings)."""

    def __init__(self, camera: Camera, settings: RayTracerSettings, device: int = -1, mode: int = _lib.MODE_RGBA8,
                 partition=None):
        self.camera = camera
        self.settings = settings
        self.device, self.mode, self.partition = device, mode, partition
        self.pipeline = None  # (RayTracePipeline, DiffusePipeline, presenter)
        self.context: Optional[HrtContext] = None
        self.frame = 0

    def open(self, image_size, render: Optional[Callable[[Image], None]] = None) -> None:
        """src/raytracing_app.rs:74-140: build pipelines, clear both images, frame -> 1."""
        self.context = HrtContext(image_size, device=self.device, mode=self.mode, partition=self.partition)
        raytrace = RayTracePipeline(self.context, image_size, self.settings)
        diffuse = DiffusePipeline(self.context, image_size)
        raytrace.init()                                         # :128
        diffuse.next_frame(self.frame, raytrace.image())        # :129 (frame 0 clears)
        if render is not None:
            render(diffuse.image())                             # :131-136
        self.pipeline = (raytrace, diffuse, render)
        self.frame += 1                                         # :139

    def close(self) -> None:
        if self.context is not None:
            self.context.close()
            self.context = None
            self.pipeline = None


def compute_then_render(app: RayTracingApp, frame_time: float = 0.0) -> None:
    """src/raytracing_app.rs:156-194 (one traced frame + accumulate + present)."""
    app.camera.do_move(frame_time)
    raytrace, diffuse, render = app.pipeline
    raytrace.compute(app.camera, app.frame)
    diffuse.next_frame(app.frame, raytrace.image())
    if render is not None:
        render(diffuse.image())
    app.frame += 1


def compute_n_then_render(app: RayTracingApp, num_renders: int) -> None:
    """src/raytracing_app.rs:196-227 (N frames chained without a host wait, then one present).

    The frame loop is one hrt_compute_n call: the same traces and accumulates byte for byte, with the
    persistent kernels tracing several frames per launch."""
    raytrace, diffuse, render = app.pipeline
    if num_renders > 0:
        if diffuse.ctx is not raytrace.ctx:
            raise ValueError("the trace and the accumulator must share one context")
        raytrace.ctx.compute_n(raytrace.push_constants(app.camera, app.frame, False), num_renders)
        app.frame += num_renders
    if render is not None:
        render(diffuse.image())
