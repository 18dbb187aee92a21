"""RayTracingApp: frame sequencing of src/raytracing_app.rs without the window.

The reference's frame counter is both the accumulator weight and the RNG ``rng_offset``:
``open`` clears the trace image and the accumulator with frame 0 (:128-129) and leaves frame = 1,
so the first traced frame uses rng_offset = 1 (:139, :181, :193).  Presentation
(RenderPassOverFrame, src/texture_draw_pipeline.rs) is out of scope: ``render`` hooks receive the
accumulated Image and may read it back.
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np

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

    def checkpoint(self, path: str) -> None:
        """Save the progressive render's state (SURVEY.md §5 checkpoint / resume, not a reference
        feature): the accumulated image in the context's own format and the frame counter."""
        ctx = self.context
        fmt = _lib.FMT_RGBA8 if ctx.mode == _lib.MODE_RGBA8 else _lib.FMT_RGBA32F
        np.savez(path, accum=ctx.read(_lib.IMG_ACCUM, fmt), frame=np.uint64(self.frame), mode=np.uint32(ctx.mode),
                 size=np.array([ctx.width, ctx.height, ctx.local_rows, ctx.row_tile, ctx.part_index, ctx.part_count],
                               np.uint32))

    def resume(self, path: str) -> None:
        """Continue a checkpointed render on an open app of the same size, mode and partition: the next
        frame traces with rng_offset = the saved frame counter, so the result equals an uninterrupted run."""
        ctx = self.context
        with np.load(path, allow_pickle=False) as z:
            size = [int(v) for v in z["size"]]
            if int(z["mode"]) != ctx.mode or size != [ctx.width, ctx.height, ctx.local_rows, ctx.row_tile,
                                                       ctx.part_index, ctx.part_count]:
                raise ValueError("checkpoint of another image size, mode or partition")
            ctx.load_accumulator(z["accum"])
            self.frame = int(z["frame"])

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
