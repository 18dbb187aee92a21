"""Host-side cost of one bench step (bench.py's compute_n_then_render shape): the time from the step's
start to hrt_compute_n's return, against the whole step (to the stream's end) and the trace launch's own
HIP-event time.  python tools/host_overhead.py [--scene island] [--steps 20] [--reps 5] [--warmup 5]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]

import epq_raytracer_amd as E  # noqa: E402
from epq_raytracer_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="island")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=5, help="frames of the warm-up hrt_compute_n")
    a = ap.parse_args()
    W, H = 1920, 1080
    camera, settings = E.preset(a.scene)
    settings.num_samples, settings.max_bounces = 64, 8
    ctx = E.HrtContext((W, H), device=0, mode=_lib.MODE_RGBA8)
    raytrace = E.RayTracePipeline(ctx, (W, H), settings)
    diffuse = E.DiffusePipeline(ctx, (W, H))
    ctx.set_option(_lib.OPT_FRAMES_PER_LAUNCH, 64)
    raytrace.init()
    diffuse.next_frame(0, raytrace.image())
    frame = 1
    ctx.compute_n(raytrace.push_constants(camera, frame, False), a.warmup)
    frame += a.warmup
    ctx.synchronize()
    for _ in range(a.reps):
        ctx.reset_stats()
        ctx.synchronize()
        t0 = time.perf_counter()
        pc = raytrace.push_constants(camera, frame, False)
        t1 = time.perf_counter()
        ctx.compute_n(pc, a.steps)
        t2 = time.perf_counter()
        ctx.synchronize()
        t3 = time.perf_counter()
        frame += a.steps
        st = ctx.stats()
        print(f"push {1e6 * (t1 - t0):.0f} us, compute_n call {1e6 * (t2 - t1):.0f} us, step {1e3 * (t3 - t0):.3f} ms, "
              f"trace kernel {st.total_trace_ms:.3f} ms, step - kernel {1e3 * (t3 - t0) - st.total_trace_ms:.3f} ms",
              flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
