"""Each row-tile partition of an N-GPU run, rendered alone on this GPU at bench.py's OWN shape (VERDICT r04
next 4): a fresh context per partition, init + frame 0 clear, the 5 warm-up frames as one hrt_compute_n,
then the 20 timed frames as one hrt_compute_n -- what one rank of `bench.py --gpus N` runs between its
barriers, minus the gather.  The whole frame (N = 1) is measured the same way in the same process, so the
line states each partition's kernel time against (whole-frame kernel time / N).

    python tools/rank_shape.py [--gpus 8] [--scene island] [--rounds 2] [--warmup 5] [--steps 20]

Prints one JSON line per (round, partition) and a summary line: per round, the slowest partition against
that round's whole frame / N (an N-GPU step waits for its slowest rank in that run); the summary's
slowest_over_fair is the worst round.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]

import epq_raytracer_amd as E  # noqa: E402
from epq_raytracer_amd import _lib  # noqa: E402


def run(args, part):
    """kernel ms per frame and wall ms per step of the timed launch, bench.py's sequence."""
    W, H = args.width, args.height
    camera, settings = E.preset(args.scene)
    settings.num_samples, settings.max_bounces = args.spp, args.bounces
    ctx = E.HrtContext((W, H), device=0, mode=_lib.MODE_RGBA8, partition=part)
    raytrace = E.RayTracePipeline(ctx, (W, H), settings)
    diffuse = E.DiffusePipeline(ctx, (W, H))
    ctx.set_option(_lib.OPT_FRAMES_PER_LAUNCH, 64)
    for k, v in args.option:
        ctx.set_option(k, v)
    raytrace.init()
    diffuse.next_frame(0, raytrace.image())
    if args.burn_ms > 0:  # (diagnosis) other GPU work right before the warm-up: does the clock ramp matter?
        burn = E.HrtContext((W, H), device=0, mode=_lib.MODE_RGBA8)
        brt = E.RayTracePipeline(burn, (W, H), settings)
        t_end = time.perf_counter() + args.burn_ms / 1e3
        k = 1
        while time.perf_counter() < t_end:
            burn.compute_n(brt.push_constants(camera, k, False), 4)
            burn.synchronize()
            k += 4
        burn.close()
    ctx.compute_n(raytrace.push_constants(camera, 1, False), args.warmup)
    ctx.synchronize()
    ctx.reset_stats()
    t0 = time.perf_counter()
    ctx.compute_n(raytrace.push_constants(camera, 1 + args.warmup, False), args.steps)
    ctx.synchronize()
    wall = (time.perf_counter() - t0) * 1e3 / args.steps
    st = ctx.stats()
    ctx.close()
    return st.total_trace_ms / max(st.traces, 1), wall, int(st.segments)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--scene", default="island")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--bounces", type=int, default=8)
    ap.add_argument("--row-tile", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--burn-ms", type=float, default=0.0, help="(diagnosis) GPU matmul work before each warm-up")
    ap.add_argument("--parts", type=int, nargs="*", default=None, help="partition indices (default all)")
    ap.add_argument("--option", type=lambda s: tuple(int(v) for v in s.split("=")), action="append", default=[],
                    help="KEY=VALUE hrt_set_option before the scene (repeatable)")
    a = ap.parse_args()
    parts = a.parts if a.parts is not None else list(range(a.gpus))
    whole, per = [], {p: [] for p in parts}
    for r in range(a.rounds):
        k, w, s = run(a, None)
        whole.append(k)
        print(json.dumps({"round": r, "part": "whole", "kernel_ms": round(k, 4), "wall_ms": round(w, 4),
                          "segments": s}), flush=True)
        for p in parts:
            k, w, s = run(a, (a.row_tile, p, a.gpus))
            per[p].append(k)
            print(json.dumps({"round": r, "part": p, "kernel_ms": round(k, 4), "wall_ms": round(w, 4),
                              "segments": s}), flush=True)
    # An N-GPU step waits for its slowest rank IN THAT RUN: per round, the slowest
    # part against that round's whole frame / N; the summary is the worst round, not each part's best.
    runs = []
    for r in range(a.rounds if parts else 0):  # (--parts with no values: whole frames only)
        fair_r = whole[r] / a.gpus
        slow_r = max(parts, key=lambda p: per[p][r])
        runs.append({"round": r, "fair_share_ms": round(fair_r, 4), "slowest_part": slow_r,
                     "slowest_ms": round(per[slow_r][r], 4), "slowest_over_fair": round(per[slow_r][r] / fair_r, 4)})
    worst = max(runs, key=lambda x: x["slowest_over_fair"]) if runs else {"slowest_over_fair": None}
    print(json.dumps({"summary": True, "scene": a.scene, "gpus": a.gpus, "shape": f"{a.warmup} warm-up + {a.steps}",
                      "whole_kernel_ms": [round(v, 4) for v in whole],
                      "part_kernel_ms": {p: [round(v, 4) for v in per[p]] for p in parts},
                      "runs": runs, "slowest_over_fair": worst["slowest_over_fair"],
                      "basis": "per run: max over parts / (that run's whole frame / N); summary = worst run",
                      "options": a.option}), flush=True)

if __name__ == "__main__":
    main()
