#!/usr/bin/env python3
"""Realtime-loop timing (compute_then_render per frame: one hrt_trace + hrt_accumulate per frame,
src/main.rs:41-57) for HRT_OPT_OVERLAP = 1..3 trace lanes, next to hrt_compute_n's batched rate.
Prints one JSON line per setting: ms per frame (wall clock over --frames frames after --warm)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]

from helpers import SceneCase, _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="island")
    ap.add_argument("--size", default="1920x1080")
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--bounces", type=int, default=8)
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--warm", type=int, default=4)
    ap.add_argument("--lanes", type=int, nargs="+", default=[1, 2, 3])
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--busy-split", type=int, nargs="+", default=[2], help="HRT_OPT_BUSY_SPLIT values")
    ap.add_argument("--defer", type=int, nargs="+", default=[1], help="HRT_OPT_DEFER_COMBINE values")
    ap.add_argument("--split", type=int, nargs="+", default=[0], help="HRT_OPT_SPLIT values (0 = auto)")
    ap.add_argument("--factor", type=int, nargs="+", default=[-1], help="HRT_OPT_SPLIT_FACTOR values (-1 = auto)")
    ap.add_argument("--no-accumulate", action="store_true",
                    help="traces only (the combine's cost and its waits left out: a lower bound)")
    ap.add_argument("--grid-cus", type=int, nargs="+", default=[0],
                    help="HRT_OPT_GRID_CUS values (libhip_raytrace_debug.so; 0 = every CU)")
    a = ap.parse_args()
    W, H = (int(v) for v in a.size.split("x"))
    case = SceneCase(a.scene, (W, H), a.spp, a.bounces)
    debug = a.grid_cus != [0]
    ctx = case.context(debug=debug)
    k = 1
    for r in range(a.rounds):
        for lanes, cus, bs, df, sp, fc in [(n, c, b, d, sp, fc) for n in a.lanes for c in a.grid_cus
                                           for b in a.busy_split for d in a.defer for sp in a.split
                                           for fc in a.factor]:
            ctx.set_option(_lib.OPT_SPLIT, sp)
            ctx.set_option(_lib.OPT_SPLIT_FACTOR, fc)
            ctx.set_option(_lib.OPT_DEFER_COMBINE, df)
            ctx.set_option(_lib.OPT_OVERLAP, lanes)
            ctx.set_option(_lib.OPT_BUSY_SPLIT, bs)
            if debug:
                ctx.set_option(_lib.OPT_GRID_CUS, cus)
            for _ in range(a.warm):
                ctx.trace(case.push(k))
                ctx.accumulate(k)
                k += 1
            ctx.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.frames):
                ctx.trace(case.push(k))
                if not a.no_accumulate:
                    ctx.accumulate(k)
                k += 1
            ctx.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / a.frames
            print(json.dumps({"round": r, "lanes": lanes, "grid_cus": cus, "busy_split": bs, "defer": df,
                              "split": sp, "factor": fc, "accumulate": not a.no_accumulate, "ms_per_frame": round(ms, 3)}), flush=True)
        if debug:
            ctx.set_option(_lib.OPT_GRID_CUS, 0)
        ctx.set_option(_lib.OPT_SPLIT, 0)
        ctx.set_option(_lib.OPT_SPLIT_FACTOR, -1)
        ctx.synchronize()
        t0 = time.perf_counter()
        ctx.compute_n(case.push(k), a.frames)
        ctx.synchronize()
        k += a.frames
        print(json.dumps({"round": r, "compute_n": a.frames,
                          "ms_per_frame": round((time.perf_counter() - t0) * 1e3 / a.frames, 3)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
