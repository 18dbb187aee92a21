"""Frame-to-frame stability of the persistent kernels' schedule: N consecutive traces of one
configuration, each planned from the previous one's tile costs.

    python tools/frames.py [--scene island --variant 0 --frames 12 --partition 16,0,8 --coop 1 --factor -1]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]

from helpers import SceneCase, _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="island")
    ap.add_argument("--size", default="1920x1080")
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--bounces", type=int, default=8)
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--frames", type=int, default=12)
    ap.add_argument("--partition", default=None)
    ap.add_argument("--coop", type=int, default=1)
    ap.add_argument("--factor", type=int, default=-1)
    ap.add_argument("--prio", type=int, default=1)
    ap.add_argument("--split", type=int, default=0)
    ap.add_argument("--ncap", type=int, default=0)
    ap.add_argument("--probe", type=int, default=1)
    ap.add_argument("--sec-batch", type=int, default=0)
    ap.add_argument("--leaf", type=int, default=0, help="> 0: BVH leaf size (HRT_OPT_BVH_LEAF_SIZE)")
    ap.add_argument("--width", type=int, default=0, help="> 0: BUNDLE_WQ group width (HRT_OPT_BVH_WIDTH)")
    ap.add_argument("--node-r", type=int, default=0, help="HRT_OPT_WQ_NODE_RADIUS (0 auto, 1 scene-wide R, 2 per node)")
    ap.add_argument("--batch", type=int, default=0,
                    help="> 0: each measurement is hrt_compute_n of this many frames (ms = per frame, wall incl. accumulates)")
    a = ap.parse_args()
    W, H = (int(v) for v in a.size.split("x"))
    case = SceneCase(a.scene, (W, H), a.spp, a.bounces)
    part = tuple(int(v) for v in a.partition.split(",")) if a.partition else None
    ctx = case.context(variant=a.variant, partition=part,
                       options={_lib.OPT_COOP: a.coop, _lib.OPT_SPLIT_FACTOR: a.factor, _lib.OPT_PRIORITY: a.prio,
                                _lib.OPT_SPLIT: a.split, _lib.OPT_SECONDARY_BATCH: a.sec_batch,
                                _lib.OPT_WQ_NODE_CAP: a.ncap, _lib.OPT_PROBE: a.probe, _lib.OPT_WQ_NODE_RADIUS: a.node_r,
                                **({_lib.OPT_BVH_LEAF_SIZE: a.leaf} if a.leaf > 0 else {}),
                                **({_lib.OPT_BVH_WIDTH: a.width} if a.width > 0 else {})},
                       debug=a.prio == 2)  # heavy tiles only: a libhip_raytrace_debug.so diagnostics mode
    pc = case.push(1)
    ms = []
    if a.batch > 0:
        import time
        ctx.set_option(_lib.OPT_FRAMES_PER_LAUNCH, a.batch)
        k = 1
        for _ in range(a.frames):
            ctx.synchronize()
            ctx.reset_stats()
            t0 = time.perf_counter()
            ctx.compute_n(case.push(k), a.batch)
            ctx.synchronize()
            ms.append(round((time.perf_counter() - t0) * 1e3 / a.batch, 3))
            k += a.batch
    for _ in range(a.frames if a.batch <= 0 else 0):
        ctx.reset_stats()
        ctx.trace(pc)
        ms.append(round(ctx.stats().total_trace_ms, 3))
    ctx.close()
    print(json.dumps({"batch": a.batch, "scene": a.scene, "variant": a.variant, "partition": a.partition, "coop": a.coop, "factor": a.factor,
                      "split": a.split, "sec_batch": a.sec_batch, "ncap": a.ncap, "probe": a.probe, "node_r": a.node_r, "leaf": a.leaf, "width": a.width, "prio": a.prio, "ms": ms}))


if __name__ == "__main__":
    main()
