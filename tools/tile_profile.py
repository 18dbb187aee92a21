"""Per-tile cost map of one trace (diagnostics build): where the frame's critical path is.

    python tools/tile_profile.py [--scene island --size 1920x1080 --spp 64 --bounces 8 --variant 0 --npz out.npz]

Prints the distribution of shader clocks per 8x8 tile, the slowest tiles (tile x, y) with their share
of the frame, and the per-lane segment counts of the slowest tile (the sequential sample chain)."""
import argparse
import json
import os
import sys

import numpy as np

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
    ap.add_argument("--split", type=int, default=0, help="HRT_OPT_SPLIT (heavy tiles as k items; 0 auto)")
    ap.add_argument("--prio", type=int, default=1, help="HRT_OPT_PRIORITY")
    ap.add_argument("--cus", type=int, default=0, help="HRT_OPT_GRID_CUS (1: tiles run near solo)")
    ap.add_argument("--npz", default=None)
    ap.add_argument("--partition", default=None, help="TILE,INDEX,COUNT: one rank's row tiles")
    a = ap.parse_args()
    W, H = (int(v) for v in a.size.split("x"))
    case = SceneCase(a.scene, (W, H), a.spp, a.bounces)
    part = tuple(int(v) for v in a.partition.split(",")) if a.partition else None
    ctx = case.context(variant=a.variant, partition=part, debug=True)  # HRT_OPT_GRID_CUS, priority 2
    pc = case.push(1)
    ctx.set_option(_lib.OPT_SPLIT, a.split)
    ctx.set_option(_lib.OPT_PRIORITY, a.prio)
    ctx.set_option(_lib.OPT_GRID_CUS, a.cus)
    ctx.trace(pc)  # warm (and the planner's tile costs)
    ctx.set_option(_lib.OPT_COUNTERS, 2)
    ctx.reset_stats()
    ctx.trace(pc)
    st = ctx.stats()
    raw = ctx.tile_profile()
    rec = raw.astype(np.float64)
    ctx.close()
    prof = rec[..., 0]
    flat = prof.ravel()
    its, surv, bcyc = (rec[..., k].ravel() for k in (1, 2, 3))
    its = (raw[..., 1].ravel() & np.uint64(0xFFFFFFFF)).astype(np.float64)
    steps = (raw[..., 1].ravel() >> np.uint64(32)).astype(np.float64)  # BUNDLE_WQ pair steps
    raw2 = raw[..., 2].ravel().astype(np.uint64)
    bvh = st.last_kernel in (6, 8, 9)  # BUNDLE_BVH*: slot 2 = node visits | (triangle tests << 32), per lane
    visits, btests = (raw2 & np.uint64(0xFFFFFFFF)).astype(np.float64), (raw2 >> np.uint64(32)).astype(np.float64)
    order = np.argsort(flat)[::-1]
    ty, tx = prof.shape
    res = {"scene": a.scene, "variant": int(st.last_kernel), "partition": a.partition, "split": a.split, "prio": a.prio, "cus": a.cus, "kernel_ms_diag": st.last_trace_ms, "tiles": int(flat.size),
           "clocks_p50": float(np.median(flat)), "clocks_p90": float(np.percentile(flat, 90)),
           "clocks_p99": float(np.percentile(flat, 99)), "clocks_max": float(flat.max()),
           "max_over_mean": float(flat.max() / flat.mean()),
           "bounce_iters_p50": float(np.median(its)), "bounce_clocks_per_iter_all": float(bcyc.sum() / max(its.sum(), 1)),
           "slowest": [{"tile_x": int(i % tx), "tile_y": int(i // tx), "clocks": float(flat[i]),
                        "bounce_iters": float(its[i]), "pair_steps": float(steps[i]),
                        **({"bvh_visits_per_lane": round(visits[i] / 64, 1), "bvh_tests_per_lane": round(btests[i] / 64, 1)}
                           if bvh else {"survivors_per_iter": round(surv[i] / max(its[i], 1), 1)}),
                        "bounce_clocks_per_iter": round(bcyc[i] / max(its[i], 1)),
                        "bounce_share": round(bcyc[i] / max(flat[i], 1), 3)} for i in order[:8]]}
    print(json.dumps(res), flush=True)
    if a.npz:
        np.savez_compressed(a.npz, tile_clocks=prof, tile_records=rec)


if __name__ == "__main__":
    main()
