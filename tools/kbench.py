"""Kernel A/B on the GPU box: trace variants interleaved in ONE process (cdna guide rule 24).

    python tools/kbench.py --variants 1 2 3 4 --rounds 3 [--scene island --size 1920x1080 --spp 64 --bounces 8]

Prints, per variant: median / min kernel ms (HIP events), Mrays/s, algorithmic TFLOP/s (38 FLOP per
reference triangle test), lane efficiency (segments / (64 * wave steps)) and whether the frame is
byte-identical to variant 1 (literal).
"""
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
    ap.add_argument("--variants", type=int, nargs="+", default=[1, 2, 3, 4, 5], help="hrt_kernel values")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--scene", default="island")
    ap.add_argument("--size", default="1920x1080")
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--bounces", type=int, default=8)
    ap.add_argument("--json", default=None)
    ap.add_argument("--no-ref", action="store_true", help="skip the literal-kernel reference frame")
    ap.add_argument("--diag", action="store_true", help="also print the bundle kernels' cull diagnostics")
    ap.add_argument("--sec-batch", type=int, nargs="+", default=[0], help="HRT_OPT_SECONDARY_BATCH values to sweep (0 = auto)")
    ap.add_argument("--split", type=int, nargs="+", default=[0], help="HRT_OPT_SPLIT values to sweep (LDS variants)")
    ap.add_argument("--prio", type=int, nargs="+", default=[1], help="HRT_OPT_PRIORITY values to sweep")
    ap.add_argument("--factor", type=int, nargs="+", default=[-1], help="HRT_OPT_SPLIT_FACTOR values to sweep")
    ap.add_argument("--coop", type=int, nargs="+", default=[1], help="HRT_OPT_COOP values to sweep")
    ap.add_argument("--leaf", type=int, default=None, help="HRT_OPT_BVH_LEAF_SIZE for the scene build")
    ap.add_argument("--partition", default=None,
                    help="TILE,INDEX,COUNT: trace only one rank's row tiles (what each GPU does at N > 1)")
    a = ap.parse_args()
    W, H = (int(v) for v in a.size.split("x"))
    case = SceneCase(a.scene, (W, H), a.spp, a.bounces)
    part = tuple(int(v) for v in a.partition.split(",")) if a.partition else None
    ctx = case.context(options={_lib.OPT_BVH_LEAF_SIZE: a.leaf} if a.leaf else None, partition=part)
    print(json.dumps({"scene_info": ctx.scene_info()}), flush=True)
    pc = case.push(1)
    # warm up + reference image (literal kernel), unless profiling one variant alone
    ref = None
    if not a.no_ref:
        ctx.set_option(_lib.OPT_KERNEL_VARIANT, 1)
        ctx.trace(pc)
        ref = ctx.read(_lib.IMG_TRACE)
    combos = [(v, sb, k) for v in a.variants for sb in (a.sec_batch if v in (0, 4, 5, 6, 7, 8) else [a.sec_batch[0]])
              for k in ([(k, p, f, c) for k in a.split for p in a.prio for f in a.factor for c in a.coop]
                        if v in (0, 7, 8) else [(a.split[0], a.prio[0], a.factor[0], a.coop[0])])]
    res = {vs: [] for vs in combos}
    stats = {}
    same = {}
    for v, sb, k in combos:  # each combo's traces back to back: the schedule plans from its own last trace
        for r in range(-1, a.rounds):
            ctx.set_option(_lib.OPT_KERNEL_VARIANT, v)
            ctx.set_option(_lib.OPT_SECONDARY_BATCH, sb)
            ctx.set_option(_lib.OPT_SPLIT, k[0])
            ctx.set_option(_lib.OPT_PRIORITY, k[1])
            ctx.set_option(_lib.OPT_SPLIT_FACTOR, k[2])
            ctx.set_option(_lib.OPT_COOP, k[3])
            ctx.reset_stats()
            ctx.trace(pc)
            st = ctx.stats()
            if r < 0:
                continue  # warm-up: this combo's tile costs for the planner
            res[(v, sb, k)].append(st.total_trace_ms)
            stats[(v, sb, k)] = (st.segments, st.tri_tests, st.wave_steps)
            if r == 0:
                same[(v, sb, k)] = None if ref is None else bool(np.array_equal(ctx.read(_lib.IMG_TRACE), ref))
    if a.diag:
        for v in a.variants:
            if v in (0, 4, 5, 6, 7, 8, 9):
                ctx.set_option(_lib.OPT_KERNEL_VARIANT, v)
                ctx.set_option(_lib.OPT_COUNTERS, 2)
                ctx.reset_stats()
                ctx.trace(pc)
                d = ctx.diagnostics()
                d["variant"] = v
                d["primary_survival"] = d["primary_survivors"] / max(d["primary_considered"], 1)
                d["bounce_survival"] = d["bounce_survivors"] / max(d["bounce_considered"], 1)
                d["bounce_lanes_per_iter"] = d["bounce_lanes"] / max(d["bounce_iters"], 1)
                d["bvh_visits_per_lane"] = d["bvh_visits"] / max(d["bounce_lanes"], 1)
                d["bvh_prims_per_lane"] = d["bvh_prim_tests"] / max(d["bounce_lanes"], 1)
                d["bvh_band_per_lane"] = d["bvh_band_tests"] / max(d["bounce_lanes"], 1)
                cyc = d["primary_cycles"] + d["bounce_cycles"] + d["shade_cycles"]
                for ph in ("primary", "bounce", "shade"):
                    d[ph + "_cycle_share"] = d[ph + "_cycles"] / max(cyc, 1)
                d["bounce_cycles_per_iter"] = d["bounce_cycles"] / max(d["bounce_iters"], 1)
                d["bounce_stage2_frac"] = d["bounce_stage2"] / max(d["bounce_survivors"], 1)
                d["bounce_front_frac"] = d["bounce_front"] / max(d["bounce_survivors"], 1)
                d["bvh_trips_per_iter"] = d["bvh_trips"] / max(d["bounce_iters"], 1)
                d["bvh_leaf_trips_per_iter"] = d["bvh_leaf_trips"] / max(d["bounce_iters"], 1)
                d["primary_cycles_per_iter"] = d["primary_cycles"] / max(d["primary_iters"], 1)
                d["primary_list_len"] = d["primary_considered"] / max(d["primary_iters"], 1)
                # fused loop (non-sky items): lanes doing primary work per primary iteration, live lanes
                # per iteration, bounce lanes per batch -- each of 64
                sky_iters = d.get("sky_items", 0) * case.settings.num_samples
                d["primary_lane_use"] = d.get("primary_lanes", 0) / max(64 * (d["primary_iters"] - sky_iters), 1)
                d["live_lane_use"] = d.get("live_lanes", 0) / max(64 * d.get("loop_iters", 0), 1)
                d["band_max_per_batch"] = d.get("band_scan_max", 0) / max(d["bounce_iters"], 1)
                d["band_len_per_lane"] = d.get("band_scan_len", 0) / max(d["bounce_lanes"], 1)
                nsteps = sum(d.get(f"wq_steps_{b}", 0) for b in (16, 32, 48, 64))
                if nsteps:  # BUNDLE_WQ node steps by fill, and the share of the 4 member slots that are valid
                    for b in (16, 32, 48, 64):
                        d[f"wq_step_share_{b}"] = d[f"wq_steps_{b}"] / nsteps
                    d["wq_pairs_per_node_step"] = d["bvh_visits"] / nsteps
                    d["wq_member_use"] = d.get("wq_members", 0) / max(4 * d["bvh_visits"], 1)
                print(json.dumps(d), flush=True)
                ctx.set_option(_lib.OPT_COUNTERS, 1)
    out = []
    for v, sb, k in combos:
        ms = np.array(res[(v, sb, k)])
        seg, tt, ws = stats[(v, sb, k)]
        med = float(np.median(ms))
        row = {"variant": v, "sec_batch": sb, "split": k[0], "prio": k[1], "factor": k[2], "coop": k[3], "ms_median": round(med, 3), "ms_min": round(float(ms.min()), 3),
               "mrays_s": round(seg / med / 1e3, 1), "tflops_alg": round(38 * tt / med / 1e9, 2),
               "lane_eff": round(seg / max(64 * ws, 1), 4), "segments": seg, "tri_tests": tt,
               "identical_to_literal": same[(v, sb, k)]}
        out.append(row)
        print(json.dumps(row), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"workload": vars(a), "results": out}, f, indent=1)
    ctx.close()


if __name__ == "__main__":
    main()
