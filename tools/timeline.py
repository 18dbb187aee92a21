"""Per-work-item timeline of one persistent trace launch at bench.py's shape (a build with -DHRT_TIMELINE=1,
passed as HRT_LIB): where a launch's time goes beyond its work -- the ramp-down tail (waves idle while the
last items finish), the heavy items' chains, the gaps between a wave's items.

    HRT_LIB=epq_raytracer_amd/build/ab_timeline/libhip_raytrace.so \\
        python tools/timeline.py [--partition 8,6,8] [--steps 20] [--warmup 5] [--json out.json]

Records (hip_raytrace.h HRT_DEBUG_OPT_TIMELINE): start, tile list built, end (s_memrealtime, 100 MHz), item word |
frame << 32 | run << 40 | sky << 47 | resident wave << 48.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]

import epq_raytracer_amd as E  # noqa: E402
from epq_raytracer_amd import _lib  # noqa: E402

TICK_US = 0.01  # s_memrealtime: 100 MHz


def records(ctx, cap):
    out = np.zeros(4 * cap, np.uint64)
    n = ctypes.c_uint32(0)
    _lib.check(ctx.lib.hrt_debug_timeline(ctx.handle, _lib.ptr(out), cap, ctypes.byref(n)), "hrt_debug_timeline",
               ctx.handle, ctx.lib)
    r = out[: 4 * min(n.value, cap)].reshape(-1, 4)
    return r, n.value


def analyse(r, waves):
    t0 = int(r[:, 0].min())
    s = (r[:, 0].astype(np.int64) - t0) * TICK_US
    su = (r[:, 1].astype(np.int64) - t0) * TICK_US
    e = (r[:, 2].astype(np.int64) - t0) * TICK_US
    w = r[:, 3]
    sky = ((w >> 47) & 1).astype(bool)
    setup = su - s
    item = (w & 0xFFFFFFFF).astype(np.uint64)
    hot = ((item >> 31) & 1).astype(bool)
    lk = ((item >> 22) & 7).astype(int)
    run = ((w >> 40) & 0x7F).astype(int)
    wave = ((w >> 48) & 0xFFFF).astype(int)
    span = float(e.max())
    dur = e - s
    # active waves over time (a wave is busy from its item's start to its end)
    grid = np.linspace(0.0, span, 201)
    busy = np.array([int(((s <= t) & (e > t)).sum()) for t in grid])
    frac = busy / max(waves, 1)

    def first_below(level):
        idx = np.nonzero((frac < level) & (grid > 0.05 * span))[0]
        return float(grid[idx[0]]) if len(idx) else span

    # per wave: its last item's end, its busy time, the gaps between its items
    last_end = np.zeros(waves)
    busy_t = np.zeros(waves)
    np.maximum.at(last_end, wave, e)
    np.add.at(busy_t, wave, dur)
    order = np.lexsort((s, wave))
    ws, we, wv = s[order], e[order], wave[order]
    same = wv[1:] == wv[:-1]
    gaps = (ws[1:] - we[:-1])[same]
    last = np.argsort(e)[-16:][::-1]
    heavy = hot | (lk > 0)
    return {
        "items": int(len(r)), "waves_seen": int(len(np.unique(wave))), "span_us": round(span, 1),
        "work_us_per_wave": round(float(dur.sum()) / waves, 1),
        "wave_utilisation": round(float(dur.sum()) / (waves * span), 4),
        "tail_us_below_90pct": round(span - first_below(0.9), 1),
        "tail_us_below_50pct": round(span - first_below(0.5), 1),
        "tail_us_below_10pct": round(span - first_below(0.1), 1),
        "wave_last_end_us": {"p10": round(float(np.percentile(last_end, 10)), 1),
                             "p50": round(float(np.percentile(last_end, 50)), 1),
                             "p90": round(float(np.percentile(last_end, 90)), 1)},
        "gap_us": {"mean": round(float(gaps.mean()), 3) if len(gaps) else None,
                   "p99": round(float(np.percentile(gaps, 99)), 3) if len(gaps) else None,
                   "sum_per_wave": round(float(gaps.sum()) / waves, 1)},
        "heavy": {"items": int(heavy.sum()),
                  "dur_us_p50": round(float(np.percentile(dur[heavy], 50)), 1) if heavy.any() else None,
                  "dur_us_max": round(float(dur[heavy].max()), 1) if heavy.any() else None,
                  "start_us_max": round(float(s[heavy].max()), 1) if heavy.any() else None,
                  "end_us_max": round(float(e[heavy].max()), 1) if heavy.any() else None},
        "tile_frames": int(run.sum()),
        "wave_us_per_tile_frame": {"all": round(float(dur.sum()) / max(int(run.sum()), 1), 2),
                                   "setup": round(float(setup.sum()) / max(int(run.sum()), 1), 2),
                                   "sky": round(float(dur[sky].sum()) / max(int(run.sum()), 1), 2),
                                   "nonsky": round(float(dur[~sky].sum()) / max(int(run.sum()), 1), 2)},
        "setup_us": {"p50": round(float(np.percentile(setup, 50)), 2), "mean": round(float(setup.mean()), 2),
                     "p99": round(float(np.percentile(setup, 99)), 2)},
        "sky_items": int(sky.sum()), "sky_runs_mean": round(float(run[sky].mean()), 2) if sky.any() else None,
        "nonsky_runs_mean": round(float(run[~sky].mean()), 2) if (~sky).any() else None,
        "nonsky_dur_us": {"p50": round(float(np.percentile(dur[~sky], 50)), 1),
                          "p99": round(float(np.percentile(dur[~sky], 99)), 1)} if (~sky).any() else None,
        "light": {"items": int((~heavy).sum()), "dur_us_p50": round(float(np.percentile(dur[~heavy], 50)), 1),
                  "dur_us_p99": round(float(np.percentile(dur[~heavy], 99)), 1),
                  "dur_us_max": round(float(dur[~heavy].max()), 1), "runs_mean": round(float(run[~heavy].mean()), 2)},
        "last_items": [{"end_us": round(float(e[i]), 1), "start_us": round(float(s[i]), 1),
                        "tile": int(item[i] & 0x3FFFFF), "lk": int(lk[i]), "hot": bool(hot[i]),
                        "frame": int((w[i] >> 32) & 0xFF), "run": int(run[i]), "sky": bool(sky[i])} for i in last],
        "busy_frac_curve": [round(float(v), 3) for v in frac[::10]],
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="island")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--bounces", type=int, default=8)
    ap.add_argument("--partition", default=None, help="TILE,INDEX,COUNT")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--cap", type=int, default=1 << 20)
    ap.add_argument("--option", type=lambda s: tuple(int(v) for v in s.split("=")), action="append", default=[])
    ap.add_argument("--json", default=None)
    ap.add_argument("--raw", default=None, help="also save the raw records (.npy)")
    ap.add_argument("--costs", default=None, help="save the warm-up launch's per-tile costs (.npy)")
    a = ap.parse_args()
    W, H = a.width, a.height
    camera, settings = E.preset(a.scene)
    settings.num_samples, settings.max_bounces = a.spp, a.bounces
    part = tuple(int(v) for v in a.partition.split(",")) if a.partition else None
    ctx = E.HrtContext((W, H), device=0, mode=_lib.MODE_RGBA8, partition=part)
    raytrace = E.RayTracePipeline(ctx, (W, H), settings)
    diffuse = E.DiffusePipeline(ctx, (W, H))
    ctx.set_option(_lib.OPT_FRAMES_PER_LAUNCH, 64)
    ctx.set_option(_lib.DEBUG_OPT_TIMELINE, a.cap)
    for k, v in a.option:
        ctx.set_option(k, v)
    raytrace.init()
    diffuse.next_frame(0, raytrace.image())
    ctx.compute_n(raytrace.push_constants(camera, 1, False), a.warmup)
    if a.costs:  # the warm-up's per-tile costs: the timed launch's plan input
        costs = np.zeros(ctx.local_rows // 8 * ((W + 7) // 8) + 64, np.uint32)
        _lib.check(ctx.lib.hrt_debug_tile_costs(ctx.handle, _lib.ptr(costs), costs.size), "tile costs", ctx.handle,
                   ctx.lib)
        np.save(a.costs, costs)
    ctx.synchronize()
    ctx.reset_stats()
    ctx.compute_n(raytrace.push_constants(camera, 1 + a.warmup, False), a.steps)
    ctx.synchronize()
    st = ctx.stats()
    r, n = records(ctx, a.cap)
    if a.raw:
        np.save(a.raw, r)
    waves = int(((r[:, 3] >> 48) & 0xFFFF).max()) + 1 if len(r) else 1  # resident waves (each takes an item)
    res = {"scene": a.scene, "partition": a.partition, "frames": a.steps, "options": a.option,
           "kernel_ms_per_frame": round(st.total_trace_ms / max(st.traces, 1), 4),
           "launch_ms": round(st.total_trace_ms / max(st.traces, 1) * a.steps, 3), "records": n,
           **analyse(r, waves)}
    ctx.close()
    print(json.dumps(res), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
