"""How long a persistent launch's workgroups hold their CUs beyond their waves' work, from the raw per-item
records tools/timeline.py --raw saves (a -DHRT_TIMELINE=1 build).

A 1,024-thread BUNDLE_WQ workgroup takes a whole CU (its LDS) and gives it back only when its last wave
ends.  In the realtime loop (one frame per launch, launches overlapped on lanes) the next frame's
workgroups can start on a CU only then, so the CU time between a wave's last item and its workgroup's end
is lost.  This prints, per launch: the span, the workgroups' end times, the CU-time held (sum over
workgroups of their end) against the wave work / waves per workgroup, and the share of held CU-time in
which fewer than 4 of the 16 waves run.

    python tools/wg_hold.py records.npy [--waves-per-wg 16]
"""
import argparse
import json

import numpy as np

TICK_US = 0.01


def analyse(r, per_wg=16):
    t0 = int(r[:, 0].min())
    s = (r[:, 0].astype(np.int64) - t0) * TICK_US
    e = (r[:, 2].astype(np.int64) - t0) * TICK_US
    wave = ((r[:, 3] >> 48) & 0xFFFF).astype(int)
    item = (r[:, 3] & 0xFFFFFFFF).astype(np.uint64)
    heavy = (((item >> 31) & 1) | ((item >> 22) & 7)) > 0
    waves = int(wave.max()) + 1
    wgs = (waves + per_wg - 1) // per_wg
    wave_end = np.zeros(waves)
    np.maximum.at(wave_end, wave, e)
    wg_end = wave_end.reshape(wgs, per_wg).max(axis=1) if waves == wgs * per_wg else \
        np.array([wave_end[g * per_wg:(g + 1) * per_wg].max() for g in range(wgs)])
    work = float((e - s).sum())
    held = float(wg_end.sum()) * per_wg  # wave-us of CU slots held
    # per workgroup: time (after its first wave ends) during which < 4 waves still run
    low = 0.0
    for g in range(wgs):
        ends = np.sort(wave_end[g * per_wg:(g + 1) * per_wg])
        if len(ends) >= 4:
            low += float(ends[-1] - ends[-4])
    heavy_wg = np.zeros(wgs, bool)
    np.logical_or.at(heavy_wg, wave[heavy] // per_wg, True)
    return {
        "items": int(len(r)), "waves": waves, "workgroups": wgs, "span_us": round(float(e.max()), 1),
        "wave_work_share_of_held": round(work / held, 4),
        "wg_end_us": {q: round(float(np.percentile(wg_end, p)), 1) for q, p in
                      (("p10", 10), ("p50", 50), ("p90", 90), ("max", 100))},
        "wave_end_us": {q: round(float(np.percentile(wave_end, p)), 1) for q, p in
                        (("p10", 10), ("p50", 50), ("p90", 90))},
        "wg_tail_under_4_waves_us_mean": round(low / wgs, 1),
        "heavy_items": int(heavy.sum()), "workgroups_with_heavy": int(heavy_wg.sum()),
        "heavy_end_us_p50": round(float(np.percentile(e[heavy], 50)), 1) if heavy.any() else None,
        "light_wg_end_us_p50": round(float(np.percentile(wg_end[~heavy_wg], 50)), 1) if (~heavy_wg).any() else None,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("raw")
    ap.add_argument("--waves-per-wg", type=int, default=16)
    a = ap.parse_args()
    r = np.load(a.raw)
    print(json.dumps({"raw": a.raw, **analyse(r, a.waves_per_wg)}))


if __name__ == "__main__":
    main()
