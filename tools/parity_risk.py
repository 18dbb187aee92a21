#!/usr/bin/env python3
"""Parity-risk study: how far can a real driver's frame sit from
the pinned oracle?  Traces the same frames with the oracle's driver-typical variants
(oracle/rt_oracle.c: ORC_DRIVER_MATH = glibc logf/sinf/cosf, ORC_DRIVER_RSQ = v * (1/sqrt),
-ffp-contract=fast, and all three) and reports the per-channel |delta| distribution of the fp32
frame (north_star's bar: |delta| <= 1e-4) and of the rgba8 frame against the pinned oracle.

    python tools/parity_risk.py [--headline-rows 9] > profiles/r02_parity_risk.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import pyoracle  # noqa: E402
from helpers import SceneCase  # noqa: E402

CASES = [  # (scene, size, spp, bounces, rows or None)
    ("cube", (256, 256), 1, 1, None),        # C1
    ("box", (512, 512), 16, 4, None),        # C2
    ("island", (192, 108), 8, 8, None),
    ("island", (64, 64), 4, 12, None),
    ("cave", (128, 72), 4, 8, None),
    ("spheres", (96, 72), 4, 8, None),
]


def stats(ref8, ref32, img8, img32):
    d = np.abs(img32[..., :3].astype(np.float64) - ref32[..., :3].astype(np.float64))
    d8 = np.abs(img8[..., :3].astype(np.int32) - ref8[..., :3].astype(np.int32))
    return {"channels": int(d.size), "frac_gt_1e-4": float((d > 1e-4).mean()), "max_abs": float(d.max()),
            "mean_abs": float(d.mean()), "p99_abs": float(np.quantile(d, 0.99)),
            "rgba8_frac_differing": float((d8 > 0).mean()), "rgba8_max_lsb": int(d8.max())}


def study(case, rows=None):
    y0, y1 = rows if rows else (0, case.size[1])
    ref8, ref32, _, _ = case.oracle(rows=rows, want_f32=True)
    out = {}
    for v in pyoracle.DRIVER_VARIANTS:
        lib = pyoracle.load_driver_variant(v)
        img8, img32, _, _ = pyoracle.trace(case.push(), case.rays, case.spheres, case.tris, case.meshes, rows=rows,
                                           want_f32=True, lib=lib)
        out[v] = stats(ref8[y0:y1], ref32[y0:y1], img8[y0:y1], img32[y0:y1])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--headline-rows", type=int, default=9, help="island 1080p 64spp 8b rows (0 = skip)")
    a = ap.parse_args()
    res = []
    for scene, size, spp, b, rows in CASES:
        t = time.time()
        r = study(SceneCase(scene, size, spp, b), rows)
        res.append({"scene": scene, "size": list(size), "spp": spp, "bounces": b, "variants": r,
                    "seconds": round(time.time() - t, 1)})
        print(json.dumps(res[-1]), file=sys.stderr)
    if a.headline_rows:
        case = SceneCase("island", (1920, 1080), 64, 8)
        for y in np.linspace(0, 1079, a.headline_rows).astype(int):
            t = time.time()
            r = study(case, (int(y), int(y) + 1))
            res.append({"scene": "island", "size": [1920, 1080], "spp": 64, "bounces": 8, "row": int(y),
                        "variants": r, "seconds": round(time.time() - t, 1)})
            print(json.dumps(res[-1]), file=sys.stderr)
    print(json.dumps({"study": "parity risk: driver-typical numerics vs the pinned oracle (fp32 frame |delta|)",
                      "threads": pyoracle.num_threads(), "cases": res}, indent=1))


if __name__ == "__main__":
    main()
