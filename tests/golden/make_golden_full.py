"""Generate tests/golden/golden_full.json: whole-frame oracle digests at the BASELINE sizes.

VERDICT r02 "Missing #2": at 1080p the GPU frames were compared with the oracle on sampled rows only.
The CPU oracle (oracle/rt_oracle.c, the restatement of assets/raytracing.glsl:355-389 and
assets/image_combiner.glsl:22-43) needs ~17 min per island 1080p 64 spp frame on 8 threads, far too
long for a test, so it runs once here and the digests are committed:

  * headline  island 1920x1080, 64 spp, 8 bounces, rng_offset 1 (BASELINE.json's metric config)
  * c3        Cave   1920x1080, 64 spp, 8 bounces, rng_offset 1 (BASELINE config C3)
  * c4        island 1920x1080, 64 spp x 4 frames (rng_offset 1..4), the rgba8 accumulator after
              the reference's frame sequence: clear (frame 0), then trace k + combine(k), k = 1..4
              (src/raytracing_app.rs:128-139,196-227; BASELINE config C4)

Each record holds the SHA-256 of the whole rgba8 image, a 16-hex-digit SHA-256 prefix per row (so a
failing test names the rows that differ) and the exact segment / triangle-test counts.  The GPU tests
(tests/test_gpu_configs.py, tests/test_gpu_parity.py) hash the HIP frames and compare.

Run (about 90 min on 8 cores; resumable -- finished frames are kept in golden_full.partial.npz):
    python tests/golden/make_golden_full.py [--threads 8]
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from helpers import SceneCase  # noqa: E402
import pyoracle  # noqa: E402

OUT = os.path.join(HERE, "golden_full.json")
PARTIAL = os.path.join(HERE, "golden_full.partial.npz")  # scratch (git-ignored)


def digest(img: np.ndarray) -> dict:
    return {"sha256_rgba8": hashlib.sha256(img.tobytes()).hexdigest(),
            "row_sha256_16": [hashlib.sha256(img[y].tobytes()).hexdigest()[:16] for y in range(img.shape[0])]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=0)
    args = ap.parse_args()
    done = dict(np.load(PARTIAL)) if os.path.exists(PARTIAL) else {}

    def frame(scene, k):
        key = f"{scene}_{k}"
        if key not in done:
            case = SceneCase(scene, (1920, 1080), 64, 8, rng_offset=k)
            t = time.time()
            img, _, seg, tt = case.oracle(nthreads=args.threads)
            print(f"{key}: {seg} segments, {tt} triangle tests, {time.time() - t:.0f} s", flush=True)
            done[key] = img
            done[key + "_counts"] = np.array([seg, tt], np.uint64)
            np.savez(PARTIAL, **done)
        return done[key], [int(v) for v in done[key + "_counts"]]

    meta = {"generator": "tests/golden/make_golden_full.py", "oracle": "oracle/rt_oracle.c", "frames": {}}
    cfg = {"scene": "island", "size": [1920, 1080], "spp": 64, "bounces": 8}
    img, (seg, tt) = frame("island", 1)
    meta["frames"]["headline"] = {**cfg, "rng_offset": 1, "segments": seg, "tri_tests": tt, **digest(img)}
    cave, (cseg, ctt) = frame("cave", 1)
    meta["frames"]["c3"] = {**cfg, "scene": "cave", "rng_offset": 1, "segments": cseg, "tri_tests": ctt,
                            **digest(cave)}
    acc = np.zeros_like(img)
    pyoracle.accumulate_rgba8(0, acc, img)  # frame 0: the clear (image_combiner.glsl:33-36)
    segs = tests = 0
    for k in range(1, 5):
        fk, (s, t) = frame("island", k)
        pyoracle.accumulate_rgba8(k, acc, fk)
        segs, tests = segs + s, tests + t
    meta["frames"]["c4"] = {**cfg, "frames": [1, 2, 3, 4], "image": "accumulator", "segments": segs,
                            "tri_tests": tests, **digest(acc)}
    with open(OUT, "w") as f:
        json.dump(meta, f, indent=0)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
