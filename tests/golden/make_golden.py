"""Generate tests/golden/golden.npz + golden.json: frames and per-pixel traces of the CPU oracle.

The reference ships no golden images and cannot run here, so these fixtures pin
the ORACLE (regression guard) and are the bar the HIP path is held to byte for byte.  The RNG KATs in
golden.json are the ones derived from assets/raytracing.glsl:13-21 in SURVEY.md 8(c).
Regenerate (only after an intended numerics-spec change):  python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from helpers import SceneCase  # noqa: E402
import pyoracle  # noqa: E402

FRAMES = {
    # name: (scene, size, spp, bounces, rng_offset)  -- SURVEY.md 8(c) fixture list + one per scene
    "cube_256_s1_b1": ("cube", (256, 256), 1, 1, 1),
    "box_128_s4_b4": ("box", (128, 128), 4, 4, 1),
    "island_96x54_s4_b8": ("island", (96, 54), 4, 8, 1),
    "cave_64x36_s2_b8": ("cave", (64, 36), 2, 8, 3),
    "spheres_64x48_s4_b8": ("spheres", (64, 48), 4, 8, 2),
}
PIXELS = [("box_128_s4_b4", 64, 64), ("box_128_s4_b4", 5, 120), ("island_96x54_s4_b8", 48, 30),
          ("cube_256_s1_b1", 128, 128)]


def main():
    arrays, meta = {}, {"frames": {}, "pixels": [], "rng": {}}
    cases = {}
    for name, (scene, size, spp, b, off) in FRAMES.items():
        case = SceneCase(scene, size, spp, b, rng_offset=off)
        cases[name] = case
        img, f32, seg, tt = case.oracle(want_f32=True)
        arrays[name] = img
        arrays[name + "_f32"] = f32
        meta["frames"][name] = {"scene": scene, "size": list(size), "spp": spp, "bounces": b, "rng_offset": off,
                                "segments": int(seg), "tri_tests": int(tt),
                                "sha256_rgba8": hashlib.sha256(img.tobytes()).hexdigest()}
    for name, x, y in PIXELS:
        c = cases[name]
        rgb, seg, tt = pyoracle.trace_pixel(c.push(), c.rays, c.spheres, c.tris, c.meshes, x, y)
        meta["pixels"].append({"frame": name, "x": x, "y": y, "rgb_bits": [int(v) for v in rgb.view(np.uint32)],
                               "segments": int(seg), "tri_tests": int(tt)})
    for seed in (719393, 0, 1, 0xFFFFFFFF):
        meta["rng"][str(seed)] = pyoracle.hash_sequence(seed, 8)
    np.savez_compressed(os.path.join(HERE, "golden.npz"), **arrays)
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote", len(arrays), "arrays")


if __name__ == "__main__":
    main()
