"""Golden fixtures (CPU): the oracle reproduces tests/golden (made by tests/golden/make_golden.py),
and its FMA and generic builds agree bit for bit (explicit fmaf either way: numerics spec S2)."""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import pyoracle
from helpers import SceneCase

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
META = json.load(open(os.path.join(GOLD, "golden.json")))


@pytest.fixture(scope="module")
def arrays():
    with np.load(os.path.join(GOLD, "golden.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize("name", sorted(META["frames"]))
def test_oracle_reproduces_golden_frame(name, arrays):
    m = META["frames"][name]
    case = SceneCase(m["scene"], tuple(m["size"]), m["spp"], m["bounces"], rng_offset=m["rng_offset"])
    img, f32, seg, tt = case.oracle(want_f32=True)
    assert hashlib.sha256(img.tobytes()).hexdigest() == m["sha256_rgba8"]
    np.testing.assert_array_equal(img, arrays[name])
    np.testing.assert_array_equal(f32.view(np.uint32), arrays[name + "_f32"].view(np.uint32))
    assert (seg, tt) == (m["segments"], m["tri_tests"])


def test_golden_pixels():
    for p in META["pixels"]:
        m = META["frames"][p["frame"]]
        c = SceneCase(m["scene"], tuple(m["size"]), m["spp"], m["bounces"], rng_offset=m["rng_offset"])
        rgb, seg, tt = pyoracle.trace_pixel(c.push(), c.rays, c.spheres, c.tris, c.meshes, p["x"], p["y"])
        assert [int(v) for v in rgb.view(np.uint32)] == p["rgb_bits"]
        assert (seg, tt) == (p["segments"], p["tri_tests"])


def test_golden_rng():
    for seed, seq in META["rng"].items():
        assert pyoracle.hash_sequence(int(seed), 8) == seq


def test_fma_and_generic_oracle_builds_agree():
    code = ("import sys, hashlib; sys.path[:0] = [%r, %r]; from helpers import SceneCase; "
            "img = SceneCase('island', (48, 27), 2, 8).oracle()[0]; print(hashlib.sha256(img.tobytes()).hexdigest())"
            % (HERE, os.path.join(os.path.dirname(HERE), "oracle")))
    outs = []
    for variant in ("fma", "generic"):
        env = dict(os.environ, ORC_VARIANT=variant, OMP_NUM_THREADS="2")
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, check=True)
        outs.append(r.stdout.strip())
    assert outs[0] == outs[1] and len(outs[0]) == 64


def test_whole_frame_digests_reproduced_on_sampled_rows():
    """tests/golden/golden_full.json (the oracle's whole-frame digests at the BASELINE sizes, which the
    GPU suite hashes its 1080p frames against) is reproduced by the oracle on sampled rows: the row
    digests of the headline and C3 frames, and the C4 accumulator rows through the combiner."""
    full = json.load(open(os.path.join(GOLD, "golden_full.json")))["frames"]
    for name, scene in (("headline", "island"), ("c3", "cave")):
        m = full[name]
        case = SceneCase(scene, tuple(m["size"]), m["spp"], m["bounces"], rng_offset=m["rng_offset"])
        for y in (0, 541):
            img = case.oracle(rows=(y, y + 1))[0]
            assert hashlib.sha256(img[y].tobytes()).hexdigest()[:16] == m["row_sha256_16"][y], (name, y)
    m = full["c4"]
    y = 620
    acc = np.zeros((1, m["size"][0], 4), np.uint8)
    pyoracle.accumulate_rgba8(0, acc, acc.copy())
    for k in m["frames"]:
        img = SceneCase("island", tuple(m["size"]), m["spp"], m["bounces"]).oracle(rng_offset=k, rows=(y, y + 1))[0]
        pyoracle.accumulate_rgba8(k, acc, np.ascontiguousarray(img[y:y + 1]))
    assert hashlib.sha256(acc[0].tobytes()).hexdigest()[:16] == m["row_sha256_16"][y]
    assert len(m["row_sha256_16"]) == m["size"][1] == 1080
