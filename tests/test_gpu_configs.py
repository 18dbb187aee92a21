"""BASELINE.json configs C3, C4 and C5 at their full sizes on the GPU.

The frame loop is the reference's progressive loop (src/raytracing_app.rs:196-227: trace with
rng_offset = k, combine with weight k).  Each config is checked three ways: against the CPU oracle on
rows / pixels it finishes in seconds, against the literal kernel or the per-frame loop at full size,
and through the exact segment / triangle-test counters.
"""
import numpy as np
import pytest

import pyoracle
from helpers import E, SceneCase, _lib, assert_frame_digest, golden_full, mismatch_report
from epq_raytracer_amd import rowtiles

pytestmark = pytest.mark.gpu


def _oracle_accumulate(case, xs, ys, frames, first=1):
    """The oracle's rgba8 accumulator at pixels (xs, ys) after frames traced from rng_offset first."""
    acc = np.zeros((len(xs), 1, 4), np.uint8)
    acc[..., 3] = 255
    segs = 0
    for k in range(first, first + frames):
        px, s, _ = pyoracle.trace_pixels(case.push(k), case.rays, case.spheres, case.tris, case.meshes, xs, ys)
        pyoracle.accumulate_rgba8(k, acc, px.reshape(-1, 1, 4))
        segs += s
    return acc.reshape(-1, 4), segs


# ---- C3: Cave.obj 1920x1080, 64 spp, 8 bounces, one GPU ----------------------------------------

@pytest.fixture(scope="module")
def cave_frame():
    case = SceneCase("cave", (1920, 1080), 64, 8, rng_offset=1)
    ctx = case.context()
    ctx.trace(case.push(1))
    auto = ctx.read(_lib.IMG_TRACE), ctx.stats()
    ctx.set_option(_lib.OPT_KERNEL_VARIANT, _lib.KERNEL_LITERAL)
    ctx.reset_stats()
    ctx.trace(case.push(1))
    literal = ctx.read(_lib.IMG_TRACE), ctx.stats()
    ctx.close()
    return case, auto, literal


def test_c3_cave_rows_match_oracle(cave_frame):
    case, (img, _), _ = cave_frame
    for y in np.linspace(0, 1079, 9).astype(int):
        ref = case.oracle(rows=(int(y), int(y) + 1))[0]
        assert np.array_equal(img[y], ref[y]), f"row {y}: " + mismatch_report(img[y:y + 1], ref[y:y + 1])


def test_c3_cave_whole_frame_matches_oracle(cave_frame):
    """The whole C3 frame against the oracle's digest and exact counters (make_golden_full.py)."""
    _, (img, st), _ = cave_frame
    rec = golden_full("c3")
    assert (st.segments, st.tri_tests) == (rec["segments"], rec["tri_tests"])
    assert_frame_digest(img, rec, "C3 cave")


def test_c3_cave_full_frame_matches_literal_kernel(cave_frame):
    _, (img, st), (lit, lst) = cave_frame
    assert np.array_equal(img, lit), mismatch_report(img, lit)
    assert (st.segments, st.tri_tests) == (lst.segments, lst.tri_tests)
    assert st.last_kernel != lst.last_kernel == _lib.KERNEL_LITERAL
    n = 1920 * 1080 * 64
    assert n <= st.segments <= 9 * n and st.tri_tests <= st.segments * 2580


# ---- C4: island 1920x1080, 64 spp x 4 frames, 8-way row tiles + gather -------------------------

def test_c4_island_eight_row_tile_parts_gathered():
    """8 row-tile partitions (8-row tiles, the bench's N = 8 layout) of hrt_compute_n(4 frames),
    rendered on the one GPU, then gathered through hrt_read_image (hrt_comm_init_all's device-copy
    transport; RCCL on 8 distinct GPUs): the gathered accumulator equals the unpartitioned one and
    the oracle's 4-frame accumulation on sampled rows; the parts' counters sum to the whole frame's."""
    case = SceneCase("island", (1920, 1080), 64, 8)
    whole = case.context()
    whole.compute_n(case.push(1), 4)
    want, wst = whole.read(_lib.IMG_ACCUM), whole.stats()
    whole.close()
    parts = []
    segs = tests = 0
    for p in range(8):
        c = case.context(partition=(8, p, 8))
        c.compute_n(case.push(1), 4)
        s = c.stats()
        segs, tests = segs + s.segments, tests + s.tri_tests
        parts.append(c)
    local = np.concatenate([c.read(_lib.IMG_ACCUM) for c in parts])
    E.HrtContext.comm_init_all(parts)
    got = parts[0].read_frame(_lib.IMG_ACCUM)
    for c in parts:
        c.close()
    assert (segs, tests) == (wst.segments, wst.tri_tests)
    assert np.array_equal(local[rowtiles.assembly_index(1080, 8, 8)], want)
    assert np.array_equal(got, want), mismatch_report(got, want)
    # the whole gathered 4-frame accumulator against the oracle's (clear, trace k + combine(k), k = 1..4)
    rec = golden_full("c4")
    assert (segs, tests) == (rec["segments"], rec["tri_tests"])
    assert_frame_digest(got, rec, "C4 accumulator")
    rng = np.random.default_rng(4)
    ys = np.repeat([5, 400, 560, 700, 1070], 48)
    xs = rng.integers(0, 1920, len(ys))
    acc, _ = _oracle_accumulate(case, xs, ys, 4)
    assert np.array_equal(got[ys, xs], acc), mismatch_report(got[ys, xs][None], acc[None])


# ---- C5: island 3840x2160, 16 spp x 64 frames, 12 bounces --------------------------------------

def test_c5_island_4k_64_progressive_frames():
    """hrt_compute_n over 64 frames (launches of up to 32 frames: the 1 GiB frame-stack cap at 4K)
    equals the per-frame hrt_trace / hrt_accumulate loop (two overlapping trace lanes) at full size,
    and the oracle's 64-frame accumulation at 256 spread pixels."""
    case = SceneCase("island", (3840, 2160), 16, 12)
    batched = case.context()
    batched.compute_n(case.push(1), 64)
    got, gst = batched.read(_lib.IMG_ACCUM), batched.stats()
    got_trace = batched.read(_lib.IMG_TRACE)
    batched.close()
    loop = case.context()
    for k in range(1, 65):
        loop.trace(case.push(k))
        loop.accumulate(k)
    want, wst = loop.read(_lib.IMG_ACCUM), loop.stats()
    want_trace = loop.read(_lib.IMG_TRACE)
    loop.close()
    assert np.array_equal(got, want), mismatch_report(got, want)
    assert np.array_equal(got_trace, want_trace)
    assert (gst.segments, gst.tri_tests, gst.traces, gst.accumulates) == \
        (wst.segments, wst.tri_tests, wst.traces, wst.accumulates) and gst.traces == 64
    ys, xs = np.meshgrid(np.linspace(3, 2156, 16).astype(int), np.linspace(7, 3832, 16).astype(int), indexing="ij")
    ys, xs = ys.ravel(), xs.ravel()
    acc, _ = _oracle_accumulate(case, xs, ys, 64)
    assert np.array_equal(got[ys, xs], acc), mismatch_report(got[ys, xs][None], acc[None])
    assert got[..., :3].any() and (got[..., 3] == 255).all()
