"""GPU tests of the drop-in boundary added in round 2 (include/hip_raytrace.h):

* trace lanes (HRT_OPT_OVERLAP): the realtime loop's consecutive traces overlap; frames, accumulator
  and counters must equal the serial loop and hrt_compute_n byte for byte, with reads interleaved;
* the framebuffer gather behind hrt_read_image (hrt_comm_*): device-copy groups on one GPU (the
  un-interleave kernel against rowtiles.assembly_index), and RCCL communicators of one rank;
* libhip_raytrace_debug.so: guard bands around every device buffer after traces at ragged sizes,
  and a failed hrt_set_scene (injected allocation failure) leaving the previous scene intact;
* the production library rejecting the diagnostics-only options.
"""
import numpy as np
import pytest

import pyoracle
from helpers import E, SceneCase, _lib, mismatch_report
from epq_raytracer_amd import rowtiles

pytestmark = pytest.mark.gpu


def _loop(case, frames, first=1, overlap=3, variant=0, mode=_lib.MODE_RGBA8, read_each=False, partition=None,
          debug=False, busy_split=2):
    ctx = E.HrtContext(case.size, device=0, mode=mode, partition=partition, debug=debug)
    ctx.set_option(_lib.OPT_KERNEL_VARIANT, variant)
    ctx.set_option(_lib.OPT_OVERLAP, overlap)
    ctx.set_option(_lib.OPT_BUSY_SPLIT, busy_split)
    ctx.set_scene(case.rays, case.spheres, case.tris, case.meshes)
    fmt = _lib.FMT_RGBA8 if mode == _lib.MODE_RGBA8 else _lib.FMT_RGBA32F
    traces = []
    for k in range(first, first + frames):
        ctx.trace(case.push(k))
        if read_each:
            traces.append(ctx.read(_lib.IMG_TRACE, fmt))
        ctx.accumulate(k)
    st = ctx.stats()
    out = ctx.read(_lib.IMG_ACCUM, fmt), ctx.read(_lib.IMG_TRACE, fmt), st, traces
    return ctx, out


@pytest.mark.parametrize("scene,size,spp,variant,mode", [
    ("island", (96, 64), 3, 9, _lib.MODE_RGBA8),
    ("island", (256, 256), 1, 0, _lib.MODE_RGBA8),      # probe-planned first trace on each lane
    ("cave", (64, 48), 2, 7, _lib.MODE_RGBA32F),
    ("box", (45, 33), 3, 5, _lib.MODE_RGBA8),           # non-persistent kernel on the lanes
    ("island", (640, 360), 8, 0, _lib.MODE_RGBA8),      # traces long enough to overlap (busy split)
])
def test_overlapped_realtime_loop_is_byte_exact(scene, size, spp, variant, mode):
    """compute_then_render per frame (src/raytracing_app.rs:156-194) with the traces alternating
    between two lanes == the same loop on one lane == hrt_compute_n, byte for byte."""
    case = SceneCase(scene, size, spp, 8)
    n = 6
    results = []
    for overlap, busy in ((3, 2), (3, 1), (2, 3), (1, 2)):
        ctx, r = _loop(case, n, first=2, overlap=overlap, variant=variant, mode=mode, busy_split=busy)
        ctx.close()
        results.append(r)
    ctx = case.context(mode=mode, variant=variant)
    ctx.compute_n(case.push(2), n)
    fmt = _lib.FMT_RGBA8 if mode == _lib.MODE_RGBA8 else _lib.FMT_RGBA32F
    batched = ctx.read(_lib.IMG_ACCUM, fmt), ctx.read(_lib.IMG_TRACE, fmt), ctx.stats()
    ctx.close()
    for acc, trace, st, _ in results:
        assert np.array_equal(acc.view(np.uint8), batched[0].view(np.uint8))
        assert np.array_equal(trace.view(np.uint8), batched[1].view(np.uint8))
        assert (st.segments, st.tri_tests, st.traces, st.accumulates) == \
            (batched[2].segments, batched[2].tri_tests, batched[2].traces, batched[2].accumulates)


@pytest.mark.parametrize("mode", [_lib.MODE_RGBA8, _lib.MODE_RGBA32F])
def test_deferred_combines_equal_immediate_ones(mode):
    """HRT_OPT_DEFER_COMBINE: the realtime loop's combines recorded and folded
    in frame order later equal one combiner dispatch per hrt_accumulate, byte for byte -- across a
    ring wrap (40 frames > 16 slots), reads of both images in between (the accumulator read folds),
    a trace read before its accumulate, an accumulate of the same image twice, a trace that is never
    accumulated, hrt_compute_n and a checkpoint restore in the middle, and the counters."""
    case = SceneCase("island", (96, 64), 2, 8)
    fmt = _lib.FMT_RGBA8 if mode == _lib.MODE_RGBA8 else _lib.FMT_RGBA32F

    def run(defer):
        ctx = case.context(mode=mode)
        ctx.set_option(_lib.OPT_DEFER_COMBINE, defer)
        seen = []
        for k in range(1, 41):
            ctx.trace(case.push(k))
            if k % 7 == 0:
                seen.append(ctx.read(_lib.IMG_TRACE, fmt))
            ctx.accumulate(k)
            if k % 11 == 0:
                seen.append(ctx.read(_lib.IMG_ACCUM, fmt))
            if k == 13:
                ctx.accumulate(k + 100)  # the same trace image again
            if k == 17:
                ctx.trace(case.push(999))  # never accumulated: the next accumulate takes the next trace
        ctx.compute_n(case.push(41), 3)
        saved = ctx.read(_lib.IMG_ACCUM, fmt)
        for k in range(44, 50):
            ctx.trace(case.push(k))
            ctx.accumulate(k)
        ctx.load_accumulator(saved)
        for k in range(44, 47):
            ctx.trace(case.push(k))
            ctx.accumulate(k)
        st = ctx.stats()
        out = ctx.read(_lib.IMG_ACCUM, fmt), ctx.read(_lib.IMG_TRACE, fmt), seen
        ctx.close()
        return out, (st.segments, st.tri_tests, st.traces, st.accumulates)

    (acc0, tr0, seen0), st0 = run(0)
    (acc1, tr1, seen1), st1 = run(1)
    assert st0 == st1
    assert np.array_equal(acc0.view(np.uint8), acc1.view(np.uint8))
    assert np.array_equal(tr0.view(np.uint8), tr1.view(np.uint8))
    assert len(seen0) == len(seen1) and all(np.array_equal(a.view(np.uint8), b.view(np.uint8))
                                            for a, b in zip(seen0, seen1))


def test_overlapped_traces_read_back_in_order():
    """Every trace image read between overlapped traces is that frame's oracle frame."""
    case = SceneCase("island", (80, 48), 2, 8)
    ctx, (_, _, _, traces) = _loop(case, 5, first=1, overlap=3, read_each=True)
    ctx.close()
    for k, img in enumerate(traces, start=1):
        ref = case.oracle(rng_offset=k)[0]
        assert np.array_equal(img, ref), f"frame {k}: " + mismatch_report(img, ref)


def test_overlap_then_compute_n_then_overlap():
    """Lanes and hrt_compute_n interleaved on one context: the accumulator equals one serial loop."""
    case = SceneCase("island", (96, 64), 2, 8)
    ref_ctx, (want, want_trace, _, _) = _loop(case, 9, first=1, overlap=1)
    ref_ctx.close()
    ctx = case.context()
    for k in (1, 2):
        ctx.trace(case.push(k))
        ctx.accumulate(k)
    ctx.compute_n(case.push(3), 4)
    for k in (7, 8, 9):
        ctx.trace(case.push(k))
        ctx.accumulate(k)
    got, got_trace = ctx.read(_lib.IMG_ACCUM), ctx.read(_lib.IMG_TRACE)
    ctx.close()
    assert np.array_equal(got, want) and np.array_equal(got_trace, want_trace)


# ---- framebuffer gather (hrt_comm_*) -----------------------------------------------------------

@pytest.mark.parametrize("parts,tile", [(2, 8), (3, 16), (8, 8), (5, 4)])
def test_gather_device_copy_group(parts, tile):
    """hrt_comm_init_all over parts contexts sharing device 0 (HRT_COMM_DEVICE_COPY): hrt_read_image
    returns the full frame, equal to rowtiles.assembly_index over the parts' local rows, to the
    unpartitioned frame and (trace image) to the oracle; rgba32f reads convert the gathered frame."""
    case = SceneCase("island", (80, 70), 2, 8)
    ref = case.oracle(rng_offset=2)[0]
    full_ctx, (want_acc, want_trace, _, _) = _loop(case, 2, first=1)
    want_acc32 = full_ctx.read(_lib.IMG_ACCUM, _lib.FMT_RGBA32F)
    full_ctx.close()
    ctxs = []
    for p in range(parts):
        c, _ = _loop(case, 2, first=1, partition=(tile, p, parts))
        ctxs.append(c)
    local = [c.read(_lib.IMG_ACCUM) for c in ctxs]
    E.HrtContext.comm_init_all(ctxs)
    assert ctxs[1].comm_info() == (1, parts, _lib.COMM_DEVICE_COPY)
    host = np.concatenate(local)[rowtiles.assembly_index(70, tile, parts)]
    for c in (ctxs[0], ctxs[-1]):  # any member may read the group's frame
        got = c.read_frame(_lib.IMG_ACCUM)
        assert np.array_equal(got, host), mismatch_report(got, host)
        assert np.array_equal(got, want_acc)
    assert np.array_equal(ctxs[0].read_frame(_lib.IMG_TRACE), ref)
    assert np.array_equal(ctxs[0].read_frame(_lib.IMG_TRACE), want_trace)
    np.testing.assert_array_equal(ctxs[0].read_frame(_lib.IMG_ACCUM, _lib.FMT_RGBA32F).view(np.uint32),
                                  want_acc32.view(np.uint32))
    # the parts keep rendering after a gather (the members' streams wait for the copies)
    for c in ctxs:
        c.trace(case.push(3))
        c.accumulate(3)
    got3 = ctxs[0].read_frame(_lib.IMG_TRACE)
    assert np.array_equal(got3, case.oracle(rng_offset=3)[0])
    ctxs[1].close()
    with pytest.raises(_lib.HrtError, match="destroyed"):
        ctxs[0].read_frame(_lib.IMG_ACCUM)
    for c in ctxs:
        c.close()


def test_gather_rccl_single_rank():
    """The RCCL paths with one rank (all a one-GPU box can form): hrt_comm_init (ncclCommInitRank +
    ncclGather to rank 0) and hrt_comm_init_all (ncclCommInitAll + grouped ncclGather) return the
    frame the context holds."""
    case = SceneCase("box", (64, 48), 2, 4)
    for mode in ("rank", "all"):
        ctx, (want_acc, want_trace, _, _) = _loop(case, 3)
        if mode == "rank":
            ctx.comm_init(E.HrtContext.comm_unique_id(), 0, 1)
            assert ctx.comm_info() == (0, 1, _lib.COMM_RCCL)
        else:
            E.HrtContext.comm_init_all([ctx])
            assert ctx.comm_info() == (0, 1, _lib.COMM_RCCL_GROUP)
        assert np.array_equal(ctx.read_frame(_lib.IMG_ACCUM), want_acc)
        assert np.array_equal(ctx.read_frame(_lib.IMG_TRACE), want_trace)
        ctx.trace(case.push(4))  # a trace after the gather
        assert np.array_equal(ctx.read_frame(_lib.IMG_TRACE), case.oracle(rng_offset=4)[0])
        ctx.close()


def test_collective_read_errors_are_agreed_not_hung():
    """VERDICT r02 weak #5 / ADVICE r02: on a context joined with hrt_comm_init, a bad argument on rank 0
    (too small a destination, an unknown image or format) is agreed on by the ranks and returned --
    rank 0 no longer returns before the gather while its peers block in it (the multi-rank protocol:
    tests/test_comm_protocol.py).  The communicator stays usable after such an error; HRT_IMG_LOCAL
    (HrtContext.read, checkpoints) reads this rank's rows without a collective."""
    case = SceneCase("box", (64, 48), 2, 4)
    ctx, (want_acc, want_trace, _, _) = _loop(case, 3)
    ctx.set_option(_lib.OPT_COMM_TIMEOUT_MS, 20000)
    ctx.comm_init(E.HrtContext.comm_unique_id(), 0, 1)
    small = np.zeros(16, np.uint8)
    with pytest.raises(_lib.HrtError, match="INVALID"):
        ctx.read_into(_lib.IMG_ACCUM, _lib.FMT_RGBA8, small.ctypes.data, small.nbytes)
    with pytest.raises(_lib.HrtError, match="INVALID"):
        ctx.read_into(7, _lib.FMT_RGBA8, small.ctypes.data, small.nbytes)
    with pytest.raises(_lib.HrtError, match="INVALID"):
        ctx.read_into(_lib.IMG_ACCUM, 9, small.ctypes.data, small.nbytes)
    assert np.array_equal(ctx.read_frame(_lib.IMG_ACCUM), want_acc)  # not broken by the errors
    assert np.array_equal(ctx.read(_lib.IMG_ACCUM), want_acc)        # local rows, no collective
    assert np.array_equal(E.Image(ctx, _lib.IMG_TRACE).read(), want_trace)  # the presenter's frame (rank 0)
    with pytest.raises(_lib.HrtError, match="INVALID"):
        ctx.set_option(_lib.OPT_COMM_TIMEOUT_MS, -1)
    ctx.close()


def test_comm_arguments_validated():
    case = SceneCase("box", (32, 32), 1, 1)
    a = case.context(partition=(8, 0, 2))
    b = case.context(partition=(8, 1, 2))
    with pytest.raises(_lib.HrtError, match="INVALID"):
        E.HrtContext.comm_init_all([b, a])  # ctxs[i] must be part i
    a.set_option(_lib.OPT_COMM_TIMEOUT_MS, 3000)  # (it joins the init, which has no peer: bounded wait)
    with pytest.raises(_lib.HrtError, match="INVALID"):
        a.comm_init(bytes(_lib.COMM_ID_BYTES), 1, 2)  # rank differs from the partition
    assert a.comm_info() == (0, 1, _lib.COMM_NONE)  # no half-formed communicator
    full = case.context()
    with pytest.raises(_lib.HrtError, match="INVALID"):
        E.HrtContext.comm_init_all([full, b])
    E.HrtContext.comm_init_all([a, b])
    with pytest.raises(_lib.HrtError, match="INVALID"):
        E.HrtContext.comm_init_all([a, b])  # already in a group
    with pytest.raises(_lib.HrtError, match="INVALID"):  # the gathered frame is the full 32 x 32
        a.read_into(_lib.IMG_ACCUM, _lib.FMT_RGBA8, np.zeros(16 * 32 * 4, np.uint8).ctypes.data, 16 * 32 * 4)
    for c in (a, b, full):
        c.close()


# ---- libhip_raytrace_debug.so: guard bands, injected failures ---------------------------------

@pytest.mark.parametrize("scene,size,spp,partition", [
    ("box", (37, 23), 3, None), ("island", (300, 1), 2, None), ("island", (1, 130), 2, None),
    ("cave", (75, 41), 2, (8, 1, 3)), ("island", (129, 67), 2, (4, 2, 3)), ("spheres", (33, 65), 2, None),
])
def test_guard_bands_intact_after_traces(scene, size, spp, partition):
    """Every device buffer (trace / accumulate images of both lanes, frame stack, camera lists, BVH
    and band lists, planner buffers, counters, gather buffers) sits between 4 KiB guard bands in the
    debug library; after every variant, compute_n batches, overlapped loops and a gather at ragged
    sizes none of the bands has changed."""
    case = SceneCase(scene, size, spp, 8)
    ctx = E.HrtContext(size, device=0, partition=partition, debug=True)
    assert ctx.lib.hrt_debug_build() == 1
    ctx.set_option(_lib.OPT_COUNTERS, 2)  # tile profile buffer too
    ctx.set_scene(case.rays, case.spheres, case.tris, case.meshes)
    for v in range(10):
        ctx.set_option(_lib.OPT_KERNEL_VARIANT, v)
        ctx.trace(case.push(v + 1))
        ctx.accumulate(v + 1)
    ctx.set_option(_lib.OPT_COUNTERS, 1)
    ctx.set_option(_lib.OPT_KERNEL_VARIANT, 0)
    ctx.set_option(_lib.OPT_FRAMES_PER_LAUNCH, 3)
    ctx.compute_n(case.push(20), 7)
    for k in range(30, 34):
        ctx.trace(case.push(k))
        ctx.accumulate(k)
    if partition is None:
        ctx.comm_init(E.HrtContext.comm_unique_id(), 0, 1)
        ctx.read_frame(_lib.IMG_ACCUM, _lib.FMT_RGBA32F)
    n, bad = ctx.check_guards()
    ctx.close()
    assert n >= 20 and bad == 0, (n, bad)


def test_failed_set_scene_keeps_the_previous_scene():
    """a failure inside hrt_set_scene (here the k-th device allocation, injected through
    libhip_raytrace_debug.so) must not leave stale counts next to freed buffers: the call reports
    HRT_ERR_OUT_OF_MEMORY and the previous scene still traces byte for byte."""
    import ctypes
    box = SceneCase("box", (48, 40), 2, 4)
    island = SceneCase("island", (48, 40), 2, 8)
    ref = box.oracle()[0]
    island_ref = island.oracle()[0]
    ctx = E.HrtContext(box.size, device=0, debug=True)
    ctx.set_scene(box.rays, box.spheres, box.tris, box.meshes)
    k, records_fallback = 1, False
    while True:
        ctx.set_option(_lib.DEBUG_OPT_FAIL_ALLOC, k)
        try:
            ctx.set_scene(island.rays, island.spheres, island.tris, island.meshes)
        except _lib.HrtError as e:
            assert "OUT_OF_MEMORY" in str(e), e
            ctx.trace(box.push())
            assert np.array_equal(ctx.read(_lib.IMG_TRACE), ref), f"allocation {k}"
            k += 1
            continue
        info = (ctypes.c_uint32 * 4)()
        _lib.check(ctx.lib.hrt_debug_band_records(ctx.handle, None, 0, None, 0, None, 0, info), "records",
                   ctx.handle, ctx.lib)
        if info[0] and not info[3]:
            # the k-th allocation was the band records' (r06): the scene is set without them and the
            # band lookups read the offsets and lists -- the same frame
            records_fallback = True
            ctx.trace(island.push())
            assert np.array_equal(ctx.read(_lib.IMG_TRACE), island_ref), "without band records"
            ctx.set_option(_lib.DEBUG_OPT_FAIL_ALLOC, 0)
            ctx.set_scene(box.rays, box.spheres, box.tris, box.meshes)
            k += 1
            continue
        break  # fewer than k allocations: the injection did not fire, the scene is island now
    assert k > 10 and records_fallback  # rays, records, camera lists of both lanes, hierarchy, band lists ...
    ctx.trace(island.push())
    assert np.array_equal(ctx.read(_lib.IMG_TRACE), island.oracle()[0])
    n, bad = ctx.check_guards()
    assert bad == 0
    ctx.close()
    fresh = E.HrtContext(box.size, device=0, debug=True)
    fresh.set_option(_lib.DEBUG_OPT_FAIL_ALLOC, 3)
    with pytest.raises(_lib.HrtError, match="OUT_OF_MEMORY"):
        fresh.set_scene(box.rays, box.spheres, box.tris, box.meshes)
    with pytest.raises(_lib.HrtError, match="NO_SCENE"):
        fresh.trace(box.push())
    fresh.close()


def test_production_library_rejects_debug_options():
    case = SceneCase("box", (16, 16), 1, 1)
    ctx = case.context()
    assert ctx.lib.hrt_debug_build() == 0
    for key, value in ((_lib.OPT_PRIORITY, 2), (_lib.OPT_GRID_CUS, 4), (_lib.DEBUG_OPT_FAIL_ALLOC, 1),
                       (_lib.DEBUG_OPT_WQ_TRI_CAP, 128), (_lib.DEBUG_OPT_GRAB_RUNS, 1)):
        with pytest.raises(_lib.HrtError, match="INVALID"):
            ctx.set_option(key, value)
    ctx.set_option(_lib.OPT_PRIORITY, 0)
    with pytest.raises(_lib.HrtError, match="INVALID"):
        ctx.check_guards()
    for bad in (-1, 4):
        with pytest.raises(_lib.HrtError, match="INVALID"):
            ctx.set_option(_lib.OPT_OVERLAP, bad)
    for ok in (0, 1, 2, 3):
        ctx.set_option(_lib.OPT_OVERLAP, ok)
    for bad in (0, 9):
        with pytest.raises(_lib.HrtError, match="INVALID"):
            ctx.set_option(_lib.OPT_BUSY_SPLIT, bad)
    ctx.close()
    dbg = E.HrtContext((16, 16), device=0, debug=True)
    dbg.set_option(_lib.OPT_PRIORITY, 2)
    dbg.set_option(_lib.OPT_GRID_CUS, 4)
    dbg.close()


def test_fast_division_and_sqrt_match_ieee():
    """hrt_math.h's shared-reciprocal normalize / division and the unscaled sqrt are the compiler's
    IEEE instruction sequences minus identities in their range: bit-identical on 16M hashed inputs
    (a third with arbitrary bit patterns -- NaN, inf, denormals, zeros -- which take the IEEE path)."""
    lib = _lib.load()
    out = np.zeros(4, np.uint64)
    for seed in (1, 2, 3, 4):
        _lib.check(lib.hrt_debug_math_check(0, 1 << 22, seed, _lib.ptr(out)), "hrt_debug_math_check")
        assert out[0] == 0 and out[1] == 0 and out[2] == 0, out
        assert out[3] > (1 << 21), out  # most of the non-wide inputs took the fast path


def test_rng_domain_shortcuts_exhaustive():
    """sqrt_rng (the unscaled sqrt) on every u01 value and every -2 log(u01), and the unguarded sin/cos
    on both angle forms of raytracing.glsl, equal the general routines for all 2^32 RNG states; and
    adjust_dir's Lambertian shortcut premise holds for all of them (a normal_dist radius is finite and
    nonzero iff u01 is neither 0 nor 1; the angle's cosine is never 0)."""
    lib = _lib.load()
    out = np.zeros(5, np.uint64)
    _lib.check(lib.hrt_debug_math_check_rng(0, _lib.ptr(out)), "hrt_debug_math_check_rng")
    print("bare hardware sqrt mismatches (u01, -2 log u01):", int(out[3]), int(out[4]))
    assert out[0] == 0 and out[1] == 0 and out[2] == 0, out


def _band_flatten_expected(n, b0):
    """Slot g of the lanes' lists laid end to end: (owner lane, entry) -- the last lane with a
    non-empty list starting at or before g."""
    pos = np.concatenate(([0], np.cumsum(n)[:-1])).astype(np.int64)
    own, ent = [], []
    for g in range(int(n.sum())):
        lane = max(l for l in range(64) if n[l] and pos[l] <= g)
        own.append(lane)
        ent.append((int(b0[lane]) + g - int(pos[lane])) & 0xFFFFFFFF)
    return np.array(own, np.uint32), np.array(ent, np.uint32)


@pytest.mark.parametrize("case", ["sparse", "dense", "long", "empty_head", "one_lane", "all_empty", "random"])
def test_band_flatten_matches_host(case):
    """The trace kernel's flattening of a wave's grazing-band lists into 64-slot rounds (BandFlat): every
    slot's owner lane and entry equal the host's, for lists of every shape -- in particular slots where
    a list starts at the slot of a lane whose own list is empty (r03: a plain LDS load there let hipcc
    forward that lane's own clearing store, so those starts were lost and their entries went to the
    previous list's ray)."""
    rng = np.random.default_rng(11 + ["sparse", "dense", "long", "empty_head", "one_lane", "all_empty", "random"].index(case))
    n = np.zeros(64, np.uint32)
    if case == "sparse":      # a bounce batch: ~40% of the lanes without a list, short lists
        n[:] = np.where(rng.random(64) < 0.4, 0, rng.integers(1, 30, 64))
    elif case == "dense":
        n[:] = rng.integers(1, 5, 64)
    elif case == "long":      # lists spanning several rounds
        n[::7] = rng.integers(60, 200, len(n[::7]))
    elif case == "empty_head":
        n[20:] = rng.integers(0, 9, 44)
    elif case == "one_lane":
        n[63] = 150
    elif case == "random":
        n[:] = rng.integers(0, 40, 64) * (rng.random(64) < 0.6)
    b0 = rng.integers(0, 1 << 20, 64).astype(np.uint32)
    total_exp = int(n.sum())
    rounds = max(1, -(-total_exp // 64)) + 1  # one round past the end, as the kernel's pipeline fetches
    out = np.zeros(rounds * 128, np.uint32)
    total = np.zeros(1, np.uint32)
    lib = _lib.load()
    _lib.check(lib.hrt_debug_band_flatten(0, _lib.ptr(n), _lib.ptr(b0), rounds, _lib.ptr(out), _lib.ptr(total)),
               "hrt_debug_band_flatten")
    assert int(total[0]) == total_exp
    own, ent = _band_flatten_expected(n, b0)
    got = out.reshape(-1, 2)[:total_exp]
    bad = np.nonzero((got[:, 0] != own) | (got[:, 1] != ent))[0]
    assert bad.size == 0, f"{bad.size} of {total_exp} slots wrong, first {bad[:5]}: got {got[bad[:3]]}, want owner {own[bad[:3]]} entry {ent[bad[:3]]}"
    assert (out.reshape(-1, 2)[total_exp:, 1] == 0).all()  # slots past the end read entry 0


@pytest.mark.parametrize("overlap", [1, 3])
def test_camera_lists_follow_the_camera(overlap):
    """A lane rebuilds its camera lists (camera_lists) only when the camera position changed since its
    last trace: a camera path A, A, B, A, B, B (across 1 or 3 trace lanes, the first trace's planning
    probe included) gives each frame exactly the image of a fresh context traced from that position."""
    case = SceneCase("island", (96, 64), 2, 4)
    a = np.asarray(case.camera.position, np.float32)
    b = a + np.float32([0.7, 0.3, -0.4])

    def push(pos, k):
        pc = case.push(k)
        pc.cam_pos[:] = [float(pos[0]), float(pos[1]), float(pos[2]), 1.0]
        return pc

    def fresh(pos, k):
        ctx = case.context()
        ctx.trace(push(pos, k))
        img = ctx.read(_lib.IMG_TRACE, _lib.FMT_RGBA8)
        ctx.close()
        return img

    path = [a, a, b, a, b, b]
    ctx = case.context()
    ctx.set_option(_lib.OPT_OVERLAP, overlap)
    for k, pos in enumerate(path, start=1):
        ctx.trace(push(pos, k))
        got = ctx.read(_lib.IMG_TRACE, _lib.FMT_RGBA8)
        want = fresh(pos, k)
        assert np.array_equal(got, want), f"frame {k}: {mismatch_report(got, want)}"
    ctx.close()


@pytest.mark.parametrize("overlap,split", [(1, 1), (3, 1), (1, 0)])
def test_tile_lists_follow_camera_jitter_and_rays(overlap, split):
    """The persistent kernels' tile lists (tile_lists, built once and kept while the camera stays): a path
    through direction-only changes (the view matrix), a jitter change, back to the first camera, and a
    re-generated ray buffer (hrt_generate_rays with another focal length) gives each trace exactly the
    image of a fresh context with that camera and those rays.  1080p-sized tile counts are not needed:
    96x72 tiles run the same kernels (the probe is off below 1,024 tiles); a long focal length keeps each
    tile's ray cone as narrow as a 1080p tile's, so that its list fits (kTileCapVgpr) and is used -- at the
    preset's focal length the 96x72 tiles' lists overflow and every tile takes the list-free path.  The
    kept lists serve whole-tile items only: with 108 tiles against 4,096 resident waves the planner splits
    every tile from the second trace on (HRT_OPT_SPLIT auto), so split = 1 keeps the tiles whole."""
    case = SceneCase("island", (96, 72), 2, 4)
    s = case.settings

    def push(k, direction=None, jitter=None):
        pc = case.push(k)
        if direction is not None:
            pc.cam_alignment_mat[:] = [float(v) for v in E.view_matrix(direction, case.camera.up)]
        if jitter is not None:
            pc.jitter_size = jitter
        return pc

    # (changes large enough that a list kept from the previous camera misses triangles: a kept list that
    # is a superset of the right one gives the right image, so small moves would not test the key --
    # tools/exp/r05_tile_list_key_mutant.patch must fail here)
    d0 = np.asarray(case.camera.direction, np.float32)
    c, sn = np.float32(np.cos(0.5)), np.float32(np.sin(0.5))
    d1 = np.float32([c * d0[0] + sn * d0[2], d0[1], -sn * d0[0] + c * d0[2]])   # yaw +0.5 rad
    d2 = np.float32([c * d0[0] - sn * d0[2], d0[1] * 0.6, sn * d0[0] + c * d0[2]])  # yaw -0.5 rad, tilt up
    path = [(1, d2, None), (2, d1, None), (3, d2, None), (4, d2, case.jitter * 8.0), (5, None, None),
            (6, None, None)]

    def fresh(pc, focal):
        ctx = E.HrtContext(case.size, device=0)
        ctx.generate_rays(focal, s.viewport_height, s.up)
        ctx.set_scene(None, case.spheres, case.tris, case.meshes)
        ctx.trace(pc)
        img = ctx.read(_lib.IMG_TRACE, _lib.FMT_RGBA8)
        ctx.close()
        return img

    ctx = E.HrtContext(case.size, device=0)
    ctx.set_option(_lib.OPT_OVERLAP, overlap)
    ctx.set_option(_lib.OPT_SPLIT, split)
    focal = s.camera_focal_length * 12.0
    ctx.generate_rays(focal, s.viewport_height, s.up)
    ctx.set_scene(None, case.spheres, case.tris, case.meshes)
    for k, direction, jitter in path:
        pc = push(k, direction, jitter)
        ctx.trace(pc)
        got = ctx.read(_lib.IMG_TRACE, _lib.FMT_RGBA8)
        want = fresh(pc, focal)
        assert np.array_equal(got, want), f"frame {k}: {mismatch_report(got, want)}"
    # new ray centres from the same camera: the lists must follow the rays (the camera key is unchanged)
    # (no hrt_set_scene in between: hrt_generate_rays alone must drop the lists built from the old rays)
    focal2 = focal * 0.5  # a wider view: the old lists miss the new edge pixels' triangles
    ctx.generate_rays(focal2, s.viewport_height, s.up)
    pc = push(7)
    ctx.trace(pc)
    got = ctx.read(_lib.IMG_TRACE, _lib.FMT_RGBA8)
    want = fresh(pc, focal2)
    ctx.close()
    assert np.array_equal(got, want), f"regenerated rays: {mismatch_report(got, want)}"


@pytest.mark.parametrize("overlap", [1, 3])
def test_probe_built_tile_lists_follow_the_camera(overlap):
    """at 1,024 tiles or more the first trace of each lane is planned from a 1-sample probe,
    which also builds the tile lists, and the main launch then skips its own list prepass.  256 x 256 (32 x
    32 tiles) with overlap 3 probes on each of the first three traces, at alternating cameras; every
    trace must equal a fresh context's with the probe off (lists built by the trace itself)."""
    case = SceneCase("island", (256, 256), 2, 4)
    s = case.settings
    d0 = np.asarray(case.camera.direction, np.float32)
    c, sn = np.float32(np.cos(0.5)), np.float32(np.sin(0.5))
    d1 = np.float32([c * d0[0] + sn * d0[2], d0[1], -sn * d0[0] + c * d0[2]])
    d2 = np.float32([c * d0[0] - sn * d0[2], d0[1] * 0.6, sn * d0[0] + c * d0[2]])
    focal = s.camera_focal_length * 12.0

    def push(k, direction):
        pc = case.push(k)
        pc.cam_alignment_mat[:] = [float(v) for v in E.view_matrix(direction, case.camera.up)]
        return pc

    def context(probe):
        ctx = E.HrtContext(case.size, device=0)
        ctx.set_option(_lib.OPT_PROBE, probe)
        ctx.set_option(_lib.OPT_OVERLAP, overlap)
        ctx.set_option(_lib.OPT_SPLIT, 1)
        ctx.generate_rays(focal, s.viewport_height, s.up)
        ctx.set_scene(None, case.spheres, case.tris, case.meshes)
        return ctx

    ctx = context(1)
    for k, direction in enumerate([d2, d1, d2, d1, d0], start=1):
        pc = push(k, direction)
        ctx.trace(pc)
        got = ctx.read(_lib.IMG_TRACE, _lib.FMT_RGBA8)
        ref = context(0)
        ref.trace(pc)
        want = ref.read(_lib.IMG_TRACE, _lib.FMT_RGBA8)
        ref.close()
        assert np.array_equal(got, want), f"frame {k}: {mismatch_report(got, want)}"
    ctx.close()


def test_camera_lists_after_a_variant_switch():
    """A kernel that neither builds nor reads the camera lists (LITERAL, BRUTE) leaves the lane's lists as
    they were: BUNDLE_WQ from position B, then LITERAL from A, then BUNDLE_WQ from A on the same lane must
    rebuild A's lists (the lane was marked as holding A's lists after the LITERAL trace, and
    the last trace read B's), giving the image of a fresh context at A."""
    case = SceneCase("island", (96, 64), 2, 4)
    a = np.asarray(case.camera.position, np.float32)
    b = a + np.float32([0.7, 0.3, -0.4])

    def push(pos, k):
        pc = case.push(k)
        pc.cam_pos[:] = [float(pos[0]), float(pos[1]), float(pos[2]), 1.0]
        return pc

    fresh = case.context(variant=_lib.KERNEL_BUNDLE_WQ)
    fresh.trace(push(a, 3))
    want = fresh.read(_lib.IMG_TRACE, _lib.FMT_RGBA8)
    fresh.close()
    ctx = case.context()
    ctx.set_option(_lib.OPT_OVERLAP, 1)
    for variant, pos, k in ((_lib.KERNEL_BUNDLE_WQ, b, 1), (_lib.KERNEL_LITERAL, a, 2), (_lib.KERNEL_BRUTE, a, 2),
                            (_lib.KERNEL_BUNDLE_WQ, a, 3)):
        ctx.set_option(_lib.OPT_KERNEL_VARIANT, variant)
        ctx.trace(push(pos, k))
    got = ctx.read(_lib.IMG_TRACE, _lib.FMT_RGBA8)
    ctx.close()
    assert np.array_equal(got, want), mismatch_report(got, want)


def _wq_protocol_model(cnt, take, tgt, val, seed):
    """Host model of hrt_debug_wq_protocol: a LIFO stack and u64 minimum slots, round by round."""
    rounds = len(take)
    stack, slots = [], [int(v) for v in seed]
    popped = np.full((rounds, 64), 0xFFFFFFFF, np.uint64)
    lo = np.zeros((rounds, 64), np.uint64)   # seen[r][l] must be <= the slot before round r's lowerings
    hi = np.zeros((rounds, 64), np.uint64)   # ... and >= the slot after them
    for r in range(rounds):
        tk = min(int(take[r]), len(stack))
        top = stack[len(stack) - tk:]
        del stack[len(stack) - tk:]
        popped[r, :tk] = top
        before = list(slots)
        for lane in range(64):
            t = int(tgt[r, lane])
            if t < 64:
                slots[t] = min(slots[t], int(val[r, lane]))
        for lane in range(64):
            t = int(tgt[r, lane])
            if t < 64:
                lo[r, lane], hi[r, lane] = slots[t], before[t]
        for k in range(4):
            room = len(stack) + 256 <= 8192  # wave-uniform, before the k-th pushes
            for lane in range(64):
                if cnt[r, lane] > k and room:
                    stack.append((r << 16) | (lane << 8) | k)
    return popped, lo, hi, np.array(slots, np.uint64), len(stack)


@pytest.mark.parametrize("case", ["balanced", "deep", "drain", "sparse_slots", "random"])
def test_wq_handoff_protocol_matches_host(case):
    """The pair traversal's cross-lane LDS handoffs (wq_push and the pops of the node / triangle stacks, the
    closest-hit slots' seed / read / lowering / final read, each ordered by wave_handoff) on scripted
    rounds of one wave: every popped entry, every slot read and the final slots equal a host model of a
    LIFO stack and u64 minimum slots (one such handoff produced wrong frames)."""
    seed_ = 100 + ["balanced", "deep", "drain", "sparse_slots", "random"].index(case)
    rng = np.random.default_rng(seed_)
    rounds = 96
    cnt = rng.integers(0, 5, (rounds, 64)).astype(np.uint32)
    take = rng.integers(0, 65, rounds).astype(np.uint32)
    if case == "deep":
        take[:] = rng.integers(0, 40, rounds)
    elif case == "drain":
        cnt[rounds // 2:] = 0
        take[rounds // 2:] = 64
    elif case == "random":
        cnt[rng.random((rounds, 64)) < 0.5] = 0
    tgt = rng.integers(0, 64, (rounds, 64)).astype(np.uint32)
    tgt[rng.random((rounds, 64)) < (0.8 if case == "sparse_slots" else 0.3)] = 64  # no slot access
    val = rng.integers(0, 1 << 62, (rounds, 64), dtype=np.uint64)
    seed = rng.integers(1 << 61, 1 << 63, 64, dtype=np.uint64)
    popped = np.zeros((rounds, 64), np.uint32)
    seen = np.zeros((rounds, 64), np.uint64)
    slots = np.zeros(64, np.uint64)
    depth = np.zeros(1, np.uint32)
    lib = _lib.load()
    _lib.check(lib.hrt_debug_wq_protocol(0, rounds, _lib.ptr(cnt), _lib.ptr(take), _lib.ptr(tgt), _lib.ptr(val),
                                         _lib.ptr(seed), _lib.ptr(popped), _lib.ptr(seen), _lib.ptr(slots),
                                         _lib.ptr(depth)), "hrt_debug_wq_protocol")
    want_pop, lo, hi, want_slots, want_depth = _wq_protocol_model(cnt, take, tgt, val, seed)
    assert int(depth[0]) == want_depth
    bad = np.argwhere(popped.astype(np.uint64) != want_pop)
    assert bad.size == 0, f"{len(bad)} popped entries differ, first (round, lane) {bad[:3].tolist()}"
    m = tgt < 64
    assert (seen[m] <= hi[m]).all(), "a slot read missed an earlier round's lowering"
    assert (seen[m] >= lo[m]).all(), "a slot read below the slot's value after its round"
    assert np.array_equal(slots, want_slots)


@pytest.mark.parametrize("scene", ["island", "cave"])
def test_band_records_match_the_lists(scene):
    """The per-cell band records BUNDLE_WQ reads (r06: one 32 B record per direction cell, built on the
    device by band_records from the uploaded offsets and 16-bit lists): for every cell, the list's start
    and length, its first 12 entries as half-words in order, and zeros past them.  Both scenes have cells
    with more than 12 entries (the lanes then read the rest from the list)."""
    import ctypes
    case = SceneCase(scene, (16, 16), 1, 2)
    ctx = case.context()
    lib = ctx.lib
    info = (ctypes.c_uint32 * 4)()
    _lib.check(lib.hrt_debug_band_records(ctx.handle, None, 0, None, 0, None, 0, info), "band records", ctx.handle, lib)
    cells, entries, wide, has_rec = list(info)
    assert cells == 6 * 1024 * 1024 and entries > 0 and wide == 0 and has_rec == 1
    rec = np.zeros(cells * 8, np.uint32)
    off = np.zeros(cells + 1, np.uint32)
    words = np.zeros((entries + 1) // 2, np.uint32)
    P = ctypes.c_void_p
    _lib.check(lib.hrt_debug_band_records(ctx.handle, P(rec.ctypes.data), rec.size, P(off.ctypes.data), off.size,
                                          P(words.ctypes.data), words.size, info), "band records", ctx.handle, lib)
    ctx.close()
    lst = words.view(np.uint16)[:entries].astype(np.uint32)
    rec = rec.reshape(cells, 8)
    n = np.diff(off.astype(np.int64))
    assert int(off[-1]) == entries and (n >= 0).all()
    assert np.array_equal(rec[:, 0], off[:-1]) and np.array_equal(rec[:, 1].astype(np.int64), n)
    assert (n > 12).any(), "no cell overflows its record: the list path is not exercised"
    half = rec[:, 2:].copy().view(np.uint16).reshape(cells, 12).astype(np.int64)
    for j in range(12):
        has = n > j
        idx = off[:-1].astype(np.int64) + j
        want = np.where(has, lst[np.minimum(idx, entries - 1)], 0)
        assert np.array_equal(half[:, j], want), f"entry {j}"


def test_tile_costs_cover_every_tile_of_the_last_launch():
    """hrt_debug_tile_costs (the planner's input, read by tools/timeline.py --costs): after a multi-frame
    persistent launch every 8x8 tile of the frame carries a cost (shader clocks / 16 summed over the
    launch's frames), and nothing is written past the frame's tiles."""
    import ctypes
    W, H = 64, 48
    tiles = (W // 8) * (H // 8)
    case = SceneCase("island", (W, H), 2, 3)
    ctx = case.context()
    ctx.trace(case.push(init=True))
    ctx.accumulate(0)
    ctx.compute_n(case.push(1), 4)
    assert ctx.stats().last_kernel == _lib.KERNEL_BUNDLE_WQ, "the persistent BUNDLE_WQ kernel records tile costs"
    costs = np.zeros(tiles + 16, np.uint32)
    _lib.check(ctx.lib.hrt_debug_tile_costs(ctx.handle, ctypes.c_void_p(costs.ctypes.data), costs.size),
               "tile costs", ctx.handle, ctx.lib)
    ctx.close()
    assert (costs[:tiles] > 0).all(), costs[:tiles]
    assert (costs[tiles:] == 0).all()


@pytest.mark.parametrize("scene", ["cave", "island"])
def test_band_lookups_agree_between_records_and_offsets(scene):
    """BUNDLE_WQ finds a bounce lane's band list through its cell record, BUNDLE_BVH through the offsets:
    the same bounce segments (the frames are byte-identical) must see the same list lengths, summed over
    every bounce lane of the frame (HRT_DIAG_BAND_SCAN_LEN).  r06: a build that cut lists at the record's
    12 entries passed every frame test -- a band entry decides a hit only in rounding-noise cases -- so
    the lookup is held here directly."""
    case = SceneCase(scene, (96, 64), 4, 8)
    sums = {}
    for variant in (6, 9):  # BUNDLE_BVH, BUNDLE_WQ
        ctx = case.context(variant=variant)
        ctx.set_option(_lib.OPT_COUNTERS, 2)
        ctx.trace(case.push(3))
        sums[variant] = ctx.diagnostics()["band_scan_len"]
        assert ctx.stats().last_kernel == variant
        ctx.close()
    assert sums[9] == sums[6] > 0, sums
