"""Checkpoint / resume of a progressive render ("dump the accumulator plus frame index;
resume = reload + continue with rng_offset = frame; deterministic seeding makes resume exact").
hrt_load_accumulator restores the bytes hrt_read_image returned; RayTracingApp.checkpoint / resume
carry them and the frame counter.  A resumed render must equal the uninterrupted one byte for byte."""
import numpy as np
import pytest

import epq_raytracer_amd as E
from epq_raytracer_amd import _lib

pytestmark = pytest.mark.gpu


def render(scene, size, mode, partition, first, second, tmp_path, resume):
    """first frames, then (optionally through a checkpoint and a new app) second more frames."""
    kw = dict(device=0, mode=mode, partition=partition)
    app = E.make_app(scene, num_samples=2, max_bounces=4, **kw)
    app.open(size)
    E.compute_n_then_render(app, first)
    if resume:
        path = str(tmp_path / "ckpt.npz")
        app.checkpoint(path)
        app.close()
        app = E.make_app(scene, num_samples=2, max_bounces=4, **kw)
        app.open(size)
        app.resume(path)
    for _ in range(second):  # the realtime loop after the restart
        E.compute_then_render(app)
    fmt = _lib.FMT_RGBA8 if mode == _lib.MODE_RGBA8 else _lib.FMT_RGBA32F
    out = app.context.read(_lib.IMG_ACCUM, fmt), app.frame
    app.close()
    return out


@pytest.mark.parametrize("scene,mode,partition", [("box", _lib.MODE_RGBA8, None), ("island", _lib.MODE_RGBA8, None),
                                                  ("box", _lib.MODE_RGBA32F, None), ("island", _lib.MODE_RGBA8, (8, 1, 3))])
def test_resume_equals_uninterrupted(tmp_path, scene, mode, partition):
    size = (160, 96)
    ref, fr_ref = render(scene, size, mode, partition, 2, 3, tmp_path, resume=False)
    got, fr_got = render(scene, size, mode, partition, 2, 3, tmp_path, resume=True)
    assert fr_got == fr_ref == 6
    assert np.array_equal(got, ref)


def test_load_accumulator_validation(tmp_path):
    app = E.make_app("box", num_samples=1, max_bounces=1, device=0)
    app.open((32, 24))
    ctx = app.context
    acc = ctx.read(_lib.IMG_ACCUM)
    with pytest.raises(_lib.HrtError):  # wrong size
        ctx.load_accumulator(acc[:-1])
    with pytest.raises(_lib.HrtError):  # another format than the context's (no conversion)
        ctx._check(ctx.lib.hrt_load_accumulator(ctx.handle, _lib.FMT_RGBA32F, _lib.ptr(acc), acc.nbytes), "x")
    E.compute_n_then_render(app, 2)
    path = str(tmp_path / "c.npz")
    app.checkpoint(path)
    app.close()
    other = E.make_app("box", num_samples=1, max_bounces=1, device=0)
    other.open((32, 16))
    with pytest.raises(ValueError):  # checkpoint of another image size
        other.resume(path)
    other.close()


def test_checkpoint_on_a_context_with_a_communicator(tmp_path):
    """RayTracingApp.checkpoint reads the local rows (HRT_IMG_LOCAL), never the collective
    gather, so a rank joined to a communicator saves its own partition's accumulator -- the same bytes
    as without the communicator -- and resumes from it."""
    size = (160, 96)
    ref, _ = render("island", size, _lib.MODE_RGBA8, None, 2, 3, tmp_path, resume=False)
    app = E.make_app("island", num_samples=2, max_bounces=4, device=0)
    app.open(size)
    app.context.comm_init(E.HrtContext.comm_unique_id(), 0, 1)
    E.compute_n_then_render(app, 2)
    path = str(tmp_path / "comm_ckpt.npz")
    app.checkpoint(path)
    app.close()
    app = E.make_app("island", num_samples=2, max_bounces=4, device=0)
    app.open(size)
    app.resume(path)
    for _ in range(3):
        E.compute_then_render(app)
    got = app.context.read(_lib.IMG_ACCUM)
    app.close()
    assert np.array_equal(got, ref)
