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
