"""Image-space data parallelism: interleaved row tiles across ranks + one gather.

Each pixel depends only on (scene, camera, rng_offset, global pixel id) (assets/raytracing.glsl:376-385),
so ranks render disjoint row tiles with no exchange at all; the only collective is the final
gather of the accumulated framebuffer.  Tile t (``row_tile`` rows) belongs to rank t % world.
Every rank stores the same number of local rows (padded), so the gather is one equal-size
``all_gather_into_tensor`` (RCCL over xGMI on the GPU box; gloo in the CPU tests).
"""
from __future__ import annotations

import numpy as np


def local_rows(height: int, row_tile: int, parts: int) -> int:
    """Rows every part stores (== hrt_layout.local_rows)."""
    if parts <= 1:
        return height
    tiles = -(-height // row_tile)
    return -(-tiles // parts) * row_tile


def global_rows(height: int, row_tile: int, parts: int, part: int) -> np.ndarray:
    """Global row of each local row of ``part`` (values >= height are padding)."""
    n = local_rows(height, row_tile, parts)
    lr = np.arange(n, dtype=np.int64)
    if parts <= 1:
        return lr
    return ((lr // row_tile) * parts + part) * row_tile + lr % row_tile


def assembly_index(height: int, row_tile: int, parts: int) -> np.ndarray:
    """For the rank-major concatenation of all parts' local rows, the source row of every global
    row 0..height-1 (so ``full = gathered[assembly_index]``)."""
    n = local_rows(height, row_tile, parts)
    src = np.empty(height, dtype=np.int64)
    for p in range(max(parts, 1)):
        g = global_rows(height, row_tile, parts, p)
        keep = g < height
        src[g[keep]] = p * n + np.nonzero(keep)[0]
    return src


def gather_frame(local, height: int, row_tile: int, group=None):
    """All-gather every rank's local rows (torch tensor, shape (local_rows, W, C)) and reassemble the
    full (height, W, C) frame on every rank.  Works with any torch.distributed backend."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    if world == 1:
        return local[:height]
    out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, local.contiguous(), group=group)
    idx = torch.as_tensor(assembly_index(height, row_tile, world), device=local.device)
    return out.index_select(0, idx)
