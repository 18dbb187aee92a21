"""Multi-GPU path logic on CPU: row-tile partition math, and the N>1 gather exercised with real
processes on the gloo backend (world_size 2 and 3).  Each rank renders ONLY its own global rows with
the oracle (standing in for its GPU) and the gathered, reassembled frame must equal the 1-rank frame
byte for byte (SURVEY.md 8(e) parity check)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from epq_raytracer_amd import rowtiles


@pytest.mark.parametrize("H,tile,parts", [(1080, 16, 1), (1080, 16, 2), (1080, 16, 8), (100, 16, 3), (7, 4, 4),
                                          (2160, 32, 8), (1, 16, 2)])
def test_partition_covers_every_row_once(H, tile, parts):
    n = rowtiles.local_rows(H, tile, parts)
    seen = np.zeros(H, int)
    for p in range(parts):
        g = rowtiles.global_rows(H, tile, parts, p)
        assert len(g) == n
        seen[g[g < H]] += 1
    assert np.all(seen == 1)
    src = rowtiles.assembly_index(H, tile, parts)
    stacked = np.concatenate([rowtiles.global_rows(H, tile, parts, p) for p in range(parts)])
    np.testing.assert_array_equal(stacked[src], np.arange(H))


def test_matches_native_layout():
    # epq_raytracer_amd.pipeline.HrtContext.global_rows uses the library's layout; same formula here
    for H, tile, parts in [(1080, 16, 8), (100, 16, 3)]:
        tiles = -(-H // tile)
        assert rowtiles.local_rows(H, tile, parts) == -(-tiles // parts) * tile


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, H, W, tile, out_dir):
    import sys
    import torch
    import torch.distributed as dist
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), os.path.join(os.path.dirname(here), "oracle"), here):
        sys.path.insert(0, p)
    from helpers import SceneCase
    from epq_raytracer_amd import rowtiles as rt

    os.environ["OMP_NUM_THREADS"] = "1"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    case = SceneCase("box", (W, H), num_samples=2, max_bounces=3)
    rows = rt.global_rows(H, tile, world, rank)
    local = np.zeros((len(rows), W, 4), np.uint8)
    for i, g in enumerate(rows):
        if g < H:
            img, _, _, _ = case.oracle(rows=(int(g), int(g) + 1), nthreads=1)
            local[i] = img[g]
    full = rt.gather_frame(torch.from_numpy(local), H, tile)
    if rank == 0:
        np.save(os.path.join(out_dir, "full.npy"), full.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_gather_reassembles_frame(tmp_path, world):
    H, W, tile = 37, 24, 4
    mp.spawn(_worker, args=(world, _free_port(), H, W, tile, str(tmp_path)), nprocs=world, join=True)
    from helpers import SceneCase
    ref, _, _, _ = SceneCase("box", (W, H), num_samples=2, max_bounces=3).oracle()
    got = np.load(tmp_path / "full.npy")
    np.testing.assert_array_equal(got, ref)
