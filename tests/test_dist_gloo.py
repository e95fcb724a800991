"""world_size-2 gloo rehearsal of the multi-GPU path on CPU: tile shards are
disjoint and complete, and gather_frame reassembles the frame exactly on rank 0."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from yrt.dist import gather_frame, tile_mask


@pytest.mark.parametrize("world", [2, 3, 8])
def test_tile_masks_partition_frame(world):
    W, H = 200, 136
    masks = [tile_mask(W, H, r, world) for r in range(world)]
    cover = np.sum(masks, axis=0)
    assert (cover == 1).all()
    # round-robin balance: tile counts differ by at most one
    ntiles = [int(m[::16, ::16].sum()) for m in masks]
    assert max(ntiles) - min(ntiles) <= 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, W, H, q):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    rng = np.random.default_rng(7)
    full = rng.random((H, W, 3), dtype=np.float32)
    mine = np.where(tile_mask(W, H, rank, world)[..., None], full, 0).astype(np.float32)
    t = torch.from_numpy(mine.copy())
    gather_frame(t, dst=0)
    if rank == 0:
        q.put(bool(np.array_equal(t.numpy(), full)))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_gather_frame_world2():
    W, H = 96, 80
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, W, H, q)) for r in range(2)]
    for p in procs:
        p.start()
    ok = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    assert ok
    assert all(p.exitcode == 0 for p in procs)
