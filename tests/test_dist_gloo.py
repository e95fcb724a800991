"""world_size-2 gloo rehearsal of the multi-GPU path on CPU: tile shards are
disjoint and complete; each rank renders only its tiles (the oracle's tile split, the same
partition yrtSetTileShard / yrtSetShardComm give the device) and gather_frame reassembles on
rank 0 a frame bit-identical to the one-process render — the per-tile Random seeds
(integratorrenderer.cpp:134) make the image partition-invariant."""
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


def _blob(W, H):
    import yrt
    from helpers import c2_args
    d = yrt.Device(host=True)
    s = yrt.Session(c2_args(W, 4) + ["-size", str(W), str(H), "-fb", "RGB_FLOAT32"], device=d)
    b = s.export_frame()
    s.close()
    d.close()
    return b


def _worker(rank, world, port, W, H, q):
    import oracle
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    img, st = oracle.render_shard(_blob(W, H), W, H, 1.0, rank, world, threads=2)
    mine = np.where(tile_mask(W, H, rank, world)[..., None], img, 0).astype(np.float32)
    assert not np.isnan(mine).any()
    t = torch.from_numpy(mine.copy())
    gather_frame(t, dst=0)
    rays = torch.tensor([st["raysClosest"] + st["raysShadow"]], dtype=torch.float64)
    dist.all_reduce(rays)
    if rank == 0:
        q.put((t.numpy(), float(rays.item())))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_tile_shards_render_and_gather(world):
    import oracle
    W, H = 88, 72
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, W, H, q)) for r in range(world)]
    for p in procs:
        p.start()
    frame, rays = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    full, st = oracle.render(_blob(W, H), W, H, 1.0)
    assert np.array_equal(frame, full)
    assert rays == st["raysClosest"] + st["raysShadow"]
