"""Multi-GPU frame sharding: one process per GPU, 16x16 tiles dealt
round-robin (tile t -> rank t mod N, t in raster tile order — the device's
yrtSetTileShard(rank, N)), and one collective per frame to bring the disjoint shards to
rank 0. The reference's multi-node analogue deals 4-row bands
(devices/device_network/api/swapchain.h:57-70)."""
from __future__ import annotations

import numpy as np

TILE = 16  # TILE_SIZE (renderers/renderer.h:34)


def tile_mask(width: int, height: int, rank: int, world: int) -> np.ndarray:
    """Pixels rendered by `rank` of `world`: bool (height, width)."""
    ntx = (width + TILE - 1) // TILE
    tile = np.arange(height)[:, None] // TILE * ntx + np.arange(width)[None, :] // TILE
    return (tile % world) == rank


def gather_frame(fb, dst: int = 0):
    """Combines per-rank framebuffers whose pixels outside the rank's tiles are zero (the
    device clears them when sharded) into the full frame on `dst`: a SUM reduce, exact
    because the supports are disjoint (x + 0 == x). `fb` is a torch tensor on the rank's
    device (CUDA -> RCCL over xGMI; CPU -> gloo)."""
    import torch.distributed as dist
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.reduce(fb, dst=dst, op=dist.ReduceOp.SUM)
    return fb
