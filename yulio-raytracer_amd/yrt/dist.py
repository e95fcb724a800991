"""Multi-GPU frame sharding: one process per GPU, 16x16 tiles dealt
round-robin (logical tile t -> rank t mod N — the device's yrtSetTileShard(rank, N)); logical
tile t of a frame covers image tile yrt_tile_scatter(t, T) (common/yrt_tile_scatter.h, a fixed
bijection that spreads every rank's tiles over the image), and one collective per frame brings
the disjoint shards to rank 0. The reference's multi-node analogue deals 4-row bands
(devices/device_network/api/swapchain.h:57-70)."""
from __future__ import annotations

from functools import lru_cache

import numpy as np

TILE = 16  # TILE_SIZE (renderers/renderer.h:34)


@lru_cache(maxsize=16)
def logical_tiles(ntiles: int) -> np.ndarray:
    """Image tile (raster order) -> the logical tile of a sharded job's frame that covers it."""
    from . import _native as N
    inv = np.empty(ntiles, np.int64)
    for t in range(ntiles):
        inv[N.dev.yrtDebugTileScatter(t, ntiles)] = t
    return inv


def tile_mask(width: int, height: int, rank: int, world: int) -> np.ndarray:
    """Pixels rendered by `rank` of `world`: bool (height, width)."""
    ntx, nty = (width + TILE - 1) // TILE, (height + TILE - 1) // TILE
    tile = np.arange(height)[:, None] // TILE * ntx + np.arange(width)[None, :] // TILE
    if world > 1:
        tile = logical_tiles(ntx * nty)[tile]
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
