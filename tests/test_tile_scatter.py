"""The sharded tile deal's image map (common/yrt_tile_scatter.h), through the device library's
host-side export (CPU only): a bijection of each frame's tiles, so a sharded frame covers every
pixel once, and a uniform spread of every shard's tiles over the image (no shard gets a column
set of a periodic scene). The GPU tests compose sharded frames bit-exactly with it
(test_tile_shards_compose_bit_exact, tests/test_gather.py)."""
import numpy as np
import pytest

from yrt import _native as N


def scatter(T):
    return np.array([N.dev.yrtDebugTileScatter(t, T) for t in range(T)])


@pytest.mark.parametrize("T", [1, 2, 3, 7, 64, 100, 96 * 96, 128 * 128, 257 * 3])
def test_scatter_is_a_bijection(T):
    p = scatter(T)
    assert sorted(p.tolist()) == list(range(T))
    assert N.dev.yrtDebugTileScatter(T, T) == -1 and N.dev.yrtDebugTileScatter(-1, T) == -1


@pytest.mark.parametrize("tx,ty", [(128, 128), (96, 96)])
@pytest.mark.parametrize("shards", [2, 3, 8])
def test_every_shard_samples_the_whole_image(tx, ty, shards):
    p = scatter(tx * ty)
    for r in range(shards):
        mine = p[r::shards]  # logical tiles r, r + N, ... -> their image tiles
        col8 = np.bincount((mine % tx) % 8, minlength=8) / len(mine)
        quarter = np.bincount(np.minimum((mine // tx) * 4 // ty, 3), minlength=4) / len(mine)
        # the plain round-robin deal puts all of a shard's tiles in one column class mod N
        assert col8.max() - col8.min() < 0.06, (r, col8)
        assert quarter.max() - quarter.min() < 0.04, (r, quarter)
