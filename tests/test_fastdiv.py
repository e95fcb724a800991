"""FastDiv (csrc/common/yrt_gpu_types.h): n / d as (umulhi(n, mul) + n) >> shift.

The kernels divide path ids by the batch's pixel count and tile indices by the tile-grid width
and the tiles per frame this way (kernels/pathtrace.hip fastdiv). This restates the host-side
construction (fastdiv_make) and the device evaluation in exact integer arithmetic and checks
them against floor division, exhaustively over small ranges and on random and boundary
dividends up to 2^31 for the divisors the renderer uses and random ones.
"""
import numpy as np


def make(d: int):
    shift = 0
    while shift < 31 and (1 << shift) < d:
        shift += 1
    magic = ((1 << 32) * ((1 << shift) - d)) // d + 1
    assert 0 < magic < (1 << 32)
    return magic, shift


def evaluate(n: np.ndarray, magic: int, shift: int) -> np.ndarray:
    n = n.astype(np.uint64)
    hi = (n * np.uint64(magic)) >> np.uint64(32)  # __umulhi
    s = (hi + n) & np.uint64(0xFFFFFFFF)  # 32-bit add: must not wrap for n < 2^31
    assert ((hi + n) >> np.uint64(32) == 0).all()
    return (s >> np.uint64(shift)).astype(np.int64)


def divisors():
    rng = np.random.default_rng(7)
    ds = list(range(1, 1025))
    ds += [256 * k for k in (1, 2, 3, 96, 1024, 9216, 12 * 9216, 65536, 262144)]  # batch pixel counts
    ds += [96, 128, 9216, 110592, 16384]  # tiles in x, tiles per frame (1536^2, 2048^2)
    ds += [(1 << k) + e for k in range(11, 31) for e in (-1, 0, 1)]
    ds += [int(x) for x in rng.integers(1, 1 << 31, 200)]
    return ds


def test_fastdiv_exhaustive_small():
    n = np.arange(0, 1 << 16, dtype=np.int64)
    for d in range(1, 1025):
        m, s = make(d)
        np.testing.assert_array_equal(evaluate(n, m, s), n // d)


def test_fastdiv_random_and_boundaries():
    rng = np.random.default_rng(11)
    base = rng.integers(0, 1 << 31, 20000, dtype=np.int64)
    for d in divisors():
        m, s = make(d)
        k = np.arange(0, (1 << 31) // d + 1, max(1, ((1 << 31) // d) // 2000), dtype=np.int64)
        edges = np.concatenate([k * d - 1, k * d, k * d + 1, [(1 << 31) - 1, (1 << 31) - 2]])
        n = np.concatenate([base, edges])
        n = n[(n >= 0) & (n < (1 << 31))]
        np.testing.assert_array_equal(evaluate(n, m, s), n // d, err_msg=f"d={d}")
