"""The oracle's integer layer pinned against the reference itself (oracle/_ref).

oracle/_ref/libref_kat.so is compiled by `make -C oracle ref` from the reference's own,
unmodified common/math/random.h, common/math/permutation.h, common/sys/stl/vector.h and
common/sys/platform.cpp (where they lie under /root/reference) behind the small driver
oracle/ref_kat.cpp. These tests compare the C restatement (oracle/yrt_oracle.c) with it bit for
bit: Random (KAT 1), Permutation, vector_t::shuffle, the per-tile set draw of
integratorrenderer.cpp:134,149, and SamplerFactory::init tables without the pixel filter
(the filter's Distribution2D lives behind default.h, which does not compile here).
"""
import ctypes as C

import numpy as np
import pytest

import oracle

if not oracle.REF_LIB.exists():
    pytest.skip("oracle/_ref not built (needs /root/reference: make -C oracle ref)", allow_module_level=True)

_ref = C.CDLL(str(oracle.REF_LIB))
SEEDS = [1, 27, 5897, 91711, 81551, 2 * 5897, 123456789, -7, 0]


def _call(name, shape, dtype, *args):
    out = np.zeros(shape, dtype)
    getattr(_ref, name)(*[C.c_int(a) for a in args], out.ctypes.data_as(C.c_void_p))
    return out


@pytest.mark.parametrize("seed", SEEDS)
def test_random_ints_and_floats(seed):
    assert np.array_equal(_call("ref_random_ints", 4096, np.int32, seed, 4096), oracle.random_ints(seed, 4096))
    assert np.array_equal(_call("ref_random_floats", 4096, np.float32, seed, 4096).view(np.uint32),
                          oracle.random_floats(seed, 4096).view(np.uint32))


@pytest.mark.parametrize("size,seed", [(1, 1), (7, 27), (64, 5897), (256, 11794), (1024, 3)])
def test_permutations(size, seed):
    assert np.array_equal(_call("ref_permutations", (9, size), np.int32, size, seed, 9),
                          oracle.permutations(size, seed, 9))


@pytest.mark.parametrize("n,seed", [(8, 1), (16, 5897), (32, 77)])
def test_vector_shuffles(n, seed):
    assert np.array_equal(_call("ref_shuffles", (12, n), np.uint32, n, seed, 12), oracle.shuffles(n, seed, 12))


@pytest.mark.parametrize("w,h", [(100, 70), (256, 256), (1536, 40)])
def test_pixel_set_draw(w, h):
    assert np.array_equal(_call("ref_pixel_sets", (h, w), np.uint8, w, h, 64), oracle.pixel_sets(w, h, 64))


@pytest.mark.parametrize("spp,iteration,n1,n2", [(1, 0, 2, 3), (16, 0, 2, 3), (64, 0, 10, 11), (256, 0, 10, 11),
                                                 (16, 5, 2, 3), (64, 3, 10, 11)])
def test_sample_tables_without_filter(spp, iteration, n1, n2):
    sets = 64
    dims = 5 + n1 + 2 * n2
    ref = _call("ref_sample_table_nofilter", (dims, sets * spp), np.float32, spp, sets, iteration, n1, n2)
    got = oracle.sample_table(spp, sets, iteration, n1, n2, filter="none")
    assert np.array_equal(ref.view(np.uint32), got.view(np.uint32))
