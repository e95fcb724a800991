"""The reference's rcp/rsqrt estimates, emulated: yrt_sse_rcp.h against the committed tables.

The reference computes rcp()/rsqrt() with the SSE estimate instructions plus one Newton step
(common/math/math.h:38-59). tests/golden/sse_rcp_tables.json holds what an Intel CPU's
rcpps/rsqrtps return (tests/golden/make_sse_tables.py); the product and the oracle share one exact
emulation of them (yulio-raytracer_amd/csrc/common/yrt_sse_rcp.h). These tests run on any host
(they do not execute the instructions): the emulation, as compiled into the oracle, against the
fixture on inputs spread over every exponent and every table entry, the special inputs, and
the Newton steps of math.h. The hardware itself is compared on every 32-bit input in
tests/test_ref_pin.py (Intel hosts), the GPU's emulation in tests/test_gpu_parity.py.
"""
import json
from pathlib import Path

import numpy as np
import pytest

import oracle

FIX = json.loads((Path(__file__).resolve().parent / "golden" / "sse_rcp_tables.json").read_text())
RCP = np.array(FIX["rcpps_mantissa12"], np.int64)
RSQ = np.array(FIX["rsqrtps_mantissa12"], np.int64)


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _inputs(seed, n=1 << 20):
    """Random sign, every biased exponent 0..255, random mantissa: each table entry many times."""
    rng = np.random.default_rng(seed)
    u = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    return u.view(np.float32)


def _expect_rcpps(x):
    u = _bits(x).astype(np.int64)
    s, e, i = u >> 31, (u >> 23) & 0xFF, (u >> 12) & 0x7FF
    out = (s << 31) | ((253 - e) << 23) | (RCP[i] << 11)
    out = np.where(e >= 253, s << 31, out)
    out = np.where(e == 255, np.where(u & 0x7FFFFF, u | 0x400000, s << 31), out)
    out = np.where(e == 0, (s << 31) | 0x7F800000, out)
    return out.astype(np.uint32)


def _expect_rsqrtps(x):
    u = _bits(x).astype(np.int64)
    s, e, j = u >> 31, (u >> 23) & 0xFF, (u >> 13) & 0x3FF
    E = e - 127
    p = E & 1
    k = (E - p) // 2
    out = ((126 - k) << 23) | (RSQ[(p << 10) | j] << 11)
    out = np.where(s == 1, 0xFFC00000, out)
    out = np.where(e == 255, np.where(u & 0x7FFFFF, u | 0x400000, np.where(s == 1, 0xFFC00000, 0)), out)
    out = np.where(e == 0, (s << 31) | 0x7F800000, out)
    return out.astype(np.uint32)


def test_fixture_is_twelve_bit_round_to_nearest_of_the_interval_midpoint():
    """What the tables are (yrt_sse_rcp.h header): RN to 12 bits of 1/mid and 1/sqrt(mid)."""
    i = np.arange(2048)
    assert np.array_equal(RCP, np.rint(4096 * (2 / (1 + (i + 0.5) / 2048) - 1)).astype(np.int64))
    j, p = np.arange(2048) & 1023, np.arange(2048) >> 10
    mid = (1 + (j + 0.5) / 1024) * 2.0 ** p
    assert np.array_equal(RSQ, np.rint(4096 * (2 / np.sqrt(mid) - 1)).astype(np.int64))


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_emulated_estimates_match_the_tables(seed):
    x = _inputs(seed)
    assert np.array_equal(_bits(oracle.vecmath("rcpps", x)), _expect_rcpps(x))
    assert np.array_equal(_bits(oracle.vecmath("rsqrtps", x)), _expect_rsqrtps(x))


def test_every_table_entry_at_both_ends():
    """Entry boundaries: the lowest and highest input of each of the 2048 intervals."""
    i = np.arange(2048, dtype=np.uint32)
    lo, hi = 0x3F800000 | (i << 12), 0x3F800000 | (i << 12) | 0xFFF
    for u in (lo, hi):
        x = u.view(np.float32)
        assert np.array_equal(_bits(oracle.vecmath("rcpps", x)), _expect_rcpps(x))
    for p in (0, 1):
        j = np.arange(1024, dtype=np.uint32)
        for low in (0, 0x1FFF):
            x = (((127 + p) << 23) | (j << 13) | low).astype(np.uint32).view(np.float32)
            assert np.array_equal(_bits(oracle.vecmath("rsqrtps", x)), _expect_rsqrtps(x))


def test_special_inputs_as_recorded():
    cases = {"+0": 0x00000000, "-0": 0x80000000, "subnormal 0x5": 0x00000005, "+inf": 0x7F800000,
             "-inf": 0xFF800000, "2^-126": 0x00800000}
    for name, u in cases.items():
        x = np.array([u], np.uint32).view(np.float32)
        for fn in ("rcpps", "rsqrtps"):
            want = float.fromhex(FIX["special"][name][fn]) if FIX["special"][name][fn] != "nan" else float("nan")
            got = float(oracle.vecmath(fn, x)[0])
            assert (np.isnan(want) and np.isnan(got)) or (got == want and np.signbit(got) == np.signbit(want)), \
                (name, fn, got, want)


def test_newton_steps_of_math_h():
    """rcp(x) = (r + r) - (r * r) * x and rsqrt(x) = 1.5 r + ((x * -0.5) * r) * (r * r), each
    operation rounded (math.h:38-42, 53-58), on the emulated estimates."""
    x = np.abs(_inputs(7, 1 << 18))
    x = x[np.isfinite(x) & (x > 2.0 ** -60) & (x < 2.0 ** 60)]
    r = oracle.vecmath("rcpps", x)
    want = (r + r) - (r * r) * x
    assert np.array_equal(_bits(oracle.vecmath("rcp", x)), _bits(want))
    q = oracle.vecmath("rsqrtps", x)
    want = np.float32(1.5) * q + ((x * np.float32(-0.5)) * q) * (q * q)
    assert np.array_equal(_bits(oracle.vecmath("rsqrt", x)), _bits(want))


def test_reference_rcp_is_not_ieee():
    """The substitution rounds 1-5 made (rcp = 1/x): how far the reference's rcp is from it."""
    x = np.abs(_inputs(9, 1 << 18))
    # beyond ~2^63 the reference's r * r underflows and rcp(x) tends to 2 rcpps(x) (reproduced)
    x = x[np.isfinite(x) & (x > 2.0 ** -60) & (x < 2.0 ** 60)]
    ulp = np.abs(_bits(oracle.vecmath("rcp", x)).astype(np.int64) - _bits(np.float32(1) / x).astype(np.int64))
    # measured: 22 % of inputs differ from the correctly rounded 1/x, by at most 2 ulp
    assert ulp.max() <= 2 and 0.15 < (ulp > 0).mean() < 0.3, (ulp.max(), (ulp > 0).mean())
    r = _bits(oracle.vecmath("rsqrt", x)).astype(np.int64)
    ulp = np.abs(r - _bits(np.float32(1) / np.sqrt(x)).astype(np.int64))
    assert ulp.max() <= 4 and (ulp > 0).mean() > 0.15, (ulp.max(), (ulp > 0).mean())
    assert float(oracle.vecmath("rcp", np.array([3.0], np.float32))[0]).hex() == "0x1.5555540000000p-2"
