"""Accuracy of yrt_libm.h, the per-ray path's elementary functions shared by the device kernels
and the oracle (evaluated here through the oracle build): ulp error against float64 numpy."""
import numpy as np
import pytest

import oracle

def _rng(name):
    """Inputs per test, independent of the order the tests run in (xdist workers)."""
    return np.random.default_rng(sum(map(ord, name)))


def _ulp(got, ref):
    sp = np.spacing(np.abs(ref.astype(np.float32))).astype(np.float64)
    return np.abs(got.astype(np.float64) - ref) / sp


@pytest.mark.parametrize("fn,np_fn,lo,hi,bound", [
    ("sin", np.sin, -20, 20, 3), ("cos", np.cos, -20, 20, 3), ("exp", np.exp, -87, 88, 2),
    ("asin", np.arcsin, -1, 1, 3), ("acos", np.arccos, -1, 1, 3), ("atan", np.arctan, -50, 50, 3)])
def test_unary_ulp(fn, np_fn, lo, hi, bound):
    x = _rng(fn).uniform(lo, hi, 200_000).astype(np.float32)
    ref = np_fn(x.astype(np.float64))
    got = oracle.libm(fn, x)
    if fn in ("sin", "cos"):
        # near a zero of sin/cos (x close to a multiple of pi/2) the three-part Cody-Waite
        # reduction leaves an absolute error of ~1e-9; relative ulps are bounded elsewhere
        far = np.abs(ref) > 1e-3
        assert np.abs(got - ref).max() < 2e-7
        assert _ulp(got[far], ref[far]).max() <= bound
    else:
        assert _ulp(got, ref).max() <= bound


def test_log_and_pow():
    x = np.exp(_rng("log").uniform(-80, 80, 200_000)).astype(np.float32)
    ref = np.log(x.astype(np.float64))
    got = oracle.libm("log", x)
    assert np.abs(got - ref).max() < 1e-5 and _ulp(got, ref)[np.abs(ref) > 0.1].max() <= 2
    # pow = exp(y log x): relative error grows with |y log x|; the renderer's exponents are
    # BRDF exponents (<= ~100) and medium depths
    x = _rng("pow x").uniform(0, 1, 200_000).astype(np.float32)
    y = _rng("pow y").uniform(0, 100, 200_000).astype(np.float32)
    ref = np.power(x.astype(np.float64), y.astype(np.float64))
    m = ref > 1e-30
    assert (np.abs(oracle.libm("pow", x, y)[m] - ref[m]) / ref[m]).max() < 2e-5


def test_atan2_and_specials():
    y = _rng("atan2 y").normal(0, 1, 200_000).astype(np.float32)
    x = _rng("atan2 x").normal(0, 1, 200_000).astype(np.float32)
    assert _ulp(oracle.libm("atan2", y, x), np.arctan2(y.astype(np.float64), x.astype(np.float64))).max() <= 4
    z = np.array([0.0, -0.0, 1.0, -1.0], np.float32)
    assert np.array_equal(oracle.libm("atan2", z, np.array([1.0, 1.0, 0.0, 0.0], np.float32)),
                          np.arctan2(z, np.array([1.0, 1.0, 0.0, 0.0], np.float32)).astype(np.float32))
    assert oracle.libm("pow", np.float32([0.0, 1.0, 2.0]), np.float32([2.0, 7.0, 0.0])).tolist() == [0.0, 1.0, 1.0]
    assert oracle.libm("exp", np.float32([0.0]))[0] == 1.0 and oracle.libm("log", np.float32([1.0]))[0] == 0.0
    assert np.isnan(oracle.libm("acos", np.float32([1.5]))[0])
