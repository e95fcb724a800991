"""Shared test helpers: BASELINE configs as session argv, and the parity criterion of
SURVEY.md §8(d) ("Parity tolerance")."""
from __future__ import annotations

from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
SCENES = ROOT / "scenes"


def c1_args(size=256, spp=1):
    """C1: models/cornell_box.ecs (256x256 1spp, depth 2, quad light)."""
    return ["-c", str(SCENES / "cornell_box.ecs"), "-size", str(size), str(size), "-spp", str(spp)]


def c2_args(size=1024, spp=16):
    """C2: models/cornell_box_spheres.ecs at 16 spp."""
    return ["-c", str(SCENES / "cornell_box_spheres.ecs"), "-size", str(size), str(size), "-spp", str(spp)]


def c4_args(size=1536, spp=256, stereo=True):
    """C4: -i test_stereo.xml -c test_stereo_view.ecs -stereo."""
    a = ["-i", str(SCENES / "test_stereo.xml"), "-c", str(SCENES / "test_stereo_view.ecs"),
         "-size", str(size), str(size), "-spp", str(spp)]
    return a + (["-stereo"] if stereo else [])


def c3_args(size=2048, spp=64):
    """C3: Sponza stand-in (yrt.standin) with the Sponza camera of test_stereo_view.ecs."""
    from yrt import standin
    x = standin.write_xml()
    return ["-i", str(x)] + standin.C3_ARGS + ["-size", str(size), str(size), "-spp", str(spp)]


def parity(g: np.ndarray, c: np.ndarray, min_frac: float, mad_rel: float | None = 1e-4, atol=1e-3, rtol=1e-3,
           exact: bool = True, nan_ok: bool = False):
    """per channel |g-c| <= atol + rtol*|c| on >= min_frac of channels, and
    mean-abs-diff <= mad_rel * mean(c). With exact (the default) the frames must also be
    bit-identical: the device and the oracle evaluate the same IEEE operations in the same order
    (no FMA contraction, shared elementary functions yrt_libm.h), so any
    difference is a defect, not rounding. nan_ok: NaN pixels allowed where the oracle has them.
    Returns a dict of the measured quantities."""
    g = np.asarray(g, np.float64)
    c = np.asarray(c, np.float64)
    assert g.shape == c.shape, (g.shape, c.shape)
    if nan_ok:
        # scenes whose reference arithmetic yields NaN samples (e.g. log(0) transmission): the
        # non-finite pixels must be the oracle's, the rest is compared as usual
        assert np.array_equal(np.isnan(g), np.isnan(c)), "NaN pixels differ from the oracle's"
        keep = ~np.isnan(c)
        g, c = g[keep], c[keep]
    assert np.isfinite(g).all(), "non-finite GPU pixels"
    d = np.abs(g - c)
    ok = d <= atol + rtol * np.abs(c)
    frac = float(ok.mean())
    mad = float(d.mean())
    mean = float(np.abs(c).mean())
    res = {"frac_within": frac, "mad": mad, "mean": mean, "max_diff": float(d.max()), "exact": float((d == 0).mean())}
    assert frac >= min_frac, res
    if mad_rel is not None:
        assert mad <= mad_rel * mean + 1e-7, res
    if exact:
        assert np.array_equal(g, c), res
    return res
