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


# ---------------------------------------------------------------- common/math (oracle/_ref/libref_math.so)
# The reference's own math.h / vec3.h (-> vector3f_sse.h) / linearspace3.h / color.h / bsphere.h,
# compiled unmodified with clang (oracle/Makefile, oracle/ref_math.cpp), against the oracle's
# helpers and the front end's camera basis, bit for bit. rcp/rsqrt go through the executing CPU's
# rcpps/rsqrtps, whose tables are vendor-specific: those comparisons need an Intel host (this
# container); tests/test_sse_rcp.py checks the same emulation against the committed Intel tables
# on any host.
import json  # noqa: E402
from pathlib import Path  # noqa: E402

_math = C.CDLL(str(oracle.REF_MATH_LIB)) if oracle.REF_MATH_LIB.exists() else None
needs_math = pytest.mark.skipif(_math is None, reason="oracle/_ref/libref_math.so not built (make -C oracle ref)")


def _vendor():
    for line in Path("/proc/cpuinfo").read_text().splitlines():
        if line.startswith("vendor_id"):
            return line.split(":", 1)[1].strip()
    return "?"


intel_only = pytest.mark.skipif(_vendor() != "GenuineIntel",
                                reason="rcpps/rsqrtps tables are vendor-specific; the fixture is Intel's")
VEC = {"dot": (0, 3, 3, 1), "cross": (1, 3, 3, 3), "normalize": (2, 3, 0, 3), "length": (3, 3, 0, 1),
       "lmul": (4, 9, 3, 3), "frame": (5, 3, 0, 9), "inverse": (6, 9, 0, 9), "color_div": (7, 3, 1, 3)}


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _ref_vec(name, a, b=None):
    fn, na, nb, no = VEC[name]
    a = np.ascontiguousarray(a, np.float32).reshape(-1, na)
    n = a.shape[0]
    b = np.zeros((n, max(nb, 1)), np.float32) if b is None else np.ascontiguousarray(b, np.float32).reshape(n, -1)
    out = np.zeros((n, no), np.float32)
    _math.ref_vec(fn, n, _p(a), _p(b), _p(out))
    return out if no > 1 else out[:, 0]


def _same(a, b, zero_sign=False):
    """Bit-identical (NaNs by bits too); zero_sign: +0 and -0 count as equal."""
    a, b = np.ascontiguousarray(a, np.float32), np.ascontiguousarray(b, np.float32)
    ok = a.view(np.uint32) == b.view(np.uint32)
    if zero_sign:
        ok |= (a == 0) & (b == 0)
    return bool(ok.all()), int((~ok).sum())


def _vectors(seed, n=1 << 16):
    """Random vectors over many magnitudes, plus axis-aligned, zero and negative-zero ones."""
    rng = np.random.default_rng(seed)
    v = (rng.standard_normal((n, 3)) * 10.0 ** rng.integers(-6, 7, (n, 1))).astype(np.float32)
    v[: n // 16] = np.float32(rng.integers(-2, 3, (n // 16, 3)))
    v[n // 16: n // 8] = rng.choice(np.array([0.0, -0.0, 1.0, -1.0, 0.5], np.float32), (n // 16, 3))
    return v


@needs_math
@intel_only
@pytest.mark.parametrize("fn,name", [(0, "rcp"), (1, "rsqrt")])
def test_reciprocals_equal_the_reference_on_every_input(fn, name):
    """math.h:38-59 rcp / rsqrt (this CPU's rcpps/rsqrtps + the Newton step) against the
    emulation the product and the oracle use (yrt_sse_rcp.h), on all 2^32 inputs, NaNs included."""
    first = C.c_uint32(0)
    _math.ref_check_sse_exhaustive.restype = C.c_uint64
    bad = _math.ref_check_sse_exhaustive(fn, min(8, oracle.cpu_count()), C.byref(first))
    assert bad == 0, (name, bad, hex(first.value))


@needs_math
@intel_only
def test_fixture_tables_are_this_cpus():
    rcp, rsq = np.zeros(2048, np.uint16), np.zeros(2048, np.uint16)
    special = np.zeros(12, np.float32)
    _math.ref_sse_tables(_p(rcp), _p(rsq), _p(special))
    fix = json.loads((Path(__file__).resolve().parent / "golden" / "sse_rcp_tables.json").read_text())
    assert rcp.tolist() == fix["rcpps_mantissa12"] and rsq.tolist() == fix["rsqrtps_mantissa12"]


@needs_math
@intel_only
@pytest.mark.parametrize("seed", [11, 12])
def test_reciprocals_on_vector_inputs(seed):
    x = np.abs(_vectors(seed)).ravel()
    for fn, name in ((0, "rcp"), (1, "rsqrt")):
        ref = np.zeros_like(x)
        _math.ref_scalar(fn, x.size, _p(x), _p(ref))
        assert _same(ref, oracle.vecmath(name, x)) == (True, 0), name


@needs_math
@intel_only
@pytest.mark.parametrize("name", ["dot", "cross", "normalize", "length", "lmul", "frame", "inverse", "color_div"])
@pytest.mark.parametrize("seed", [21, 22])
def test_vector_helpers_equal_the_reference(name, seed):
    """vector3f_sse.h dot (_mm_dp_ps) / cross / normalize / length, linearspace3.h L * v, frame,
    inverse, color_sse.h Color / float: the oracle's helpers (the product's yrt_math.h twins are
    bit-exact to them through every render test) on the reference's own code. dot's only
    difference is the sign of an exactly zero sum: dp_ps adds its masked fourth lane's +0
    (DESIGN.md §4); nothing downstream reads that sign."""
    _, na, nb, _ = VEC[name]
    rng = np.random.default_rng(seed)
    v = _vectors(seed)
    a = np.concatenate([v, _vectors(seed + 100), _vectors(seed + 200)], 1)[:, :na] if na == 9 else v
    b = None
    if nb == 3:
        b = _vectors(seed + 1)
    elif nb == 1:
        b = (rng.standard_normal(v.shape[0]) * 10.0 ** rng.integers(-3, 4, v.shape[0])).astype(np.float32)
    ref = _ref_vec(name, a, b)
    got = oracle.vecmath(name, a, b)
    assert _same(ref, got, zero_sign=(name == "dot")) == (True, 0)


@needs_math
def test_bounding_sphere_equals_the_reference():
    """getBSphere (bbox.h:75-78) + BSphere::rayIntersect (bsphere.h:93-100) + solveQuadratic
    (math.h:174-208): no rcp/rsqrt inside, so any host."""
    rng = np.random.default_rng(5)
    n = 1 << 15
    lo = (rng.standard_normal((n, 3)) * 50).astype(np.float32)
    hi = lo + np.abs(rng.standard_normal((n, 3)) * 80).astype(np.float32)
    org = (rng.standard_normal((n, 3)) * 100).astype(np.float32)
    d = rng.standard_normal((n, 3)).astype(np.float32)
    d[:64] = 0.0  # the linear and no-solution cases
    ref = np.zeros((n, 4), np.float32)
    _math.ref_bsphere(n, *[_p(np.ascontiguousarray(x)) for x in (lo, hi, org, d)], _p(ref))
    got = oracle.bsphere(lo, hi, org, d)
    assert _same(ref, got) == (True, 0) and 0.1 < ref[:, 0].mean() < 0.9


def _session_camera(args):
    import yrt
    from dae_scene import blob_objects
    dev = yrt.Device(host=True)
    s = yrt.Session(args, device=dev)
    blob = s.export_frame()
    s.close()
    dev.close()
    cams = [p for k, _, p in blob_objects(blob) if k == "CAMERA"]
    assert len(cams) == 1
    return blob, cams[0]


@needs_math
@intel_only
def test_front_end_camera_basis():
    """The .ecs camera (-vp -vi -vu) -> local2world: renderer.cpp's AffineSpace3f::lookAtPoint
    (affinespace.h:72-77), here with the reference's Vector3f normalize / cross (ref_look_at)."""
    from helpers import c1_args, c3_args
    for args, (vp, vi, vu) in [(c3_args(64, 1), ((2.25067, 8.24132, -0.0492483), (3.15037, 7.8048, -0.0501832),
                                                  (0.436514, 0.899693, -0.00291584))),
                               (c1_args(64, 1), ((278, 273, -800), (278, 273, 0), (0, 1, 0)))]:
        _, cam = _session_camera(args)
        want = np.zeros(12, np.float32)
        e, p, u = (np.array(x, np.float32) for x in (vp, vi, vu))
        _math.ref_look_at(1, _p(e), _p(p), _p(u), _p(want))
        assert _same(np.array(cam["local2world"], np.float32), want) == (True, 0), (cam["local2world"], want)


@needs_math
@intel_only
@pytest.mark.parametrize("which", ["c1", "c3"])
def test_pinhole_camera_rays_equal_the_reference(which):
    """PinHoleCamera (pinholecamera.h:30-40): the oracle's camera rays of the exported frame (the
    device's are bit-exact to the oracle's, tests/test_gpu_parity.py) against the reference's
    Vector3f arithmetic on the same local2world, angle and aspect ratio."""
    from helpers import c1_args, c3_args
    blob, cam = _session_camera(c1_args(64, 1) if which == "c1" else c3_args(64, 1))
    l2w = np.array(cam["local2world"], np.float32)
    angle, ar = float(cam["angle"][0]), float(cam["aspectRatio"][0])
    rng = np.random.default_rng(3)
    px = rng.random((4096, 2)).astype(np.float32)
    want = np.zeros((4096, 3), np.float32)
    _math.ref_pinhole_dir(4096, _p(l2w[:9].copy()), C.c_float(angle), C.c_float(ar), _p(px), _p(want))
    org, got = oracle.camera_rays(blob, px)
    assert _same(got, want) == (True, 0)
    assert np.array_equal(org, np.broadcast_to(l2w[9:], org.shape))
