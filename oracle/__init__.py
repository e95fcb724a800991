"""ctypes wrapper of liboracle.so — the CPU restatement of the reference render path.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker. The product (yulio-raytracer_amd/) never imports it.
See yrt_oracle.h for what it restates (reference file:line) and its documented substitutions.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"


def build():
    import subprocess
    subprocess.run(["make", "-C", str(HERE)], check=True, stdout=subprocess.DEVNULL)


if not LIB.exists():
    build()
REF_LIB = HERE / "_ref" / "libref_kat.so"  # reference-compiled KAT library (make -C oracle ref)
REF_MATH_LIB = HERE / "_ref" / "libref_math.so"  # the reference's common/math, compiled (make -C oracle ref)
IEEE_LIB = HERE / "liboracle_ieee.so"  # rcp = 1/x, rsqrt = 1/sqrt(x): tools/rcp_sensitivity.py only
_lib = C.CDLL(str(LIB))

vp, sz, i32, PF = C.c_void_p, C.c_size_t, C.c_int, C.POINTER(C.c_float)


class OracleStats(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("raysClosest", "raysShadow", "samples", "seconds", "nodeVisits",
                                          "triVisits")]


def _sig(name, res, *args):
    f = getattr(_lib, name)
    f.restype, f.argtypes = res, list(args)


_sig("oracle_render", i32, vp, sz, i32, i32, C.c_float, i32, i32, i32, i32, i32, vp, C.POINTER(OracleStats))
_sig("oracle_trace", i32, vp, sz, vp, vp, i32, i32, vp)
_sig("oracle_debug_pixel", i32, vp, sz, i32, i32, i32, i32, vp, i32)
_sig("oracle_debug_path", i32, vp, sz, i32, i32, i32, i32, i32, vp)
_sig("oracle_render_shard", i32, vp, sz, i32, i32, C.c_float, i32, i32, i32, i32, i32, i32, i32, vp,
     C.POINTER(OracleStats))
_sig("oracle_count_visits", i32, vp, sz, vp, sz, vp, vp, i32, i32, C.POINTER(C.c_double),
     C.POINTER(C.c_double), vp, sz)
_sig("oracle_count_visits_q", i32, vp, sz, vp, sz, vp, vp, i32, i32, C.POINTER(C.c_double),
     C.POINTER(C.c_double), vp, sz)
_sig("oracle_random_ints", None, i32, i32, vp)
_sig("oracle_sample_table", i32, i32, i32, i32, i32, i32, C.c_char_p, vp, sz)
_sig("oracle_pixel_sets", None, i32, i32, i32, vp)
_sig("oracle_scene_triangles", i32, vp, sz, vp, i32)
_sig("oracle_last_error", C.c_char_p)
_sig("oracle_random_floats", None, i32, i32, vp)
_sig("oracle_permutations", None, i32, i32, i32, vp)
_sig("oracle_shuffles", None, i32, i32, i32, vp)
_sig("oracle_libm", None, i32, i32, vp, vp, vp)
_sig("oracle_vecmath", None, i32, i32, vp, vp, vp)
_sig("oracle_bsphere", None, i32, vp, vp, vp, vp, vp)
_sig("oracle_camera_rays", i32, vp, sz, i32, vp, vp, vp)


def _err():
    e = _lib.oracle_last_error()
    return e.decode() if e else "?"


_ieee = None


def _ieee_lib():
    """liboracle_ieee.so: the same restatement with rcp = 1/x, rsqrt = 1/sqrt(x) (the substitution
    of rounds 1-5), for tools/rcp_sensitivity.py."""
    global _ieee
    if _ieee is None:
        _ieee = C.CDLL(str(IEEE_LIB))
        _ieee.oracle_render.restype = i32
        _ieee.oracle_render.argtypes = _lib.oracle_render.argtypes
    return _ieee


def render(blob: bytes, width, height, gamma=1.0, rect=None, threads=0, ieee_rcp=False):
    """RGB_FLOAT32 image (H, W, 3) of the frame blob; pixels outside rect stay NaN."""
    threads = threads or cpu_count()
    x0, y0, x1, y1 = rect if rect is not None else (0, 0, width, height)
    out = np.full((height, width, 3), np.nan, np.float32)
    st = OracleStats()
    lib = _ieee_lib() if ieee_rcp else _lib
    rc = lib.oracle_render(blob, len(blob), width, height, gamma, x0, y0, x1, y1, threads, out.ctypes.data,
                           C.byref(st))
    if rc != 0:
        raise RuntimeError(f"oracle_render: {_err()}")
    return out, {n: getattr(st, n) for n, _ in st._fields_}


def render_shard(blob: bytes, width, height, gamma, index, count, threads=0):
    """The tiles t % count == index of the frame (SURVEY §8(e) split); other pixels NaN."""
    threads = threads or cpu_count()
    out = np.full((height, width, 3), np.nan, np.float32)
    st = OracleStats()
    rc = _lib.oracle_render_shard(blob, len(blob), width, height, gamma, 0, 0, width, height, index, count, threads,
                                  out.ctypes.data, C.byref(st))
    if rc != 0:
        raise RuntimeError(f"oracle_render_shard: {_err()}")
    return out, {n: getattr(st, n) for n, _ in st._fields_}


def debug_pixel(blob: bytes, width, height, x, y, max_spp=1 << 16):
    """Per-sample radiance of pixel (x, y): float32 (spp, 3), in the pixel's summation order."""
    out = np.zeros((max_spp, 3), np.float32)
    n = _lib.oracle_debug_pixel(blob, len(blob), width, height, x, y, out.ctypes.data, max_spp)
    if n < 0:
        raise RuntimeError(f"oracle_debug_pixel: {_err()}")
    return out[:min(n, max_spp)]


# fields of a debug_path record (32 floats per depth)
PATH_FIELDS = ["valid", "tri", "t", "u", "v", "thr", "thr", "thr", "P", "P", "P", "Ns", "Ns", "Ns", "L", "L", "L",
               "wi", "wi", "wi", "pdf", "c", "c", "c", "nthr", "nthr", "nthr", "dir", "dir", "dir", "org_x", "useDirect"]


def debug_path(blob: bytes, width, height, x, y, sample):
    """Per-depth record of sample `sample` of pixel (x, y): float32 (depths, 32), PATH_FIELDS."""
    out = np.zeros((32, 32), np.float32)
    if _lib.oracle_debug_path(blob, len(blob), width, height, x, y, sample, out.ctypes.data) < 0:
        raise RuntimeError(f"oracle_debug_path: {_err()}")
    return out[: int((out[:, 0] != 0).sum())]


def trace(blob: bytes, org4: np.ndarray, dir4: np.ndarray, any_hit=False):
    org4 = np.ascontiguousarray(org4, np.float32)
    dir4 = np.ascontiguousarray(dir4, np.float32)
    n = org4.shape[0]
    hit = np.zeros((n, 4), np.float32)
    rc = _lib.oracle_trace(blob, len(blob), org4.ctypes.data, dir4.ctypes.data, n, int(any_hit), hit.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"oracle_trace: {_err()}")
    return hit


def count_visits(nodes: np.ndarray, tris: np.ndarray, org4, dir4, any_hit=False, tri_bytes=48, qnodes=None):
    """Node / triangle visits of the device traversal order over an exported BVH (tri_bytes:
    the scene's triRecordBytes); qnodes: traverse the quantized nodes (Device.export_qbvh)
    instead of the float ones."""
    org4 = np.ascontiguousarray(org4, np.float32)
    dir4 = np.ascontiguousarray(dir4, np.float32)
    n = org4.shape[0]
    nv, tv = C.c_double(), C.c_double()
    hit = np.zeros((n, 4), np.float32)
    fn, nd, nb = (_lib.oracle_count_visits, nodes, 128) if qnodes is None else (_lib.oracle_count_visits_q, qnodes, 64)
    rc = fn(nd.ctypes.data, nd.nbytes // nb, tris.ctypes.data, tris.nbytes // tri_bytes,
            org4.ctypes.data, dir4.ctypes.data, n, int(any_hit), C.byref(nv), C.byref(tv),
            hit.ctypes.data, tri_bytes)
    if rc != 0:
        raise RuntimeError(f"oracle_count_visits: {_err()}")
    return nv.value, tv.value, hit


def random_ints(seed, n):
    out = np.zeros(n, np.int32)
    _lib.oracle_random_ints(seed, n, out.ctypes.data)
    return out


def random_floats(seed, n):
    out = np.zeros(n, np.float32)
    _lib.oracle_random_floats(seed, n, out.ctypes.data)
    return out


LIBM = {"sin": 0, "cos": 1, "exp": 2, "log": 3, "pow": 4, "asin": 5, "acos": 6, "atan": 7, "atan2": 8}


def libm(fn, x, y=None):
    """yrt_libm.h (the per-ray path's elementary functions, shared with the device) on float32 x[, y]."""
    x = np.ascontiguousarray(x, np.float32)
    y = np.ascontiguousarray(y if y is not None else np.zeros_like(x), np.float32)
    out = np.zeros_like(x)
    _lib.oracle_libm(LIBM[fn], x.size, x.ctypes.data, y.ctypes.data, out.ctypes.data)
    return out


VECMATH = {"dot": (0, 3, 3, 1), "cross": (1, 3, 3, 3), "normalize": (2, 3, 0, 3), "length": (3, 3, 0, 1),
           "lmul": (4, 9, 3, 3), "frame": (5, 3, 0, 9), "inverse": (6, 9, 0, 9), "color_div": (7, 3, 1, 3),
           "rcp": (8, 1, 0, 1), "rsqrt": (9, 1, 0, 1), "rcpps": (10, 1, 0, 1), "rsqrtps": (11, 1, 0, 1)}


def vecmath(name, a, b=None):
    """The oracle's vector helper `name` element-wise (VECMATH: fn, floats per item of a, of b, of out)."""
    fn, na, nb, no = VECMATH[name]
    a = np.ascontiguousarray(a, np.float32).reshape(-1, na)
    n = a.shape[0]
    b = np.zeros((n, max(nb, 1)), np.float32) if b is None else np.ascontiguousarray(b, np.float32).reshape(n, -1)
    out = np.zeros((n, no), np.float32)
    _lib.oracle_vecmath(fn, n, a.ctypes.data, b.ctypes.data, out.ctypes.data)
    return out if no > 1 else out[:, 0]


def bsphere(lo, hi, org, dir_):
    """AmbientLight's bounding sphere intersection: (n, 4) hit, near, far, radius."""
    arrs = [np.ascontiguousarray(x, np.float32).reshape(-1, 3) for x in (lo, hi, org, dir_)]
    out = np.zeros((arrs[0].shape[0], 4), np.float32)
    _lib.oracle_bsphere(arrs[0].shape[0], *[x.ctypes.data for x in arrs], out.ctypes.data)
    return out


def camera_rays(blob: bytes, px):
    """The frame blob camera's rays for pixel coordinates px (n, 2) = (fx, fy): org, dir (n, 3)."""
    px = np.ascontiguousarray(px, np.float32).reshape(-1, 2)
    org = np.zeros((px.shape[0], 3), np.float32)
    dir_ = np.zeros_like(org)
    if _lib.oracle_camera_rays(blob, len(blob), px.shape[0], px.ctypes.data, org.ctypes.data, dir_.ctypes.data):
        raise RuntimeError(f"oracle_camera_rays: {_err()}")
    return org, dir_


def permutations(size, seed, count):
    out = np.zeros((count, size), np.int32)
    _lib.oracle_permutations(size, seed, count, out.ctypes.data)
    return out


def shuffles(n, seed, count):
    out = np.zeros((count, n), np.uint32)
    _lib.oracle_shuffles(n, seed, count, out.ctypes.data)
    return out


def sample_table(spp, sets, iteration, num1D, num2D, filter="bspline"):
    n = _lib.oracle_sample_table(spp, sets, iteration, num1D, num2D, filter.encode(), None, 0)
    if n < 0:
        raise RuntimeError(f"oracle_sample_table: {_err()}")
    dims = 5 + num1D + 2 * num2D
    out = np.zeros(dims * n, np.float32)
    _lib.oracle_sample_table(spp, sets, iteration, num1D, num2D, filter.encode(), out.ctypes.data, out.size)
    return out.reshape(dims, n)


def pixel_sets(width, height, sets):
    out = np.zeros(width * height, np.uint8)
    _lib.oracle_pixel_sets(width, height, sets, out.ctypes.data)
    return out.reshape(height, width)


def scene_triangles(blob: bytes):
    n = _lib.oracle_scene_triangles(blob, len(blob), None, 0)
    if n < 0:
        raise RuntimeError(f"oracle_scene_triangles: {_err()}")
    out = np.zeros((n, 9), np.float32)
    _lib.oracle_scene_triangles(blob, len(blob), out.ctypes.data, n)
    return out


def cpu_count():
    """CPUs this process can use: the affinity mask, capped at the cgroup CPU quota (the GPU
    box grants a 16-CPU share of a larger host)."""
    n = len(os.sched_getaffinity(0))
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()
        if q != "max":
            n = max(1, min(n, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return n
