"""Deterministic Sponza-class atrium (BASELINE config C3 stand-in).

The reference's Sponza.DAE is absent (.MISSING_LARGE_BLOBS:11), so config C3 renders this
procedural stand-in instead: an open-roofed two-storey colonnade courtyard in Sponza's frame
(x ∈ [-19, 18] m, y ∈ [0, 15] m, z ∈ [-8, 8] m, matching the camera of
models/test_stereo_view.ecs:2-10), ≈66 k triangles, Uber materials textured with the
reference's own models/Sponza/*.JPG, hanging cloth with smooth normals, lit by the dome
(`-ambientlight 8 8 8`). Generated with seed 1234; the XML goes through the same loader as
any scene (devices/device/loaders/xml_loader.cpp restated in csrc/frontend/loaders.cpp).
"""
from __future__ import annotations

import os
from pathlib import Path

import numpy as np

SEED = 1234
HERE = Path(__file__).resolve().parent
SCENES = HERE.parent.parent / "scenes"

# BASELINE config C3 camera/params (models/test_stereo_view.ecs:2-10 Sponza block)
C3_ARGS = ["-vp", "2.25067", "8.24132", "-0.0492483", "-vi", "3.15037", "7.8048", "-0.0501832",
           "-vu", "0.436514", "0.899693", "-0.00291584", "-fov", "96.6708", "-ambientlight", "8", "8", "8",
           "-depth", "10", "-tMaxShadowRay", "120", "-renderer", "pathtracer"]


class _Mesh:
    def __init__(self, material):
        self.material = material
        self.P, self.N, self.T, self.I = [], [], [], []
        self.n = 0
        self.smooth = False

    def add(self, P, T, I, N=None):
        self.P.append(P.reshape(-1, 3))
        self.T.append(T.reshape(-1, 2))
        if N is not None:
            self.N.append(N.reshape(-1, 3))
            self.smooth = True
        self.I.append(I.reshape(-1, 3) + self.n)
        self.n += P.reshape(-1, 3).shape[0]

    def arrays(self):
        P = np.concatenate(self.P).astype(np.float32)
        T = np.concatenate(self.T).astype(np.float32)
        I = np.concatenate(self.I).astype(np.int32)
        N = np.concatenate(self.N).astype(np.float32) if self.smooth else None
        return P, N, T, I


def _grid_indices(nu, nv):
    i = np.arange(nu)[:, None]
    j = np.arange(nv)[None, :]
    a = i * (nv + 1) + j
    b = a + (nv + 1)
    t1 = np.stack([a, b, a + 1], -1)
    t2 = np.stack([a + 1, b, b + 1], -1)
    return np.concatenate([t1.reshape(-1, 3), t2.reshape(-1, 3)])


def _quad(m, origin, du, dv, nu, nv, uvscale=1.0):
    """Flat nu x nv subdivided quad origin + s*du + t*dv (geometric normals)."""
    s = np.linspace(0, 1, nu + 1)[:, None, None]
    t = np.linspace(0, 1, nv + 1)[None, :, None]
    P = np.asarray(origin) + s * np.asarray(du) + t * np.asarray(dv)
    lu, lv = np.linalg.norm(du), np.linalg.norm(dv)
    T = np.concatenate([np.broadcast_to(s * lu, P.shape[:2] + (1,)), np.broadcast_to(t * lv, P.shape[:2] + (1,))],
                       -1) / uvscale
    m.add(P, T, _grid_indices(nu, nv))


def _box(m, lo, hi, n=(2, 2, 2), uvscale=1.0):
    lo, hi = np.asarray(lo, float), np.asarray(hi, float)
    d = hi - lo
    ex, ey, ez = np.array([d[0], 0, 0]), np.array([0, d[1], 0]), np.array([0, 0, d[2]])
    _quad(m, lo, ey, ex, n[1], n[0], uvscale)           # -z
    _quad(m, lo + ez, ex, ey, n[0], n[1], uvscale)      # +z
    _quad(m, lo, ez, ey, n[2], n[1], uvscale)           # -x
    _quad(m, lo + ex, ey, ez, n[1], n[2], uvscale)      # +x
    _quad(m, lo, ex, ez, n[0], n[2], uvscale)           # -y
    _quad(m, lo + ey, ez, ex, n[2], n[0], uvscale)      # +y


def _lathe(m, base, radius_fn, y0, y1, seg, rings):
    """Surface of revolution about the vertical axis through base (smooth normals)."""
    th = np.linspace(0, 2 * np.pi, seg + 1)[None, :]
    ys = np.linspace(y0, y1, rings + 1)[:, None]
    shape = (rings + 1, seg + 1)
    r = np.broadcast_to(radius_fn((ys - y0) / (y1 - y0)), (rings + 1, 1))
    dr = np.gradient(r[:, 0], ys[:, 0])[:, None]
    P = np.stack([base[0] + r * np.cos(th), np.broadcast_to(ys, shape), base[2] + r * np.sin(th)], -1)
    N = np.stack([np.broadcast_to(np.cos(th), shape), np.broadcast_to(-dr, shape),
                  np.broadcast_to(np.sin(th), shape)], -1)
    N = N / np.linalg.norm(N, axis=-1, keepdims=True)
    T = np.stack([np.broadcast_to(th / np.pi, shape), np.broadcast_to(ys / 2.0, shape)], -1)
    m.add(P, T, _grid_indices(rings, seg), N)


def _arch(m, x0, x1, z, y_spring, depth, thick, seg):
    """Semicircular arch between two column centres in the plane z (extruded along z)."""
    cx, r = 0.5 * (x0 + x1), 0.5 * (x1 - x0)
    a = np.linspace(np.pi, 0, seg + 1)
    inner = np.stack([cx + r * np.cos(a), y_spring + r * np.sin(a)], -1)
    outer = np.stack([cx + (r + thick) * np.cos(a), y_spring + (r + thick) * np.sin(a)], -1)
    for zz in (z - depth / 2, z + depth / 2):      # two faces: annulus strip
        P = np.stack([np.stack([inner[:, 0], inner[:, 1], np.full(seg + 1, zz)], -1),
                      np.stack([outer[:, 0], outer[:, 1], np.full(seg + 1, zz)], -1)], 1)
        T = P[..., :2] / 2.0
        m.add(P, T, _grid_indices(seg, 1))
    for curve in (inner, outer):                  # soffit / extrados
        P = np.stack([np.stack([curve[:, 0], curve[:, 1], np.full(seg + 1, z - depth / 2)], -1),
                      np.stack([curve[:, 0], curve[:, 1], np.full(seg + 1, z + depth / 2)], -1)], 1)
        T = np.stack([np.linspace(0, 3, seg + 1)[:, None] * np.ones((1, 2)), np.array([[0, 1]]) * np.ones((seg + 1, 1))],
                     -1)
        m.add(P, T, _grid_indices(seg, 1))


def _curtain(m, rng, x0, x1, z, ytop, ybot, nu, nv):
    """Draped cloth: folds along x, billowing toward the courtyard (smooth normals)."""
    u = np.linspace(0, 1, nu + 1)[:, None]
    v = np.linspace(0, 1, nv + 1)[None, :]
    k = rng.integers(5, 9)
    ph = rng.uniform(0, 2 * np.pi)
    amp = 0.12 + 0.25 * v                     # folds deepen toward the hem
    sway = 0.35 * np.sin(np.pi * v) * np.sign(-z)
    X = x0 + (x1 - x0) * u + 0.0 * v
    Y = ytop - (ytop - ybot) * v + 0.15 * np.cos(np.pi * (2 * u - 1)) * v ** 2 + 0.0 * u
    Z = z + amp * np.sin(2 * np.pi * k * u + ph) + sway + 0.0 * u
    P = np.stack([X, Y, Z], -1)
    du = np.gradient(P, axis=0)
    dv = np.gradient(P, axis=1)
    N = np.cross(du, dv)
    N /= np.linalg.norm(N, axis=-1, keepdims=True)
    T = np.stack([np.broadcast_to(u, X.shape) * 4, np.broadcast_to(v, X.shape) * 4], -1)
    m.add(P, T, _grid_indices(nu, nv), N)


def build_meshes():
    rng = np.random.default_rng(SEED)
    floor = _Mesh(("KAMEN.JPG", None))
    walls = _Mesh(("x01_st.JPG", None))
    columns = _Mesh(("KAMEN-stup.JPG", None))
    arches = _Mesh(("sp_luk.JPG", None))
    slabs = _Mesh(("01_STUB.JPG", None))
    trims = _Mesh(("00_skap.JPG", None))
    cloth = [_Mesh((None, c)) for c in ((0.55, 0.08, 0.06), (0.10, 0.35, 0.12), (0.12, 0.14, 0.45))]

    X0, X1, Z = -19.0, 18.0, 8.0
    _quad(floor, (X0, 0, -Z), (0, 0, 2 * Z), (X1 - X0, 0, 0), 40, 96, 2.0)
    for s in (-1, 1):
        _quad(walls, (X0, 0, s * Z), (X1 - X0, 0, 0) if s < 0 else (0, 15, 0),
              (0, 15, 0) if s < 0 else (X1 - X0, 0, 0), *((64, 24) if s < 0 else (24, 64)), 3.0)
    _quad(walls, (X0, 0, -Z), (0, 15, 0), (0, 0, 2 * Z), 24, 32, 3.0)
    _quad(walls, (X1, 0, -Z), (0, 0, 2 * Z), (0, 15, 0), 32, 24, 3.0)

    xs = np.linspace(-16.0, 15.0, 11)
    for s in (-1, 1):
        zc = s * 4.6
        for storey, (y0, y1, rad) in enumerate(((0.0, 4.6, 0.42), (6.2, 10.4, 0.32))):
            for x in xs:
                jit = rng.uniform(-0.01, 0.01)
                _lathe(columns, (x + jit, 0, zc), lambda t, r=rad: r * (1.0 - 0.08 * t + 0.05 * np.sin(9 * t)),
                       y0 + 0.3, y1 - 0.35, 20, 9)
                _lathe(columns, (x + jit, 0, zc), lambda t, r=rad: r * (1.0 + 0.6 * t), y1 - 0.35, y1, 20, 2)
                _box(trims, (x - rad - 0.15, y0, zc - rad - 0.15), (x + rad + 0.15, y0 + 0.3, zc + rad + 0.15),
                     (2, 1, 2))
            for a, b in zip(xs[:-1], xs[1:]):
                _arch(arches, a, b, zc, y1, 0.7 if storey == 0 else 0.5, 0.45, 16)
        # gallery slabs and parapets between colonnade and outer wall
        for y in (6.0, 11.6):
            _box(slabs, (X0, y - 0.25, min(zc, s * Z)), (X1, y, max(zc, s * Z)), (48, 1, 4), 3.0)
            _box(trims, (X0, y, zc - 0.15), (X1, y + 1.0, zc + 0.15), (64, 2, 1), 1.5)
        # cornice at the roof line
        _box(trims, (X0, 14.6, s * Z - s * 0.8 - 0.0 if s > 0 else -Z), (X1, 15.0, Z if s > 0 else -Z + 0.8),
             (96, 1, 2), 1.5)
        # curtains hanging in the upper gallery bays
        for k, (a, b) in enumerate(zip(xs[1:-1:2], xs[2::2])):
            _curtain(cloth[(k + (s > 0)) % 3], rng, a + 0.4, b - 0.4, zc + s * 0.7, 10.2, 6.6, 48, 16)
    return [floor, walls, columns, arches, slabs, trims] + cloth


def _fmt(a):
    return " ".join("%.9g" % v for v in np.asarray(a).reshape(-1))


def write_xml(path: Path | None = None) -> Path:
    """Writes the stand-in scene XML (textures referenced from scenes/Sponza)."""
    path = Path(path) if path else SCENES / "_generated" / "sponza_standin.xml"
    path.parent.mkdir(parents=True, exist_ok=True)
    tex_dir = SCENES / "Sponza"
    out = ["<?xml version=\"1.0\"?>", "<scene>", "  <Group>"]
    for m in build_meshes():
        P, N, T, I = m.arrays()
        tex, color = m.material
        out.append("    <TriangleMesh>")
        out.append("      <positions>" + _fmt(P) + "</positions>")
        if N is not None:
            out.append("      <normals>" + _fmt(N) + "</normals>")
        out.append("      <texcoords>" + _fmt(T) + "</texcoords>")
        out.append("      <triangles>" + " ".join(map(str, I.reshape(-1))) + "</triangles>")
        out.append("      <material>\n        <code>\"Uber\"</code>\n        <parameters>")
        if tex:
            rel = Path("..") / tex_dir.name / tex if path.parent.parent == tex_dir.parent else tex_dir / tex
            out.append(f"          <texture name=\"Kd\">\"{rel}\"</texture>")
        else:
            out.append("          <float3 name=\"diffuse\">%g %g %g</float3>" % color)
            out.append("          <float name=\"reflectivity\">0.08</float>")
        out.append("          <float2 name=\"s0\">0 0</float2>\n          <float2 name=\"ds\">1 1</float2>")
        out.append("        </parameters>\n      </material>\n    </TriangleMesh>")
    out += ["  </Group>", "</scene>", ""]
    tmp = path.with_suffix(f".{os.getpid()}.tmp")  # per process: concurrent writers never share it
    tmp.write_text("\n".join(out))
    tmp.replace(path)
    return path


def triangle_count() -> int:
    return sum(m.arrays()[3].shape[0] for m in build_meshes())


if __name__ == "__main__":
    p = write_xml()
    print(p, triangle_count())
