"""Deterministic 22 Frederick St. interior stand-in (BASELINE config C5).

The reference's own scene `sample_scene/22_Frederick_St_good_tempo_to_execute.dae.zip` is
absent (.MISSING_LARGE_BLOBS:13); its 152 textures are present. BASELINE.md:56 prescribes a
procedural interior stand-in with seed 2217, so config C5 renders this instead: a furnished
open-plan apartment (living room, kitchen/dining, hallway; ≈140 k triangles) written as a
SketchUp-style COLLADA 1.4.1 file — inches, Z_UP, `<lambert>`/`<phong>` effects with diffuse
textures taken from the reference's own `sample_scene/22 Frederick St. good_tempo/` (copied to
scenes/frederick/), A_ONE-transparent window glass (ThinDielectric), GOOGLEEARTH double-sided
foliage and curtains, two `YULIO_FPR_VIEW_` cameras and a `YULIO_CAMERA_ALIGNED_` cut-out
billboard. It goes through the same Collada loader and FPR stereo loop as a real Yulio export
(StartRT, devices/renderer/renderer.cpp:543-737; devices/device/loaders/ColladaLoader.cpp).
Lighting is the DLL's: the dome light `ambientlight` (.83 .95 .98) through the windows, shadow
rays 120 in long (tMaxShadowRay x sceneScale).
"""
from __future__ import annotations

import math
import os
from pathlib import Path

import numpy as np

SEED = 2217
HERE = Path(__file__).resolve().parent
SCENES = HERE.parent.parent / "scenes"
TEX = SCENES / "frederick"
UNIT = 0.0254  # SketchUp exports inches
H_CEIL = 108.0

# name: (texture or None, diffuse rgb, reflectivity (Collada, inverted by the loader), transparent alpha
# or None, double sided, texture tile size in inches)
MATERIALS = {
    "floor_wood": ("PDM_Wood_floor_Cherry_01.jpg", None, 1.0, None, False, 72.0),
    "floor_kitchen": ("PDM_Concrete_09.jpg", None, 1.0, None, False, 48.0),
    "wall_paint": (None, (0.82, 0.80, 0.74), 1.0, None, False, 0),
    "wall_brick": ("Brick_Antique_01.jpg", None, 1.0, None, False, 48.0),
    "ceiling": (None, (0.88, 0.88, 0.86), 1.0, None, False, 0),
    "trim": (None, (0.92, 0.92, 0.90), 0.85, None, False, 0),
    "rug": ("Carpet_Plush_Charcoal.jpg", None, 1.0, None, False, 24.0),
    "fabric": ("Turner_-_Chinchilla.jpg", None, 1.0, None, False, 18.0),
    "wood": ("Wood_Cherry_Original.jpg", None, 0.9, None, False, 24.0),
    "cabinet": ("Wood_Board_Cork.jpg", None, 1.0, None, False, 24.0),
    "steel": ("PDM_Stainless_steel.jpg", None, 0.55, None, False, 30.0),
    "aluminum": ("Metal_Aluminum_Anodized.jpg", None, 0.7, None, False, 12.0),
    "sink": ("Kitchen_Sink.jpg", None, 0.6, None, False, 24.0),
    "book_cover": ("Notebook_Cover.jpg", None, 1.0, None, False, 10.0),
    "cardboard": ("Cardboard_Texture.jpg", None, 1.0, None, False, 20.0),
    "curtain": ("Mesh_-_Sterling.jpg", None, 1.0, None, True, 30.0),
    "screen": ("iMac.jpeg", None, 0.8, None, False, 0),
    "picture": ("PDM_Picture_01_MacBook.jpg", None, 0.9, None, False, 0),
    "leaf": (None, (0.18, 0.42, 0.14), 1.0, None, True, 0),
    "pot": (None, (0.62, 0.32, 0.20), 0.9, None, False, 0),
    "lampshade": (None, (0.95, 0.90, 0.78), 1.0, None, True, 0),
    "ground": ("PDM_Concrete_09.jpg", None, 1.0, None, False, 200.0),
    "glass": (None, (0.85, 0.92, 0.95), 0.9, 0.25, False, 0),
    "cutout": ("material_77.png", None, 1.0, None, True, 0),
    "book_red": (None, (0.55, 0.10, 0.08), 1.0, None, False, 0),
    "book_blue": (None, (0.10, 0.18, 0.45), 1.0, None, False, 0),
    "book_green": (None, (0.12, 0.35, 0.18), 1.0, None, False, 0),
    "book_cream": (None, (0.85, 0.80, 0.65), 1.0, None, False, 0),
    "ceramic": (None, (0.90, 0.88, 0.84), 0.8, None, False, 0),
}

# FPR views: name -> (eye, target) in file coordinates (inches, Z up)
CAMERAS = {
    "Living": ((150.0, 70.0, 64.0), (150.0, 200.0, 58.0)),
    "Kitchen": ((372.0, 80.0, 64.0), (456.0, 110.0, 52.0)),
}


class Mesh:
    def __init__(self):
        self.P, self.N, self.T, self.I = [], [], [], []
        self.n = 0

    def add(self, P, N, T, I):
        P = np.asarray(P, np.float64).reshape(-1, 3)
        self.P.append(P)
        self.N.append(np.asarray(N, np.float64).reshape(-1, 3))
        self.T.append(np.asarray(T, np.float64).reshape(-1, 2))
        self.I.append(np.asarray(I, np.int64).reshape(-1, 3) + self.n)
        self.n += P.shape[0]

    def arrays(self):
        return (np.concatenate(self.P), np.concatenate(self.N), np.concatenate(self.T), np.concatenate(self.I))

    @property
    def triangles(self):
        return sum(i.shape[0] for i in self.I)


def _grid(nu, nv):
    i = np.arange(nu)[:, None]
    j = np.arange(nv)[None, :]
    a = i * (nv + 1) + j
    b = a + (nv + 1)
    return np.concatenate([np.stack([a, b, a + 1], -1).reshape(-1, 3), np.stack([a + 1, b, b + 1], -1).reshape(-1, 3)])


class Builder:
    def __init__(self):
        self.meshes: dict[str, Mesh] = {}
        self.rng = np.random.default_rng(SEED)

    def m(self, mat):
        return self.meshes.setdefault(mat, Mesh())

    def quad(self, mat, o, du, dv, nu=1, nv=1, tile=None, flip=False):
        """Flat quad o + s du + t dv, normal du x dv (or its negation), nu x nv cells."""
        o, du, dv = (np.asarray(x, np.float64) for x in (o, du, dv))
        s = np.linspace(0, 1, nu + 1)[:, None, None]
        t = np.linspace(0, 1, nv + 1)[None, :, None]
        P = o + s * du + t * dv
        n = np.cross(du, dv)
        n /= np.linalg.norm(n)
        tile = tile if tile is not None else (MATERIALS[mat][5] or 0)
        if tile:
            T = np.concatenate([np.broadcast_to(s * np.linalg.norm(du), P.shape[:2] + (1,)),
                                np.broadcast_to(t * np.linalg.norm(dv), P.shape[:2] + (1,))], -1) / tile
        else:
            T = np.concatenate([np.broadcast_to(s, P.shape[:2] + (1,)), np.broadcast_to(t, P.shape[:2] + (1,))], -1)
        I = _grid(nu, nv)
        if flip:
            I = I[:, ::-1]
            n = -n
        self.m(mat).add(P, np.broadcast_to(n, P.shape), T, I)

    def box(self, mat, lo, hi, cell=None):
        """Axis-aligned box, outward faces; `cell` subdivides faces into ~cell-inch cells."""
        lo, hi = np.asarray(lo, np.float64), np.asarray(hi, np.float64)
        d = hi - lo
        ex, ey, ez = np.array([d[0], 0, 0]), np.array([0, d[1], 0]), np.array([0, 0, d[2]])

        def k(a, b):
            if not cell:
                return 1, 1
            return max(1, int(round(a / cell))), max(1, int(round(b / cell)))
        self.quad(mat, lo, ey, ex, *k(d[1], d[0]))            # -z
        self.quad(mat, lo + ez, ex, ey, *k(d[0], d[1]))       # +z
        self.quad(mat, lo, ez, ey, *k(d[2], d[1]))            # -x
        self.quad(mat, lo + ex, ey, ez, *k(d[1], d[2]))       # +x
        self.quad(mat, lo, ex, ez, *k(d[0], d[2]))            # -y
        self.quad(mat, lo + ey, ez, ex, *k(d[2], d[0]))       # +y

    def lathe(self, mat, base, radius, z0, z1, seg=32, rings=8, cap=False):
        """Surface of revolution about the vertical axis through base; radius(t), t in [0, 1]."""
        th = np.linspace(0, 2 * np.pi, seg + 1)[None, :]
        ts = np.linspace(0, 1, rings + 1)[:, None]
        r = np.asarray(radius(ts), np.float64) * np.ones_like(ts)
        z = z0 + (z1 - z0) * ts
        dr = np.gradient(r[:, 0], z[:, 0]) if rings > 0 else np.zeros(rings + 1)
        shape = (rings + 1, seg + 1)
        P = np.stack([base[0] + r * np.cos(th), base[1] + r * np.sin(th), np.broadcast_to(z, shape)], -1)
        N = np.stack([np.broadcast_to(np.cos(th), shape), np.broadcast_to(np.sin(th), shape),
                      np.broadcast_to(-dr[:, None], shape)], -1)
        N /= np.linalg.norm(N, axis=-1, keepdims=True)
        T = np.stack([np.broadcast_to(th / (2 * np.pi), shape), np.broadcast_to(ts, shape)], -1)
        self.m(mat).add(P, N, T, _grid(rings, seg)[:, ::-1])
        if cap:  # flat top disk
            rr = r[-1, 0]
            a = np.linspace(0, 2 * np.pi, seg + 1)[:-1]
            P = np.concatenate([[[base[0], base[1], z1]], np.stack([base[0] + rr * np.cos(a), base[1] + rr * np.sin(a),
                                                                     np.full(seg, z1)], -1)])
            I = np.stack([np.zeros(seg, int), 1 + np.arange(seg), 1 + (np.arange(seg) + 1) % seg], -1)
            self.m(mat).add(P, np.broadcast_to([0, 0, 1.0], P.shape), P[:, :2] / 24.0, I)

    def cylinder(self, mat, base, r, z0, z1, seg=16):
        self.lathe(mat, base, lambda t: r, z0, z1, seg, 1, cap=True)

    def sheet(self, mat, P, nu, nv, tile=24.0):
        """Smooth grid surface from a (nu+1, nv+1, 3) point array (normals from the grid)."""
        du = np.gradient(P, axis=0)
        dv = np.gradient(P, axis=1)
        N = np.cross(du, dv)
        N /= np.maximum(np.linalg.norm(N, axis=-1, keepdims=True), 1e-12)
        s = np.linspace(0, 1, nu + 1)[:, None]
        t = np.linspace(0, 1, nv + 1)[None, :]
        ext = (np.linalg.norm(P[-1, 0] - P[0, 0]), np.linalg.norm(P[0, -1] - P[0, 0]))
        T = np.stack([np.broadcast_to(s * ext[0] / tile, P.shape[:2]), np.broadcast_to(t * ext[1] / tile, P.shape[:2])], -1)
        self.m(mat).add(P, N, T, _grid(nu, nv))


# ------------------------------------------------------------------ the apartment
def _walls(b: Builder):
    t = 6.0
    X1, Y1 = 456.0, 216.0
    # floor finishes, ceiling slab, outer ground
    b.quad("floor_wood", (0, 0, 0), (288, 0, 0), (0, Y1, 0), 48, 36)
    b.quad("floor_kitchen", (288, 0, 0), (X1 - 288, 0, 0), (0, Y1, 0), 28, 36)
    b.quad("floor_wood", (0, Y1, 0), (120, 0, 0), (0, 84, 0), 20, 14)
    b.box("ceiling", (-t, -t, H_CEIL), (X1 + t, 300 + t, H_CEIL + 8), cell=24)
    b.box("ceiling", (-t, -t, -8), (X1 + t, 300 + t, 0), cell=48)
    b.quad("ground", (-2000, -2000, -130), (4000 + X1, 0, 0), (0, 4000 + Y1, 0), 8, 8)

    def wall_x(y0, y1, x0, x1, openings, mat="wall_paint"):
        """Wall along x from x0 to x1, thickness y0..y1, with openings (xa, xb, za, zb)."""
        xs = x0
        for xa, xb, za, zb in sorted(openings):
            b.box(mat, (xs, y0, 0), (xa, y1, H_CEIL), cell=24)
            if za > 0:
                b.box(mat, (xa, y0, 0), (xb, y1, za), cell=24)
            b.box(mat, (xa, y0, zb), (xb, y1, H_CEIL), cell=24)
            xs = xb
        b.box(mat, (xs, y0, 0), (x1, y1, H_CEIL), cell=24)

    def wall_y(x0, x1, y0, y1, openings, mat="wall_paint"):
        ys = y0
        for ya, yb, za, zb in sorted(openings):
            b.box(mat, (x0, ys, 0), (x1, ya, H_CEIL), cell=24)
            if za > 0:
                b.box(mat, (x0, ya, 0), (x1, yb, za), cell=24)
            b.box(mat, (x0, ya, zb), (x1, yb, H_CEIL), cell=24)
            ys = yb
        b.box(mat, (x0, ys, 0), (x1, y1, H_CEIL), cell=24)

    wins_s = [(30, 102, 30, 90), (126, 198, 30, 90), (222, 270, 30, 90), (318, 414, 36, 90)]
    wall_x(-t, 0, -t, X1 + t, wins_s)
    wall_y(X1, X1 + t, 0, Y1 + 84, [(120, 180, 40, 86)])
    wall_y(-t, 0, 0, 300, [], mat="wall_brick")
    wall_x(Y1, Y1 + t, 120, X1, [(300, 336, 0, 84)])
    wall_x(Y1, Y1 + t, 0, 120, [(40, 80, 0, 84)])
    wall_x(300, 300 + t, -t, 126, [])
    wall_y(120, 126, Y1, 300, [(240, 276, 0, 84)])
    wall_y(288, 294, 0, Y1, [(48, 168, 0, 84)])   # living | kitchen partition with a wide opening
    # window glass and frames
    for xa, xb, za, zb in wins_s:
        b.quad("glass", (xa, -3, za), (xb - xa, 0, 0), (0, 0, zb - za))
        for z in (za, zb - 1.5):
            b.box("trim", (xa, -4, z), (xb, -2, z + 1.5))
        for x in (xa, (xa + xb) / 2 - 0.75, xb - 1.5):
            b.box("trim", (x, -4, za), (x + 1.5, -2, zb))
    b.quad("glass", (X1 + 3, 120, 40), (0, 60, 0), (0, 0, 46))
    # skirting boards
    for (x0, y0, x1, y1) in ((0, 0, 288, 0.75), (0, Y1 - 0.75, 288, Y1), (0.0, 0, 0.75, Y1), (294, 0, X1, 0.75)):
        b.box("trim", (x0, y0, 0), (x1, y1, 4))


def _curtain(b: Builder, x0, x1, y, z0, z1, nu=96, nv=48):
    rng = b.rng
    u = np.linspace(0, 1, nu + 1)[:, None]
    v = np.linspace(0, 1, nv + 1)[None, :]
    k = rng.integers(9, 14)
    ph = rng.uniform(0, 2 * np.pi)
    amp = 1.2 + 1.3 * (1 - v)
    X = x0 + (x1 - x0) * u + 0 * v
    Y = y + amp * np.sin(2 * np.pi * k * u + ph) + 0 * v
    Z = z1 - (z1 - z0) * (1 - v) + 0 * u
    b.sheet("curtain", np.stack([X, Y, Z], -1), nu, nv, tile=30.0)


def _plant(b: Builder, x, y, h=40.0, leaves=220):
    rng = b.rng
    b.lathe("pot", (x, y), lambda t: 7 + 3 * t - 1.5 * t * t, 0, 14, 40, 10, cap=False)
    b.cylinder("cardboard", (x, y), 8.2, 12.5, 13.0, 24)  # soil
    for _ in range(leaves):
        a = rng.uniform(0, 2 * np.pi)
        lift = rng.uniform(0.25, 1.0)
        base = np.array([x + rng.normal(0, 1.5), y + rng.normal(0, 1.5), 13 + h * lift * rng.uniform(0.2, 0.8)])
        L, W = rng.uniform(7, 13), rng.uniform(1.6, 3.0)
        d = np.array([math.cos(a), math.sin(a), rng.uniform(0.1, 0.7)])
        d /= np.linalg.norm(d)
        side = np.cross(d, [0, 0, 1.0])
        side /= np.linalg.norm(side)
        s = np.linspace(0, 1, 5)[:, None, None]
        w = np.linspace(-1, 1, 3)[None, :, None]
        P = base + s * L * d + w * (W * np.sin(np.pi * np.clip(s, 0.05, 1))) * side - (s ** 2) * np.array([0, 0, 3.0])
        b.sheet("leaf", P, 4, 2, tile=8.0)


def _bookshelf(b: Builder, x0, y0, y1, h=84.0, shelves=6):
    rng = b.rng
    d = 12.0
    b.box("wood", (x0, y0, 0), (x0 + d, y0 + 1, h))
    b.box("wood", (x0, y1 - 1, 0), (x0 + d, y1, h))
    b.box("wood", (x0, y0, 0), (x0 + 0.75, y1, h))
    colors = ["book_red", "book_blue", "book_green", "book_cream", "book_cover"]
    for k in range(shelves + 1):
        z = k * (h - 1) / shelves
        b.box("wood", (x0, y0 + 1, z), (x0 + d, y1 - 1, z + 1))
        if k == shelves:
            break
        y = y0 + 1.5
        while True:
            w = rng.uniform(0.8, 2.2)
            bh = rng.uniform(7, min(12, (h - 1) / shelves - 2))
            if y + w > y1 - 1.5:
                break
            if rng.uniform() < 0.08:  # gap
                y += w
                continue
            dd = rng.uniform(6, 9)
            b.box(colors[rng.integers(len(colors))], (x0 + 1, y, z + 1), (x0 + 1 + dd, y + w, z + 1 + bh))
            y += w + 0.05


def _chair(b: Builder, x, y, rot):
    c, s = math.cos(rot), math.sin(rot)

    def P(dx, dy):
        return (x + c * dx - s * dy, y + s * dx + c * dy)
    for dx, dy in ((-8, -8), (8, -8), (-8, 8), (8, 8)):
        b.cylinder("wood", P(dx, dy), 0.8, 0, 18, 12)
    lo = np.array(P(-9.5, -9.5))
    hi = np.array(P(9.5, 9.5))
    b.box("fabric", (min(lo[0], hi[0]), min(lo[1], hi[1]), 18), (max(lo[0], hi[0]), max(lo[1], hi[1]), 20.5), cell=4)
    bx = np.array([P(-9.5, 8), P(9.5, 9.5)])
    b.box("wood", (bx[:, 0].min(), bx[:, 1].min(), 20.5), (bx[:, 0].max(), bx[:, 1].max(), 36))


def _lamp(b: Builder, x, y):
    b.cylinder("aluminum", (x, y), 7, 0, 1.2, 32)
    b.cylinder("aluminum", (x, y), 0.6, 1.2, 58, 12)
    b.lathe("lampshade", (x, y), lambda t: 9 - 3.5 * t, 54, 66, 48, 12)


def _vase(b: Builder, x, y, z, h, r, mat="ceramic"):
    b.lathe(mat, (x, y), lambda t: r * (0.55 + 0.5 * np.sin(np.pi * (0.15 + 0.8 * t)) - 0.25 * t), z, z + h, 64, 32)


def _living(b: Builder):
    rng = b.rng
    b.box("rug", (40, 70, 0), (220, 170, 0.6), cell=12)
    # sofa: base, seat and back cushions, arms
    b.box("fabric", (50, 168, 0), (190, 204, 15), cell=6)
    for k in range(3):
        x0 = 56 + k * 43
        b.box("fabric", (x0 + 0.5, 170, 15), (x0 + 42.5, 198, 21), cell=3)
        b.box("fabric", (x0 + 0.5, 194, 21), (x0 + 42.5, 204, 40), cell=3)
    for x0 in (50, 184):
        b.box("fabric", (x0, 168, 15), (x0 + 6, 204, 27), cell=4)
    # throw pillows: squashed lathes
    for px in (64, 176):
        b.lathe("book_red", (px, 190), lambda t: 7 * np.sin(np.pi * np.clip(t, 0.02, 0.98)) + 0.5, 21, 35, 32, 16)
    # coffee table
    b.box("wood", (90, 100, 15), (150, 130, 16.5))
    b.box("wood", (92, 102, 5), (148, 128, 6))
    for x, y in ((92, 102), (148, 102), (92, 128), (148, 128)):
        b.cylinder("wood", (x, y), 1.0, 0, 15, 12)
    _vase(b, 110, 115, 16.5, 10, 3.5)
    b.box("book_cover", (126, 108, 16.5), (139, 118, 17.5))
    b.box("book_blue", (127, 109, 17.5), (138, 117, 18.4))
    # TV console and TV
    b.box("cabinet", (90, 6, 0), (190, 22, 20), cell=6)
    b.box("aluminum", (108, 12, 20), (172, 16, 21))
    b.box("aluminum", (138, 13, 21), (142, 15, 26))
    b.box("aluminum", (110, 12.5, 26), (170, 14.5, 60))
    b.quad("screen", (111, 12.4, 27), (58, 0, 0), (0, 0, 32), flip=True)
    # armchairs
    b.box("fabric", (214, 96, 0), (246, 130, 16), cell=4)
    b.box("fabric", (240, 96, 16), (246, 130, 36), cell=4)
    b.box("fabric", (214, 96, 16), (246, 100, 24), cell=4)
    b.box("fabric", (214, 126, 16), (246, 130, 24), cell=4)
    _bookshelf(b, 0, 24, 132)
    _lamp(b, 34, 190)
    _lamp(b, 204, 190)
    _plant(b, 264, 28)
    _plant(b, 20, 160, h=30, leaves=160)
    # pictures on the north wall
    for x0, w, h in ((70, 40, 26), (128, 30, 40), (176, 24, 18)):
        b.box("wood", (x0 - 1, Y_N - 1.5, 52), (x0 + w + 1, Y_N, 53 + h + 1))
        b.quad("picture", (x0, Y_N - 1.6, 53), (w, 0, 0), (0, 0, h))
    # curtains at the living-room windows
    for xa, xb in ((24, 108), (120, 204), (216, 276)):
        _curtain(b, xa, xb, 4.0, 0.5, 100)
    # a sculpture on a plinth: displaced sphere (dense, smooth)
    b.box("trim", (250, 180, 0), (266, 196, 32))
    nu, nv = 96, 64
    th = np.linspace(0, np.pi, nv + 1)[None, :]
    ph = np.linspace(0, 2 * np.pi, nu + 1)[:, None]
    rr = 6 + 0.9 * np.sin(5 * ph) * np.sin(4 * th) + 0.4 * np.cos(9 * th)
    P = np.stack([258 + rr * np.sin(th) * np.cos(ph), 188 + rr * np.sin(th) * np.sin(ph), 39 - rr * np.cos(th)], -1)
    b.sheet("steel", P, nu, nv, tile=12.0)


Y_N = 216.0


def _kitchen(b: Builder):
    rng = b.rng
    X1 = 456.0
    # counter run along the east wall and the north wall, cabinets under, uppers above
    b.box("cabinet", (430, 10, 0), (X1, 206, 34), cell=8)
    b.box("steel", (428, 8, 34), (X1, 208, 35.5), cell=8)
    b.box("cabinet", (300, 184, 0), (430, 210, 34), cell=8)
    b.box("steel", (300, 182, 34), (430, 210, 35.5), cell=8)
    b.box("cabinet", (440, 10, 54), (X1, 116, 90), cell=8)
    b.box("cabinet", (440, 184, 54), (X1, 206, 90), cell=8)
    for y in np.arange(14, 200, 16.0):  # handles
        b.cylinder("aluminum", (429.2, y), 0.4, 26, 31, 8)
    # sink
    b.box("sink", (432, 130, 27), (452, 152, 35.6))
    b.cylinder("steel", (452, 141), 0.7, 35.5, 48, 16)
    b.box("steel", (442, 140.3, 46.5), (452, 141.7, 48))
    # fridge
    b.box("steel", (300, 186, 0), (334, 214, 72), cell=6)
    b.box("aluminum", (302, 185, 36), (303, 186, 60))
    # island with stools
    b.box("cabinet", (350, 60, 0), (410, 96, 34), cell=6)
    b.box("wood", (346, 56, 34), (414, 100, 36))
    for x in (358, 380, 402):
        b.lathe("aluminum", (x, 48), lambda t: 5.5 - 4.6 * t + 1.2 * t * t, 0, 26, 24, 6)
        b.cylinder("fabric", (x, 48), 7.0, 26, 28.5, 32)
    # dining table and chairs
    b.box("wood", (322, 120, 29), (414, 162, 30.5))
    for x, y in ((326, 124), (410, 124), (326, 158), (410, 158)):
        b.cylinder("wood", (x, y), 1.2, 0, 29, 12)
    for k, x in enumerate((338, 368, 398)):
        _chair(b, x, 112, 0.0)
        _chair(b, x, 170, math.pi)
    for x in (350, 386):  # pendant lamps
        b.cylinder("aluminum", (x, 141), 0.15, 78, H_CEIL, 6)
        b.lathe("lampshade", (x, 141), lambda t: 1.5 + 8 * t * t, 66, 78, 48, 12)
    # kitchen clutter: bowls, jars, a plant, moving boxes
    for _ in range(10):
        x, y = rng.uniform(432, 452), rng.uniform(20, 120)
        _vase(b, x, y, 35.5, rng.uniform(3, 9), rng.uniform(1.5, 3), "ceramic")
    _vase(b, 380, 80, 36, 6, 6, "ceramic")
    _plant(b, 300, 24, h=34, leaves=180)


def _hallway(b: Builder):
    rng = b.rng
    for k in range(9):  # a stack of moving boxes
        x0 = 10 + (k % 3) * 26 + rng.uniform(-2, 2)
        y0 = 250 + rng.uniform(-3, 3)
        z0 = (k // 3) * 18
        b.box("cardboard", (x0, y0, z0), (x0 + 24, y0 + 20, z0 + 17.8), cell=6)
    b.box("wood", (60, 276, 0), (110, 294, 30))
    _vase(b, 90, 285, 30, 12, 3, "ceramic")


def _cutout(b: Builder):
    """YULIO_CAMERA_ALIGNED_ billboard (faceCamera): a vertical textured card."""
    return np.array([[-12, 0, 0], [12, 0, 0], [12, 0, 66], [-12, 0, 66]], np.float64)


def build() -> Builder:
    b = Builder()
    _walls(b)
    _living(b)
    _kitchen(b)
    _hallway(b)
    return b


def triangle_count() -> int:
    return sum(m.triangles for m in build().meshes.values()) + 2


# ------------------------------------------------------------------ COLLADA writer
def _f(a, fmt="%.6g"):
    return " ".join(fmt % v for v in np.asarray(a, np.float64).reshape(-1))


def _lookat(pos, dst, up=(0, 0, 1.0)):
    pos, dst, up = (np.asarray(v, np.float64) for v in (pos, dst, up))
    d = (dst - pos) / np.linalg.norm(dst - pos)
    r = np.cross(d, up)
    r /= np.linalg.norm(r)
    u = np.cross(r, d)
    m = np.eye(4)
    m[:3, 0], m[:3, 1], m[:3, 2], m[:3, 3] = r, u, -d, pos
    return m


def write_dae(path: Path | None = None) -> Path:
    """Writes the stand-in .dae (texture paths relative to scenes/frederick); returns it."""
    path = Path(path) if path else SCENES / "_generated" / "frederick_standin.dae"
    path.parent.mkdir(parents=True, exist_ok=True)
    b = build()
    rel = os.path.relpath(TEX, path.parent)
    imgs, fx, mats, geos, nodes = [], [], [], [], []
    for name, (tex, col, refl, alpha, ds, _tile) in MATERIALS.items():
        if tex:
            imgs.append(f'<image id="img_{name}"><init_from>{rel}/{tex}</init_from></image>')
            diffuse = f'<diffuse><texture texture="{name}-sampler" texcoord="UVSET0"/></diffuse>'
            params = (f'<newparam sid="{name}-surface"><surface type="2D"><init_from>img_{name}</init_from></surface>'
                      f'</newparam><newparam sid="{name}-sampler"><sampler2D><source>{name}-surface</source>'
                      f'</sampler2D></newparam>')
        else:
            diffuse = f'<diffuse><color>{_f(col)} 1</color></diffuse>'
            params = ""
        extra = ""
        if alpha is not None:
            extra += f'<transparent opaque="A_ONE"><color>1 1 1 {alpha}</color></transparent>'
        body = f'{diffuse}<reflectivity><float>{refl}</float></reflectivity>{extra}'
        shade = "phong" if refl < 1.0 else "lambert"
        ds_xml = '<extra><technique profile="GOOGLEEARTH"><double_sided>1</double_sided></technique></extra>' if ds else ""
        fx.append(f'<effect id="fx_{name}"><profile_COMMON>{params}<technique sid="common"><{shade}>{body}</{shade}>'
                  f'</technique>{ds_xml}</profile_COMMON></effect>')
        mats.append(f'<material id="mat_{name}" name="{name}"><instance_effect url="#fx_{name}"/></material>')

    def geometry(gid, gname, P, N, T, I, mat):
        n = len(P)
        geos.append(
            f'<geometry id="{gid}" name="{gname}"><mesh>'
            f'<source id="{gid}-p"><float_array id="{gid}-pa" count="{3 * n}">{_f(P)}</float_array><technique_common>'
            f'<accessor source="#{gid}-pa" count="{n}" stride="3"><param name="X" type="float"/><param name="Y" type="float"/>'
            f'<param name="Z" type="float"/></accessor></technique_common></source>'
            f'<source id="{gid}-n"><float_array id="{gid}-na" count="{3 * n}">{_f(N, "%.5f")}</float_array><technique_common>'
            f'<accessor source="#{gid}-na" count="{n}" stride="3"><param name="X" type="float"/><param name="Y" type="float"/>'
            f'<param name="Z" type="float"/></accessor></technique_common></source>'
            f'<source id="{gid}-t"><float_array id="{gid}-ta" count="{2 * n}">{_f(T, "%.5f")}</float_array><technique_common>'
            f'<accessor source="#{gid}-ta" count="{n}" stride="2"><param name="S" type="float"/><param name="T" type="float"/>'
            f'</accessor></technique_common></source>'
            f'<vertices id="{gid}-v"><input semantic="POSITION" source="#{gid}-p"/></vertices>'
            f'<triangles material="sym" count="{len(I)}"><input semantic="VERTEX" source="#{gid}-v" offset="0"/>'
            f'<input semantic="NORMAL" source="#{gid}-n" offset="0"/>'
            f'<input semantic="TEXCOORD" source="#{gid}-t" offset="0" set="0"/>'
            f'<p>{" ".join(map(str, np.asarray(I).reshape(-1)))}</p></triangles></mesh></geometry>')
        nodes.append(f'<node id="n_{gid}" name="{gname}"><instance_geometry url="#{gid}"><bind_material>'
                     f'<technique_common><instance_material symbol="sym" target="#mat_{mat}">'
                     f'<bind_vertex_input semantic="UVSET0" input_semantic="TEXCOORD" input_set="0"/></instance_material>'
                     f'</technique_common></bind_material></instance_geometry></node>')

    for k, (mat, m) in enumerate(b.meshes.items()):
        P, N, T, I = m.arrays()
        geometry(f"g{k}", f"{mat}_mesh", P, N, T, I, mat)
    C = _cutout(b)
    geometry("g_cut", "YULIO_CAMERA_ALIGNED_visitor", C, np.broadcast_to([0, -1.0, 0], C.shape),
             np.array([[0, 0], [1, 0], [1, 1], [0, 1.0]]), np.array([[0, 1, 2], [0, 2, 3]]), "cutout")
    # the cut-out stands in the living room (its node translation is the billboard pivot)
    nodes[-1] = nodes[-1].replace('name="YULIO_CAMERA_ALIGNED_visitor">',
                                  'name="YULIO_CAMERA_ALIGNED_visitor"><translate>236 150 0</translate>')
    cams = []
    for name, (eye, dst) in CAMERAS.items():
        m = _lookat(eye, dst)
        cams.append(f'<node id="cam_{name}" name="YULIO_FPR_VIEW_{name}"><matrix>{_f(m)}</matrix>'
                    f'<instance_camera url="#cam0"/></node>')
    doc = ('<?xml version="1.0" encoding="utf-8"?>\n'
           '<COLLADA xmlns="http://www.collada.org/2005/11/COLLADASchema" version="1.4.1">\n'
           '<asset><contributor><authoring_tool>yrt frederick stand-in (seed 2217)</authoring_tool></contributor>'
           f'<unit name="inch" meter="{UNIT}"/><up_axis>Z_UP</up_axis></asset>\n'
           f'<library_images>{"".join(imgs)}</library_images>\n'
           f'<library_effects>{"".join(fx)}</library_effects>\n'
           f'<library_materials>{"".join(mats)}</library_materials>\n'
           f'<library_geometries>{"".join(geos)}</library_geometries>\n'
           '<library_cameras><camera id="cam0"><optics><technique_common><perspective><xfov>90</xfov>'
           '<aspect_ratio>1</aspect_ratio><znear>1</znear><zfar>10000</zfar></perspective></technique_common>'
           '</optics></camera></library_cameras>\n'
           f'<library_visual_scenes><visual_scene id="scene0" name="Frederick">{"".join(nodes)}{"".join(cams)}'
           '</visual_scene></library_visual_scenes>\n'
           '<scene><instance_visual_scene url="#scene0"/></scene>\n</COLLADA>\n')
    tmp = path.with_suffix(f".{os.getpid()}.tmp")
    tmp.write_text(doc)
    tmp.replace(path)
    return path


if __name__ == "__main__":
    p = write_dae()
    print(p, triangle_count(), f"{p.stat().st_size / 1e6:.1f} MB")
