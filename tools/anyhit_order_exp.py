#!/usr/bin/env python3
"""Child visiting orders for the any-hit traversal on the C3 shadow streams
(gpurun_out/shadow_c3.npz, tools/dump_shadow_stream.py): node steps and triangle tests per query
until the first occluder, for the device's order (farthest entry first, the others in slot
order), nearest first, slot order, and two static per-node orders that need no per-ray sort —
largest child box first, and an order learned from where the first occluders of half of the
depth-0 stream lie (tools/anyhit_order_exp.c).
usage: python tools/anyhit_order_exp.py [npz]"""
import ctypes as C
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
so = Path("/tmp/aho.so")
subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", str(so), str(ROOT / "tools" / "anyhit_order_exp.c"), "-lm"],
               check=True)
lib = C.CDLL(str(so))
d = np.load(sys.argv[1] if len(sys.argv) > 1 else ROOT / "gpurun_out" / "shadow_c3.npz")
nodes, tris = np.ascontiguousarray(d["nodes"]), np.ascontiguousarray(d["tris"])
nn = nodes.size * nodes.itemsize // 128
nf = np.frombuffer(nodes.tobytes(), np.float32).reshape(nn, 32)
ni = np.frombuffer(nodes.tobytes(), np.int32).reshape(nn, 32)
lox, hix, loy, hiy, loz, hiz = (nf[:, 4 * k:4 * k + 4] for k in range(6))
child = ni[:, 24:28]
ext = np.maximum(0, np.stack([hix - lox, hiy - loy, hiz - loz], -1))
area = ext[..., 0] * ext[..., 1] + ext[..., 1] * ext[..., 2] + ext[..., 2] * ext[..., 0]

# leaf-slot range [lo, hi) under every child
rng = np.zeros((nn, 4, 2), np.int64)
sys.setrecursionlimit(10000)


def span(c):
    if c == -1:
        return (1 << 40, -1)
    if c & 31:
        return (c >> 5, (c >> 5) + (c & 31))
    n = c >> 5
    los, his = [], []
    for k in range(4):
        lo, hi = span(int(child[n, k]))
        rng[n, k] = (lo, hi)
        los.append(lo)
        his.append(hi)
    return (min(los), max(his))


span(0)


def run(org, dr, mode, perm=None):
    n = org.shape[0]
    steps = np.zeros((n, 2), np.int32)
    occ = np.zeros(n, np.int32)
    p = perm if perm is not None else np.zeros((nn, 4), np.int32)
    lib.anyhit_order(C.c_void_p(nodes.ctypes.data), C.c_void_p(tris.ctypes.data), C.c_void_p(org.ctypes.data),
                     C.c_void_p(dr.ctypes.data), n, mode, C.c_void_p(p.ctypes.data), C.c_void_p(steps.ctypes.data),
                     C.c_void_p(occ.ctypes.data))
    return steps, occ


streams = {k: (np.ascontiguousarray(d[f"s{k}_org"], np.float32), np.ascontiguousarray(d[f"s{k}_dir"], np.float32))
           for k in range(3) if f"s{k}_org" in d}
org0, dir0 = streams[0]
half = org0.shape[0] // 2
_, occ_tr = run(np.ascontiguousarray(org0[:half]), np.ascontiguousarray(dir0[:half]), 0)
cnt = np.zeros((nn, 4), np.int64)
for s in occ_tr[occ_tr >= 0]:
    n = 0
    while True:
        k = int(np.nonzero((rng[n, :, 0] <= s) & (s < rng[n, :, 1]))[0][0])
        cnt[n, k] += 1
        c = int(child[n, k])
        if c & 31:
            break
        n = c >> 5
perm_area = np.ascontiguousarray(np.argsort(-area, axis=1, kind="stable"), np.int32)
perm_learn = np.ascontiguousarray(
    np.array([sorted(range(4), key=lambda k: (-cnt[i, k], -area[i, k])) for i in range(nn)], np.int32))
modes = [("far first, others by slot (device)", 0, None), ("nearest first", 1, None), ("slot order", 2, None),
         ("largest box first (static)", 3, perm_area), ("learned occluder order (static)", 3, perm_learn),
         ("all by entry distance, far first", 4, None), ("all by exit distance, far first", 5, None)]
for depth, (org, dr) in streams.items():
    if depth == 0:
        org, dr = np.ascontiguousarray(org[half:]), np.ascontiguousarray(dr[half:])
    for name, mode, perm in modes:
        steps, occ = run(org, dr, mode, perm)
        print(f"depth {depth} ({org.shape[0]} queries, {(occ >= 0).mean():.3f} occluded): {name:36s} "
              f"{steps[:, 0].mean():6.3f} nodes {steps[:, 1].mean():6.3f} tris per query")
