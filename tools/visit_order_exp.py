#!/usr/bin/env python3
"""Node/triangle visits per query for several BVH4 child orders (tools/visit_order_exp.c) on
the captured C3 query streams (tools/dump_rays.py -> gpurun_out/rays_c3.npz). CPU only."""
import ctypes as C
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
so = "/tmp/voe.so"
subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-ffp-contract=off", "-o", so,
                str(ROOT / "tools" / "visit_order_exp.c"), "-lm"], check=True)
lib = C.CDLL(so)
lib.visit_counts.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                            C.POINTER(C.c_double)]
z = np.load(sys.argv[1] if len(sys.argv) > 1 else ROOT / "gpurun_out" / "rays_c3.npz")
nodes, tris = z["nodes"], z["tris"]
nn = len(nodes) // 128
modes = {0: "distance", 1: "octant", 2: "slot", 3: "area-desc", 4: "area-asc", 5: "far-first", 6: "oct-rev", 7: "far1+slot", 8: "far-net3", 9: "octfar1", 10: "bound", 11: "near-net3", 12: "near-net4", 13: "axis-cent", 14: "axis-box"}
for kind in ("c", "s"):
    tot = {m: np.zeros(3) for m in modes}
    wsum = 0.0
    for d in range(10):
        k = f"{kind}{d}"
        if k + "_org" not in z:
            continue
        org = np.ascontiguousarray(z[k + "_org"], np.float32)
        dr = np.ascontiguousarray(z[k + "_dir"], np.float32)
        w = float(z[k + "_tot"])
        wsum += w
        for m in modes:
            out = (C.c_double * 3)()
            lib.visit_counts(nodes.ctypes.data, C.c_size_t(nn), tris.ctypes.data, org.ctypes.data, dr.ctypes.data,
                             len(org), int(kind == "s"), m, out)
            tot[m] += w * np.array(out[:])
    print("closest" if kind == "c" else "shadow")
    for m, v in tot.items():
        v = v / wsum
        print(f"  {modes[m]:9s} nodes {v[0]:6.2f}  tris {v[1]:5.2f}  pushes {v[2]:5.2f}")

lib.visit_counts8.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                              C.POINTER(C.c_double)]
for kind in ("c", "s"):
    tot = np.zeros(3)
    wsum = 0.0
    for d in range(10):
        k = f"{kind}{d}"
        if k + "_org" not in z:
            continue
        org = np.ascontiguousarray(z[k + "_org"], np.float32)
        dr = np.ascontiguousarray(z[k + "_dir"], np.float32)
        w = float(z[k + "_tot"])
        wsum += w
        out = (C.c_double * 3)()
        n8 = lib.visit_counts8(nodes.ctypes.data, C.c_size_t(nn), tris.ctypes.data, org.ctypes.data, dr.ctypes.data,
                               len(org), int(kind == "s"), out)
        tot += w * np.array(out[:])
    v = tot / wsum
    print(f"BVH8 ({n8} nodes vs {nn}) {'closest' if kind == 'c' else 'shadow'}: nodes {v[0]:6.2f}  tris {v[1]:5.2f}  "
          f"pushes {v[2]:5.2f}")
