#!/usr/bin/env python3
"""Node / triangle visits per shadow query, 4-wide (farthest child first) vs the 8-wide BVH
collapsed from it (tools/bvh8_visits_exp.c), on the C3 shadow streams dumped by
tools/dump_shadow_stream.py (gpurun_out/shadow_c3.npz).
usage: python tools/bvh8_visits_exp.py [npz]"""
import ctypes as C
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
so = Path("/tmp/b8v.so")
subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", str(so), str(ROOT / "tools" / "bvh8_visits_exp.c"), "-lm"],
               check=True)
lib = C.CDLL(str(so))
lib.bvh8_visits.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
d = np.load(sys.argv[1] if len(sys.argv) > 1 else ROOT / "gpurun_out" / "shadow_c3.npz")
nodes, tris = np.ascontiguousarray(d["nodes"]), np.ascontiguousarray(d["tris"])
for depth in range(3):
    org = np.ascontiguousarray(d[f"s{depth}_org"], np.float32)
    dr = np.ascontiguousarray(d[f"s{depth}_dir"], np.float32)
    out = np.zeros(7)
    lib.bvh8_visits(nodes.ctypes.data, nodes.nbytes // 128, tris.ctypes.data, org.ctypes.data, dr.ctypes.data,
                    org.shape[0], out.ctypes.data)
    print(f"depth {depth}: {org.shape[0]} queries  4-wide {out[0]:.2f} nodes {out[1]:.2f} tris  |  "
          f"8-wide {out[2]:.2f} nodes {out[3]:.2f} tris  (8-wide nodes {out[5]:.0f}, {out[6]:.2f} children avg; "
          f"occlusion disagreements {out[4]:.0f})")
