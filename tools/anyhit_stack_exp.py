#!/usr/bin/env python3
"""Stack depth of the any-hit traversal on the C3 shadow streams (tools/dump_shadow_stream.py ->
gpurun_out/shadow_c3.npz): distribution of the deepest stack per query and the pushes an LDS
ring of 8 / 16 / 32 entries would evict (tools/anyhit_stack_exp.c).
usage: python tools/anyhit_stack_exp.py [npz]"""
import ctypes as C
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
so = Path("/tmp/ase.so")
subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", str(so), str(ROOT / "tools" / "anyhit_stack_exp.c"), "-lm"],
               check=True)
lib = C.CDLL(str(so))
lib.stack_depths.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
lib.closest_stack_depths.argtypes = lib.stack_depths.argtypes
d = np.load(sys.argv[1] if len(sys.argv) > 1 else ROOT / "gpurun_out" / "shadow_c3.npz")
nodes, tris = np.ascontiguousarray(d["nodes"]), np.ascontiguousarray(d["tris"])
for kind, depth in [(k, dd) for k in ("s", "c") for dd in range(3)]:
    if f"{kind}{depth}_org" not in d:
        continue
    org = np.ascontiguousarray(d[f"{kind}{depth}_org"], np.float32)
    dr = np.ascontiguousarray(d[f"{kind}{depth}_dir"], np.float32)
    fn = lib.stack_depths if kind == "s" else lib.closest_stack_depths
    if kind == "c":  # the closest-hit traversal is slower on the CPU: a strided sample
        org, dr = np.ascontiguousarray(org[::8]), np.ascontiguousarray(dr[::8])
    n = org.shape[0]
    out = np.zeros(n, np.int32)
    ev = np.zeros((n, 3), np.int32)
    fn(nodes.ctypes.data, tris.ctypes.data, org.ctypes.data, dr.ctypes.data, n, out.ctypes.data,
                     ev.ctypes.data)
    q = np.percentile(out, [50, 90, 99, 99.9])
    print(f"{'shadow' if kind == 's' else 'closest'} depth {depth}: {n} queries, max stack p50/p90/p99/p99.9 {q.tolist()} max {out.max()}; "
          f"queries over 8/16/32 entries {[(out > r).mean().round(5) for r in (8, 16, 32)]}; "
          f"evictions per query ring 8/16/32 {ev.mean(0).round(4).tolist()}")
