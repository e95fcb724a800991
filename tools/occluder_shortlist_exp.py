#!/usr/bin/env python3
"""Occluder shortlist on the C3 shadow streams (tools/dump_shadow_stream.py ->
gpurun_out/shadow_c3.npz): the K leaf slots that occlude most often on the depth-0 stream's
first half, tested before the BVH on the rest — the share of queries they end, and the node
steps / triangle tests saved against the K tests added (tools/occluder_shortlist_exp.c).
usage: python tools/occluder_shortlist_exp.py [npz]"""
import ctypes as C
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
so = Path("/tmp/osl.so")
subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", str(so), str(ROOT / "tools" / "occluder_shortlist_exp.c"),
                "-lm"], check=True)
lib = C.CDLL(str(so))
d = np.load(sys.argv[1] if len(sys.argv) > 1 else ROOT / "gpurun_out" / "shadow_c3.npz")
nodes, tris = np.ascontiguousarray(d["nodes"]), np.ascontiguousarray(d["tris"])


def run(org, dr):
    n = org.shape[0]
    steps = np.zeros((n, 2), np.int32)
    occ = np.zeros(n, np.int32)
    lib.anyhit(C.c_void_p(nodes.ctypes.data), C.c_void_p(tris.ctypes.data), C.c_void_p(org.ctypes.data),
               C.c_void_p(dr.ctypes.data), n, C.c_void_p(steps.ctypes.data), C.c_void_p(occ.ctypes.data))
    return steps, occ


streams = {k: (np.ascontiguousarray(d[f"s{k}_org"], np.float32), np.ascontiguousarray(d[f"s{k}_dir"], np.float32))
           for k in range(3) if f"s{k}_org" in d}
org0, dir0 = streams[0]
half = org0.shape[0] // 2
_, occ_train = run(np.ascontiguousarray(org0[:half]), np.ascontiguousarray(dir0[:half]))
slots, counts = np.unique(occ_train[occ_train >= 0], return_counts=True)
order = slots[np.argsort(-counts)]
print(f"training: depth-0 first half, {half} queries, {(occ_train >= 0).mean():.3f} occluded by "
      f"{slots.size} distinct slots; top 8 / 32 / 128 slots cover "
      f"{[round(float(np.sort(counts)[::-1][:k].sum()) / max(1, (occ_train >= 0).sum()), 3) for k in (8, 32, 128)]}")
for depth, (org, dr) in streams.items():
    if depth == 0:
        org, dr = np.ascontiguousarray(org[half:]), np.ascontiguousarray(dr[half:])
    steps, occ = run(org, dr)
    n = org.shape[0]
    for K in (8, 16, 32, 64):
        lst = np.ascontiguousarray(order[:K], np.int32)
        pos = np.zeros(n, np.int32)
        lib.shortlist(C.c_void_p(tris.ctypes.data), C.c_void_p(org.ctypes.data), C.c_void_p(dr.ctypes.data), n,
                      C.c_void_p(lst.ctypes.data), K, C.c_void_p(pos.ctypes.data))
        ended = pos > 0
        # tests run: the position of the first occluder for ended queries, K for the rest
        tests_added = np.where(ended, pos, K).sum() / n
        nodes_saved = steps[ended, 0].sum() / n
        tris_saved = steps[ended, 1].sum() / n
        print(f"depth {depth}: {n} queries ({(occ >= 0).mean():.3f} occluded, {steps[:, 0].mean():.2f} nodes "
              f"{steps[:, 1].mean():.2f} tris each); K={K:3d}: ends {ended.mean():.3f} of the queries, saves "
              f"{nodes_saved:.2f} node steps + {tris_saved:.2f} tri tests per query, adds {tests_added:.2f} tri tests")
