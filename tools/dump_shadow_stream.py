#!/usr/bin/env python3
"""Dumps the C3 frame's complete shadow- and closest-query streams of depths 0-2 (batch 0, queue order) plus the
uploaded BVH to gpurun_out/shadow_c3.npz, for CPU-side any-hit experiments
(tools/occluder_cache_exp.c). usage: python tools/dump_shadow_stream.py [size] [spp]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "yulio-raytracer_amd"), str(ROOT / "tests")]
import numpy as np  # noqa: E402

import yrt  # noqa: E402
from helpers import c3_args  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 192
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 16
dev = yrt.Device(0)
s = yrt.Session(c3_args(size, spp), device=dev)
S = s.info()["scene"]
dev.set_ray_capture(size * size * spp)  # >= every queue of the frame: stride 1
s.render()
dev.set_ray_capture(0)
out = {}
for depth in range(3):
    org, dr, tot = dev.captured_rays(1, depth)
    out[f"s{depth}_org"], out[f"s{depth}_dir"] = org, dr
    org, dr, tot = dev.captured_rays(0, depth)  # the closest-hit queries entering this depth
    out[f"c{depth}_org"], out[f"c{depth}_dir"] = org, dr
nodes, tris = dev.export_bvh(S)
out["nodes"], out["tris"] = nodes, tris
Path(ROOT / "gpurun_out").mkdir(exist_ok=True)
np.savez_compressed(ROOT / "gpurun_out" / "shadow_c3.npz", **out)
print("saved", {k: v.shape for k, v in out.items() if k.endswith("_org")})
