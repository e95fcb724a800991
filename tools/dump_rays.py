#!/usr/bin/env python3
"""Dumps a strided sample of the C3 frame's real query streams (closest and shadow, per depth)
plus the uploaded BVH to gpurun_out/rays_c3.npz, for CPU-side traversal-order experiments
(tools/visit_order_exp.c). usage: python tools/dump_rays.py [per_depth] [size] [spp]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "yulio-raytracer_amd"), str(ROOT / "tests")]
import numpy as np  # noqa: E402

import yrt  # noqa: E402
from helpers import c3_args  # noqa: E402

per = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
size = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 16
dev = yrt.Device(0)
s = yrt.Session(c3_args(size, spp), device=dev)
S = s.info()["scene"]
dev.set_ray_capture(per)
s.render()
dev.set_ray_capture(0)
out = {}
for shadow in (0, 1):
    for depth in range(10):
        org, dr, tot = dev.captured_rays(shadow, depth)
        if len(org):
            k = f"{'s' if shadow else 'c'}{depth}"
            out[k + "_org"], out[k + "_dir"], out[k + "_tot"] = org, dr, np.float64(tot)
nodes, tris = dev.export_bvh(S)
out["nodes"], out["tris"] = nodes, tris
Path(ROOT / "gpurun_out").mkdir(exist_ok=True)
np.savez_compressed(ROOT / "gpurun_out" / "rays_c3.npz", **out)
print("saved", {k: v.shape for k, v in out.items() if k.endswith("_org")})
