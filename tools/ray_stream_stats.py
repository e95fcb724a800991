#!/usr/bin/env python3
"""Per-depth statistics of the captured query streams of one C3 frame (GPU): how many rays have a
NaN or infinite component in their origin or direction, the spread of |dir|, and the oracle's node
and triangle visits per query for the finite rays and the non-finite ones separately. Run once
per library (YRT_LIB_DIR) to compare ray streams of two builds.

    python tools/ray_stream_stats.py [size] [spp] [max_per_depth]
"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "yulio-raytracer_amd"), str(ROOT / "tests")]
import oracle  # noqa: E402  (the checker: counts visits on the captured rays)
import yrt  # noqa: E402
from helpers import c3_args  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 512
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 16
cap = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 20
dev = yrt.Device(0)
s = yrt.Session(c3_args(size, spp), device=dev)
s.render(read=False)
dev.set_ray_capture(cap)
s.render(read=False)
dev.set_ray_capture(0)
scene = s.info()["scene"]
sinfo = dev.scene_info(scene)
nodes, tris = dev.export_bvh(scene)
qnodes = dev.export_qbvh(scene)
out = {"size": size, "spp": spp, "max_per_depth": cap, "kinds": {}}
for shadow in (0, 1):
    rows = []
    for depth in range(64):
        org, dr, total = dev.captured_rays(shadow, depth)
        if not len(org):
            continue
        bad = ~(np.isfinite(org[:, :3]).all(1) & np.isfinite(dr[:, :3]).all(1))
        ln = np.sqrt((dr[:, :3].astype(np.float64) ** 2).sum(1))
        row = {"depth": depth, "total": total, "sampled": int(len(org)), "nonfinite": int(bad.sum()),
               "len_dev_max": float(np.nanmax(np.abs(ln[~bad] - 1.0))) if (~bad).any() else None}
        for name, m in (("finite", ~bad), ("nonfinite", bad)):
            if m.any():
                o, d = np.ascontiguousarray(org[m]), np.ascontiguousarray(dr[m])
                nv, tv, _ = oracle.count_visits(nodes, tris, o, d, any_hit=bool(shadow),
                                                tri_bytes=sinfo["triRecordBytes"],
                                                qnodes=qnodes if (shadow and sinfo["nodeBytesAny"] == 64) else None)
                row[name + "_nodes_per_ray"] = nv / m.sum()
                row[name + "_tris_per_ray"] = tv / m.sum()
        rows.append(row)
        print(("shadow" if shadow else "closest"), json.dumps(row), flush=True)
    out["kinds"]["shadow" if shadow else "closest"] = rows
print(json.dumps(out))
