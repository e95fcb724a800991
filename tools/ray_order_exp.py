#!/usr/bin/env python3
"""Experiment: how much does the ORDER of a query stream change k_trace's time? Captures the
full closest-hit and shadow query streams of one C3 frame (batch 0, every depth), then traces
each stream through yrtIntersect / yrtOccluded in (a) queue order, (b) a stable sort by
direction octant, (c) octant then a Morton code of the origin, (d) random order — same rays,
so the visit counts are identical and only SIMD coherence changes.
usage: python tools/ray_order_exp.py [size] [spp]"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "yulio-raytracer_amd"), str(ROOT / "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import yrt  # noqa: E402
from helpers import c3_args  # noqa: E402


def morton3(q):  # q: (n,3) int in [0, 1024)
    def spread(x):
        x = x.astype(np.uint64) & 0x3FF
        x = (x | (x << 16)) & 0x030000FF
        x = (x | (x << 8)) & 0x0300F00F
        x = (x | (x << 4)) & 0x030C30C3
        x = (x | (x << 2)) & 0x09249249
        return x
    return spread(q[:, 0]) | (spread(q[:, 1]) << 1) | (spread(q[:, 2]) << 2)


def orders(org, dr):
    n = len(org)
    octant = ((dr[:, 0] < 0).astype(np.int64) | ((dr[:, 1] < 0).astype(np.int64) << 1) |
              ((dr[:, 2] < 0).astype(np.int64) << 2))
    lo, hi = org[:, :3].min(0), org[:, :3].max(0)
    q = np.clip(((org[:, :3] - lo) / np.maximum(hi - lo, 1e-9) * 1023).astype(np.int64), 0, 1023)
    mo = morton3(q).astype(np.int64)
    rng = np.random.default_rng(7)
    return {
        "queue": np.arange(n),
        "octant": np.argsort(octant, kind="stable"),
        "octant+morton": np.lexsort((mo, octant)),
        "morton": np.argsort(mo, kind="stable"),
        "random": rng.permutation(n),
    }


def time_stream(dev, scene, org, dr, shadow, reps=3):
    o = torch.from_numpy(np.ascontiguousarray(org)).cuda()
    d = torch.from_numpy(np.ascontiguousarray(dr)).cuda()
    n = len(org)
    out = torch.empty((n, 4), dtype=torch.float32, device="cuda") if not shadow else \
        torch.empty(n, dtype=torch.int32, device="cuda")
    fn = dev.occluded if shadow else dev.intersect
    fn(scene, o.data_ptr(), d.data_ptr(), n, out.data_ptr())
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t = time.perf_counter()
        fn(scene, o.data_ptr(), d.data_ptr(), n, out.data_ptr())
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    return best, out.cpu().numpy()


def main():
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    dev = yrt.Device(0)
    s = yrt.Session(c3_args(size, spp), device=dev)
    info = s.info()
    dev.set_ray_capture(1 << 30)
    s.render()
    dev.set_ray_capture(0)
    scene = info["scene"]
    for shadow in (0, 1):
        for depth in (0, 1, 2, 4):
            org, dr, tot = dev.captured_rays(shadow, depth)
            if len(org) < 100000:
                continue
            res = {}
            ref = None
            for name, idx in orders(org, dr).items():
                dt, out = time_stream(dev, scene, org[idx], dr[idx], shadow)
                inv = np.empty_like(idx)
                inv[idx] = np.arange(len(idx))
                out = out[inv]
                if ref is None:
                    ref = out
                same = bool(np.array_equal(out.view(np.int32), ref.view(np.int32)))
                res[name] = (dt, same)
            base = res["queue"][0]
            print(f"{'shadow' if shadow else 'closest'} depth {depth}: {len(org)} rays, queue order "
                  f"{len(org) / base / 1e6:.0f} Mrays/s; " +
                  ", ".join(f"{k} {base / v[0]:.3f}x{'' if v[1] else ' (DIFFERENT RESULTS)'}"
                            for k, v in res.items() if k != "queue"), flush=True)
    s.close()
    dev.close()


if __name__ == "__main__":
    main()
