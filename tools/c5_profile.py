#!/usr/bin/env python3
"""GPU-box: one C5 FPR view (the Frederick stand-in, yrt.frederick) as one cube job at the DLL's
defaults (1536^2, depth 10, tMaxShadowRay 120 x sceneScale, ambient .83 .95 .98, toe-in), for
rocprofv3 kernel statistics and PMC passes of the north-star path (tools/gpu_profile_cmd.sh).
One untimed warm-up view at 4 spp, then --views timed views at --spp. Prints one JSON line
whose "config" identifies the workload.

usage: python tools/c5_profile.py [--spp 64] [--views 1] [--face-loop]
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "yulio-raytracer_amd"), str(ROOT)]
import yrt  # noqa: E402
from yrt import frederick  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--size", type=int, default=1536)
    ap.add_argument("--views", type=int, default=1)
    ap.add_argument("--face-loop", action="store_true", help="per-face rtRenderFrame (the reference's loop)")
    a = ap.parse_args()
    dae = frederick.write_dae(ROOT / "scenes" / "_generated" / "frederick_c5" / "frederick.dae")
    dev = yrt.Device(0)
    args = ["-fprCollada", "-faceCullingMode", "default", "-i", str(dae), "-stereo", "-size", str(a.size),
            str(a.size), "-spp", str(a.spp), "-depth", "10", "-tMaxShadowRay", "120", "-ambientlight", "0.83",
            "0.95", "0.98", "-toeIn"]
    s = yrt.Session(args, device=dev)
    s.render_scene_camera(0)  # warm-up: BVH upload, allocations, sample table
    rays, t = 0.0, 0.0
    for v in range(a.views):
        t0 = time.perf_counter()
        if a.face_loop:
            for f in range(12):
                s.render_scene_camera(12 * (v % 2) + f, )
                st = dev.render_stats()
                rays += st["raysClosest"] + st["raysShadow"]
        else:
            s.render_scene_cube(v % 2, read=False)
            st = dev.render_stats()
            rays += st["raysClosest"] + st["raysShadow"]
        t += time.perf_counter() - t0
    info = dev.scene_info(s.info()["scene"])
    out = {"metric": "Mrays/s (C5 FPR view)", "value": round(rays / t / 1e6, 1), "ms_per_view": round(t / a.views * 1e3, 1),
           "config": {"workload": f"C5 frederick_standin FPR view 12x{a.size}^2 {a.spp}spp depth10 DLL defaults",
                      "width": a.size, "height": a.size, "spp": a.spp, "triangles": info["numTriangles"],
                      "bvh_nodes": info["numNodes"], "batch_capacity": "default",
                      "mode": "face-loop" if a.face_loop else "cube-job"}}
    print(json.dumps(out), flush=True)
    s.close()
    dev.close()


if __name__ == "__main__":
    main()
