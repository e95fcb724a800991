#!/usr/bin/env python3
"""GPU-box: every BASELINE.json config on one MI355X, with the CPU restatement beside it.

C1 cornell 256^2 1spp and C2 cornell-spheres 1024^2 16spp: full frames on GPU and CPU (the
BASELINE plan's "full run"). C3 Sponza stand-in 2048^2 64spp: GPU full frame (bench.py has
the CPU sample). C4 test_stereo cubemap 12 x 1536^2 256spp: GPU all 12 faces, CPU one face
at spp 16 scaled x16 x12 ("spp 16, scaled x16, stated"). One line per config.
"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "yulio-raytracer_amd"), str(ROOT / "tests")]
import oracle  # noqa: E402
import yrt  # noqa: E402
from helpers import c1_args, c2_args, c3_args, c4_args  # noqa: E402

dev = yrt.Device(0)
threads = oracle.cpu_count()  # all logical cores


def gpu_frames(ses, faces, reps=2):
    for f in faces[:1]:
        ses.render(f)  # warm-up: allocations, sample table
    best = None
    for _ in range(reps):
        t = time.perf_counter()
        rays = 0.0
        for f in faces:
            ses.render(f)
            st = dev.render_stats()
            rays += st["raysClosest"] + st["raysShadow"]
        dt = time.perf_counter() - t
        best = (dt, rays) if best is None or dt < best[0] else best
    return best


def cpu_frame(ses, w, h, face=-1):
    blob = ses.export_frame(face)
    t = time.perf_counter()
    _, st = oracle.render(blob, w, h, ses.info()["gamma"], threads=threads)
    return time.perf_counter() - t, st["raysClosest"] + st["raysShadow"]


rows = []
for name, args, size, spp, faces in [("C1 cornell_box 256^2 1spp", c1_args(256, 1), 256, 1, [-1]),
                                      ("C2 cornell_box_spheres 1024^2 16spp", c2_args(1024, 16), 1024, 16, [-1]),
                                      ("C3 sponza_standin 2048^2 64spp", c3_args(2048, 64), 2048, 64, [-1]),
                                      ("C4 test_stereo cubemap 12x1536^2 256spp", c4_args(1536, 256), 1536, 256,
                                       list(range(12)))]:
    ses = yrt.Session(args + ["-fb", "RGB_FLOAT32"], device=dev)
    dt, rays = gpu_frames(ses, faces)
    samples = size * size * spp * len(faces)
    row = {"config": name, "gpu_ms": round(dt * 1e3, 2), "gpu_Mrays_s": round(rays / dt / 1e6, 1),
           "gpu_Msamples_s": round(samples / dt / 1e6, 1)}
    if name.startswith(("C1", "C2")):
        cdt, crays = cpu_frame(ses, size, size)
        row.update({"cpu_ms": round(cdt * 1e3, 1), "cpu_Mrays_s": round(crays / cdt / 1e6, 2), "cpu_threads": threads,
                    "speedup": round(cdt / dt, 1)})
    elif name.startswith("C4"):
        # CPU: face 0 at spp 16, scaled x16 (spp) x12 (faces) to the cubemap (stated)
        ses16 = yrt.Session(c4_args(1536, 16) + ["-fb", "RGB_FLOAT32"], device=dev)
        cdt, crays = cpu_frame(ses16, 1536, 1536, face=0)
        ses16.close()
        est = cdt * 16 * 12
        row.update({"cpu_ms_scaled": round(est * 1e3, 0), "cpu_Mrays_s": round(crays / cdt / 1e6, 2),
                    "cpu_threads": threads, "cpu_sample": "face 0 at 16 spp, x16 x12", "speedup": round(est / dt, 0)})
    ses.close()
    rows.append(row)
    print(json.dumps(row), flush=True)
