#!/usr/bin/env python3
"""GPU-box: where a C4 cubemap's time goes, cube job vs face loop: the render calls alone
(framebuffers stay on the device side of the session) and the host readback of the 12 faces,
timed separately, 3 repetitions each after a warm-up. usage: python tools/cube_face_split.py"""
import ctypes as C
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "yulio-raytracer_amd"), str(ROOT), str(ROOT / "tests")]
import yrt  # noqa: E402
from yrt import _native as N  # noqa: E402
from helpers import c4_args  # noqa: E402

dev = yrt.Device(0)
ses = yrt.Session(c4_args(1536, 256), device=dev)
ses.render_cube(read=False)
for f in range(12):
    ses.render(f)
res = {}
for rep in range(3):
    t = time.perf_counter(); ses.render_cube(read=False); t1 = time.perf_counter()
    ses._cube_faces(); t2 = time.perf_counter()
    ms_dev = dev.render_stats().get("msTotal", 0)
    res.setdefault("cube_render_ms", []).append(round((t1 - t) * 1e3, 1))
    res.setdefault("cube_readback_ms", []).append(round((t2 - t1) * 1e3, 1))
    res.setdefault("cube_msTotal", []).append(round(ms_dev, 1))
    tr, tmt = 0.0, 0.0
    t = time.perf_counter()
    for f in range(12):
        a = time.perf_counter()
        ses.render(f, read=False)
        tr += time.perf_counter() - a
        tmt += dev.render_stats().get("msTotal", 0)
    res.setdefault("face_render_ms", []).append(round(tr * 1e3, 1))
    res.setdefault("face_msTotal_sum", []).append(round(tmt, 1))
    res.setdefault("face_loop_total_ms", []).append(round((time.perf_counter() - t) * 1e3, 1))
print(json.dumps(res), flush=True)
