#!/usr/bin/env python3
"""Phase breakdown of k_shade on the C3 stand-in or a C4 stereo face (needs a -DYRT_SHADE_PROF
build, selected with YRT_LIB_DIR): shader-clock cycles per phase summed over the waves of every
shade launch of one frame.
usage: YRT_LIB_DIR=... python tools/shade_profile.py [C3|C4] [size] [spp] [fine]"""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "yulio-raytracer_amd"), str(ROOT / "tests")]
import yrt  # noqa: E402
from yrt import _native as N  # noqa: E402
from helpers import c3_args, c4_args  # noqa: E402

PHASES = ["queue record + pixel/sample record", "misses (env/backplate)", "postIntersect",
          "material shade + emission", "continuation sample", "continuation append/stores",
          "direct light + shadow append", "loop overhead"]
FINE = ["record .. RR (before BRDF sample)", "CompositedBRDF::sample", "rest of continuation + append",
        "Light::sample", "CompositedBRDF::eval", "jitter + contribution", "shadow append + stores",
        "loop overhead"]
argv = sys.argv[1:]
cfg = argv.pop(0) if argv and argv[0] in ("C3", "C4") else "C3"
if len(argv) > 2 and argv[2] == "fine":  # a -DYRT_SHADE_PROF=2 build
    PHASES = FINE

size = int(argv[0]) if len(argv) > 0 else 1024
spp = int(argv[1]) if len(argv) > 1 else 16
dev = yrt.Device(0)
s = yrt.Session((c4_args if cfg == "C4" else c3_args)(size, spp), device=dev)
dev.set_kernel_timing(True)
s.render()  # warm-up
buf = (C.c_uint64 * 8)()
N.dev.yrtDebugTraceProfile(dev.h, buf, 1)
s.render()
rc = N.dev.yrtDebugTraceProfile(dev.h, buf, 1)
st = dev.render_stats()
v = list(buf)
if rc != 0:
    sys.exit("not a YRT_SHADE_PROF build")
tot = sum(v)
items = st["raysClosest"]
if tot == 0:
    sys.exit(f"{cfg}: no phase cycles recorded (the profile counters stayed 0)")
print(f"{cfg} {size}^2 {spp}spp: shade items {items:.0f}, shade ms {st['msShade']:.1f}")
for name, x in zip(PHASES, v):
    print(f"  {name:38s} {100.0 * x / tot:6.2f} %   {x / max(items, 1) * 64:9.1f} wave-cycles per 64 items")
