#!/usr/bin/env python3
"""SIMD utilization of the traversal kernel on the C3 stand-in (needs a -DYRT_PROFILE build,
selected with YRT_LIB_DIR)."""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "yulio-raytracer_amd"), str(ROOT / "tests")]
import yrt  # noqa: E402
from yrt import _native as N  # noqa: E402
from helpers import c3_args  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 512
dev = yrt.Device(0)
s = yrt.Session(c3_args(size, 16), device=dev)
buf = (C.c_uint64 * 8)()
N.dev.yrtDebugTraceProfile(dev.h, buf, 1)
s.render()
rc = N.dev.yrtDebugTraceProfile(dev.h, buf, 1)
v = list(buf)
print("rc", rc, v)
if rc == 0:
    print(f"outer iterations/wave-steps {v[0]}, lanes with ray {v[1] / max(v[0], 1) / 64:.3f}")
    print(f"node-phase iterations {v[2]}, node-lane utilization {v[3] / max(v[2], 1) / 64:.3f}")
    print(f"leaf passes {v[4]}, tri-loop iterations {v[5]}, tri-lane utilization {v[6] / max(v[5], 1) / 64:.3f}")
    print(f"node iterations per outer {v[2] / max(v[0], 1):.2f}, tri iterations per outer {v[5] / max(v[0], 1):.2f}")
