#!/usr/bin/env python3
"""GPU-box parity debugging, one level below tools/c5_pixel_debug.py: the per-depth record of one
sample of one pixel of a C5 FPR face (1536^2, 1024 spp) from the device (a -DYRT_PATH_DEBUG build
of the library: YRT_LIB_DIR=yulio-raytracer_amd/lib_variants/pathdbg) and from the oracle
(oracle.debug_path), printed side by side with the first differing field.

usage: YRT_LIB_DIR=... python tools/c5_path_debug.py cam x y sample
"""
import ctypes as C
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "yulio-raytracer_amd"), str(ROOT)]
import numpy as np  # noqa: E402

import oracle  # noqa: E402
import yrt  # noqa: E402
from yrt import _native, frederick  # noqa: E402

cam, x, y, sample = (int(a) for a in sys.argv[1:5])
W = H = 1536
SPP = 1024
lib = C.CDLL(str(Path(os.environ["YRT_LIB_DIR"]) / "libdevice_singleray_mi355x.so"))
fn = lib.yrt_debug_path
fn.restype = C.c_int
fn.argtypes = [C.c_int, C.c_int, C.c_void_p]
dev = yrt.Device(0)
s = yrt.Session(["-fprCollada", "-faceCullingMode", "default", "-i", str(frederick.write_dae()), "-stereo", "-size",
                 str(W), str(H), "-spp", str(SPP), "-fb", "RGB_FLOAT32", "-tMaxShadowRay", "120", "-ambientlight", "0.83",
                 "0.95", "0.98", "-depth", "10", "-toeIn"], device=dev)
assert fn(y * W + x, sample, None) == 0
s.render_scene_camera(cam)
g = np.zeros((32, 32), np.float32)
assert fn(0, 0, g.ctypes.data) == 0
g = g[: int((g[:, 0] != 0).sum())]
blob = s.export_frame(camera=s.scene_camera(cam))
o = oracle.debug_path(blob, W, H, x, y, sample)
print(json.dumps({"cam": cam, "pixel": [x, y], "sample": sample, "depths_gpu": len(g), "depths_oracle": len(o),
                  "lib": _native.LIB_DIR.name}), flush=True)
F = oracle.PATH_FIELDS
for d in range(max(len(g), len(o))):
    a = g[d] if d < len(g) else np.full(32, np.nan, np.float32)
    b = o[d] if d < len(o) else np.full(32, np.nan, np.float32)
    diff = [k for k in range(32) if not (a[k] == b[k] or (np.isnan(a[k]) and np.isnan(b[k])))]
    print(json.dumps({"depth": d, "first_diff": F[diff[0]] if diff else None, "diff_fields": sorted({F[k] for k in diff}),
                      "gpu": [float(v) for v in a], "oracle": [float(v) for v in b]}), flush=True)
np.savez_compressed(ROOT / "gpurun_out" / f"c5_path_debug_{cam}_{x}_{y}_{sample}.npz", gpu=g, oracle=o)
s.close()
dev.close()
