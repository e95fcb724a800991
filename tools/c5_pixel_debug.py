#!/usr/bin/env python3
"""GPU-box parity debugging: C5 FPR face `cam` at 1536^2 / 1024 spp (the configuration of
tests/test_cubes.py::test_c5_full_size_face_band_parity) against the oracle on a row band;
for the first mismatching pixels, the per-sample radiance of the device (yrtDebugPixelSamples)
and of the oracle (oracle_debug_pixel) side by side -> gpurun_out/c5_pixel_debug_<cam>.npz.

usage: python tools/c5_pixel_debug.py [cam] [y0] [rows] [max_pixels]
"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "yulio-raytracer_amd"), str(ROOT)]
import numpy as np  # noqa: E402

import oracle  # noqa: E402
import yrt  # noqa: E402
from yrt import frederick  # noqa: E402

cam = int(sys.argv[1]) if len(sys.argv) > 1 else 2
y0 = int(sys.argv[2]) if len(sys.argv) > 2 else 760
rows = int(sys.argv[3]) if len(sys.argv) > 3 else 16
maxpix = int(sys.argv[4]) if len(sys.argv) > 4 else 4
W = H = 1536
SPP = 1024
dev = yrt.Device(0)
s = yrt.Session(["-fprCollada", "-faceCullingMode", "default", "-i", str(frederick.write_dae()), "-stereo", "-size",
                 str(W), str(H), "-spp", str(SPP), "-fb", "RGB_FLOAT32", "-tMaxShadowRay", "120", "-ambientlight", "0.83",
                 "0.95", "0.98", "-depth", "10", "-toeIn"], device=dev)
img = s.render_scene_camera(cam)
blob = s.export_frame(camera=s.scene_camera(cam))
ref, _ = oracle.render(blob, W, H, 1.0, rect=(0, y0, W, y0 + rows))
g, c = img[y0:y0 + rows], ref[y0:y0 + rows]
bad = np.argwhere(g != c)
print(json.dumps({"cam": cam, "band": [y0, y0 + rows], "mismatching_channels": int(len(bad))}), flush=True)
pix = []
for yy, xx, ch in bad:
    p = (int(xx), int(yy) + y0)
    if p not in pix:
        pix.append(p)
res = {}
for (x, y) in pix[:maxpix]:
    dev.debug_pixel_arm(x, y, W, 0, SPP)
    s.render_scene_camera(cam)
    gs = dev.debug_pixel_samples(SPP)
    dev.debug_pixel_arm(-1, 0, W)
    os_ = oracle.debug_pixel(blob, W, H, x, y)
    diff = np.argwhere(np.any(gs != os_, axis=1)).ravel()
    print(json.dumps({"pixel": [x, y], "gpu": img[y, x].tolist(), "oracle": ref[y, x].tolist(),
                      "sum_gpu": gs.sum(0).tolist(), "sum_oracle": os_.sum(0).tolist(),
                      "differing_samples": diff.tolist()[:20],
                      "values": [[int(k), gs[k].tolist(), os_[k].tolist()] for k in diff[:8]]}), flush=True)
    res[f"{x}_{y}"] = np.stack([gs, os_])
np.savez_compressed(ROOT / "gpurun_out" / f"c5_pixel_debug_{cam}.npz", **res)
s.close()
dev.close()
