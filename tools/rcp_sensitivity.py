#!/usr/bin/env python3
"""What the reciprocal substitution of rounds 1-5 cost, measured on the CPU alone.

Rounds 1-5 computed rcp(x) as 1/x and rsqrt(x) as 1/sqrt(x) (correctly rounded) on the GPU and in
the oracle alike. The reference uses the SSE estimates plus one Newton step (common/math/math.h:
38-59), which round 6 reproduces exactly (yrt_sse_rcp.h). This renders the same frame blobs with
both oracle builds — liboracle.so (the reference's reciprocals) and liboracle_ieee.so (the old
substitution) — and applies the SURVEY §8(d) gate to the pair: per channel |g - c| <= 1e-3 +
1e-3 |c| on >= 99.9 % (C1/C2) / 99.5 % (C3-C5) of channels, mean abs diff <= 1e-4 mean(c). The
GPU is bit-exact to liboracle.so in every parity test, so the IEEE column is the distance rounds
1-5's product had from the reference's arithmetic.

    python tools/rcp_sensitivity.py [--threads N] > profiles/r06/rcp_sensitivity_r06.txt
"""
from __future__ import annotations

import argparse
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "yulio-raytracer_amd"), str(ROOT / "tests")]

import oracle  # noqa: E402
import yrt  # noqa: E402
from helpers import c1_args, c2_args, c3_args, c4_args  # noqa: E402
from yrt import frederick  # noqa: E402

DLL = ["-tMaxShadowRay", "120", "-ambientlight", "0.83", "0.95", "0.98", "-depth", "10", "-toeIn"]


def gate(g, c, min_frac):
    ok = np.abs(g - c) <= 1e-3 + 1e-3 * np.abs(c)
    frac = float(ok.mean())
    mad = float(np.abs(g - c).mean() / max(float(np.abs(c).mean()), 1e-30))
    return frac, mad, float(np.abs(g - c).max()), float((g.view(np.uint32) == c.view(np.uint32)).mean()), \
        frac >= min_frac and mad <= 1e-4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=0)
    a = ap.parse_args()
    dev = yrt.Device(host=True)
    rows = []
    tmp = Path(tempfile.mkdtemp())
    dae = frederick.write_dae(tmp / "frederick.dae")
    cases = [("C1 256^2 1spp (full)", c1_args(256, 1), -1, None, 256, 0.999),
             ("C2 256^2 16spp", c2_args(256, 16), -1, None, 256, 0.999),
             ("C3 128^2 16spp", c3_args(128, 16), -1, None, 128, 0.995),
             ("C4 face 3 128^2 16spp", c4_args(128, 16), 3, None, 128, 0.995),
             ("C4 face 7 128^2 16spp", c4_args(128, 16), 7, None, 128, 0.995),
             ("C5 camera 2 96^2 16spp", None, -1, 2, 96, 0.995),
             ("C5 camera 19 96^2 16spp", None, -1, 19, 96, 0.995)]
    print("# CPU only (this container, %s threads): the same frame blob through liboracle.so (the"
          % (a.threads or oracle.cpu_count()))
    print("# reference's rcp/rsqrt: Intel rcpps/rsqrtps emulated + math.h's Newton steps) and through")
    print("# liboracle_ieee.so (rounds 1-5: 1/x, 1/sqrt(x)). Gate: SURVEY 8(d), per channel")
    print("# |g-c| <= 1e-3 + 1e-3|c| on >= 99.9 % (C1/C2) / 99.5 % (C3-C5), mad <= 1e-4 mean.")
    print("%-26s %-11s %-11s %-9s %-13s %s" % ("config", "within-gate", "mad/mean", "max|d|", "bit-identical", "gate"))
    for name, args, face, cam, size, min_frac in cases:
        if cam is not None:
            s = yrt.Session(["-fprCollada", "-faceCullingMode", "default", "-i", str(dae), "-stereo", "-size",
                             str(size), str(size), "-spp", "16", "-fb", "RGB_FLOAT32"] + DLL, device=dev)
            blob = s.export_frame(camera=s.scene_camera(cam))
        else:
            s = yrt.Session(args + ["-fb", "RGB_FLOAT32"], device=dev)
            blob = s.export_frame(face)
        gamma = s.info()["gamma"]
        s.close()
        t0 = time.time()
        ref, _ = oracle.render(blob, size, size, gamma, threads=a.threads)
        ieee, _ = oracle.render(blob, size, size, gamma, threads=a.threads, ieee_rcp=True)
        frac, mad, mx, same, ok = gate(ieee, ref, min_frac)
        print("%-26s %-11.4f %-11.2e %-9.3g %-13.4f %s   (%.0f s)" % (name, frac, mad, mx, same,
                                                                     "pass" if ok else "FAIL", time.time() - t0))
        sys.stdout.flush()
    dev.close()


if __name__ == "__main__":
    main()
