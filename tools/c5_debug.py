"""Debug: GPU vs oracle on one C5 FPR face; saves both images for offline analysis."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "yulio-raytracer_amd"), str(ROOT)]
import numpy as np
import oracle
import yrt
from yrt import frederick
cam = int(sys.argv[1]) if len(sys.argv) > 1 else 0
size, spp = 64, 4
dev = yrt.Device(0)
dae = frederick.write_dae()
extra = sys.argv[2:]  # extra session args
s = yrt.Session(["-fprCollada", "-faceCullingMode", "default", "-i", str(dae), "-stereo", "-size", str(size), str(size),
                 "-spp", str(spp), "-fb", "RGB_FLOAT32", "-tMaxShadowRay", "120", "-ambientlight", "0.83", "0.95",
                 "0.98", "-depth", "10", "-toeIn"] + extra, device=dev)
img = s.render_scene_camera(cam)
blob = s.export_frame(camera=s.scene_camera(cam))
ref, _ = oracle.render(blob, size, size, s.info()["gamma"])
d = np.abs(img - ref)
print("cam", cam, "frac_ok", ((d <= 1e-3 + 1e-3 * np.abs(ref)).mean()), "mad", d.mean(), "mean", ref.mean())
out = ROOT / "gpurun_out" / f"c5dbg_{cam}.npz"
np.savez_compressed(out, img=img, ref=ref, blob=np.frombuffer(blob, np.uint8))
