"""Debug: yrtIntersect / yrtOccluded vs the oracle on the C5 stand-in (incoherent rays)."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "yulio-raytracer_amd"), str(ROOT)]
import numpy as np
import torch
import oracle
import yrt
from yrt import frederick
dev = yrt.Device(0)
s = yrt.Session(["-fprCollada", "-faceCullingMode", "default", "-i", str(frederick.write_dae()), "-stereo", "-size", "32",
                 "32", "-spp", "1", "-fb", "RGB_FLOAT32"], device=dev)
scene = s.info()["scene"]
blob = s.export_frame(camera=s.scene_camera(0))
n = 1 << 18
rng = np.random.default_rng(7)
lo = np.array([0.0, 0.05, -5.5]); hi = np.array([11.5, 2.7, 0.0])   # inside the apartment (metres, Y up)
tri = oracle.scene_triangles(blob).reshape(-1, 3, 3)
print("bbox", tri.min((0, 1)), tri.max((0, 1)))
org = np.zeros((n, 4), np.float32); org[:, :3] = lo + (hi - lo) * rng.random((n, 3))
d = rng.normal(size=(n, 3)); d /= np.linalg.norm(d, axis=1, keepdims=True)
# a quarter of the rays axis-aligned-ish (walls are axis aligned)
d[: n // 4] = np.eye(3)[rng.integers(0, 3, n // 4)] * rng.choice([-1, 1], (n // 4, 1)) + 1e-4 * rng.normal(size=(n // 4, 3))
d /= np.linalg.norm(d, axis=1, keepdims=True)
dr = np.zeros((n, 4), np.float32); dr[:, :3] = d; dr[:, 3] = np.inf
do = dr.copy(); do[:, 3] = 3.0
ref = oracle.trace(blob, org, dr)
ref_occ = oracle.trace(blob, org, do, any_hit=True)[:, 3].view(np.int32)
hit = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
occ = torch.zeros(n, dtype=torch.int32, device="cuda")
o_t, d_t, do_t = (torch.from_numpy(a).cuda() for a in (org, dr, do))
torch.cuda.synchronize()
dev.intersect(scene, o_t.data_ptr(), d_t.data_ptr(), n, hit.data_ptr())
dev.occluded(scene, o_t.data_ptr(), do_t.data_ptr(), n, occ.data_ptr())
h = hit.cpu().numpy(); oc = occ.cpu().numpy()
tg, tc = h[:, 3].view(np.int32), ref[:, 3].view(np.int32)
mm = np.nonzero(tg != tc)[0]
print("closest mismatches", len(mm), "of", n, "occluded mismatches", int((oc != ref_occ).sum()))
for i in mm[:10]:
    print(i, org[i], dr[i], "gpu", h[i], tg[i], "ref", ref[i], tc[i])
np.savez_compressed(ROOT / "gpurun_out" / "c5trace.npz", org=org, dr=dr, do=do, h=h, ref=ref, oc=oc, ref_occ=ref_occ)
