"""BASELINE config C5: the 22 Frederick St. interior stand-in (yrt.frederick, seed 2217) through
the Collada loader and the FPR stereo path (StartRT, renderer.cpp:543-737).

CPU: the stand-in is deterministic, loads through the Collada path with 2 FPR views x 12 stereo
cube cameras, window glass as ThinDielectric, one faceCamera billboard.
GPU: FPR faces of both views against the oracle at reduced size with the DLL's own defaults
(ambient .83 .95 .98, tMaxShadowRay 120 x sceneScale, depth 10; SURVEY §8(d) gate), and a small
StartRT run writing one strip per view.
"""
import hashlib

import numpy as np
import pytest

import oracle
import yrt
from yrt import frederick
from helpers import parity
from dae_scene import blob_objects

DLL = ["-tMaxShadowRay", "120", "-ambientlight", "0.83", "0.95", "0.98", "-depth", "10", "-toeIn"]


def _session(device, dae, size, spp):
    return yrt.Session(["-fprCollada", "-faceCullingMode", "default", "-i", str(dae), "-stereo", "-size", str(size),
                        str(size), "-spp", str(spp), "-fb", "RGB_FLOAT32"] + DLL, device=device)


def test_standin_is_deterministic(tmp_path):
    a = frederick.write_dae(tmp_path / "a.dae").read_bytes()
    b = frederick.write_dae(tmp_path / "b.dae").read_bytes()
    assert hashlib.sha256(a).digest() == hashlib.sha256(b).digest()
    assert 120_000 < frederick.triangle_count() < 200_000


def test_standin_loads_through_collada(host_device):
    dae = frederick.write_dae()
    s = _session(host_device, dae, 32, 1)
    assert s.num_scene_cameras() == 12 * len(frederick.CAMERAS)
    objs = blob_objects(s.export_frame(camera=s.scene_camera(0)))
    types = {o[1] for o in objs if o[0] == "MATERIAL"}
    assert {"Uber", "ThinDielectric"} <= types, types
    tris = oracle.scene_triangles(s.export_frame(camera=s.scene_camera(0)))
    # FindDegenerates drops the zero-area triangles at lathe poles (assimp post-process chain)
    assert 0.98 * frederick.triangle_count() < len(tris) <= frederick.triangle_count()
    # world in metres (unit 0.0254, Z_UP -> Y_UP): the apartment is ~11.6 x 2.7 x 7.6 m
    t = tris.reshape(-1, 3, 3)
    inside = t[(t[:, :, 1] > -0.5).all(1)]
    ext = inside.reshape(-1, 3).max(0) - inside.reshape(-1, 3).min(0)
    assert 11 < ext[0] < 12.5 and 2.7 < ext[1] < 3.2, ext
    s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cam", [0, 4, 9, 14, 21])
def test_c5_fpr_face_parity(gpu_device, cam):
    """FPR faces of both views (faceCamera billboard re-oriented per face, GPU refit) against
    the oracle on the same committed frame, 64^2 at 4 spp, depth 10."""
    s = _session(gpu_device, frederick.write_dae(), 64, 4)
    img = s.render_scene_camera(cam)
    ref, _ = oracle.render(s.export_frame(camera=s.scene_camera(cam)), 64, 64, s.info()["gamma"])
    r = parity(img, ref, 0.995)
    print(f"C5 face {cam}", r)
    s.close()


@pytest.mark.gpu
def test_c5_startrt_writes_both_views(tmp_path):
    """StartRT on the stand-in with DLL defaults (reduced size/spp): one 12-face strip per FPR
    view, named <dae>_<view>.jpg (renderer.cpp:719-720)."""
    PIL = pytest.importorskip("PIL.Image")
    dae = frederick.write_dae(tmp_path / "frederick.dae")
    p = yrt.InitParamsRT()
    p.size, p.spp = 48, 2
    assert yrt.StartRT(dae, p)
    assert yrt.WaitRT()
    assert yrt.GetLastErrorRT() == 0
    for view in frederick.CAMERAS:
        out = tmp_path / f"frederick_{view}.jpg"
        assert out.exists(), out
        a = np.asarray(PIL.open(out))
        assert a.shape == (48, 12 * 48, 3) and a.mean() > 10
