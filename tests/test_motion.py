"""Motion blur and mesh tangents (the last shape features of
devices/device_singleray/shapes/trianglemesh_full.cpp):

* moving geometry: TriangleMeshFull "motions" (one vector per vertex, :29-33) and Sphere dPdt
  (sphere.h:38,67) — the triangle at ray time t is p + t * m (:104-109, :211-215), the BVH bounds
  both ends of the frame time (:152-166), the time is the sample's (integratorrenderer.cpp:159)
  and shadow / continuation rays inherit it (pathtraceintegrator.cpp:158,210). The reference's
  own scene models/sphere_motion.{ecs,xml} (copied to scenes/samples/) has a moving sphere and a
  moving quad.
* tangent_x / tangent_y arrays (:39-48, :244-263): interpolated per hit instead of derived from
  dP/dst, read by the anisotropic BrushedMetal microfacet.

Embree's motion-blur intersection is binary-only (unpinned); the parity reference is the oracle
restatement (bit-exact)."""
import numpy as np
import pytest

import oracle
import yrt
from helpers import SCENES, parity

MOTION = ["-c", str(SCENES / "samples" / "sphere_motion.ecs")]


def _static_copy():
    """sphere_motion.xml with the motions removed (same geometry at t = 0)."""
    import re
    src = (SCENES / "samples" / "sphere_motion.xml").read_text()
    txt = re.sub(r"<motion>[^<]*</motion>", "", src)
    txt = re.sub(r"<motions>.*?</motions>", "", txt, flags=re.S)
    assert txt != src
    gen = SCENES / "_generated"
    gen.mkdir(parents=True, exist_ok=True)
    (gen / "sphere_static.xml").write_text(txt.replace('"lines.ppm"', f'"{SCENES / "lines.ppm"}"'))
    ecs = (SCENES / "samples" / "sphere_motion.ecs").read_text().replace("sphere_motion.xml", "sphere_static.xml")
    (gen / "sphere_static.ecs").write_text(ecs)
    return ["-c", str(gen / "sphere_static.ecs")]


def test_motion_scene_loads_and_blurs(host_device):
    """The moving sphere and quad load (no 'outside scope') and the oracle's image differs from
    the same scene without motion."""
    s = yrt.Session(MOTION + ["-size", "40", "40", "-spp", "4"], device=host_device)
    info = host_device.scene_info(s.info()["scene"])
    img, st = oracle.render(s.export_frame(), 40, 40, s.info()["gamma"])
    s0 = yrt.Session(_static_copy() + ["-size", "40", "40", "-spp", "4"], device=host_device)
    info0 = host_device.scene_info(s0.info()["scene"])
    img0, _ = oracle.render(s0.export_frame(), 40, 40, s0.info()["gamma"])
    assert info["numTriangles"] == info0["numTriangles"]
    assert np.isfinite(img).all() and not np.array_equal(img, img0)
    s.close()
    s0.close()


def _tangent_scene(d, width, spp, tangents=True):
    """A BrushedMetal quad whose tangent_x / tangent_y arrays rotate the anisotropy by 30 degrees
    against the dP/dst frame, under a dome and a quad light."""
    from test_cpu_host import yrt_lookat
    mesh = d.rtNewShape("trianglemesh")
    pos = np.array([[-300, 0, -300], [300, 0, -300], [300, 0, 300], [-300, 0, 300]], np.float32)
    nor = np.array([[0, 1, 0]] * 4, np.float32)
    uv = np.array([[0, 0], [1, 0], [1, 1], [0, 1]], np.float32)
    c, s_ = np.cos(np.pi / 6), np.sin(np.pi / 6)
    tx = np.array([[c, 0, s_]] * 4, np.float32)
    ty = np.array([[-s_, 0, c]] * 4, np.float32)
    idx = np.array([[0, 2, 1], [0, 3, 2]], np.int32)
    arrays = [("positions", pos, "float3"), ("normals", nor, "float3"), ("texcoords", uv, "float2"),
              ("indices", idx, "int3")]
    if tangents:
        arrays += [("tangent_x", tx, "float3"), ("tangent_y", ty, "float3")]
    for name, arr, typ in arrays:
        dh = d.rtNewData("immutable", arr)
        d.rtSetArray(mesh, name, typ, dh, len(arr), arr.itemsize * arr.shape[1])
    d.rtCommit(mesh)
    mat = d.rtNewMaterial("BrushedMetal")
    d.rtSetFloat3(mat, "reflectance", 0.9, 0.8, 0.6)
    d.rtSetFloat1(mat, "roughnessX", 0.02)
    d.rtSetFloat1(mat, "roughnessY", 0.5)
    d.rtCommit(mat)
    amb = d.rtNewLight("ambientlight")
    d.rtSetFloat3(amb, "L", 0.3, 0.3, 0.35)
    d.rtCommit(amb)
    tl = d.rtNewLight("trianglelight")
    for n, v in (("v0", (-60, 200, -60)), ("v1", (60, 200, -60)), ("v2", (0, 200, 80)), ("L", (40, 38, 30))):
        d.rtSetFloat3(tl, n, *v)
    d.rtCommit(tl)
    scene = d.rtNewScene("default")
    d.rtSetPrimitive(scene, 0, d.rtNewShapePrimitive(mesh, mat))
    d.rtSetPrimitive(scene, 1, d.rtNewLightPrimitive(amb))
    d.rtSetPrimitive(scene, 2, d.rtNewLightPrimitive(tl))
    d.rtCommit(scene)
    cam = d.rtNewCamera("pinhole")
    d.rtSetTransform(cam, "local2world", yrt_lookat((0, 250, -420), (0, 0, 0), (0, 1, 0)))
    d.rtSetFloat1(cam, "angle", 60.0)
    d.rtSetFloat1(cam, "aspectRatio", 1.0)
    d.rtCommit(cam)
    r = d.rtNewRenderer("pathtracer")
    d.rtSetInt1(r, "maxDepth", 3)
    d.rtSetInt1(r, "sampler.spp", spp)
    d.rtSetFloat1(r, "tMaxShadowRay", 1e4)
    d.rtCommit(r)
    tm = d.rtNewToneMapper("default")
    d.rtCommit(tm)
    fb = d.rtNewFrameBuffer("RGB_FLOAT32", width, width)
    return r, cam, scene, tm, fb


def test_tangent_arrays_change_the_brushed_frame(host_device):
    """The tangent arrays reach the oracle through the frame blob and steer the anisotropic
    highlight: the image differs from the same quad without them."""
    d = host_device
    r, cam, scene, tm, fb = _tangent_scene(d, 32, 4)
    img, _ = oracle.render(d.export_frame(r, cam, scene), 32, 32, 1.0)
    blob = d.export_frame(r, cam, scene)
    assert b"tangent_x" in blob and b"tangent_y" in blob
    assert np.isfinite(img).all() and img.mean() > 0
    r0, cam0, scene0, _, _ = _tangent_scene(d, 32, 4, tangents=False)
    img0, _ = oracle.render(d.export_frame(r0, cam0, scene0), 32, 32, 1.0)
    assert not np.array_equal(img, img0)


@pytest.mark.gpu
def test_motion_blur_parity(gpu_device):
    """sphere_motion (the reference's scene) on the GPU against the oracle, RGB_FLOAT32,
    bit-exact: the moving-triangle trace kernels, the per-ray time queues and the moving
    vertices in postIntersect."""
    s = yrt.Session(MOTION + ["-size", "80", "60", "-spp", "8", "-fb", "RGB_FLOAT32"], device=gpu_device)
    img = s.render()
    ref, st = oracle.render(s.export_frame(), 80, 60, s.info()["gamma"])
    parity(img, ref, 0.999)
    assert gpu_device.render_stats()["raysClosest"] == st["raysClosest"]
    s.close()


@pytest.mark.gpu
def test_tangent_arrays_parity(gpu_device):
    d = gpu_device
    r, cam, scene, tm, fb = _tangent_scene(d, 64, 8)
    d.rtRenderFrame(r, cam, scene, tm, fb, 0)
    img = d.framebuffer_array(fb, 64, 64, "RGB_FLOAT32")
    ref, _ = oracle.render(d.export_frame(r, cam, scene), 64, 64, 1.0)
    parity(img, ref, 0.999)


def _sphere_scene(d, dpdt=None):
    """A Matte sphere under a dome; `dpdt` sets the sphere's motion (sphere.h:38,67)."""
    from test_cpu_host import yrt_lookat
    sph = d.rtNewShape("sphere")
    d.rtSetFloat3(sph, "P", 0.0, 0.0, 0.0)
    d.rtSetFloat1(sph, "r", 1.0)
    d.rtSetInt1(sph, "numTheta", 16)
    d.rtSetInt1(sph, "numPhi", 32)
    if dpdt is not None:
        d.rtSetFloat3(sph, "dPdt", *dpdt)
    d.rtCommit(sph)
    mat = d.rtNewMaterial("Matte")
    d.rtSetFloat3(mat, "reflectance", 0.7, 0.5, 0.3)
    d.rtCommit(mat)
    amb = d.rtNewLight("ambientlight")
    d.rtSetFloat3(amb, "L", 1.0, 1.0, 1.0)
    d.rtCommit(amb)
    cam = d.rtNewCamera("pinhole")
    d.rtSetTransform(cam, "local2world", yrt_lookat((0, 0, -4), (0, 0, 0), (0, 1, 0)))
    d.rtSetFloat1(cam, "angle", 50.0)
    d.rtSetFloat1(cam, "aspectRatio", 1.0)
    d.rtCommit(cam)
    r = d.rtNewRenderer("pathtracer")
    d.rtSetInt1(r, "maxDepth", 2)
    d.rtSetInt1(r, "sampler.spp", 8)
    d.rtCommit(r)
    tm = d.rtNewToneMapper("default")
    d.rtCommit(tm)
    fb = d.rtNewFrameBuffer("RGB_FLOAT32", 48, 48)
    return sph, mat, amb, cam, r, tm, fb


@pytest.mark.gpu
def test_recommit_with_changed_motion_rebuilds(gpu_device):
    """A scene re-committed after its sphere gained a dPdt (same vertices at t = 0) must render
    the moving sphere: the faceCamera refit re-uploads positions and normals only, so the commit
    rebuilds instead (the old compare saw 'same geometry' and kept the static scene)."""
    d = gpu_device
    sph, mat, amb, cam, r, tm, fb = _sphere_scene(d)
    scene = d.rtNewScene("default")
    d.rtSetPrimitive(scene, 0, d.rtNewShapePrimitive(sph, mat))
    d.rtSetPrimitive(scene, 1, d.rtNewLightPrimitive(amb))
    d.rtCommit(scene)
    d.rtRenderFrame(r, cam, scene, tm, fb, 0)
    static = d.framebuffer_array(fb, 48, 48, "RGB_FLOAT32").copy()
    d.rtSetFloat3(sph, "dPdt", 0.6, 0.0, 0.0)
    d.rtCommit(sph)
    d.rtSetPrimitive(scene, 0, d.rtNewShapePrimitive(sph, mat))
    d.rtCommit(scene)
    assert d.scene_refits(scene) == 0  # rebuilt, not refit
    d.rtRenderFrame(r, cam, scene, tm, fb, 0)
    moving = d.framebuffer_array(fb, 48, 48, "RGB_FLOAT32")
    ref, _ = oracle.render(d.export_frame(r, cam, scene), 48, 48, 1.0)
    assert not np.array_equal(moving, static)
    parity(moving, ref, 0.999)
