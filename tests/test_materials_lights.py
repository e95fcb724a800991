"""the reference materials and lights outside the BASELINE configs —
Plastic, Dielectric (with medium tracking and the volumetric transmission term), Mirror,
Metal, BrushedMetal, Velvet (devices/device_singleray/materials/*.h) and point, spot,
directional, distant lights (lights/*.h) — through the XML loader and the command-line tags
(scenes/materials_lights.{xml,ecs}, written by tools/make_materials_scene.py), GPU against
the oracle restatement on the same frame."""
import numpy as np
import pytest

import dae_scene
import oracle
import yrt
from helpers import SCENES, parity

ARGS = ["-c", str(SCENES / "materials_lights.ecs")]


def test_scene_objects_and_defaults(host_device):
    s = yrt.Session(ARGS + ["-size", "32", "32"], device=host_device)
    objs = dae_scene.blob_objects(s.export_frame())
    mats = sorted({o[1] for o in objs if o[0] == "MATERIAL"})
    lights = sorted({o[1] for o in objs if o[0] == "LIGHT"})
    assert mats == ["BrushedMetal", "Dielectric", "Matte", "Metal", "Mirror", "Plastic", "Velvet"]
    assert lights == ["ambientlight", "directionallight", "distantlight", "pointlight", "spotlight"]
    spot = [o[2] for o in objs if o[1] == "spotlight"][0]
    assert spot["D"][:3] == pytest.approx((0.0, -1.0, 0.0))  # AffineSpace column vz (xml_loader.cpp:293)
    assert spot["angleMin"][0] == 35 and spot["angleMax"][0] == 55
    s.close()


def test_masked_pointlight_tag(host_device):
    s = yrt.Session(ARGS + ["-size", "16", "16", "-masked_pointlight", "1", "2", "3", "10", "10", "10", "2", "5"],
                    device=host_device)
    assert oracle.render(s.export_frame(), 16, 16, 1.0)[0].mean() > 0
    s.close()


def test_oracle_render(host_device):
    s = yrt.Session(ARGS + ["-size", "24", "18", "-spp", "2"], device=host_device)
    img, st = oracle.render(s.export_frame(), 24, 18, 1.0)
    assert np.isfinite(img).all() and img.mean() > 0.02
    assert st["raysShadow"] > st["raysClosest"]  # five lights per diffuse vertex
    s.close()


def test_unknown_types_raise(host_device):
    with pytest.raises(RuntimeError, match="unknown material type"):
        host_device.rtNewMaterial("Chrome")
    with pytest.raises(RuntimeError, match="unknown light type"):
        host_device.rtNewLight("arealight")


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [2, 6])
def test_materials_lights_parity(gpu_device, depth):
    """GPU vs oracle, RGB_FLOAT32: every new BRDF component (reflection, conductor, rough and
    anisotropic conductor microfacets, Minnaert, Velvety, dielectric transmission through two
    interfaces with the in-medium attenuation) and every light sampler."""
    s = yrt.Session(ARGS + ["-size", "96", "72", "-spp", "8", "-depth", str(depth), "-fb", "RGB_FLOAT32"],
                    device=gpu_device)
    img = s.render()
    ref, _ = oracle.render(s.export_frame(), 96, 72, s.info()["gamma"])
    parity(img, ref, 0.995)
    s.close()


def test_depth_of_field_camera_object(host_device):
    """-radius r selects DepthOfFieldCamera (renderer.cpp:312-331): lensRadius r and the
    focal distance |lookAt - position|."""
    s = yrt.Session(ARGS + ["-size", "24", "18", "-radius", "6"], device=host_device)
    objs = dae_scene.blob_objects(s.export_frame())
    cam = [o for o in objs if o[0] == "CAMERA"][0]
    assert cam[1] == "depthoffield" and cam[2]["lensRadius"][0] == 6.0
    assert cam[2]["focalDistance"][0] == pytest.approx(float(np.linalg.norm([0, 440, 720])), rel=1e-6)
    assert np.isfinite(oracle.render(s.export_frame(), 24, 18, 1.0)[0]).all()
    s.close()


@pytest.mark.gpu
def test_depth_of_field_parity(gpu_device):
    """Thin-lens rays from the sampler's lens dimensions (sample.getLens()), GPU vs oracle."""
    s = yrt.Session(ARGS + ["-size", "80", "60", "-spp", "8", "-radius", "12", "-fb", "RGB_FLOAT32"],
                    device=gpu_device)
    img = s.render()
    ref, _ = oracle.render(s.export_frame(), 80, 60, s.info()["gamma"])
    parity(img, ref, 0.995)
    s.close()


def test_backplate_oracle(host_device):
    """-backplate (renderer.cpp:1259-1263; pathtraceintegrator.cpp:80-84): straight camera
    rays that miss the scene see the backplate at their image-plane position instead of the
    environment; bent paths still see the environment."""
    from helpers import c4_args, SCENES
    base = c4_args(48, 1, stereo=False)
    s0 = yrt.Session(base + ["-fb", "RGB_FLOAT32"], device=host_device)
    s1 = yrt.Session(base + ["-backplate", str(SCENES / "logo.png"), "-fb", "RGB_FLOAT32"], device=host_device)
    objs = dae_scene.blob_objects(s1.export_frame())
    rend = [o for o in objs if o[0] == "RENDERER"][0]
    assert "backplate" in rend[2]
    a, _ = oracle.render(s0.export_frame(), 48, 48, 1.0)
    b, _ = oracle.render(s1.export_frame(), 48, 48, 1.0)
    assert not np.array_equal(a, b)
    s0.close()
    s1.close()


@pytest.mark.gpu
def test_backplate_parity(gpu_device):
    """The backplate on the device, bit-identical to the oracle (C4 view: most camera rays
    leave toward the sky, so the backplate fills the background)."""
    from helpers import c4_args, SCENES
    s = yrt.Session(c4_args(96, 4, stereo=False) + ["-backplate", str(SCENES / "lines.ppm"), "-fb", "RGB_FLOAT32"],
                    device=gpu_device)
    img = s.render()
    ref, _ = oracle.render(s.export_frame(), 96, 96, s.info()["gamma"])
    parity(img, ref, 0.999)
    s.close()


# the camera of models/cornell_box_spheres.ecs:2
CAM = ["-vp", "278", "273", "-800", "-vi", "278", "273", "0", "-vu", "0", "1", "0", "-fov", "37"]


def _glitter_scene():
    """models/cornell_box_spheres.xml with metallic glitter on both MetallicPaint spheres
    (materials/metallicpaint.h:36-42 parameters glitterColor / glitterSpread): the red sphere
    with broad silver flakes, the green one with tight gold flakes."""
    src = (SCENES / "cornell_box_spheres.xml").read_text()
    red = '<float3 name="shadeColor">0.5 0.0 0.0</float3>'
    green = '<float3 name="shadeColor">0.0 0.5 0.0</float3>'
    assert red in src and green in src
    txt = src.replace(red, red + '<float3 name="glitterColor">0.8 0.8 0.8</float3><float name="glitterSpread">0.5</float>')
    txt = txt.replace(green, green + '<float3 name="glitterColor">0.9 0.7 0.2</float3>'
                                     '<float name="glitterSpread">0.05</float>')
    out = SCENES / "_generated" / "cornell_box_spheres_glitter.xml"
    out.parent.mkdir(parents=True, exist_ok=True)
    out.write_text(txt)
    return out


def _glitter_args(size, spp, depth=4):
    return ["-i", str(_glitter_scene())] + CAM + ["-size", str(size), str(size), "-spp", str(spp), "-depth", str(depth)]


def test_glitter_oracle_brightens_spheres(host_device):
    """The glitter layer (a third, glossy component) adds flake reflections: the oracle's image of
    the spheres with glitter is brighter than without, with the same geometry and lights."""
    from helpers import c2_args
    s = yrt.Session(_glitter_args(48, 4), device=host_device)
    objs = dae_scene.blob_objects(s.export_frame())
    paints = [o[2] for o in objs if o[0] == "MATERIAL" and o[1] == "MetallicPaint"]
    assert len(paints) == 2 and all("glitterColor" in p for p in paints)
    img, _ = oracle.render(s.export_frame(), 48, 48, 1.0)
    s.close()
    s0 = yrt.Session(c2_args(48, 4) + ["-depth", "4"], device=host_device)
    img0, _ = oracle.render(s0.export_frame(), 48, 48, 1.0)
    s0.close()
    assert np.isfinite(img).all() and img.mean() > img0.mean()


@pytest.mark.gpu
def test_glitter_parity(gpu_device):
    """MetallicPaint with glitter (DielectricLayer<Microfacet<FresnelConductor, PowerCosine>>,
    metallicpaint.h:63-70) on the GPU against the oracle, RGB_FLOAT32, bit-exact."""
    s = yrt.Session(_glitter_args(96, 8) + ["-fb", "RGB_FLOAT32"], device=gpu_device)
    img = s.render()
    ref, _ = oracle.render(s.export_frame(), 96, 96, s.info()["gamma"])
    parity(img, ref, 0.999)
    s.close()


def _disk_scene():
    """models/cornell_box_spheres.xml plus three reference Disk shapes (xml_loader.cpp:491-504,
    shapes/disk.h): a flat disk on the floor, a cone (height > 0) and a coarse 5-triangle fan
    under a rotation, which exercises all three fan windings (phi % 3)."""
    src = (SCENES / "cornell_box_spheres.xml").read_text()
    mat = '<material><code>"Matte"</code><parameters><float3 name="reflectance">{}</float3></parameters></material>'
    disks = (f'<Disk><position>400 0.5 120</position><radius>80</radius><numTriangles>48</numTriangles>'
             f'{mat.format("0.2 0.3 0.8")}</Disk>'
             f'<Transform><AffineSpace>1 0 0 0  0 0 -1 0  0 1 0 0</AffineSpace>'
             f'<Disk><position>120 -400 0</position><radius>60</radius><height>150</height>'
             f'<numTriangles>24</numTriangles>{mat.format("0.8 0.7 0.2")}</Disk></Transform>'
             f'<Transform><AffineSpace>0 0 1 420  0 1 0 260  -1 0 0 380</AffineSpace>'
             f'<Disk><position>0 0 0</position><radius>70</radius><height>-40</height>'
             f'<numTriangles>5</numTriangles>{mat.format("0.7 0.7 0.7")}</Disk></Transform>')
    assert src.count("</Group>") == 1
    out = SCENES / "_generated" / "cornell_box_spheres_disks.xml"
    out.parent.mkdir(parents=True, exist_ok=True)
    out.write_text(src.replace("</Group>", disks + "</Group>"))
    return out


def test_disk_shapes_tessellate(host_device):
    """Disk (shapes/disk.h:45-65): numTriangles + 1 vertices (rim + apex), numTriangles
    triangles; the oracle rebuilds the same triangles from the frame blob."""
    s = yrt.Session(["-i", str(_disk_scene())] + CAM + ["-size", "32", "32"], device=host_device)
    info = host_device.scene_info(s.info()["scene"])
    base = yrt.Session(["-i", str(SCENES / "cornell_box_spheres.xml")] + CAM + ["-size", "32", "32"],
                       device=host_device)
    assert info["numTriangles"] - host_device.scene_info(base.info()["scene"])["numTriangles"] == 48 + 24 + 5
    tris = oracle.scene_triangles(s.export_frame())
    assert len(tris) == info["numTriangles"]
    img, _ = oracle.render(s.export_frame(), 32, 32, 1.0)
    assert np.isfinite(img).all()
    s.close()
    base.close()


@pytest.mark.gpu
def test_disk_parity(gpu_device):
    """Disk and cone shapes on the GPU against the oracle, RGB_FLOAT32, bit-exact."""
    s = yrt.Session(["-i", str(_disk_scene())] + CAM + ["-size", "96", "96", "-spp", "8", "-depth", "3", "-fb",
                                                         "RGB_FLOAT32"], device=gpu_device)
    img = s.render()
    ref, _ = oracle.render(s.export_frame(), 96, 96, s.info()["gamma"])
    parity(img, ref, 0.999)
    s.close()
