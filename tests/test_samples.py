"""The reference's own sample scenes (models/*.xml, *.ecs, copied as data into scenes/samples/):
glass, mirror and car-paint spheres over a textured floor under the HDRI light, the
transmissive-materials scene, through the reference's own stereo view (sphere_view.ecs:
-stereo, -depth 8, -ambientlight 1 0 0). The reference ships no rendered images of them, so
parity is against the oracle restatement on the same committed frame (bit-exact), at reduced
size; the CPU test checks that each loads and renders on the oracle."""
import numpy as np
import pytest

import oracle
import yrt
from helpers import SCENES, parity

S = SCENES / "samples"
SCENES_ARGS = {
    "sphere_glass": ["-c", str(S / "sphere_glass.ecs")],
    "sphere_mirror": ["-c", str(S / "sphere_mirror.ecs")],
    "sphere_carpaint": ["-i", str(S / "sphere_carpaint.xml"), "-c", str(S / "sphere_view.ecs")],
    "test_transmissive": ["-i", str(S / "test_transmissive.xml"), "-c", str(S / "sphere_view.ecs")],
}


@pytest.mark.parametrize("name", sorted(SCENES_ARGS))
def test_sample_scene_loads_and_renders_on_oracle(host_device, name):
    s = yrt.Session(SCENES_ARGS[name] + ["-size", "24", "24", "-spp", "2"], device=host_device)
    info = s.info()
    assert info["stereo"] == 1  # sphere_view.ecs:11
    img, st = oracle.render(s.export_frame(0), 24, 24, info["gamma"])
    assert np.isfinite(img).all() and img.mean() > 0 and st["raysClosest"] > 0
    s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(SCENES_ARGS))
@pytest.mark.parametrize("face", [0, 5, 8])
def test_sample_scene_parity(gpu_device, name, face):
    s = yrt.Session(SCENES_ARGS[name] + ["-size", "64", "64", "-spp", "4", "-fb", "RGB_FLOAT32"], device=gpu_device)
    img = s.render(face)
    ref, _ = oracle.render(s.export_frame(face), 64, 64, s.info()["gamma"])
    # test_transmissive's ThinDielectric spheres (eta 1, transmission with zero channels): the
    # restated reference arithmetic gives NaN samples on some paths (log(0) absorption), the
    # GPU must give them on the same pixels
    parity(img, ref, 0.999, nan_ok=name == "test_transmissive")
    s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("face", [0, 5])
def test_zero_radiance_lights_parity(gpu_device, face):
    """A second dome light with L = 0 0 0 on the transmissive scene: the device leaves it out of
    the direct-light and miss loops (its terms are exactly 0), but a path whose throughput is
    already NaN (this scene's ThinDielectric log(0) * 0) must still turn NaN at a miss, as the
    reference's `L += throughput * 0` does. Bit-exact against the oracle, NaN masks included."""
    s = yrt.Session(SCENES_ARGS["test_transmissive"] + ["-ambientlight", "0", "0", "0", "-size", "64", "64", "-spp",
                                                        "4", "-fb", "RGB_FLOAT32"], device=gpu_device)
    img = s.render(face)
    ref, _ = oracle.render(s.export_frame(face), 64, 64, s.info()["gamma"])
    parity(img, ref, 0.999, nan_ok=True)
    s.close()
