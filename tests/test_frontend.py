"""Front-end outputs: JPEG writer pinned against libjpeg-turbo (via PIL), stereo cube strip
layout, StartRT/WaitRT/StopRT file contract (renderer.cpp:543-737, 1483-1657)."""
import io
import shutil

import numpy as np
import pytest

import yrt
from helpers import SCENES


def _requant(img):
    """Image3c -> Color4 -> byte round trip (common/math/color_scalar.h:45-60)."""
    return (np.clip(img.astype(np.float32) * np.float32(1.0 / 255.0), 0, 1) * np.float32(255.0)).astype(np.uint8)


@pytest.mark.parametrize("shape", [(64, 64), (37, 53), (16, 16), (100, 1), (48, 200)])
@pytest.mark.parametrize("quality", [90, 75, 50, 10, 100])
def test_jpeg_writer_matches_libjpeg(tmp_path, shape, quality):
    """Baseline 4:2:0 JPEG: same DCT coefficients as libjpeg-turbo at the same quality
    (decoded pixels identical). The reference stores through FreeImage (freeimage.cpp:191-232)."""
    PIL = pytest.importorskip("PIL.Image")
    rng = np.random.default_rng(shape[0] * 1000 + shape[1] + quality)
    h, w = shape
    img = np.clip(np.cumsum(rng.integers(-40, 41, (h, w, 3)), axis=1) + 128, 0, 255).astype(np.uint8)
    f = tmp_path / "a.jpg"
    yrt.store_image(f, img, quality)
    mine = np.asarray(PIL.open(f).convert("RGB"))
    bio = io.BytesIO()
    PIL.fromarray(_requant(img)).save(bio, "JPEG", quality=quality, subsampling=2)
    ref = np.asarray(PIL.open(io.BytesIO(bio.getvalue())).convert("RGB"))
    assert np.array_equal(mine, ref)


def test_store_ppm_png_roundtrip(tmp_path):
    PIL = pytest.importorskip("PIL.Image")
    img = (np.arange(30 * 20 * 3) % 251).astype(np.uint8).reshape(20, 30, 3)
    for ext in ("ppm", "png"):
        f = tmp_path / f"a.{ext}"
        yrt.store_image(f, img)
        assert np.array_equal(np.asarray(PIL.open(f).convert("RGB")), img)


def test_store_rejects_unknown_format(tmp_path):
    with pytest.raises(RuntimeError, match="not supported"):
        yrt.store_image(tmp_path / "a.tga", np.zeros((4, 4, 3), np.uint8))


def test_watermark_resource_decodes():
    from pathlib import Path
    f = Path(yrt.__file__).resolve().parent.parent / "resources" / "watermarkwhitetrasp_100x100.png"
    px = yrt.decode_image(f)
    assert px.shape == (100, 100, 4) and px[..., 3].max() > 0


# ----------------------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_stereo_strip_layout(gpu_device, tmp_path):
    """-stereo -o: 12 faces in one strip, right eye first, each eye L,R,U,D,B,F
    (renderer.cpp:820-877), bytes through Color4 (Q7)."""
    args = ["-i", str(SCENES / "test_stereo.xml"), "-c", str(SCENES / "test_stereo_view.ecs"), "-size", "32", "32",
            "-spp", "1", "-stereo"]
    s = yrt.Session(args, device=gpu_device)
    faces = [s.render(i) for i in range(12)]
    out = tmp_path / "strip.ppm"
    s.output(str(out))
    PIL = pytest.importorskip("PIL.Image")
    strip = np.asarray(PIL.open(out).convert("RGB"))
    assert strip.shape == (32, 12 * 32, 3)
    order = [3, 1, 4, 5, 2, 0]
    for seg in range(12):
        eye = 1 if seg < 6 else 0
        face = 6 * eye + order[seg % 6]
        assert np.array_equal(strip[:, seg * 32:(seg + 1) * 32], _requant(faces[face])), seg
    s.close()


@pytest.mark.gpu
def test_startrt_writes_cubemap_jpeg(tmp_path):
    """StartRT on an .ecs scene renders the stereo rig and writes <name>_cubemap.jpg; the
    watermark changes only the front/back/side faces (renderer.cpp:636-655)."""
    PIL = pytest.importorskip("PIL.Image")
    for f in ("cornell_box.ecs", "cornell_box.obj", "cornell_box.mtl"):
        shutil.copy(SCENES / f, tmp_path / f)
    imgs = {}
    for wm in (False, True):
        p = yrt.InitParamsRT()
        p.size, p.spp, p.depth = 128, 1, 2
        p.waterMark = wm
        assert yrt.StartRT(tmp_path / "cornell_box.ecs", p)
        assert yrt.WaitRT()
        st = yrt.GetCurrentStatusRT()
        assert st.state == 4 and yrt.GetLastErrorRT() == 0  # Done, NoError
        out = tmp_path / "cornell_box_cubemap.jpg"
        assert out.exists()
        imgs[wm] = np.asarray(PIL.open(out).convert("RGB")).astype(int)
        out.unlink()
    a, b = imgs[False], imgs[True]
    assert a.shape == (128, 12 * 128, 3)
    diff = np.abs(a - b).reshape(128, 12, 128, 3).max(axis=(0, 2, 3))
    # strip segments L,R,U,D,B,F per eye: U and D (2,3 / 8,9) carry no watermark
    assert all(diff[k] > 0 for k in (0, 1, 4, 5, 6, 7, 10, 11)), diff
    assert all(diff[k] <= 2 for k in (2, 3, 8, 9)), diff


@pytest.mark.gpu
def test_stoprt_cancels_a_running_render(tmp_path):
    """StopRT during a long StartRT (default ParamsRT but 4096 spp: 1536^2 faces; the cubemap
    at the default 256 spp — a camera outside the open box, mostly sky — now renders in about
    a second, within the sleep below): a second StartRT is refused with RenderingIsInProgress,
    the stop flag ends the render at the next wavefront batch, the state becomes Stopped and,
    keepResults = false, no image is left (renderer.cpp:724-731, 1606-1641)."""
    import time
    for f in ("cornell_box.ecs", "cornell_box.obj", "cornell_box.mtl"):
        shutil.copy(SCENES / f, tmp_path / f)
    p = yrt.InitParamsRT()
    p.spp = 4096
    assert yrt.StartRT(tmp_path / "cornell_box.ecs", p)
    assert not yrt.StartRT(tmp_path / "cornell_box.ecs", p)
    assert yrt.GetLastErrorRT() == 1  # RenderingIsInProgress
    time.sleep(1.0)
    t0 = time.time()
    assert yrt.StopRT(False)
    assert time.time() - t0 < 60
    st = yrt.GetCurrentStatusRT()
    assert st.state == 3  # Stopped
    assert not (tmp_path / "cornell_box_cubemap.jpg").exists()
    assert not yrt.WaitRT()  # nothing left to wait for


@pytest.mark.parametrize("mangle", [
    ("<!-- light -->", "<!-\r light -->"),          # a broken comment opener (fuzz finding, r05)
    ('<float name="eta">', '<float name="eta>'),    # an attribute value without its closing quote
    ('<float name="eta">', '<float name=eta>'),     # an unquoted attribute value
    ("</scene>", "</scene"),                        # an end tag without '>'
    ("<Group>", "<>"),                              # an empty element name
], ids=["comment", "quote", "unquoted", "endtag", "noname"])
def test_malformed_xml_fails_cleanly(host_device, tmp_path, mangle):
    """The XML scene reader refuses malformed text with an error instead of looping: a mangled
    comment opener once wrapped its scan index past npos back to 0 and parsed forever
    (tools/run_sanitizers.sh mutation fuzz, profiles/r05/sanitizers_r05.txt)."""
    import time
    src = (SCENES / "cornell_box_spheres.xml").read_text()
    assert mangle[0] in src
    f = tmp_path / "mangled.xml"
    f.write_text(src.replace(mangle[0], mangle[1], 1))
    t = time.perf_counter()
    with pytest.raises(RuntimeError):
        yrt.Session(["-i", str(f), "-size", "16", "16"], device=host_device)
    assert time.perf_counter() - t < 10


def test_obj_short_faces_and_mixed_normals(host_device, tmp_path):
    """OBJ faces of fewer than three vertices yield no triangle (the fan read face[1] of a
    one-vertex face: a heap overread under ASan, tools/run_sanitizers.sh mutation fuzz), and a
    group mixing vertices with and without normals is refused instead of handing the mesh a
    normal array shorter than its positions."""
    f = tmp_path / "short.obj"
    f.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1\nf 1 2\nf 1 2 3\n")
    s = yrt.Session(["-i", str(f), "-size", "16", "16"], device=host_device)
    assert host_device.scene_info(s.info()["scene"])["numTriangles"] == 1
    s.close()
    h = tmp_path / "stray_cr.obj"  # a '\r' inside a face line once looped forever (fuzz finding)
    h.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2\r 3\n")
    with pytest.raises(RuntimeError, match="malformed face"):
        yrt.Session(["-i", str(h), "-size", "16", "16"], device=host_device)
    g = tmp_path / "mixed.obj"
    g.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nv 1 1 0\nvn 0 0 1\nf 1//1 2//1 3//1\nf 2 4 3\n")
    with pytest.raises(RuntimeError, match="normals"):
        yrt.Session(["-i", str(g), "-size", "16", "16"], device=host_device)
