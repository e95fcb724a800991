"""Parity of the MI355X HIP path (through the C ABI) with the CPU oracle.

Oracle: oracle/ (CPU restatement of the reference's device_singleray path, see its header
for the file:line it follows). Tolerances: SURVEY.md §8(d) — |g-c| <= 1e-3 + 1e-3|c| on
>= 99.9 % of channels (C1/C2) / 99.5 % (C3/C4) and mean-abs-diff <= 1e-4 * mean; integer
outputs (debug renderer ids, hit triangle ids, occlusion flags) bit-exact.
"""
import numpy as np
import pytest

import oracle
import yrt
from helpers import c1_args, c2_args, c3_args, c4_args, parity

pytestmark = pytest.mark.gpu


def _session(dev, args):
    return yrt.Session(args + ["-fb", "RGB_FLOAT32"], device=dev)


def _render_pair(dev, args, face=-1, threads=0):
    s = _session(dev, args)
    info = s.info()
    img = s.render(face)
    blob = s.export_frame(face)
    ref, _ = oracle.render(blob, info["width"], info["height"], info["gamma"], threads=threads)
    stats = dev.render_stats()
    s.close()
    return img, ref, stats


# ----------------------------------------------------------------------------- debug renderer
@pytest.mark.parametrize("args", [c1_args(128), c2_args(128, 1), c4_args(96, 1, stereo=False)],
                         ids=["C1", "C2", "C4"])
def test_debug_renderer_bit_exact(gpu_device, args):
    """DebugRenderer (renderers/debugrenderer.cpp:66-140) id-hash image: integer-exact traversal KAT."""
    img, ref, _ = _render_pair(gpu_device, args + ["-renderer", "debug"])
    assert np.array_equal(img, ref), np.argwhere(img != ref)[:5]


# ----------------------------------------------------------------------------- arithmetic
def test_fast_reciprocal_is_correctly_rounded(gpu_device):
    """The kernels' rcp_rn (v_rcp_f32 + one FMA Newton step, IEEE division outside
    [2^-124, 2^124)) equals the IEEE division 1.0f/x for all 2^32 inputs, so shading stays
    bit-exact with the oracle's 1/x."""
    import ctypes as C
    from yrt import _native as N
    out = (C.c_uint64 * 2)()
    assert N.dev.yrtDebugCheckMath(gpu_device.h, 0, out) == 0, gpu_device.error()
    assert out[0] == 0, f"{out[0]} mismatches, first input bits {out[1]:#x}"


@pytest.mark.parametrize("fn,key", [(1, "rcpps_mantissa12"), (2, "rsqrtps_mantissa12")])
def test_sse_estimates_match_the_intel_tables(gpu_device, fn, key):
    """The kernels' emulation of rcpps / rsqrtps (the estimates the reference's rcp/rsqrt start
    from, common/math/math.h:38-59; yrt_sse_rcp.h) equals the committed Intel tables
    (tests/golden/sse_rcp_tables.json) on all 2^32 inputs: the GPU computes the reference's
    reciprocals bit for bit, like the host and the oracle (tests/test_sse_rcp.py,
    tests/test_ref_pin.py)."""
    import ctypes as C
    import json
    from pathlib import Path
    from yrt import _native as N
    fix = json.loads((Path(__file__).resolve().parent / "golden" / "sse_rcp_tables.json").read_text())
    tab = np.ascontiguousarray(fix[key], np.uint16)
    out = (C.c_uint64 * 2)()
    assert N.dev.yrtDebugCheckMathTable(gpu_device.h, fn, tab.ctypes.data, out) == 0, gpu_device.error()
    assert out[0] == 0, f"{out[0]} mismatches, first input bits {out[1]:#x}"


# ----------------------------------------------------------------------------- ray queries
def _rays(blob, n, seed=42):
    """SURVEY §8(d)(ii) incoherent rays: origins uniform in the scene AABB, directions on S^2."""
    tris = oracle.scene_triangles(blob).reshape(-1, 3, 3)
    lo, hi = tris.min(axis=(0, 1)), tris.max(axis=(0, 1))
    rng = np.random.default_rng(seed)
    org = rng.uniform(lo, hi, size=(n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    org4 = np.concatenate([org, np.zeros((n, 1), np.float32)], 1).astype(np.float32)
    dir4 = np.concatenate([d.astype(np.float32), np.full((n, 1), np.inf, np.float32)], 1)
    return org4, dir4


@pytest.mark.parametrize("which", ["C2", "C3", "C4"])
def test_intersect_and_occluded(gpu_device, which):
    import torch
    args = {"C2": c2_args(64, 1), "C3": c3_args(64, 1), "C4": c4_args(64, 1, stereo=False)}[which]
    s = _session(gpu_device, args)
    info = s.info()
    scene = info["scene"]
    blob = s.export_frame()
    org4, dir4 = _rays(blob, 1 << 16)
    # finite tfar for half the occlusion queries
    dir4_occ = dir4.copy()
    dir4_occ[::2, 3] = 50.0
    ref = oracle.trace(blob, org4, dir4)
    ref_occ = oracle.trace(blob, org4, dir4_occ, any_hit=True)[:, 3].view(np.int32)
    o = torch.from_numpy(org4).cuda()
    dd = torch.from_numpy(dir4).cuda()
    do = torch.from_numpy(dir4_occ).cuda()
    hit = torch.zeros((len(org4), 4), dtype=torch.float32, device="cuda")
    occ = torch.zeros(len(org4), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    gpu_device.intersect(scene, o.data_ptr(), dd.data_ptr(), len(org4), hit.data_ptr())
    gpu_device.occluded(scene, o.data_ptr(), do.data_ptr(), len(org4), occ.data_ptr())
    h = hit.cpu().numpy()
    tri_g = h[:, 3].view(np.int32)
    tri_c = ref[:, 3].view(np.int32)
    mism = tri_g != tri_c
    assert mism.mean() == 0.0, (mism.sum(), np.argwhere(mism)[:5])
    m = tri_c >= 0
    np.testing.assert_allclose(h[m, :3], ref[m, :3], rtol=1e-5, atol=1e-6)
    assert np.array_equal(occ.cpu().numpy(), ref_occ)
    s.close()


@pytest.mark.parametrize("name", ["c2", "c3"])
def test_intersect_golden_records(gpu_device, name):
    """KAT 4 on the device: yrtIntersect / yrtOccluded on the committed incoherent rays give
    the committed triangle ids and occlusion flags bit-exactly, t/u/v within 1e-5."""
    import torch
    from pathlib import Path
    g = np.load(Path(__file__).parent / "golden" / f"hits_{name}_4096.npz")
    args = {"c2": c2_args(32, 1), "c3": c3_args(32, 1)}[name]
    s = _session(gpu_device, args)
    scene = s.info()["scene"]
    n = len(g["org"])
    o = torch.from_numpy(g["org"]).cuda()
    dd = torch.from_numpy(g["dir"]).cuda()
    do = torch.from_numpy(g["occ_dir"]).cuda()
    hit = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
    occ = torch.zeros(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    gpu_device.intersect(scene, o.data_ptr(), dd.data_ptr(), n, hit.data_ptr())
    gpu_device.occluded(scene, o.data_ptr(), do.data_ptr(), n, occ.data_ptr())
    h = hit.cpu().numpy()
    ref = g["hit"]
    assert np.array_equal(h[:, 3].view(np.int32), ref[:, 3].view(np.int32))
    m = ref[:, 3].view(np.int32) >= 0
    np.testing.assert_allclose(h[m, :3], ref[m, :3], rtol=1e-5, atol=1e-6)
    assert np.array_equal(occ.cpu().numpy(), g["occ"])
    s.close()


# ----------------------------------------------------------------------------- full renders
# Every render comparison uses the SURVEY §8(d) gate at its stated bound: |g-c| <= 1e-3 +
# 1e-3|c| on >= 99.9 % (C1/C2) / 99.5 % (C3-C5) of channels and mean-abs-diff <= 1e-4 * mean.
def test_c1_pathtracer_parity(gpu_device):
    img, ref, st = _render_pair(gpu_device, c1_args(256, 1))
    parity(img, ref, 0.999)
    assert st["raysClosest"] > 0 and st["samples"] == 256 * 256


def test_c2_pathtracer_parity(gpu_device):
    img, ref, _ = _render_pair(gpu_device, c2_args(256, 16))
    parity(img, ref, 0.999)


def test_c2_full_size_parity(gpu_device):
    """C2 at its BASELINE size: cornell_box_spheres 1024^2 at 16 spp, the whole frame."""
    img, ref, st = _render_pair(gpu_device, c2_args(1024, 16))
    r = parity(img, ref, 0.999)
    assert st["samples"] == 1024 * 1024 * 16
    print("C2 1024^2 16spp", r)


def test_c3_standin_parity(gpu_device):
    img, ref, _ = _render_pair(gpu_device, c3_args(128, 4))
    parity(img, ref, 0.995)


def test_c3_full_size_band_parity(gpu_device):
    """C3 at its BASELINE size (2048^2, 64 spp, depth 10, 64 M-path batches over two lanes):
    the GPU frame against the oracle on a centred band of 64 full rows (same frame blob)."""
    s = _session(gpu_device, c3_args(2048, 64))
    info = s.info()
    img = s.render()
    y0 = 992
    ref, _ = oracle.render(s.export_frame(), 2048, 2048, info["gamma"], rect=(0, y0, 2048, y0 + 64))
    r = parity(img[y0:y0 + 64], ref[y0:y0 + 64], 0.995)
    assert np.isfinite(img).all()
    print("C3 band", r)
    s.close()


@pytest.mark.parametrize("face", [0, 3, 7, 10])
def test_c4_stereo_face_parity(gpu_device, face):
    img, ref, _ = _render_pair(gpu_device, c4_args(96, 4), face=face)
    parity(img, ref, 0.995)


@pytest.mark.parametrize("which", ["C2 200x120", "C4 face 0 72^2", "C4 face 5 72^2"])
def test_partial_tile_sizes_parity(gpu_device, which):
    """Images whose sides are not multiples of the 16-pixel tile (the last tile row/column
    overhangs the image): the batch pixel mapping (multiply-high tile division, overhang lanes
    left out of the queues) and the stereo camera's host-side terms on a non-square tile grid."""
    if which.startswith("C2"):
        img, ref, st = _render_pair(gpu_device, c2_args(200, 4) + ["-size", "200", "120"])
        assert img.shape[:2] == (120, 200) and st["samples"] == 200 * 120 * 4
        parity(img, ref, 0.999)
    else:
        img, ref, _ = _render_pair(gpu_device, c4_args(72, 4), face=int(which.split()[2]))
        parity(img, ref, 0.995)


def _hdri_scene(L=(2.0, 1.5, 1.2)):
    """models/test_stereo.xml with the HDRI radiance its authors left commented out
    (test_stereo.xml:100 `<L>2.0 1.5 1.2</L>`) switched on; texture paths made absolute."""
    from helpers import SCENES
    src = (SCENES / "test_stereo.xml").read_text()
    assert "<L>0.0 0.0 0.0</L>" in src
    txt = src.replace("<L>0.0 0.0 0.0</L>", "<L>%g %g %g</L>" % L)
    for f in ("logo.png", "lines.ppm"):
        txt = txt.replace(f'"{f}"', f'"{SCENES / f}"')
    out = SCENES / "_generated" / "test_stereo_hdri.xml"
    out.parent.mkdir(parents=True, exist_ok=True)
    out.write_text(txt)
    return out


@pytest.mark.parametrize("face", [0, 4, 9])
def test_hdri_light_parity(gpu_device, face):
    """HDRILight with non-zero radiance (lights/hdrilight.cpp:39-112): lat-long Le on misses and
    importance-sampled direct light from the precomputed per-record light samples."""
    from helpers import SCENES
    args = ["-i", str(_hdri_scene()), "-c", str(SCENES / "test_stereo_view.ecs"), "-size", "96", "96",
            "-spp", "4", "-stereo"]
    img, ref, st = _render_pair(gpu_device, args, face=face)
    parity(img, ref, 0.995)
    # the HDRI really contributes: the same face without it is darker
    img0, _, _ = _render_pair(gpu_device, c4_args(96, 4), face=face)
    assert img.mean() > img0.mean() * 1.2, (img.mean(), img0.mean())


def test_white_furnace_gpu(gpu_device):
    """KAT 5 on the device: an open Lambertian plane (albedo 0.5) under a constant dome L = 2 with
    nothing above it: camera rays hitting the plane return L * albedo (one diffuse vertex, the
    dome sample's Lambertian weight is exactly albedo), sky pixels L, and the image equals the
    oracle's."""
    from test_cpu_host import yrt_lookat
    d = gpu_device
    L, albedo = 2.0, 0.5
    mesh = d.rtNewShape("trianglemesh")
    pos = np.array([[-1e3, 0, -1e3], [1e3, 0, -1e3], [1e3, 0, 1e3], [-1e3, 0, 1e3]], np.float32)
    idx = np.array([[0, 2, 1], [0, 3, 2]], np.int32)
    dp, di = d.rtNewData("immutable", pos), d.rtNewData("immutable", idx)
    d.rtSetArray(mesh, "positions", "float3", dp, 4, 12)
    d.rtSetArray(mesh, "indices", "int3", di, 2, 12)
    d.rtCommit(mesh)
    mat = d.rtNewMaterial("Matte")
    d.rtSetFloat3(mat, "reflectance", albedo, albedo, albedo)
    d.rtCommit(mat)
    amb = d.rtNewLight("ambientlight")
    d.rtSetFloat3(amb, "L", L, L, L)
    d.rtCommit(amb)
    scene = d.rtNewScene("default")
    d.rtSetPrimitive(scene, 0, d.rtNewShapePrimitive(mesh, mat))
    d.rtSetPrimitive(scene, 1, d.rtNewLightPrimitive(amb))
    d.rtCommit(scene)
    cam = d.rtNewCamera("pinhole")
    d.rtSetTransform(cam, "local2world", yrt_lookat((0, 10, 0), (0, 10, 1), (0, 1, 0)))
    d.rtSetFloat1(cam, "angle", 60.0)
    d.rtSetFloat1(cam, "aspectRatio", 1.0)
    d.rtCommit(cam)
    r = d.rtNewRenderer("pathtracer")
    d.rtSetInt1(r, "maxDepth", 2)
    d.rtSetInt1(r, "sampler.spp", 4)
    d.rtSetFloat1(r, "tMaxShadowRay", 1e4)
    d.rtCommit(r)
    tm = d.rtNewToneMapper("default")
    d.rtCommit(tm)
    fb = d.rtNewFrameBuffer("RGB_FLOAT32", 64, 64)
    d.rtRenderFrame(r, cam, scene, tm, fb, 0)
    img = d.framebuffer_array(fb, 64, 64, "RGB_FLOAT32")
    ref, _ = oracle.render(d.export_frame(r, cam, scene), 64, 64, 1.0)
    parity(img, ref, 0.999)
    plane = np.isclose(img, L * albedo, rtol=2e-3)
    sky = np.isclose(img, L, rtol=2e-3)
    assert plane.mean() > 0.3 and sky.mean() > 0.3, (plane.mean(), sky.mean())
    assert (img >= L * albedo * (1 - 2e-3)).all() and (img <= L * (1 + 2e-3)).all()


# ----------------------------------------------------------------------------- invariances
def test_tile_shards_compose_bit_exact(gpu_device):
    """tiles round-robin over ranks; the union of shards equals the full frame."""
    args = c2_args(200, 4) + ["-fb", "RGB_FLOAT32"]
    s = yrt.Session(args, device=gpu_device)
    full = s.render()
    parts = []
    try:
        for k in range(3):
            gpu_device.set_tile_shard(k, 3)
            parts.append(s.render())
            # the same shard again: its frame block already holds the zeros outside the shard
            # and is not cleared again (device.cpp FrameBlock::zeroKey)
            assert np.array_equal(s.render(), parts[-1])
        gpu_device.set_tile_shard(0, 1)
        assert np.array_equal(s.render(), full)
        gpu_device.set_tile_shard(1, 3)  # after a whole frame the block is cleared again
        again = s.render()
    finally:
        gpu_device.set_tile_shard(0, 1)
    from yrt.dist import tile_mask
    for k, p in enumerate(parts):
        assert not p[~tile_mask(200, 200, k, 3)].any()
    assert np.array_equal(again, parts[1])
    assert np.array_equal(sum(parts), full)
    s.close()


def test_multi_device_tile_shards_compose_bit_exact(gpu_device):
    """A process of two logical devices (devices=0,0) rendering a process-level shard
    (yrtSetTileShard(k, 3), no communicator): the pixels of the other processes' shards read as
    zeros in every render, including a fresh frame block and one that held a whole frame, so the
    three per-process images sum to the one-device frame (device.cpp shard clear)."""
    from yrt.dist import tile_mask
    args = c2_args(200, 4) + ["-fb", "RGB_FLOAT32"]
    s = yrt.Session(args, device=gpu_device)
    full = s.render()
    s.close()
    multi = yrt.Device(devices=[0, 0])
    try:
        s = yrt.Session(args, device=multi)
        assert np.array_equal(s.render(), full)  # the block now holds a whole frame
        parts = []
        for k in range(3):
            multi.set_tile_shard(k, 3)
            parts.append(s.render())
            assert np.array_equal(s.render(), parts[-1])
        multi.set_tile_shard(0, 1)
        s.close()
    finally:
        multi.close()
    for k, p in enumerate(parts):
        assert not p[~tile_mask(200, 200, k, 3)].any(), k
    assert np.array_equal(sum(parts), full)


def test_batch_capacity_invariance(gpu_device):
    s = _session(gpu_device, c2_args(160, 4))
    a = s.render()
    gpu_device.set_batch_capacity(256 * 4 * 3)  # 3 tiles per wavefront batch (34 batches, both lanes)
    try:
        b = s.render()
    finally:
        gpu_device.set_batch_capacity(64 << 20)
    assert np.array_equal(a, b)
    s.close()


@pytest.mark.parametrize("which", ["C3", "C4"])
def test_fused_primary_invariance(gpu_device, monkeypatch, which):
    """Depth 0 as one kernel (camera rays generated inside the closest-hit trace,
    launch_trace_primary: hits queued, misses resolved there; YRT_PRIMARY=2) against k_raygen +
    the queued trace (0): bit-identical frames and the same query counts; C3's dome and C4's
    zero HDRI both qualify (C3: pinhole camera, C4: stereo)."""
    out = []
    for prim in ("0", "2"):
        monkeypatch.setenv("YRT_PRIMARY", prim)
        gpu_device.set_batch_capacity(256 * 16 * 5)  # several batches on both lanes
        try:
            if which == "C3":
                s = _session(gpu_device, c3_args(96, 4))
                img = [s.render()]
            else:
                s = _session(gpu_device, c4_args(64, 2))
                img = s.render_cube()
            st = gpu_device.render_stats()
        finally:
            gpu_device.set_batch_capacity(64 << 20)
        s.close()
        out.append((img, st["raysClosest"], st["raysShadow"]))
    for o in out[1:]:
        for a, b in zip(out[0][0], o[0]):
            assert np.array_equal(a, b)
        assert out[0][1:] == o[1:]


def test_lanes_invariance(monkeypatch):
    """Batches spread over one to four lanes (streams; three is the default) give bit-identical
    frames; lanes 0 restores the default."""
    imgs = []
    for lanes in ("1", "2", "3", "4"):
        monkeypatch.setenv("YRT_LANES", lanes)
        d = yrt.Device(0)
        d.set_batch_capacity(256 * 4 * 5)
        s = _session(d, c2_args(160, 4))
        imgs.append(s.render())
        if lanes == "1":
            d.set_lanes(0)  # the default again (YRT_LANES = 1 here)
            assert np.array_equal(s.render(), imgs[-1])
        s.close()
        d.close()
    for k in range(1, 4):
        assert np.array_equal(imgs[0], imgs[k]), k


def test_rgb8_framebuffer_quantization(gpu_device):
    """RGB8 output (api/framebuffer.h:194-226): truncating quantization, <= 1 LSB vs oracle."""
    s = yrt.Session(c1_args(128, 1), device=gpu_device)
    img8 = s.render().astype(np.int32)
    info = s.info()
    ref, _ = oracle.render(s.export_frame(), 128, 128, info["gamma"])
    ref8 = np.clip(ref * 255.0, 0, 255).astype(np.int32)
    d = np.abs(img8 - ref8)
    assert (d <= 1).mean() >= 0.99, d.max()  # SURVEY §8(d) 8-bit gate
    assert np.array_equal(img8, ref8)  # and bit-identical (truncation of identical floats)
    s.close()


def test_progressive_accumulate(gpu_device):
    """rtRenderFrame(accumulate=1) averages successive frames (AccuBuffer, integratorrenderer.cpp:166)."""
    s = _session(gpu_device, c1_args(64, 1))
    i = s.info()
    cam = s.camera()
    d = gpu_device
    d.rtRenderFrame(i["renderer"], cam, i["scene"], i["tonemapper"], i["framebuffer"], 0)
    a = d.framebuffer_array(i["framebuffer"], 64, 64, "RGB_FLOAT32")
    d.rtRenderFrame(i["renderer"], cam, i["scene"], i["tonemapper"], i["framebuffer"], 1)
    b = d.framebuffer_array(i["framebuffer"], 64, 64, "RGB_FLOAT32")
    assert np.isfinite(b).all() and not np.array_equal(a, b)
    assert abs(float(b.mean()) - float(a.mean())) < 0.25 * float(a.mean()) + 1e-3
    s.close()


def test_pick(gpu_device):
    """rtPick (singleray_device.cpp:692-708): the centre of the Cornell view hits the tall
    block's front face, at the oracle's closest hit on the same ray; the top edge of the
    image plane sees the ceiling."""
    s = _session(gpu_device, c1_args(64, 1))
    i = s.info()
    cam = s.camera()
    hit, p = gpu_device.rtPick(cam, 0.5, 0.5, i["scene"])
    assert hit
    blob = s.export_frame()
    # the pinhole ray through (0.5, 0.5): origin (278, 273, -800), towards +z
    org = np.array([[278.0, 273.0, -800.0, 0.0]], np.float32)
    d = np.array(p, np.float64) - org[0, :3]
    dir4 = np.array([[*(d / np.linalg.norm(d)), np.inf]], np.float32)
    ref = oracle.trace(blob, org, dir4)
    q = org[0, :3] + ref[0, 0] * dir4[0, :3]
    np.testing.assert_allclose(p, q, rtol=1e-4, atol=1e-2)
    assert 0.0 < p[2] < 559.3
    hit, p = gpu_device.rtPick(cam, 0.5, 0.0, i["scene"])
    assert hit and abs(p[1] - 548.8) < 1.0
    s.close()


# ----------------------------------------------------------------------------- multi-GPU (C++)
@pytest.mark.parametrize("replica", [False, True])
def test_multi_device_shards_bit_exact(gpu_device, monkeypatch, replica):
    """yrtNewDevice("devices=0,0,0"): the frame's tiles dealt over three logical shards (one
    host thread and one set of streams each), packed into slabs and gathered on the first
    (SURVEY §8(e)); identical to the one-device frame, RGB_FLOAT32 and RGB8, progressive too.
    replica: the scene is peer-copied to every shard (the multi-GPU replication path)."""
    if replica:
        monkeypatch.setenv("YRT_FORCE_SCENE_REPLICA", "1")
    multi = yrt.Device(devices=[0, 0, 0])
    assert multi.device_count() == 3
    try:
        for args in (c2_args(200, 4) + ["-fb", "RGB_FLOAT32"], c4_args(96, 2) + ["-fb", "RGB8"]):
            face = 3 if "-stereo" in args else -1
            imgs = []
            for d in (gpu_device, multi):
                s = yrt.Session(args, device=d)
                a = s.render(face)
                i = s.info()
                d.rtRenderFrame(i["renderer"], s.camera(face), i["scene"], i["tonemapper"], i["framebuffer"], 1)
                fmt = "RGB_FLOAT32" if "RGB_FLOAT32" in args else "RGB8"
                b = d.framebuffer_array(i["framebuffer"], i["width"], i["height"], fmt)
                imgs.append((a, b, d.render_stats()["raysClosest"]))
                s.close()
            assert np.array_equal(imgs[0][0], imgs[1][0])
            assert np.array_equal(imgs[0][1], imgs[1][1])
            assert imgs[0][2] == imgs[1][2]
    finally:
        multi.close()


def test_startrt_multi_device_equals_single(tmp_path, monkeypatch):
    """StartRT over YRT_DEVICES=0,0 (two logical shards of the GPU) writes the same strips as
    over one device."""
    from dae_scene import write
    outs = []
    for k, devs in enumerate(("0", "0,0")):
        monkeypatch.setenv("YRT_DEVICES", devs)
        d = tmp_path / f"r{k}"
        f = write(d)
        p = yrt.InitParamsRT()
        p.size, p.spp, p.depth = 32, 2, 3
        assert yrt.StartRT(f, p) and yrt.WaitRT()
        assert yrt.GetLastErrorRT() == 0
        outs.append([(d / f"room_{n}.jpg").read_bytes() for n in ("Kitchen", "Hall")])
    assert outs[0] == outs[1]


def test_debug_pixel_samples_match_oracle(gpu_device):
    """yrtDebugPixelSamples (the parity-debugging capture): the per-sample radiance of one pixel,
    in the pixel's summation order, equals the oracle's per-sample radiance bit for bit; the
    capture disarms, and reading without an armed capture on a fresh device raises."""
    s = yrt.Session(c2_args(64, 16) + ["-fb", "RGB_FLOAT32"], device=gpu_device)
    x, y = 37, 22
    gpu_device.debug_pixel_arm(x, y, 64, 0, 16)
    try:
        s.render()
        g = gpu_device.debug_pixel_samples(16)
    finally:
        gpu_device.debug_pixel_arm(-1, 0, 64)
    o = oracle.debug_pixel(s.export_frame(), 64, 64, x, y)
    assert g.shape == o.shape == (16, 3)
    assert np.array_equal(g, o)
    s.close()
    fresh = yrt.Device(0)
    try:
        with pytest.raises(RuntimeError):
            fresh.debug_pixel_samples(4)
    finally:
        fresh.close()


@pytest.mark.gpu
def test_framebuffer_read_back_at_map(gpu_device):
    """rtRenderFrame leaves the frame in HBM and rtMapFrameBuffer reads it back on first access
    (device.cpp fb_read_back): frames rendered into several framebuffers before any map — the
    frame blocks ping-pong, a third live one is allocated, a re-rendered framebuffer drops its
    older frame — all read back equal to frames mapped right after their render."""
    s = yrt.Session(c4_args(64, 2) + ["-fb", "RGB_FLOAT32"], device=gpu_device)
    i = s.info()
    R, S, T = i["renderer"], i["scene"], i["tonemapper"]
    ref = {f: s.render(f) for f in (0, 5, 9)}
    d = gpu_device
    fa, fb, fc = (d.rtNewFrameBuffer("RGB_FLOAT32", 64, 64) for _ in range(3))
    d.rtRenderFrame(R, s.camera(0), S, T, fa, 0)
    d.rtRenderFrame(R, s.camera(5), S, T, fb, 0)
    d.rtRenderFrame(R, s.camera(9), S, T, fa, 0)
    d.rtRenderFrame(R, s.camera(0), S, T, fc, 0)
    assert np.array_equal(d.framebuffer_array(fa, 64, 64, "RGB_FLOAT32"), ref[9])
    assert np.array_equal(d.framebuffer_array(fb, 64, 64, "RGB_FLOAT32"), ref[5])
    assert np.array_equal(d.framebuffer_array(fc, 64, 64, "RGB_FLOAT32"), ref[0])
    assert np.array_equal(d.framebuffer_array(fa, 64, 64, "RGB_FLOAT32"), ref[9])  # a second map: same pixels
    # eight framebuffers rendered before any map: past three live frame blocks the block about to
    # be reused is read back to its framebuffers' host pixels (GpuCtx::kMaxFrameBlocks)
    fbs = [d.rtNewFrameBuffer("RGB_FLOAT32", 64, 64) for _ in range(8)]
    faces = [0, 5, 9, 0, 5, 9, 0, 5]
    for f, cam in zip(fbs, faces):
        d.rtRenderFrame(R, s.camera(cam), S, T, f, 0)
    for f, cam in zip(fbs, faces):
        assert np.array_equal(d.framebuffer_array(f, 64, 64, "RGB_FLOAT32"), ref[cam])
    s.close()
