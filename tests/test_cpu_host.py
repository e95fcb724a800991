"""CPU suite: oracle against golden vectors, host logic of the device plugin (loaders, BVH,
sampler, decoders, frame export) and the C-ABI surface. No GPU calls."""
import ctypes
import json
import re

import numpy as np
import pytest

import oracle
import yrt
from helpers import ROOT, SCENES, c1_args, c2_args, c3_args, c4_args

GOLDEN = ROOT / "tests" / "golden"


# ----------------------------------------------------------------------------- Random (KAT 1)
def _random_ref(seed, n):
    """Independent restatement of embree::Random (common/math/random.h:31-65): Park-Miller
    minimal standard with a 32-entry Bays-Durham shuffle, 32-bit signed arithmetic."""
    a, m, q, r = 16807, 2147483647, 127773, 2836
    s = 1 if seed == 0 else (-seed if seed < 0 else seed)
    table = [0] * 32
    for j in range(39, -1, -1):
        k = int(s / q)
        s = a * (s - k * q) - r * k
        if s < 0:
            s += m
        if j < 32:
            table[j] = s
    state = table[0]
    out = []
    for _ in range(n):
        k = int(s / q)
        s = a * (s - k * q) - r * k
        if s < 0:
            s += m
        j = state // (1 + (2147483647 - 1) // 32)
        state = table[j]
        table[j] = s
        out.append(state)
    return out


@pytest.mark.parametrize("seed", [0, 1, 27, 3433, 81551, 91711, 91711 * 5 + 81551 * 3])
def test_random_matches_restatement(seed):
    assert oracle.random_ints(seed, 200).tolist() == _random_ref(seed, 200)


def test_random_golden():
    g = json.loads((GOLDEN / "random_ints.json").read_text())
    for seed, vals in g.items():
        assert oracle.random_ints(int(seed), len(vals)).tolist() == vals


# ----------------------------------------------------------------------------- sampler (KAT 2)
@pytest.mark.parametrize("spp,depth", [(1, 2), (16, 2), (64, 10), (3, 4)])
def test_sample_table_host_equals_oracle(spp, depth):
    """Product host sampler (csrc/device/sampler.cpp) vs oracle restatement: bit-exact."""
    a = yrt.sample_table(spp, 64, 0, depth, depth + 1)
    b = oracle.sample_table(spp, 64, 0, depth, depth + 1)
    assert a.shape == b.shape
    assert np.array_equal(a, b)


@pytest.mark.parametrize("spp,depth", [(1, 2), (16, 2), (64, 10)])
def test_sample_table_golden(spp, depth):
    g = np.load(GOLDEN / f"sample_table_spp{spp}_d{depth}.npy")
    b = oracle.sample_table(spp, 64, 0, depth, depth + 1)
    assert np.array_equal(g, b)


def test_sample_table_spp_rounds_up_to_pow2():
    """Quirk Q5 (samplers/sampler.cpp:91): spp is rounded up to a power of two."""
    assert yrt.sample_table(3, 64, 0, 1, 2).shape[1] == 4 * 64
    assert yrt.sample_table(33, 8, 0, 1, 2).shape[1] == 64 * 8


def test_pixel_sets_golden():
    g = np.load(GOLDEN / "pixel_sets_100x70.npy")
    assert np.array_equal(oracle.pixel_sets(100, 70, 64), g)


# ----------------------------------------------------------------------------- decoders
@pytest.mark.parametrize("name", sorted(p.name for p in (SCENES / "Sponza").glob("*.JPG")) + ["../logo.png"])
def test_image_decoders_match_pil(name):
    """Baseline JPEG (islow IDCT, fancy upsampling) and PNG decoders vs libjpeg-turbo/zlib via PIL."""
    PIL = pytest.importorskip("PIL.Image")
    f = SCENES / "Sponza" / name
    a = yrt.decode_image(f)
    b = np.asarray(PIL.open(f))
    if b.ndim == 2:
        b = b[..., None]
    assert a.shape == b.shape and np.array_equal(a, b)


# ----------------------------------------------------------------------------- loaders + commit
@pytest.mark.parametrize("args,tris,lights", [
    (c1_args(32), 36, 2),           # 34 OBJ triangles + quad light (2 triangle lights)
    (c2_args(32, 1), 2 * 4900 + 10 + 2, 2),
    (c4_args(32, 1, stereo=False), 3 * 4900 + 2 + 2, 2),
])
def test_scene_load_counts(host_device, args, tris, lights):
    s = yrt.Session(args, device=host_device)
    info = host_device.scene_info(s.info()["scene"])
    assert info["numTriangles"] == tris
    assert info["numLights"] == lights
    s.close()


def test_standin_is_deterministic_and_sized():
    from yrt import standin
    a = [m.arrays() for m in standin.build_meshes()]
    b = [m.arrays() for m in standin.build_meshes()]
    for x, y in zip(a, b):
        for u, v in zip(x, y):
            assert (u is None and v is None) or np.array_equal(u, v)
    n = sum(x[3].shape[0] for x in a)
    assert 60000 <= n <= 70000


def _incoherent(blob, n, seed=42):
    tris = oracle.scene_triangles(blob).reshape(-1, 3, 3)
    lo, hi = tris.min(axis=(0, 1)), tris.max(axis=(0, 1))
    rng = np.random.default_rng(seed)
    org = rng.uniform(lo, hi, size=(n, 3))
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    org4 = np.concatenate([org, np.zeros((n, 1))], 1).astype(np.float32)
    dir4 = np.concatenate([d, np.full((n, 1), np.inf)], 1).astype(np.float32)
    return org4, dir4


@pytest.mark.parametrize("sbvh", [0, 1], ids=["sah", "sbvh"])
@pytest.mark.parametrize("which", ["C1", "C2", "C3", "C4"])
def test_device_bvh_gives_oracle_hits(host_device, which, sbvh, monkeypatch):
    """The product's SAH BVH (csrc/device/bvh_build.cpp; sbvh: with spatial splits, triangles
    referenced from several leaves with clipped boxes), traversed in the device kernel's
    order by the oracle, returns the same closest hits as the oracle's own BVH: the
    (t, triangle id) tie-break makes the hit independent of the tree."""
    monkeypatch.setenv("YRT_SBVH", str(sbvh))
    args = {"C1": c1_args(32), "C2": c2_args(32, 1), "C3": c3_args(32, 1),
            "C4": c4_args(32, 1, stereo=False)}[which]
    s = yrt.Session(args, device=host_device)
    if sbvh:
        info = host_device.scene_info(s.info()["scene"])
        assert info["numTriRefs"] >= info["numTriangles"]
    scene = s.info()["scene"]
    blob = s.export_frame()
    nodes, tris = host_device.export_bvh(scene)
    org4, dir4 = _incoherent(blob, 4096)
    ref = oracle.trace(blob, org4, dir4)
    nv, tv, hit = oracle.count_visits(nodes, tris, org4, dir4,
                                      tri_bytes=host_device.scene_info(scene)["triRecordBytes"])
    assert np.array_equal(hit[:, 3].view(np.int32), ref[:, 3].view(np.int32))
    m = ref[:, 3].view(np.int32) >= 0
    assert np.array_equal(hit[m, :3], ref[m, :3])
    assert nv > 0 and tv > 0
    s.close()


def _qnode_planes(q):
    """Dequantized planes of exported quantized nodes, exactly (float64): origin + q * 2^e."""
    rec = q.reshape(-1, 64)
    origin = rec[:, 0:12].copy().view(np.float32).astype(np.float64)          # (n, 3)
    exps = rec[:, 12:16].copy().view(np.uint32)[:, 0]
    child = rec[:, 16:32].copy().view(np.int32)                                # (n, 4)
    words = rec[:, 32:56].copy().view(np.uint32)                               # (n, 6)
    scale = np.stack([2.0 ** (((exps >> (8 * a)) & 0xFF).astype(np.int64) - 127) for a in range(3)], 1)
    byte = (words[:, :, None] >> (8 * np.arange(4))[None, None, :]) & 0xFF      # (n, 6, 4)
    lo = origin[:, :, None] + byte[:, 0::2, :] * scale[:, :, None]              # (n, 3, 4)
    hi = origin[:, :, None] + byte[:, 1::2, :] * scale[:, :, None]
    return lo, hi, scale, child


@pytest.mark.parametrize("which", ["C2", "C3", "C4", "C5"])
def test_quantized_nodes_contain_the_float_boxes(host_device, which):
    """The any-hit kernel's 64-B nodes (common/yrt_qnode.h): node for node the same children,
    and every dequantized child box contains the float node's child box widened by one quantum
    on every side (the slack that keeps the kernel's box test conservative)."""
    if which == "C5":
        from yrt import frederick
        dae = frederick.write_dae()
        s = yrt.Session(["-fprCollada", "-i", str(dae), "-stereo", "-size", "32", "32", "-spp", "1"],
                        device=host_device)
    else:
        s = yrt.Session({"C2": c2_args(32, 1), "C3": c3_args(32, 1), "C4": c4_args(32, 1)}[which], device=host_device)
    scene = s.info()["scene"]
    nodes, _ = host_device.export_bvh(scene)
    q = host_device.export_qbvh(scene)
    nd = nodes.reshape(-1, 128)
    planes = nd[:, :96].copy().view(np.float32).reshape(-1, 6, 4).astype(np.float64)  # lox hix loy hiy loz hiz
    fchild = nd[:, 96:112].copy().view(np.int32)
    lo, hi, scale, qchild = _qnode_planes(q)
    assert np.array_equal(fchild, qchild)
    valid = fchild != -1
    for a in range(3):
        s_ = scale[:, a][:, None]
        assert np.all((lo[:, a, :] <= planes[:, 2 * a, :] - s_) | ~valid)
        assert np.all((hi[:, a, :] >= planes[:, 2 * a + 1, :] + s_) | ~valid)
    # the quantum is a small fraction of the node: at most 1/250 of its extent, or 2 float ulps
    v3 = valid[:, None, :]
    L = np.where(v3, planes[:, 0::2, :], np.inf).min(2)
    H = np.where(v3, planes[:, 1::2, :], -np.inf).max(2)
    ok = valid.any(1)
    E = (H - L)[ok]
    m = np.maximum(np.abs(L), np.abs(H))[ok]
    assert np.all(scale[ok] <= np.maximum(E / 125.0, 2.0 ** -100) + 4 * m * 2.0 ** -23)
    s.close()


@pytest.mark.parametrize("which", ["C2", "C3"])
def test_quantized_nodes_give_the_same_hits(host_device, which):
    """Closest hits and occlusion of 4096 incoherent rays through the quantized nodes, in the
    kernel's traversal order, equal the float nodes' (and so the oracle's own BVH's)."""
    s = yrt.Session({"C2": c2_args(32, 1), "C3": c3_args(32, 1)}[which], device=host_device)
    scene = s.info()["scene"]
    blob = s.export_frame()
    nodes, tris = host_device.export_bvh(scene)
    q = host_device.export_qbvh(scene)
    tb = host_device.scene_info(scene)["triRecordBytes"]
    org4, dir4 = _incoherent(blob, 4096)
    for any_hit in (False, True):
        d = dir4.copy()
        if any_hit:
            d[::2, 3] = 50.0
        nv, tv, h = oracle.count_visits(nodes, tris, org4, d, any_hit=any_hit, tri_bytes=tb)
        nq, tq, hq = oracle.count_visits(nodes, tris, org4, d, any_hit=any_hit, tri_bytes=tb, qnodes=q)
        if any_hit:
            assert np.array_equal(h[:, 3].view(np.int32) >= 0, hq[:, 3].view(np.int32) >= 0)
        else:
            assert np.array_equal(h.view(np.uint32), hq.view(np.uint32))
        assert nv <= nq < 1.5 * nv, (nv, nq)
    s.close()


def test_bvh_depth_within_stack(host_device):
    s = yrt.Session(c3_args(32, 1), device=host_device)
    info = host_device.scene_info(s.info()["scene"])
    assert info["bvhDepth"] <= 63  # YRT_STACK_DEPTH - 1
    s.close()


def test_export_frame_deterministic(host_device):
    s1 = yrt.Session(c2_args(32, 1), device=host_device)
    s2 = yrt.Session(c2_args(32, 1), device=host_device)
    assert s1.export_frame() == s2.export_frame()
    s1.close()
    s2.close()


# ----------------------------------------------------------------------------- oracle goldens
@pytest.mark.parametrize("name,args", [
    ("c1_64", c1_args(64, 1)), ("c2_64", c2_args(64, 4)), ("c4_face3_64", c4_args(64, 4)),
])
def test_oracle_thumbnails_golden(host_device, name, args):
    """Oracle 64x64 thumbnails (KAT 6) stay bit-identical to the committed fixtures."""
    g = np.load(GOLDEN / f"thumb_{name}.npy")
    face = 3 if "face3" in name else -1
    s = yrt.Session(args + ["-fb", "RGB_FLOAT32"], device=host_device)
    img, _ = oracle.render(s.export_frame(face), 64, 64, s.info()["gamma"])
    assert np.array_equal(img, g)
    s.close()


@pytest.mark.parametrize("name", ["c2", "c3"])
def test_oracle_hit_records_golden(host_device, name):
    """KAT 4: the oracle's closest hits (t, u, v, triangle id) and occlusion flags for 4096
    incoherent rays stay bit-identical to the committed records (tests/golden/make_golden.py)."""
    g = np.load(GOLDEN / f"hits_{name}_4096.npz")
    args = {"c2": c2_args(32, 1), "c3": c3_args(32, 1)}[name]
    s = yrt.Session(args, device=host_device)
    blob = s.export_frame()
    assert np.array_equal(oracle.trace(blob, g["org"], g["dir"]).view(np.uint32), g["hit"].view(np.uint32))
    assert np.array_equal(oracle.trace(blob, g["org"], g["occ_dir"], any_hit=True)[:, 3].view(np.int32), g["occ"])
    assert (g["hit"][:, 3].view(np.int32) >= 0).mean() > 0.5 and 0 < g["occ"].mean() < 1
    s.close()


def test_oracle_debug_renderer_golden(host_device):
    g = np.load(GOLDEN / "debug_c2_64.npy")
    s = yrt.Session(c2_args(64, 1) + ["-renderer", "debug", "-fb", "RGB_FLOAT32"], device=host_device)
    img, _ = oracle.render(s.export_frame(), 64, 64, 1.0)
    assert np.array_equal(img, g)
    s.close()


def test_white_furnace(host_device):
    """KAT 5: an open Lambertian plane under a constant dome with nothing above it: every
    primary hit returns the dome radiance times the albedo (one diffuse vertex)."""
    d = host_device
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
    blob = d.export_frame(r, cam, scene)
    img, _ = oracle.render(blob, 32, 32, 1.0)
    # every pixel sees either the dome (L) or the plane (L * albedo); filter-blended horizon
    # pixels lie in between
    plane = np.isclose(img, L * albedo, rtol=2e-3)
    sky = np.isclose(img, L, rtol=2e-3)
    assert plane.mean() > 0.3 and sky.mean() > 0.3, (plane.mean(), sky.mean())
    assert (img >= L * albedo * (1 - 2e-3)).all() and (img <= L * (1 + 2e-3)).all()


def yrt_lookat(eye, point, up):
    """lookAtPoint (common/math/affinespace.h:72-77) as the 12-float rtSetTransform layout."""
    eye, point, up = (np.asarray(v, np.float64) for v in (eye, point, up))
    z = point - eye
    z /= np.linalg.norm(z)
    u = np.cross(up, z)
    u /= np.linalg.norm(u)
    v = np.cross(z, u)
    v /= np.linalg.norm(v)
    return np.concatenate([u, v, z, eye]).astype(np.float32)


# ----------------------------------------------------------------------------- C-ABI surface
def _declared(header):
    txt = (ROOT / "include" / header).read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    txt = "\n".join(l for l in txt.splitlines() if not l.lstrip().startswith("#"))
    names = re.findall(r"(?:YRT_API|YULIO_DLL_EXPORT)[^;(]*?\b(\w+)\s*\(", txt)
    return sorted(set(names))


@pytest.mark.parametrize("header,lib", [("yrt_device.h", "dev"), ("yrt_frontend.h", "fe"), ("YulioRT.h", "fe")])
def test_every_declared_symbol_is_exported(header, lib):
    from yrt import _native
    so = getattr(_native, lib)
    names = _declared(header)
    assert len(names) >= 5
    missing = [n for n in names if not hasattr(so, n)]
    assert not missing, missing


def test_host_device_refuses_rendering(host_device):
    s = yrt.Session(c1_args(16), device=host_device)
    with pytest.raises(RuntimeError, match="host-only"):
        s.render()
    s.close()


def test_out_of_scope_types_fail_loudly(host_device):
    with pytest.raises(RuntimeError, match="scope"):
        host_device.rtNewShape("cylinder")
    with pytest.raises(RuntimeError, match="unknown camera type"):
        host_device.rtNewCamera("orthographic")


def test_params_rt_defaults():
    """InitParamsRT fills the YulioRT.h:37-50 defaults."""
    p = yrt.InitParamsRT()
    assert p.renderer == b"pathtracer" and p.size == 1536 and p.depth == 10 and p.spp == 256
    assert abs(p.tMaxShadowRay - 120.0) < 1e-6 and p.toeIn and not p.waterMark
    assert list(p.ambientlight) == pytest.approx([0.83, 0.95, 0.98])
    assert p.faceCullingMode == b"default"


def test_start_rt_rejects_missing_and_collada(tmp_path):
    assert not yrt.StartRT(tmp_path / "x.txt")
    assert yrt.GetLastErrorRT() == 2  # MissingColladaFile


# ----------------------------------------------------------------------------- remaining Device API
def _quad_scene(d, face_camera):
    mesh = d.rtNewShape("trianglemesh")
    # authored lying in the XZ plane: the update's -90 degree turn about `right` stands it up
    pos = np.array([[-1, 0, 0], [1, 0, 0], [1, 0, 2], [-1, 0, 2]], np.float32)
    idx = np.array([[0, 1, 2], [2, 3, 0]], np.int32)
    d.rtSetArray(mesh, "positions", "float3", d.rtNewData("immutable", pos), 4, 12)
    d.rtSetArray(mesh, "indices", "int3", d.rtNewData("immutable", idx), 2, 12)
    d.rtCommit(mesh)
    mat = d.rtNewMaterial("Matte")
    d.rtCommit(mat)
    xf = np.array([2, 0, 0, 0, 2, 0, 0, 0, 2, 5, 0, 5], np.float32)  # scale 2, at (5, 0, 5)
    prim = d.rtNewShapePrimitive(mesh, mat, xf, face_camera)
    scene = d.rtNewScene("default")
    d.rtSetPrimitive(scene, 0, prim)
    d.rtCommit(scene)
    return scene, prim


def _tris(d, scene):
    cam = d.rtNewCamera("pinhole")
    d.rtCommit(cam)
    r = d.rtNewRenderer("pathtracer")
    d.rtCommit(r)
    return oracle.scene_triangles(d.export_frame(r, cam, scene)).reshape(-1, 3, 3)


def test_update_primitive_faces_camera(host_device):
    """rtUpdatePrimitive (singleray_device.cpp:354-398): the faceCamera quad turns to face the
    floor-projected camera direction, keeping its position and scale."""
    d = host_device
    scene, prim = _quad_scene(d, True)
    cam_pos = (5.0, 3.0, 20.0)
    d.rtUpdatePrimitive(scene, 0, prim, cam_pos, (0.0, 1.0, 0.0))
    d.rtCommit(scene)
    t = _tris(d, scene)
    n = np.cross(t[0, 1] - t[0, 0], t[0, 2] - t[0, 0])
    n /= np.linalg.norm(n)
    to_eye = np.array([0.0, 0.0, 1.0])  # (cam - prim) projected on the floor
    assert abs(abs(np.dot(n, to_eye)) - 1.0) < 1e-5
    c = t.reshape(-1, 3).mean(0)
    assert np.allclose(c[[0, 2]], [5.0, 5.0], atol=1e-4)
    ext = t.reshape(-1, 3).max(0) - t.reshape(-1, 3).min(0)
    assert np.isclose(max(ext), 4.0, atol=1e-4)  # 2 (mesh) x 2 (scale)


def test_update_primitive_ignores_static(host_device):
    d = host_device
    scene, prim = _quad_scene(d, False)
    before = _tris(d, scene)
    d.rtUpdatePrimitive(scene, 0, prim, (0.0, 0.0, 50.0), (0.0, 1.0, 0.0))
    d.rtCommit(scene)
    assert np.array_equal(before, _tris(d, scene))


def test_transform_primitive_composes(host_device):
    """rtTransformPrimitive: new transform = given * primitive's (api/instance.h:47-51)."""
    d = host_device
    scene, prim = _quad_scene(d, False)
    moved = d.rtTransformPrimitive(prim, np.array([1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 10, 0], np.float32))
    s2 = d.rtNewScene("default")
    d.rtSetPrimitive(s2, 0, moved)
    d.rtCommit(s2)
    a, b = _tris(d, scene), _tris(d, s2)
    assert np.allclose(b - a, np.array([0, 10, 0], np.float32))


def test_getters_and_data_from_file(host_device, tmp_path):
    d = host_device
    cam = d.rtNewCamera("pinhole")
    d.rtSetFloat1(cam, "sceneScale", 2.5)
    d.rtSetString(cam, "name", "cam_front")
    xf = np.arange(12, dtype=np.float32)
    d.rtSetTransform(cam, "local2world", xf)
    assert d.rtGetFloat1(cam, "sceneScale") == 2.5
    assert d.rtGetFloat1(cam, "unset") == 0.0
    assert d.rtGetString(cam, "name") == "cam_front"
    assert np.array_equal(d.rtGetTransform(cam, "local2world"), xf)
    assert np.array_equal(d.rtGetTransform(cam, "nothing"), [1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0])
    d.rtSetBool2(cam, "b2", 1, 0)
    d.rtSetBool4(cam, "b4", 1, 0, 1, 0)
    f = tmp_path / "blob.bin"
    f.write_bytes(bytes(range(64)))
    assert d.rtNewDataFromFile("immutable", f, 8, 16)
    with pytest.raises(RuntimeError):
        d.rtNewDataFromFile("immutable", f, 60, 16)
