"""Stereo cubes as one wavefront job (yrtRenderFrames, SURVEY §8(a) a19 + §8(e)) and the
multi-GPU gathers.

The reference renders the 12 faces of a stereo cube one rtRenderFrame at a time
(devices/renderer/renderer.cpp:543-737 FPR, :742-878 non-FPR). yrtRenderFrames renders them as
one job: the faces' 16x16 tiles form one sequence that fills the batches and is dealt over
shards and GPUs as a whole. Every per-pixel input depends on the face's own pixel only (the
per-tile Random of integratorrenderer.cpp:134 is seeded by tile coordinates), so the faces must
equal the face-by-face loop bit for bit — whatever the batch boundaries, shards or devices.

Full-size parity bands: C4 (1536^2 at 256 spp) and C5 (1536^2 at 1024 spp) faces against the
oracle on bands of the configs' own frames (large-spp sample-record indexing, 2.4 G-path faces
split into 64 M-path batches).
"""
import multiprocessing as mp

import numpy as np
import pytest

import oracle
import yrt
from helpers import c4_args, parity
from yrt import _native as N
from yrt import frederick

FPR = ["-tMaxShadowRay", "120", "-ambientlight", "0.83", "0.95", "0.98", "-depth", "10", "-toeIn"]


def _fpr_args(dae, size, spp, fb="RGB_FLOAT32"):
    return ["-fprCollada", "-faceCullingMode", "default", "-i", str(dae), "-stereo", "-size", str(size), str(size),
            "-spp", str(spp), "-fb", fb] + FPR


def _gpu_count():
    d = yrt.Device(devices="all")
    n = d.device_count()
    d.close()
    return n


# ----------------------------------------------------------------------------- one job = face loop
@pytest.mark.gpu
@pytest.mark.parametrize("capacity", [0, 256 * 4 * 7])
def test_cube_job_equals_face_loop_c4(gpu_device, capacity):
    """C4 (96^2, 4 spp): the 12 faces as one job equal 12 rtRenderFrame calls, bit for bit, and
    trace the same rays. capacity 7 tiles per batch: batches straddle face boundaries (36 tiles
    per face)."""
    s = yrt.Session(c4_args(96, 4) + ["-fb", "RGB_FLOAT32"], device=gpu_device)
    loop, rays = [], 0.0
    for f in range(12):
        loop.append(s.render(f))
        st = gpu_device.render_stats()
        rays += st["raysClosest"] + st["raysShadow"]
    if capacity:
        gpu_device.set_batch_capacity(capacity)
    try:
        cube = s.render_cube()
        st = gpu_device.render_stats()
    finally:
        gpu_device.set_batch_capacity(64 << 20)
    for f in range(12):
        assert np.array_equal(cube[f], loop[f]), f
    assert st["raysClosest"] + st["raysShadow"] == rays
    assert st["samples"] == 12 * 96 * 96 * 4
    s.close()


@pytest.mark.gpu
def test_cube_job_shards_compose(gpu_device):
    """The cube's tile sequence dealt round-robin over 3 shards: the shards' faces are disjoint
    and sum to the whole cube (C4's 110,592 tiles dealt tile_id mod N; logical
    tile l of a face covers image tile yrt_tile_scatter(l, T), common/yrt_tile_scatter.h)."""
    s = yrt.Session(c4_args(80, 2) + ["-fb", "RGB_FLOAT32"], device=gpu_device)
    full = s.render_cube()
    parts = []
    try:
        for k in range(3):
            gpu_device.set_tile_shard(k, 3)
            parts.append(s.render_cube())
    finally:
        gpu_device.set_tile_shard(0, 1)
    tpf = 5 * 5  # 80^2 -> 5 x 5 tiles per face
    logical = {N.dev.yrtDebugTileScatter(l, tpf): l for l in range(tpf)}  # image tile -> logical
    assert sorted(logical) == list(range(tpf))
    for f in range(12):
        assert np.array_equal(sum(p[f] for p in parts), full[f])
        for k in range(3):
            for t in range(tpf):
                ty, tx = divmod(t, 5)
                blk = parts[k][f][16 * ty:16 * ty + 16, 16 * tx:16 * tx + 16]
                mine = (f * tpf + logical[t]) % 3 == k
                assert mine or not blk.any(), (f, t, k)
    s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [8, 4])
def test_batch_grow_invariance(gpu_device, monkeypatch, n):
    """A rank's share of the full-size C4 cube job runs 7 (N = 8) or 14 (N = 4) batches per lane
    at the default capacity, so Device::render_shard grows them to 2x / 1.5x the size; the faces
    are bit-identical to the share rendered without growing (YRT_BATCH_GROW=0)."""
    s = yrt.Session(c4_args() + ["-fb", "RGB8"], device=gpu_device)
    faces = []
    try:
        gpu_device.set_tile_shard(n - 1, n)
        for grow in ("0", "1"):
            monkeypatch.setenv("YRT_BATCH_GROW", grow)
            faces.append(s.render_cube())
    finally:
        gpu_device.set_tile_shard(0, 1)
    s.close()
    for a, b in zip(faces[0], faces[1]):
        assert a.any() and np.array_equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("fb", ["RGB_FLOAT32", "RGB8"])
def test_cube_job_multi_device(gpu_device, fb):
    """devices=0,0,0 (three logical shards, slab gather on the first; RGB8 framebuffers move
    4-byte slab words): the cube equals the one-device cube."""
    multi = yrt.Device(devices=[0, 0, 0])
    try:
        cubes = []
        for d in (gpu_device, multi):
            s = yrt.Session(c4_args(96, 2) + ["-fb", fb], device=d)
            cubes.append(s.render_cube())
            s.close()
        for f in range(12):
            assert np.array_equal(cubes[0][f], cubes[1][f]), f
    finally:
        multi.close()


@pytest.mark.gpu
def test_scene_cube_equals_face_loop_c5(gpu_device):
    """C5 FPR views (48^2, 2 spp): one faceCamera update + refit per view and the 12 faces as
    one job equal the reference's per-face loop (update, commit, render per face)."""
    s = yrt.Session(_fpr_args(frederick.write_dae(), 48, 2), device=gpu_device)
    nviews = s.num_scene_cameras() // 12
    assert nviews == len(frederick.CAMERAS)
    for v in range(nviews):
        loop = [s.render_scene_camera(12 * v + f) for f in range(12)]
        cube = s.render_scene_cube(v)
        for f in range(12):
            assert np.array_equal(cube[f], loop[f]), (v, f)
    s.close()


@pytest.mark.gpu
def test_startrt_cube_equals_face_loop(tmp_path, monkeypatch):
    """StartRT on the C5 stand-in writes the same strips with the views rendered as one job each
    as with the reference's face-by-face loop (YRT_FACE_LOOP=1)."""
    outs = []
    for k, loop in enumerate((True, False)):
        if loop:
            monkeypatch.setenv("YRT_FACE_LOOP", "1")
        else:
            monkeypatch.delenv("YRT_FACE_LOOP", raising=False)
        d = tmp_path / f"r{k}"
        dae = frederick.write_dae(d / "frederick.dae")
        p = yrt.InitParamsRT()
        p.size, p.spp, p.depth = 32, 2, 4
        assert yrt.StartRT(dae, p) and yrt.WaitRT()
        assert yrt.GetLastErrorRT() == 0
        outs.append([(d / f"frederick_{v}.jpg").read_bytes() for v in frederick.CAMERAS])
    assert outs[0] == outs[1]


# ----------------------------------------------------------------------------- full-size bands
@pytest.mark.gpu
def test_c4_full_size_face_band_parity(gpu_device):
    """C4 at its BASELINE size and spp (1536^2, 256 spp, 64 sets x 256 sample records): stereo
    face 3 against the oracle on a centred band of 32 full rows of the same frame."""
    s = yrt.Session(c4_args(1536, 256) + ["-fb", "RGB_FLOAT32"], device=gpu_device)
    img = s.render(3)
    y0 = 752
    ref, st = oracle.render(s.export_frame(3), 1536, 1536, s.info()["gamma"], rect=(0, y0, 1536, y0 + 32))
    r = parity(img[y0:y0 + 32], ref[y0:y0 + 32], 0.995)
    print("C4 face 3 band", r, st["raysClosest"] + st["raysShadow"])
    s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cam", [2, 19])
def test_c5_full_size_face_band_parity(gpu_device, cam):
    """C5 at its own size and spp (1536^2, 1024 spp: sample records set * 1024 + s up to 65,535,
    a 2.4 G-path face in 64 M-path batches): one FPR face of each view against the oracle on a
    16-row band of the same frame (faceCamera billboard re-oriented, DLL defaults)."""
    s = yrt.Session(_fpr_args(frederick.write_dae(), 1536, 1024), device=gpu_device)
    img = s.render_scene_camera(cam)
    y0 = 760
    ref, st = oracle.render(s.export_frame(camera=s.scene_camera(cam)), 1536, 1536, s.info()["gamma"],
                            rect=(0, y0, 1536, y0 + 16))
    r = parity(img[y0:y0 + 16], ref[y0:y0 + 16], 0.995)
    print(f"C5 face {cam} band", r, st["raysClosest"] + st["raysShadow"])
    s.close()


# ----------------------------------------------------------------------------- distinct GPUs (RCCL)
@pytest.mark.gpu
def test_multi_gpu_devices_equal_single(gpu_device):
    """devices=0,1 (two distinct GPUs in one process: scene peer-copied, tile slabs gathered by
    RCCL grouped send/recv over xGMI, ncclCommInitAll): frames and cubes equal one GPU's.
    Skipped on a one-GPU box."""
    if _gpu_count() < 2:
        pytest.skip("needs two GPUs")
    multi = yrt.Device(devices=[0, 1])
    try:
        for fb in ("RGB_FLOAT32", "RGB8"):
            res = []
            for d in (gpu_device, multi):
                s = yrt.Session(c4_args(96, 2) + ["-fb", fb], device=d)
                res.append((s.render(3), s.render_cube()))
                s.close()
            assert np.array_equal(res[0][0], res[1][0])
            for f in range(12):
                assert np.array_equal(res[0][1][f], res[1][1][f])
    finally:
        multi.close()


def _comm_rank(rank, world, q_uid, q_out, fail_rank):
    import yrt as y
    from helpers import c4_args as args4
    d = y.Device(rank)
    if rank == 0:
        uid = y.Device.shard_comm_unique_id()
        for _ in range(world - 1):
            q_uid.put(uid)
    else:
        uid = q_uid.get(timeout=60)
    d.set_shard_comm(rank, world, uid)
    s = y.Session(args4(96, 2) + ["-fb", "RGB8"], device=d)
    out = {"rank": rank}
    try:
        out["cube"] = s.render_cube()
        out["face"] = s.render(5)
    except RuntimeError as e:
        out["err"] = str(e)
    if fail_rank is not None:
        i = s.info()
        sc = d.rtNewScene() if rank == fail_rank else i["scene"]  # uncommitted scene: this rank fails
        try:
            d.rtRenderFrame(i["renderer"], s.camera(0), sc, i["tonemapper"], i["framebuffer"], 0)
            out["fail_err"] = None
        except RuntimeError as e:
            out["fail_err"] = str(e)
    s.close()
    d.set_shard_comm(0, 1, uid)
    d.close()
    q_out.put(out)


@pytest.mark.gpu
def test_process_rccl_gather_equals_single(gpu_device):
    """One process per GPU (yrtSetShardComm over RCCL, bench.py's N-GPU path): rank 0's gathered
    cube and frame equal one GPU's; a rank whose render fails makes every rank's call fail
    (status exchange before the gather) instead of hanging rank 0. Skipped on a one-GPU box."""
    if _gpu_count() < 2:
        pytest.skip("needs two GPUs")
    s = yrt.Session(c4_args(96, 2) + ["-fb", "RGB8"], device=gpu_device)
    ref_cube, ref_face = s.render_cube(), s.render(5)
    s.close()
    ctx = mp.get_context("spawn")
    q_uid, q_out = ctx.Queue(), ctx.Queue()
    procs = [ctx.Process(target=_comm_rank, args=(r, 2, q_uid, q_out, 1)) for r in range(2)]
    for p in procs:
        p.start()
    outs = {}
    for _ in procs:
        o = q_out.get(timeout=240)
        outs[o["rank"]] = o
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert "err" not in outs[0] and "err" not in outs[1], outs
    for f in range(12):
        assert np.array_equal(outs[0]["cube"][f], ref_cube[f]), f
    assert np.array_equal(outs[0]["face"], ref_face)
    assert "not committed" in outs[1]["fail_err"]
    assert "peer rank" in outs[0]["fail_err"]


# ----------------------------------------------------------------------------- bench.py N>1 path
@pytest.mark.gpu
def test_bench_two_ranks_cubemap_gather_check(tmp_path):
    """bench.py at N=2 as the driver launches it (torch.distributed.run, one process per rank),
    rehearsed with two gloo ranks on this GPU: the line carries the strong-scaling cubemap
    (default at N>1) and its gather check against rank 0's one-GPU render is bit-exact. RCCL
    refuses two ranks on one GPU, so the rehearsal gathers with torch's reduce (the line says
    which); the C++ RCCL gather itself is test_process_rccl_gather_equals_single on >= 2 GPUs."""
    import json
    import os
    import socket
    import subprocess
    import sys
    from helpers import ROOT
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, YRT_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1",
           "--warmup", "0", "--size", "256", "--spp", "4", "--capture", "0", "--no-cpu-baseline",
           "--stereo-size", "128", "--stereo-spp", "4"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["ranks"] == 2 and line["n_gpus"] == 1  # two ranks, one physical GPU
    sc = line["stereo_cubemap"]
    assert sc is not None and sc["scaling"] == "strong" and sc["value"] > 0
    assert sc["ranks"] == 2 and sc["n_gpus"] == 1
    assert sc["gather_check"] == "bit_exact", sc
    assert sc["single_gpu_ms_per_cubemap"] > 0
    # several cubemaps by default at N > 1, reported as median and min per cubemap
    assert sc["frames"] == 6 and 0 < sc["ms_per_cubemap_min"] <= sc["ms_per_cubemap_median"]
    assert "note" in line["roofline"]["kernel_ms_per_step"]
