"""Python host binding of the MI355X device plugin.

``Device`` mirrors embree::Device (devices/device/device.h:51-330): the same rt* method names,
argument meaning and error behaviour (a failing call raises ``RuntimeError`` with the
device's message, as the reference throws std::runtime_error). Every call goes through the
C ABI of ``lib/libdevice_singleray_mi355x.so``; there is no Python or CPU compute path.

``Session`` wraps the command-line front end (devices/renderer/renderer.cpp:240-1474) and
``StartRT``/``WaitRT``/... the DLL API (YulioRT.h).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native as N
from ._native import ParamsRT, RenderStats, SceneInfo, SessionInfo, StatusRT  # noqa: F401

__all__ = ["Device", "Session", "ParamsRT", "StatusRT", "RenderStats", "SceneInfo", "sample_table",
           "StartRT", "WaitRT", "StopRT", "GetLastErrorRT", "GetCurrentStatusRT", "InitParamsRT"]


def _b(s):
    return s.encode() if isinstance(s, str) else s


def _xfm(t):
    if t is None:
        t = (1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0)
    a = (C.c_float * 12)(*[float(x) for x in np.asarray(t, dtype=np.float32).reshape(-1)])
    return a


class Device:
    """One MI355X (HIP device ``device``); several (``devices=[0, 1, ...]`` or ``"all"``: the
    frame's tiles dealt over them, gathered on the first; an id may repeat for logical shards
    of one GPU); or, with ``host=True``, a host-only device that loads, commits and exports
    scenes but cannot render (used by the CPU test suite)."""

    def __init__(self, device: int = 0, host: bool = False, handle=None, devices=None):
        self._owned = handle is None
        if handle is not None:
            self.h = handle
        else:
            if host:
                parms = "host"
            elif devices is not None:
                parms = "devices=" + (devices if isinstance(devices, str) else ",".join(str(int(d)) for d in devices))
            else:
                parms = f"device={device}"
            self.h = N.dev.yrtNewDevice(_b(parms), 0, 0, b"")
            if not self.h:
                raise RuntimeError(f"yrtNewDevice({parms!r}) failed (no HIP device?)")
        self._keep = []  # ctypes objects that must outlive the device (callbacks)

    def close(self):
        if self.h and self._owned:
            N.dev.yrtDeleteDevice(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- error convention
    def error(self) -> str:
        e = N.dev.yrtGetLastError(self.h)
        return e.decode() if e else ""

    def _h(self, h, what):
        if not h:
            raise RuntimeError(f"{what}: {self.error()}")
        return h

    def _rc(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what}: {self.error()}")

    # -- object creation (device.h:126-214)
    def rtNewCamera(self, type="pinhole"):
        return self._h(N.dev.yrtNewCamera(self.h, _b(type)), "rtNewCamera")

    def rtNewData(self, type, data):
        buf = np.ascontiguousarray(data)
        return self._h(N.dev.yrtNewData(self.h, _b(type), buf.nbytes, buf.ctypes.data), "rtNewData")

    def rtNewImage(self, type, width, height, data):
        buf = np.ascontiguousarray(data)
        return self._h(N.dev.yrtNewImage(self.h, _b(type), width, height, buf.ctypes.data), "rtNewImage")

    def rtNewImageFromFile(self, file):
        return self._h(N.dev.yrtNewImageFromFile(self.h, _b(str(file))), "rtNewImageFromFile")

    def rtNewTexture(self, type="bilinear"):
        return self._h(N.dev.yrtNewTexture(self.h, _b(type)), "rtNewTexture")

    def rtNewMaterial(self, type):
        return self._h(N.dev.yrtNewMaterial(self.h, _b(type)), "rtNewMaterial")

    def rtNewShape(self, type):
        return self._h(N.dev.yrtNewShape(self.h, _b(type)), "rtNewShape")

    def rtNewLight(self, type):
        return self._h(N.dev.yrtNewLight(self.h, _b(type)), "rtNewLight")

    def rtNewShapePrimitive(self, shape, material, transform=None, faceCamera=False):
        return self._h(N.dev.yrtNewShapePrimitive(self.h, shape, material, _xfm(transform), int(faceCamera)),
                       "rtNewShapePrimitive")

    def rtNewLightPrimitive(self, light, material=None, transform=None):
        return self._h(N.dev.yrtNewLightPrimitive(self.h, light, material, _xfm(transform)), "rtNewLightPrimitive")

    def rtNewScene(self, type="default"):
        return self._h(N.dev.yrtNewScene(self.h, _b(type)), "rtNewScene")

    def rtSetPrimitive(self, scene, slot, prim):
        self._rc(N.dev.yrtSetPrimitive(self.h, scene, slot, prim), "rtSetPrimitive")

    def rtNewToneMapper(self, type="default"):
        return self._h(N.dev.yrtNewToneMapper(self.h, _b(type)), "rtNewToneMapper")

    def rtNewRenderer(self, type="pathtracer"):
        return self._h(N.dev.yrtNewRenderer(self.h, _b(type)), "rtNewRenderer")

    def rtNewFrameBuffer(self, type, width, height, buffers=1):
        return self._h(N.dev.yrtNewFrameBuffer(self.h, _b(type), width, height, buffers, None), "rtNewFrameBuffer")

    # -- properties (device.h:237-312)
    def rtIncRef(self, h):
        self._rc(N.dev.yrtIncRef(self.h, h), "rtIncRef")

    def rtDecRef(self, h):
        self._rc(N.dev.yrtDecRef(self.h, h), "rtDecRef")

    def rtSetBool1(self, h, p, x):
        self._rc(N.dev.yrtSetBool1(self.h, h, _b(p), int(bool(x))), "rtSetBool1")

    def rtSetInt1(self, h, p, x):
        self._rc(N.dev.yrtSetInt1(self.h, h, _b(p), int(x)), "rtSetInt1")

    def rtSetInt2(self, h, p, x, y):
        self._rc(N.dev.yrtSetInt2(self.h, h, _b(p), int(x), int(y)), "rtSetInt2")

    def rtSetFloat1(self, h, p, x):
        self._rc(N.dev.yrtSetFloat1(self.h, h, _b(p), float(x)), "rtSetFloat1")

    def rtSetFloat2(self, h, p, x, y):
        self._rc(N.dev.yrtSetFloat2(self.h, h, _b(p), float(x), float(y)), "rtSetFloat2")

    def rtSetFloat3(self, h, p, x, y, z):
        self._rc(N.dev.yrtSetFloat3(self.h, h, _b(p), float(x), float(y), float(z)), "rtSetFloat3")

    def rtSetFloat4(self, h, p, x, y, z, w):
        self._rc(N.dev.yrtSetFloat4(self.h, h, _b(p), float(x), float(y), float(z), float(w)), "rtSetFloat4")

    def rtGetFloat3(self, h, p):
        x, y, z = C.c_float(), C.c_float(), C.c_float()
        self._rc(N.dev.yrtGetFloat3(self.h, h, _b(p), C.byref(x), C.byref(y), C.byref(z)), "rtGetFloat3")
        return x.value, y.value, z.value

    def rtSetBool2(self, h, p, x, y):
        self._rc(N.dev.yrtSetBool2(self.h, h, _b(p), int(bool(x)), int(bool(y))), "rtSetBool2")

    def rtSetBool3(self, h, p, x, y, z):
        self._rc(N.dev.yrtSetBool3(self.h, h, _b(p), int(bool(x)), int(bool(y)), int(bool(z))), "rtSetBool3")

    def rtSetBool4(self, h, p, x, y, z, w):
        self._rc(N.dev.yrtSetBool4(self.h, h, _b(p), *[int(bool(v)) for v in (x, y, z, w)]), "rtSetBool4")

    def rtGetFloat1(self, h, p):
        x = C.c_float()
        self._rc(N.dev.yrtGetFloat1(self.h, h, _b(p), C.byref(x)), "rtGetFloat1")
        return x.value

    def rtGetString(self, h, p):
        n = N.dev.yrtGetString(self.h, h, _b(p), None, 0)
        if n < 0:
            raise RuntimeError(f"rtGetString: {self.error()}")
        buf = C.create_string_buffer(n + 1)
        N.dev.yrtGetString(self.h, h, _b(p), buf, n + 1)
        return buf.value.decode()

    def rtGetTransform(self, h, p):
        out = (C.c_float * 12)()
        self._rc(N.dev.yrtGetTransform(self.h, h, _b(p), out), "rtGetTransform")
        return np.array(out, np.float32)

    def rtNewDataFromFile(self, type, file, offset, bytes_):
        return self._h(N.dev.yrtNewDataFromFile(self.h, _b(type), _b(str(file)), offset, bytes_), "rtNewDataFromFile")

    def rtTransformPrimitive(self, prim, transform):
        return self._h(N.dev.yrtTransformPrimitive(self.h, prim, _xfm(transform)), "rtTransformPrimitive")

    def rtUpdatePrimitive(self, scene, slot, prim, camPos, camUp):
        pos = (C.c_float * 3)(*camPos)
        up = (C.c_float * 3)(*camUp)
        self._rc(N.dev.yrtUpdatePrimitive(self.h, scene, slot, prim, pos, up), "rtUpdatePrimitive")

    def rtPick(self, camera, x, y, scene):
        px, py, pz = C.c_float(), C.c_float(), C.c_float()
        r = N.dev.yrtPick(self.h, camera, float(x), float(y), scene, C.byref(px), C.byref(py), C.byref(pz))
        if r < 0:
            raise RuntimeError(f"rtPick: {self.error()}")
        return bool(r), (px.value, py.value, pz.value)

    def rtSetArray(self, h, p, type, data, size, stride, ofs=0):
        self._rc(N.dev.yrtSetArray(self.h, h, _b(p), _b(type), data, size, stride, ofs), "rtSetArray")

    def rtSetString(self, h, p, s):
        self._rc(N.dev.yrtSetString(self.h, h, _b(p), _b(s)), "rtSetString")

    def rtSetImage(self, h, p, image):
        self._rc(N.dev.yrtSetImage(self.h, h, _b(p), image), "rtSetImage")

    def rtSetTexture(self, h, p, tex):
        self._rc(N.dev.yrtSetTexture(self.h, h, _b(p), tex), "rtSetTexture")

    def rtSetTransform(self, h, p, t):
        self._rc(N.dev.yrtSetTransform(self.h, h, _b(p), _xfm(t)), "rtSetTransform")

    def rtClear(self, h):
        self._rc(N.dev.yrtClear(self.h, h), "rtClear")

    def rtCommit(self, h):
        self._rc(N.dev.yrtCommit(self.h, h), "rtCommit")

    # -- rendering (device.h:223-234)
    def rtRenderFrame(self, renderer, camera, scene, toneMapper, frameBuffer, accumulate=0):
        self._rc(N.dev.yrtRenderFrame(self.h, renderer, camera, scene, toneMapper, frameBuffer, int(accumulate)),
                 "rtRenderFrame")

    def rtRenderFrames(self, renderer, cameras, scene, toneMapper, frameBuffers, accumulate=0):
        """yrtRenderFrames: frame k through cameras[k] into frameBuffers[k], one wavefront job."""
        n = len(cameras)
        if len(frameBuffers) != n:
            raise ValueError("one framebuffer per camera")
        cams = (C.c_void_p * n)(*cameras)
        fbs = (C.c_void_p * n)(*frameBuffers)
        self._rc(N.dev.yrtRenderFrames(self.h, renderer, cams, n, scene, toneMapper, fbs, int(accumulate)),
                 "rtRenderFrames")

    def rtMapFrameBuffer(self, frameBuffer, bufID=-1):
        return self._h(N.dev.yrtMapFrameBuffer(self.h, frameBuffer, bufID), "rtMapFrameBuffer")

    def rtUnmapFrameBuffer(self, frameBuffer, bufID=-1):
        self._rc(N.dev.yrtUnmapFrameBuffer(self.h, frameBuffer, bufID), "rtUnmapFrameBuffer")

    def rtSwapBuffers(self, frameBuffer):
        self._rc(N.dev.yrtSwapBuffers(self.h, frameBuffer), "rtSwapBuffers")

    def rtSetStatusCallback(self, renderer, fn):
        cb = N.STATUS_CB(lambda s, p, u: fn(s, p))
        self._keep.append(cb)
        self._rc(N.dev.yrtSetStatusCallback(self.h, renderer, cb, None), "rtSetStatusCallback")

    # -- framebuffer readback helpers
    def framebuffer_array(self, frameBuffer, width, height, format):
        """Copy of the mapped framebuffer as numpy (H, W, c) in the reference's row order."""
        p = self.rtMapFrameBuffer(frameBuffer)
        if format == "RGB_FLOAT32":
            a = np.ctypeslib.as_array((C.c_float * (width * height * 3)).from_address(p)).reshape(height, width, 3)
        elif format == "RGBA_FLOAT32":
            a = np.ctypeslib.as_array((C.c_float * (width * height * 4)).from_address(p)).reshape(height, width, 4)
        elif format == "RGBA8":
            a = np.ctypeslib.as_array((C.c_uint8 * (width * height * 4)).from_address(p)).reshape(height, width, 4)
        elif format == "RGB8":
            stride = (3 * width + 3) // 4 * 4  # api/framebuffer.h:194-226
            a = np.ctypeslib.as_array((C.c_uint8 * (stride * height)).from_address(p)).reshape(height, stride)
            a = a[:, :3 * width].reshape(height, width, 3)
        else:
            raise ValueError(format)
        a = a.copy()
        self.rtUnmapFrameBuffer(frameBuffer)
        return a

    # -- hot-path ray queries (device pointers: e.g. torch.cuda tensors' data_ptr())
    def intersect(self, scene, org4_ptr, dir4_ptr, n, hit4_ptr, stream=None):
        self._rc(N.dev.yrtIntersect(self.h, scene, org4_ptr, dir4_ptr, n, hit4_ptr, stream), "rtcIntersect")

    def occluded(self, scene, org4_ptr, dir4_ptr, n, occ_ptr, stream=None):
        self._rc(N.dev.yrtOccluded(self.h, scene, org4_ptr, dir4_ptr, n, occ_ptr, stream), "rtcOccluded")

    def triangle_ids(self, scene, tri):
        g, p = C.c_int32(), C.c_int32()
        self._rc(N.dev.yrtTriangleIds(self.h, scene, int(tri), C.byref(g), C.byref(p)), "triangle_ids")
        return g.value, p.value

    # -- stats / control
    def render_stats(self) -> dict:
        s = RenderStats()
        self._rc(N.dev.yrtGetRenderStats(self.h, C.byref(s)), "render_stats")
        return s.as_dict()

    def set_kernel_timing(self, on=True):
        self._rc(N.dev.yrtSetKernelTiming(self.h, int(on)), "set_kernel_timing")

    def set_lanes(self, lanes):
        """Wavefront lanes (overlapping HIP streams), 1..4 (0: the default, 4 or YRT_LANES); with 1
        no two kernels overlap."""
        self._rc(N.dev.yrtSetLanes(self.h, int(lanes)), "set_lanes")

    def scene_info(self, scene) -> dict:
        s = SceneInfo()
        self._rc(N.dev.yrtGetSceneInfo(self.h, scene, C.byref(s)), "scene_info")
        d = {n: getattr(s, n) for n, _ in s._fields_}
        d["bboxLo"], d["bboxHi"] = list(s.bboxLo), list(s.bboxHi)
        return d

    def export_bvh(self, scene):
        """Host mirror of the uploaded BVH: (nodes uint8[numNodes*128],
        tris uint8[numTriRefs*triRecordBytes])."""
        info = self.scene_info(scene)
        nodes = np.zeros(info["numNodes"] * 128, np.uint8)
        tris = np.zeros(info["numTriRefs"] * info["triRecordBytes"], np.uint8)
        self._rc(N.dev.yrtExportBVH(self.h, scene, nodes.ctypes.data, nodes.nbytes, tris.ctypes.data, tris.nbytes),
                 "export_bvh")
        return nodes, tris

    def export_qbvh(self, scene):
        """The any-hit traversal's quantized nodes (uint8[numNodes*64], common/yrt_qnode.h)."""
        info = self.scene_info(scene)
        q = np.zeros(info["numNodes"] * 64, np.uint8)
        self._rc(N.dev.yrtExportQuantizedBVH(self.h, scene, q.ctypes.data, q.nbytes), "export_qbvh")
        return q

    def export_frame(self, renderer, camera, scene) -> bytes:
        n = N.dev.yrtExportFrame(self.h, renderer, camera, scene, None, 0)
        if n < 0:
            raise RuntimeError(f"export_frame: {self.error()}")
        buf = C.create_string_buffer(n)
        m = N.dev.yrtExportFrame(self.h, renderer, camera, scene, buf, n)
        if m != n:
            raise RuntimeError(f"export_frame: {self.error()}")
        return buf.raw

    def set_frame_seed(self, seed):
        self._rc(N.dev.yrtSetFrameSeed(self.h, seed & 0xFFFFFFFF), "set_frame_seed")

    def set_batch_capacity(self, paths):
        self._rc(N.dev.yrtSetBatchCapacity(self.h, int(paths)), "set_batch_capacity")

    def set_ray_capture(self, max_per_depth):
        self._rc(N.dev.yrtSetRayCapture(self.h, int(max_per_depth)), "set_ray_capture")

    def captured_rays(self, shadow, depth):
        """(org4, dir4, total) strided sample of one depth's query stream of the last frame."""
        tot = C.c_double()
        m = N.dev.yrtGetCapturedRays(self.h, int(shadow), depth, None, None, 0, C.byref(tot))
        if m < 0:
            raise RuntimeError(f"captured_rays: {self.error()}")
        org = np.zeros((m, 4), np.float32)
        dir_ = np.zeros((m, 4), np.float32)
        N.dev.yrtGetCapturedRays(self.h, int(shadow), depth, org.ctypes.data, dir_.ctypes.data, m, C.byref(tot))
        return org, dir_, tot.value

    def debug_pixel_arm(self, x, y, width, frame=0, max_samples=1 << 16):
        """Capture the per-sample radiance of pixel (x, y) of frame `frame` in later renders."""
        self._rc(N.dev.yrtDebugPixelSamples(self.h, int(y * width + x) if x >= 0 else -1, int(frame), None,
                                            int(max_samples)), "debug_pixel_arm")

    def debug_pixel_samples(self, spp):
        """The captured per-sample radiance: float32 (spp, 3)."""
        out = np.zeros((spp, 4), np.float32)
        n = N.dev.yrtDebugPixelSamples(self.h, 0, 0, out.ctypes.data, int(spp))
        if n < 0:
            raise RuntimeError(f"debug_pixel_samples: {self.error()}")
        return out[:n, :3]

    def set_refit_commits(self, on=True):
        self._rc(N.dev.yrtSetRefitCommits(self.h, int(on)), "set_refit_commits")

    def scene_refits(self, scene) -> int:
        n = N.dev.yrtGetSceneRefits(self.h, scene)
        if n < 0:
            raise RuntimeError(f"scene_refits: {self.error()}")
        return n

    def set_tile_shard(self, index, count):
        self._rc(N.dev.yrtSetTileShard(self.h, int(index), int(count)), "set_tile_shard")

    def device_count(self) -> int:
        return int(N.dev.yrtGetDeviceCount(self.h))

    @staticmethod
    def rccl_available() -> bool:
        """librccl loads (checked on every rank before the collective communicator init)."""
        return bool(N.dev.yrtRcclAvailable())

    @staticmethod
    def shard_comm_unique_id() -> bytes:
        """128-byte RCCL unique id (rank 0), to broadcast to the other ranks."""
        buf = (C.c_uint8 * 128)()
        if N.dev.yrtShardCommUniqueId(buf) != 0:
            raise RuntimeError("yrtShardCommUniqueId failed (librccl unavailable?)")
        return bytes(buf)

    def set_shard_comm(self, rank, world, uid: bytes):
        """Tiles dealt round-robin over `world` processes; each frame is gathered on rank 0
        inside rtRenderFrame (grouped RCCL send/recv, yrtSetShardComm)."""
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        self._rc(N.dev.yrtSetShardComm(self.h, int(rank), int(world), buf), "set_shard_comm")

    def set_shard_hub(self, hub, rank):
        """Arms rank `rank` of an in-process ShardHub (yrtSetShardHub): tiles dealt round-robin
        over the hub's devices, every frame gathered on rank 0's device inside rtRenderFrame
        (the process gather's bookkeeping with peer / device-to-device copies). hub=None disarms."""
        self._rc(N.dev.yrtSetShardHub(self.h, hub.h if hub is not None else None, int(rank)), "set_shard_hub")

    def set_gather_timeout(self, seconds):
        """Bound of every wait of a multi-GPU gather (yrtSetGatherTimeout)."""
        self._rc(N.dev.yrtSetGatherTimeout(self.h, float(seconds)), "set_gather_timeout")


GATHER_PATHS = {0: "none", 1: "d2d", 2: "rccl-local", 3: "peer-copy", 4: "rccl-process", 5: "hub"}


class ShardHub:
    """The in-process meeting point of a multi-device gather (yrtNewShardHub). status() and
    slab() drive its two phases on host memory (CPU tests of the deadlines and size checks)."""

    def __init__(self, world):
        self.h = N.dev.yrtNewShardHub(int(world))
        if not self.h:
            raise RuntimeError(f"yrtNewShardHub: {N.dev.yrtShardHubLastError().decode()}")
        self.world = int(world)

    def close(self):
        if self.h:
            N.dev.yrtDeleteShardHub(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass

    def status(self, rank, flag, timeout):
        """Min of every rank's flag; raises RuntimeError (naming the missing ranks) on timeout."""
        r = N.dev.yrtShardHubStatus(self.h, int(rank), int(flag), float(timeout))
        if r < 0:
            raise RuntimeError(N.dev.yrtShardHubLastError().decode())
        return r

    def slab(self, rank, data=b"", recv_bytes_per_rank=0, timeout=10.0):
        """rank > 0 sends `data` to rank 0; rank 0 returns the peers' slabs (rank order)."""
        src = np.frombuffer(bytes(data), np.uint8) if len(data) else np.zeros(1, np.uint8)
        out = np.zeros(max(1, (self.world - 1) * recv_bytes_per_rank), np.uint8) if rank == 0 else None
        r = N.dev.yrtShardHubSlab(self.h, int(rank), src.ctypes.data, len(data),
                                  out.ctypes.data if out is not None else None, int(recv_bytes_per_rank),
                                  float(timeout))
        if r < 0:
            raise RuntimeError(N.dev.yrtShardHubLastError().decode())
        return out[:(self.world - 1) * recv_bytes_per_rank] if out is not None else None


def sample_table(spp, sets, iteration, num1D, num2D, filter="bspline"):
    """Host sampler's SoA table (dims x records), see yrtDebugSampleTable."""
    n = N.dev.yrtDebugSampleTable(spp, sets, iteration, num1D, num2D, _b(filter), None, 0)
    if n < 0:
        raise RuntimeError("yrtDebugSampleTable failed")
    dims = 5 + num1D + 2 * num2D
    out = np.zeros(dims * n, np.float32)
    N.dev.yrtDebugSampleTable(spp, sets, iteration, num1D, num2D, _b(filter),
                              out.ctypes.data_as(N.PF), out.size)
    return out.reshape(dims, n)


def decode_image(file):
    """(H, W, C) uint8 pixels decoded by the device's own JPEG/PNG decoder, top row first."""
    w, h, c = C.c_int(), C.c_int(), C.c_int()
    rc = N.dev.yrtDebugDecodeImage(_b(str(file)), C.byref(w), C.byref(h), C.byref(c), None, 0)
    if rc != 0:
        raise RuntimeError(f"decode_image({file}) failed: {rc}")
    out = np.zeros((h.value, w.value, c.value), np.uint8)
    N.dev.yrtDebugDecodeImage(_b(str(file)), C.byref(w), C.byref(h), C.byref(c), out.ctypes.data, out.nbytes)
    return out


class Session:
    """Command-line session (renderer.cpp parseCommandLine/outputMode) over a Device."""

    def __init__(self, args, device: Device | None = None):
        args = [str(a) for a in args]
        argv = (C.c_char_p * len(args))(*[_b(a) for a in args])
        self.device = device
        self.h = N.fe.yrtSessionCreate(device.h if device else None, len(args), argv)
        if not self.h:
            raise RuntimeError(N.fe.yrtFrontendLastError().decode())
        if device is None:
            self.device = Device(handle=self.info()["device"])

    def close(self):
        if self.h:
            N.fe.yrtSessionDestroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def info(self) -> dict:
        s = SessionInfo()
        if N.fe.yrtSessionInfo(self.h, C.byref(s)) != 0:
            raise RuntimeError(N.fe.yrtFrontendLastError().decode())
        return {n: getattr(s, n) for n, _ in s._fields_}

    def camera(self, face=-1):
        h = N.fe.yrtSessionCamera(self.h, face)
        if not h:
            raise RuntimeError(N.fe.yrtFrontendLastError().decode())
        return h

    def render(self, face=-1, read=True):
        """Renders one frame (mono face=-1, stereo cube face 0..11) and returns it as numpy
        (None when read=False: the frame stays in the session's framebuffer)."""
        p = N.fe.yrtSessionRender(self.h, face)
        if not p:
            raise RuntimeError(N.fe.yrtFrontendLastError().decode())
        i = self.info()
        N.dev.yrtUnmapFrameBuffer(self.device.h, i["framebuffer"], -1)
        if not read:
            return None
        fmt = ("RGB8", "RGBA8", "RGB_FLOAT32", "RGBA_FLOAT32")[i["framebufferFormat"]]
        return self.device.framebuffer_array(i["framebuffer"], i["width"], i["height"], fmt)

    def _cube_faces(self):
        i = self.info()
        fmt = ("RGB8", "RGBA8", "RGB_FLOAT32", "RGBA_FLOAT32")[i["framebufferFormat"]]
        out = []
        for f in range(12):
            fb = N.fe.yrtSessionCubeFrameBuffer(self.h, f)
            if not fb:
                raise RuntimeError(N.fe.yrtFrontendLastError().decode())
            out.append(self.device.framebuffer_array(fb, i["width"], i["height"], fmt))
        return out

    def render_cube(self, read=True):
        """The 12 stereo cube faces as one job (yrtSessionRenderCube); list of 12 numpy images
        (None when read=False: the faces stay in the session's framebuffers)."""
        if N.fe.yrtSessionRenderCube(self.h) != 0:
            raise RuntimeError(N.fe.yrtFrontendLastError().decode())
        return self._cube_faces() if read else None

    def render_scene_cube(self, view=0, read=True):
        """The 12 faces of FPR view `view` as one job (yrtSessionRenderSceneCube)."""
        if N.fe.yrtSessionRenderSceneCube(self.h, int(view)) != 0:
            raise RuntimeError(N.fe.yrtFrontendLastError().decode())
        return self._cube_faces() if read else None

    def export_frame(self, face=-1, camera=None) -> bytes:
        i = self.info()
        return self.device.export_frame(i["renderer"], camera if camera else self.camera(face), i["scene"])

    # -- Collada scenes: stereo cube cameras of the FPR views (12 per view)
    def num_scene_cameras(self) -> int:
        return int(N.fe.yrtSessionNumSceneCameras(self.h))

    def scene_camera(self, i):
        h = N.fe.yrtSessionSceneCamera(self.h, i)
        if not h:
            raise RuntimeError(N.fe.yrtFrontendLastError().decode())
        return h

    def render_scene_camera(self, i, read=True):
        """One FPR face (faceCamera update, scene commit, render) of scene camera i (numpy, or
        None when read=False)."""
        p = N.fe.yrtSessionRenderSceneCamera(self.h, i)
        if not p:
            raise RuntimeError(N.fe.yrtFrontendLastError().decode())
        info = self.info()
        N.dev.yrtUnmapFrameBuffer(self.device.h, info["framebuffer"], -1)
        if not read:
            return None
        fmt = ("RGB8", "RGBA8", "RGB_FLOAT32", "RGBA_FLOAT32")[info["framebufferFormat"]]
        return self.device.framebuffer_array(info["framebuffer"], info["width"], info["height"], fmt)

    def output(self, file=None):
        if N.fe.yrtSessionOutput(self.h, _b(file) if file else None) != 0:
            raise RuntimeError(N.fe.yrtFrontendLastError().decode())


def store_image(file, img, quality=90):
    """storeImage: numpy (H, W, 3|4) uint8 or float32 -> .jpg/.png/.ppm/.pfm."""
    a = np.ascontiguousarray(img)
    h, w, c = a.shape
    fmt = {(np.dtype(np.uint8), 3): 0, (np.dtype(np.uint8), 4): 1, (np.dtype(np.float32), 3): 2,
           (np.dtype(np.float32), 4): 3}[(a.dtype, c)]
    if N.fe.yrtStoreImage(_b(str(file)), w, h, fmt, a.ctypes.data, a.strides[0], int(quality)) != 0:
        raise RuntimeError(N.fe.yrtFrontendLastError().decode())


# ---- DLL API (YulioRT.h)
def InitParamsRT() -> ParamsRT:
    p = ParamsRT()
    N.fe.InitParamsRT(C.byref(p))
    return p


def StartRT(file, params: ParamsRT | None = None) -> bool:
    return bool(N.fe.StartRT(_b(str(file)), C.byref(params) if params is not None else None))


def WaitRT() -> bool:
    return bool(N.fe.WaitRT())


def StopRT(keepResults=False) -> bool:
    return bool(N.fe.StopRT(bool(keepResults)))


def GetLastErrorRT() -> int:
    return int(N.fe.GetLastErrorRT())


def GetCurrentStatusRT() -> StatusRT:
    s = StatusRT()
    N.fe.GetCurrentStatusRT(C.byref(s))
    return s
