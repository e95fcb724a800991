"""ctypes bindings of the two C-ABI libraries (include/yrt_device.h, include/yrt_frontend.h,
include/YulioRT.h).

The libraries are built in-tree by ``make -C yulio-raytracer_amd`` (``__graft_entry__.build()``)
into ``yulio-raytracer_amd/lib``. There is no fallback: when they are missing, importing this
module raises, so no caller can silently run without the HIP path.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

# YRT_LIB_DIR selects an alternative in-tree build (e.g. a tuning variant under lib_variants/)
LIB_DIR = Path(os.environ.get("YRT_LIB_DIR", Path(__file__).resolve().parent.parent / "lib"))
DEVICE_LIB = LIB_DIR / "libdevice_singleray_mi355x.so"
FRONTEND_LIB = LIB_DIR / "libYulioRT_mi355x.so"


class NativeLibraryMissing(ImportError):
    pass


def _load(path: Path) -> C.CDLL:
    if not path.exists():
        raise NativeLibraryMissing(
            f"{path} is missing: build it with `make -C yulio-raytracer_amd` "
            "(or __graft_entry__.build()); the MI355X path has no CPU fallback")
    return C.CDLL(str(path), mode=os.RTLD_NOW | C.RTLD_GLOBAL)


dev = _load(DEVICE_LIB)
fe = _load(FRONTEND_LIB)

vp = C.c_void_p
cstr = C.c_char_p
f32 = C.c_float
i32 = C.c_int
sz = C.c_size_t
PF = C.POINTER(C.c_float)


class RenderStats(C.Structure):
    _fields_ = [(n, C.c_double) for n in (
        "raysClosest", "raysShadow", "samples", "msTotal", "msTraceClosest", "msTraceShadow", "msShade",
        "msOther", "launchesClosest", "launchesShadow", "nodeVisits", "triVisits", "gather", "msRender",
        "msGather")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class SceneInfo(C.Structure):
    _fields_ = [("numTriangles", C.c_int64), ("numGeometries", C.c_int64), ("numNodes", C.c_int64),
                ("bvhDepth", C.c_int64), ("numLights", C.c_int64), ("buildSeconds", C.c_double),
                ("bboxLo", C.c_float * 3), ("bboxHi", C.c_float * 3), ("numTriRefs", C.c_int64),
                ("triRecordBytes", C.c_int64), ("nodeBytesClosest", C.c_int64), ("nodeBytesAny", C.c_int64)]


class SessionInfo(C.Structure):
    _fields_ = [("device", vp), ("renderer", vp), ("tonemapper", vp), ("framebuffer", vp), ("scene", vp),
                ("width", i32), ("height", i32), ("stereo", i32), ("numFrames", i32),
                ("framebufferFormat", i32), ("gamma", f32)]


class ParamsRT(C.Structure):
    """include/YulioRT.h ParamsRT (devices/renderer/YulioRT.h:37-50)."""
    _fields_ = [("renderer", cstr), ("size", i32), ("depth", i32), ("tMaxShadowRay", f32), ("spp", i32),
                ("ambientlight", f32 * 3), ("eyeSeparation", f32), ("toeIn", C.c_bool), ("zeroParallax", f32),
                ("jpegQuality", i32), ("debug", C.c_bool), ("threadsPriority", i32), ("waterMark", C.c_bool),
                ("faceCullingMode", cstr)]


class StatusRT(C.Structure):
    _fields_ = [("state", i32), ("progress", f32), ("lastError", i32)]


def _sig(lib, name, res, *args):
    fn = getattr(lib, name)
    fn.restype = res
    fn.argtypes = list(args)
    return fn


# ---- device plugin (include/yrt_device.h)
_sig(dev, "yrtNewDevice", vp, cstr, sz, i32, cstr)
_sig(dev, "yrtDeleteDevice", None, vp)
_sig(dev, "yrtGetLastError", cstr, vp)
for _n in ("yrtNewCamera", "yrtNewTexture", "yrtNewMaterial", "yrtNewShape", "yrtNewLight", "yrtNewScene",
           "yrtNewToneMapper", "yrtNewRenderer"):
    _sig(dev, _n, vp, vp, cstr)
_sig(dev, "yrtNewData", vp, vp, cstr, sz, vp)
_sig(dev, "yrtNewImage", vp, vp, cstr, sz, sz, vp)
_sig(dev, "yrtNewImageFromFile", vp, vp, cstr)
_sig(dev, "yrtNewShapePrimitive", vp, vp, vp, vp, PF, i32)
_sig(dev, "yrtNewLightPrimitive", vp, vp, vp, vp, PF)
_sig(dev, "yrtSetPrimitive", i32, vp, vp, sz, vp)
_sig(dev, "yrtNewFrameBuffer", vp, vp, cstr, sz, sz, sz, vp)
_sig(dev, "yrtIncRef", i32, vp, vp)
_sig(dev, "yrtDecRef", i32, vp, vp)
_sig(dev, "yrtSetBool1", i32, vp, vp, cstr, i32)
_sig(dev, "yrtSetBool2", i32, vp, vp, cstr, i32, i32)
_sig(dev, "yrtSetBool3", i32, vp, vp, cstr, i32, i32, i32)
_sig(dev, "yrtSetBool4", i32, vp, vp, cstr, i32, i32, i32, i32)
_sig(dev, "yrtSetInt1", i32, vp, vp, cstr, i32)
_sig(dev, "yrtSetInt2", i32, vp, vp, cstr, i32, i32)
_sig(dev, "yrtSetInt3", i32, vp, vp, cstr, i32, i32, i32)
_sig(dev, "yrtSetInt4", i32, vp, vp, cstr, i32, i32, i32, i32)
_sig(dev, "yrtSetFloat1", i32, vp, vp, cstr, f32)
_sig(dev, "yrtSetFloat2", i32, vp, vp, cstr, f32, f32)
_sig(dev, "yrtSetFloat3", i32, vp, vp, cstr, f32, f32, f32)
_sig(dev, "yrtSetFloat4", i32, vp, vp, cstr, f32, f32, f32, f32)
_sig(dev, "yrtGetFloat1", i32, vp, vp, cstr, PF)
_sig(dev, "yrtGetFloat3", i32, vp, vp, cstr, PF, PF, PF)
_sig(dev, "yrtGetString", i32, vp, vp, cstr, C.c_char_p, sz)
_sig(dev, "yrtGetTransform", i32, vp, vp, cstr, PF)
_sig(dev, "yrtNewDataFromFile", vp, vp, cstr, cstr, sz, sz)
_sig(dev, "yrtTransformPrimitive", vp, vp, vp, PF)
_sig(dev, "yrtUpdatePrimitive", i32, vp, vp, sz, vp, PF, PF)
_sig(dev, "yrtPick", i32, vp, vp, f32, f32, vp, PF, PF, PF)
_sig(dev, "yrtSetArray", i32, vp, vp, cstr, cstr, vp, sz, sz, sz)
_sig(dev, "yrtSetString", i32, vp, vp, cstr, cstr)
_sig(dev, "yrtSetImage", i32, vp, vp, cstr, vp)
_sig(dev, "yrtSetTexture", i32, vp, vp, cstr, vp)
_sig(dev, "yrtSetTransform", i32, vp, vp, cstr, PF)
_sig(dev, "yrtSetPointer", i32, vp, vp, cstr, vp)
_sig(dev, "yrtClear", i32, vp, vp)
_sig(dev, "yrtCommit", i32, vp, vp)
_sig(dev, "yrtRenderFrame", i32, vp, vp, vp, vp, vp, vp, i32)
_sig(dev, "yrtRenderFrames", i32, vp, vp, C.POINTER(vp), i32, vp, vp, C.POINTER(vp), i32)
_sig(dev, "yrtMapFrameBuffer", vp, vp, vp, i32)
_sig(dev, "yrtUnmapFrameBuffer", i32, vp, vp, i32)
_sig(dev, "yrtSwapBuffers", i32, vp, vp)
STATUS_CB = C.CFUNCTYPE(None, i32, f32, vp)
_sig(dev, "yrtSetStatusCallback", i32, vp, vp, STATUS_CB, vp)
_sig(dev, "yrtSetStopFlag", i32, vp, vp, C.POINTER(C.c_int))
_sig(dev, "yrtIntersect", i32, vp, vp, vp, vp, C.c_uint32, vp, vp)
_sig(dev, "yrtOccluded", i32, vp, vp, vp, vp, C.c_uint32, vp, vp)
_sig(dev, "yrtTriangleIds", i32, vp, vp, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32))
_sig(dev, "yrtGetRenderStats", i32, vp, C.POINTER(RenderStats))
_sig(dev, "yrtSetKernelTiming", i32, vp, i32)
_sig(dev, "yrtSetLanes", i32, vp, i32)
_sig(dev, "yrtGetSceneInfo", i32, vp, vp, C.POINTER(SceneInfo))
_sig(dev, "yrtExportBVH", i32, vp, vp, vp, sz, vp, sz)
try:  # round 6; absent from older builds selected with YRT_LIB_DIR (same-box A/B against round 5)
    _sig(dev, "yrtExportQuantizedBVH", i32, vp, vp, vp, sz)
except AttributeError:
    pass
_sig(dev, "yrtExportFrame", C.c_int64, vp, vp, vp, vp, vp, sz)
_sig(dev, "yrtSetFrameSeed", i32, vp, C.c_uint32)
_sig(dev, "yrtSetBatchCapacity", i32, vp, C.c_int64)
_sig(dev, "yrtSetTileShard", i32, vp, i32, i32)
_sig(dev, "yrtShardCommUniqueId", i32, vp)
_sig(dev, "yrtSetShardComm", i32, vp, i32, i32, vp)
_sig(dev, "yrtRcclAvailable", i32)
try:  # absent from builds before round 4 selected with YRT_LIB_DIR (same-box A/B variants)
    _sig(dev, "yrtNewShardHub", vp, i32)
    _sig(dev, "yrtDeleteShardHub", None, vp)
    _sig(dev, "yrtSetShardHub", i32, vp, vp, i32)
    _sig(dev, "yrtSetGatherTimeout", i32, vp, C.c_double)
    _sig(dev, "yrtShardHubStatus", i32, vp, i32, i32, C.c_double)
    _sig(dev, "yrtShardHubSlab", i32, vp, i32, vp, sz, vp, sz, C.c_double)
    _sig(dev, "yrtShardHubLastError", cstr)
except AttributeError:
    pass
_sig(dev, "yrtGetDeviceCount", i32, vp)
_sig(dev, "yrtSetRefitCommits", i32, vp, i32)
_sig(dev, "yrtGetSceneRefits", i32, vp, vp)
_sig(dev, "yrtSetRayCapture", i32, vp, i32)
_sig(dev, "yrtGetCapturedRays", C.c_int64, vp, i32, i32, vp, vp, sz, C.POINTER(C.c_double))
_sig(dev, "yrtDebugTraceProfile", i32, vp, C.POINTER(C.c_uint64), i32)
try:  # debug-only entry; absent from older tuning builds selected with YRT_LIB_DIR
    _sig(dev, "yrtDebugCheckMath", i32, vp, i32, C.POINTER(C.c_uint64))
    _sig(dev, "yrtDebugCheckMathTable", i32, vp, i32, vp, C.POINTER(C.c_uint64))
    _sig(dev, "yrtDebugPixelSamples", i32, vp, i32, i32, vp, i32)
except AttributeError:
    pass
try:  # round 6; absent from older tuning builds selected with YRT_LIB_DIR
    _sig(dev, "yrtDebugTileScatter", i32, i32, i32)
except AttributeError:
    pass
_sig(dev, "yrtDebugDecodeImage", i32, cstr, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32), vp, sz)
_sig(dev, "yrtDebugSampleTable", i32, i32, i32, i32, i32, i32, cstr, PF, sz)

# ---- front end (include/yrt_frontend.h, include/YulioRT.h)
_sig(fe, "yrtSessionCreate", vp, vp, i32, C.POINTER(cstr))
_sig(fe, "yrtSessionDestroy", None, vp)
_sig(fe, "yrtFrontendLastError", cstr)
_sig(fe, "yrtSessionInfo", i32, vp, C.POINTER(SessionInfo))
_sig(fe, "yrtSessionCamera", vp, vp, i32)
_sig(fe, "yrtSessionRender", vp, vp, i32)
_sig(fe, "yrtSessionRenderCube", i32, vp)
_sig(fe, "yrtSessionRenderSceneCube", i32, vp, i32)
_sig(fe, "yrtSessionCubeFrameBuffer", vp, vp, i32)
_sig(fe, "yrtSessionNumSceneCameras", i32, vp)
_sig(fe, "yrtSessionSceneCamera", vp, vp, i32)
_sig(fe, "yrtSessionRenderSceneCamera", vp, vp, i32)
_sig(fe, "yrtSessionOutput", i32, vp, cstr)
_sig(fe, "yrtMain", i32, i32, C.POINTER(cstr))
_sig(fe, "yrtStoreImage", i32, cstr, i32, i32, i32, vp, sz, i32)
_sig(fe, "InitParamsRT", None, C.POINTER(ParamsRT))
_sig(fe, "StartRT", C.c_bool, cstr, C.POINTER(ParamsRT))
_sig(fe, "WaitRT", C.c_bool)
_sig(fe, "StopRT", C.c_bool, C.c_bool)
_sig(fe, "GetLastErrorRT", i32)
_sig(fe, "GetCurrentStatusRT", None, C.POINTER(StatusRT))
