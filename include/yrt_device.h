/* yrt_device.h — C ABI of the MI355X path-tracing device plugin (libdevice_singleray_mi355x.so).
 *
 * This is the reference's device plugin boundary made C-callable. Each entry point
 * replaces one virtual method of embree::Device (devices/device/device.h:51-330) with the
 * same arguments and semantics; the plugin factory replaces
 * `extern "C" Device* create(const char* parms, size_t numThreads, int threadsPriority,
 * const char* rtcore_cfg)` (devices/device_singleray/api/singleray_device.cpp:105-107,
 * resolved by devices/device/device.cpp:24-35).
 *
 * Conventions
 *   - Handles are opaque pointers to ref-counted objects starting at refcount 1
 *     (device_singleray/api/handle.h:26-31). yrtIncRef/yrtDecRef mirror rtIncRef/rtDecRef.
 *   - rtSet* values are buffered; yrtCommit (re)constructs the object (api/handle.h:99-103).
 *   - The reference throws std::runtime_error; here every call returns 0 on success and a
 *     negative code on failure, with the message in yrtGetLastError(device). No exception
 *     crosses the ABI.
 *   - Every call on one device is serialized by a device mutex (singleray_device.cpp:97).
 *   - yrtRenderFrame is synchronous (integratorrenderer.cpp:90-93); yrtMapFrameBuffer
 *     returns the host pixel pointer (singleray_device.cpp:439-447). The frame stays in HBM
 *     until the first yrtMapFrameBuffer of that buffer copies it to the host pixels (every
 *     read of the pixels goes through the map, as in the reference); framebuffers created
 *     over user pointers (yrtNewFrameBuffer ptrs) receive the pixels at the end of the render.
 */
#ifndef YRT_DEVICE_H
#define YRT_DEVICE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define YRT_API __attribute__((visibility("default")))

typedef struct YRTDevice_* YRTDevice;
typedef void* YRTHandle;

/* ---- device lifetime (Device::rtCreateDevice / create) ------------------------------ */
/* parms: "" or "device=N" to pick a HIP device; "host" creates a host-only device (loaders,
 * scene commit, BVH build, yrtExportFrame/BVH; rendering and ray queries fail) used by the
 * CPU test suite. numThreads / threadsPriority are accepted
 * for signature parity (they size the CPU TaskScheduler in the reference and are unused
 * on the GPU). */
/* parms: "" or "device=<k>": one HIP device; "devices=<a,b,...>" / "devices=all": the frame's
 * 16x16 tiles are dealt round-robin over several HIP devices, one host
 * thread each, and gathered on the first (RCCL over xGMI between distinct GPUs; an id may
 * repeat for logical shards of one GPU); "host": no GPU (loaders, BVH, frame export). */
YRT_API YRTDevice yrtNewDevice(const char* parms, size_t numThreads, int threadsPriority, const char* rtcore_cfg);
YRT_API void yrtDeleteDevice(YRTDevice dev);
YRT_API const char* yrtGetLastError(YRTDevice dev);

/* ---- object creation (device.h:126-214) ---------------------------------------------- */
YRT_API YRTHandle yrtNewCamera(YRTDevice dev, const char* type);        /* "pinhole", "stereo" */
YRT_API YRTHandle yrtNewData(YRTDevice dev, const char* type, size_t bytes, const void* data);
/* rtNewDataFromFile (device.h:144, singleray_device.cpp:204-222): "immutable" only. */
YRT_API YRTHandle yrtNewDataFromFile(YRTDevice dev, const char* type, const char* file, size_t offset, size_t bytes);
YRT_API YRTHandle yrtNewImage(YRTDevice dev, const char* type, size_t width, size_t height, const void* data);
                                                                       /* "RGB8","RGBA8","RGB_FLOAT32","RGBA_FLOAT32" */
YRT_API YRTHandle yrtNewImageFromFile(YRTDevice dev, const char* file); /* .ppm/.png/.jpg */
YRT_API YRTHandle yrtNewTexture(YRTDevice dev, const char* type);       /* "bilinear","nearest","image" */
YRT_API YRTHandle yrtNewMaterial(YRTDevice dev, const char* type);
YRT_API YRTHandle yrtNewShape(YRTDevice dev, const char* type);         /* "trianglemesh","sphere","triangle" */
YRT_API YRTHandle yrtNewLight(YRTDevice dev, const char* type);         /* "ambientlight","trianglelight","hdrilight" */
YRT_API YRTHandle yrtNewShapePrimitive(YRTDevice dev, YRTHandle shape, YRTHandle material, const float* transform12,
                                       int faceCamera);
YRT_API YRTHandle yrtNewLightPrimitive(YRTDevice dev, YRTHandle light, YRTHandle material, const float* transform12);
/* rtTransformPrimitive (device.h:197): new primitive with transform * prim.transform. */
YRT_API YRTHandle yrtTransformPrimitive(YRTDevice dev, YRTHandle prim, const float* transform12);
YRT_API YRTHandle yrtNewScene(YRTDevice dev, const char* type);
YRT_API int yrtSetPrimitive(YRTDevice dev, YRTHandle scene, size_t slot, YRTHandle prim);
/* rtUpdatePrimitive (device.h:207, singleray_device.cpp:354-398): re-aims a faceCamera
 * primitive at camPos (floor-projected) with up camUp; no-op for other primitives. The scene
 * must be re-committed afterwards, as renderer.cpp:550-559 does per cube face. */
YRT_API int yrtUpdatePrimitive(YRTDevice dev, YRTHandle scene, size_t slot, YRTHandle prim, const float* camPos3,
                               const float* camUp3);
YRT_API YRTHandle yrtNewToneMapper(YRTDevice dev, const char* type);    /* "default" */
YRT_API YRTHandle yrtNewRenderer(YRTDevice dev, const char* type);      /* "pathtracer", "debug" */
YRT_API YRTHandle yrtNewFrameBuffer(YRTDevice dev, const char* type, size_t width, size_t height, size_t buffers,
                                    void** ptrs);

/* ---- reference counting / properties (device.h:237-312) ----------------------------- */
YRT_API int yrtIncRef(YRTDevice dev, YRTHandle h);
YRT_API int yrtDecRef(YRTDevice dev, YRTHandle h);
YRT_API int yrtSetBool1(YRTDevice dev, YRTHandle h, const char* property, int x);
YRT_API int yrtSetBool2(YRTDevice dev, YRTHandle h, const char* property, int x, int y);
YRT_API int yrtSetBool3(YRTDevice dev, YRTHandle h, const char* property, int x, int y, int z);
YRT_API int yrtSetBool4(YRTDevice dev, YRTHandle h, const char* property, int x, int y, int z, int w);
YRT_API int yrtSetInt1(YRTDevice dev, YRTHandle h, const char* property, int x);
YRT_API int yrtSetInt2(YRTDevice dev, YRTHandle h, const char* property, int x, int y);
YRT_API int yrtSetInt3(YRTDevice dev, YRTHandle h, const char* property, int x, int y, int z);
YRT_API int yrtSetInt4(YRTDevice dev, YRTHandle h, const char* property, int x, int y, int z, int w);
YRT_API int yrtSetFloat1(YRTDevice dev, YRTHandle h, const char* property, float x);
YRT_API int yrtSetFloat2(YRTDevice dev, YRTHandle h, const char* property, float x, float y);
YRT_API int yrtSetFloat3(YRTDevice dev, YRTHandle h, const char* property, float x, float y, float z);
YRT_API int yrtSetFloat4(YRTDevice dev, YRTHandle h, const char* property, float x, float y, float z, float w);
YRT_API int yrtGetFloat1(YRTDevice dev, YRTHandle h, const char* property, float* x);
YRT_API int yrtGetFloat3(YRTDevice dev, YRTHandle h, const char* property, float* x, float* y, float* z);
/* rtGetString (device.h:293): copies at most bufSize-1 bytes + NUL; returns the full length. */
YRT_API int yrtGetString(YRTDevice dev, YRTHandle h, const char* property, char* buf, size_t bufSize);
/* rtGetTransform (device.h:303): 12 floats (vx, vy, vz, p); identity when unset. */
YRT_API int yrtGetTransform(YRTDevice dev, YRTHandle h, const char* property, float* transform12);
YRT_API int yrtSetArray(YRTDevice dev, YRTHandle h, const char* property, const char* type, YRTHandle data,
                        size_t size, size_t stride, size_t ofs);
YRT_API int yrtSetString(YRTDevice dev, YRTHandle h, const char* property, const char* str);
YRT_API int yrtSetImage(YRTDevice dev, YRTHandle h, const char* property, YRTHandle image);
YRT_API int yrtSetTexture(YRTDevice dev, YRTHandle h, const char* property, YRTHandle texture);
YRT_API int yrtSetTransform(YRTDevice dev, YRTHandle h, const char* property, const float* transform12);
YRT_API int yrtSetPointer(YRTDevice dev, YRTHandle h, const char* property, void* p);
YRT_API int yrtClear(YRTDevice dev, YRTHandle h);
YRT_API int yrtCommit(YRTDevice dev, YRTHandle h);

/* ---- rendering (device.h:223-234, 322) ----------------------------------------------- */
YRT_API int yrtRenderFrame(YRTDevice dev, YRTHandle renderer, YRTHandle camera, YRTHandle scene,
                           YRTHandle tonemapper, YRTHandle framebuffer, int accumulate);
/* Several frames of one scene in one wavefront job: frame k seen through cameras[k] into
 * framebuffers[k] (all the same size and format). With accumulate = 0 the result equals
 * numFrames rtRenderFrame calls with accumulate = 0, bit for bit (the per-tile Random of
 * integratorrenderer.cpp:134 and every per-pixel input depend on the frame's own pixel only),
 * but the frames' 16x16 tiles form one sequence (frame-major) that fills the batches and is
 * dealt over shards and GPUs as a whole, with one gather per job. This is the loop of the
 * stereo-cube drivers over the 12 faces of a view (renderer.cpp:543-737, 742-878) when no
 * primitive changes between the faces. accumulate != 0 is accepted for numFrames == 1 only (a
 * job keeps one sampler iteration and no per-frame accumulation state across calls). */
YRT_API int yrtRenderFrames(YRTDevice dev, YRTHandle renderer, const YRTHandle* cameras, int numFrames,
                            YRTHandle scene, YRTHandle tonemapper, const YRTHandle* framebuffers, int accumulate);
YRT_API void* yrtMapFrameBuffer(YRTDevice dev, YRTHandle framebuffer, int bufID);
YRT_API int yrtUnmapFrameBuffer(YRTDevice dev, YRTHandle framebuffer, int bufID);
YRT_API int yrtSwapBuffers(YRTDevice dev, YRTHandle framebuffer);
/* rtPick (device.h:329, singleray_device.cpp:692-708): world position of the closest hit of
 * the camera ray through image-plane point (x, y) in [0,1]^2. Returns 1 hit, 0 miss, <0 error. */
YRT_API int yrtPick(YRTDevice dev, YRTHandle camera, float x, float y, YRTHandle scene, float* px, float* py,
                    float* pz);
/* Renderer status callback (device.h:335-347): state 0 Inactive, 1 Rendering, 2 Done. */
typedef void (*YRTStatusCallback)(int state, float progress, void* user);
YRT_API int yrtSetStatusCallback(YRTDevice dev, YRTHandle renderer, YRTStatusCallback cb, void* user);
/* Stop flag polled between wavefront iterations (renderer "stopFlag", integratorrenderer.h:100). */
YRT_API int yrtSetStopFlag(YRTDevice dev, YRTHandle renderer, volatile int* flag);

/* ---- hot-path ray queries: rtcIntersect / rtcOccluded over device-resident streams ---- */
/* org4[i] = (org.xyz, tnear), dir4[i] = (dir.xyz, tfar) ; hit4[i] = (t, u, v, triId bits)
 * occluded[i] = 1/0. All pointers are HIP device pointers; stream may be NULL (default).
 * Replaces rtcIntersect (pathtraceintegrator.cpp:72) and rtcOccluded (:160). */
YRT_API int yrtIntersect(YRTDevice dev, YRTHandle scene, const float* org4, const float* dir4, uint32_t n,
                         float* hit4, void* stream);
YRT_API int yrtOccluded(YRTDevice dev, YRTHandle scene, const float* org4, const float* dir4, uint32_t n,
                        int32_t* occluded, void* stream);
/* Maps a global triangle id (hit4.w) to Embree's (geomID, primID). */
YRT_API int yrtTriangleIds(YRTDevice dev, YRTHandle scene, int32_t tri, int32_t* geomID, int32_t* primID);

/* ---- statistics of the last yrtRenderFrame (integratorrenderer.cpp:96-116) ------------ */
typedef struct YRTRenderStats {
  double raysClosest;     /* rtcIntersect-equivalent queries  */
  double raysShadow;      /* rtcOccluded-equivalent queries   */
  double samples;         /* W*H*spp                          */
  double msTotal;         /* wall time of yrtRenderFrame      */
  double msTraceClosest;  /* summed kernel time (HIP events) when timing enabled */
  double msTraceShadow;
  double msShade;
  double msOther;
  double launchesClosest; /* kernel launches of each kind */
  double launchesShadow;
  double nodeVisits;      /* reserved (0): visit counts come from oracle_count_visits */
  double triVisits;
  double gather;          /* how the frame was gathered: YRT_GATHER_* */
  double msRender;        /* wall time until this process's tiles were rendered (multi-GPU diagnosis) */
  double msGather;        /* wall time of the gather after that (0 without one; includes waiting for peers) */
} YRTRenderStats;
#define YRT_GATHER_NONE 0           /* one device, no gather */
#define YRT_GATHER_D2D 1            /* logical shards of one GPU: device-to-device copy */
#define YRT_GATHER_RCCL_LOCAL 2     /* distinct GPUs of one process: RCCL (ncclCommInitAll) send/recv */
#define YRT_GATHER_PEER_COPY 3      /* distinct GPUs, RCCL unavailable or timed out: hipMemcpyPeerAsync */
#define YRT_GATHER_RCCL_PROCESS 4   /* one process per GPU: RCCL communicator (yrtSetShardComm) */
#define YRT_GATHER_HUB 5            /* several devices of one process: shard hub (yrtSetShardHub) */
YRT_API int yrtGetRenderStats(YRTDevice dev, YRTRenderStats* out);
/* 1 = bracket every kernel with HIP events (adds sync-free event records). */
YRT_API int yrtSetKernelTiming(YRTDevice dev, int enable);
/* Wavefront lanes (HIP streams whose batches overlap) of every render context, 1..4; 0 = the
 * default (3, or YRT_LANES). With one lane no two kernels of a frame overlap, so the kernel
 * timings above are each kernel's own duration (bench.py's roofline uses such a frame). */
YRT_API int yrtSetLanes(YRTDevice dev, int lanes);
/* Scene info: triangles, geometries, BVH nodes, BVH depth, build seconds; numTriRefs = leaf
 * triangle records (>= numTriangles: spatial splits reference a triangle from several leaves). */
typedef struct YRTSceneInfo {
  int64_t numTriangles, numGeometries, numNodes, bvhDepth, numLights;
  double buildSeconds;
  float bboxLo[3], bboxHi[3];
  int64_t numTriRefs;
  int64_t triRecordBytes;  /* bytes per leaf triangle record (48, or 64 with a stored normal) */
  /* bytes per BVH node the closest-hit / any-hit traversal reads: 128 (float planes) or 64
   * (8-bit quantized planes, yulio-raytracer_amd/csrc/common/yrt_qnode.h) */
  int64_t nodeBytesClosest, nodeBytesAny;
} YRTSceneInfo;
YRT_API int yrtGetSceneInfo(YRTDevice dev, YRTHandle scene, YRTSceneInfo* out);
/* Copies the host mirror of the BVH (4-wide nodes: 128 B each, numTriRefs leaf tris: 48 B each). */
YRT_API int yrtExportBVH(YRTDevice dev, YRTHandle scene, void* nodes, size_t nodesBytes, void* tris,
                         size_t trisBytes);
/* The same tree with the any-hit traversal's 64-byte quantized nodes (node i = node i of
 * yrtExportBVH; layout yulio-raytracer_amd/csrc/common/yrt_qnode.h): numNodes * 64 bytes. */
YRT_API int yrtExportQuantizedBVH(YRTDevice dev, YRTHandle scene, void* qnodes, size_t qnodesBytes);
/* Serializes the committed scene graph + renderer + camera as the oracle's input blob
 * (format: oracle/yrt_oracle.h). Returns the byte count; call with buf=NULL to size. */
YRT_API int64_t yrtExportFrame(YRTDevice dev, YRTHandle renderer, YRTHandle camera, YRTHandle scene, void* buf,
                               size_t bytes);
/* Frame seed of the shadow-jitter hash (replaces C rand(), pathtraceintegrator.cpp:151). */
YRT_API int yrtSetFrameSeed(YRTDevice dev, uint32_t seed);
/* Paths in flight per wavefront batch (default 64M, ~10 GB of wavefront state); smaller for tests. */
YRT_API int yrtSetBatchCapacity(YRTDevice dev, int64_t paths);
/* Tile sharding across processes: this process renders only the tiles with
 * (tileIndex % count) == index (dealt further over its own HIP devices, see yrtNewDevice);
 * without a communicator (yrtSetShardComm) the other tiles' pixels are left zero. With a
 * communicator, only its own (rank, world) shard is accepted. */
YRT_API int yrtSetTileShard(YRTDevice dev, int index, int count);
/* Multi-GPU, one process per GPU (the reference's device_network image split,
 * devices/device_network/network_device.cpp:255-300, as an RCCL gather over xGMI):
 * yrtShardCommUniqueId fills 128 bytes on rank 0 (ncclGetUniqueId), which the caller
 * broadcasts; every rank then calls yrtSetShardComm with it. Tiles are dealt round-robin
 * (tile % world == rank) and every rtRenderFrame ends with a grouped RCCL send of each rank's
 * tile slab to rank 0, whose framebuffer then holds the whole frame. */
YRT_API int yrtShardCommUniqueId(void* id128);
/* Every rank of a job calls yrtSetShardComm (collective: RCCL ncclCommInitRank). Before each
 * gather the ranks exchange their render status, so a rank whose render throws (or whose
 * render call fails on its arguments) makes every rank's yrtRenderFrame fail instead of
 * leaving rank 0 waiting. Every wait of the gather is bounded (yrtSetGatherTimeout): on expiry
 * the communicator is aborted (ncclCommAbort) and the call fails with the phase that timed
 * out; later gathers on it fail at once. world = 1 drops the communicator. The gathered slabs carry 4 bytes per pixel for RGB8 framebuffers (16 else).
 * Only rank 0's framebuffers receive pixels; the other ranks' host framebuffers are left as
 * they were (their part of the frame is already on rank 0). */
YRT_API int yrtSetShardComm(YRTDevice dev, int rank, int world, const void* id128);
/* The same gather between several devices of one process (threads; they may share a GPU):
 * yrtNewShardHub(world) is the meeting point, and yrtSetShardHub(dev, hub, rank) arms device
 * `rank` (tile shard rank of world) exactly as yrtSetShardComm would; hub = NULL disarms. The
 * slabs move by hipMemcpyPeerAsync (device-to-device on one GPU). This runs the process
 * gather's bookkeeping — status exchange, per-rank tile counts, pack, unpack, the failing-rank
 * path — on one GPU. A device keeps the hub alive; yrtDeleteShardHub drops the caller's. */
typedef struct YRTShardHub_* YRTShardHub;
YRT_API YRTShardHub yrtNewShardHub(int world);
YRT_API void yrtDeleteShardHub(YRTShardHub hub);
YRT_API int yrtSetShardHub(YRTDevice dev, YRTShardHub hub, int rank);
/* Bound, in seconds, of the waits of a gather; default YRT_GATHER_TIMEOUT_S or 300. The slab
 * send/recv wait at most this long; the status exchange, which also waits for the slowest rank's
 * render, this plus ten times the calling rank's render time of the frame. */
YRT_API int yrtSetGatherTimeout(YRTDevice dev, double seconds);
/* Host-memory forms of the hub's two phases (CPU tests of its deadlines and size checks):
 * yrtShardHubStatus returns the min of the ranks' flags (or -1), yrtShardHubSlab sends `bytes`
 * to rank 0 (rank > 0) or receives every peer's recvBytesPerRank bytes into recv in rank
 * order (rank 0). Errors: -1 and yrtShardHubLastError() (per calling thread). */
YRT_API int yrtShardHubStatus(YRTShardHub hub, int rank, int flag, double timeoutS);
YRT_API int yrtShardHubSlab(YRTShardHub hub, int rank, const void* slab, size_t bytes, void* recv,
                            size_t recvBytesPerRank, double timeoutS);
YRT_API const char* yrtShardHubLastError(void);
/* 1 when librccl can be loaded (checked on every rank before the collective comm init). */
YRT_API int yrtRcclAvailable(void);
/* HIP devices (logical shards) this device renders on (yrtNewDevice "devices=..."). */
YRT_API int yrtGetDeviceCount(YRTDevice dev);
/* Scene commits that only move the vertices of some primitives (faceCamera re-orientation by
 * rtUpdatePrimitive, the FPR loop of renderer.cpp:550-559) refit the BVH on the GPU instead of
 * rebuilding it (on by default). yrtGetSceneRefits: refit commits since the last rebuild. */
YRT_API int yrtSetRefitCommits(YRTDevice dev, int on);
YRT_API int yrtGetSceneRefits(YRTDevice dev, YRTHandle scene);
/* Host sampler check: writes the SoA sample table (dims x (sets*spp)) that the frame
 * renderer uploads (sampler/sampler.cpp:46-126 restated); returns sets*spp records. */
/* Ray capture for the roofline's algorithmic bytes: while maxPerDepth > 0,
 * yrtRenderFrame keeps a strided sample (<= maxPerDepth rays) of the closest-hit and shadow
 * query streams of every depth of its first wavefront batch (synchronizes per depth: use on
 * an untimed frame). yrtGetCapturedRays returns the sample size and the stream's full size. */
YRT_API int yrtSetRayCapture(YRTDevice dev, int maxPerDepth);
YRT_API int64_t yrtGetCapturedRays(YRTDevice dev, int shadow, int depth, float* org4, float* dir4, size_t maxRays,
                                   double* totalInBatch);
/* Profiling builds (-DYRT_PROFILE) only: k_trace SIMD-utilization counters since the last
 * reset (outer iterations, lanes with a ray, node-phase iterations, lanes at a node, leaf
 * passes, triangle-loop iterations, useful triangle tests, 0). Returns -1 otherwise. */
YRT_API int yrtDebugTraceProfile(YRTDevice dev, uint64_t* out8, int reset);
/* Arithmetic self-check on the device: fn 0 compares the kernels' correctly rounded fast
 * reciprocal (rcp_rn, common/yrt_math.h) with the IEEE division 1.0f/x for all 2^32 inputs.
 * out2[0] = mismatches, out2[1] = the smallest mismatching input (or UINT64_MAX). */
YRT_API int yrtDebugCheckMath(YRTDevice dev, int fn, uint64_t* out2);
/* Arithmetic self-check of the emulated SSE estimates the reference's rcp/rsqrt start from
 * (common/yrt_sse_rcp.h; common/math/math.h:38-59): fn 1 rcpps, fn 2 rsqrtps, each against its
 * reconstruction from table2048 (the 12-bit mantissas of tests/golden/sse_rcp_tables.json) for
 * all 2^32 inputs. out2 as yrtDebugCheckMath. */
YRT_API int yrtDebugCheckMathTable(YRTDevice dev, int fn, const uint16_t* table2048, uint64_t* out2);
/* The image tile that logical tile t of a sharded job's frame of T tiles covers
 * (common/yrt_tile_scatter.h: a fixed bijection of [0, T), used by the renderer and the gather
 * whenever the tile stride is above 1). Host-side; -1 for t outside [0, T). */
YRT_API int yrtDebugTileScatter(int t, int T);
/* Parity debugging: out4 == NULL arms the capture of the per-sample radiance (the pathL terms
 * the resolve sums, in s order) of pixel id y*width+x (-1 disarms) of frame `frame` for the
 * following renders (buffer of maxSamples float4); out4 != NULL copies the captured samples
 * and returns their count (at most maxSamples: the kernel writes no more than the buffer
 * holds). Captures on the device's first GPU only (a multi-GPU device's other GPUs render
 * their tiles uncaptured). Compare with oracle_debug_pixel. */
YRT_API int yrtDebugPixelSamples(YRTDevice dev, int pixelId, int frame, float* out4, int maxSamples);
/* Decoder check: 8-bit pixels of a .jpg/.png in file row order (top row first), before the
 * Image4c flip/requantization of rtNewImageFromFile. Call with out=NULL to get the size. */
YRT_API int yrtDebugDecodeImage(const char* file, int* width, int* height, int* channels, uint8_t* out,
                                size_t outBytes);
YRT_API int yrtDebugSampleTable(int spp, int sets, int iteration, int num1D, int num2D, const char* filter,
                                float* out, size_t outFloats);

#ifdef __cplusplus
}
#endif

#endif /* YRT_DEVICE_H */
