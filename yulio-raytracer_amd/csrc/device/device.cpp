// device.cpp — the MI355X device plugin: C-ABI entry points (include/yrt_device.h) over the
// object model, scene commit and the wavefront frame renderer.
//
// Reference counterparts: SingleRayDevice (device_singleray/api/singleray_device.cpp:99-709),
// IntegratorRenderer::renderFrame/RenderJob (renderers/integratorrenderer.cpp:63-185),
// DebugRenderer (renderers/debugrenderer.cpp:66-140).
#include "../../../include/yrt_device.h"
#include "../common/yrt_tile_scatter.h"

#include <string.h>
#include <strings.h>

#include <chrono>
#include <cmath>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <memory>
#include <deque>
#include <thread>

#include "../kernels/yrt_kernels.h"
#include "image_io.h"
#include "objects.h"
#include "scene_gpu.h"
#include "gather.h"
#include "rccl_comm.h"
#include "sampler.h"

namespace yrt {

#ifndef YRT_STACK_DEPTH
#define YRT_STACK_DEPTH 64
#endif

struct FrameCache {
  std::string key;
  SampleTable table;
  DevBuf dims, light;
  std::vector<uint8_t> slotLive;  // per light-sample slot: some record's radiance is not exactly 0
};

// One HIP device's rendering state: its streams (lanes), the frame buffers, the wavefront
// queues and the sample tables uploaded to it. A Device renders on one or several of these
// (yrtNewDevice "devices=..."): 16x16 tiles are dealt round-robin over them,
// one host thread drives each, and the frame is gathered on the first (rccl_comm.h).
struct GpuCtx {
  int hipDevice = 0;
  hipStream_t stream = nullptr;  // lanes[0].stream
  // A wavefront lane: a stream and the batch state it owns. Batches alternate between the
  // lanes so one batch's kernels run beside the other's (the VALU-bound traversal next to the
  // latency-bound shading).
  struct Lane {
    hipStream_t stream = nullptr;
    DevBuf qPath[2], qOrg[2], qDir[2], qThr[2], hit, hitGeom, pathL, shFirst, sOrg, sDir, sContrib, sOcc, counters, spill;
    DevBuf qTime[2], sTime;  // ray times (moving scenes only)
    int64_t pathCap = 0, shadowCap = 0;
    // Batches enqueued whose queue counters are not yet accounted, oldest first: a pinned
    // copy of the counters (written by the stream after the batch's last trace), the event
    // after that copy, the batch's tiles (progress) and its place in the job (seq). A lane
    // takes its next batch once its previous batch's counters have arrived — before that
    // batch's pixel resolve, so the host enqueues while the resolve runs. Two batches ahead
    // per lane measured the same (profiles/r04/ab_r04k.txt).
    struct Pend {
      unsigned* hc = nullptr;
      size_t hcWords = 0;
      hipEvent_t done = nullptr;
      int64_t tiles = 0;
      int64_t seq = 0;
      bool fused = false;  // depth 0 ran as k_trace's camera-ray instantiation (hits queued only)
    };
    static constexpr int kPendDepth = 1;
    Pend pend[kPendDepth];
    int pendHead = 0, pendCount = 0;
  };
#ifndef YRT_MAX_LANES
#define YRT_MAX_LANES 4  // one HIP stream each; HIP gives a process 4 hardware queues by default
#endif
  static constexpr int kMaxLanes = YRT_MAX_LANES;  // YRT_LANES may ask for up to this many
  // three: a process gets 4 hardware queues (GPU_MAX_HW_QUEUES), and four lane streams plus the
  // context's own stream (clears, copies, the gather) share them. Same box against four
  // (profiles/r06/ab_r06r.txt): C3 +3.4 %, C4 cube job -1.7 %, C5 -2.7 %, N = 8 rank shares C3
  // -13.5 % (slowest) and C4 -5 %. (Round 5: four over two C3 +1.4 %, ab_lanes_r05q.txt; rounds
  // 1-2: two +4 % over one.)
  static constexpr int kDefaultLanes = 3;
  static int default_lanes() {
    int lanes = kDefaultLanes;
    if (const char* e = getenv("YRT_LANES")) lanes = std::max(1, std::min(kMaxLanes, atoi(e)));
    return lanes;
  }
  Lane lanes[kMaxLanes];
  int numLanes = kDefaultLanes;
  DevBuf dRp, dCam, dPixelSets, dAccu, dCount, dSpill, dSlab, dDirect;
  // The frames a job renders into (float RGB and RGB8 rows, frame-major). On the primary
  // device a job's framebuffers keep a reference to their block until rtMapFrameBuffer reads
  // them back, so the next job renders into the spare (or a fresh) block meanwhile.
  struct FrameBlock {
    DevBuf fbFloat, fbRGB8;
    // the shard layout (index, count, width, height, frames) whose other shards' pixels this
    // block holds as zeros (a one-shard render writes only its own tiles); -1: unknown
    long long zeroKey[5] = {-1, -1, -1, -1, -1};
  };
  std::shared_ptr<FrameBlock> blk = std::make_shared<FrameBlock>(), spareBlk;
  // every block allocated after the first two (weak: a block lives while a framebuffer's
  // unread frame or blk / spareBlk holds it); at most kMaxFrameBlocks stay alive
  static constexpr int kMaxFrameBlocks = 3;
  std::vector<std::weak_ptr<FrameBlock>> extraBlocks;
  float* fbFloat() const { return blk->fbFloat.as<float>(); }
  uint8_t* fbRGB8() const { return blk->fbRGB8.as<uint8_t>(); }
  std::vector<int> hDirect;        // the frame's direct-light list (uploaded to dDirect)
  std::vector<GpuCamera> hCams;  // the job's cameras, one per frame (uploaded to dCam)
  DevBuf dBackplate;                       // the renderer's backplate image (texels)
  uint64_t backplateSerial = 0;            // ImageObj::serial of the image dBackplate holds
  // (width, height, sets) of the pixel-set map dPixelSets holds: the map depends on nothing else
  // (integratorrenderer.cpp:126-131 seeds by tile position), so a frame of the same size reuses it
  long long pixelSetsKey[3] = {-1, -1, -1};
  // per committed scene (GpuScene::serial): camera rays traced by fused depth-0 batches
  // (launch_trace_primary) and how many of them left the scene; their ratio picks the depth-0
  // kernels (a running total: one batch's share varies with the faces it covers)
  std::map<uint64_t, std::pair<double, double>> missFrac;
  std::map<int, DevBuf> recvSlabs;  // gather on the first device: one slab per peer
  // sample tables by request (a progressive or multi-GPU weak-scaling run cycles through a
  // few sampler iterations; rebuilding a table costs ~9 ms of host time per frame)
  static constexpr size_t kMaxFrameCaches = 16;
  std::map<std::string, std::unique_ptr<FrameCache>> fcaches;
  std::deque<std::string> fcacheOrder;
  std::vector<hipEvent_t> eventPool;
  YRTRenderStats stats{};
  struct Captured { std::vector<float> org, dir; double total = 0; };
  std::vector<Captured> capClosest, capShadow;

  GpuCtx(int dev, int lanesWanted) : hipDevice(dev), numLanes(lanesWanted) {
    HIP_CHECK(hipSetDevice(hipDevice));
    ensure_streams(1);
    stream = lanes[0].stream;
  }
  // A lane's stream is created when a render first uses the lane: several contexts
  // in one process (e.g. devices=[0,0]) all map their lanes onto the process's 4 hardware queues
  // (GPU_MAX_HW_QUEUES), so streams nobody renders on only add to that sharing.
  void ensure_streams(int n) {
    for (int l = 0; l < n && l < kMaxLanes; ++l)
      if (!lanes[l].stream) HIP_CHECK(hipStreamCreateWithFlags(&lanes[l].stream, hipStreamNonBlocking));
  }
  ~GpuCtx() {
    (void)hipSetDevice(hipDevice);
    for (auto e : eventPool) (void)hipEventDestroy(e);
    for (Lane& L : lanes) {
      for (Lane::Pend& P : L.pend) {
        if (P.hc) (void)hipHostFree(P.hc);
        if (P.done) (void)hipEventDestroy(P.done);
      }
      if (L.stream) (void)hipStreamDestroy(L.stream);
    }
  }
  hipEvent_t ev() {
    hipEvent_t e;
    HIP_CHECK(hipEventCreate(&e));
    eventPool.push_back(e);
    return e;
  }
  int* spill() {
    dSpill.alloc(YRT_TRACE_SPILL_INTS * sizeof(int));
    return dSpill.as<int>();
  }
  // P paths per batch; queues hold YRT_QSEGS segments of qseg_capacity(P) slots
  static void ensure_paths(Lane& L, int64_t P, int numLights, bool motion) {
    const int64_t Q = (int64_t)YRT_QSEGS * qseg_capacity(P);
    if (Q > L.pathCap) {
      for (int k = 0; k < 2; ++k) {
        L.qPath[k].alloc(Q * 4);
        L.qOrg[k].alloc(Q * 16);
        L.qDir[k].alloc(Q * 16);
        L.qThr[k].alloc(Q * 16);
      }
      L.hit.alloc(Q * 16);
      if (trace_hit_geom()) L.hitGeom.alloc(Q * 4);
      L.pathL.alloc(Q * 16);
      L.pathCap = Q;
    }
    const int64_t S = Q * std::max(1, numLights);
    if (S > L.shadowCap) {
      L.shFirst.alloc(S * 4);
      L.sOrg.alloc(S * 16);
      L.sDir.alloc(S * 16);
      L.sContrib.alloc(S * 16);
      L.sOcc.alloc(S * 4);
      L.shadowCap = S;
    }
    if (motion) {
      for (int k = 0; k < 2; ++k) L.qTime[k].alloc(Q * 4);
      L.sTime.alloc(S * 4);
    }
  }
  // ray capture (roofline accounting): strided sample of each depth's query streams, batch 0
  // counts: the queue's first segment counter; segments of segCap slots
  void capture(int captureMax, std::vector<Captured>& out, int depth, const float4* org, const float4* dir,
               const unsigned* counts, int segCap, hipStream_t st) {
    std::vector<unsigned> cs((size_t)YRT_QSEGS * YRT_QCSTRIDE);
    HIP_CHECK(hipMemcpyAsync(cs.data(), counts, cs.size() * sizeof(unsigned), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    size_t n = 0;
    for (int k = 0; k < YRT_QSEGS; ++k) n += cs[(size_t)k * YRT_QCSTRIDE];
    if ((int)out.size() <= depth) out.resize(depth + 1);
    Captured& c = out[depth];
    c.total = (double)n;
    c.org.clear();
    c.dir.clear();
    const size_t stride = std::max<size_t>(1, (n + captureMax - 1) / captureMax);
    for (int k = 0; k < YRT_QSEGS; ++k) {
      const size_t nk = cs[(size_t)k * YRT_QCSTRIDE];
      const size_t m = nk ? (nk + stride - 1) / stride : 0;
      if (!m) continue;
      const size_t at = c.org.size();
      c.org.resize(at + m * 4);
      c.dir.resize(at + m * 4);
      HIP_CHECK(hipMemcpy2D(c.org.data() + at, 16, org + (size_t)k * segCap, stride * 16, 16, m,
                            hipMemcpyDeviceToHost));
      HIP_CHECK(hipMemcpy2D(c.dir.data() + at, 16, dir + (size_t)k * segCap, stride * 16, 16, m,
                            hipMemcpyDeviceToHost));
    }
  }
};

// the tiles of shard (index, count): tile = index + j * count, j < shard_tiles
static int shard_tiles(int numTiles, int index, int count) {
  return numTiles > index ? (numTiles - index + count - 1) / count : 0;
}

void fb_read_back(FrameBufferObj& F, int id);

class Device {
 public:
  std::recursive_mutex mu;
  std::string lastError;
  std::set<HandleRef*> handles;
  std::vector<std::unique_ptr<GpuCtx>> ctx;  // ctx[0]: the primary device (commits, queries, output)
  int hipDevice = 0;                         // ctx[0]'s
  hipStream_t stream = nullptr;              // ctx[0]'s
  uint32_t frameSeed = 0x2545F491u;
#ifndef YRT_DEFAULT_CAPACITY_M
#define YRT_DEFAULT_CAPACITY_M 64
#endif
  int64_t capacity = (int64_t)YRT_DEFAULT_CAPACITY_M << 20;  // paths per batch: C3 +4 % over 16 M (fewer launch tails), ~10 GB
  // process-level shard (yrtSetTileShard / yrtSetShardComm): this process renders tiles
  // t = shardIndex (mod shardCount), dealt over its own devices
  int shardIndex = 0, shardCount = 1;
  // process-level gather to rank 0 (gather.h): RCCL (yrtSetShardComm) or an in-process hub
  // of several Device objects (yrtSetShardHub)
  std::unique_ptr<GatherTransport> proc;
  int commRank = 0, commWorld = 1;   // proc's rank / size: the only shard it gathers
  double gatherTimeout = default_gather_timeout();  // bound of every gather wait (yrtSetGatherTimeout)
  ncclComm_t localComm = nullptr;    // the ctx devices' gather (distinct devices only): rank 0's
  std::vector<ncclComm_t> localComms;  // one per ctx device (ncclCommInitAll)
  // ncclCommInitAll failed (or a gather over it timed out): distinct devices gather with
  // hipMemcpyPeerAsync instead, reported as YRT_GATHER_PEER_COPY in the render stats
  bool localRcclOff = getenv("YRT_NO_LOCAL_RCCL") != nullptr;
  std::string localRcclWhy;
  bool refitCommits = true;  // SceneObj::commit refits faceCamera-only changes (yrtSetRefitCommits)
  bool kernelTiming = false;
  YRTRenderStats stats{};
  int captureMax = 0;

  bool gpu = true;  // false: host-only device (loaders, BVH, export; no rendering) for CPU tests
  Device(const std::vector<int>& devs, bool useGpu) : gpu(useGpu) {
    if (!gpu) return;
    const int lanes = GpuCtx::default_lanes();
    for (int d : devs) ctx.emplace_back(new GpuCtx(d, lanes));
    hipDevice = ctx[0]->hipDevice;
    stream = ctx[0]->stream;
    HIP_CHECK(hipSetDevice(hipDevice));
  }
  DevBuf dbgPixelBuf;   // yrtDebugPixelSamples capture (a debugging aid), armed on this device
  int dbgPixelCap = 0;
  ~Device() {
    if (dbgPixelBuf.p) (void)debug_pixel_capture(-1, -1, nullptr, 0);  // no kernel may write it once freed
    for (auto* h : handles) delete h;
    handles.clear();
    try {
      for (auto c : localComms) rccl().CommDestroy(c);
    } catch (...) {
    }
    proc.reset();
  }

  YRTHandle wrap(std::shared_ptr<Object> o) {
    o->dev = this;
    auto* h = new HandleRef();
    h->obj = std::move(o);
    handles.insert(h);
    return (YRTHandle)h;
  }
  HandleRef* ref(YRTHandle h) {
    auto* r = (HandleRef*)h;
    if (!r || handles.find(r) == handles.end()) throw std::runtime_error("invalid handle");
    return r;
  }
  template <class T>
  std::shared_ptr<T> get(YRTHandle h, const char* what) {
    if (!h) return nullptr;
    auto o = std::dynamic_pointer_cast<T>(ref(h)->obj);
    if (!o) throw std::runtime_error(std::string("invalid ") + what + " handle");
    return o;
  }

  int* spill() { return ctx[0]->spill(); }

  // the committed scene as seen by one of the devices (a peer copy, refreshed after rebuilds
  // and refits; logical shards on the primary's own device share its buffers)
  // YRT_FORCE_SCENE_REPLICA=1 (tests): peer-copy the scene even onto the primary's own device,
  // so a one-GPU box exercises the replication path of multi-GPU renders
  GpuScene& scene_on(SceneObj& S, int dev, bool primary) {
    static const bool force = getenv("YRT_FORCE_SCENE_REPLICA") != nullptr;
    if (dev == S.gpu->device && (primary || !force)) return *S.gpu;
    auto& r = S.replicas[dev];
    if (!r || r->serial != S.gpu->serial || r->refits != S.gpu->refits) r = replicate_gpu_scene(*S.gpu, dev);
    return *r;
  }

  // one or several frames of the same size and format in one wavefront job (yrtRenderFrames):
  // their tiles form one sequence, frame-major, dealt over shards and devices
  void render(RendererObj& R, const std::vector<CameraObj*>& C, SceneObj& S, ToneMapperObj& T,
              const std::vector<FrameBufferObj*>& F, int accumulate);
  void render_shard(GpuCtx& g, GpuScene& G, RendererObj& R, const std::vector<CameraObj*>& C, ToneMapperObj& T,
                    int W, int H, int index, int count, int accumulate, bool reportProgress);
  int gather_local(const SlabLayout& base, int numTiles);
  // the render's output is this shard alone (no gather fills the other shards' tiles): those
  // pixels must read as zeros, so per-shard images compose by sum
  bool shardZero = true;
  // renderSeconds: this rank's render time of the call; the status exchange waits for the
  // slowest rank's render, so its deadline is gatherTimeout + kStatusRenderFactor x that time
  // (a peer may take ten times as long before the gather gives up; the slab transfers keep
  // gatherTimeout)
  static constexpr double kStatusRenderFactor = 10.0;
  void gather_process(const SlabLayout& base, int numTiles, bool localOk, double renderSeconds);
  // copies every unread frame held in block b into its framebuffer's host pixels
  void read_back_block(const void* b) {
    for (HandleRef* h : handles)
      if (auto* F = dynamic_cast<FrameBufferObj*>(h->obj.get()))
        for (int id = 0; id < (int)F->pending.size(); ++id)
          if (F->pending[id].keep.get() == b) fb_read_back(*F, id);
  }
  // a process gather is armed: every render of this device joins the ranks' status exchange
  bool proc_gather_armed() const {
    return proc && shardCount > 1 && shardIndex == commRank && shardCount == commWorld;
  }
  // A render call that fails before reaching render() (bad handles, host-only device) still
  // joins the status exchange with flag 0, so the peers fail instead of waiting for it.
  void fail_proc_gather() {
    if (!proc_gather_armed() || proc->aborted()) return;
    try {
      (void)proc->exchange_status(0, hipDevice, stream, gatherTimeout);
    } catch (...) {
    }
  }
  void intersect(SceneObj& S, const float* org4, const float* dir4, uint32_t n, float* hit4, int32_t* occ,
                 hipStream_t st);
};

// ---------------------------------------------------------------- rendering
static void status(RendererObj& R, int state, float progress) {
  if (R.statusCallback) ((YRTStatusCallback)R.statusCallback)(state, progress, R.statusUser);
}

// Copies the frame framebuffer F's buffer `id` still holds in HBM (FrameBufferObj::Pending)
// into its host pixels, converting float RGB to the RGBA / RGBA8 formats.
void fb_read_back(FrameBufferObj& F, int id) {
  if (id < 0 || id >= (int)F.pending.size() || !F.pending[id].keep) return;
  FrameBufferObj::Pending pf = F.pending[id];
  F.pending[id] = FrameBufferObj::Pending();
  HIP_CHECK(hipSetDevice(pf.hipDevice));
  const int W = F.width, H = F.height;
  void* dst = F.buffer(id);
  if (F.format == FB_RGB8) {
    HIP_CHECK(hipMemcpy(dst, pf.src, F.stride * H, hipMemcpyDeviceToHost));
    return;
  }
  if (F.format == FB_RGB_FLOAT32) {
    HIP_CHECK(hipMemcpy(dst, pf.src, (size_t)W * H * 3 * sizeof(float), hipMemcpyDeviceToHost));
    return;
  }
  std::vector<float> tmp((size_t)W * H * 3);
  HIP_CHECK(hipMemcpy(tmp.data(), pf.src, tmp.size() * sizeof(float), hipMemcpyDeviceToHost));
  if (F.format == FB_RGBA_FLOAT32) {
    float* o = (float*)dst;
    for (size_t i = 0; i < (size_t)W * H; ++i) {
      o[4 * i] = tmp[3 * i]; o[4 * i + 1] = tmp[3 * i + 1]; o[4 * i + 2] = tmp[3 * i + 2]; o[4 * i + 3] = 1.0f;
    }
  } else {  // RGBA8: pixel[3] = 0 (framebuffer.h:170-178)
    uint8_t* o = (uint8_t*)dst;
    for (size_t i = 0; i < (size_t)W * H; ++i) {
      for (int c = 0; c < 3; ++c) o[4 * i + c] = (uint8_t)clampf(tmp[3 * i + c] * 255.0f, 0.0f, 255.0f);
      o[4 * i + 3] = 0;
    }
  }
}

void Device::render(RendererObj& R, const std::vector<CameraObj*>& C, SceneObj& S, ToneMapperObj& T,
                    const std::vector<FrameBufferObj*>& F, int accumulate) {
  auto t0 = std::chrono::steady_clock::now();
  auto tRendered = t0;  // this process's tiles rendered (before any gather)
  // A process-level gather (yrtSetShardComm) is collective: every rank must reach it, so any
  // failure of this rank's part (arguments, scene, kernels) is reported to the peers through
  // the status exchange at its start instead of being thrown past it.
  const bool procGather = !R.debug && proc_gather_armed();
  const int nf = (int)F.size();
  const int W = nf ? F[0]->width : 0, H = nf ? F[0]->height : 0;
  const int tilesPerFrame = ((W + 15) / 16) * ((H + 15) / 16);
  const int numTiles = tilesPerFrame * nf;
  const bool rgb8 = nf && F[0]->format == FB_RGB8;
  SlabLayout base{W, H, (3 * W + 3) / 4 * 4, tilesPerFrame, 0, 1, rgb8 ? 1 : 0, 0};
  const int N = (int)ctx.size();
  // the debug renderer is a one-pass traversal KAT: the primary device renders every tile
  const int nr = R.debug ? 1 : N;
  std::string localErr;
  int gatherPath = YRT_GATHER_NONE;
  try {
    if (!S.gpu) throw std::runtime_error("scene not committed");
    if (S.gpu->device != hipDevice) throw std::runtime_error("scene committed on another HIP device");
    if (nf < 1 || (int)C.size() != nf) throw std::runtime_error("rtRenderFrames: one camera per framebuffer");
    for (const FrameBufferObj* f : F)
      if (f->width != W || f->height != H || f->format != F[0]->format)
        throw std::runtime_error("rtRenderFrames: framebuffers differ in size or format");
    if (R.debug && nf > 1) {
      // the debug renderer is a one-frame traversal KAT: its frames go one by one
      YRTRenderStats acc{};
      for (int k = 0; k < nf; ++k) {
        render(R, {C[k]}, S, T, {F[k]}, accumulate);
        acc.raysClosest += stats.raysClosest;
        acc.samples += stats.samples;
      }
      acc.msTotal = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      stats = acc;
      return;
    }
    memset(&stats, 0, sizeof(stats));
    if (!accumulate) R.iteration = 0;
    {
      // frames of an earlier job not yet read back: this job renders into another block. With
      // blk and spareBlk both holding unread frames a new block is allocated, up to
      // kMaxFrameBlocks alive; past that the block about to be reused is read back into its
      // framebuffers' host pixels first (rtMapFrameBuffer then finds them there), so frames
      // nobody maps cannot pin HBM without bound
      GpuCtx& g0 = *ctx[0];
      if (g0.blk.use_count() > 1) {
        std::swap(g0.blk, g0.spareBlk);
        if (!g0.blk || g0.blk.use_count() > 1) {
          auto& xb = g0.extraBlocks;
          xb.erase(std::remove_if(xb.begin(), xb.end(), [](const std::weak_ptr<GpuCtx::FrameBlock>& w) {
                     return w.expired();
                   }), xb.end());
          // blocks alive: blk, spareBlk and the extra ones (spareBlk is usually one of those)
          int live = (g0.blk ? 1 : 0) + (g0.spareBlk ? 1 : 0);
          for (const auto& w : xb) {
            const auto b = w.lock();
            live += b && b != g0.blk && b != g0.spareBlk;
          }
          if (g0.blk && live >= GpuCtx::kMaxFrameBlocks) {
            read_back_block(g0.blk.get());
          } else {
            g0.blk = std::make_shared<GpuCtx::FrameBlock>();
            xb.push_back(g0.blk);
          }
        }
      }
    }
    std::vector<GpuScene*> scenes(nr);
    for (int k = 0; k < nr; ++k) scenes[k] = &scene_on(S, ctx[k]->hipDevice, k == 0);
    // Without a process gather, the pixels of the other processes' shards (yrtSetTileShard)
    // must read as zeros so per-process images compose by sum: ctx[0]'s block is cleared
    // outside the tiles this call writes. With several devices in the process and no
    // process-level shard (shardCount 1), the local gather writes every tile: no clear.
    shardZero = !procGather && (nr == 1 || shardCount > 1);
    if (nr == 1) {
      render_shard(*ctx[0], *scenes[0], R, C, T, W, H, shardIndex, shardCount, accumulate, true);
      tRendered = std::chrono::steady_clock::now();
    } else {
      // device k of this process renders the tiles t = shardIndex + k * shardCount (mod shardCount * N)
      std::vector<std::string> errs(nr);
      std::vector<std::thread> th;
      for (int k = 0; k < nr; ++k)
        th.emplace_back([&, k] {
          try {
            render_shard(*ctx[k], *scenes[k], R, C, T, W, H, shardIndex + k * shardCount, shardCount * nr,
                         accumulate, k == 0);
          } catch (const std::exception& e) {
            errs[k] = e.what();
          }
        });
      for (auto& t : th) t.join();
      for (auto& e : errs)
        if (!e.empty()) throw std::runtime_error(e);
      tRendered = std::chrono::steady_clock::now();
      gatherPath = gather_local(base, numTiles);
    }
  } catch (const std::exception& e) {
    if (!procGather) throw;
    localErr = e.what();
  }
  if (procGather) {
    gather_process(base, numTiles, localErr.empty(),
                   std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    gatherPath = proc->kind()[0] == 'r' ? YRT_GATHER_RCCL_PROCESS : YRT_GATHER_HUB;
  }
  if (!localErr.empty()) throw std::runtime_error(localErr);
  R.iteration++;
  for (int k = 0; k < nr; ++k) {
    const YRTRenderStats& s = ctx[k]->stats;
    stats.raysClosest += s.raysClosest;
    stats.raysShadow += s.raysShadow;
    stats.launchesClosest += s.launchesClosest;
    stats.launchesShadow += s.launchesShadow;
    stats.msTraceClosest = std::max(stats.msTraceClosest, s.msTraceClosest);
    stats.msTraceShadow = std::max(stats.msTraceShadow, s.msTraceShadow);
    stats.msShade = std::max(stats.msShade, s.msShade);
  }

  // framebuffer write-back (api/framebuffer.h:93-226) from the primary device, frame by frame.
  // The other ranks of a process gather hold only their tiles: their host pixels are not
  // written (rank 0's framebuffers receive the gathered frames). A framebuffer with its own
  // host pixels keeps a reference to the frame in HBM instead, read back by rtMapFrameBuffer
  // (the reference's only access to the pixels, singleray_device.cpp:439-447): frames nobody
  // maps cross no PCIe.
  GpuCtx& g0 = *ctx[0];
  HIP_CHECK(hipSetDevice(g0.hipDevice));
  const size_t rgb8Stride = ((size_t)3 * W + 3) / 4 * 4;
  for (int k = 0; k < nf && !(procGather && shardIndex != 0); ++k) {
    FrameBufferObj& Fk = *F[k];
    FrameBufferObj::Pending pf;
    pf.keep = g0.blk;
    pf.src = Fk.format == FB_RGB8 ? (const void*)(g0.fbRGB8() + (size_t)k * rgb8Stride * H)
                                  : (const void*)(g0.fbFloat() + (size_t)k * W * H * 3);
    pf.hipDevice = g0.hipDevice;
    if ((int)Fk.pending.size() < Fk.depth) Fk.pending.resize(Fk.depth);
    Fk.pending[Fk.cur] = pf;
    if (!Fk.userPtrs.empty()) fb_read_back(Fk, Fk.cur);
  }
  stats.samples = ctx[0]->stats.samples;
  stats.gather = gatherPath;
  const auto tEnd = std::chrono::steady_clock::now();
  if (tRendered == t0) tRendered = tEnd;  // the render threw before its end (collective error path)
  stats.msTotal = std::chrono::duration<double, std::milli>(tEnd - t0).count();
  stats.msRender = std::chrono::duration<double, std::milli>(tRendered - t0).count();
  stats.msGather = std::chrono::duration<double, std::milli>(tEnd - tRendered).count();
  status(R, 2, 1.f);
}

// Renders the tiles of shard (index, count) of the frame into g's full-size buffers (the other
// tiles' pixels are left zero when count > 1).
void Device::render_shard(GpuCtx& g, GpuScene& G, RendererObj& R, const std::vector<CameraObj*>& C,
                          ToneMapperObj& T, int W, int H, int index, int count, int accumulate, bool reportProgress) {
  const int nf = (int)C.size();
  HIP_CHECK(hipSetDevice(g.hipDevice));
  memset(&g.stats, 0, sizeof(g.stats));
  SceneView sv = G.view;
  sv.traceSpill = g.spill();
  const hipStream_t stream = g.stream;

  GpuRenderParams rp;
  memset(&rp, 0, sizeof(rp));
  rp.width = W;
  rp.height = H;
  rp.numTilesX = (W + 15) / 16;
  rp.numTilesY = (H + 15) / 16;
  rp.rcpWidth = rcpf_(float(W));
  rp.rcpHeight = rcpf_(float(H));
  rp.gamma = T.gamma;
  rp.rcpGamma = rcpf_(T.gamma);
  rp.frameSeed = frameSeed;
  rp.maxDepth = R.maxDepth;
  rp.rrDepth = R.rrDepth;
  rp.minContribution = R.minContribution;
  rp.epsilon = R.epsilon;
  rp.tMaxShadowRay = R.tMaxShadowRay;
  rp.tMaxShadowJitter = R.tMaxShadowJitter;
  rp.up[0] = R.up.x; rp.up[1] = R.up.y; rp.up[2] = R.up.z;
  rp.numLights = G.view.numLights;
  rp.numEnvLights = G.view.numEnvLights;
  rp.numPrecomp = (int)G.precomputed.size();
  rp.numFrames = nf;
  rp.tilesPerFrame = rp.numTilesX * rp.numTilesY;
  rp.divTilesX = fastdiv_make((uint32_t)rp.numTilesX);
  rp.divTilesPerFrame = fastdiv_make((uint32_t)rp.tilesPerFrame);

  // samples: PathTraceIntegrator::requestSamples (pathtraceintegrator.cpp:35-47)
  SampleRequest req;
  req.spp = R.debug ? 1 : R.spp;
  req.sets = R.sets;
  req.iteration = R.iteration;
  req.num1D = R.debug ? 0 : R.maxDepth;
  req.num2D = R.debug ? 0 : 1 + R.maxDepth;
  req.filter = R.filter;
  if (!R.debug) req.lights = G.precomputed;
  rp.dim1D = req.num1D;
  rp.dim2D = req.num2D;
  rp.lightSampleID = 0;
  rp.firstScatterSampleID = 1;
  rp.firstScatterTypeSampleID = 0;
  char keybuf[256];
  snprintf(keybuf, sizeof(keybuf), "%d/%d/%d/%d/%d/%s/%llu", req.spp, req.sets, req.iteration, req.num1D, req.num2D,
           req.filter.c_str(), (unsigned long long)G.serial);
  auto fit = g.fcaches.find(keybuf);
  if (fit == g.fcaches.end()) {
    if (g.fcaches.size() >= GpuCtx::kMaxFrameCaches) {
      g.fcaches.erase(g.fcacheOrder.front());
      g.fcacheOrder.pop_front();
    }
    auto fc = std::make_unique<FrameCache>();
    build_sample_table(req, fc->table);
    const SampleTable& t = fc->table;
    fc->slotLive.assign(t.numLightSlots, 0);
    for (int r = 0; r < t.numRecords; ++r)
      for (int k = 0; k < t.numLightSlots; ++k) {
        const float* ls = &t.light[((size_t)r * t.numLightSlots + k) * 8];
        if (!(ls[4] == 0.f && ls[5] == 0.f && ls[6] == 0.f)) fc->slotLive[k] = 1;
      }
    fc->dims.upload(fc->table.dims);
    fc->light.upload(fc->table.light);
    fc->key = keybuf;
    g.fcacheOrder.push_back(keybuf);
    fit = g.fcaches.emplace(keybuf, std::move(fc)).first;
  }
  FrameCache& fcache = *fit->second;
  const SampleTable& tab = fcache.table;
  rp.spp = tab.spp;
  rp.sets = tab.sets;
  // direct lighting (pathtraceintegrator.cpp:123-167) skips a light whose sample radiance is
  // exactly 0 for every sample of the frame (a zero L, e.g. C4's HDRILight L = 0 0 0): its
  // shadow ray is never cast, so dropping it from the loop changes no pixel, and a frame left
  // with one such light fuses the shadow resolve into the any-hit kernel. The loop keeps the
  // lights' own indices (shadow jitter hash, light order).
  g.hDirect.clear();
  for (int li = 0; li < (int)G.hLights.size(); ++li) {
    const GpuLight& lt = G.hLights[li];
    const bool live = lt.precomputed >= 0 ? (lt.precomputed < (int)fcache.slotLive.size() && fcache.slotLive[lt.precomputed])
                                          : !(lt.L[0] == 0.f && lt.L[1] == 0.f && lt.L[2] == 0.f);
    if (live || getenv("YRT_ALL_DIRECT_LIGHTS")) g.hDirect.push_back(li);
  }
  g.dDirect.alloc(sizeof(int) * std::max<size_t>(1, g.hDirect.size()));
  if (!g.hDirect.empty())
    HIP_CHECK(hipMemcpyAsync(g.dDirect.p, g.hDirect.data(), sizeof(int) * g.hDirect.size(), hipMemcpyHostToDevice,
                             stream));
  sv.directLights = g.dDirect.as<int>();
  sv.numDirectLights = (int)g.hDirect.size();
  const int numDirect = sv.numDirectLights;

  // a fused depth 0's miss radiance (PrimaryRays)
  for (int k = 0; k < 4; ++k) rp.missL[k] = 0.f;
  for (int j : G.hEnvLights) {
    const float* Le = G.hLights[j].L;
    for (int k = 0; k < 3; ++k) rp.missL[k] = rp.missL[k] + 1.0f * Le[k];
  }
  g.dRp.alloc(sizeof(rp));
  g.hCams.resize(nf);
  for (int k = 0; k < nf; ++k) g.hCams[k] = C[k]->cam;
  g.dCam.alloc(sizeof(GpuCamera) * nf);
  HIP_CHECK(hipMemcpyAsync(g.dRp.p, &rp, sizeof(rp), hipMemcpyHostToDevice, stream));
  HIP_CHECK(hipMemcpyAsync(g.dCam.p, g.hCams.data(), sizeof(GpuCamera) * nf, hipMemcpyHostToDevice, stream));
  g.dPixelSets.alloc((size_t)W * H);
  const size_t rgb8Stride = ((size_t)3 * W + 3) / 4 * 4;
  GpuCtx::FrameBlock& B = *g.blk;
  const void* const oldF = B.fbFloat.p;
  const void* const oldB = B.fbRGB8.p;
  B.fbFloat.alloc((size_t)nf * W * H * 3 * sizeof(float));
  B.fbRGB8.alloc((size_t)nf * rgb8Stride * H);
  const long long zkey[5] = {index, count, W, H, nf};
  if (B.fbFloat.p != oldF || B.fbRGB8.p != oldB) B.zeroKey[0] = -1;
  if (count > 1 && shardZero && &g == ctx[0].get() && !R.debug) {
    // pixels of other shards stay 0 so per-shard images compose by sum; a block that already
    // holds this layout's zeros (the same shard rendered into it before) is not cleared again.
    // Only ctx[0]'s block is output: the other devices of the process send their tiles to it.
    // Their (index, count) = (shardIndex, shardCount·N) identify the process's layout, since N
    // is fixed per Device (the debug renderer, which renders on ctx[0] alone, resets the key).
    if (memcmp(B.zeroKey, zkey, sizeof(zkey)) != 0) {
      HIP_CHECK(hipMemsetAsync(B.fbFloat.p, 0, (size_t)nf * W * H * 3 * sizeof(float), stream));
      HIP_CHECK(hipMemsetAsync(B.fbRGB8.p, 0, (size_t)nf * rgb8Stride * H, stream));
      memcpy(B.zeroKey, zkey, sizeof(zkey));
    }
  } else {
    B.zeroKey[0] = -1;  // every tile gets written (one shard, the gather, the debug renderer)
  }

  FrameView fv;
  fv.rp = g.dRp.as<GpuRenderParams>();
  fv.cam = g.dCam.as<GpuCamera>();
  fv.samples = fcache.dims.as<float>();
  fv.lightSamples = fcache.light.as<float>();
  fv.pixelSets = g.dPixelSets.as<uint8_t>();
  fv.numRecords = tab.numRecords;
  fv.numLightSlots = std::max(1, tab.numLightSlots);
  memset(&fv.backplate, 0, sizeof(fv.backplate));
  fv.backplateTexels = nullptr;
  if (R.backplate && !R.debug) {
    const ImageObj& im = *R.backplate;
    if (g.backplateSerial != im.serial) {
      g.dBackplate.upload(im.data);
      g.backplateSerial = im.serial;
    }
    fv.backplate.width = im.width;
    fv.backplate.height = im.height;
    fv.backplate.format = im.format;
    fv.backplate.offset = 0;
    fv.backplateTexels = g.dBackplate.as<uint8_t>();
  }

  if (reportProgress) status(R, 1, 0.f);
  const int numTiles = rp.tilesPerFrame * nf;
  const int shardTiles = shard_tiles(numTiles, index, count);

  if (R.debug) {
    launch_debug_render(sv, fv, R.maxDepth, R.spp, numTiles, g.fbFloat(), g.fbRGB8(),
                        (int)rgb8Stride, stream);
  } else {
    if (g.pixelSetsKey[0] != W || g.pixelSetsKey[1] != H || g.pixelSetsKey[2] != rp.sets) {
      launch_pixel_sets(fv, g.dPixelSets.as<uint8_t>(), W, H, rp.sets, stream);
      g.pixelSetsKey[0] = W;
      g.pixelSetsKey[1] = H;
      g.pixelSetsKey[2] = rp.sets;
    }
    g.capClosest.clear();
    g.capShadow.clear();
    const int spp = rp.spp;
    int64_t tilesPerBatch = std::max<int64_t>(1, capacity / (256ll * spp));
    // a multiple of the lanes in batches (evenly sized), so both lanes have work even when a
    // shard of the frame fits one batch (multi-GPU shards, small frames)
    if (captureMax == 0 && g.numLanes > 1 && shardTiles > 1) {
      int64_t nb = (shardTiles + tilesPerBatch - 1) / tilesPerBatch;
      nb = (nb + g.numLanes - 1) / g.numLanes * g.numLanes;
      // At the default capacity, a lane that would run 5-8 batches runs half as many of twice
      // the size: each batch pays a fixed chain of 10 depths x 3 launches and a ramp-down, which
      // outweighs the overlap the extra batches buy there (C4 N = 8 rank share 51.0 -> 48.7 ms;
      // at 27+ batches per lane, N = 1 / 2, twice the size measured +1 / +4 %,
      // profiles/r04/ab_r04k.txt, scaling_prediction_c4_r04z.txt). YRT_BATCH_GROW=0: off.
      const bool grow = capacity == ((int64_t)YRT_DEFAULT_CAPACITY_M << 20) &&
                        !(getenv("YRT_BATCH_GROW") && atoi(getenv("YRT_BATCH_GROW")) == 0);
      if (grow && nb > 4 * g.numLanes && nb <= 8 * g.numLanes) {
        nb = (nb / 2 + g.numLanes - 1) / g.numLanes * g.numLanes;
      } else if (grow && nb > 8 * g.numLanes && nb <= 16 * g.numLanes) {
        // 9-16 per lane: 1.5x the size (C4 N = 4 share, 96 M paths: 100 -> 95 ms, ab_r04k.txt)
        nb = (nb * 2 / 3 + g.numLanes - 1) / g.numLanes * g.numLanes;
      }
      tilesPerBatch = (shardTiles + nb - 1) / nb;
    }
    const int64_t P = std::min<int64_t>(tilesPerBatch, shardTiles) * 256 * spp;
    const int64_t numBatches = (shardTiles + tilesPerBatch - 1) / tilesPerBatch;
    // the capture frame (roofline accounting) reads batch 0's queues synchronously: one lane
    const int nl = captureMax > 0 ? 1 : (int)std::max<int64_t>(1, std::min<int64_t>(g.numLanes, numBatches));
    const int levels = rp.maxDepth + 1;
    // the queue counters, then one word: the camera rays a fused depth 0 traced
    // (PrimaryRays::traced)
    const size_t counterWords = qcounter_words(levels) + 1;
    const size_t tracedWord = counterWords - 1;
    g.dAccu.alloc((size_t)nf * W * H * 16);
    g.ensure_streams(nl);
    for (int l = 0; l < nl; ++l) {
      GpuCtx::Lane& L = g.lanes[l];
      GpuCtx::ensure_paths(L, std::max<int64_t>(P, 256ll * spp), numDirect, G.hasMotion);
      L.counters.alloc(counterWords * sizeof(unsigned));
      L.spill.alloc(YRT_TRACE_SPILL_INTS * sizeof(int));
      for (GpuCtx::Lane::Pend& Pd : L.pend) {
        if (Pd.hcWords < counterWords) {
          if (Pd.hc) HIP_CHECK(hipHostFree(Pd.hc));
          Pd.hc = nullptr;
          Pd.hcWords = 0;
          HIP_CHECK(hipHostMalloc((void**)&Pd.hc, counterWords * sizeof(unsigned), hipHostMallocDefault));
          Pd.hcWords = counterWords;
        }
        if (!Pd.done) HIP_CHECK(hipEventCreateWithFlags(&Pd.done, hipEventDisableTiming));
      }
      L.pendHead = L.pendCount = 0;
    }
    // the other lanes start after the frame setup enqueued on lane 0 (uploads, pixel sets)
    if (nl > 1) {
      hipEvent_t setup = g.ev();
      HIP_CHECK(hipEventRecord(setup, stream));
      for (int l = 1; l < nl; ++l) HIP_CHECK(hipStreamWaitEvent(g.lanes[l].stream, setup, 0));
    }
    auto lane_buffers = [&](GpuCtx::Lane& L) {
      PathBuffers pb;
      for (int k = 0; k < 2; ++k) {
        pb.qPath[k] = L.qPath[k].as<int>();
        pb.qOrg[k] = L.qOrg[k].as<float4>();
        pb.qDir[k] = L.qDir[k].as<float4>();
        pb.qThr[k] = L.qThr[k].as<float4>();
      }
      pb.hit = L.hit.as<float4>();
      pb.hitGeom = L.hitGeom.as<int>();
      pb.pathL = L.pathL.as<float4>();
      pb.shFirst = L.shFirst.as<int>();
      pb.sOrg = L.sOrg.as<float4>();
      pb.sDir = L.sDir.as<float4>();
      pb.sContrib = L.sContrib.as<float4>();
      pb.sOcc = L.sOcc.as<int>();
      pb.counters = L.counters.as<unsigned>();
      for (int k = 0; k < 2; ++k) pb.qTime[k] = G.hasMotion ? L.qTime[k].as<float>() : nullptr;
      pb.sTime = G.hasMotion ? L.sTime.as<float>() : nullptr;
      pb.capacity = (int)std::max<int64_t>(P, 256ll * spp);
      pb.segCap = qseg_capacity(pb.capacity);
      pb.shSegCap = pb.segCap * std::max(1, numDirect);
      // one light: shadow contributions are added by k_trace<true> itself (no resolve pass)
      pb.fuseShadow = numDirect == 1 && !getenv("YRT_NO_SHADOW_FUSE");
      return pb;
    };
    auto mit = g.missFrac.find(G.serial);
    double missEst = mit == g.missFrac.end() ? -1.0 : mit->second.first / mit->second.second;
    // accounts the queue counters of the lane's oldest pending batch; without `wait` only if
    // the batch's counters have arrived (returns whether it accounted one)
    int64_t tilesDone = 0;
    auto drain_one = [&](GpuCtx::Lane& L, bool wait) -> bool {
      if (L.pendCount == 0) return false;
      GpuCtx::Lane::Pend& Pd = L.pend[L.pendHead];
      if (wait) {
        HIP_CHECK(hipEventSynchronize(Pd.done));
      } else {
        const hipError_t q = hipEventQuery(Pd.done);
        if (q == hipErrorNotReady) return false;
        HIP_CHECK(q);
      }
      for (int d = 0; d < levels; ++d) {
        double nc = 0, ns = 0;
        for (int k = 0; k < YRT_QSEGS; ++k) {
          nc += Pd.hc[qcounter_index(d, 0, k)];
          ns += Pd.hc[qcounter_index(d, 1, k)];
        }
        if (d == 0 && Pd.fused && Pd.hc[tracedWord] > 0) {
          if (g.missFrac.size() > 64 && !g.missFrac.count(G.serial)) g.missFrac.clear();
          auto& acc = g.missFrac[G.serial];
          acc.first += (double)Pd.hc[tracedWord] - nc;  // a fused depth 0 queues its hits only
          acc.second += (double)Pd.hc[tracedWord];
          missEst = acc.first / acc.second;
        }
        if (d < rp.maxDepth) {  // level maxDepth counts continuations that are never traced
          // a fused depth 0 queues its hits only: the camera rays it traced are counted apart
          const double traced = d == 0 && Pd.fused ? (double)Pd.hc[tracedWord] : nc;
          g.stats.raysClosest += traced;
          if (traced) g.stats.launchesClosest += 1;
        }
        g.stats.raysShadow += ns;
        if (d < rp.maxDepth && ns) g.stats.launchesShadow += 1;
      }
      L.pendHead = (L.pendHead + 1) % GpuCtx::Lane::kPendDepth;
      L.pendCount -= 1;
      tilesDone += Pd.tiles;
      if (reportProgress) status(R, 1, float(tilesDone) / float(std::max(1, shardTiles)));
      return true;
    };

    struct EvPair { hipEvent_t a, b; int kind; };
    std::vector<EvPair> evs;
    int64_t batch = 0;
    // Depth 0 as one kernel (launch_trace_primary): camera rays generated inside the closest-hit
    // trace, misses resolved there, only hits queued for k_shade — for static scenes whose
    // depth-0 miss radiance is a constant: no backplate, every environment light ambient
    // (k_shade's miss branch then adds thr * L = L per light in envLights order, thr = 1).
    // Not in the capture frame (it copies the depth-0 queue). It pays where camera rays miss
    // (C4: cube job -11 %, -1.3 % more at 96 VGPRs / 5 waves since round 5) and costs where they
    // hit (C3 -2.5 %, C5 -1.3 %: its hits are appended in completion order, profiles/r04/
    // ab_r04d.txt; a path-ordered "identity" layout measured no better, profiles/r05/
    // ab_prim_r05j.txt), so a batch is fused while the scene's measured miss share (missFrac, over
    // its fused batches so far) is at least YRT_PRIMARY_MISS (default 0.5) or unknown.
    // YRT_PRIMARY=0: never, 2: always.
    const int primMode = getenv("YRT_PRIMARY") ? atoi(getenv("YRT_PRIMARY")) : 1;
    const double primMiss = getenv("YRT_PRIMARY_MISS") ? atof(getenv("YRT_PRIMARY_MISS")) : 0.5;
    // Toe-in stereo cameras (the DLL's FPR default) are left to k_raygen: the fused kernel is
    // compiled without that branch (camera_ray<false>, pathtrace.hip).
    bool toeIn = false;
    for (const GpuCamera& c : g.hCams) toeIn |= c.type == CAM_STEREO && c.toeIn != 0;
    const bool fusedPrimary = captureMax == 0 && !G.hasMotion && !fv.backplateTexels && sv.numEnvDir == 0 &&
                              primMode != 0 && !toeIn;
    // A lane's batch is enqueued a step at a time — its prologue (counter clear, camera rays),
    // one depth (closest trace, shade, shadow trace), its epilogue (counter copy, pixel resolve)
    // — round-robin over the lanes that hold a batch, so every lane's first kernels are queued
    // within a few launches of the job's start. A whole batch at a time (≈ 33 launches at
    // ≈ 58 µs of host time each), lane k started k × 1.9 ms after lane 0 and the job's end waited
    // as long for the last lane (C3 N = 8 share: lanes starting 0 / 1.1 / 3.1 / 5.1 ms into a
    // 52.7 ms job, profiles/r05/timeline_c3_n8_r05v.txt). A lane takes its next batch once its
    // previous batch's counters have arrived (Pend); the batch goes to the first such lane, so a
    // lane that finishes early is refilled at once (lanes in turn: C4 N = 3 rank share 160 ms,
    // profiles/r04/ab_r04i.txt). When every lane is full the host blocks on the batch enqueued
    // first (hipEventSynchronize) instead of spinning a core.
    struct LaneJob {
      bool active = false;
      int step = 0;  // 0: prologue, 1..maxDepth: depth step - 1, maxDepth + 1: epilogue
      int64_t first = 0, seq = 0;
      BatchInfo bi{};
      bool fused = false;
    };
    std::vector<LaneJob> jobs(nl);
    int64_t nextFirst = 0;  // the next batch's first tile of the shard
    auto enqueue_step = [&](GpuCtx::Lane& L, LaneJob& J) {
      const hipStream_t st = L.stream;
      const PathBuffers pb = lane_buffers(L);
      SceneView lsv = sv;
      lsv.traceSpill = L.spill.as<int>();
      const BatchInfo& bi = J.bi;
      if (J.step == 0) {
        HIP_CHECK(hipMemsetAsync(L.counters.p, 0, counterWords * sizeof(unsigned), st));
        if (!J.fused) launch_raygen(fv, pb, bi, st);
      } else if (J.step <= rp.maxDepth) {
        const int d = J.step - 1;
        const int cur = d & 1;
        EvPair e1{};
        if (kernelTiming) { e1 = {g.ev(), g.ev(), 0}; HIP_CHECK(hipEventRecord(e1.a, st)); }
        if (d == 0 && J.fused) {
          PrimaryRays pr;
          pr.fv = fv;
          pr.bi = bi;
          pr.qPath = pb.qPath[0];
          pr.qOrg = pb.qOrg[0];
          pr.qDir = pb.qDir[0];
          pr.pathL = pb.pathL;
          pr.counts = pb.counters + qcounter_index(0, 0, 0);
          pr.segCap = pb.segCap;
          pr.traced = pb.counters + tracedWord;
          pr.numPaths = (long long)bi.numPixels * spp;
          launch_trace_primary(lsv, pr, pb.hit, pb.hitGeom, st);
        } else {
          launch_trace_closest(lsv, pb.qOrg[cur], pb.qDir[cur], pb.counters + qcounter_index(d, 0, 0), YRT_QSEGS,
                               pb.segCap, pb.hit, st, pb.qTime[cur], pb.hitGeom);
        }
        if (kernelTiming) { HIP_CHECK(hipEventRecord(e1.b, st)); evs.push_back(e1); }
        if (captureMax > 0 && J.first == 0)
          g.capture(captureMax, g.capClosest, d, pb.qOrg[cur], pb.qDir[cur], pb.counters + qcounter_index(d, 0, 0),
                    pb.segCap, st);
        EvPair e2{};
        if (kernelTiming) { e2 = {g.ev(), g.ev(), 2}; HIP_CHECK(hipEventRecord(e2.a, st)); }
        launch_shade(lsv, fv, pb, bi, d, G.materialMask, st);
        if (kernelTiming) { HIP_CHECK(hipEventRecord(e2.b, st)); evs.push_back(e2); }
        if (numDirect > 0) {
          EvPair e3{};
          if (kernelTiming) { e3 = {g.ev(), g.ev(), 1}; HIP_CHECK(hipEventRecord(e3.a, st)); }
          const ShadowFuse sf{pb.fuseShadow ? pb.sContrib : nullptr, pb.pathL};
          launch_trace_any(lsv, pb.sOrg, pb.sDir, pb.counters + qcounter_index(d, 1, 0), YRT_QSEGS, pb.shSegCap,
                           pb.sOcc, st, &sf, pb.sTime);
          if (kernelTiming) { HIP_CHECK(hipEventRecord(e3.b, st)); evs.push_back(e3); }
          if (captureMax > 0 && J.first == 0)
            g.capture(captureMax, g.capShadow, d, pb.sOrg, pb.sDir, pb.counters + qcounter_index(d, 1, 0),
                      pb.shSegCap, st);
          if (!pb.fuseShadow) launch_shadow_resolve(pb, d, numDirect, st);
        }
      } else {
        // the counters are final after the last trace: their copy runs before the pixel resolve,
        // so the host learns the batch's queue sizes while the resolve still runs
        GpuCtx::Lane::Pend& Pd = L.pend[(L.pendHead + L.pendCount) % GpuCtx::Lane::kPendDepth];
        HIP_CHECK(hipMemcpyAsync(Pd.hc, L.counters.p, counterWords * sizeof(unsigned), hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipEventRecord(Pd.done, st));
        Pd.tiles = bi.numPixels / 256;
        Pd.fused = J.fused;
        Pd.seq = J.seq;
        L.pendCount += 1;
        launch_resolve_pixels(fv, pb, bi, g.fbFloat(), g.fbRGB8(), (int)rgb8Stride, g.dAccu.as<float4>(),
                              accumulate ? 1 : 0, st);
        J.active = false;
      }
      J.step += 1;
    };
    for (;;) {
      if (R.stopFlag && R.stopFlag->load()) nextFirst = shardTiles;  // no new batches
      for (int l = 0; l < nl; ++l)
        while (drain_one(g.lanes[l], false)) {}
      for (int l = 0; l < nl && nextFirst < shardTiles; ++l) {
        LaneJob& J = jobs[l];
        if (J.active || g.lanes[l].pendCount >= GpuCtx::Lane::kPendDepth) continue;
        J = LaneJob{};
        J.active = true;
        J.seq = batch++;
        const int64_t batchTiles = std::min<int64_t>(tilesPerBatch, shardTiles - nextFirst);
        J.first = nextFirst;
        J.bi.firstTile = (int)nextFirst;
        J.bi.tileStride = count;
        J.bi.tileOffset = index;
        nextFirst += batchTiles;
        J.bi.numPixels = (int)(batchTiles * 256);
        J.bi.divPixels = fastdiv_make((uint32_t)J.bi.numPixels);
        // fused (hits queued) while camera rays mostly miss, k_raygen + the queued trace otherwise
        J.fused = fusedPrimary && (primMode == 2 || (primMode == 1 && (missEst < 0 || missEst >= primMiss)));
      }
      bool enqueued = false;
      for (int l = 0; l < nl; ++l)
        if (jobs[l].active) {
          enqueue_step(g.lanes[l], jobs[l]);
          enqueued = true;
        }
      if (enqueued) continue;
      if (nextFirst >= shardTiles) break;  // every batch enqueued
      // every lane holds a batch whose counters have not arrived: wait for the oldest
      int oldest = 0;
      for (int l = 1; l < nl; ++l)
        if (g.lanes[l].pend[g.lanes[l].pendHead].seq < g.lanes[oldest].pend[g.lanes[oldest].pendHead].seq) oldest = l;
      drain_one(g.lanes[oldest], true);
    }
    for (int l = 0; l < nl; ++l)
      while (drain_one(g.lanes[l], true)) {}
    for (auto& e : evs) {
      float ms = 0;
      HIP_CHECK(hipEventElapsedTime(&ms, e.a, e.b));
      if (e.kind == 0) g.stats.msTraceClosest += ms;
      else if (e.kind == 1) g.stats.msTraceShadow += ms;
      else g.stats.msShade += ms;
    }
    for (auto e : g.eventPool) (void)hipEventDestroy(e);
    g.eventPool.clear();
  }
  for (int l = 0; l < GpuCtx::kMaxLanes; ++l)
    if (g.lanes[l].stream) HIP_CHECK(hipStreamSynchronize(g.lanes[l].stream));
  g.stats.samples = (double)nf * W * H * (R.debug ? 1 : rp.spp);
}

// The ctx devices' shards onto ctx[0]: every peer packs its tiles into a slab, the slabs go to
// the first device (RCCL grouped send/recv when the devices are distinct GPUs — one xGMI link
// per peer; hipMemcpyPeerAsync when ncclCommInitAll is unavailable; a device-to-device copy
// when logical shards share a GPU) and are unpacked there. Every wait is bounded by
// gatherTimeout; a timed-out RCCL gather aborts the communicators and later frames use peer
// copies. Returns the YRT_GATHER_* path taken.
int Device::gather_local(const SlabLayout& base, int numTiles) {
  const int N = (int)ctx.size();
  bool distinct = true;
  for (int a = 0; a < N; ++a)
    for (int b = a + 1; b < N; ++b) distinct &= ctx[a]->hipDevice != ctx[b]->hipDevice;
  GpuCtx& g0 = *ctx[0];
  const size_t eb = slab_element_bytes(base.rgb8);
  std::vector<int> tiles(N);
  std::vector<SlabLayout> lay(N, base);
  for (int k = 1; k < N; ++k) {
    GpuCtx& g = *ctx[k];
    lay[k].tileOffset = shardIndex + k * shardCount;
    lay[k].tileStride = shardCount * N;
    tiles[k] = shard_tiles(numTiles, lay[k].tileOffset, lay[k].tileStride);
    HIP_CHECK(hipSetDevice(g.hipDevice));
    g.dSlab.alloc((size_t)std::max(1, tiles[k]) * 256 * eb);
    launch_pack_tiles(g.fbFloat(), g.fbRGB8(), lay[k], tiles[k], g.dSlab.p, g.stream);
    HIP_CHECK(hipSetDevice(g0.hipDevice));
    g0.recvSlabs[k].alloc((size_t)std::max(1, tiles[k]) * 256 * eb);
  }
  const Clock::time_point deadline =
      Clock::now() + std::chrono::microseconds((long long)(gatherTimeout * 1e6));
  auto wait_ctx = [&](int k, const char* phase) {
    HIP_CHECK(hipSetDevice(ctx[k]->hipDevice));
    if (!stream_wait_until(ctx[k]->stream, deadline))
      throw std::runtime_error(std::string("multi-GPU gather: ") + phase + " on HIP device " +
                               std::to_string(ctx[k]->hipDevice) + " timed out after " +
                               std::to_string(gatherTimeout) + " s");
  };
  int path = distinct ? YRT_GATHER_RCCL_LOCAL : YRT_GATHER_D2D;
  if (distinct && !localRcclOff && !localComm) {
    try {
      const RcclApi& nc = rccl();
      std::vector<int> devs;
      for (auto& g : ctx) devs.push_back(g->hipDevice);
      std::vector<ncclComm_t> comms(N);
      rccl_check(nc.CommInitAll(comms.data(), N, devs.data()), "ncclCommInitAll");
      localComms.assign(comms.begin(), comms.end());
      localComm = comms[0];
    } catch (const std::exception& e) {
      localRcclOff = true;
      localRcclWhy = e.what();
      fprintf(stderr, "yrt: %s; the multi-GPU gather uses hipMemcpyPeerAsync instead\n", e.what());
    }
  }
  if (distinct && localRcclOff) path = YRT_GATHER_PEER_COPY;
  if (path == YRT_GATHER_RCCL_LOCAL) {
    const RcclApi& nc = rccl();
    rccl_check(nc.GroupStart(), "ncclGroupStart");
    for (int k = 1; k < N; ++k) {
      const size_t bytes = (size_t)tiles[k] * 256 * eb;
      if (!bytes) continue;
      rccl_check(nc.Send(ctx[k]->dSlab.p, bytes, ncclUint8, 0, localComms[k], ctx[k]->stream), "ncclSend");
      rccl_check(nc.Recv(g0.recvSlabs[k].p, bytes, ncclUint8, k, localComms[0], g0.stream), "ncclRecv");
    }
    rccl_check(nc.GroupEnd(), "ncclGroupEnd");
  } else {
    for (int k = 1; k < N; ++k) {
      wait_ctx(k, "tile pack");
      const size_t bytes = (size_t)tiles[k] * 256 * eb;
      if (bytes)
        HIP_CHECK(hipMemcpyPeerAsync(g0.recvSlabs[k].p, g0.hipDevice, ctx[k]->dSlab.p, ctx[k]->hipDevice, bytes,
                                     g0.stream));
    }
  }
  HIP_CHECK(hipSetDevice(g0.hipDevice));
  for (int k = 1; k < N; ++k)
    launch_unpack_tiles(g0.recvSlabs[k].p, g0.fbFloat(), g0.fbRGB8(), lay[k], tiles[k],
                        g0.stream);
  try {
    for (int k = 0; k < N; ++k) wait_ctx(k, path == YRT_GATHER_RCCL_LOCAL ? "RCCL slab send/recv" : "slab copy");
  } catch (...) {
    if (path == YRT_GATHER_RCCL_LOCAL) {
      // the communicators may hold a send/recv that never matches: abort them and gather with
      // peer copies from now on
      try {
        const RcclApi& nc = rccl();
        for (auto c : localComms) (nc.CommAbort ? nc.CommAbort : nc.CommDestroy)(c);
      } catch (...) {
      }
      localComms.clear();
      localComm = nullptr;
      localRcclOff = true;
      localRcclWhy = "an RCCL gather timed out";
    }
    throw;
  }
  HIP_CHECK(hipSetDevice(g0.hipDevice));
  return path;
}

// This process's tiles (shard shardIndex of shardCount, already gathered on ctx[0]) to rank 0
// of the process transport (gather.h: RCCL, yrtSetShardComm, or the in-process hub,
// yrtSetShardHub): the ranks first exchange their render status (the min of every rank's
// flag, so a rank whose render failed makes every rank fail instead of leaving rank 0 waiting
// for its slab), then every rank packs its tiles and rank 0 receives each peer's slab and
// unpacks it into its frames. Every wait is bounded: the status exchange by gatherTimeout plus
// kStatusRenderFactor times this rank's render time, the transfers by gatherTimeout.
void Device::gather_process(const SlabLayout& base, int numTiles, bool localOk, double renderSeconds) {
  GpuCtx& g0 = *ctx[0];
  HIP_CHECK(hipSetDevice(g0.hipDevice));
  const int P = shardCount;
  const int flag = proc->exchange_status(localOk ? 1 : 0, g0.hipDevice, g0.stream,
                                         gatherTimeout + kStatusRenderFactor * std::max(0.0, renderSeconds));
  if (!flag) {
    if (localOk) throw std::runtime_error("rtRenderFrame: a peer rank's render failed (no frame gathered)");
    return;  // the caller rethrows this rank's own error
  }
  const size_t eb = slab_element_bytes(base.rgb8);
  SlabLayout L = base;
  L.tileStride = P;
  if (shardIndex != 0) {
    L.tileOffset = shardIndex;
    const int tiles = shard_tiles(numTiles, shardIndex, P);
    g0.dSlab.alloc((size_t)std::max(1, tiles) * 256 * eb);
    launch_pack_tiles(g0.fbFloat(), g0.fbRGB8(), L, tiles, g0.dSlab.p, g0.stream);
    proc->send_root(g0.dSlab.p, (size_t)tiles * 256 * eb, g0.hipDevice, g0.stream, gatherTimeout);
  } else {
    std::vector<int> tiles(P);
    std::vector<void*> bufs(P, nullptr);
    std::vector<size_t> bytes(P, 0);
    for (int r = 1; r < P; ++r) {
      tiles[r] = shard_tiles(numTiles, r, P);
      g0.recvSlabs[r].alloc((size_t)std::max(1, tiles[r]) * 256 * eb);
      bufs[r] = g0.recvSlabs[r].p;
      bytes[r] = (size_t)tiles[r] * 256 * eb;
    }
    proc->recv_all(bufs, bytes, g0.hipDevice, g0.stream, gatherTimeout);
    for (int r = 1; r < P; ++r) {
      L.tileOffset = r;
      launch_unpack_tiles(g0.recvSlabs[r].p, g0.fbFloat(), g0.fbRGB8(), L, tiles[r],
                          g0.stream);
    }
    HIP_CHECK(hipStreamSynchronize(g0.stream));
  }
}

// ---------------------------------------------------------------- ray queries
void Device::intersect(SceneObj& S, const float* org4, const float* dir4, uint32_t n, float* hit4, int32_t* occ,
                       hipStream_t st) {
  HIP_CHECK(hipSetDevice(hipDevice));
  if (!S.gpu) throw std::runtime_error("scene not committed");
  GpuCtx& g = *ctx[0];
  g.dCount.alloc(sizeof(unsigned));
  HIP_CHECK(hipMemcpyAsync(g.dCount.p, &n, sizeof(unsigned), hipMemcpyHostToDevice, st));
  SceneView sv = S.gpu->view;
  sv.traceSpill = spill();
  if (occ)
    launch_trace_any(sv, (const float4*)org4, (const float4*)dir4, g.dCount.as<unsigned>(), 1, (int)n, occ, st);
  else
    launch_trace_closest(sv, (const float4*)org4, (const float4*)dir4, g.dCount.as<unsigned>(), 1, (int)n,
                         (float4*)hit4, st);
  HIP_CHECK(hipStreamSynchronize(st));
}

// ---------------------------------------------------------------- scene commit
void SceneObj::commit() {
  std::vector<std::shared_ptr<ScenePrim>> prims = slots;
  Device* d = static_cast<Device*>(dev);
  // per-face commits of the FPR loop (renderer.cpp:550-559) only re-orient faceCamera
  // meshes: refit on the GPU instead of rebuilding
  if (gpu && d->gpu && d->refitCommits) {
    HIP_CHECK(hipSetDevice(d->hipDevice));
    if (refit_gpu_scene(*gpu, prims, d->stream)) return;
  }
  gpu = build_gpu_scene(prims, YRT_STACK_DEPTH, d->gpu);
}

}  // namespace yrt

// ====================================================================== C ABI
using namespace yrt;

struct YRTDevice_ {
  Device* d;
};

#define DEV_GUARD(dev, failret)                                         \
  if (!dev || !dev->d) return failret;                                  \
  std::lock_guard<std::recursive_mutex> _lk(dev->d->mu);                \
  try {
#define DEV_END(failret)                                                \
  }                                                                     \
  catch (const std::exception& e) {                                     \
    dev->d->lastError = e.what();                                       \
    return failret;                                                     \
  }

extern "C" {

// parms: "" or "device=<k>" (one HIP device), "devices=<a,b,...>" or "devices=all" (tiles dealt
// over several; a device id may repeat: logical shards on one GPU), "host" (no GPU: loaders,
// BVH and frame export only, for CPU tests)
YRTDevice yrtNewDevice(const char* parms, size_t, int, const char*) {
  std::vector<int> devs = {0};
  bool gpu = true;
  try {
    if (parms && strncmp(parms, "device=", 7) == 0) devs = {atoi(parms + 7)};
    if (parms && strncmp(parms, "devices=", 8) == 0) {
      devs.clear();
      if (!strcmp(parms + 8, "all")) {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n < 1) return nullptr;
        for (int k = 0; k < n; ++k) devs.push_back(k);
      } else {
        for (const char* p = parms + 8; *p;) {
          devs.push_back(atoi(p));
          while (*p && *p != ',') ++p;
          if (*p == ',') ++p;
        }
      }
      if (devs.empty()) return nullptr;
    }
    if (parms && strcmp(parms, "host") == 0) gpu = false;
    auto* d = new YRTDevice_;
    d->d = new Device(devs, gpu);
    return d;
  } catch (...) {
    return nullptr;
  }
}

void yrtDeleteDevice(YRTDevice dev) {
  if (!dev) return;
  delete dev->d;
  delete dev;
}

const char* yrtGetLastError(YRTDevice dev) { return dev && dev->d ? dev->d->lastError.c_str() : "no device"; }

static bool ieq(const char* a, const char* b) { return a && b && strcasecmp(a, b) == 0; }

YRTHandle yrtNewCamera(YRTDevice dev, const char* type) {
  DEV_GUARD(dev, nullptr)
  if (!ieq(type, "pinhole") && !ieq(type, "depthoffield") && !ieq(type, "stereo"))
    throw std::runtime_error(std::string("unknown camera type: ") + type);
  return dev->d->wrap(std::make_shared<CameraObj>(type));
  DEV_END(nullptr)
}

YRTHandle yrtNewData(YRTDevice dev, const char* type, size_t bytes, const void* data) {
  DEV_GUARD(dev, nullptr)
  auto o = std::make_shared<DataObj>();
  o->type = type ? type : "immutable";
  o->bytes.assign((const uint8_t*)data, (const uint8_t*)data + bytes);
  return dev->d->wrap(o);
  DEV_END(nullptr)
}

// SingleRayDevice::rtNewDataFromFile (singleray_device.cpp:204-222)
YRTHandle yrtNewDataFromFile(YRTDevice dev, const char* type, const char* file, size_t offset, size_t bytes) {
  DEV_GUARD(dev, nullptr)
  if (!file) throw std::runtime_error("invalid file name");
  if (!strncmp(file, "server:", 7)) file += 7;
  if (strcasecmp(type, "immutable") != 0) throw std::runtime_error(std::string("unknown data buffer type: ") + type);
  FILE* f = fopen(file, "rb");
  if (!f) throw std::runtime_error(std::string("cannot open file ") + file);
  auto d = std::make_shared<DataObj>();
  d->bytes.resize(bytes);
  fseek(f, (long)offset, SEEK_SET);
  const size_t got = fread(d->bytes.data(), 1, bytes, f);
  fclose(f);
  if (got != bytes) throw std::runtime_error("error filling data buffer from file");
  return dev->d->wrap(d);
  DEV_END(nullptr)
}

YRTHandle yrtNewImage(YRTDevice dev, const char* type, size_t width, size_t height, const void* data) {
  DEV_GUARD(dev, nullptr)
  auto o = std::make_shared<ImageObj>();
  image_from_memory(type, (int)width, (int)height, data, *o);
  return dev->d->wrap(o);
  DEV_END(nullptr)
}

YRTHandle yrtNewImageFromFile(YRTDevice dev, const char* file) {
  DEV_GUARD(dev, nullptr)
  auto o = std::make_shared<ImageObj>();
  // SingleRayDevice::rtNewImageFromFile (singleray_device.cpp:238-251): failed load -> 1x1 white
  if (!image_load(file, *o)) {
    o->width = o->height = 1;
    o->format = IMG_RGBA8;
    o->data = {255, 255, 255, 255};
  }
  return dev->d->wrap(o);
  DEV_END(nullptr)
}

YRTHandle yrtNewTexture(YRTDevice dev, const char* type) {
  DEV_GUARD(dev, nullptr)
  if (!ieq(type, "bilinear") && !ieq(type, "nearest") && !ieq(type, "image"))
    throw std::runtime_error(std::string("unsupported texture type: ") + type);
  return dev->d->wrap(std::make_shared<TextureObj>(type));
  DEV_END(nullptr)
}

YRTHandle yrtNewMaterial(YRTDevice dev, const char* type) {
  DEV_GUARD(dev, nullptr)
  // SingleRayDevice::rtNewMaterial (api/singleray_device.cpp:262-280)
  static const char* ok[] = {"Matte", "Plastic", "Dielectric", "Glass", "ThinDielectric", "ThinGlass", "Mirror",
                             "Metal", "BrushedMetal", "MetallicPaint", "MatteTextured", "Uber", "Obj", "Velvet"};
  bool found = false;
  for (auto* n : ok) found |= ieq(type, n);
  if (!found) throw std::runtime_error(std::string("unknown material type: ") + type);
  return dev->d->wrap(std::make_shared<MaterialObj>(type));
  DEV_END(nullptr)
}

YRTHandle yrtNewShape(YRTDevice dev, const char* type) {
  DEV_GUARD(dev, nullptr)
  if (!ieq(type, "trianglemesh") && !ieq(type, "sphere") && !ieq(type, "triangle") && !ieq(type, "disk"))
    throw std::runtime_error(std::string("shape type '") + type + "' is outside the MI355X device's scope");
  return dev->d->wrap(std::make_shared<ShapeObj>(type));
  DEV_END(nullptr)
}

YRTHandle yrtNewLight(YRTDevice dev, const char* type) {
  DEV_GUARD(dev, nullptr)
  // SingleRayDevice::rtNewLight (api/singleray_device.cpp:293-302)
  static const char* ok[] = {"ambientlight", "pointlight", "spotlight", "directionallight", "distantlight",
                             "hdrilight", "trianglelight"};
  bool found = false;
  for (auto* n : ok) found |= ieq(type, n);
  if (!found) throw std::runtime_error(std::string("unknown light type: ") + type);
  return dev->d->wrap(std::make_shared<LightObj>(type));
  DEV_END(nullptr)
}

static A3 xfm_or_identity(const float* t) {
  if (!t) return a3_identity();
  return a3(l3(v3(t[0], t[1], t[2]), v3(t[3], t[4], t[5]), v3(t[6], t[7], t[8])), v3(t[9], t[10], t[11]));
}

YRTHandle yrtNewShapePrimitive(YRTDevice dev, YRTHandle shape, YRTHandle material, const float* transform12,
                               int faceCamera) {
  DEV_GUARD(dev, nullptr)
  auto p = std::make_shared<PrimitiveObj>();
  p->shapeHandle = dev->d->get<ShapeObj>(shape, "shape");
  p->materialHandle = dev->d->get<MaterialObj>(material, "material");
  if (!p->shapeHandle) throw std::runtime_error("invalid shape handle");
  p->transform = xfm_or_identity(transform12);
  p->faceCamera = faceCamera != 0;
  return dev->d->wrap(p);
  DEV_END(nullptr)
}

YRTHandle yrtNewLightPrimitive(YRTDevice dev, YRTHandle light, YRTHandle material, const float* transform12) {
  DEV_GUARD(dev, nullptr)
  auto p = std::make_shared<PrimitiveObj>();
  p->lightHandle = dev->d->get<LightObj>(light, "light");
  p->materialHandle = dev->d->get<MaterialObj>(material, "material");
  if (!p->lightHandle) throw std::runtime_error("invalid light handle");
  p->transform = xfm_or_identity(transform12);
  return dev->d->wrap(p);
  DEV_END(nullptr)
}

// SingleRayDevice::rtTransformPrimitive (singleray_device.cpp:328-334) ->
// PrimitiveHandle(space, other): transform = space * other.transform (api/instance.h:47-51)
YRTHandle yrtTransformPrimitive(YRTDevice dev, YRTHandle prim, const float* transform12) {
  DEV_GUARD(dev, nullptr)
  auto o = dev->d->get<PrimitiveObj>(prim, "primitive");
  if (!o) throw std::runtime_error("invalid primitive handle");
  auto p = std::make_shared<PrimitiveObj>(*o);
  p->transform = mul(xfm_or_identity(transform12), o->transform);
  return dev->d->wrap(p);
  DEV_END(nullptr)
}

YRTHandle yrtNewScene(YRTDevice dev, const char* type) {
  DEV_GUARD(dev, nullptr)
  return dev->d->wrap(std::make_shared<SceneObj>(type ? type : "default"));
  DEV_END(nullptr)
}

// BackendSceneFlat::Handle::setPrimitive (api/scene_flat.h:48-58)
int yrtSetPrimitive(YRTDevice dev, YRTHandle scene, size_t slot, YRTHandle prim) {
  DEV_GUARD(dev, -1)
  auto s = dev->d->get<SceneObj>(scene, "scene");
  auto p = dev->d->get<PrimitiveObj>(prim, "primitive");
  if (!s || !p) throw std::runtime_error("invalid scene or primitive");
  if (slot >= s->slots.size()) s->slots.resize(slot + 1);
  auto sp = std::make_shared<ScenePrim>();
  std::shared_ptr<const MeshInst> shape;
  std::shared_ptr<const LightInst> light;
  if (p->shapeHandle) {
    if (!p->shapeHandle->inst) throw std::runtime_error("shape not committed");
    shape = p->shapeHandle->inst;
  }
  if (p->lightHandle) {
    if (!p->lightHandle->inst) throw std::runtime_error("light not committed");
    light = p->lightHandle->inst;
    shape = light->shape;
  }
  if (shape) sp->shape = shape->transform(p->transform);
  if (light) sp->light = light->transform(p->transform, p->illumMask, p->shadowMask);
  if (p->materialHandle) {
    if (!p->materialHandle->inst) throw std::runtime_error("material not committed");
    sp->material = p->materialHandle->inst;
  }
  sp->illumMask = p->illumMask;
  sp->shadowMask = p->shadowMask;
  sp->faceCamera = p->faceCamera;
  sp->prim = p;
  s->slots[slot] = sp;
  return 0;
  DEV_END(-1)
}

// SingleRayDevice::rtUpdatePrimitive (singleray_device.cpp:354-398): re-orients a faceCamera
// primitive toward the camera position projected on the floor and replaces the scene slot
// (BackendSceneFlat::Handle::updatePrimitive, api/scene_flat.h:75-85). The caller re-commits
// the scene (renderer.cpp:550-559).
int yrtUpdatePrimitive(YRTDevice dev, YRTHandle scene, size_t slot, YRTHandle prim, const float* camPos3,
                       const float* camUp3) {
  DEV_GUARD(dev, -1)
  auto s = dev->d->get<SceneObj>(scene, "scene");
  if (!s) throw std::runtime_error("invalid scene handle");
  if (!prim) {
    if (slot < s->slots.size()) s->slots[slot].reset();
    return 0;
  }
  auto p = dev->d->get<PrimitiveObj>(prim, "primitive");
  if (!p->faceCamera) return 0;
  const V3 camPos = v3(camPos3[0], camPos3[1], camPos3[2]);
  const V3 camUp = v3(camUp3[0], camUp3[1], camUp3[2]);
  const V3 primPos = p->transform.p;
  V3 toEye = camPos - primPos;
  toEye.y = 0.f;
  toEye = normalize(toEye);
  const A3 lookAt = lookAtPoint(v3s(0.f), toEye, camUp);
  V3 right = cross(camUp, v3(0.f, 0.f, 1.f));
  if (right.x == 0.f && right.y == 0.f && right.z == 0.f) right = cross(camUp, v3(0.f, 1.f, 0.f));
  if (right.x == 0.f && right.y == 0.f && right.z == 0.f) right = cross(camUp, v3(1.f, 0.f, 0.f));
  const A3 makeVertical = a3_rotate_about(v3s(0.f), right, deg2rad(-90.f));
  A3 xf = mul(mul(a3_translate(primPos), lookAt), makeVertical);
  // glm::decompose scale: column lengths, negated when the linear part flips orientation
  const L3& l = p->transform.l;
  V3 sc = v3(length(l.vx), length(l.vy), length(l.vz));
  if (dot(l.vx, cross(l.vy, l.vz)) < 0.f) sc = -sc;
  if (sc.x != 0.f && sc.y != 0.f && sc.z != 0.f) xf = mul(xf, a3_scale(sc));
  if (slot > s->slots.size()) return 0;
  if (slot == s->slots.size()) s->slots.resize(slot + 1);
  auto sp = std::make_shared<ScenePrim>();
  std::shared_ptr<const MeshInst> shape;
  std::shared_ptr<const LightInst> light;
  if (p->shapeHandle && p->shapeHandle->inst) shape = p->shapeHandle->inst;
  if (p->lightHandle && p->lightHandle->inst) {
    light = p->lightHandle->inst;
    shape = light->shape;
  }
  if (shape) sp->shape = shape->transform(xf);
  if (light) sp->light = light->transform(xf, p->illumMask, p->shadowMask);
  if (p->materialHandle) sp->material = p->materialHandle->inst;
  sp->illumMask = p->illumMask;
  sp->shadowMask = p->shadowMask;
  sp->faceCamera = true;
  auto exportPrim = std::make_shared<PrimitiveObj>(*p);
  exportPrim->transform = xf;  // the frame blob carries the applied transform
  exportPrim->faceCamera = false;
  sp->prim = exportPrim;
  s->slots[slot] = sp;
  return 0;
  DEV_END(-1)
}

YRTHandle yrtNewToneMapper(YRTDevice dev, const char* type) {
  DEV_GUARD(dev, nullptr)
  if (!ieq(type, "default")) throw std::runtime_error(std::string("unknown tonemapper: ") + type);
  return dev->d->wrap(std::make_shared<ToneMapperObj>(type));
  DEV_END(nullptr)
}

YRTHandle yrtNewRenderer(YRTDevice dev, const char* type) {
  DEV_GUARD(dev, nullptr)
  if (!ieq(type, "pathtracer") && !ieq(type, "pt") && !ieq(type, "debug") && !ieq(type, "integrator"))
    throw std::runtime_error(std::string("unknown renderer: ") + type);
  return dev->d->wrap(std::make_shared<RendererObj>(type));
  DEV_END(nullptr)
}

YRTHandle yrtNewFrameBuffer(YRTDevice dev, const char* type, size_t width, size_t height, size_t buffers, void** ptrs) {
  DEV_GUARD(dev, nullptr)
  auto f = std::make_shared<FrameBufferObj>(type);
  if (ieq(type, "RGB8")) { f->format = FB_RGB8; f->stride = (3 * width + 3) / 4 * 4; }
  else if (ieq(type, "RGBA8")) { f->format = FB_RGBA8; f->stride = 4 * width; }
  else if (ieq(type, "RGB_FLOAT32")) { f->format = FB_RGB_FLOAT32; f->stride = 12 * width; }
  else if (ieq(type, "RGBA_FLOAT32")) { f->format = FB_RGBA_FLOAT32; f->stride = 16 * width; }
  else throw std::runtime_error(std::string("unknown framebuffer format: ") + type);
  f->width = (int)width;
  f->height = (int)height;
  f->depth = (int)std::max<size_t>(1, buffers);
  if (ptrs) f->userPtrs.assign(ptrs, ptrs + f->depth);
  else
    for (int i = 0; i < f->depth; ++i) f->host.emplace_back(new HostPixels(f->stride * height, dev->d->gpu));
  return dev->d->wrap(f);
  DEV_END(nullptr)
}

int yrtIncRef(YRTDevice dev, YRTHandle h) {
  DEV_GUARD(dev, -1)
  dev->d->ref(h)->refs++;
  return 0;
  DEV_END(-1)
}

int yrtDecRef(YRTDevice dev, YRTHandle h) {
  DEV_GUARD(dev, -1)
  HandleRef* r = dev->d->ref(h);
  if (--r->refs == 0) {
    dev->d->handles.erase(r);
    delete r;
  }
  return 0;
  DEV_END(-1)
}

static int set_variant(YRTDevice dev, YRTHandle h, const char* prop, const Variant& v) {
  DEV_GUARD(dev, -1)
  if (!prop) throw std::runtime_error("invalid property");
  auto& obj = dev->d->ref(h)->obj;
  obj->parms.set(prop, v);
  // PrimitiveHandle::set applies immediately (api/instance.h:54-60)
  if (auto p = std::dynamic_pointer_cast<PrimitiveObj>(obj)) {
    if (!strcmp(prop, "illumMask")) p->illumMask = v.i[0];
    else if (!strcmp(prop, "shadowMask")) p->shadowMask = v.i[0];
    else if (!strcmp(prop, "faceCamera")) p->faceCamera = v.i[0] != 0;
  }
  return 0;
  DEV_END(-1)
}

int yrtSetBool1(YRTDevice dev, YRTHandle h, const char* p, int x) {
  Variant v; v.type = Variant::BOOL1; v.i[0] = x != 0;
  return set_variant(dev, h, p, v);
}
int yrtSetBool2(YRTDevice dev, YRTHandle h, const char* p, int x, int y) {
  Variant v; v.type = Variant::BOOL2; v.i[0] = x != 0; v.i[1] = y != 0;
  return set_variant(dev, h, p, v);
}
int yrtSetBool3(YRTDevice dev, YRTHandle h, const char* p, int x, int y, int z) {
  Variant v; v.type = Variant::BOOL3; v.i[0] = x != 0; v.i[1] = y != 0; v.i[2] = z != 0;
  return set_variant(dev, h, p, v);
}
int yrtSetBool4(YRTDevice dev, YRTHandle h, const char* p, int x, int y, int z, int w) {
  Variant v; v.type = Variant::BOOL4; v.i[0] = x != 0; v.i[1] = y != 0; v.i[2] = z != 0; v.i[3] = w != 0;
  return set_variant(dev, h, p, v);
}
int yrtSetInt1(YRTDevice dev, YRTHandle h, const char* p, int x) {
  Variant v; v.type = Variant::INT1; v.i[0] = x;
  return set_variant(dev, h, p, v);
}
int yrtSetInt2(YRTDevice dev, YRTHandle h, const char* p, int x, int y) {
  Variant v; v.type = Variant::INT2; v.i[0] = x; v.i[1] = y;
  return set_variant(dev, h, p, v);
}
int yrtSetInt3(YRTDevice dev, YRTHandle h, const char* p, int x, int y, int z) {
  Variant v; v.type = Variant::INT3; v.i[0] = x; v.i[1] = y; v.i[2] = z;
  return set_variant(dev, h, p, v);
}
int yrtSetInt4(YRTDevice dev, YRTHandle h, const char* p, int x, int y, int z, int w) {
  Variant v; v.type = Variant::INT4; v.i[0] = x; v.i[1] = y; v.i[2] = z; v.i[3] = w;
  return set_variant(dev, h, p, v);
}
int yrtSetFloat1(YRTDevice dev, YRTHandle h, const char* p, float x) {
  Variant v; v.type = Variant::FLOAT1; v.f[0] = x;
  return set_variant(dev, h, p, v);
}
int yrtSetFloat2(YRTDevice dev, YRTHandle h, const char* p, float x, float y) {
  Variant v; v.type = Variant::FLOAT2; v.f[0] = x; v.f[1] = y;
  return set_variant(dev, h, p, v);
}
int yrtSetFloat3(YRTDevice dev, YRTHandle h, const char* p, float x, float y, float z) {
  Variant v; v.type = Variant::FLOAT3; v.f[0] = x; v.f[1] = y; v.f[2] = z;
  return set_variant(dev, h, p, v);
}
int yrtSetFloat4(YRTDevice dev, YRTHandle h, const char* p, float x, float y, float z, float w) {
  Variant v; v.type = Variant::FLOAT4; v.f[0] = x; v.f[1] = y; v.f[2] = z; v.f[3] = w;
  return set_variant(dev, h, p, v);
}
int yrtGetFloat3(YRTDevice dev, YRTHandle h, const char* p, float* x, float* y, float* z) {
  DEV_GUARD(dev, -1)
  const Variant* v = dev->d->ref(h)->obj->parms.find(p);
  if (!v || v->type != Variant::FLOAT3) throw std::runtime_error(std::string("no float3 property ") + p);
  *x = v->f[0]; *y = v->f[1]; *z = v->f[2];
  return 0;
  DEV_END(-1)
}
// rtGetFloat1 / rtGetString / rtGetTransform (singleray_device.cpp:548-555, 616-622, 651-657):
// the reference reads the handle's current value; unset properties read as 0 / "" / identity.
int yrtGetFloat1(YRTDevice dev, YRTHandle h, const char* p, float* x) {
  DEV_GUARD(dev, -1)
  if (!h) return 0;
  const Variant* v = dev->d->ref(h)->obj->parms.find(p);
  *x = 0.f;
  if (v) {
    if (v->type >= Variant::FLOAT1 && v->type <= Variant::FLOAT4) *x = v->f[0];
    else if (v->type >= Variant::BOOL1 && v->type <= Variant::INT4) *x = (float)v->i[0];
  }
  return 0;
  DEV_END(-1)
}
int yrtGetString(YRTDevice dev, YRTHandle h, const char* p, char* buf, size_t bufSize) {
  DEV_GUARD(dev, -1)
  if (!h) return 0;
  const Variant* v = dev->d->ref(h)->obj->parms.find(p);
  const std::string str = (v && v->type == Variant::STRING) ? v->str : std::string();
  if (buf && bufSize) {
    const size_t n = std::min(bufSize - 1, str.size());
    memcpy(buf, str.data(), n);
    buf[n] = 0;
  }
  return (int)str.size();
  DEV_END(-1)
}
int yrtGetTransform(YRTDevice dev, YRTHandle h, const char* p, float* transform12) {
  DEV_GUARD(dev, -1)
  if (!h) return 0;
  const Variant* v = dev->d->ref(h)->obj->parms.find(p);
  static const float I[12] = {1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0};
  memcpy(transform12, (v && v->type == Variant::TRANSFORM) ? v->f : I, sizeof(I));
  return 0;
  DEV_END(-1)
}
int yrtSetArray(YRTDevice dev, YRTHandle h, const char* p, const char* type, YRTHandle data, size_t size,
                size_t stride, size_t ofs) {
  DEV_GUARD(dev, -1)
  auto d = dev->d->get<DataObj>(data, "data");
  if (!d) throw std::runtime_error("invalid data handle");
  Variant v;
  v.type = Variant::DATA;
  v.obj = d;
  v.dataType = type;
  v.size = size;
  size_t es = 0;
  if (ieq(type, "float2")) es = 8;
  else if (ieq(type, "float3") || ieq(type, "int3")) es = 12;
  else if (ieq(type, "float4") || ieq(type, "int4")) es = 16;
  else if (ieq(type, "float1") || ieq(type, "int1")) es = 4;
  else if (ieq(type, "int2")) es = 8;
  else throw std::runtime_error(std::string("unknown array type: ") + type);
  v.stride = stride == (size_t)-1 ? es : stride;
  v.ofs = ofs;
  if (size && v.ofs + (size - 1) * v.stride + es > d->bytes.size()) throw std::runtime_error("array exceeds data");
  dev->d->ref(h)->obj->parms.set(p, v);
  return 0;
  DEV_END(-1)
}
int yrtSetString(YRTDevice dev, YRTHandle h, const char* p, const char* str) {
  Variant v; v.type = Variant::STRING; v.str = str ? str : "";
  return set_variant(dev, h, p, v);
}
int yrtSetImage(YRTDevice dev, YRTHandle h, const char* p, YRTHandle image) {
  DEV_GUARD(dev, -1)
  Variant v;
  v.type = Variant::IMAGE;
  v.obj = dev->d->get<ImageObj>(image, "image");
  dev->d->ref(h)->obj->parms.set(p, v);
  return 0;
  DEV_END(-1)
}
int yrtSetTexture(YRTDevice dev, YRTHandle h, const char* p, YRTHandle texture) {
  DEV_GUARD(dev, -1)
  Variant v;
  v.type = Variant::TEXTURE;
  v.obj = dev->d->get<TextureObj>(texture, "texture");
  dev->d->ref(h)->obj->parms.set(p, v);
  return 0;
  DEV_END(-1)
}
int yrtSetTransform(YRTDevice dev, YRTHandle h, const char* p, const float* t) {
  Variant v;
  v.type = Variant::TRANSFORM;
  for (int i = 0; i < 12; ++i) v.f[i] = t[i];
  return set_variant(dev, h, p, v);
}
int yrtSetPointer(YRTDevice dev, YRTHandle h, const char* p, void* ptr) {
  Variant v; v.type = Variant::POINTER; v.ptr = ptr;
  return set_variant(dev, h, p, v);
}
int yrtClear(YRTDevice dev, YRTHandle h) {
  DEV_GUARD(dev, -1)
  dev->d->ref(h)->obj->parms.clear();
  return 0;
  DEV_END(-1)
}
int yrtCommit(YRTDevice dev, YRTHandle h) {
  DEV_GUARD(dev, -1)
  if (dev->d->gpu) HIP_CHECK(hipSetDevice(dev->d->hipDevice));
  dev->d->ref(h)->obj->commit();
  return 0;
  DEV_END(-1)
}

int yrtRenderFrame(YRTDevice dev, YRTHandle renderer, YRTHandle camera, YRTHandle scene, YRTHandle tonemapper,
                   YRTHandle framebuffer, int accumulate) {
  DEV_GUARD(dev, -1)
  std::shared_ptr<RendererObj> R;
  std::shared_ptr<CameraObj> C;
  std::shared_ptr<SceneObj> S;
  std::shared_ptr<ToneMapperObj> T;
  std::shared_ptr<FrameBufferObj> F;
  try {
    R = dev->d->get<RendererObj>(renderer, "renderer");
    C = dev->d->get<CameraObj>(camera, "camera");
    S = dev->d->get<SceneObj>(scene, "scene");
    T = dev->d->get<ToneMapperObj>(tonemapper, "tonemapper");
    F = dev->d->get<FrameBufferObj>(framebuffer, "framebuffer");
    if (!R || !C || !S || !T || !F) throw std::runtime_error("rtRenderFrame: null handle");
    if (!dev->d->gpu) throw std::runtime_error("rtRenderFrame: host-only device (created with parms \"host\")");
  } catch (...) {
    dev->d->fail_proc_gather();  // the peers of a process gather must not wait for this rank
    throw;
  }
  dev->d->render(*R, {C.get()}, *S, *T, {F.get()}, accumulate);
  return 0;
  DEV_END(-1)
}

int yrtRenderFrames(YRTDevice dev, YRTHandle renderer, const YRTHandle* cameras, int numFrames, YRTHandle scene,
                    YRTHandle tonemapper, const YRTHandle* framebuffers, int accumulate) {
  DEV_GUARD(dev, -1)
  std::shared_ptr<RendererObj> R;
  std::shared_ptr<SceneObj> S;
  std::shared_ptr<ToneMapperObj> T;
  std::vector<std::shared_ptr<CameraObj>> cs;
  std::vector<std::shared_ptr<FrameBufferObj>> fs;
  std::vector<CameraObj*> cp;
  std::vector<FrameBufferObj*> fp;
  try {
    if (numFrames < 1 || !cameras || !framebuffers) throw std::runtime_error("rtRenderFrames: no frames");
    R = dev->d->get<RendererObj>(renderer, "renderer");
    S = dev->d->get<SceneObj>(scene, "scene");
    T = dev->d->get<ToneMapperObj>(tonemapper, "tonemapper");
    if (!R || !S || !T) throw std::runtime_error("rtRenderFrames: null handle");
    // one accumulation state per framebuffer and sampler iteration per job: a multi-frame job
    // equals a loop of yrtRenderFrame calls only for non-accumulating frames (yrt_device.h)
    if (numFrames > 1 && accumulate) throw std::runtime_error("rtRenderFrames: accumulate needs numFrames == 1");
    cs.resize(numFrames);
    fs.resize(numFrames);
    cp.resize(numFrames);
    fp.resize(numFrames);
    for (int k = 0; k < numFrames; ++k) {
      cs[k] = dev->d->get<CameraObj>(cameras[k], "camera");
      fs[k] = dev->d->get<FrameBufferObj>(framebuffers[k], "framebuffer");
      if (!cs[k] || !fs[k]) throw std::runtime_error("rtRenderFrames: null camera or framebuffer handle");
      cp[k] = cs[k].get();
      fp[k] = fs[k].get();
    }
    if (!dev->d->gpu) throw std::runtime_error("rtRenderFrames: host-only device (created with parms \"host\")");
  } catch (...) {
    dev->d->fail_proc_gather();
    throw;
  }
  dev->d->render(*R, cp, *S, *T, fp, accumulate);
  return 0;
  DEV_END(-1)
}

void* yrtMapFrameBuffer(YRTDevice dev, YRTHandle fb, int bufID) {
  DEV_GUARD(dev, nullptr)
  auto F = dev->d->get<FrameBufferObj>(fb, "framebuffer");
  const int id = bufID < 0 ? F->cur : bufID;
  if (id < 0 || id >= F->depth) throw std::runtime_error("rtMapFrameBuffer: invalid buffer id");
  fb_read_back(*F, id);  // a frame still in HBM comes to the host pixels now
  return F->buffer(id);
  DEV_END(nullptr)
}
int yrtUnmapFrameBuffer(YRTDevice dev, YRTHandle fb, int) {
  DEV_GUARD(dev, -1)
  (void)dev->d->get<FrameBufferObj>(fb, "framebuffer");
  return 0;
  DEV_END(-1)
}
int yrtSwapBuffers(YRTDevice dev, YRTHandle fb) {
  DEV_GUARD(dev, -1)
  auto F = dev->d->get<FrameBufferObj>(fb, "framebuffer");
  F->cur = (F->cur + 1) % F->depth;
  return 0;
  DEV_END(-1)
}
int yrtSetStatusCallback(YRTDevice dev, YRTHandle renderer, YRTStatusCallback cb, void* user) {
  DEV_GUARD(dev, -1)
  auto R = dev->d->get<RendererObj>(renderer, "renderer");
  R->statusCallback = (void*)cb;
  R->statusUser = user;
  return 0;
  DEV_END(-1)
}
int yrtSetStopFlag(YRTDevice dev, YRTHandle renderer, volatile int* flag) {
  DEV_GUARD(dev, -1)
  auto R = dev->d->get<RendererObj>(renderer, "renderer");
  R->stopFlag = (std::atomic<bool>*)flag;  // polled as a byte-sized bool between batches
  return 0;
  DEV_END(-1)
}

int yrtIntersect(YRTDevice dev, YRTHandle scene, const float* org4, const float* dir4, uint32_t n, float* hit4,
                 void* stream) {
  DEV_GUARD(dev, -1)
  auto S = dev->d->get<SceneObj>(scene, "scene");
  dev->d->intersect(*S, org4, dir4, n, hit4, nullptr, stream ? (hipStream_t)stream : dev->d->stream);
  return 0;
  DEV_END(-1)
}
int yrtOccluded(YRTDevice dev, YRTHandle scene, const float* org4, const float* dir4, uint32_t n, int32_t* occ,
                void* stream) {
  DEV_GUARD(dev, -1)
  auto S = dev->d->get<SceneObj>(scene, "scene");
  dev->d->intersect(*S, org4, dir4, n, nullptr, occ, stream ? (hipStream_t)stream : dev->d->stream);
  return 0;
  DEV_END(-1)
}
int yrtTriangleIds(YRTDevice dev, YRTHandle scene, int32_t tri, int32_t* geomID, int32_t* primID) {
  DEV_GUARD(dev, -1)
  auto S = dev->d->get<SceneObj>(scene, "scene");
  if (!S->gpu) throw std::runtime_error("scene not committed");
  if (tri < 0 || tri >= S->gpu->numTris) { *geomID = -1; *primID = -1; return 0; }
  const int g = S->gpu->hTriGeom[tri];
  *geomID = g;
  *primID = tri - S->gpu->hGeoms[g].triBase;
  return 0;
  DEV_END(-1)
}
int yrtPick(YRTDevice dev, YRTHandle camera, float x, float y, YRTHandle scene, float* px, float* py, float* pz) {
  DEV_GUARD(dev, -1)
  Device& D = *dev->d;
  if (!D.gpu) throw std::runtime_error("rtPick: host-only device");
  auto C = D.get<CameraObj>(camera, "camera");
  auto S = D.get<SceneObj>(scene, "scene");
  if (!C || !S || !S->gpu) throw std::runtime_error("rtPick: invalid camera or uncommitted scene");
  HIP_CHECK(hipSetDevice(D.hipDevice));
  GpuCtx& g = *D.ctx[0];
  g.dCam.alloc(sizeof(GpuCamera));
  g.dCount.alloc(sizeof(float4));
  HIP_CHECK(hipMemcpyAsync(g.dCam.p, &C->cam, sizeof(GpuCamera), hipMemcpyHostToDevice, D.stream));
  launch_pick(S->gpu->view, g.dCam.as<GpuCamera>(), x, y, g.dCount.as<float4>(), D.stream);
  float4 r;
  HIP_CHECK(hipMemcpyAsync(&r, g.dCount.p, sizeof(r), hipMemcpyDeviceToHost, D.stream));
  HIP_CHECK(hipStreamSynchronize(D.stream));
  *px = r.x;
  *py = r.y;
  *pz = r.z;
  return __builtin_bit_cast(int, r.w) >= 0 ? 1 : 0;
  DEV_END(-1)
}

int yrtGetRenderStats(YRTDevice dev, YRTRenderStats* out) {
  DEV_GUARD(dev, -1)
  *out = dev->d->stats;
  return 0;
  DEV_END(-1)
}
int yrtSetKernelTiming(YRTDevice dev, int enable) {
  DEV_GUARD(dev, -1)
  dev->d->kernelTiming = enable != 0;
  return 0;
  DEV_END(-1)
}
int yrtSetLanes(YRTDevice dev, int lanes) {
  DEV_GUARD(dev, -1)
  if (lanes < 0 || lanes > GpuCtx::kMaxLanes)
    throw std::runtime_error("yrtSetLanes: 1.." + std::to_string(GpuCtx::kMaxLanes) + " lanes (YRT_MAX_LANES), 0 = default");
  for (auto& c : dev->d->ctx) c->numLanes = lanes ? lanes : GpuCtx::default_lanes();
  return 0;
  DEV_END(-1)
}
int yrtGetSceneInfo(YRTDevice dev, YRTHandle scene, YRTSceneInfo* out) {
  DEV_GUARD(dev, -1)
  auto S = dev->d->get<SceneObj>(scene, "scene");
  if (!S->gpu) throw std::runtime_error("scene not committed");
  out->numTriangles = S->gpu->numTris;
  out->numGeometries = S->gpu->numGeoms;
  out->numNodes = (int64_t)S->gpu->hNodes.size();
  out->numTriRefs = (int64_t)S->gpu->hTris.size();
  out->triRecordBytes = (int64_t)sizeof(GpuTri);
  out->nodeBytesClosest = trace_node_bytes(false);
  out->nodeBytesAny = trace_node_bytes(true);
  out->bvhDepth = S->gpu->bvhDepth;
  out->numLights = S->gpu->view.numLights;
  out->buildSeconds = S->gpu->buildSeconds;
  for (int k = 0; k < 3; ++k) { out->bboxLo[k] = S->gpu->bboxLo[k]; out->bboxHi[k] = S->gpu->bboxHi[k]; }
  return 0;
  DEV_END(-1)
}
int yrtExportBVH(YRTDevice dev, YRTHandle scene, void* nodes, size_t nodesBytes, void* tris, size_t trisBytes) {
  DEV_GUARD(dev, -1)
  auto S = dev->d->get<SceneObj>(scene, "scene");
  if (!S->gpu) throw std::runtime_error("scene not committed");
  sync_host_bvh(*S->gpu);
  const size_t nb = S->gpu->hNodes.size() * sizeof(GpuNode), tb = S->gpu->hTris.size() * sizeof(GpuTri);
  if (nodesBytes < nb || trisBytes < tb) throw std::runtime_error("buffers too small");
  memcpy(nodes, S->gpu->hNodes.data(), nb);
  memcpy(tris, S->gpu->hTris.data(), tb);
  return 0;
  DEV_END(-1)
}
int yrtExportQuantizedBVH(YRTDevice dev, YRTHandle scene, void* qnodes, size_t qnodesBytes) {
  DEV_GUARD(dev, -1)
  auto S = dev->d->get<SceneObj>(scene, "scene");
  if (!S->gpu) throw std::runtime_error("scene not committed");
  sync_host_bvh(*S->gpu);
  const size_t nb = S->gpu->hQNodes.size() * sizeof(GpuQNode);
  if (qnodesBytes < nb) throw std::runtime_error("buffer too small");
  memcpy(qnodes, S->gpu->hQNodes.data(), nb);
  return 0;
  DEV_END(-1)
}
int yrtSetFrameSeed(YRTDevice dev, uint32_t seed) {
  DEV_GUARD(dev, -1)
  dev->d->frameSeed = seed;
  return 0;
  DEV_END(-1)
}
int yrtSetBatchCapacity(YRTDevice dev, int64_t paths) {
  DEV_GUARD(dev, -1)
  if (paths < 256) throw std::runtime_error("capacity must be >= 256 paths");
  dev->d->capacity = paths;
  return 0;
  DEV_END(-1)
}
int64_t yrt_export_frame_impl(const Object* renderer, const Object* camera, const SceneObj* scene, uint32_t frameSeed,
                              void* buf, size_t bytes);
int64_t yrtExportFrame(YRTDevice dev, YRTHandle renderer, YRTHandle camera, YRTHandle scene, void* buf, size_t bytes) {
  DEV_GUARD(dev, -1)
  auto R = dev->d->get<RendererObj>(renderer, "renderer");
  auto C = dev->d->get<CameraObj>(camera, "camera");
  auto S = dev->d->get<SceneObj>(scene, "scene");
  if (!R || !C || !S) throw std::runtime_error("yrtExportFrame: null handle");
  return yrt_export_frame_impl(R.get(), C.get(), S.get(), dev->d->frameSeed, buf, bytes);
  DEV_END(-1)
}

int yrtDebugSampleTable(int spp, int sets, int iteration, int num1D, int num2D, const char* filter, float* out,
                        size_t outFloats) {
  try {
    SampleRequest req;
    req.spp = spp;
    req.sets = sets;
    req.iteration = iteration;
    req.num1D = num1D;
    req.num2D = num2D;
    req.filter = filter ? filter : "bspline";
    SampleTable t;
    build_sample_table(req, t);
    if (out && outFloats >= t.dims.size()) memcpy(out, t.dims.data(), t.dims.size() * sizeof(float));
    return t.numRecords;
  } catch (...) {
    return -1;
  }
}

int yrtDebugDecodeImage(const char* file, int* width, int* height, int* channels, uint8_t* out, size_t outBytes) {
  try {
    FILE* f = fopen(file, "rb");
    if (!f) return -1;
    std::vector<uint8_t> bytes;
    uint8_t buf[65536];
    size_t n;
    while ((n = fread(buf, 1, sizeof(buf), f)) > 0) bytes.insert(bytes.end(), buf, buf + n);
    fclose(f);
    std::string err;
    std::vector<uint8_t> px;
    int w = 0, h = 0, c = 3;
    const char* dot = strrchr(file, '.');
    if (dot && (!strcasecmp(dot, ".jpg") || !strcasecmp(dot, ".jpeg"))) {
      if (!decode_jpeg(bytes, w, h, px, err)) return -2;
    } else if (dot && !strcasecmp(dot, ".png")) {
      if (!decode_png(bytes, w, h, c, px, err)) return -2;
    } else {
      return -3;
    }
    *width = w;
    *height = h;
    *channels = c;
    if (out && outBytes >= px.size()) memcpy(out, px.data(), px.size());
    return 0;
  } catch (...) {
    return -4;
  }
}

int yrtSetRayCapture(YRTDevice dev, int maxPerDepth) {
  DEV_GUARD(dev, -1)
  dev->d->captureMax = std::max(0, maxPerDepth);
  return 0;
  DEV_END(-1)
}

int64_t yrtGetCapturedRays(YRTDevice dev, int shadow, int depth, float* org4, float* dir4, size_t maxRays,
                           double* totalInBatch) {
  DEV_GUARD(dev, -1)
  if (dev->d->ctx.empty()) throw std::runtime_error("host-only device");
  auto& v = shadow ? dev->d->ctx[0]->capShadow : dev->d->ctx[0]->capClosest;
  if (depth < 0 || depth >= (int)v.size()) {
    if (totalInBatch) *totalInBatch = 0;
    return 0;
  }
  const auto& c = v[depth];
  const size_t m = c.org.size() / 4;
  if (totalInBatch) *totalInBatch = c.total;
  if (org4 && dir4) {
    const size_t k = std::min(m, maxRays);
    memcpy(org4, c.org.data(), k * 16);
    memcpy(dir4, c.dir.data(), k * 16);
  }
  return (int64_t)m;
  DEV_END(-1)
}

int yrtDebugTraceProfile(YRTDevice dev, uint64_t* out8, int reset) {
  DEV_GUARD(dev, -1)
  HIP_CHECK(hipDeviceSynchronize());
  return trace_profile((unsigned long long*)out8, reset);
  DEV_END(-1)
}

int yrtDebugPixelSamples(YRTDevice dev, int pixelId, int frame, float* out4, int maxSamples) {
  DEV_GUARD(dev, -1)
  Device& D = *dev->d;
  if (!D.gpu) throw std::runtime_error("host-only device");
  HIP_CHECK(hipSetDevice(D.hipDevice));
  // one capture at a time per process (the kernel-side target is a module global)
  DevBuf& buf = D.dbgPixelBuf;
  if (!out4) {
    if (pixelId < 0) return debug_pixel_capture(-1, -1, nullptr, 0);
    if (maxSamples < 1) throw std::runtime_error("yrtDebugPixelSamples: maxSamples < 1");
    buf.alloc((size_t)maxSamples * sizeof(float4));
    HIP_CHECK(hipMemset(buf.p, 0, (size_t)maxSamples * sizeof(float4)));
    D.dbgPixelCap = maxSamples;
    return debug_pixel_capture(pixelId, frame, buf.as<float4>(), maxSamples);
  }
  if (!buf.p) throw std::runtime_error("yrtDebugPixelSamples: no capture armed on this device");
  const int n = std::min(maxSamples, D.dbgPixelCap);
  HIP_CHECK(hipDeviceSynchronize());
  HIP_CHECK(hipMemcpy(out4, buf.p, (size_t)n * sizeof(float4), hipMemcpyDeviceToHost));
  return n;
  DEV_END(-1)
}

int yrtDebugCheckMath(YRTDevice dev, int fn, uint64_t* out2) {
  DEV_GUARD(dev, -1)
  if (fn != 0 || !out2) throw std::runtime_error("yrtDebugCheckMath: fn 0 only");
  HIP_CHECK(hipSetDevice(dev->d->hipDevice));
  if (check_math(fn, (unsigned long long*)out2) != 0) throw std::runtime_error("check_math failed");
  return 0;
  DEV_END(-1)
}

int yrtDebugCheckMathTable(YRTDevice dev, int fn, const uint16_t* table2048, uint64_t* out2) {
  DEV_GUARD(dev, -1)
  if ((fn != 1 && fn != 2) || !table2048 || !out2) throw std::runtime_error("yrtDebugCheckMathTable: fn 1 or 2");
  HIP_CHECK(hipSetDevice(dev->d->hipDevice));
  if (check_math_table(fn, table2048, (unsigned long long*)out2) != 0) throw std::runtime_error("check_math_table failed");
  return 0;
  DEV_END(-1)
}

int yrtDebugTileScatter(int t, int T) {
  if (T < 1 || t < 0 || t >= T) return -1;
  return yrt_tile_scatter(t, T);
}

int yrtSetTileShard(YRTDevice dev, int index, int count) {
  DEV_GUARD(dev, -1)
  if (count < 1 || index < 0 || index >= count) throw std::runtime_error("invalid shard");
  // a process communicator gathers exactly its own shard (rank of world): another shard would
  // post sends/receives its peers never match
  if (dev->d->proc && (index != dev->d->commRank || count != dev->d->commWorld))
    throw std::runtime_error("yrtSetTileShard: shard differs from the process communicator's (rank " +
                             std::to_string(dev->d->commRank) + " of " + std::to_string(dev->d->commWorld) +
                             "); call yrtSetShardComm(dev, 0, 1, id) or yrtSetShardHub(dev, NULL, 0) first to drop it");
  dev->d->shardIndex = index;
  dev->d->shardCount = count;
  return 0;
  DEV_END(-1)
}

int yrtRcclAvailable(void) {
  try {
    (void)rccl();
    return 1;
  } catch (...) {
    return 0;
  }
}

int yrtShardCommUniqueId(void* id128) {
  try {
    ncclUniqueId id;
    rccl_check(rccl().GetUniqueId(&id), "ncclGetUniqueId");
    memcpy(id128, &id, sizeof(id));
    return 0;
  } catch (...) {
    return -1;
  }
}

int yrtSetShardComm(YRTDevice dev, int rank, int world, const void* id128) {
  DEV_GUARD(dev, -1)
  Device& D = *dev->d;
  if (world < 1 || rank < 0 || rank >= world) throw std::runtime_error("invalid shard");
  if (!D.gpu) throw std::runtime_error("host-only device");
  HIP_CHECK(hipSetDevice(D.hipDevice));
  D.proc.reset();
  D.commRank = 0;
  D.commWorld = 1;
  if (world > 1) {
    D.proc = make_rccl_transport(rank, world, id128);
    D.commRank = rank;
    D.commWorld = world;
  }
  D.shardIndex = rank;
  D.shardCount = world;
  return 0;
  DEV_END(-1)
}

struct YRTShardHub_ {
  std::shared_ptr<ShardHub> hub;
};
static thread_local std::string t_hubError;

YRTShardHub yrtNewShardHub(int world) {
  try {
    auto* h = new YRTShardHub_;
    h->hub = make_shard_hub(world);
    return h;
  } catch (const std::exception& e) {
    t_hubError = e.what();
    return nullptr;
  }
}

void yrtDeleteShardHub(YRTShardHub hub) { delete hub; }

int yrtSetShardHub(YRTDevice dev, YRTShardHub hub, int rank) {
  DEV_GUARD(dev, -1)
  Device& D = *dev->d;
  D.proc.reset();
  D.commRank = 0;
  D.commWorld = 1;
  D.shardIndex = 0;
  D.shardCount = 1;
  if (!hub) return 0;
  const int world = shard_hub_world(*hub->hub);
  if (rank < 0 || rank >= world) throw std::runtime_error("yrtSetShardHub: invalid rank");
  if (!D.gpu && world > 1) throw std::runtime_error("host-only device");
  if (world > 1) {
    D.proc = make_hub_transport(hub->hub, rank);
    D.commRank = rank;
    D.commWorld = world;
  }
  D.shardIndex = rank;
  D.shardCount = world;
  return 0;
  DEV_END(-1)
}

int yrtSetGatherTimeout(YRTDevice dev, double seconds) {
  DEV_GUARD(dev, -1)
  if (!(seconds > 0)) throw std::runtime_error("yrtSetGatherTimeout: seconds must be > 0");
  dev->d->gatherTimeout = seconds;
  return 0;
  DEV_END(-1)
}

int yrtShardHubStatus(YRTShardHub hub, int rank, int flag, double timeoutS) {
  try {
    if (!hub) throw std::runtime_error("null hub");
    return hub_host_status(*hub->hub, rank, flag, timeoutS);
  } catch (const std::exception& e) {
    t_hubError = e.what();
    return -1;
  }
}

int yrtShardHubSlab(YRTShardHub hub, int rank, const void* slab, size_t bytes, void* recv, size_t recvBytesPerRank,
                    double timeoutS) {
  try {
    if (!hub) throw std::runtime_error("null hub");
    hub_host_slab(*hub->hub, rank, slab, bytes, recv, recvBytesPerRank, timeoutS);
    return 0;
  } catch (const std::exception& e) {
    t_hubError = e.what();
    return -1;
  }
}

const char* yrtShardHubLastError(void) { return t_hubError.c_str(); }

int yrtGetDeviceCount(YRTDevice dev) {
  DEV_GUARD(dev, -1)
  return (int)dev->d->ctx.size();
  DEV_END(-1)
}

int yrtSetRefitCommits(YRTDevice dev, int on) {
  DEV_GUARD(dev, -1)
  dev->d->refitCommits = on != 0;
  return 0;
  DEV_END(-1)
}

int yrtGetSceneRefits(YRTDevice dev, YRTHandle scene) {
  DEV_GUARD(dev, -1)
  auto S = dev->d->get<SceneObj>(scene, "scene");
  if (!S || !S->gpu) throw std::runtime_error("scene not committed");
  return S->gpu->refits;
  DEV_END(-1)
}

}  // extern "C"
