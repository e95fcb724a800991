// scene_gpu.h — a committed scene flattened into HBM (layout: common/yrt_gpu_types.h).
#pragma once

#include <hip/hip_runtime.h>

#include <memory>
#include <stdexcept>
#include <string>
#include <atomic>
#include <vector>

#include "../kernels/yrt_kernels.h"
#include "objects.h"
#include "sampler.h"

namespace yrt {

#define HIP_CHECK(x)                                                                              \
  do {                                                                                            \
    hipError_t _e = (x);                                                                          \
    if (_e != hipSuccess)                                                                         \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " #x);    \
  } while (0)

// RAII device allocation
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() {}
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  void alloc(size_t n) {
    if (n <= bytes && p) return;
    release();
    if (n == 0) n = 16;
    HIP_CHECK(hipMalloc(&p, n));
    bytes = n;
  }
  template <class T>
  void upload(const std::vector<T>& v) {
    alloc(v.size() * sizeof(T));
    if (!v.empty()) HIP_CHECK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  }
  template <class T>
  T* as() const { return (T*)p; }
};

struct GpuScene {
  int device = 0;
  uint64_t serial = next_serial();  // identifies the committed scene in caches (addresses get reused)
  static uint64_t next_serial() {
    static std::atomic<uint64_t> n{1};
    return n++;
  }
  DevBuf nodes, qnodes, tris, triGeom, indices, positions, normals, texcoords, geoms, materials, textures, images, texels, texQuads,
      lights, envLights, hdriDist, media, geomRecs, motions, tangents, triMotion, triShade;
  bool hasMotion = false;  // moving geometry: time-aware trace kernels, no refit
  SceneView view{};
  unsigned materialMask = 0;  // bit MAT_x per material type, bit 16+LIGHT_x per light type used (shade kernel variant)
  size_t texels8Bytes = 0;    // the 8-bit images' part of the texel pool (float images follow it)
  // host mirrors (BVH export, precomputed light sampling, stats)
  std::vector<GpuNode> hNodes;
  std::vector<GpuQNode> hQNodes;  // the same tree with 64-B quantized nodes (common/yrt_qnode.h)
  std::vector<GpuTri> hTris;
  std::vector<GpuGeom> hGeoms;
  std::vector<int> hTriGeom;
  std::vector<std::shared_ptr<const LightInst>> allLights;
  std::vector<GpuLight> hLights;                // the uploaded light table
  std::vector<int> hEnvLights;                  // the uploaded envLights (indices into hLights)
  std::vector<LightSampleSource> precomputed;   // LightSampleSource per precompute() light
  // incremental commits (faceCamera refit, refit_gpu_scene): the slots this scene was built
  // from, slot -> geometry, gid -> leaf position, and the node indices grouped by tree depth
  std::vector<std::shared_ptr<ScenePrim>> slotsCommitted;
  std::vector<int> slotGeom;
  std::vector<int> levelStart;  // nodes of depth d: levelNodes[levelStart[d] .. levelStart[d+1])
  DevBuf triLeaf, levelNodes;
  bool hostBvhStale = false;    // hNodes/hTris lag a device refit until sync_host_bvh
  int refits = 0;               // refit commits since the build (stats)
  int numTris = 0, numGeoms = 0, bvhDepth = 0;
  double buildSeconds = 0;
  float bboxLo[3] = {0, 0, 0}, bboxHi[3] = {0, 0, 0};
};

std::shared_ptr<GpuScene> build_gpu_scene(const std::vector<std::shared_ptr<ScenePrim>>& prims, int stackDepth,
                                          bool upload);
// A copy of an uploaded scene's device buffers on another HIP device (peer copies over xGMI),
// for multi-GPU tile rendering; the host-side mirrors stay with the source.
std::shared_ptr<GpuScene> replicate_gpu_scene(const GpuScene& src, int device);
// Commits `prims` onto an uploaded scene without a rebuild when only vertex positions/normals
// of some primitives changed (faceCamera re-orientation): uploads the moved vertices and
// refits the BVH on the GPU. Returns false (scene untouched) when a rebuild is needed.
bool refit_gpu_scene(GpuScene& S, const std::vector<std::shared_ptr<ScenePrim>>& prims, hipStream_t stream);
// Brings the host BVH mirrors (export, stats) up to date after device refits.
void sync_host_bvh(GpuScene& S);

}  // namespace yrt
