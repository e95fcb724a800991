// objects.h — device objects behind the C-ABI handles.
//
// Mirrors device_singleray/api/handle.h: an object buffers rtSet* values in a Parms bag and
// rtCommit builds an immutable instance from them (constructor defaults restated from the
// reference classes). Primitives capture the instances current at creation time, scenes
// flatten their primitives into GPU buffers at commit.
#pragma once

#include <hip/hip_runtime.h>

#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../common/yrt_gpu_types.h"
#include "../common/yrt_math.h"
#include "parms.h"

namespace yrt {

enum class Kind { CAMERA, DATA, IMAGE, TEXTURE, MATERIAL, SHAPE, LIGHT, PRIMITIVE, SCENE, TONEMAPPER, RENDERER, FRAMEBUFFER };
const char* kind_name(Kind k);

class Device;

struct Object {
  Kind kind;
  std::string type;
  Parms parms;
  Device* dev = nullptr;
  Object(Kind k, const std::string& t) : kind(k), type(t) {}
  virtual ~Object() {}
  virtual void commit() {}
};

// C-ABI handle: a counted reference to an object (api/handle.h:26-31, refcount starts at 1).
struct HandleRef {
  std::shared_ptr<Object> obj;
  std::atomic<int> refs{1};
  uint32_t magic = 0x59525448;  // 'YRTH'
};

// ---------------------------------------------------------------- data / images
struct DataObj : Object {
  std::vector<uint8_t> bytes;
  DataObj() : Object(Kind::DATA, "immutable") {}
};

// Image4c semantics: RGBA8 texels as stored after the loader's float round trip
// (common/image/*.cpp store Color4 through Col4c: char(clamp(c)*255)); or RGBA float.
struct ImageObj : Object {
  int width = 0, height = 0;
  ImageFormat format = IMG_RGBA8;
  std::vector<uint8_t> data;  // width*height*4 bytes (RGBA8) or *16 (RGBAF32)
  // process-unique identity (device caches key on it: a freed image's address can be reused)
  const uint64_t serial = next_serial();
  ImageObj() : Object(Kind::IMAGE, "image") {}
  static uint64_t next_serial() {
    static std::atomic<uint64_t> n{0};
    return ++n;
  }
  void get(int x, int y, float c[4]) const;
};

struct TextureInst {
  std::shared_ptr<ImageObj> image;
  TexFilter filter = TEX_BILINEAR;
  bool invert = false;
};
struct TextureObj : Object {
  std::shared_ptr<const TextureInst> inst;
  explicit TextureObj(const std::string& t) : Object(Kind::TEXTURE, t) {}
  void commit() override;
};

// ---------------------------------------------------------------- materials
struct MaterialInst {
  GpuMaterial gm;
  std::shared_ptr<const TextureInst> tex[5];
};
struct MaterialObj : Object {
  std::shared_ptr<const MaterialInst> inst;
  explicit MaterialObj(const std::string& t) : Object(Kind::MATERIAL, t) {}
  void commit() override;
};

// ---------------------------------------------------------------- shapes
struct MeshInst {
  GeomKind kind = GEOM_MESH_FULL;
  std::vector<V3> pos, nor;
  std::vector<float> uv;      // 2 per vertex
  std::vector<int> tri;       // 3 per triangle
  std::vector<V3> mot;        // per-vertex motion ("motions", Sphere dPdt): empty when static
  std::vector<V3> tanX, tanY; // per-vertex tangents ("tangent_x" / "tangent_y"): empty when absent
  bool cull = false;
  V3 Ng = v3s(0.f);           // GEOM_TRIANGLE: normalize(cross(v2-v0, v1-v0))
  std::shared_ptr<const MeshInst> transform(const A3& xfm) const;
};
struct ShapeObj : Object {
  std::shared_ptr<const MeshInst> inst;
  explicit ShapeObj(const std::string& t) : Object(Kind::SHAPE, t) {}
  void commit() override;
};

// ---------------------------------------------------------------- lights
struct LightInst {
  LightType type = LIGHT_AMBIENT;
  V3 L = v3s(0.f);
  V3 v0 = v3s(0.f), v1 = v3s(0.f), v2 = v3s(0.f), e1 = v3s(0.f), e2 = v3s(0.f), Ng = v3s(0.f);
  A3 l2w = a3_identity(), w2l = a3_identity();
  std::shared_ptr<ImageObj> image;
  // HDRI importance distribution (lights/hdrilight.cpp:35-40): yCDF/yPDF + per-row x CDF/PDF
  std::vector<float> ycdf, ypdf, xcdf, xpdf;
  int illumMask = -1, shadowMask = -1;
  float cosAngleMin = 1.f, cosAngleMax = 1.f;   // spot (spotlight.h:29-30)
  float halfAngle = 0.f, cosHalfAngle = 1.f;    // distant (distantlight.h:28-29)
  std::shared_ptr<const MeshInst> shape;  // TriangleLight::shape()
  std::shared_ptr<const LightInst> transform(const A3& xfm, int illumMask, int shadowMask) const;
  bool precompute() const { return type == LIGHT_HDRI; }
};
struct LightObj : Object {
  std::shared_ptr<const LightInst> inst;
  explicit LightObj(const std::string& t) : Object(Kind::LIGHT, t) {}
  void commit() override;
};

// ---------------------------------------------------------------- primitives / scene
struct PrimitiveObj : Object {
  std::shared_ptr<ShapeObj> shapeHandle;
  std::shared_ptr<LightObj> lightHandle;
  std::shared_ptr<MaterialObj> materialHandle;
  std::shared_ptr<const MeshInst> shape;
  std::shared_ptr<const LightInst> light;
  std::shared_ptr<const MaterialInst> material;
  A3 transform = a3_identity();
  bool faceCamera = false;
  int illumMask = -1, shadowMask = -1;
  PrimitiveObj() : Object(Kind::PRIMITIVE, "primitive") {}
  void commit() override;
};

// One world-space primitive after rtSetPrimitive (api/scene_flat.h:48-58)
struct ScenePrim {
  std::shared_ptr<const MeshInst> shape;       // world space
  std::shared_ptr<const LightInst> light;      // world space
  std::shared_ptr<const MaterialInst> material;
  int illumMask = -1, shadowMask = -1;
  bool faceCamera = false;
  std::shared_ptr<PrimitiveObj> prim;          // for yrtExportFrame
};

struct GpuScene;  // scene_gpu.h
struct SceneObj : Object {
  std::vector<std::shared_ptr<ScenePrim>> slots;
  std::shared_ptr<GpuScene> gpu;
  // copies of `gpu` on the other HIP devices of a multi-GPU device (by HIP device id),
  // re-made when the scene is rebuilt or refit (device.cpp scene_on)
  std::map<int, std::shared_ptr<GpuScene>> replicas;
  explicit SceneObj(const std::string& t) : Object(Kind::SCENE, t) {}
  void commit() override;
};

// ---------------------------------------------------------------- camera / renderer / fb
struct CameraObj : Object {
  GpuCamera cam;
  explicit CameraObj(const std::string& t) : Object(Kind::CAMERA, t) {}
  void commit() override;
};

struct ToneMapperObj : Object {
  float gamma = 1.f;
  bool vignetting = false;
  explicit ToneMapperObj(const std::string& t) : Object(Kind::TONEMAPPER, t) {}
  void commit() override;
};

struct RendererStatusC {
  int state;       // 0 Inactive, 1 Rendering, 2 Done (device/device.h:335-347)
  float progress;
};
typedef void (*YrtStatusCallback)(const RendererStatusC* status, void* user);

struct RendererObj : Object {
  bool debug = false;
  int maxDepth = 10, rrDepth = 5, spp = 1, sets = 64;
  float minContribution = .02f, epsilon = 32.f * kUlp, tMaxShadowRay = INFINITY, tMaxShadowJitter = .15f;
  V3 up = v3(0.f, 1.f, 0.f);
  std::string filter = "bspline";
  std::shared_ptr<ImageObj> backplate;  // pathtraceintegrator.cpp:32, used at :80-84
  std::atomic<bool>* stopFlag = nullptr;
  void* statusCallback = nullptr;   // RendererStatusCallback* (C++ ref) or YrtStatusCallback
  void* statusUser = nullptr;
  int iteration = 0;
  explicit RendererObj(const std::string& t) : Object(Kind::RENDERER, t) {}
  void commit() override;
};

enum FbFormat { FB_RGB8 = 0, FB_RGBA8 = 1, FB_RGB_FLOAT32 = 2, FB_RGBA_FLOAT32 = 3 };
// Host pixels of a framebuffer: page-locked when the device has a GPU, so the per-frame
// write-back (a 12-face C4 cube is 85 MB of RGB8) runs at DMA speed instead of staging
// through pageable memory; zero-filled either way.
struct HostPixels {
  uint8_t* p = nullptr;
  size_t bytes = 0;
  bool pinned = false;
  HostPixels(size_t n, bool pin) : bytes(n) {
    if (pin && hipHostMalloc((void**)&p, n ? n : 1, hipHostMallocDefault) == hipSuccess) pinned = true;
    else p = (uint8_t*)malloc(n ? n : 1);
    if (!p) throw std::bad_alloc();
    memset(p, 0, n);
  }
  ~HostPixels() {
    if (pinned) (void)hipHostFree(p);
    else free(p);
  }
  HostPixels(const HostPixels&) = delete;
  HostPixels& operator=(const HostPixels&) = delete;
};

struct FrameBufferObj : Object {
  FbFormat format = FB_RGB8;
  int width = 0, height = 0, depth = 1, cur = 0;
  size_t stride = 0;
  std::vector<std::unique_ptr<HostPixels>> host;  // one per swapchain buffer (or user pointers)
  std::vector<void*> userPtrs;
  std::vector<float> accu;                 // AccuBuffer (x,y,z,w) per pixel
  // A frame still on the device (per buffer id): rtRenderFrame leaves it in HBM and
  // rtMapFrameBuffer copies it to the host pixels on first access (device.cpp fb_read_back).
  struct Pending {
    std::shared_ptr<void> keep;  // the device block holding the frame (kept alive until read)
    const void* src = nullptr;   // RGB8 rows (RGB8 framebuffers) or RGB float32 (the others)
    int hipDevice = 0;
  };
  std::vector<Pending> pending;
  explicit FrameBufferObj(const std::string& t) : Object(Kind::FRAMEBUFFER, t) {}
  void* buffer(int id) { return userPtrs.size() ? userPtrs[id] : host[id]->p; }
};

}  // namespace yrt
