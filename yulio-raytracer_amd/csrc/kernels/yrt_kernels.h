// yrt_kernels.h — launch interface of the wavefront path tracer (C++ linkage, used by the
// device plugin's host code only; the exported C ABI lives in include/yrt_device.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../common/yrt_gpu_types.h"

namespace yrt {

struct SceneView {
  const GpuNode* nodes;
  const GpuTri* tris;
  const int* triGeom;
  const int4* indices;
  const float4* positions;
  const float4* normals;
  const float2* texcoords;
  const GpuGeom* geoms;
  const GpuMaterial* materials;
  const GpuTexture* textures;
  const GpuImage* images;
  const uint8_t* texels;
  const GpuLight* lights;
  const int* envLights;
  const float* hdriDist;
  int numLights, numEnvLights, numNodes, numTris;
};

struct FrameView {
  const GpuRenderParams* rp;   // device copy
  const GpuCamera* cam;        // device copy
  const float* samples;        // [numDims][numRecords]
  const float* lightSamples;   // [numRecords][numLightSlots][8]
  const uint8_t* pixelSets;    // W*H set index per pixel
  int numRecords, numLightSlots;
};

// Wavefront state for one batch of P = numPixels * spp paths (SoA, device memory).
struct PathBuffers {
  int* qPath[2];
  float4* qOrg[2];   // xyz, tnear
  float4* qDir[2];   // xyz, tfar
  float4* hit;       // t, u, v, tri (bits)
  float4* thr;       // per path throughput
  float4* L;         // per path radiance
  int* meta;         // per path: depth | ignoreVL<<8 | unbent<<9
  int* shFirst;      // per (queue entry, light): shadow-ray slot or -1
  float4* sOrg;      // shadow rays
  float4* sDir;
  float4* sContrib;
  int* sOcc;
  unsigned* counters;  // [depth*4 + 0] queue size at depth, [depth*4+1] shadow rays at depth
  int capacity;        // max paths
  int shadowCapacity;  // max shadow rays per depth
};

struct BatchInfo {
  int firstTile;       // first tile of the batch, counted in this shard's tile sequence
  int numPixels;       // pixels in the batch (multiple of 256, may overhang the image)
  int tileStride;      // shard: image tile = tileOffset + localTile * tileStride
  int tileOffset;
};

// Kernel launchers (kernels/pathtrace.hip)
void launch_pixel_sets(const FrameView& fv, uint8_t* pixelSets, int width, int height, int sets, hipStream_t s);
void launch_raygen(const FrameView& fv, const PathBuffers& pb, const BatchInfo& bi, hipStream_t s);
void launch_trace_closest(const SceneView& sv, const float4* org, const float4* dir, const unsigned* count,
                          int maxCount, float4* hit, hipStream_t s);
void launch_trace_any(const SceneView& sv, const float4* org, const float4* dir, const unsigned* count, int maxCount,
                      int* occluded, hipStream_t s);
void launch_shade(const SceneView& sv, const FrameView& fv, const PathBuffers& pb, const BatchInfo& bi, int depth,
                  hipStream_t s);
void launch_shadow_resolve(const PathBuffers& pb, int depth, int numLights, hipStream_t s);
void launch_resolve_pixels(const FrameView& fv, const PathBuffers& pb, const BatchInfo& bi, float* fbFloat,
                           uint8_t* fbRGB8, int rgb8Stride, float4* accu, int accumulate, hipStream_t s);
void launch_pick(const SceneView& sv, const GpuCamera* cam, float x, float y, float4* out, hipStream_t s);
void launch_debug_render(const SceneView& sv, const FrameView& fv, int maxDepth, int spp, int numTiles, float* fbFloat,
                         uint8_t* fbRGB8, int rgb8Stride, hipStream_t s);

}  // namespace yrt
