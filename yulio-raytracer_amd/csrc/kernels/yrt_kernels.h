// yrt_kernels.h — launch interface of the wavefront path tracer (C++ linkage, used by the
// device plugin's host code only; the exported C ABI lives in include/yrt_device.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../common/yrt_gpu_types.h"
#include "../common/yrt_qnode.h"
#include "yrt_traverse.h"

namespace yrt {

struct SceneView {
  const GpuNode* nodes;
  const GpuQNode* qnodes;  // the same tree, 64-B quantized nodes (any-hit traversal)
  const GpuTri* tris;
  const int* triGeom;
  const int4* indices;
  const float4* positions;
  const float4* normals;
  const float2* texcoords;
  const GpuGeom* geoms;
  const GpuGeomRec* geomRecs;  // per geometry: geometry + material + tex[0] descriptor (k_shade)
  const GpuTriShade* triShade; // per triangle: k_shade's postIntersect record
  const GpuMaterial* materials;
  const GpuTexture* textures;
  const GpuImage* images;
  const uint8_t* texels;
  const uint8_t* texQuads;  // per 8-bit texel i: texels i, i+1, i+W, i+W+1 (16 B at 4x its texel offset)
  const GpuLight* lights;
  const int* envLights;
  const int* directLights;  // the lights whose samples can carry radiance (Device::render), in light order
  const float* hdriDist;
  const float4* media;  // medium table (transmission.rgb, eta); [0] = vacuum (materials/medium.h)
  const float4* motions;            // per vertex (moving scenes only, else null)
  const float4* tangents;           // per vertex: tangent_x, tangent_y (meshes with tangents, else null)
  const GpuTriMotion* triMotion;    // per leaf slot (moving scenes only, else null)
  int* traceSpill;   // deep traversal-stack entries: YRT_TRACE_SPILL_INTS ints
  int numLights, numEnvLights, numNodes, numTris;
  int numDirectLights;  // k_shade's direct-light loop and the per-path shadow slots
  int numEnvZero;       // environment lights left out of envLights: radiance exactly 0 (scene_gpu.cpp)
  int numEnvDir;        // envLights whose Le depends on the direction (HDRI, distant; not ambient)
};

// Trace grid: 16384 blocks (swept with 128-lane blocks; with 64-lane blocks 32768 is -0.5 %),
// several times the resident blocks (256 CUs x ~9),
// so a CU always has a queued block when one drains and the other lane's kernels interleave
// (sweep 1024..16384 blocks: 16384 best, +1.2 % over 8192 with the 32-entry LDS stack).
#ifndef YRT_TRACE_GRID
#define YRT_TRACE_GRID 16384
#endif
// spilled stack entries per lane: the one-ray kernels' (YRT_STACK_DEPTH - ring), or two ray slots'
// of k_occluded2 (one 64-lane wave per block, YRT_TRACE_GRID blocks at most)
#define YRT_SPILL_1 (YRT_STACK_DEPTH - YRT_LDS_STACK_MIN)
#define YRT_SPILL_2 (YRT_ANY2 ? 2 * (YRT_STACK_DEPTH - YRT_ANY2_LDS) : 0)
#define YRT_TRACE_SPILL_INTS \
  ((size_t)YRT_TRACE_GRID * (YRT_TRACE_BLOCK > 64 ? YRT_TRACE_BLOCK : 64) * (YRT_SPILL_1 > YRT_SPILL_2 ? YRT_SPILL_1 : YRT_SPILL_2))

struct FrameView {
  const GpuRenderParams* rp;   // device copy
  const GpuCamera* cam;        // device copy: one per frame (rp->numFrames)
  const float* samples;        // [numDims][numRecords]
  const float* lightSamples;   // [numRecords][numLightSlots][8]
  const uint8_t* pixelSets;    // W*H set index per pixel
  int numRecords, numLightSlots;
  GpuImage backplate;           // PathTraceIntegrator backplate (offset 0 in backplateTexels)
  const uint8_t* backplateTexels;  // null: none
};

// Queues are split into YRT_QSEGS segments, each with its own append counter on its own
// 256-B line: one returning atomic on a single word saturates near 88 M/s on MI355X
// (MI355X_MICROARCH.md, 'dequeue'), which bounded raygen/shade with one counter per queue.
// Input item q appends into segment (q/64) % YRT_QSEGS, so a segment never receives more
// than capacity/YRT_QSEGS + 64 items per input item's fan-out. Consumers map a logical index
// to (segment, offset) through the exclusive prefix of the segment counts.
#define YRT_QSEGS 32
#define YRT_QCSTRIDE 64  // unsigned words between two segment counters
// counters[((level * 2 + kind) * YRT_QSEGS + seg) * YRT_QCSTRIDE], kind 0 = closest queue
// entering depth `level`, kind 1 = shadow rays emitted at depth `level`; except that the
// closest queue entering depth level > 0 counts in the word after the shadow counter of depth
// level - 1 (same segment).
inline __host__ __device__ size_t qcounter_index(int level, int kind, int seg) {
  if (kind == 0 && level > 0) return ((size_t)((level - 1) * 2 + 1) * YRT_QSEGS + seg) * YRT_QCSTRIDE + 1;
  return ((size_t)(level * 2 + kind) * YRT_QSEGS + seg) * YRT_QCSTRIDE;
}
// counter words of a batch of depth levels 0 .. levels - 1
inline __host__ __device__ size_t qcounter_words(int levels) {
  return (size_t)(levels * 2) * YRT_QSEGS * YRT_QCSTRIDE;
}
inline __host__ __device__ int qseg_capacity(long long items) {
  return (int)(((items + 63) / 64 + YRT_QSEGS - 1) / YRT_QSEGS * 64 + 64);
}

// Wavefront state for one batch of P = numPixels * spp paths (SoA, device memory).
// Path state travels with the queue entry (coalesced in queue order); radiance lives in the
// path-indexed pathL and is only touched when a vertex adds emission or direct light.
struct PathBuffers {
  int* qPath[2];
  float4* qOrg[2];   // xyz, tnear
  float4* qDir[2];   // xyz, tfar
  float4* qThr[2];   // throughput xyz, w = meta bits: depth | ignoreVL<<8 | unbent<<9
  float4* hit;       // t, u, v, tri (bits), per closest-queue slot
  int* hitGeom;      // the hit triangle's geometry id, per closest-queue slot: k_shade loads its
                     // geometry record beside the shading record instead of after it
  float4* pathL;     // per path id: radiance so far (emission and unoccluded direct light are
                     // read-modify-written in the reference's order; one writer per path at a time)
  int* shFirst;      // per (queue slot, light): shadow-ray slot or -1
  float4* sOrg;      // shadow rays: origin xyz, tnear
  float4* sDir;
  float4* sContrib;
  int* sOcc;
  float* qTime[2];   // moving scenes: ray time per closest-queue slot (else null)
  float* sTime;      // moving scenes: ray time per shadow slot (else null)
  unsigned* counters;  // segment counters, see qcounter_index
  int capacity;        // max paths
  int segCap;          // closest-queue slots per segment (qPath/qOrg/qDir/hit: YRT_QSEGS * segCap)
  int shSegCap;        // shadow slots per segment (sOrg/sDir/sContrib/sOcc: YRT_QSEGS * shSegCap)
  // 1 (one light): k_shade stores each shadow ray's path id in sContrib.w and k_trace<true>
  // adds the contribution to pathL itself when the ray is unoccluded — one writer per path,
  // so the sum is deterministic and in the reference's order; k_shadow_resolve is not
  // launched. 0: sOcc + shFirst + k_shadow_resolve (several lights, light order kept).
  int fuseShadow;
};

// Fused shadow resolve: sContrib.w = path id (bits) whose pathL receives the contribution.
struct ShadowFuse {
  const float4* contrib;  // null: not fused, k_trace<true> writes occlusion flags
  float4* pathL;
};

struct BatchInfo {
  int firstTile;       // first tile of the batch, counted in this shard's tile sequence
  int numPixels;       // pixels in the batch (multiple of 256, may overhang the image)
  int tileStride;      // shard: image tile = tileOffset + localTile * tileStride
  int tileOffset;
  FastDiv divPixels;   // fastdiv_make(numPixels): path id -> (sample, batch pixel)
};

// Camera rays generated inside the closest-hit kernel (k_trace<false, false, PRIM>):
// depth 0 without a raygen pass. A lane takes the batch's next path id, computes its camera ray
// as k_raygen does, traces it and, when it is done, either appends it with its hit to the
// depth-0 queue (qPath/qOrg/qDir/hit, the segment of its path id's 64-group) or, on a miss,
// writes the path's radiance: the environment's (GpuRenderParams::missL; direction-independent environment
// lights only, k_shade's depth-0 miss branch). Paths outside the image get radiance 0.
struct PrimaryRays {
  FrameView fv;
  BatchInfo bi;
  int* qPath;
  float4* qOrg;
  float4* qDir;
  float4* pathL;
  unsigned* counts;   // depth-0 closest-queue counters: qcounter_index(0, 0, 0), segments YRT_QCSTRIDE apart
  int segCap;
  unsigned* traced;   // camera rays traced (valid paths); one atomic per wave
  long long numPaths; // numPixels * spp (grid size)
};

// Kernel launchers (kernels/pathtrace.hip)
void launch_pixel_sets(const FrameView& fv, uint8_t* pixelSets, int width, int height, int sets, hipStream_t s);
void launch_raygen(const FrameView& fv, const PathBuffers& pb, const BatchInfo& bi, hipStream_t s);
// counts: first segment counter of the queue (segments YRT_QCSTRIDE apart), numSegs segments
// of segCap slots; hit/occluded are indexed by physical slot.
// Every launch gets the full grid for the queue's capacity: the kernels grid-stride over the
// device-side count and idle waves exit at once.
// time (moving scenes): per-slot ray time (Ray::time); null: static scene (or time 0)
// hitGeom (optional): the hit triangle's geometry id per slot
void launch_trace_closest(const SceneView& sv, const float4* org, const float4* dir, const unsigned* counts,
                          int numSegs, int segCap, float4* hit, hipStream_t s, const float* time = nullptr,
                          int* hitGeom = nullptr);
// depth 0 of a batch: camera rays generated, traced and queued (hits) or resolved (misses) in
// one kernel, see PrimaryRays; replaces launch_raygen + the depth-0 launch_trace_closest for
// static scenes without a backplate or direction-dependent environment lights
void launch_trace_primary(const SceneView& sv, const PrimaryRays& pr, float4* hit, int* hitGeom, hipStream_t s);
void launch_trace_any(const SceneView& sv, const float4* org, const float4* dir, const unsigned* counts, int numSegs,
                      int segCap, int* occluded, hipStream_t s, const ShadowFuse* fuse = nullptr,
                      const float* time = nullptr);
// materialMask: bit MAT_x set for every material type the scene uses (selects a specialized
// instantiation of the shade kernel)
void launch_shade(const SceneView& sv, const FrameView& fv, const PathBuffers& pb, const BatchInfo& bi, int depth,
                  unsigned materialMask, hipStream_t s);
void launch_shadow_resolve(const PathBuffers& pb, int depth, int numLights, hipStream_t s);
void launch_resolve_pixels(const FrameView& fv, const PathBuffers& pb, const BatchInfo& bi, float* fbFloat,
                           uint8_t* fbRGB8, int rgb8Stride, float4* accu, int accumulate, hipStream_t s);
// YRT_PROFILE builds only: SIMD-utilization counters of k_trace (see pathtrace.hip); -1 otherwise
int trace_profile(unsigned long long* out8, int reset);
// Debug capture: per-sample radiance of pixel id (y * width + x) of frame `frame` written to
// out[s] by the next resolves (pixelId -1: off)
int debug_pixel_capture(int pixelId, int frame, float4* out, int capacity);
// Arithmetic self-check of the correctly rounded fast reciprocal (rcp_rn): see pathtrace.hip
int check_math(int fn, unsigned long long* host2);
int check_math_table(int fn, const uint16_t* table2048, unsigned long long* host2);
// Multi-GPU gather (device.cpp): the pixels of the tiles of one shard (job tile =
// tileOffset + j * tileStride, j < numTiles, over numFrames stacked frames of tilesPerFrame
// tiles) as a slab of numTiles * 256 elements in tile order j and scan order within the tile;
// unpack scatters a slab back into the frames. Elements are 32-bit RGB8 words (rgb8 = 1: the
// framebuffer is RGB8, a quarter of the bytes) or float4 (rgb float, w = the RGB8 bytes).
// Pixels outside the image are zero in the slab and skipped on unpack.
struct SlabLayout {
  int width, height, rgb8Stride, tilesPerFrame;
  int tileOffset, tileStride, rgb8, pad;
};
inline size_t slab_element_bytes(int rgb8) { return rgb8 ? 4 : 16; }
void launch_pack_tiles(const float* fbFloat, const uint8_t* fbRGB8, const SlabLayout& L, int numTiles, void* slab,
                       hipStream_t s);
void launch_unpack_tiles(const void* slab, float* fbFloat, uint8_t* fbRGB8, const SlabLayout& L, int numTiles,
                         hipStream_t s);
void launch_pick(const SceneView& sv, const GpuCamera* cam, float x, float y, float4* out, hipStream_t s);
// BVH refit after faceCamera updates: rewrite triangles [firstTri, firstTri+numTris) (global
// ids) from the vertex buffer in every leaf slot that references them (leafSlots[leafStart[g]
// .. leafStart[g+1])), then refit one tree level of nodes (call deepest level first)
void launch_refit_tris(GpuTri* tris, GpuTriShade* triShade, const int4* indices, const float4* positions,
                       const float4* normals, const int* leafStart, const int* leafSlots, int firstTri, int numTris,
                       hipStream_t s);
void launch_refit_nodes(GpuNode* nodes, const GpuTri* tris, const int4* indices, const float4* positions,
                        const int* levelNodes, int count, hipStream_t s);
// the quantized copy of every node (yrt_quantize_node), after a refit of the float nodes
void launch_quantize_nodes(const GpuNode* nodes, GpuQNode* qnodes, int count, hipStream_t s);
// bytes per node of the closest-hit / any-hit traversal as built (YRT_QNODES_CLOSEST / _ANY)
int trace_node_bytes(bool anyHit);
// whether the closest-hit kernels store each hit's geometry id (YRT_HIT_GEOM)
bool trace_hit_geom();
void launch_debug_render(const SceneView& sv, const FrameView& fv, int maxDepth, int spp, int numTiles, float* fbFloat,
                         uint8_t* fbRGB8, int rgb8Stride, hipStream_t s);

}  // namespace yrt
