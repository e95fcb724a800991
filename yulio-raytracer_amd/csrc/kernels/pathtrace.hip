// pathtrace.hip — wavefront path tracer for gfx950 (MI355X).
//
// The reference's per-pixel integrator (integrators/pathtraceintegrator.cpp:50-217 called
// from renderers/integratorrenderer.cpp:118-185) becomes, per batch of pixels x spp paths:
//
//   k_raygen -> for depth d: k_trace_closest -> k_shade -> k_trace_any -> k_shadow_resolve
//            -> k_resolve_pixels
//
// Queues are compacted with one wave-wide ballot/prefix + one atomic per wave.  Per-path
// radiance is accumulated in the same order as the reference's sequential loop (env or
// emission first, then the direct-light terms in light order), and the pixel sum over
// samples runs s = 0..spp-1, so results do not depend on queue order.
//
// Wave64: every cross-lane primitive below is written for 64 lanes (ballot is 64-bit).

#include <hip/hip_runtime.h>
#include <stdio.h>

#include <mutex>
#include <set>

#include "../common/yrt_tile_scatter.h"
#include "yrt_kernels.h"
#include "yrt_shade.h"
#include "yrt_traverse.h"

namespace yrt {

#ifndef YRT_BLOCK
#define YRT_BLOCK 64  // raygen / shade / resolve blocks: one wave (128: +0.5 %, 64: +0.9 % over 256, two lanes)
#endif

// ---------------------------------------------------------------- wave helpers
__device__ __forceinline__ int lane_id() { return __lane_id(); }
// 0.0f computed where it is used (volatile: not hoisted out of a loop)
__device__ __forceinline__ float opaque_zero() {
  float z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
  return z;
}
// set bits of a wave mask below this lane (v_mbcnt: no per-lane mask register kept live)
__device__ __forceinline__ unsigned lanes_below(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

// Reserve k slots (k >= 0 per lane) in *counter; returns this lane's first slot.
// Every lane of the wave must call it (no divergent callers).
__device__ __forceinline__ unsigned wave_reserve(unsigned* counter, unsigned k) {
  const int lane = lane_id();
  unsigned incl = k;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    unsigned y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  const unsigned total = __shfl(incl, 63, 64);
  unsigned base = 0;
  if (lane == 0 && total) base = atomicAdd(counter, total);
  base = __shfl(base, 0, 64);
  return base + incl - k;
}

// Ballot of a bool (the builtin on the i1 lane mask; HIP's __ballot takes an int).
__device__ __forceinline__ unsigned long long ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

__device__ __forceinline__ unsigned wave_append(unsigned* counter, bool pred, bool& got) {
  const unsigned long long mask = ballot(pred);
  got = pred;
  if (mask == 0) return 0;
  const int lane = lane_id();
  const int leader = __ffsll((long long)mask) - 1;
  unsigned base = 0;
  if (lane == leader) base = atomicAdd(counter, (unsigned)__popcll(mask));
  base = __shfl(base, leader, 64);
  return base + (unsigned)__popcll(mask & ((1ull << lane) - 1ull));
}

// ---------------------------------------------------------------- segmented queues
struct QMap {
  unsigned pre[YRT_QSEGS + 1];  // exclusive prefix of the segment counts; pre[numSegs] = total
};

// Every thread of the block must call it (barrier inside).
__device__ __forceinline__ void qmap_load(QMap& m, const unsigned* counts, int numSegs) {
  if (threadIdx.x == 0) {
    unsigned c[YRT_QSEGS];
#pragma unroll
    for (int k = 0; k < YRT_QSEGS; ++k) c[k] = k < numSegs ? counts[(size_t)k * YRT_QCSTRIDE] : 0u;
    unsigned acc = 0;
#pragma unroll
    for (int k = 0; k < YRT_QSEGS; ++k) {
      m.pre[k] = acc;
      acc += c[k];
    }
    m.pre[YRT_QSEGS] = acc;
  }
  __syncthreads();
}

// Physical slot of logical queue index q < total.
__device__ __forceinline__ int qmap_phys(const QMap& m, int segCap, unsigned q) {
  int lo = 0;
#pragma unroll
  for (int step = YRT_QSEGS / 2; step > 0; step >>= 1)
    if (m.pre[lo + step] <= q) lo += step;
  return lo * segCap + (int)(q - m.pre[lo]);
}

// Segment that input item q appends into (uniform across a wave: q >> 6 is).
__device__ __forceinline__ int qseg_of(unsigned q) { return (int)((q >> 6) % YRT_QSEGS); }

// ---------------------------------------------------------------- reference RNG
// Park-Miller minimal standard + Bays-Durham shuffle (common/math/random.h:24-78).
struct DevRandom {
  int seed, state;
  int table[32];
  __device__ void setSeed(int s) {
    const int a = 16807, m = 2147483647, q = 127773, r = 2836;
    if (s == 0) seed = 1;
    else if (s < 0) seed = -s;
    else seed = s;
    for (int j = 32 + 7; j >= 0; j--) {
      int k = seed / q;
      seed = a * (seed - k * q) - r * k;
      if (seed < 0) seed += m;
      if (j < 32) table[j] = seed;
    }
    state = table[0];
  }
  __device__ int getInt() {
    const int a = 16807, m = 2147483647, q = 127773, r = 2836;
    int k = seed / q;
    seed = a * (seed - k * q) - r * k;
    if (seed < 0) seed += m;
    int j = state / (1 + (2147483647 - 1) / 32);
    state = table[j];
    table[j] = seed;
    return state;
  }
  __device__ int getInt(int limit) { return getInt() % limit; }
  __device__ float getFloat() { return fminf(getInt() / 2147483647.0f, 1.0f - kUlp); }
};

// Counter-based replacement for C rand() in the shadow-ray jitter
// (pathtraceintegrator.cpp:151; the reference calls rand() from worker threads, so it
// is not reproducible). Same function in oracle/yrt_oracle.c: hash_u01.
__device__ __forceinline__ uint32_t mix32(uint32_t h) {
  h ^= h >> 16; h *= 0x7feb352dU; h ^= h >> 15; h *= 0x846ca68bU; h ^= h >> 16;
  return h;
}
__device__ __forceinline__ float hash_u01(uint32_t seed, uint32_t pixel, uint32_t sample, uint32_t depthLight) {
  uint32_t h = mix32(seed ^ 0x9e3779b9U);
  h = mix32(h ^ pixel);
  h = mix32(h ^ (sample * 0x85ebca6bU));
  h = mix32(h ^ (depthLight * 0xc2b2ae35U));
  return (float)(h >> 8) * (1.0f / 16777216.0f);
}

// Records every lane of a wave reads at one address (the render parameters, the frame's
// camera) are read through the constant address space: scalar loads into SGPRs instead of
// per-lane vector loads held in VGPRs (the kernels never write them).
#define YRT_CONST __attribute__((address_space(4)))
template <class T>
__device__ __forceinline__ const YRT_CONST T& const_ref(const T* p) {
  return *(const YRT_CONST T*)p;
}

template <class F>
__device__ __forceinline__ V3 ld3(const F* p) { return v3(p[0], p[1], p[2]); }
__device__ __forceinline__ V3 ld3(const float4& p) { return v3(p.x, p.y, p.z); }
template <class F>
__device__ __forceinline__ A3 ldA3(const F* m) {
  return a3(l3(v3(m[0], m[1], m[2]), v3(m[3], m[4], m[5]), v3(m[6], m[7], m[8])), v3(m[9], m[10], m[11]));
}

// ---------------------------------------------------------------- cameras
// PinHoleCamera::ray (cameras/pinholecamera.h:23-25)
// StereoCubeCamera::ray (cameras/StereoCubeCamera.h:68-161)
// DepthOfFieldCamera::ray (cameras/depthoffieldcamera.h:20-26); (lx, ly) = the lens sample
template <class CAM>
__device__ __forceinline__ void pinhole_ray(const CAM& cam, float fx, float fy, V3& org, V3& dir) {
  A3 p2w = ldA3(cam.p2w[0]);
  org = p2w.p;
  dir = normalize(fx * p2w.l.vx + (1.0f - fy) * p2w.l.vy + p2w.l.vz);
}
// TOEIN = false drops the toe-in stereo branch: the fused depth-0 trace kernel takes no toe-in
// camera (the host routes those frames through k_raygen). Its two rotations about per-ray
// points and the reference's rcp/rsqrt sequences need ~40 more VGPRs than the rest of the
// camera code (k_raygen 37 -> 76), which at the fused kernel's 96-VGPR cap spilled 60-76 B
// into its traversal loop.
template <bool TOEIN = true, class CAM>  // GpuCamera, or a YRT_CONST one (scalar loads)
__device__ void camera_ray(const CAM& cam, float fx, float fy, V3& org, V3& dir, float lx = 0.f,
                           float ly = 0.f) {
  if (cam.type == CAM_PINHOLE) {
    pinhole_ray(cam, fx, fy, org, dir);
    return;
  }
  if (cam.type == CAM_DOF) {
    const A3 p2w = ldA3(cam.p2w[0]), l2w = ldA3(cam.p2w[1]);
    const float lensRadius = cam.xyzStraight[0], focalDistance = cam.xyzStraight[1];
    // uniformSampleDisk (samplers/shapesampler.h:187-191)
    const float r = sqrtf(lx), theta = kTwoPi * ly;
    const V3 begin = xfmPoint(l2w, v3(lensRadius * r * yrt_cosf(theta), lensRadius * r * yrt_sinf(theta), 0.0f));
    const V3 end = p2w.p + focalDistance * (fx * p2w.l.vx + (1.0f - fy) * p2w.l.vy + p2w.l.vz);
    org = begin;
    dir = normalize(end - begin);
    return;
  }
  const A3 pixel2world = ldA3(cam.p2w[0]);
  const int eyeCubeFaceIndex = cam.cubeFaceIndex % 6;
  const float yPixel = 1.0f - fy;
  A3 p2w = ldA3(cam.p2w[eyeCubeFaceIndex]);
  const V3 xyzStraight = ld3(cam.xyzStraight);
  float theta = 0.f;
  float absoluteVerticalAngle = 0.f;
  if (eyeCubeFaceIndex <= 3) {
    const V3 xDir = normalize(fx * pixel2world.l.vx + .5f * pixel2world.l.vy + pixel2world.l.vz);
    theta = yrt_acosf(clampf(dot(xDir, xyzStraight), -1.f, 1.f)) * signf_(fx - .5f);
    const V3 yDir = normalize(.5f * pixel2world.l.vx + yPixel * pixel2world.l.vy + pixel2world.l.vz);
    const float yAngle = rad2deg(yrt_acosf(clampf(dot(yDir, xyzStraight), -1.f, 1.f))) * signf_(yPixel - .5f);
    absoluteVerticalAngle = fabsf(yAngle);
  } else {
    const V3 xyDir = v3(fx - .5f, yPixel - .5f, 0.f);
    const V3 xyDirNorm = normalize(xyDir);
    const V3 xyUp = v3(0.f, eyeCubeFaceIndex == 4 ? -1.f : 1.f, 0.f);
    theta = yrt_acosf(clampf(dot(xyDirNorm, xyUp), -1.f, 1.f)) * signf_(fx - .5f);
    const V3 xyzDir = normalize(fx * pixel2world.l.vx + yPixel * pixel2world.l.vy + pixel2world.l.vz);
    const float xyzAngle = rad2deg(yrt_acosf(clampf(dot(xyzDir, xyzStraight), -1.f, 1.f)));
    absoluteVerticalAngle = 90.f - fabsf(xyzAngle);
  }
  float eyeOffset = cam.eyeSeparation * (cam.cubeFaceIndex < 6 ? -.5f : .5f);
  if (absoluteVerticalAngle > cam.falloffAngle) {
    const float coef = 1.f - smoothstepf(0.f, 1.f, smoothstepf(cam.falloffAngle, 90.f, absoluteVerticalAngle));
    eyeOffset *= coef;
  }
  if (TOEIN && cam.toeIn) {
    p2w = mul(p2w, a3_translate(v3(eyeOffset, 0.f, 0.f)));
    const V3 origin = ld3(cam.origin), up = ld3(cam.up);
    const A3 rayRotationSpace = a3_rotate_about(origin, up, theta);
    const V3 rayOrigin = mul(rayRotationSpace, p2w).p;
    const float toeInCorrection = -yrt_atanf(eyeOffset * cam.rcpZeroParallaxDistance);
    p2w = mul(a3_rotate_about(rayOrigin, up, toeInCorrection), p2w);
    org = rayOrigin;
    dir = normalize(fx * p2w.l.vx + yPixel * p2w.l.vy + p2w.l.vz);
    return;
  }
  // Without toe-in the same products with the pixel-independent terms taken from the camera
  // record (objects.cpp): translate(origin) * rotate(up, theta) * translate(-origin) has the
  // rotation as its linear part (the identity factors' ones and zeros only add exact zeros),
  // and its point is rotation * (-origin) + rotP; the shifted eye point is
  // p2w.p + eyeOffset * p2w.vx plus the translation's zero products.
  const auto* R = cam.rot;  // u.xyz, uxx, 1-uxx, uyy, 1-uyy, uzz, 1-uzz, uxy, uxz, uyz
  const float sn = yrt_sinf(theta), cs = yrt_cosf(theta), omc = 1 - cs;
  const V3 rvx = v3(R[3] + R[4] * cs, R[9] * omc + R[2] * sn, R[10] * omc - R[1] * sn);
  const V3 rvy = v3(R[9] * omc - R[2] * sn, R[5] + R[6] * cs, R[11] * omc + R[0] * sn);
  const V3 rvz = v3(R[10] * omc + R[1] * sn, R[11] * omc - R[0] * sn, R[7] + R[8] * cs);
  // the rotation's products through the fused LinearSpace3 * v helper, as the oracle's lmul
  const L3 rot = l3(rvx, rvy, rvz);
  const V3 bp = mul(rot, ld3(cam.negO)) + ld3(cam.rotP);
  const auto* z = cam.zero[eyeCubeFaceIndex];
  const V3 eye = v3(eyeOffset * p2w.l.vx.x + z[0], eyeOffset * p2w.l.vx.y + z[1], eyeOffset * p2w.l.vx.z + z[2]) + p2w.p;
  org = mul(rot, eye) + bp;
  const auto* m = cam.lin[eyeCubeFaceIndex];
  dir = normalize(fx * v3(m[0], m[1], m[2]) + yPixel * v3(m[3], m[4], m[5]) + v3(m[6], m[7], m[8]));
}

// ---------------------------------------------------------------- batch pixel mapping
// Batch pixel i -> (frame f, pixel x, y). A batch holds whole 16x16 tiles of the job's tile
// sequence (all frames' tiles, frame-major); the 256 pixels of a tile are consecutive, so the
// 64 lanes of a wave (64-aligned i) always share the tile and the frame.
template <class D>  // FastDiv, or a YRT_CONST one
__device__ __forceinline__ int fastdiv(int n, const D& d) {  // n in [0, 2^31)
  return (int)((__umulhi((unsigned)n, d.mul) + (unsigned)n) >> d.shift);
}
// the tile of batch-pixel block ib = i >> 8: its frame and first pixel (false past the job)
template <class RP>
__device__ __forceinline__ bool batch_tile(const RP& rp, const BatchInfo& bi, int ib, int& x0, int& y0,
                                           int& f) {
  int tile = bi.tileOffset + (bi.firstTile + ib) * bi.tileStride;
  f = 0;
  if (tile >= rp.tilesPerFrame * rp.numFrames) return false;
  if (rp.numFrames > 1) {
    f = fastdiv(tile, rp.divTilesPerFrame);
    tile -= f * rp.tilesPerFrame;
  }
  // sharded jobs: the logical tile's image tile (common/yrt_tile_scatter.h; slab_pixel agrees)
  if (bi.tileStride > 1) tile = yrt_tile_scatter(tile, rp.tilesPerFrame);
  const int ty = fastdiv(tile, rp.divTilesX);
  x0 = (tile - ty * rp.numTilesX) * 16;
  y0 = ty * 16;
  return true;
}
template <class RP>
__device__ __forceinline__ bool batch_pixel(const RP& rp, const BatchInfo& bi, int i, int& x, int& y,
                                            int& f) {
  int x0 = 0, y0 = 0;
  if (!batch_tile(rp, bi, i >> 8, x0, y0, f)) return false;
  x = x0 + (i & 15);
  y = y0 + ((i >> 4) & 15);
  return x < rp.width && y < rp.height;
}
template <class RP>
__device__ __forceinline__ bool batch_pixel(const RP& rp, const BatchInfo& bi, int i, int& x, int& y) {
  int f;
  return batch_pixel(rp, bi, i, x, y, f);
}

__device__ __forceinline__ float samp(const FrameView& fv, int dim, int rec) {
  return fv.samples[(size_t)dim * fv.numRecords + rec];
}

// ---------------------------------------------------------------- kernels
__global__ void k_pixel_sets(const GpuRenderParams* __restrict__ rpp, uint8_t* __restrict__ sets) {
  const GpuRenderParams rp = *rpp;
  const int tile = blockIdx.x * blockDim.x + threadIdx.x;
  if (tile >= rp.numTilesX * rp.numTilesY) return;
  const int tile_x = (tile % rp.numTilesX) * 16;
  const int tile_y = (tile / rp.numTilesX) * 16;
  DevRandom rng;
  rng.setSeed(tile_x * 91711 + tile_y * 81551 + 3433 * 0);
  for (int dy = 0; dy < 16; dy++) {
    const int y = tile_y + dy;
    if (y >= rp.height) continue;
    for (int dx = 0; dx < 16; dx++) {
      const int x = tile_x + dx;
      if (x >= rp.width) continue;
      sets[(size_t)y * rp.width + x] = (uint8_t)rng.getInt(rp.sets);
    }
  }
}

__global__ __launch_bounds__(YRT_BLOCK) void k_raygen(FrameView fv, PathBuffers pb, BatchInfo bi) {
  static_assert(YRT_BLOCK <= 256 && 256 % YRT_BLOCK == 0, "a raygen block lies in one 256-pixel tile");
  const YRT_CONST GpuRenderParams& rp = const_ref(fv.rp);
  const int P = bi.numPixels * rp.spp;
  for (int base = blockIdx.x * blockDim.x; base < P; base += gridDim.x * blockDim.x) {
    // P is a multiple of 256 and base of the block size: every lane has p < P
    const int p = base + threadIdx.x;
    // the block's paths share the sample index, the tile and the frame (numPixels is a
    // multiple of 256): computed once from the block base, on the scalar unit
    const int s = fastdiv(base, bi.divPixels);
    int x0 = 0, y0 = 0, f = 0;
    const bool tileOk = batch_tile(rp, bi, (base - s * bi.numPixels) >> 8, x0, y0, f);
    const int x = x0 + (p & 15), y = y0 + ((p >> 4) & 15);
    // a pixel of the image, and the loop head of Li: depth < maxDepth and
    // max(throughput) = 1 >= minContribution
    const bool valid = tileOk && x < rp.width && y < rp.height && rp.maxDepth > 0 && !(1.0f < rp.minContribution);
    // queue slots first: the append's atomic is issued before the camera ray is computed and
    // its result is read at the stores, so its round trip overlaps the sample loads and the
    // camera arithmetic (the leader lane's counter value is broadcast after)
    const int seg = qseg_of((unsigned)base + (threadIdx.x & ~63u));
    const unsigned long long vmask = ballot(valid);
    const int leader = vmask ? __ffsll((long long)vmask) - 1 : 0;
    unsigned qbase = 0;
    if (vmask && lane_id() == leader) qbase = atomicAdd(pb.counters + qcounter_index(0, 0, seg), (unsigned)__popcll(vmask));
    if (valid) {
      const YRT_CONST GpuCamera& cam = const_ref(fv.cam + f);  // scalar loads
      const int set = fv.pixelSets[(size_t)y * rp.width + x];
      const int rec = set * rp.spp + s;
      const float fx = (float(x) + samp(fv, 0, rec)) * rp.rcpWidth;
      const float fy = (float(y) + samp(fv, 1, rec)) * rp.rcpHeight;
      V3 org, dir;
      camera_ray(cam, fx, fy, org, dir, samp(fv, 2, rec), samp(fv, 3, rec));  // sample.getLens()
      // the camera ray's throughput (1, 1, 1), its meta word (depth 0, unbent) and its zero
      // radiance are implicit at depth 0: k_shade starts from them and writes pathL of every
      // queued path, so only the paths that are not queued get their zero radiance here
      const unsigned q = seg * pb.segCap + (unsigned)__builtin_amdgcn_readlane((int)qbase, leader) +
                         (unsigned)__popcll(vmask & ((1ull << lane_id()) - 1ull));
      pb.qPath[0][q] = p;
      pb.qOrg[0][q] = make_float4(org.x, org.y, org.z, 0.f);
      pb.qDir[0][q] = make_float4(dir.x, dir.y, dir.z, __int_as_float(0x7f800000));
      if (pb.qTime[0]) pb.qTime[0][q] = samp(fv, 4, rec);  // primary.time = sample.getTime() (:159)
    } else {
      pb.pathL[p] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}

// Ray-query kernel with lane refill (persistent-wave traversal, after Aila & Laine 2009):
// each wave owns a contiguous chunk of the queue; the traversal advances one node visit or
// one leaf per iteration, and whenever at least YRT_REFILL lanes of the wave have finished
// their ray, those lanes take the next rays of the chunk (ballot + popcount, no atomics).
// This keeps 64-wide waves busy although ray costs differ by 10-100x. Same visit order and
// the same (t, triangle id) closest-hit rule as traverse<>.
#ifndef YRT_REFILL
#define YRT_REFILL 40  // 24/6 +1.3 % over 16/4; with 64-lane blocks 28/6 +0.4 %, then 40/8 +0.9 % over 28/6;
                        // with four lanes 48 everywhere: C4 -0.8 %, C3 +0.2 %, C5 +1.6 % (r05cc/dd/ee)
#endif
#if defined(YRT_PROFILE) && defined(YRT_SHADE_PROF)
#error "YRT_PROFILE and YRT_SHADE_PROF share the profile counters: build one at a time"
#endif
#if defined(YRT_PROFILE) || defined(YRT_SHADE_PROF)
// YRT_PROFILE: [0] outer iterations x waves, [1] lanes holding a ray at outer iterations,
// [2] node-phase iterations, [3] lanes visiting a node, [4] leaf passes with work,
// [5] triangle-loop iterations (max leaf size per pass), [6] useful triangle tests
// YRT_SHADE_PROF: [0..6] k_shade shader-clock cycles per phase summed over waves, [7] wave
// iterations (see k_shade)
__device__ unsigned long long g_traceProfile[8];
#endif
#ifdef YRT_PROFILE
#ifndef YRT_PROFILE_ANY
#define YRT_PROFILE_ANY 0  // which instantiation counts: 0 closest hit, 1 any hit
#endif
#define YRT_PROF(i, v) (ANY == (YRT_PROFILE_ANY != 0) ? (void)(prof[i] += (unsigned long long)(v)) : (void)0)
#else
#define YRT_PROF(i, v) ((void)0)
#endif

#ifndef YRT_REFILL_ANY
#define YRT_REFILL_ANY 32  // any hit: with node bias 20, C3 +1.5 %, C4 / C5 within the spread (r05ii)
#endif
#ifndef YRT_REFILL_PRIM
#define YRT_REFILL_PRIM YRT_REFILL  // refill threshold of the fused depth-0 instantiation
#endif
#ifndef YRT_TRI_STEP
#define YRT_TRI_STEP 2  // triangles per lane per leaf step (0 = whole leaf): 2 is +0.7 % over whole leaves
#endif
#ifndef YRT_TRI_STEP_ANY
#define YRT_TRI_STEP_ANY YRT_TRI_STEP  // any-hit: triangles per lane per leaf step (sequential, early exit)
#endif
#ifndef YRT_NODE_BIAS
#define YRT_NODE_BIAS 8  // node step iff lanes at a node * 4 > blocked lanes * YRT_NODE_BIAS
#endif
// The closest-hit kernels can store each hit's geometry id (hitGeom) so that k_shade loads the
// geometry record beside the shading record instead of after it (one dependent level fewer).
// Measured same box (profiles/r06/ab_r06a.txt): k_shade 2.663 ms per launch with it, 2.617
// without, C3 and C4 within the spread: the 4-byte store and load per ray cost what the shorter
// chain saves. Off by default; -DYRT_HIT_GEOM=1 for the A/B.
#ifndef YRT_HIT_GEOM
#define YRT_HIT_GEOM 0
#endif
// Node format per traversal kind: 1 = the 64-B quantized nodes (common/yrt_qnode.h), 0 = the
// 128-B float nodes. Both give the same query results bit for bit (conservative boxes).
// Closest hit: neutral at a 32-entry LDS ring (LDS-bound 4.75 waves/SIMD); with a 16-entry ring
// the quantized kernel runs 74 VGPRs at 6 waves/SIMD and the smaller node footprint pays for the
// extra waves' cache interference that the float nodes lose to (same box, profiles/r06/
// ab_r06j.txt: C3 +5.3 %, C4 -1.8 %, C5 -2.5 %; float nodes with the 16-entry ring C3 -2 %).
#ifndef YRT_QNODES_ANY
#define YRT_QNODES_ANY 1
#endif
#ifndef YRT_QNODES_CLOSEST
#define YRT_QNODES_CLOSEST 1
#endif
#ifndef YRT_NODE_BIAS_ANY
#define YRT_NODE_BIAS_ANY 20  // any hit: 12 over 8 -1.7 % on C3, C5 within the spread (r03 anyk); 4 +2.4 %;
                              // four lanes (r05gg-ii): 24 / 32 C3 -2.0 / -2.8 % but C5 +1.6 / +2.3 %
                              // unless refill 32 (20 / 32: C3 -1.5 %, C5 +0.0 %)
#endif
#ifndef YRT_NODE_UNROLL_ANY
#define YRT_NODE_UNROLL_ANY 1  // any-hit: node steps between two node/leaf-phase checks
#endif
#ifndef YRT_TRACE_WAVES
// 6: a scheduling target — the 16 KB LDS stack of a 128-lane block holds the kernels at 5
// waves/SIMD, but code scheduled for 6 (78/74 VGPRs with SGPR-based node addressing) runs
// +0.6 % on C3 over code scheduled for 5 (profiles/r01/variants_r01.txt)
#define YRT_TRACE_WAVES 6
#endif
#ifndef YRT_TRACE_WAVES_PRIM
// the camera-ray (fused depth-0) instantiations: register target of 5 waves/SIMD (96 VGPRs)
#define YRT_TRACE_WAVES_PRIM 5
#endif
#ifndef YRT_TRACE_WAVES_ANY
// occupancy target of the shadow-ray instantiation: 8 waves/SIMD (64 VGPRs, no scratch; the
// 16-entry LDS ring allows 9): same box against 7 (profiles/r06/ab_r06g.txt) C3 +1.9 / +0.8 %,
// C4 -0.7 / -1.1 %, C5 -1.4 %
#define YRT_TRACE_WAVES_ANY 8
#endif
// A finished shadow query: the occlusion flag, or (fused, PathBuffers::fuseShadow) the
// light's contribution added to its path's radiance when unoccluded (k_shadow_resolve order).
__device__ __forceinline__ void shadow_done(const ShadowFuse& sf, int* __restrict__ occOut, int q, bool occluded) {
  if (sf.contrib) {
    if (!occluded) {
      const float4 c = sf.contrib[q];
      const int tg = __float_as_int(c.w);
      float4* Lp = sf.pathL + tg;
      const float4 l = *Lp;
      *Lp = make_float4(l.x + c.x, l.y + c.y, l.z + c.z, l.w);
    }
  } else {
    occOut[q] = occluded ? 1 : 0;
  }
}

// A leaf triangle as tested at ray time t: static scenes read the GpuTri as stored; moving
// scenes (MOTION) rebuild v0, e1, e2 from p + t * m (trianglemesh_full.cpp:104-109, the same
// operations as the oracle's trace), keeping the record's id and flag words.
template <bool MOTION>
__device__ __forceinline__ GpuTri tri_at(const GpuTri* __restrict__ tris, const GpuTriMotion* __restrict__ tms,
                                         int slot, float time) {
  GpuTri t = tris[slot];
  if constexpr (MOTION) {
    const GpuTriMotion m = tms[slot];
    const float p0x = t.v0[0] + time * m.m0[0], p0y = t.v0[1] + time * m.m0[1], p0z = t.v0[2] + time * m.m0[2];
    const float p1x = m.p1[0] + time * m.m1[0], p1y = m.p1[1] + time * m.m1[1], p1z = m.p1[2] + time * m.m1[2];
    const float p2x = m.p2[0] + time * m.m2[0], p2y = m.p2[1] + time * m.m2[1], p2z = m.p2[2] + time * m.m2[2];
    t.v0[0] = p0x; t.v0[1] = p0y; t.v0[2] = p0z;
    t.e1[0] = p0x - p1x; t.e1[1] = p0y - p1y; t.e1[2] = p0z - p1z;
    t.e2[0] = p2x - p0x; t.e2[1] = p2y - p0y; t.e2[2] = p2z - p0z;
  }
  return t;
}

// MOTION: moving geometry; rayTime[q] is query q's time (Ray::time, set from sample.getTime()
// for camera rays and inherited by shadow and continuation rays, pathtraceintegrator.cpp:158,210)
// PRIM = 1 (closest hit, static scenes): depth 0 from the batch's path ids instead of a queue —
// camera rays generated at refill, hits appended to the depth-0 queue, misses resolved
// (PrimaryRays)
template <bool ANY, bool MOTION, int PRIM = 0>
__global__ __launch_bounds__(YRT_TRACE_BLOCK) __attribute__((amdgpu_waves_per_eu(
    ANY ? YRT_TRACE_WAVES_ANY : PRIM ? YRT_TRACE_WAVES_PRIM : YRT_TRACE_WAVES))) void k_trace(
    SceneView sv, const float4* __restrict__ org,
                                                         const float4* __restrict__ dir,
                                                         const unsigned* __restrict__ counts, int numSegs,
                                                         int segCap, float4* __restrict__ hitOut,
                                                         int* __restrict__ occOut, int* __restrict__ spillBuf,
                                                         ShadowFuse sf, const float* __restrict__ rayTime,
                                                         PrimaryRays pr) {
  static_assert(!PRIM || (!ANY && !MOTION), "camera rays: closest hit, static scenes");
  constexpr int kLds = ANY ? YRT_LDS_STACK_ANY : PRIM ? YRT_LDS_STACK_PRIM : YRT_LDS_STACK;
  __shared__ int lstack[kLds * YRT_TRACE_BLOCK];
  __shared__ QMap qm;
  unsigned n;
  if constexpr (PRIM) {
    n = (unsigned)pr.bi.numPixels * (unsigned)const_ref(pr.fv.rp).spp;
  } else {
    qmap_load(qm, counts, numSegs);
    n = qm.pre[YRT_QSEGS];
  }
  const int lane = lane_id();
  const unsigned wavesPerBlock = YRT_TRACE_BLOCK / 64;
  const unsigned gw = blockIdx.x * wavesPerBlock + (threadIdx.x >> 6);
  const unsigned numWaves = gridDim.x * wavesPerBlock;
  unsigned chunk = (n + numWaves - 1) / numWaves;
  chunk = chunk < 64u ? 64u : chunk;
  unsigned next = gw * chunk;
  const unsigned end = min(n, next + chunk);
  if (next >= end) return;  // wave-uniform

  const GpuNode* __restrict__ nodes = sv.nodes;
  const GpuQNode* __restrict__ qnodes = sv.qnodes;
  const GpuTri* __restrict__ tris = sv.tris;
  int* stack = lstack + threadIdx.x;
  // Deep stack entries (rare) spill to global memory, [entry][thread]: a private array here
  // would let the compiler fuse LDS and scratch pops into one slow flat load.
  const size_t spillStride = (size_t)gridDim.x * YRT_TRACE_BLOCK;
  int* __restrict__ spill = spillBuf + blockIdx.x * YRT_TRACE_BLOCK + threadIdx.x;

  bool has = false;
  // cur: next entry to process (count 0 = inner node, >0 = leaf range, -1 = stack exhausted)
  // pend: a leaf parked during the inner-node phase (count 0 = none)
  int q = 0, sp = 0, curIdx = 0, curCnt = 0, pendIdx = 0, pendCnt = 0;
  // The LDS stack is a ring holding the top YRT_LDS_STACK entries; older entries are evicted
  // to global memory on push and restored into the freed slot on pop (both rare). Every pop
  // returns an LDS value, so the hot path stays a ds_read.
#define YRT_SLOT(i) ((((i) & (kLds - 1))) * YRT_TRACE_BLOCK)
#define YRT_POP_READ(e_)                                                          \
  do {                                                                            \
    e_ = (unsigned)stack[YRT_SLOT(sp)];                                           \
    if (sp >= kLds) stack[YRT_SLOT(sp)] = spill[(size_t)(sp - kLds) * spillStride]; \
  } while (0)
#define YRT_PUSH(e)                                                               \
  do {                                                                            \
    if (sp >= kLds) spill[(size_t)(sp - kLds) * spillStride] = stack[YRT_SLOT(sp)]; \
    stack[YRT_SLOT(sp)] = (e);                                                    \
    sp += 1;                                                                      \
  } while (0)
#define YRT_POP()                                                                 \
  do {                                                                            \
    if (sp == 0) {                                                                \
      curCnt = -1;                                                                \
    } else {                                                                      \
      sp -= 1;                                                                    \
      unsigned e_;                                                                \
      YRT_POP_READ(e_);                                                           \
      curIdx = (int)(e_ >> 5);                                                    \
      curCnt = (int)(e_ & 31u);                                                   \
    }                                                                             \
  } while (0)
  // ray kept as plain vectors across iterations (a loop-carried RayPre struct ends up in
  // scratch: the vectorizer's straddling loads defeat SROA); rebuilt in registers per step
  float4 ro = make_float4(0.f, 0.f, 0.f, 0.f), rd = ro, ri = ro, rc = ro;
  float rtime = 0.f;
  Hit best;
  best.t = best.u = best.v = 0.f;
  best.tri = -1;
  // closest hit: the accepted triangle's undivided barycentrics (U, V) and |den| are kept, and
  // u = U/|den|, v = V/|den| are divided once, when the finished query is stored at the next
  // refill (or at the wave's end), instead of at every accepted hit; q = -1: nothing to store
  float bestDen = 1.f;
  // closest hit: the accepted triangle's geometry id (GpuTri::e2[3]), stored beside the hit
  // (occOut) so k_shade loads the geometry record beside the shading record, not after it
  int bestGeom = 0;
  q = -1;
  // PRIM: a finished camera ray (q = its path id) — a hit is appended with its ray and hit
  // record to the depth-0 queue segment of its path id's 64-group (one atomic per segment among
  // the storing lanes); a miss gets the environment's radiance, loaded from the render
  // parameters where it is stored (a value held in registers through the loop costs four of
  // them). The camera rays traced are counted after the loop, no counter is carried through it.
  auto prim_store = [&]() {
    const bool hitp = best.tri >= 0;
    if (!hitp) {
      const float* mL = pr.fv.rp->missL;
      pr.pathL[q] = make_float4(mL[0], mL[1], mL[2], mL[3]);
    }
    const int seg = qseg_of((unsigned)q);
    unsigned long long m = ballot(hitp);
    while (m) {
      const int l0 = __ffsll((long long)m) - 1;
      const int seg0 = __builtin_amdgcn_readlane(seg, l0);
      const unsigned long long sub = ballot(hitp && seg == seg0);
      unsigned base = 0;
      if (lane == l0) base = atomicAdd(pr.counts + (size_t)seg0 * YRT_QCSTRIDE, (unsigned)__popcll(sub));
      base = (unsigned)__builtin_amdgcn_readlane((int)base, l0);
      if (hitp && seg == seg0) {
        const unsigned slot = (unsigned)seg0 * (unsigned)pr.segCap + base + lanes_below(sub);
        pr.qPath[slot] = q;
        pr.qOrg[slot] = ro;
        pr.qDir[slot] = rd;
        hitOut[slot] = make_float4(best.t, best.u / bestDen, best.v / bestDen, __int_as_float(best.tri));
        if (YRT_HIT_GEOM && occOut) occOut[slot] = bestGeom;
      }
      m &= ~sub;
    }
  };
#define YRT_STORE_HIT()                                                                              \
  do {                                                                                               \
    if constexpr (PRIM)                                                                              \
      prim_store();                                                                                  \
    else {                                                                                           \
      hitOut[q] = make_float4(best.t, best.u / bestDen, best.v / bestDen, __int_as_float(best.tri)); \
      if (YRT_HIT_GEOM && occOut) occOut[q] = bestGeom;                                              \
    }                                                                                                \
    q = -1;                                                                                          \
  } while (0)

#ifdef YRT_PROFILE
  unsigned long long prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  while (true) {
    // retire lanes whose traversal is complete
    if (has && curCnt < 0 && pendCnt == 0) {
      if (ANY) shadow_done(sf, occOut, q, false);
      has = false;
    }
    const unsigned long long idle = ballot(!has);
    const int nIdle = __popcll(idle);
    YRT_PROF(0, 1);
    YRT_PROF(1, 64 - nIdle);
    if (nIdle >= (ANY ? YRT_REFILL_ANY : PRIM ? YRT_REFILL_PRIM : YRT_REFILL)) {
      if (next < end) {
        const unsigned li = next + lanes_below(idle);
        if (!has) {
          if (!ANY && q >= 0) YRT_STORE_HIT();
          if (li < end) {
            if constexpr (PRIM) {
              // k_raygen's camera ray of path li (same operations, bit-identical rays)
              const YRT_CONST GpuRenderParams& rp = const_ref(pr.fv.rp);
              const int p = (int)li;
              const int smp = fastdiv(p, pr.bi.divPixels);
              int x = 0, y = 0, f = 0;
              const bool valid = batch_pixel(rp, pr.bi, p - smp * pr.bi.numPixels, x, y, f) && rp.maxDepth > 0 &&
                                 !(1.0f < rp.minContribution);
              if (valid) {
                const int rec = pr.fv.pixelSets[(size_t)y * rp.width + x] * rp.spp + smp;
                const float fx = (float(x) + samp(pr.fv, 0, rec)) * rp.rcpWidth;
                const float fy = (float(y) + samp(pr.fv, 1, rec)) * rp.rcpHeight;
                const float lx = samp(pr.fv, 2, rec), ly = samp(pr.fv, 3, rec);
                V3 o3 = v3s(0.f), d3 = v3s(0.f);
                // one pass per frame among the refilled lanes (almost always one): the frame's
                // camera record is read with scalar loads, as in k_raygen
                for (bool todo = true; todo;) {
                  const int f0 = __builtin_amdgcn_readfirstlane(f);
                  if (f == f0) {
                    const YRT_CONST GpuCamera& cam = const_ref(pr.fv.cam + f0);
                    camera_ray<false>(cam, fx, fy, o3, d3, lx, ly);
                    todo = false;
                  }
                }
                ro = make_float4(o3.x, o3.y, o3.z, 0.f);
                rd = make_float4(d3.x, d3.y, d3.z, __int_as_float(0x7f800000));
                q = p;
              } else {
                // a zero made here: a constant zero vector is hoisted out of the loop and held in
                // four registers (spilled at a 5-wave register target)
                const float z = opaque_zero();
                pr.pathL[p] = make_float4(z, z, z, z);  // not a pixel of the image
                q = -1;
                ro = make_float4(0.f, 0.f, 0.f, 1.f);  // tfar < tnear: nothing to traverse
                rd = make_float4(0.f, 0.f, 1.f, 0.f);
              }
            } else {
            q = qmap_phys(qm, segCap, li);
            ro = org[q];
            rd = dir[q];
            if (MOTION) rtime = rayTime[q];
            }
            ri = make_float4(safe_inv(rd.x), safe_inv(rd.y), safe_inv(rd.z), 0.f);
            ri.w = __int_as_float(plane_offsets(ri.x, ri.y, ri.z));
            {
              V3 oi;
              float mg;
              ray_slab_consts(v3(ro.x, ro.y, ro.z), v3(ri.x, ri.y, ri.z), oi, mg);
              rc = make_float4(oi.x, oi.y, oi.z, mg);
            }
            best.t = rd.w;
            best.u = best.v = 0.f;
            best.tri = -1;
            bestDen = 1.f;
            sp = 0;
            curIdx = 0;
            curCnt = 0;
            pendCnt = 0;
            // NaN tfar (tMaxShadowRay = inf): no hit, nothing to traverse
            has = rd.w >= ro.w;
            if (!has) {
              if (ANY) shadow_done(sf, occOut, q, false);
            }
          }
        }
        next += (unsigned)nIdle;
      } else if (nIdle == 64) {
        if (!ANY && q >= 0) YRT_STORE_HIT();
        if constexpr (PRIM) {
          // the camera rays this wave traced: the valid path ids of its chunk (the refill's
          // test again, after the loop, so that no count is carried through it)
          const YRT_CONST GpuRenderParams& rp = const_ref(pr.fv.rp);
          unsigned t = 0;
          if (rp.maxDepth > 0 && !(1.0f < rp.minContribution)) {
            for (unsigned b = gw * chunk; b < end; b += 64) {
              const unsigned p = b + (unsigned)lane;
              bool v = false;
              if (p < end) {
                const int smp = fastdiv((int)p, pr.bi.divPixels);
                int x, y, f;
                v = batch_pixel(rp, pr.bi, (int)p - smp * pr.bi.numPixels, x, y, f);
              }
              t += (unsigned)__popcll(ballot(v));
            }
          }
          if (lane == 0 && t) atomicAdd(pr.traced, t);
        }
#ifdef YRT_PROFILE
        if (lane == 0)
          for (int k = 0; k < 8; ++k) atomicAdd(&g_traceProfile[k], prof[k]);
#endif
        break;
      }
    }
    RayPre r;
    r.org = v3(ro.x, ro.y, ro.z);
    r.dir = v3(rd.x, rd.y, rd.z);
    r.inv = v3(ri.x, ri.y, ri.z);
    r.tnear = ro.w;
    r.tfar = rd.w;
    r.oi = v3(rc.x, rc.y, rc.z);
    r.margin = rc.w;

    // One step per iteration, chosen wave-uniformly ("while-while" with speculative leaf
    // parking, Aila & Laine 2009): node steps while any lane still searches for its first
    // leaf (a lane reaching a leaf parks it and keeps descending), then one leaf step in
    // which every lane tests one leaf. Refill above runs every iteration, so lanes that
    // finish rejoin at once instead of idling until the wave's phase ends.
    // node step when more lanes can descend than are blocked on a leaf (cur is a leaf while
    // another is parked, or only a parked leaf is left); otherwise a leaf step
    // lane masks of plain comparisons (one v_cmp each) combined on the scalar unit: a ballot of
    // has && ... re-materializes the predicate per ballot (8 -> 3 VALU per node-step check,
    // closest-hit trace -2.1 % on C3, profiles/r02/trace_variants_r02.txt); has does not change
    // inside the node loop, so its mask is taken once here
    const unsigned long long hasB = ballot(has);
#define YRT_NNODE() __popcll(ballot(curCnt == 0) & hasB)
#define YRT_NBLOCKED() __popcll(ballot(max(pendCnt, curCnt) > 0) & ~ballot(curCnt == 0) & hasB)
    const int nNode = YRT_NNODE();
    const int nBlocked = YRT_NBLOCKED();
    if (nNode * 4 > nBlocked * (ANY ? YRT_NODE_BIAS_ANY : YRT_NODE_BIAS)) {
     // consecutive node steps without the retire/refill block in between (+1.5 % on C3)
     while (true) {
#pragma unroll
      for (int nu = 0; nu < (ANY ? YRT_NODE_UNROLL_ANY : 1); ++nu) {
      YRT_PROF(2, 1);
      YRT_PROF(3, __popcll(ballot(has && curCnt == 0)));
      if (has && curCnt == 0) {
        float t[4];
        int c[4];
        // sign-ordered slab planes (+1.5 % on C3 with two lanes, bit-identical distances)
        if (ANY ? YRT_QNODES_ANY : YRT_QNODES_CLOSEST)
          box4_quant<ANY>(r, __float_as_int(ri.w), best.t, t, c, qnodes, curIdx);
        else
          box4_ordered<ANY>(r, __float_as_int(ri.w), best.t, t, c, nodes, curIdx);
        // closest-hit rays sort the hit children by entry distance (nearest next, the others
        // pushed farthest-first); any-hit rays take the farthest hit child next and push the
        // others in slot order (sort3_far: -22 % node visits against slot order)
        if (!ANY) sort4(t, c);
        else sort3_far(t, c);
        const float MISS = __int_as_float(ANY ? 0xff800000 : 0x7f800000);
#define YRT_HIT(x) (ANY ? (x) > MISS : (x) < MISS)
        if (sp + 3 <= kLds) {
          // all three candidates fit in free ring slots: store unconditionally, advance sp
          // only past the hit ones (a store of a missed child lands on a free slot);
          // shadow rays -4..9 %, closest neutral (profiles/r01)
          const int h3 = YRT_HIT(t[3]), h2 = YRT_HIT(t[2]), h1 = YRT_HIT(t[1]);
          stack[YRT_SLOT(sp)] = c[3];
          stack[YRT_SLOT(sp + h3)] = c[2];
          stack[YRT_SLOT(sp + h3 + h2)] = c[1];
          sp += h3 + h2 + h1;
        } else {
          if (YRT_HIT(t[3])) YRT_PUSH(c[3]);
          if (YRT_HIT(t[2])) YRT_PUSH(c[2]);
          if (YRT_HIT(t[1])) YRT_PUSH(c[1]);
        }
        if (YRT_HIT(t[0])) {
          curIdx = c[0] >> 5;
          curCnt = c[0] & 31;
        } else {
          YRT_POP();
        }
#undef YRT_HIT
        if (curCnt > 0 && pendCnt == 0) {
          pendIdx = curIdx;
          pendCnt = curCnt;
          YRT_POP();
        }
      }
      }  // YRT_NODE_UNROLL_ANY
      const int nNode2 = YRT_NNODE();
      const int nBlocked2 = YRT_NBLOCKED();
      if (!(nNode2 * 4 > nBlocked2 * (ANY ? YRT_NODE_BIAS_ANY : YRT_NODE_BIAS))) break;
     }
    } else {
      // leaf step: the parked leaf, or else the current entry when it is a leaf
      const bool usePend = pendCnt > 0;
      const int lIdx = usePend ? pendIdx : curIdx;
      const int lCnt = !has ? 0 : usePend ? pendCnt : (curCnt > 0 ? curCnt : 0);
#ifdef YRT_PROFILE
      {
        const int lc_ = YRT_TRI_STEP ? min(lCnt, ANY ? YRT_TRI_STEP_ANY : YRT_TRI_STEP) : lCnt;  // triangles this step
        int mx = lc_;
        for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o, 64));
        int sm = lc_;
        for (int o = 32; o > 0; o >>= 1) sm += __shfl_xor(sm, o, 64);
        YRT_PROF(4, mx > 0 ? 1 : 0);
        YRT_PROF(5, mx);
        YRT_PROF(6, sm);
      }
#endif
      bool found = false;
#if YRT_TRI_STEP
      // at most YRT_TRI_STEP (YRT_TRI_STEP_ANY) triangles per lane per leaf step (the rest of
      // the leaf stays current / parked): less intra-leaf divergence
      constexpr int kTriStep = ANY ? YRT_TRI_STEP_ANY : YRT_TRI_STEP;
      const int lTake = min(lCnt, kTriStep);
#else
      const int lTake = lCnt;
#endif
      if (!ANY && YRT_TRI_STEP >= 2) {
        // closest hit: all triangles of the step loaded up front (one memory round trip instead
        // of one per triangle: closest trace -4.6 % on C3, profiles/r02/trace_variants_r02.txt),
        // then accepted in leaf order exactly as the loop below does; lanes with fewer
        // triangles repeat their last one and ignore it
        constexpr int K = YRT_TRI_STEP >= 2 ? YRT_TRI_STEP : 2;
        if (lTake > 0) {
          GpuTri tt[K];
#pragma unroll
          for (int k = 0; k < K; ++k) tt[k] = tri_at<MOTION>(tris, sv.triMotion, lIdx + min(k, lTake - 1), rtime);
#pragma unroll
          for (int k = 0; k < K; ++k) {
            float t, U, V, absDen;
            const bool g = tri_test_g(tt[k], r, t, U, V, absDen);
            const int gid = __float_as_int(tt[k].v0[3]);
            // range test against the current closest hit; on a tie (t == best.t) the smaller
            // triangle id wins
            // a tie with an accepted hit (best.tri >= 0, so best.t < tfar) passes the range test
            // by itself: one predicate instead of a re-test against tfar (C3 -0.35 %, C5 -0.3 %)
            const bool tie = (t == best.t) & (best.tri >= 0) & (gid < best.tri);
            const bool ok = g & (t > r.tnear) & ((t < best.t + 0.0f) | tie);
            if (ok & (k < lTake)) {
              best.t = t; best.u = U; best.v = V; bestDen = absDen; best.tri = gid;
              if (YRT_HIT_GEOM) bestGeom = __float_as_int(tt[k].e2[3]);
            }
          }
        }
      } else {
        for (int i = 0; i < lTake && !found; ++i) {
          const GpuTri tr = tri_at<MOTION>(tris, sv.triMotion, lIdx + i, rtime);
          float t, U, V, absDen;
          bool ok = tri_test_t(tr, r, ANY ? r.tfar : best.t + 0.0f, t, U, V, absDen);
          const int gid = __float_as_int(tr.v0[3]);
          if (ANY) {
            found = ok;
          } else {
            // ties (t == best.t) were rejected by the strict test: smaller id wins
            if (!ok && best.tri >= 0 && t == best.t && gid < best.tri) {
              float t2, U2, V2, a2;
              ok = tri_test_t(tr, r, r.tfar, t2, U2, V2, a2);
            }
            if (ok) {
              best.t = t; best.u = U; best.v = V; bestDen = absDen; best.tri = gid;
              if (YRT_HIT_GEOM) bestGeom = __float_as_int(tr.e2[3]);
            }
          }
        }
      }
#if YRT_TRI_STEP
      if (lCnt > 0) {
        if (usePend) {
          pendIdx += lTake;
          pendCnt -= lTake;
        } else if (curCnt > lTake) {
          curIdx += lTake;
          curCnt -= lTake;
        } else {
          YRT_POP();
        }
      }
#else
      if (lCnt > 0) {
        if (usePend) pendCnt = 0;
        else YRT_POP();
      }
#endif
      if (ANY && found) {
        shadow_done(sf, occOut, q, true);
        has = false;
      }
    }
  }
}

#if YRT_ANY2
// ---------------------------------------------------------------- any hit, two rays per lane
// k_occluded2: the shadow query of k_trace<true, false> (the same quantized box test, the same
// farthest-child-first order, the same triangle test, so the same occlusion answers) with TWO
// independent rays per lane. A node step loads both rays' nodes before testing either, a leaf
// step both rays' triangles, so each lane keeps two dependent load -> test -> push chains in
// flight. Round 5 measured this on the 128-B float nodes (k_occluded): 146 VGPRs, 3 waves/SIMD,
// frame -2.7 %; the 64-B quantized node is 14 words instead of 28 per ray. Each ray slot has a
// YRT_ANY2_LDS-entry LDS ring (2 x 16 x 256 B = 8 KB per wave, the one-ray kernel's LDS);
// older entries spill to global memory. Slots without work load node 0 / triangle 0 (L2 hits)
// so the loads stay unconditional and issue back to back.
#ifndef YRT_ANY2_REFILL
#define YRT_ANY2_REFILL 64  // refill when this many of the wave's 128 ray slots are idle
#endif
#ifndef YRT_ANY2_BIAS
#define YRT_ANY2_BIAS 20  // node step iff slots at a node * 4 > blocked slots * YRT_ANY2_BIAS
#endif
#ifndef YRT_ANY2_WAVES
#define YRT_ANY2_WAVES 4
#endif
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(YRT_ANY2_WAVES))) void k_occluded2(
    SceneView sv, const float4* __restrict__ org, const float4* __restrict__ dir, const unsigned* __restrict__ counts,
    int numSegs, int segCap, int* __restrict__ occOut, int* __restrict__ spillBuf, ShadowFuse sf) {
  constexpr int R = YRT_ANY2_LDS;
  __shared__ int lstack[2 * R * 64];
  __shared__ QMap qm;
  qmap_load(qm, counts, numSegs);
  const unsigned n = qm.pre[YRT_QSEGS];
  const int lane = lane_id();
  unsigned chunk = (n + gridDim.x - 1) / gridDim.x;
  chunk = chunk < 128u ? 128u : chunk;
  unsigned next = blockIdx.x * chunk;
  const unsigned end = min(n, next + chunk);
  if (next >= end) return;  // wave-uniform

  const GpuQNode* __restrict__ qnodes = sv.qnodes;
  const GpuTri* __restrict__ tris = sv.tris;
  int* stack = lstack + lane;
  // spilled entries: [entry][slot][thread] (YRT_TRACE_SPILL_INTS covers 2 x (YRT_STACK_DEPTH - R)
  // entries per thread of a 64-lane block)
  const size_t spillStride = (size_t)gridDim.x * 64;
  int* __restrict__ spill = spillBuf + blockIdx.x * 64 + lane;
#define A2_SLOT(s, i) ((((s) * R) + ((i) & (R - 1))) * 64)
#define A2_SPILL(s, i) spill[((size_t)((i) - R) * 2 + (s)) * spillStride]
#define A2_PUSH(s, e)                                              \
  do {                                                             \
    if (sp[s] >= R) A2_SPILL(s, sp[s]) = stack[A2_SLOT(s, sp[s])]; \
    stack[A2_SLOT(s, sp[s])] = (e);                                \
    sp[s] += 1;                                                    \
  } while (0)
#define A2_POP(s)                                                          \
  do {                                                                     \
    if (sp[s] == 0) {                                                      \
      cur[s] = -1;                                                         \
    } else {                                                               \
      sp[s] -= 1;                                                          \
      cur[s] = stack[A2_SLOT(s, sp[s])];                                   \
      if (sp[s] >= R) stack[A2_SLOT(s, sp[s])] = A2_SPILL(s, sp[s]);       \
    }                                                                      \
  } while (0)
  // per slot: the ray (org.xyz, tnear | dir.xyz, tfar | inv.xyz, plane offsets), its query
  // index, stack pointer, current entry (index << 5 | count; count 0 = inner node, -1 = stack
  // exhausted) and a parked leaf (0 = none). The slab constants org * inv and margin are
  // recomputed per step instead of held in four more registers per slot.
  float4 ro[2], rd[2], ri[2];
  int q[2], sp[2], cur[2], pend[2];
  bool has[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    ro[s] = rd[s] = ri[s] = make_float4(0.f, 0.f, 0.f, 0.f);
    q[s] = sp[s] = pend[s] = 0;
    cur[s] = -1;
    has[s] = false;
  }
  auto ray_of = [&](int s) {
    RayPre r;
    r.org = v3(ro[s].x, ro[s].y, ro[s].z);
    r.dir = v3(rd[s].x, rd[s].y, rd[s].z);
    r.inv = v3(ri[s].x, ri[s].y, ri[s].z);
    r.tnear = ro[s].w;
    r.tfar = rd[s].w;
    ray_slab_consts(r.org, r.inv, r.oi, r.margin);
    return r;
  };
#define A2_INNER(s) (cur[s] >= 0 && (cur[s] & 31) == 0)
#define A2_NNODE() (__popcll(ballot(A2_INNER(0)) & hasB0) + __popcll(ballot(A2_INNER(1)) & hasB1))
#define A2_NBLOCKED()                                                       \
  (__popcll(ballot(!A2_INNER(0) && (pend[0] != 0 || cur[0] > 0)) & hasB0) + \
   __popcll(ballot(!A2_INNER(1) && (pend[1] != 0 || cur[1] > 0)) & hasB1))
  while (true) {
    // retire slots whose traversal is complete (unoccluded)
#pragma unroll
    for (int s = 0; s < 2; ++s)
      if (has[s] && cur[s] < 0 && pend[s] == 0) {
        shadow_done(sf, occOut, q[s], false);
        has[s] = false;
      }
    const unsigned long long idle0 = ballot(!has[0]), idle1 = ballot(!has[1]);
    const int nIdle0 = __popcll(idle0);
    const int nIdle = nIdle0 + __popcll(idle1);
    if (nIdle >= YRT_ANY2_REFILL) {
      if (next < end) {
        // idle slot 0s take the next rays of the chunk in lane order, then idle slot 1s
        bool take[2];
        float4 lo[2], ld[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const unsigned li = next + (s ? (unsigned)nIdle0 : 0u) + (unsigned)lanes_below(s ? idle1 : idle0);
          take[s] = !has[s] && li < end;
          if (take[s]) {
            q[s] = qmap_phys(qm, segCap, li);
            lo[s] = org[q[s]];
            ld[s] = dir[q[s]];
          }
        }
#pragma unroll
        for (int s = 0; s < 2; ++s)
          if (take[s]) {
            ro[s] = lo[s];
            rd[s] = ld[s];
            ri[s] = make_float4(safe_inv(rd[s].x), safe_inv(rd[s].y), safe_inv(rd[s].z), 0.f);
            ri[s].w = __int_as_float(plane_offsets(ri[s].x, ri[s].y, ri[s].z));
            sp[s] = 0;
            cur[s] = 0;
            pend[s] = 0;
            // NaN tfar (tMaxShadowRay = inf): nothing to traverse, unoccluded
            has[s] = rd[s].w >= ro[s].w;
            if (!has[s]) shadow_done(sf, occOut, q[s], false);
          }
        next += (unsigned)nIdle;
      } else if (nIdle == 128) {
        break;
      }
    }
    // node steps while more slots can descend than are blocked on a leaf, else a leaf step
    // (the one-ray kernel's rule, counted over both slots)
    const unsigned long long hasB0 = ballot(has[0]), hasB1 = ballot(has[1]);
    if (A2_NNODE() * 4 > A2_NBLOCKED() * YRT_ANY2_BIAS) {
      while (true) {
        bool act[2];
        QNodeData nd[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          act[s] = has[s] && A2_INNER(s);
          nd[s] = qnode_load(qnodes, act[s] ? (cur[s] >> 5) : 0);
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const RayPre r = ray_of(s);
          float t[4];
          int c[4];
          box4_qdata<true>(nd[s], r, __float_as_int(ri[s].w), r.tfar, t, c);
          sort3_far(t, c);
          if (act[s]) {
            const float MISS = __int_as_float(0xff800000);
            const int h3 = t[3] > MISS, h2 = t[2] > MISS, h1 = t[1] > MISS;
            if (sp[s] + 3 <= R) {
              // unconditional stores into free ring slots, sp advanced past the hit children
              stack[A2_SLOT(s, sp[s])] = c[3];
              stack[A2_SLOT(s, sp[s] + h3)] = c[2];
              stack[A2_SLOT(s, sp[s] + h3 + h2)] = c[1];
              sp[s] += h3 + h2 + h1;
            } else {
              if (h3) A2_PUSH(s, c[3]);
              if (h2) A2_PUSH(s, c[2]);
              if (h1) A2_PUSH(s, c[1]);
            }
            if (t[0] > MISS) cur[s] = c[0];
            else A2_POP(s);
            // a leaf reached while none is parked: park it and keep descending
            if (cur[s] > 0 && (cur[s] & 31) != 0 && pend[s] == 0) {
              pend[s] = cur[s];
              A2_POP(s);
            }
          }
        }
        if (!(A2_NNODE() * 4 > A2_NBLOCKED() * YRT_ANY2_BIAS)) break;
      }
    } else {
      // leaf step: one triangle per slot, the parked leaf or else the current entry
      int lf[2];
      bool usePend[2];
      GpuTri tr[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        usePend[s] = pend[s] != 0;
        lf[s] = !has[s] ? 0 : usePend[s] ? pend[s] : (cur[s] > 0 && (cur[s] & 31) != 0) ? cur[s] : 0;
        tr[s] = tris[lf[s] > 0 ? (lf[s] >> 5) : 0];
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if (lf[s] > 0) {
          const RayPre r = ray_of(s);
          float t, U, V, absDen;
          const bool found = tri_test_t(tr[s], r, r.tfar, t, U, V, absDen);
          // the leaf's next triangle (index + 1, count - 1), or the leaf is done
          const int rest = (lf[s] & 31) > 1 ? lf[s] + 31 : 0;
          if (usePend[s]) pend[s] = rest;
          else if (rest) cur[s] = rest;
          else A2_POP(s);
          if (found) {
            shadow_done(sf, occOut, q[s], true);
            has[s] = false;
          }
        }
      }
    }
  }
#undef A2_INNER
#undef A2_NNODE
#undef A2_NBLOCKED
#undef A2_SLOT
#undef A2_SPILL
#undef A2_PUSH
#undef A2_POP
}
#endif  // YRT_ANY2

// ---------------------------------------------------------------- shading helpers
// BackendSceneFlat::postIntersect -> Shape::postIntersect
// geom: the hit triangle's geometry record (sv.geoms / the geometry part of sv.geomRecs)
// time: the ray's time (moving geometry, GF_MOTION: vertices p + time * m, trianglemesh_full.cpp:211-215)
__device__ __forceinline__ void post_intersect_g(const SceneView& sv, const GpuGeom& geom, V3 org, V3 dir, float t,
                                                 float u, float v, int gid, DG& dg, bool wantTangents,
                                                 float time = 0.f) {
  dg.material = geom.material;
  dg.light = geom.light;
  dg.illumMask = geom.illumMask;
  dg.shadowMask = geom.shadowMask;
  dg.P = org + t * dir;
  if (geom.kind == GEOM_TRIANGLE) {
    // shapes/triangle.h:69-78
    dg.Ng = v3(geom.Ng[0], geom.Ng[1], geom.Ng[2]);
    dg.Ns = dg.Ng;
    dg.s = u;
    dg.t = v;
    dg.Tx = dg.Ty = v3s(0.f);
  } else {
    const int4 idx = sv.indices[gid];
    V3 p0 = ld3(sv.positions[idx.x]), p1 = ld3(sv.positions[idx.y]), p2 = ld3(sv.positions[idx.z]);
    if (geom.flags & GF_MOTION) {
      p0 = p0 + time * ld3(sv.motions[idx.x]);
      p1 = p1 + time * ld3(sv.motions[idx.y]);
      p2 = p2 + time * ld3(sv.motions[idx.z]);
    }
    const float w = 1.0f - u - v;
    const V3 dPdu = p1 - p0, dPdv = p2 - p0;
    dg.Ng = normalize(cross(p0 - p1, p2 - p0));  // ray.Ng (unnormalized Embree Ng)
    if (geom.kind == GEOM_MESH_NORMALS) {
      // shapes/trianglemesh_normals.cpp:125-147
      dg.s = u;
      dg.t = v;
      const V3 n0 = ld3(sv.normals[idx.x]), n1 = ld3(sv.normals[idx.y]), n2 = ld3(sv.normals[idx.z]);
      V3 Ns = w * n0 + u * n1 + v * n2;
      const float len2 = dot(Ns, Ns);
      Ns = len2 > 0 ? Ns * rsqrtf_(len2) : dg.Ng;
      if (dot(Ns, dg.Ng) < 0) Ns = -Ns;
      dg.Ns = Ns;
      dg.Tx = dPdu;
      dg.Ty = dPdv;
    } else {
      // shapes/trianglemesh_full.cpp:192-260
      float dsdu, dtdu, dsdv, dtdv;
      if (geom.flags & GF_TEXCOORDS) {
        const float2 st0 = sv.texcoords[idx.x], st1 = sv.texcoords[idx.y], st2 = sv.texcoords[idx.z];
        dg.s = st0.x * w + st1.x * u + st2.x * v;
        dg.t = st0.y * w + st1.y * u + st2.y * v;
        dsdu = st1.x - st0.x; dtdu = st1.y - st0.y;
        dsdv = st2.x - st0.x; dtdv = st2.y - st0.y;
      } else {
        dg.s = u;
        dg.t = v;
        dsdu = 1; dtdu = 0;
        dsdv = 0; dtdv = 1;
      }
      if (geom.flags & GF_NORMALS) {
        const V3 n0 = ld3(sv.normals[idx.x]), n1 = ld3(sv.normals[idx.y]), n2 = ld3(sv.normals[idx.z]);
        V3 Ns = w * n0 + u * n1 + v * n2;
        const float len2 = dot(Ns, Ns);
        Ns = len2 > 0 ? Ns * rsqrtf_(len2) : dg.Ng;
        if (dot(Ns, dg.Ng) < 0) Ns = -Ns;
        dg.Ns = Ns;
      } else {
        dg.Ns = dg.Ng;
      }
      if (wantTangents) {
        // trianglemesh_full.cpp:244-263: interpolated tangents when the mesh has them
        if (geom.flags & GF_TANGENT_X) {
          dg.Tx = w * ld3(sv.tangents[2 * idx.x]) + u * ld3(sv.tangents[2 * idx.y]) + v * ld3(sv.tangents[2 * idx.z]);
        } else {
          const V3 dPds = normalize(dPdu * dtdv - dPdv * dtdu);
          dg.Tx = normalize(dPds - dot(dPds, dg.Ns) * dg.Ns);
        }
        if (geom.flags & GF_TANGENT_Y) {
          dg.Ty = w * ld3(sv.tangents[2 * idx.x + 1]) + u * ld3(sv.tangents[2 * idx.y + 1]) +
                  v * ld3(sv.tangents[2 * idx.z + 1]);
        } else {
          const V3 dPdt = normalize(dPdv * dsdu - dPdu * dsdv);
          dg.Ty = normalize(dPdt - dot(dPdt, dg.Ns) * dg.Ns);
        }
      } else {
        dg.Tx = dg.Ty = v3s(0.f);
      }
    }
  }
  dg.error = fmaxf(fabsf(t), reduce_max(absv(dg.P)));
}
// k_shade's postIntersect: static mesh triangles read their GpuTriShade record (r0 = its
// first 16 bytes, already loaded for the geometry id) instead of the index record and the
// vertex arrays; the same operations as post_intersect_g on the same values, so the same bits.
// Single triangles, moving meshes and meshes with tangent arrays take post_intersect_g.
__device__ __forceinline__ void post_intersect_rec(const SceneView& sv, const GpuGeom& geom,
                                                   const float4* __restrict__ rec, float4 r0, V3 org, V3 dir, float t,
                                                   float u, float v, int gid, DG& dg, bool wantTangents, float time) {
  if (geom.kind == GEOM_TRIANGLE || (geom.flags & (GF_MOTION | GF_TANGENT_X | GF_TANGENT_Y))) {
    post_intersect_g(sv, geom, org, dir, t, u, v, gid, dg, wantTangents, time);
    return;
  }
  dg.material = geom.material;
  dg.light = geom.light;
  dg.illumMask = geom.illumMask;
  dg.shadowMask = geom.shadowMask;
  dg.P = org + t * dir;
  const float4 r1 = rec[1];
  const V3 e1 = v3(r0.x, r0.y, r0.z), e2 = v3(r1.x, r1.y, r1.z);  // p0 - p1, p2 - p0
  const float w = 1.0f - u - v;
  const V3 dPdu = -e1, dPdv = e2;  // p1 - p0 (negation is exact), p2 - p0
  dg.Ng = normalize(cross(e1, e2));
  const bool meshNormals = geom.kind == GEOM_MESH_NORMALS;
  if (meshNormals || (geom.flags & GF_NORMALS)) {
    const float4 r2 = rec[2], r3 = rec[3], r4 = rec[4];
    const V3 n0 = v3(r2.x, r2.y, r2.z), n1 = v3(r2.w, r3.x, r3.y), n2 = v3(r3.z, r3.w, r4.x);
    V3 Ns = w * n0 + u * n1 + v * n2;
    const float len2 = dot(Ns, Ns);
    Ns = len2 > 0 ? Ns * rsqrtf_(len2) : dg.Ng;
    if (dot(Ns, dg.Ng) < 0) Ns = -Ns;
    dg.Ns = Ns;
  } else {
    dg.Ns = dg.Ng;
  }
  if (meshNormals) {
    // shapes/trianglemesh_normals.cpp:125-147
    dg.s = u;
    dg.t = v;
    dg.Tx = dPdu;
    dg.Ty = dPdv;
  } else {
    // shapes/trianglemesh_full.cpp:192-260
    float dsdu, dtdu, dsdv, dtdv;
    if (geom.flags & GF_TEXCOORDS) {
      const float4 r4 = rec[4], r5 = rec[5];
      const float2 st0 = make_float2(r4.y, r4.z), st1 = make_float2(r4.w, r5.x), st2 = make_float2(r5.y, r5.z);
      dg.s = st0.x * w + st1.x * u + st2.x * v;
      dg.t = st0.y * w + st1.y * u + st2.y * v;
      dsdu = st1.x - st0.x; dtdu = st1.y - st0.y;
      dsdv = st2.x - st0.x; dtdv = st2.y - st0.y;
    } else {
      dg.s = u;
      dg.t = v;
      dsdu = 1; dtdu = 0;
      dsdv = 0; dtdv = 1;
    }
    if (wantTangents) {
      const V3 dPds = normalize(dPdu * dtdv - dPdv * dtdu);
      dg.Tx = normalize(dPds - dot(dPds, dg.Ns) * dg.Ns);
      const V3 dPdt = normalize(dPdv * dsdu - dPdu * dsdv);
      dg.Ty = normalize(dPdt - dot(dPdt, dg.Ns) * dg.Ns);
    } else {
      dg.Tx = dg.Ty = v3s(0.f);
    }
  }
  dg.error = fmaxf(fabsf(t), reduce_max(absv(dg.P)));
}

__device__ __forceinline__ void post_intersect(const SceneView& sv, V3 org, V3 dir, float t, float u, float v, int gid,
                                               DG& dg, bool wantTangents) {
  const int g = sv.indices[gid].w;  // geometry id rides in the index record
  post_intersect_g(sv, sv.geoms[g], org, dir, t, u, v, gid, dg, wantTangents);
}

__device__ __forceinline__ void add_comp(BRDFSet& bs, int kind, uint32_t type, V3 R, float a = 0.f, float b = 0.f,
                                         float c = 0.f) {
  (void)type;  // == comp_type(kind), documented at each call
  // Unconditional constant-index stores of selected values: a conditional store lets the
  // optimizer merge the slots into a pointer phi, which pins the set in scratch memory.
#pragma unroll
  for (int i = 0; i < YRT_MAX_COMPS; ++i) {
    const bool w = i == bs.n;
    bs.c[i].kind = w ? kind : bs.c[i].kind;
    bs.c[i].R = v3(w ? R.x : bs.c[i].R.x, w ? R.y : bs.c[i].R.y, w ? R.z : bs.c[i].R.z);
    bs.c[i].a = w ? a : bs.c[i].a;
    bs.c[i].b = w ? b : bs.c[i].b;
    bs.c[i].c = w ? c : bs.c[i].c;
  }
  bs.n = bs.n < YRT_MAX_COMPS ? bs.n + 1 : bs.n;
}

// Material::shade for the in-scope materials (materials/*.h). May modify dg.Ns (Obj bump).
template <unsigned MM>
// t0: the descriptor of m.tex[0] (GpuGeomRec::t0)
__device__ __forceinline__ void shade_material(const SceneView& sv, const GpuMaterial& m, const GpuTexture& t0, int matId,
                                               int medium, DG& dg, BRDFSet& bs) {
  bs.n = 0;
  // each case is compiled only when the instantiation's material set MM holds its type
  const float idBits = __int_as_float(matId);
  switch (m.type) {
    case MAT_PLASTIC:
      if constexpr (!(MM & mat_bit(MAT_PLASTIC))) break;
      // p: pigment[0..2], eta[3], roughness[4], rcpRoughness[5], layer etait[6], etati[7], eta_[8]
      add_comp(bs, C_DIEL_LAYER_LAMB, BT_DIFFUSE_REFLECTION, v3(m.p[0], m.p[1], m.p[2]), m.p[6], m.p[7]);
      if (m.p[4] == 0.0f) add_comp(bs, C_DIEL_REFL, BT_SPECULAR_REFLECTION, v3s(0.f), m.p[8], 1.0f);
      else add_comp(bs, C_MICROFACET, BT_GLOSSY_REFLECTION, v3s(1.f), 1.0f, m.p[3], m.p[5]);
      break;
    case MAT_DIELECTRIC:
      if constexpr (!(MM & mat_bit(MAT_DIELECTRIC))) break;
      // outside -> inside when the ray travels in the outside medium (dielectric.h:42-52)
      if (medium == m.media[0]) {
        add_comp(bs, C_DIEL_REFL, BT_SPECULAR_REFLECTION, v3s(0.f), m.p[8], 1.0f);
        add_comp(bs, C_DIEL_TRANS, BT_SPECULAR_TRANSMISSION, v3s(0.f), m.p[8]);
      } else {
        add_comp(bs, C_DIEL_REFL, BT_SPECULAR_REFLECTION, v3s(0.f), m.p[9], 1.0f);
        add_comp(bs, C_DIEL_TRANS, BT_SPECULAR_TRANSMISSION, v3s(0.f), m.p[9]);
      }
      break;
    case MAT_MIRROR:
      if constexpr (!(MM & mat_bit(MAT_MIRROR))) break;
      add_comp(bs, C_REFLECTION, BT_SPECULAR_REFLECTION, v3(m.p[0], m.p[1], m.p[2]));
      break;
    case MAT_METAL:
      if constexpr (!(MM & mat_bit(MAT_METAL))) break;
      // p: R[0..2], eta[3..5], k[6..8], roughness[9], rcpRoughness[10]
      if (m.p[9] == 0.0f) add_comp(bs, C_CONDUCTOR, BT_SPECULAR_REFLECTION, v3(m.p[0], m.p[1], m.p[2]), 0.f, 0.f, idBits);
      else add_comp(bs, C_MICRO_COND, BT_GLOSSY_REFLECTION, v3(m.p[0], m.p[1], m.p[2]), m.p[10], 0.f, idBits);
      break;
    case MAT_BRUSHED_METAL:
      if constexpr (!(MM & mat_bit(MAT_BRUSHED_METAL))) break;
      // p: R[0..2], eta[3..5], k[6..8], roughnessX[9], roughnessY[10], rcp[11], rcp[12]
      if (m.p[9] == 0.0f || m.p[10] == 0.0f)
        add_comp(bs, C_CONDUCTOR, BT_SPECULAR_REFLECTION, v3(m.p[0], m.p[1], m.p[2]), 0.f, 0.f, idBits);
      else
        add_comp(bs, C_MICRO_ANISO, BT_GLOSSY_REFLECTION, v3(m.p[0], m.p[1], m.p[2]), m.p[11], m.p[12], idBits);
      break;
    case MAT_VELVET:
      if constexpr (!(MM & mat_bit(MAT_VELVET))) break;
      add_comp(bs, C_MINNAERT, BT_DIFFUSE_REFLECTION, v3(m.p[0], m.p[1], m.p[2]), m.p[3]);
      add_comp(bs, C_VELVETY, BT_DIFFUSE_REFLECTION, v3(m.p[4], m.p[5], m.p[6]), m.p[7]);
      break;
    case MAT_MATTE:
      if constexpr (!(MM & mat_bit(MAT_MATTE))) break;
      add_comp(bs, C_LAMBERT, BT_DIFFUSE_REFLECTION, v3(m.p[0], m.p[1], m.p[2]));
      break;
    case MAT_MATTE_TEXTURED:
      if constexpr (!(MM & mat_bit(MAT_MATTE_TEXTURED))) break;
      if (m.tex[0] >= 0) {
        float c[4];
        tex_get_rec(t0, sv.texels, sv.texQuads, m.p[2] * dg.s + m.p[0], m.p[3] * dg.t + m.p[1], c);
        add_comp(bs, C_LAMBERT, BT_DIFFUSE_REFLECTION, v3(c[0], c[1], c[2]));
      }
      break;
    case MAT_METALLIC_PAINT:
      if constexpr (!(MM & mat_bit(MAT_METALLIC_PAINT))) break;
      // p: shadeColor[0..2], eta[3], reflection eta_ [4], layer etait [5], etati [6]
      add_comp(bs, C_DIEL_REFL, BT_SPECULAR_REFLECTION, v3s(0.f), m.p[4], 1.0f);
      add_comp(bs, C_DIEL_LAYER_LAMB, BT_DIFFUSE_REFLECTION, v3(m.p[0], m.p[1], m.p[2]), m.p[5], m.p[6]);
      break;
    case MAT_METALLIC_GLITTER:
      if constexpr (!(MM & mat_bit(MAT_METALLIC_GLITTER))) break;
      // MetallicPaint::shade (metallicpaint.h:58-71); p as above + glitterColor [7..9], n = 1/spread [10]
      add_comp(bs, C_DIEL_REFL, BT_SPECULAR_REFLECTION, v3s(0.f), m.p[4], 1.0f);
      add_comp(bs, C_DIEL_LAYER_LAMB, BT_DIFFUSE_REFLECTION, v3(m.p[0], m.p[1], m.p[2]), m.p[5], m.p[6]);
      add_comp(bs, C_DIEL_LAYER_GLITTER, BT_GLOSSY_REFLECTION, v3(m.p[7], m.p[8], m.p[9]), m.p[5], m.p[6], m.p[10]);
      break;
    case MAT_OBJ: {
      if constexpr (!(MM & mat_bit(MAT_OBJ))) break;
      // p: d[0], Kd[1..3], Ks[4..6], Ns[7]; tex: map_d, map_Kd, map_Ks, map_Ns, map_Bump
      float c[4];
      if (m.tex[4] >= 0) {
        tex_get(sv.textures, sv.images, sv.texels, sv.texQuads, m.tex[4], dg.s, dg.t, c);
        const V3 b = v3(2.0f * c[0] - 1.0f, 2.0f * c[1] - 1.0f, 2.0f * c[2] - 1.0f);
        dg.Ns = normalize(b.x * dg.Tx + b.y * dg.Ty + b.z * dg.Ns);
      }
      float d = m.p[0];
      if (m.tex[0] >= 0) {
        tex_get_rec(t0, sv.texels, sv.texQuads, dg.s, dg.t, c);
        d *= c[0];
      }
      if (d < 1.0f) add_comp(bs, C_TRANSMISSION, BT_SPECULAR_TRANSMISSION, v3s(1.0f - d));
      V3 Kd = d * v3(m.p[1], m.p[2], m.p[3]);
      if (m.tex[1] >= 0) {
        tex_get(sv.textures, sv.images, sv.texels, sv.texQuads, m.tex[1], dg.s, dg.t, c);
        Kd = Kd * v3(c[0], c[1], c[2]);
      }
      if (Kd != v3s(0.f)) add_comp(bs, C_LAMBERT, BT_DIFFUSE_REFLECTION, Kd);
      float Ns = m.p[7];
      if (m.tex[3] >= 0) {
        tex_get(sv.textures, sv.images, sv.texels, sv.texQuads, m.tex[3], dg.s, dg.t, c);
        Ns *= c[0];
      }
      V3 Ks = d * v3(m.p[4], m.p[5], m.p[6]);
      if (m.tex[2] >= 0) {
        tex_get(sv.textures, sv.images, sv.texels, sv.texQuads, m.tex[2], dg.s, dg.t, c);
        Ks = Ks * v3(c[0], c[1], c[2]);
      }
      if (Ks != v3s(0.f)) add_comp(bs, C_SPECULAR, BT_GLOSSY_REFLECTION, Ks, Ns);
      break;
    }
    case MAT_UBER: {
      if constexpr (!(MM & mat_bit(MAT_UBER))) break;
      // p: diffuse[0..2], s0[3..4], ds[5..6], eta[7], roughness[8], reflectivity[9],
      //    rcpRoughness[10], eta_ = 1*rcp(eta) [11]
      float dc[4] = {m.p[0], m.p[1], m.p[2], 1.f};
      float alpha = 1.f, opacity = 0.f;
      if (m.tex[0] >= 0) {
        tex_get_rec(t0, sv.texels, sv.texQuads, m.p[5] * dg.s + m.p[3], m.p[6] * dg.t + m.p[4], dc);
        alpha = dc[3];
        opacity = 1.f - alpha;
      }
      add_comp(bs, C_LAMBERT, BT_DIFFUSE_REFLECTION, v3(dc[0] * alpha, dc[1] * alpha, dc[2] * alpha));
      if (alpha < 1.f) add_comp(bs, C_CONST_DIEL_TRANS, BT_SPECULAR_TRANSMISSION, v3s(opacity));
      if (m.p[9] > 0.f) add_comp(bs, C_DIEL_REFL, BT_SPECULAR_REFLECTION, v3s(0.f), m.p[11], alpha * m.p[9]);
      else if (m.p[8] == 0.f) add_comp(bs, C_DIEL_REFL, BT_SPECULAR_REFLECTION, v3s(0.f), m.p[11], alpha);
      else add_comp(bs, C_MICROFACET, BT_GLOSSY_REFLECTION, v3s(alpha), 1.f, m.p[7], m.p[10]);
      break;
    }
    case MAT_THIN_DIELECTRIC: {
      if constexpr (!(MM & mat_bit(MAT_THIN_DIELECTRIC))) break;
      // p: transmission[0..2], s0[3..4], ds[5..6], eta[7], thickness[8], transparency[9], eta_[10]
      add_comp(bs, C_DIEL_REFL, BT_SPECULAR_REFLECTION, v3s(0.f), m.p[10], 1.0f);
      float dc[4] = {m.p[0], m.p[1], m.p[2], 1.f};
      if (m.tex[0] >= 0)
        tex_get_rec(t0, sv.texels, sv.texQuads, m.p[5] * dg.s + m.p[3], m.p[6] * dg.t + m.p[4], dc);
      const float tr = m.p[9];
      const V3 T = v3(dc[0] * tr, dc[1] * tr, dc[2] * tr);
      add_comp(bs, C_THIN_DIEL_TRANS, BT_SPECULAR_TRANSMISSION, v3(yrt_logf(T.x), yrt_logf(T.y), yrt_logf(T.z)), m.p[10],
               m.p[8]);
      break;
    }
    default:
      break;
  }
}

__device__ __forceinline__ void img_get(const SceneView& sv, int image, int x, int y, float c[4]) {
  texel(sv.images[image], sv.texels, x, y, c);
}

// HDRILight::Le (lights/hdrilight.cpp:43-71)
template <class LT>  // GpuLight, or a YRT_CONST one (scalar loads)
__device__ __forceinline__ V3 hdri_Le(const SceneView& sv, const LT& lt, V3 wo) {
  const A3 w2l = ldA3(lt.w2l);
  const V3 wi = xfmVector(w2l, -wo);
  const float theta = yrt_acosf(clampf(wi.y, -1.0f, 1.0f));
  float phi = yrt_atan2f(-wi.z, -wi.x);
  if (phi < 0) phi += 2.0f * kPi;
  const float u = 1.0f - (phi * kOneOverTwoPi);
  const float v = theta * kOneOverPi;
  const int width = lt.hdriW, height = lt.hdriH;
  int x = max(0, min((int)(u * width), width - 1));
  int xNext = x + 1;
  if (xNext == width) xNext = 0;
  const float alpha = u * width - x;
  int y = max(0, min((int)(v * height), height - 1));
  int yNext = y + 1;
  if (yNext == height) yNext = height - 1;
  const float beta = v * height - y;
  float c0[4], c1[4], c2[4], c3[4];
  img_get(sv, lt.image, x, y, c0);
  img_get(sv, lt.image, xNext, y, c1);
  img_get(sv, lt.image, xNext, yNext, c2);
  img_get(sv, lt.image, x, yNext, c3);
  V3 r;
  float* rr = &r.x;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float temp0 = beta * c3[k] + (1 - beta) * c0[k];
    const float temp1 = beta * c2[k] + (1 - beta) * c1[k];
    rr[k] = lt.L[k] * (alpha * temp1 + (1 - alpha) * temp0);
  }
  return r;
}

// LM: the light types (bit LIGHT_x) an instantiation handles: bits 16.. of the shade kernel's
// instantiation mask (light_bit), which the launcher picks as a superset of the scene's lights.
constexpr unsigned kAllLights = 0x7Fu;
template <unsigned MM>
constexpr unsigned lights_of() { return (MM >> 16) & kAllLights; }
template <unsigned LM, class LT>
__device__ __forceinline__ V3 env_Le(const SceneView& sv, const LT& lt, V3 wo) {
  if ((LM & (1u << LIGHT_AMBIENT)) && lt.type == LIGHT_AMBIENT) return v3(lt.L[0], lt.L[1], lt.L[2]);
  if ((LM & (1u << LIGHT_DISTANT)) && lt.type == LIGHT_DISTANT)  // DistantLight::Le (distantlight.h:38-41)
    return dot(-wo, ld3(lt.e1)) >= lt.bsphere[1] ? v3(lt.L[0], lt.L[1], lt.L[2]) : v3s(0.f);
  if ((LM & (1u << LIGHT_HDRI)) && lt.type == LIGHT_HDRI) return hdri_Le(sv, lt, wo);
  return v3s(0.f);
}

// Light::sample for a non-precomputed light; returns L, sets wi/pdf.
template <unsigned LM, class LT>
__device__ __forceinline__ V3 light_sample(const LT& lt, const DG& dg, float sx, float sy, V3& wi, float& pdf) {
  if ((LM & (1u << LIGHT_AMBIENT)) && lt.type == LIGHT_AMBIENT) {
    // lights/ambientlight.h:52-65 (the bsphere tMax is overwritten by the integrator)
    wi = cosine_hemi_dg(sx, sy, dg, pdf);
    return v3(lt.L[0], lt.L[1], lt.L[2]);
  }
  if ((LM & (1u << LIGHT_TRIANGLE)) && lt.type == LIGHT_TRIANGLE) {
    // lights/trianglelight.h:77-85
    const V3 A = ld3(lt.v0), B = ld3(lt.v1), C = ld3(lt.v2);
    const float su = sqrtf(sx);
    const V3 d = (C + (1.0f - su) * (A - C) + (sy * su) * (B - C)) - dg.P;
    const float tMax = length(d);
    const float dDotNg = dot(d, ld3(lt.Ng));
    if (dDotNg >= 0) {
      pdf = 0.f;
      wi = v3s(0.f);
      return v3s(0.f);
    }
    wi = d * rcpf_(tMax);
    pdf = 2.0f * tMax * tMax * tMax * rcpf_(fabsf(dDotNg));
    return v3(lt.L[0], lt.L[1], lt.L[2]);
  }
  if ((LM & (1u << LIGHT_POINT)) && lt.type == LIGHT_POINT) {  // pointlight.h:36-42
    const V3 d = ld3(lt.v0) - dg.P;
    const float distance = length(d);
    wi = d / distance;
    pdf = distance * distance;
    return v3(lt.L[0], lt.L[1], lt.L[2]);
  }
  if ((LM & (1u << LIGHT_SPOT)) && lt.type == LIGHT_SPOT) {  // spotlight.h:41-52
    const V3 d = ld3(lt.v0) - dg.P;
    const float distance = length(d);
    wi = d * rcpf_(distance);
    pdf = distance * distance;
    const float cosAngle = dot(wi, ld3(lt.e1));
    const float cosMin = lt.bsphere[0], cosMax = lt.bsphere[1];
    if (cosMin != cosMax) return v3(lt.L[0], lt.L[1], lt.L[2]) * clampf((cosAngle - cosMax) * rcpf_(cosMin - cosMax));
    if (cosAngle > cosMin) return v3(lt.L[0], lt.L[1], lt.L[2]);
    return v3s(0.f);
  }
  if ((LM & (1u << LIGHT_DIRECTIONAL)) && lt.type == LIGHT_DIRECTIONAL) {  // directionallight.h:31-33 (Sample3f pdf defaults to 1)
    wi = ld3(lt.e1);
    pdf = 1.0f;
    return v3(lt.L[0], lt.L[1], lt.L[2]);
  }
  if ((LM & (1u << LIGHT_DISTANT)) && lt.type == LIGHT_DISTANT) {  // distantlight.h:46-50, uniformSampleCone (shapesampler.h:149-165)
    const float angle = lt.bsphere[0];
    const float phi = kTwoPi * sx;
    const float cosTheta = 1.0f - sy * (1.0f - yrt_cosf(angle));
    const float sinTheta = cos2sin(cosTheta);
    const V3 l = v3(yrt_cosf(phi) * sinTheta, yrt_sinf(phi) * sinTheta, cosTheta);
    pdf = rcpf_(4.0f * kPi * sqrf(yrt_sinf(0.5f * angle)));
    wi = mul(frame(ld3(lt.e1)), l);
    return v3(lt.L[0], lt.L[1], lt.L[2]);
  }
  pdf = 0.f;
  wi = v3s(0.f);
  return v3s(0.f);
}

// Occupancy target for k_shade. With the material / component / light cases pruned per
// instantiation (if constexpr), the Uber kernel needs 125 VGPRs: 4 waves/SIMD. Same box, C3:
// 3 waves 420.4, 4 waves 419.5, 5 waves 436.9 ms/frame (profiles/r02/shade_prune_r02.txt).
#ifndef YRT_SHADE_WAVES
#define YRT_SHADE_WAVES 4
#endif
#ifndef YRT_SHADE_WAVES_ALL
#define YRT_SHADE_WAVES_ALL 2  // the generic all-types instantiation (rare scenes): no spills at 2
#endif
#ifndef YRT_SHADE_WAVES_MP
#define YRT_SHADE_WAVES_MP YRT_SHADE_WAVES  // instantiations with MetallicPaint (C4's set)
#endif
#ifdef YRT_PATH_DEBUG
// Debug builds only (-DYRT_PATH_DEBUG): per-vertex record of one path (pixel id, sample) of the
// shade kernel, 32 floats per depth, laid out as oracle_debug_path's (tools/c5_path_debug.py).
__device__ int g_dbgPath[2] = {-1, -1};
__device__ float g_dbgTrace[32 * 32];
extern "C" int yrt_debug_path(int pixelId, int sample, float* out) {
  if (!out) {
    const int v[2] = {pixelId, sample};
    static const float z[32 * 32] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_dbgTrace), z, sizeof(z)) != hipSuccess) return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_dbgPath), v, sizeof(v)) == hipSuccess ? 0 : -1;
  }
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dbgTrace), sizeof(g_dbgTrace)) == hipSuccess ? 0 : -1;
}
#endif

template <unsigned MM>
__global__ __launch_bounds__(YRT_BLOCK) __attribute__((amdgpu_waves_per_eu(
    MM == (YRT_ALL_MATS | YRT_ALL_LIGHTS) ? YRT_SHADE_WAVES_ALL
    : (MM & mat_bit(MAT_METALLIC_PAINT)) ? YRT_SHADE_WAVES_MP
                                         : YRT_SHADE_WAVES))) void k_shade(SceneView sv, FrameView fv, PathBuffers pb, BatchInfo bi,
                                                   int depthLevel) {
#ifdef YRT_SHADE_PROF
  // shader-clock cycles per phase (wave-uniform points only), summed over the waves
  unsigned long long sprof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tprev = __builtin_amdgcn_s_memtime();
#define SPROF_AT(k)                                            \
  do {                                                         \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    sprof[k] += t_ - tprev;                                    \
    tprev = t_;                                                \
  } while (0)
#endif
  // YRT_SHADE_PROF=1: one slot per phase; =2: the continuation and direct-light phases split
#if defined(YRT_SHADE_PROF) && YRT_SHADE_PROF == 1
#define SPROF_MARK(k) SPROF_AT(k)
#else
#define SPROF_MARK(k) ((void)0)
#endif
#if defined(YRT_SHADE_PROF) && YRT_SHADE_PROF == 2
#define SPROF_FINE(k) SPROF_AT(k)
#else
#define SPROF_FINE(k) ((void)0)
#endif
  const YRT_CONST GpuRenderParams& rp = const_ref(fv.rp);
  __shared__ QMap qm;
  __shared__ float sstash[7 * YRT_MAX_COMPS * YRT_BLOCK];  // set_sample candidates, [slot][lane]
  qmap_load(qm, pb.counters + qcounter_index(depthLevel, 0, 0), YRT_QSEGS);
  const int n = (int)qm.pre[YRT_QSEGS];
  const int cur = depthLevel & 1;
  const int numDirect = sv.numDirectLights;
  for (int base = blockIdx.x * blockDim.x; base < n; base += gridDim.x * blockDim.x) {
    const unsigned ql = (unsigned)base + threadIdx.x;
    const bool active = (int)ql < n;
    const int q = active ? qmap_phys(qm, pb.segCap, ql) : 0;
    const int oseg = qseg_of((unsigned)base + (threadIdx.x & ~63u));
    unsigned* nextCount = pb.counters + qcounter_index(depthLevel + 1, 0, oseg);
    unsigned* shadowCount = pb.counters + qcounter_index(depthLevel, 1, oseg);
    int path = 0;
    V3 org = v3s(0.f), dir = v3s(0.f), thr = v3s(0.f), L = v3s(0.f);
    int meta = 0, depth = 0, rec = 0, pixelId = 0, s = 0, medium = 0;
    bool ignoreVL = false, unbent = false, isHit = false, useDirect = false;
    bool haveL = false;  // L holds pathL[path] plus this vertex's emission (written back below)
    float4 h = make_float4(0.f, 0.f, 0.f, 0.f);
    int hg = 0;
    DG dg;
    BRDFSet bs;
    bs.n = 0;
#pragma unroll
    for (int k = 0; k < YRT_MAX_COMPS; ++k) {
      bs.c[k].kind = 0;
      bs.c[k].R = v3s(0.f);
      bs.c[k].a = bs.c[k].b = bs.c[k].c = 0.f;
    }
    V3 wo = v3s(0.f);
    int px = 0, py = 0;
    SPROF_MARK(7);
    SPROF_FINE(7);
    if (active) {
      path = pb.qPath[cur][q];
      h = pb.hit[q];
#if YRT_HIT_GEOM
      hg = pb.hitGeom[q];
#endif
      if (depthLevel == 0) {
        // camera rays (k_raygen): throughput 1, depth 0, unbent, vacuum, zero radiance so far;
        // pathL is written below for every queued path
        thr = v3s(1.f);
        meta = 1 << 9;
        L = v3s(0.f);
        haveL = true;
      } else {
        const float4 t4 = pb.qThr[cur][q];
        thr = v3(t4.x, t4.y, t4.z);
        meta = __float_as_int(t4.w);
      }
      depth = meta & 255;
      ignoreVL = (meta >> 8) & 1;
      unbent = (meta >> 9) & 1;
      medium = (meta >> 10) & 0xFFFF;  // LightPath::lastMedium as a medium-table index
      s = fastdiv(path, bi.divPixels);
      const int i = path - s * bi.numPixels;
      batch_pixel(rp, bi, i, px, py);
      pixelId = py * rp.width + px;
      isHit = __float_as_int(h.w) >= 0;
    }
    // the ray's direction, origin and sample record are read where they are used: a miss
    // reads the direction only for an emitting environment light whose Le depends on it, and
    // neither the origin nor the sample record unless it looks up the backplate (a hit issues
    // these loads beside its shading record's, off its dependent chain)
    if (active && (isHit || sv.numEnvDir > 0)) {
      const float4 d = pb.qDir[cur][q];
      dir = v3(d.x, d.y, d.z);
      wo = -dir;
    }
    SPROF_MARK(0);  // queue record, pixel and sample record
    if (active && !isHit) {
      {
        const int x = px, y = py;
        // environment shading (pathtraceintegrator.cpp:79-92): the backplate for a straight
        // camera ray, looked up at the sample's image-plane position (state.pixel)
        if (fv.backplateTexels && unbent) {
          rec = fv.pixelSets[pixelId] * rp.spp + s;
          const float fx = (float(x) + samp(fv, 0, rec)) * rp.rcpWidth;
          const float fy = (float(y) + samp(fv, 1, rec)) * rp.rcpHeight;
          const GpuImage& bp = fv.backplate;
          const int bx = max(0, min((int)(fx * (float)bp.width), bp.width - 1));
          const int by = max(0, min((int)(fy * (float)bp.height), bp.height - 1));
          float c[4];
          texel(bp, fv.backplateTexels, bx, by, c);
          if (!haveL) { const float4 l4 = pb.pathL[path]; L = v3(l4.x, l4.y, l4.z); haveL = true; }
          L = L + thr * v3(c[0], c[1], c[2]);
        } else if (!ignoreVL) {
          for (int j = 0; j < sv.numEnvLights; ++j) {
            if (!haveL) { const float4 l4 = pb.pathL[path]; L = v3(l4.x, l4.y, l4.z); haveL = true; }
            L = L + thr * env_Le<lights_of<MM>()>(sv, const_ref(sv.lights + const_ref(sv.envLights + j)), wo);
          }
          // the zero environment lights' throughput * 0: a no-op unless the throughput is not
          // finite, where the reference's add makes the radiance NaN
          if (sv.numEnvZero > 0 && !(fabsf(thr.x) <= 3.40282347e38f && fabsf(thr.y) <= 3.40282347e38f && fabsf(thr.z) <= 3.40282347e38f)) {
            if (!haveL) { const float4 l4 = pb.pathL[path]; L = v3(l4.x, l4.y, l4.z); haveL = true; }
            L = L + thr * v3s(0.f);
          }
        }
      }
    }
    SPROF_MARK(1);  // misses: environment / backplate
    bool backfacing = false;
    int g = 0;  // the hit's geometry (sv.geomRecs)
    if (active && isHit) {
      const int gid = __float_as_int(h.w);
      const float4* tsr = (const float4*)(sv.triShade + gid);
      const float4 r0 = tsr[0];
      const float4 o = pb.qOrg[cur][q];
      org = v3(o.x, o.y, o.z);
      rec = fv.pixelSets[pixelId] * rp.spp + s;
      // the geometry id comes with the hit (k_trace's hitGeom), so its record is loaded beside
      // the shading record: hit -> {shading record, geometry record} -> texels
#if YRT_HIT_GEOM
      g = hg;
#else
      g = __float_as_int(r0.w);  // geometry id rides in the shading record
#endif
      const GpuGeomRec& gr = sv.geomRecs[g];
      const int mat = gr.g.material;
      // tangents only feed the Obj bump map and the anisotropic microfacet
      const bool wantT = mat >= 0 && (((MM & mat_bit(MAT_OBJ)) && gr.m.type == MAT_OBJ && gr.m.tex[4] >= 0) ||
                                      ((MM & mat_bit(MAT_BRUSHED_METAL)) && gr.m.type == MAT_BRUSHED_METAL));
      post_intersect_rec(sv, gr.g, tsr, r0, org, dir, h.x, h.y, h.z, gid, dg, wantT,
                         pb.qTime[0] ? samp(fv, 4, rec) : 0.f);
      if (dot(dg.Ng, dir) > 0.f) {
        backfacing = true;
        dg.Ng = -dg.Ng;
        dg.Ns = -dg.Ns;
      }
    }
    SPROF_MARK(2);  // postIntersect
    if (active && isHit) {
      if (dg.material >= 0) shade_material<MM>(sv, sv.geomRecs[g].m, sv.geomRecs[g].t0, dg.material, medium, dg, bs);
      if (!ignoreVL && dg.light >= 0 && !backfacing) {
        const GpuLight& al = sv.lights[dg.light];
        if (!haveL) { const float4 l4 = pb.pathL[path]; L = v3(l4.x, l4.y, l4.z); haveL = true; }
        L = L + thr * v3(al.L[0], al.L[1], al.L[2]);
      }
#pragma unroll
      for (int k = 0; k < YRT_MAX_COMPS; ++k)
        if (k < bs.n) useDirect |= (comp_type(bs.c[k].kind) & BT_DIFFUSE) != 0;
      dg_frame(dg);
    }
    SPROF_MARK(3);  // material::shade (textures), emission

    // continuation (pathtraceintegrator.cpp:169-213)
    bool cont = false;
    V3 nwi = v3s(0.f), nthr = v3s(0.f);
    int nmeta = 0;
    bool doSample = false;
    float sx = 0.f, sy = 0.f, ss = 0.f;
    if (active && isHit) {
      bool stop = depth >= rp.maxDepth - 1;
      if (!stop && rp.rrDepth > 0 && depth >= rp.rrDepth - 1) {  // size_t compare in the reference
        const float qrr = fminf(reduce_max(thr) * 1.f * 1.f, .95f);  // eta == 1
        if (samp(fv, 5 + rp.firstScatterTypeSampleID + depth, rec) >= qrr) stop = true;
      }
      if (!stop) {
        const int d2 = rp.firstScatterSampleID + depth;
        sx = samp(fv, 5 + rp.dim1D + 2 * d2, rec);
        sy = samp(fv, 5 + rp.dim1D + 2 * d2 + 1, rec);
        ss = samp(fv, 5 + rp.firstScatterTypeSampleID + depth, rec);
        doSample = true;
      }
    }
    SPROF_FINE(0);  // everything before CompositedBRDF::sample
    float spdf = 0.f;
    uint32_t stype = 0;
    V3 sc = v3s(0.f);
    if (doSample)
      sc = set_sample<comps_of(MM)>(bs, sv.materials, wo, dg, sx, sy, ss, nwi, spdf, stype, sstash + threadIdx.x);
    SPROF_FINE(1);  // CompositedBRDF::sample
    if (doSample) {
      {
        V3 c = sc;
        const float pdf = spdf;
        const uint32_t type = stype;
        if (!(c == v3s(0.f) || pdf <= 0.f)) {
          if (MM & mat_bit(MAT_DIELECTRIC)) {
            // simple volumetric effect and medium tracking (pathtraceintegrator.cpp:197-207)
            const float4 T = sv.media[medium];
            if (!(T.x == 1.f && T.y == 1.f && T.z == 1.f)) c = c * v3(yrt_powf(T.x, h.x), yrt_powf(T.y, h.x), yrt_powf(T.z, h.x));
            if ((type & BT_TRANSMISSION) && dg.material >= 0) {
              const GpuMaterial& mt = sv.materials[dg.material];
              if (mt.type == MAT_DIELECTRIC) medium = medium == mt.media[1] ? mt.media[0] : mt.media[1];
            }
          }
          nthr = thr * c * rcpf_(pdf);
          const bool nIgnore = (type & BT_DIFFUSE) != 0;
          const bool nUnbent = unbent && (nwi == dir);
          // loop head of the next iteration: depth+1 < maxDepth holds; minContribution test
          if (!(reduce_max(nthr) < rp.minContribution)) {
            cont = true;
            nmeta = (depth + 1) | ((nIgnore ? 1 : 0) << 8) | ((nUnbent ? 1 : 0) << 9) | (medium << 10);
          }
        }
      }
    }
    SPROF_MARK(4);  // continuation: CompositedBRDF::sample, Russian roulette
    if (haveL) pb.pathL[path] = make_float4(L.x, L.y, L.z, 0.f);
    // the continuation's records (pathtraceintegrator.cpp:169-213) at queue slot nq
    auto cont_store = [&](unsigned nq) {
      if (pb.qTime[0]) pb.qTime[cur ^ 1][nq] = samp(fv, 4, rec);  // lastRay.time (:210)
      pb.qPath[cur ^ 1][nq] = path;
      pb.qOrg[cur ^ 1][nq] = make_float4(dg.P.x, dg.P.y, dg.P.z, dg.error * rp.epsilon);
      pb.qDir[cur ^ 1][nq] = make_float4(nwi.x, nwi.y, nwi.z, __int_as_float(0x7f800000));
      pb.qThr[cur ^ 1][nq] = make_float4(nthr.x, nthr.y, nthr.z, __int_as_float(nmeta));
    };
    // direct lighting: one shadow ray per light (pathtraceintegrator.cpp:123-167); its
    // contribution is added to pathL[path] after the emission above (reference order)
    auto light_term = [&](int k, V3& wi, float& tfar, V3& contrib) -> bool {
      const int li = const_ref(sv.directLights + k);
      const YRT_CONST GpuLight& lt = const_ref(sv.lights + li);  // scalar loads
      const bool lit = active && isHit && useDirect && (lt.illumMask & dg.illumMask) != 0;
      V3 Ls = v3s(0.f);
      float pdf = 0.f;
      if (lit) {
        if (lt.precomputed >= 0) {
          const float* ls = fv.lightSamples + ((size_t)rec * fv.numLightSlots + lt.precomputed) * 8;
          wi = v3(ls[0], ls[1], ls[2]);
          pdf = ls[3];
          Ls = v3(ls[4], ls[5], ls[6]);
        } else {
          const float lsx = samp(fv, 5 + rp.dim1D + 2 * rp.lightSampleID, rec);
          const float lsy = samp(fv, 5 + rp.dim1D + 2 * rp.lightSampleID + 1, rec);
          Ls = light_sample<lights_of<MM>()>(lt, dg, lsx, lsy, wi, pdf);
        }
      }
      SPROF_FINE(3);  // Light::sample
      const bool lsOk = lit && !(Ls == v3s(0.f) || pdf == 0.f);
      V3 brdf = v3s(0.f);
      if (lsOk) brdf = set_eval<comps_of(MM)>(bs, sv.materials, wo, dg, wi, BT_DIFFUSE);
      SPROF_FINE(4);  // CompositedBRDF::eval
      if (lsOk && !(brdf == v3s(0.f))) {
        const float r01 = hash_u01(rp.frameSeed, (uint32_t)pixelId, (uint32_t)s, (uint32_t)(depth * 64 + li));
        const float shadowRayJitterLength = 2.f * rp.tMaxShadowRay * rp.tMaxShadowJitter * r01 -
                                            rp.tMaxShadowRay * rp.tMaxShadowJitter;
        float tMax = rp.tMaxShadowRay + shadowRayJitterLength;
        const float dotProduct = dot(wi, ld3(rp.up));
        if (dotProduct <= 0.f) tMax += rp.tMaxShadowRay * 100.f * smoothstepf(0.f, 1.f, fabsf(dotProduct));
        tfar = tMax - dg.error * rp.epsilon;
        contrib = thr * Ls * brdf * rcpf_(pdf);
        return true;
      }
      return false;
    };
    // shadow ray records at slot si: origin (dg.P, dg.error * epsilon), direction and tfar, the
    // light's contribution and the path id
    auto shadow_store = [&](unsigned si, const V3& wi, float tfar, const V3& contrib) {
      if (pb.sTime) pb.sTime[si] = samp(fv, 4, rec);  // lastRay.time (:158)
      pb.sOrg[si] = make_float4(dg.P.x, dg.P.y, dg.P.z, dg.error * rp.epsilon);
      pb.sDir[si] = make_float4(wi.x, wi.y, wi.z, tfar);
      pb.sContrib[si] = make_float4(contrib.x, contrib.y, contrib.z, __int_as_float(path));
    };
    {
      bool got;
      const unsigned nq = oseg * pb.segCap + wave_append(nextCount, cont, got);
      if (got) cont_store(nq);
      SPROF_MARK(5);  // continuation append and stores
      SPROF_FINE(2);  // rest of the continuation, append and stores
      for (int k = 0; k < numDirect; ++k) {
        V3 wi = v3s(0.f), contrib = v3s(0.f);
        float tfar = 0.f;
        const bool pred = light_term(k, wi, tfar, contrib);
        SPROF_FINE(5);  // shadow-ray jitter, contribution
        bool sgot;
        const unsigned si = oseg * pb.shSegCap + wave_append(shadowCount, pred, sgot);
        if (sgot) shadow_store(si, wi, tfar, contrib);
        if (active && !pb.fuseShadow) pb.shFirst[(size_t)q * numDirect + k] = sgot ? (int)si : -1;
        SPROF_FINE(6);  // shadow-ray append and stores
      }
    }
    SPROF_MARK(6);  // direct light: light sample, BRDF eval, shadow-ray append and stores
#ifdef YRT_PATH_DEBUG
    if (active && pixelId == g_dbgPath[0] && s == g_dbgPath[1] && depth < 32) {
      float* o = g_dbgTrace + depth * 32;
      if (!haveL) { const float4 l4 = pb.pathL[path]; L = v3(l4.x, l4.y, l4.z); }
      const float r[32] = {1.f, isHit ? (float)__float_as_int(h.w) : -1.f, h.x, h.y, h.z, thr.x, thr.y, thr.z,
                           dg.P.x, dg.P.y, dg.P.z, dg.Ns.x, dg.Ns.y, dg.Ns.z, L.x, L.y, L.z, nwi.x, nwi.y, nwi.z,
                           spdf, sc.x, sc.y, sc.z, nthr.x, nthr.y, nthr.z, dir.x, dir.y, dir.z, org.x, (float)useDirect};
      for (int k = 0; k < 32; ++k) o[k] = r[k];
    }
#endif
  }
#ifdef YRT_SHADE_PROF
  if (threadIdx.x == 0)
    for (int k = 0; k < 8; ++k) atomicAdd(&g_traceProfile[k], sprof[k]);
#endif
}

// Adds the unoccluded direct-light terms in light order.
__global__ __launch_bounds__(YRT_BLOCK) void k_shadow_resolve(PathBuffers pb, int depthLevel, int numLights) {
  __shared__ QMap qm;
  qmap_load(qm, pb.counters + qcounter_index(depthLevel, 0, 0), YRT_QSEGS);
  const int n = (int)qm.pre[YRT_QSEGS];
  const int cur = depthLevel & 1;
  for (int ql = blockIdx.x * blockDim.x + threadIdx.x; ql < n; ql += gridDim.x * blockDim.x) {
    const int q = qmap_phys(qm, pb.segCap, (unsigned)ql);
    bool any = false;
    for (int li = 0; li < numLights; ++li) any |= pb.shFirst[(size_t)q * numLights + li] >= 0;
    if (!any) continue;
    float4* Lp = &pb.pathL[pb.qPath[cur][q]];
    const float4 l4 = *Lp;
    V3 L = v3(l4.x, l4.y, l4.z);
    for (int li = 0; li < numLights; ++li) {
      const int si = pb.shFirst[(size_t)q * numLights + li];
      if (si < 0 || pb.sOcc[si]) continue;
      const float4 c = pb.sContrib[si];
      L = L + v3(c.x, c.y, c.z);
    }
    *Lp = make_float4(L.x, L.y, L.z, 0.f);
  }
}

// Debug capture (yrtDebugPixelSamples): the per-sample radiance of one pixel of one frame,
// in the pixel's summation order, for parity debugging against oracle_debug_pixel.
__device__ int g_dbgPixel[3] = {-1, -1, 0};  // pixel id (y * width + x), frame, capacity of g_dbgOut
__device__ float4* g_dbgOut = nullptr;

// AccuBuffer::update (api/framebuffer.h:289-304) + DefaultToneMapper::eval
// (tonemappers/defaulttonemapper.h:23-36) + FrameBufferRGB8::set (api/framebuffer.h:220-226)
__global__ __launch_bounds__(YRT_BLOCK) void k_resolve_pixels(FrameView fv, PathBuffers pb, BatchInfo bi,
                                                            float* __restrict__ fbFloat, uint8_t* __restrict__ fbRGB8,
                                                            int rgb8Stride, float4* __restrict__ accu, int accumulate) {
  const YRT_CONST GpuRenderParams& rp = const_ref(fv.rp);
  const size_t frameStride = (size_t)rp.width * rp.height;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < bi.numPixels; i += gridDim.x * blockDim.x) {
    int x, y, f;
    if (!batch_pixel(rp, bi, i, x, y, f)) continue;
    V3 L = v3s(0.f);
    for (int s = 0; s < rp.spp; ++s) {
      const float4 l4 = pb.pathL[(size_t)s * bi.numPixels + i];
      L = L + v3(l4.x, l4.y, l4.z);
    }
    if (g_dbgPixel[0] == y * rp.width + x && g_dbgPixel[1] == f && g_dbgOut)
      for (int s = 0; s < min(rp.spp, g_dbgPixel[2]); ++s) g_dbgOut[s] = pb.pathL[(size_t)s * bi.numPixels + i];
    // AccuBuffer::update: non-accumulating frames store (L, spp), accumulating ones add
    const size_t pix = (size_t)f * frameStride + (size_t)y * rp.width + x;
    float4 a = make_float4(L.x, L.y, L.z, (float)rp.spp);
    if (accumulate) {
      const float4 c = accu[pix];
      a = make_float4(c.x + L.x, c.y + L.y, c.z + L.z, c.w + (float)rp.spp);
    }
    accu[pix] = a;
    V3 L0 = accumulate ? v3(a.x, a.y, a.z) * rcpf_(a.w) : L * rcpf_((float)rp.spp);
    if (rp.gamma != 1.0f) L0 = v3(yrt_powf(L0.x, rp.rcpGamma), yrt_powf(L0.y, rp.rcpGamma), yrt_powf(L0.z, rp.rcpGamma));
    if (fbFloat) {
      float* o = fbFloat + pix * 3;
      o[0] = L0.x;
      o[1] = L0.y;
      o[2] = L0.z;
    }
    if (fbRGB8) {
      uint8_t* o = fbRGB8 + ((size_t)f * rp.height + y) * rgb8Stride + 3 * x;
      o[0] = (uint8_t)clampf(L0.x * 255.0f, 0.0f, 255.0f);
      o[1] = (uint8_t)clampf(L0.y * 255.0f, 0.0f, 255.0f);
      o[2] = (uint8_t)clampf(L0.z * 255.0f, 0.0f, 255.0f);
    }
  }
}

// DebugRenderer (renderers/debugrenderer.cpp:66-140): one thread per 16x16 tile, since the
// per-tile Random is consumed sequentially in scan order.
__global__ __launch_bounds__(64) void k_debug(SceneView sv, FrameView fv, int maxDepth, int spp,
                                             float* __restrict__ fbFloat, uint8_t* __restrict__ fbRGB8,
                                             int rgb8Stride) {
  __shared__ int stack[YRT_LDS_STACK * YRT_TRACE_BLOCK];
  const GpuRenderParams& rp = *fv.rp;
  const GpuCamera& cam = *fv.cam;
  const int tile = blockIdx.x * blockDim.x + threadIdx.x;
  if (tile >= rp.numTilesX * rp.numTilesY) return;
  DevRandom rnd;
  rnd.setSeed(tile * 1024);
  const int x0 = (tile % rp.numTilesX) * 16, y0 = (tile / rp.numTilesX) * 16;
  for (int dy = 0; dy < 16; dy++) {
    const int iy = y0 + dy;
    const float fy = iy * rp.rcpHeight;
    if (iy >= rp.height) continue;
    for (int dx = 0; dx < 16; dx++) {
      const int ix = x0 + dx;
      const float fx = ix * rp.rcpWidth;
      if (ix >= rp.width) continue;
      for (int i = 0; i < spp; i++) {
        V3 org, dir;
        camera_ray(cam, fx, fy, org, dir);
        float tnear = 0.f, tfar = __int_as_float(0x7f800000);
        Hit h;
        h.tri = -1;
        int id0 = -1, id1 = -1;
        for (int depth = 0; depth < maxDepth; depth++) {
          RayPre r;
          r.org = org;
          r.dir = dir;
          r.inv = v3(safe_inv(dir.x), safe_inv(dir.y), safe_inv(dir.z));
          r.tnear = tnear;
          r.tfar = tfar;
          h = traverse<false>(sv.nodes, sv.tris, r, stack + threadIdx.x);
          if (h.tri < 0) {
            id0 = id1 = -1;
            break;
          }
          const int g = sv.triGeom[h.tri];
          id0 = g;
          id1 = h.tri - sv.geoms[g].triBase;
          if (depth + 1 < maxDepth) {
            const int4 idx = sv.indices[h.tri];
            const V3 p0 = ld3(sv.positions[idx.x]), p1 = ld3(sv.positions[idx.y]), p2 = ld3(sv.positions[idx.z]);
            const V3 Ng = cross(p0 - p1, p2 - p0);  // ray.Ng
            V3 Nf = normalize(Ng);
            if (dot(-dir, Nf) < 0) Nf = -Nf;
            const float u1 = rnd.getFloat();
            const float u2 = rnd.getFloat();
            float pdf;
            const V3 norg = org + 0.999f * h.t * dir;
            dir = cosine_hemi(u1, u2, Nf, pdf);
            org = norg;
            tnear = 4.0f * kUlp;
            tfar = __int_as_float(0x7f800000);
          }
        }
        V3 c;
        if (id0 < 0) c = v3s(1.0f);
        else
          c = v3(((3434553u * ((unsigned)(id0 + id1 + 3243))) % 255) / 255.0f,
                 ((7342453u * ((unsigned)(id0 + id1 + 8237))) % 255) / 255.0f,
                 ((9234454u * ((unsigned)(id0 + id1 + 2343))) % 255) / 255.0f);
        if (fbFloat) {
          float* o = fbFloat + ((size_t)iy * rp.width + ix) * 3;
          o[0] = c.x;
          o[1] = c.y;
          o[2] = c.z;
        }
        if (fbRGB8) {
          uint8_t* o = fbRGB8 + (size_t)iy * rgb8Stride + 3 * ix;
          o[0] = (uint8_t)clampf(c.x * 255.0f, 0.0f, 255.0f);
          o[1] = (uint8_t)clampf(c.y * 255.0f, 0.0f, 255.0f);
          o[2] = (uint8_t)clampf(c.z * 255.0f, 0.0f, 255.0f);
        }
      }
    }
  }
}

// ---------------------------------------------------------------- launchers

static inline int grid_for(long long n, int block, int maxBlocks) {
  long long g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > maxBlocks) g = maxBlocks;
  return (int)g;
}

void launch_pixel_sets(const FrameView& fv, uint8_t* pixelSets, int width, int height, int sets, hipStream_t s) {
  const int tiles = ((width + 15) / 16) * ((height + 15) / 16);
  hipLaunchKernelGGL(k_pixel_sets, dim3((tiles + 63) / 64), dim3(64), 0, s, fv.rp, pixelSets);
}

void launch_raygen(const FrameView& fv, const PathBuffers& pb, const BatchInfo& bi, hipStream_t s) {
  // spp is read on device; the host passes the path count through capacity sizing.
#ifndef YRT_RAYGEN_GRID
#define YRT_RAYGEN_GRID 16384
#endif
  hipLaunchKernelGGL(k_raygen, dim3(grid_for(pb.capacity, YRT_BLOCK, YRT_RAYGEN_GRID)), dim3(YRT_BLOCK), 0, s, fv, pb, bi);
}

// closest hit: the kernel's int output (occOut, the any-hit occlusion flags) carries the hit's
// geometry id
void launch_trace_closest(const SceneView& sv, const float4* org, const float4* dir, const unsigned* counts,
                          int numSegs, int segCap, float4* hit, hipStream_t s, const float* time, int* hitGeom) {
  if (!YRT_HIT_GEOM) hitGeom = nullptr;
  const dim3 grid(grid_for((long long)numSegs * segCap, YRT_TRACE_BLOCK, YRT_TRACE_GRID));
  if (time)
    hipLaunchKernelGGL((k_trace<false, true>), grid, dim3(YRT_TRACE_BLOCK), 0, s, sv, org, dir, counts, numSegs, segCap,
                       hit, hitGeom, sv.traceSpill, ShadowFuse{}, time, PrimaryRays{});
  else
    hipLaunchKernelGGL((k_trace<false, false>), grid, dim3(YRT_TRACE_BLOCK), 0, s, sv, org, dir, counts, numSegs,
                       segCap, hit, hitGeom, sv.traceSpill, ShadowFuse{}, (const float*)nullptr, PrimaryRays{});
}

void launch_trace_primary(const SceneView& sv, const PrimaryRays& pr, float4* hit, int* hitGeom, hipStream_t s) {
  if (!YRT_HIT_GEOM) hitGeom = nullptr;
  const dim3 grid(grid_for(pr.numPaths, YRT_TRACE_BLOCK, YRT_TRACE_GRID));
  hipLaunchKernelGGL((k_trace<false, false, 1>), grid, dim3(YRT_TRACE_BLOCK), 0, s, sv, (const float4*)nullptr,
                     (const float4*)nullptr, (const unsigned*)nullptr, 0, 0, hit, hitGeom, sv.traceSpill,
                     ShadowFuse{}, (const float*)nullptr, pr);
}

void launch_trace_any(const SceneView& sv, const float4* org, const float4* dir, const unsigned* counts, int numSegs,
                      int segCap, int* occluded, hipStream_t s, const ShadowFuse* fuse, const float* time) {
  const dim3 grid(grid_for((long long)numSegs * segCap, YRT_TRACE_BLOCK, YRT_TRACE_GRID));
  const ShadowFuse sf = fuse ? *fuse : ShadowFuse{};
#if YRT_ANY2
  if (!time) {
    hipLaunchKernelGGL(k_occluded2, grid, dim3(64), 0, s, sv, org, dir, counts, numSegs, segCap, occluded,
                       sv.traceSpill, sf);
    return;
  }
#endif
  if (time)
    hipLaunchKernelGGL((k_trace<true, true>), grid, dim3(YRT_TRACE_BLOCK), 0, s, sv, org, dir, counts, numSegs,
                       segCap, (float4*)nullptr, occluded, sv.traceSpill, sf, time, PrimaryRays{});
  else
    hipLaunchKernelGGL((k_trace<true, false>), grid, dim3(YRT_TRACE_BLOCK), 0, s, sv, org, dir, counts, numSegs,
                       segCap, (float4*)nullptr, occluded, sv.traceSpill, sf, (const float*)nullptr, PrimaryRays{});
}

// Instantiated material sets (bitmask of MAT_x): the launcher picks the smallest superset of
// the scene's material and light types; YRT_SV_ALL is the generic fallback.
// Bits 16.. select the light types (light_bit); the first four cover the reference's scenes
// (dome / quad / HDRI lights).
#define YRT_SV_UBER (mat_bit(MAT_UBER) | YRT_BASIC_LIGHTS)                                   // Collada (Sponza)
#define YRT_SV_OBJ (mat_bit(MAT_OBJ) | YRT_BASIC_LIGHTS)                                     // OBJ scenes
#define YRT_SV_SPHERES (mat_bit(MAT_MATTE) | mat_bit(MAT_METALLIC_PAINT) | YRT_BASIC_LIGHTS)  // cornell spheres
#define YRT_SV_STEREO \
  (mat_bit(MAT_UBER) | mat_bit(MAT_MATTE_TEXTURED) | mat_bit(MAT_METALLIC_PAINT) | YRT_BASIC_LIGHTS)  // test_stereo
// the material types DAELoader emits (Matte default, Uber, ThinDielectric for A_ONE
// transparency; devices/device/loaders/ColladaLoader.cpp:102,210-294): every StartRT .dae job
#define YRT_SV_COLLADA \
  (mat_bit(MAT_MATTE) | mat_bit(MAT_UBER) | mat_bit(MAT_THIN_DIELECTRIC) | YRT_BASIC_LIGHTS)
#define YRT_SV_ALL (YRT_ALL_MATS | YRT_ALL_LIGHTS)
static const unsigned kShadeVariants[] = {YRT_SV_UBER,   YRT_SV_OBJ,     YRT_SV_SPHERES,
                                          YRT_SV_STEREO, YRT_SV_COLLADA, YRT_SV_ALL};

template <unsigned MM>
static void launch_shade_t(const SceneView& sv, const FrameView& fv, const PathBuffers& pb, const BatchInfo& bi,
                           int depth, hipStream_t s) {
#ifndef YRT_SHADE_GRID
#define YRT_SHADE_GRID 16384  // blocks of YRT_BLOCK; swept 2048..32768 (x 256 and 64 lanes)
#endif
  hipLaunchKernelGGL(k_shade<MM>, dim3(grid_for(pb.capacity, YRT_BLOCK, YRT_SHADE_GRID)),
                     dim3(YRT_BLOCK), 0, s, sv, fv, pb,
                     bi, depth);
}

void launch_shade(const SceneView& sv, const FrameView& fv, const PathBuffers& pb, const BatchInfo& bi, int depth,
                  unsigned materialMask, hipStream_t s) {
  unsigned pick = YRT_SV_ALL;
  for (unsigned v : kShadeVariants)
    if ((materialMask & ~v) == 0) {
      pick = v;
      break;
    }
  switch (pick) {
    case YRT_SV_UBER: launch_shade_t<YRT_SV_UBER>(sv, fv, pb, bi, depth, s); break;
    case YRT_SV_OBJ: launch_shade_t<YRT_SV_OBJ>(sv, fv, pb, bi, depth, s); break;
    case YRT_SV_SPHERES: launch_shade_t<YRT_SV_SPHERES>(sv, fv, pb, bi, depth, s); break;
    case YRT_SV_STEREO: launch_shade_t<YRT_SV_STEREO>(sv, fv, pb, bi, depth, s); break;
    case YRT_SV_COLLADA: launch_shade_t<YRT_SV_COLLADA>(sv, fv, pb, bi, depth, s); break;
    default: {
      // the generic kernel (every material and light type) holds ~218 VGPRs, 2 waves/SIMD:
      // say so once per material set, so a scene outside the specialized sets is not slow
      // without a trace
      static std::mutex mu;
      static std::set<unsigned> warned;
      {
        std::lock_guard<std::mutex> lk(mu);
        if (warned.insert(materialMask).second)
          fprintf(stderr,
                  "yrt: material/light set 0x%x has no specialized k_shade; using the generic kernel "
                  "(2 waves/SIMD, slower shading)\n",
                  materialMask);
      }
      launch_shade_t<YRT_SV_ALL>(sv, fv, pb, bi, depth, s);
      break;
    }
  }
}

void launch_shadow_resolve(const PathBuffers& pb, int depth, int numLights, hipStream_t s) {
  hipLaunchKernelGGL(k_shadow_resolve, dim3(grid_for(pb.capacity, YRT_BLOCK, 8192)), dim3(YRT_BLOCK),
                     0, s, pb, depth,
                     numLights);
}

void launch_resolve_pixels(const FrameView& fv, const PathBuffers& pb, const BatchInfo& bi, float* fbFloat,
                           uint8_t* fbRGB8, int rgb8Stride, float4* accu, int accumulate, hipStream_t s) {
  hipLaunchKernelGGL(k_resolve_pixels, dim3(grid_for(bi.numPixels, YRT_BLOCK, 8192)), dim3(YRT_BLOCK), 0, s, fv, pb, bi,
                     fbFloat, fbRGB8, rgb8Stride, accu, accumulate);
}

// ---------------------------------------------------------------- multi-GPU tile slabs
// Slab pixel i of a shard's tile sequence -> (frame f, x, y); frames are numFrames images of
// width x height stacked in memory, tile t = frame t / tilesPerFrame.
__device__ __forceinline__ bool slab_pixel(const SlabLayout& L, int i, int& f, int& x, int& y) {
  const int ntx = (L.width + 15) >> 4;
  int t = L.tileOffset + (i >> 8) * L.tileStride;
  f = t / L.tilesPerFrame;
  t -= f * L.tilesPerFrame;
  if (L.tileStride > 1) t = yrt_tile_scatter(t, L.tilesPerFrame);  // as batch_tile
  x = (t % ntx) * 16 + (i & 15);
  y = (t / ntx) * 16 + ((i >> 4) & 15);
  return x < L.width && y < L.height;
}

// rgb8: the slab holds one 32-bit word per pixel (the RGB8 bytes, what an RGB8 framebuffer
// maps); else float4 (the float pixel, w = the RGB8 bytes)
__global__ __launch_bounds__(256) void k_pack_tiles(const float* __restrict__ fbFloat,
                                                    const uint8_t* __restrict__ fbRGB8, SlabLayout L, int n,
                                                    void* __restrict__ slab) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    int f, x, y;
    const bool in = slab_pixel(L, i, f, x, y);
    unsigned c = 0;
    if (in) {
      const uint8_t* p = fbRGB8 + ((size_t)f * L.height + y) * L.rgb8Stride + 3 * x;
      c = (unsigned)p[0] | ((unsigned)p[1] << 8) | ((unsigned)p[2] << 16);
    }
    if (L.rgb8) {
      ((unsigned*)slab)[i] = c;
    } else {
      float4 v = make_float4(0.f, 0.f, 0.f, __uint_as_float(c));
      if (in) {
        const float* fp = fbFloat + (((size_t)f * L.height + y) * L.width + x) * 3;
        v.x = fp[0];
        v.y = fp[1];
        v.z = fp[2];
      }
      ((float4*)slab)[i] = v;
    }
  }
}

__global__ __launch_bounds__(256) void k_unpack_tiles(const void* __restrict__ slab, float* __restrict__ fbFloat,
                                                      uint8_t* __restrict__ fbRGB8, SlabLayout L, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    int f, x, y;
    if (!slab_pixel(L, i, f, x, y)) continue;
    unsigned c;
    if (L.rgb8) {
      c = ((const unsigned*)slab)[i];
    } else {
      const float4 v = ((const float4*)slab)[i];
      float* fp = fbFloat + (((size_t)f * L.height + y) * L.width + x) * 3;
      fp[0] = v.x;
      fp[1] = v.y;
      fp[2] = v.z;
      c = __float_as_uint(v.w);
    }
    uint8_t* o = fbRGB8 + ((size_t)f * L.height + y) * L.rgb8Stride + 3 * x;
    o[0] = (uint8_t)(c & 255u);
    o[1] = (uint8_t)((c >> 8) & 255u);
    o[2] = (uint8_t)((c >> 16) & 255u);
  }
}

void launch_pack_tiles(const float* fbFloat, const uint8_t* fbRGB8, const SlabLayout& L, int numTiles, void* slab,
                       hipStream_t s) {
  const int n = numTiles * 256;
  if (n <= 0) return;
  hipLaunchKernelGGL(k_pack_tiles, dim3(grid_for(n, 256, 16384)), dim3(256), 0, s, fbFloat, fbRGB8, L, n, slab);
}

void launch_unpack_tiles(const void* slab, float* fbFloat, uint8_t* fbRGB8, const SlabLayout& L, int numTiles,
                         hipStream_t s) {
  const int n = numTiles * 256;
  if (n <= 0) return;
  hipLaunchKernelGGL(k_unpack_tiles, dim3(grid_for(n, 256, 16384)), dim3(256), 0, s, slab, fbFloat, fbRGB8, L, n);
}

// SingleRayDevice::rtPick (api/singleray_device.cpp:692-708): one camera ray at image-plane
// (x, y), lens sample (0.5, 0.5), closest hit.
__global__ __launch_bounds__(YRT_TRACE_BLOCK) void k_pick(SceneView sv, const GpuCamera* camp, float x, float y,
                                                          float4* out) {
  __shared__ int stack[YRT_LDS_STACK * YRT_TRACE_BLOCK];
  if (threadIdx.x != 0) return;
  V3 org, dir;
  camera_ray(*camp, x, y, org, dir);
  RayPre r;
  r.org = org;
  r.dir = dir;
  r.inv = v3(safe_inv(dir.x), safe_inv(dir.y), safe_inv(dir.z));
  r.tnear = 0.f;
  r.tfar = __int_as_float(0x7f800000);
  const Hit h = traverse<false>(sv.nodes, sv.tris, r, stack + threadIdx.x);
  const V3 p = org + h.t * dir;
  out[0] = make_float4(p.x, p.y, p.z, __int_as_float(h.tri));
}

// ---------------------------------------------------------------- arithmetic checks
// fn 0: rcp_rn(x) against the IEEE division 1.0f/x for every 32-bit pattern x.
// Mismatches are counted in out[0]; out[1] = the smallest mismatching input bits.
__global__ __launch_bounds__(256) void k_check_math(int fn, unsigned long long* out) {
  unsigned long long bad = 0, first = ~0ull;
  if (fn == 0) {
    for (unsigned long long i = blockIdx.x * 256ull + threadIdx.x; i < (1ull << 32);
         i += (unsigned long long)gridDim.x * 256ull) {
      const float x = __uint_as_float((uint32_t)i);
      const float got = rcp_rn(x), want = 1.0f / x;
      if (!(__float_as_uint(got) == __float_as_uint(want) || (got != got && want != want))) {
        ++bad;
        first = i < first ? i : first;
      }
    }
  }
  if (bad) {
    atomicAdd(&out[0], bad);
    atomicMin(&out[1], first);
  }
}

// fn 1 / 2: the emulated SSE estimates yrt_rcpps / yrt_rsqrtps (common/yrt_sse_rcp.h) against a
// reconstruction from the 2048-entry table `tab` of 12-bit mantissas (the Intel fixture,
// tests/golden/sse_rcp_tables.json), for every 32-bit pattern; written independently of the
// emulation (the reconstruction of tests/test_sse_rcp.py).
__device__ __forceinline__ uint32_t sse_expect(int fn, uint32_t u, const uint16_t* tab) {
  const uint32_t s = u >> 31, e = (u >> 23) & 0xffu, mant = u & 0x7fffffu;
  if (fn == 1) {
    if (e == 0u) return (s << 31) | 0x7f800000u;
    if (e == 255u) return mant ? (u | 0x400000u) : (s << 31);
    if (e >= 253u) return s << 31;
    return (s << 31) | ((253u - e) << 23) | ((uint32_t)tab[(u >> 12) & 0x7ffu] << 11);
  }
  if (e == 0u) return (s << 31) | 0x7f800000u;
  if (e == 255u && mant) return u | 0x400000u;
  if (s) return 0xffc00000u;
  if (e == 255u) return 0u;
  const int E = (int)e - 127, p = E & 1, k = (E - p) / 2;
  return ((uint32_t)(126 - k) << 23) | ((uint32_t)tab[((uint32_t)p << 10) | ((u >> 13) & 0x3ffu)] << 11);
}
__global__ __launch_bounds__(256) void k_check_math_table(int fn, const uint16_t* __restrict__ tab,
                                                          unsigned long long* out) {
  unsigned long long bad = 0, first = ~0ull;
  for (unsigned long long i = blockIdx.x * 256ull + threadIdx.x; i < (1ull << 32);
       i += (unsigned long long)gridDim.x * 256ull) {
    const uint32_t u = (uint32_t)i;
    const float x = __uint_as_float(u);
    const uint32_t got = __float_as_uint(fn == 1 ? yrt_rcpps(x) : yrt_rsqrtps(x));
    if (got != sse_expect(fn, u, tab)) {
      ++bad;
      first = i < first ? i : first;
    }
  }
  if (bad) {
    atomicAdd(&out[0], bad);
    atomicMin(&out[1], first);
  }
}

int check_math_table(int fn, const uint16_t* table2048, unsigned long long* host2) {
  if (fn != 1 && fn != 2) return -1;
  unsigned long long* d = nullptr;
  uint16_t* t = nullptr;
  if (hipMalloc(&d, 16) != hipSuccess) return -1;
  if (hipMalloc(&t, 4096) != hipSuccess) { (void)hipFree(d); return -1; }
  const unsigned long long init[2] = {0ull, ~0ull};
  int rc = 0;
  if (hipMemcpy(d, init, 16, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(t, table2048, 4096, hipMemcpyHostToDevice) != hipSuccess)
    rc = -1;
  if (!rc) {
    hipLaunchKernelGGL(k_check_math_table, dim3(8192), dim3(256), 0, 0, fn, t, d);
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(host2, d, 16, hipMemcpyDeviceToHost) != hipSuccess) rc = -1;
  }
  (void)hipFree(t);
  (void)hipFree(d);
  return rc;
}

int check_math(int fn, unsigned long long* host2) {
  unsigned long long* d = nullptr;
  if (hipMalloc(&d, 16) != hipSuccess) return -1;
  const unsigned long long init[2] = {0ull, ~0ull};
  int rc = 0;
  if (hipMemcpy(d, init, 16, hipMemcpyHostToDevice) != hipSuccess) rc = -1;
  if (!rc) {
    hipLaunchKernelGGL(k_check_math, dim3(8192), dim3(256), 0, 0, fn, d);
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(host2, d, 16, hipMemcpyDeviceToHost) != hipSuccess) rc = -1;
  }
  (void)hipFree(d);
  return rc;
}

int debug_pixel_capture(int pixelId, int frame, float4* out, int capacity) {
  const int v[3] = {pixelId, frame, out ? capacity : 0};
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_dbgPixel), v, sizeof(v)) != hipSuccess) return -1;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_dbgOut), &out, sizeof(out)) != hipSuccess) return -1;
  return 0;
}

int trace_profile(unsigned long long* out8, int reset) {
#if defined(YRT_PROFILE) || defined(YRT_SHADE_PROF)
  if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_traceProfile), 8 * sizeof(unsigned long long)) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_traceProfile), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
#else
  (void)out8;
  (void)reset;
  return -1;
#endif
}

void launch_pick(const SceneView& sv, const GpuCamera* cam, float x, float y, float4* out, hipStream_t s) {
  hipLaunchKernelGGL(k_pick, dim3(1), dim3(YRT_TRACE_BLOCK), 0, s, sv, cam, x, y, out);
}

void launch_debug_render(const SceneView& sv, const FrameView& fv, int maxDepth, int spp, int numTiles, float* fbFloat,
                         uint8_t* fbRGB8, int rgb8Stride, hipStream_t s) {
  hipLaunchKernelGGL(k_debug, dim3((numTiles + 63) / 64), dim3(64), 0, s, sv, fv, maxDepth, spp, fbFloat, fbRGB8,
                     rgb8Stride);
}

}  // namespace yrt

namespace yrt {

// ---------------------------------------------------------------- BVH refit (faceCamera)
// Per-face dynamic geometry (rtUpdatePrimitive of YULIO_CAMERA_ALIGNED_ meshes,
// singleray_device.cpp:354-398) keeps the BVH topology and only moves vertices: the moved
// triangles' Moeller-Trumbore records are rewritten from the new world vertices, then the
// node boxes are refit bottom-up, one launch per tree level (deepest first). The reference
// rebuilt the whole Embree BVH on every face commit. Boxes stay the exact
// union of the original vertex bounds (what the builder computes), so the hits are identical
// to a rebuild's: the closest hit is the smallest (t, triangle id) whatever the tree.
__global__ __launch_bounds__(YRT_BLOCK) void k_refit_tris(GpuTri* __restrict__ tris, GpuTriShade* __restrict__ triShade,
                                                         const int4* __restrict__ indices,
                                                         const float4* __restrict__ positions,
                                                         const float4* __restrict__ normals,
                                                         const int* __restrict__ leafStart,
                                                         const int* __restrict__ leafSlots, int firstTri, int numTris) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= numTris) return;
  const int gid = firstTri + i;
  const int4 ix = indices[gid];
  const float4 a = positions[ix.x], b = positions[ix.y], c = positions[ix.z];
  // the shading record's edges and vertex normals (scene_gpu.cpp builds it the same way)
  GpuTriShade& ts = triShade[gid];
  ts.e1[0] = a.x - b.x; ts.e1[1] = a.y - b.y; ts.e1[2] = a.z - b.z;
  ts.e2[0] = c.x - a.x; ts.e2[1] = c.y - a.y; ts.e2[2] = c.z - a.z;
  const float4 na = normals[ix.x], nb = normals[ix.y], nc = normals[ix.z];
  ts.n[0] = na.x; ts.n[1] = na.y; ts.n[2] = na.z;
  ts.n[3] = nb.x; ts.n[4] = nb.y; ts.n[5] = nb.z;
  ts.n[6] = nc.x; ts.n[7] = nc.y; ts.n[8] = nc.z;
  // every leaf slot referencing the triangle (spatial splits duplicate references)
  for (int k = leafStart[gid]; k < leafStart[gid + 1]; ++k) {
    GpuTri& t = tris[leafSlots[k]];
    // e1 = v0 - v1, e2 = v2 - v0 (device/bvh_build.cpp, rtcore convention); .w words kept
    t.v0[0] = a.x; t.v0[1] = a.y; t.v0[2] = a.z;
    t.e1[0] = a.x - b.x; t.e1[1] = a.y - b.y; t.e1[2] = a.z - b.z;
    t.e2[0] = c.x - a.x; t.e2[1] = c.y - a.y; t.e2[2] = c.z - a.z;
  }
}

__global__ __launch_bounds__(YRT_BLOCK) void k_refit_nodes(GpuNode* __restrict__ nodes, const GpuTri* __restrict__ tris,
                                                          const int4* __restrict__ indices,
                                                          const float4* __restrict__ positions,
                                                          const int* __restrict__ levelNodes, int count) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  GpuNode& n = nodes[levelNodes[i]];
  for (int k = 0; k < 4; ++k) {
    const int c = n.child[k];
    if (c == -1) continue;
    const int idx = c >> 5, cnt = c & 31;
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    if (cnt > 0) {
      for (int t = 0; t < cnt; ++t) {
        const int gid = __float_as_int(tris[idx + t].v0[3]);
        const int4 ix = indices[gid];
        const float4 p[3] = {positions[ix.x], positions[ix.y], positions[ix.z]};
        for (int v = 0; v < 3; ++v) {
          lo[0] = fminf(lo[0], p[v].x); hi[0] = fmaxf(hi[0], p[v].x);
          lo[1] = fminf(lo[1], p[v].y); hi[1] = fmaxf(hi[1], p[v].y);
          lo[2] = fminf(lo[2], p[v].z); hi[2] = fmaxf(hi[2], p[v].z);
        }
      }
    } else {
      const GpuNode& ch = nodes[idx];
      for (int j = 0; j < 4; ++j) {
        if (ch.child[j] == -1) continue;
        lo[0] = fminf(lo[0], ch.lox[j]); hi[0] = fmaxf(hi[0], ch.hix[j]);
        lo[1] = fminf(lo[1], ch.loy[j]); hi[1] = fmaxf(hi[1], ch.hiy[j]);
        lo[2] = fminf(lo[2], ch.loz[j]); hi[2] = fmaxf(hi[2], ch.hiz[j]);
      }
    }
    n.lox[k] = lo[0]; n.hix[k] = hi[0];
    n.loy[k] = lo[1]; n.hiy[k] = hi[1];
    n.loz[k] = lo[2]; n.hiz[k] = hi[2];
  }
}

__global__ __launch_bounds__(YRT_BLOCK) void k_quantize_nodes(const GpuNode* __restrict__ nodes,
                                                             GpuQNode* __restrict__ qnodes, int count) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  GpuQNode q;
  yrt_quantize_node(nodes[i], q);  // the host builder's function: the same bytes
  qnodes[i] = q;
}

bool trace_hit_geom() { return YRT_HIT_GEOM != 0; }

int trace_node_bytes(bool anyHit) {
  return (anyHit ? YRT_QNODES_ANY : YRT_QNODES_CLOSEST) ? (int)sizeof(GpuQNode) : (int)sizeof(GpuNode);
}

void launch_quantize_nodes(const GpuNode* nodes, GpuQNode* qnodes, int count, hipStream_t s) {
  if (count <= 0) return;
  hipLaunchKernelGGL(k_quantize_nodes, dim3((count + YRT_BLOCK - 1) / YRT_BLOCK), dim3(YRT_BLOCK), 0, s, nodes, qnodes,
                     count);
}

void launch_refit_tris(GpuTri* tris, GpuTriShade* triShade, const int4* indices, const float4* positions,
                       const float4* normals, const int* leafStart, const int* leafSlots, int firstTri, int numTris,
                       hipStream_t s) {
  if (numTris <= 0) return;
  hipLaunchKernelGGL(k_refit_tris, dim3((numTris + YRT_BLOCK - 1) / YRT_BLOCK), dim3(YRT_BLOCK), 0, s, tris, triShade,
                     indices, positions, normals, leafStart, leafSlots, firstTri, numTris);
}

void launch_refit_nodes(GpuNode* nodes, const GpuTri* tris, const int4* indices, const float4* positions,
                        const int* levelNodes, int count, hipStream_t s) {
  if (count <= 0) return;
  hipLaunchKernelGGL(k_refit_nodes, dim3((count + YRT_BLOCK - 1) / YRT_BLOCK), dim3(YRT_BLOCK), 0, s, nodes, tris,
                     indices, positions, levelNodes, count);
}

}  // namespace yrt
