// yrt_traverse.h — 4-wide BVH traversal + Embree-convention triangle test, device side.
//
// Replaces Embree 2.15 rtcIntersect / rtcOccluded (call sites
// integrators/pathtraceintegrator.cpp:72,160, renderers/debugrenderer.cpp:109).
//
// Hit convention (restated from the in-tree copy lights/trianglelight.h:55-65 and the
// rtcore triangle layout; Embree itself is binary-only so this is "parity unpinned"
// against Embree and pinned against oracle/):
//   e1 = v0-v1, e2 = v2-v0, Ng = cross(e1,e2), C = v0-O, R = cross(D,C)  (tri_cross)
//   den = dot(Ng,D), U = dot(R,e2)*sgn(den), V = dot(R,e1)*sgn(den), T = dot(Ng,C)*sgn(den)
//   valid: den != 0, U >= 0, V >= 0, U+V <= |den|, tnear < t=T/|den| < tfar
//   back-face filter (cullBackFaces meshes, shapes/trianglemesh_full.cpp:86-106): reject den <= 0
//   closest hit: smallest (t, global triangle id) — order independent, so any BVH gives
//   the same answer (used to pin the GPU against the oracle's own BVH).
// Stack: per-lane short stack in LDS, [depth][lane] so a wave's pushes hit 64 distinct
// banks. Only the top entries live in LDS, a ring of 16 per lane (4 KB per 64-lane block) for
// every traversal kind since round 6; deeper entries spill to global memory. History: closest
// hit on the float nodes, 32 entries instead of 16: +4.9 % on C3 in round 1, still +2 % in
// round 6; on the 64-B quantized nodes 16 entries win (6 waves/SIMD, C3 +5.3 %, pathtrace.hip).
// The builder bounds the tree depth to YRT_STACK_DEPTH-1 (device/bvh_build.cpp).
#pragma once

#include "../common/yrt_gpu_types.h"
#include "../common/yrt_math.h"
#include "../common/yrt_qnode.h"

#ifndef YRT_STACK_DEPTH
#define YRT_STACK_DEPTH 64   // bound on traversal stack entries + 1 (device/bvh_build.cpp enforces it)
#endif
#ifndef YRT_LDS_STACK
#define YRT_LDS_STACK 16     // top entries kept in LDS; deeper ones spill (power of two); Makefile LDSSTACK
#endif
static_assert((YRT_LDS_STACK & (YRT_LDS_STACK - 1)) == 0, "YRT_LDS_STACK must be a power of two");
#ifndef YRT_LDS_STACK_ANY
// LDS ring of the any-hit (shadow) instantiation: 16 entries (4.2 KB per wave). On the 64-B
// quantized nodes that kernel needs 72 VGPRs, so with 32 entries (8.3 KB) LDS held it at 4.75
// waves/SIMD and with 16 registers allow 7: same box (profiles/r06/ab_r06f.txt) C5 -5.0 %, C4
// -1 %, C3 +0.2 %. (On the float nodes, at 5 waves either way, 16 entries were 3.3 % slower.)
#define YRT_LDS_STACK_ANY 16
#endif
static_assert((YRT_LDS_STACK_ANY & (YRT_LDS_STACK_ANY - 1)) == 0, "YRT_LDS_STACK_ANY must be a power of two");
#ifndef YRT_LDS_STACK_PRIM
// LDS ring of the fused depth-0 (camera ray) instantiation: 16 entries. The kernel stays at 5
// waves/SIMD (96 VGPRs) either way, but the 4 KB ring leaves LDS for the other lanes' kernels
// running beside it: same box (profiles/r06/ab_r06i.txt) C4 -1.3 %, its N = 8 share -2 %, C3
// and C5 within the spread (on the float nodes, when the queued closest-hit kernels kept 32).
#define YRT_LDS_STACK_PRIM 16
#endif
static_assert((YRT_LDS_STACK_PRIM & (YRT_LDS_STACK_PRIM - 1)) == 0, "YRT_LDS_STACK_PRIM must be a power of two");
#define YRT_LDS_STACK_MIN2 (YRT_LDS_STACK < YRT_LDS_STACK_ANY ? YRT_LDS_STACK : YRT_LDS_STACK_ANY)
#define YRT_LDS_STACK_MIN (YRT_LDS_STACK_MIN2 < YRT_LDS_STACK_PRIM ? YRT_LDS_STACK_MIN2 : YRT_LDS_STACK_PRIM)
#ifndef YRT_ANY2
#define YRT_ANY2 0  // 1: static scenes' shadow queries run two rays per lane (k_occluded2)
#endif
#ifndef YRT_ANY2_LDS
#define YRT_ANY2_LDS 16  // LDS ring entries per ray slot of k_occluded2
#endif
static_assert((YRT_ANY2_LDS & (YRT_ANY2_LDS - 1)) == 0, "YRT_ANY2_LDS must be a power of two");
#ifndef YRT_TRACE_BLOCK
// one wave per block (8 KB of LDS stack): +1.0 % on C3 over 128-lane blocks once the trace code
// was scheduled for a 6-wave target (profiles/r01/variants_r01.txt)
#define YRT_TRACE_BLOCK 64
#endif

namespace yrt {

struct Hit {
  float t, u, v;
  int tri;  // global triangle id, -1 = miss
};

// Slab exit-distance factor 1 + 2^-16 (robust box test; Embree flags ROBUST,
// api/scene_flat.h:75-80). The triangle test accepts hits a rounding error outside the
// triangle: on a sliver-thin or tiny triangle that is more than the 1 + 2*gamma(3) a box test
// needs for its own rounding (C5, pixel 1081,772 sample 191: a hit 1.2e-6 of the distance
// outside its leaf box, tests/test_cubes.py full-size band). The closest hit is the smallest
// (t, triangle id) over every triangle the test accepts only if no box holding one is culled,
// so the factor is wide enough for the triangle test's errors; the oracle uses the same one.
#ifndef YRT_BOX_ROBUST
#define YRT_BOX_ROBUST 1.0000152587890625f
#endif

__device__ __forceinline__ float safe_inv(float d) {
  return rcp_rn(fabsf(d) > 1e-20f ? d : copysignf(1e-20f, d));  // correctly rounded: the bits of 1.0f / x
}

struct RayPre {
  V3 org, dir, inv;
  float tnear, tfar;
  V3 oi;         // org * inv (rounded): slab distances as fma(plane, inv, -oi) (box4_ordered)
  float margin;  // absolute slack of those distances: 2^-22 * max |oi| (see box4_ordered)
};

// Per-ray constants of box4_ordered's fused slab test.
__device__ __forceinline__ void ray_slab_consts(const V3& org, const V3& inv, V3& oi, float& margin) {
  oi = v3(org.x * inv.x, org.y * inv.y, org.z * inv.z);
  margin = fmaxf(fmaxf(fabsf(oi.x), fabsf(oi.y)), fabsf(oi.z)) * 2.384185791015625e-07f;  // 2^-22
}

// Entry distances of the four children of a 4-wide node (INFINITY = missed / empty slot).
// Slab distances (b - o) * inv are computed two children at a time with packed ops
// (v_pk_add_f32 / v_pk_mul_f32); the robust factor widens the exit distance as before.
__device__ __forceinline__ void box4(const GpuNode* __restrict__ np, const RayPre& r, float tmax, float t[4],
                                     int c[4]) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  const float4* q = (const float4*)np;
  const float4 lx = q[0], hx = q[1], ly = q[2], hy = q[3], lz = q[4], hz = q[5];
  const int4 ch = *(const int4*)(q + 6);
  const f2 ox = {r.org.x, r.org.x}, oy = {r.org.y, r.org.y}, oz = {r.org.z, r.org.z};
  const f2 ix = {r.inv.x, r.inv.x}, iy = {r.inv.y, r.inv.y}, iz = {r.inv.z, r.inv.z};
  const f2 lx01 = (f2{lx.x, lx.y} - ox) * ix, lx23 = (f2{lx.z, lx.w} - ox) * ix;
  const f2 hx01 = (f2{hx.x, hx.y} - ox) * ix, hx23 = (f2{hx.z, hx.w} - ox) * ix;
  const f2 ly01 = (f2{ly.x, ly.y} - oy) * iy, ly23 = (f2{ly.z, ly.w} - oy) * iy;
  const f2 hy01 = (f2{hy.x, hy.y} - oy) * iy, hy23 = (f2{hy.z, hy.w} - oy) * iy;
  const f2 lz01 = (f2{lz.x, lz.y} - oz) * iz, lz23 = (f2{lz.z, lz.w} - oz) * iz;
  const f2 hz01 = (f2{hz.x, hz.y} - oz) * iz, hz23 = (f2{hz.z, hz.w} - oz) * iz;
  const float INF = __int_as_float(0x7f800000);
#define YRT_CHILD(k, LX, HX, LY, HY, LZ, HZ, CH)                                                          \
  do {                                                                                                    \
    const float nn = fmaxf(fmaxf(fminf(LX, HX), fminf(LY, HY)), fmaxf(fminf(LZ, HZ), r.tnear));          \
    const float ff = fminf(fminf(fmaxf(LX, HX), fmaxf(LY, HY)), fminf(fmaxf(LZ, HZ), tmax));             \
    t[k] = ((nn <= ff * YRT_BOX_ROBUST) && (CH) != -1) ? nn : INF;                                        \
    c[k] = (CH);                                                                                          \
  } while (0)
  YRT_CHILD(0, lx01.x, hx01.x, ly01.x, hy01.x, lz01.x, hz01.x, ch.x);
  YRT_CHILD(1, lx01.y, hx01.y, ly01.y, hy01.y, lz01.y, hz01.y, ch.y);
  YRT_CHILD(2, lx23.x, hx23.x, ly23.x, hy23.x, lz23.x, hz23.x, ch.z);
  YRT_CHILD(3, lx23.y, hx23.y, ly23.y, hy23.y, lz23.y, hz23.y, ch.w);
#undef YRT_CHILD
}

// Same entry distances as box4, with the near/far plane of each axis picked per ray by the
// sign of its inverse direction instead of a min/max per slab: planeOff packs the byte
// offsets (0 or 16) of the near plane within the lo/hi pair of x, y, z in bits 0-7, 8-15,
// 16-23. Rounding is monotonic, so for lo <= hi the ordered planes give bit-identical slab
// distances to min/max and the traversal is unchanged; it saves 24 VALU ops per node.
__device__ __forceinline__ int plane_offsets(float ix, float iy, float iz) {
  return ((__float_as_uint(ix) >> 27) & 16) | ((__float_as_uint(iy) >> 19) & (16 << 8)) |
         ((__float_as_uint(iz) >> 11) & (16 << 16));
}
// Empty slots carry inverted infinite boxes (device/bvh_build.cpp), which the ordered-plane
// test culls by itself, so no child-reference check is needed. The six plane loads and the
// child load address the node array as a uniform (SGPR) base plus a 32-bit per-lane byte
// offset (global_load saddr form) instead of six 64-bit per-lane pointers (78/74 VGPRs instead
// of 82/84). nodeIdx < 2^25 (node byte offsets fit 32 bits; bvh_build.cpp enforces it).
// MISS: the entry distance reported for a missed child (+INF for closest-hit rays, which sort
// ascending; -INF for any-hit rays, which visit the farthest child first, see sort3_far).
// The ray's near/far planes and the child references of one node, as loaded.
struct NodeData {
  float4 nx, fx, ny, fy, nz, fz;
  int4 ch;
};
__device__ __forceinline__ NodeData node_load(const GpuNode* __restrict__ base, int nodeIdx, int planeOff) {
  const char* b0 = (const char*)base;
  const unsigned nb = (unsigned)nodeIdx << 7;
  const unsigned ox = (unsigned)planeOff & 0xffu, oy = ((unsigned)planeOff >> 8) & 0xffu,
                 oz = (unsigned)planeOff >> 16;
  NodeData d;
  d.nx = *(const float4*)(b0 + (nb + ox));
  d.fx = *(const float4*)(b0 + (nb + (16u - ox)));
  d.ny = *(const float4*)(b0 + (nb + (32u + oy)));
  d.fy = *(const float4*)(b0 + (nb + (48u - oy)));
  d.nz = *(const float4*)(b0 + (nb + (64u + oz)));
  d.fz = *(const float4*)(b0 + (nb + (80u - oz)));
  d.ch = *(const int4*)(b0 + (nb + 96u));
  return d;
}
template <bool ANY = false>
__device__ __forceinline__ void box4_data(const NodeData& d, const RayPre& r, float tmax, float t[4], int c[4]);
template <bool ANY = false>
__device__ __forceinline__ void box4_ordered(const RayPre& r, int planeOff, float tmax, float t[4], int c[4],
                                             const GpuNode* __restrict__ base, int nodeIdx) {
  box4_data<ANY>(node_load(base, nodeIdx, planeOff), r, tmax, t, c);
}
template <bool ANY>
__device__ __forceinline__ void box4_data(const NodeData& d, const RayPre& r, float tmax, float t[4], int c[4]) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  const float4 nx = d.nx, fx = d.fx, ny = d.ny, fy = d.fy, nz = d.nz, fz = d.fz;
  const int4 ch = d.ch;
  // slab distance t = fma(plane, inv, -org*inv): one fused op per plane instead of a subtract
  // and a multiply. Against (plane - org) * inv it carries an extra absolute error of at most
  // one rounding of org*inv (u * |oi|, u = 2^-24) on each of the near and far distances; the
  // far plane is widened by margin = 4u * max|oi| on top of the robust factor (relative
  // errors, as before), so the test stays conservative: a box the ray meets is never culled,
  // and the closest hit (smallest (t, triangle id)) is the same for any visit order.
  const f2 ix = {r.inv.x, r.inv.x}, iy = {r.inv.y, r.inv.y}, iz = {r.inv.z, r.inv.z};
  const f2 mx = {-r.oi.x, -r.oi.x}, my = {-r.oi.y, -r.oi.y}, mz = {-r.oi.z, -r.oi.z};
#define YRT_SLAB(P, I, M) __builtin_elementwise_fma(P, I, M)
  const f2 nx01 = YRT_SLAB((f2{nx.x, nx.y}), ix, mx), nx23 = YRT_SLAB((f2{nx.z, nx.w}), ix, mx);
  const f2 fx01 = YRT_SLAB((f2{fx.x, fx.y}), ix, mx), fx23 = YRT_SLAB((f2{fx.z, fx.w}), ix, mx);
  const f2 ny01 = YRT_SLAB((f2{ny.x, ny.y}), iy, my), ny23 = YRT_SLAB((f2{ny.z, ny.w}), iy, my);
  const f2 fy01 = YRT_SLAB((f2{fy.x, fy.y}), iy, my), fy23 = YRT_SLAB((f2{fy.z, fy.w}), iy, my);
  const f2 nz01 = YRT_SLAB((f2{nz.x, nz.y}), iz, mz), nz23 = YRT_SLAB((f2{nz.z, nz.w}), iz, mz);
  const f2 fz01 = YRT_SLAB((f2{fz.x, fz.y}), iz, mz), fz23 = YRT_SLAB((f2{fz.z, fz.w}), iz, mz);
#undef YRT_SLAB
  const float MISS = __int_as_float(ANY ? 0xff800000 : 0x7f800000);
  // v_max/v_min written out (+1.5 % on C3, shadow trace 5.84 -> 5.38 ms/launch,
  // profiles/r02/trace_variants_r02.txt): fmaxf/fminf on the loop-carried tnear / tfar make
  // the compiler re-quiet (canonicalize) them with an extra v_max every node step (IEEE mode). A signalling
  // NaN never reaches here (ray records are computed values), and the hardware min/max give
  // the same result as fmaxf/fminf for every other input.
#define YRT_CHILD(k, NX, FX, NY, FY, NZ, FZ, CH)                                            \
  do {                                                                                      \
    float nn, ff, a_, b_;                                                                   \
    asm("v_max_f32 %0, %1, %2" : "=v"(a_) : "v"(NZ), "v"(r.tnear));                         \
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(nn) : "v"(NX), "v"(NY), "v"(a_));                \
    asm("v_min_f32 %0, %1, %2" : "=v"(b_) : "v"(FZ), "v"(tmax));                            \
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(ff) : "v"(FX), "v"(FY), "v"(b_));                \
    t[k] = nn <= __builtin_fmaf(ff, YRT_BOX_ROBUST, r.margin) ? nn : MISS;                  \
    c[k] = (CH);                                                                            \
  } while (0)
  YRT_CHILD(0, nx01.x, fx01.x, ny01.x, fy01.x, nz01.x, fz01.x, ch.x);
  YRT_CHILD(1, nx01.y, fx01.y, ny01.y, fy01.y, nz01.y, fz01.y, ch.y);
  YRT_CHILD(2, nx23.x, fx23.x, ny23.x, fy23.x, nz23.x, fz23.x, ch.z);
  YRT_CHILD(3, nx23.y, fx23.y, ny23.y, fy23.y, nz23.y, fz23.y, ch.w);
#undef YRT_CHILD
}

// box4_ordered on the 64-B quantized node of the same index (common/yrt_qnode.h): one 64-B line
// (four loads: origin + quantum exponents, children, lo/hi words of x and y, of z) instead of
// seven 16-B loads from 128 B. Per axis a = fma(origin, inv, -org * inv) and s = 2^e * inv
// (exact); per plane one v_cvt_f32_ubyte and one FMA (packed two children at a time), the near
// and far words picked by the ray's direction signs (planeOff, as box4_ordered). The planes lie
// at least one quantum outside the float node's child boxes, which covers a's rounding (see
// yrt_qnode.h), so the same boxes are never culled and every query returns the same bits.
// Empty slots are tested by their child reference.
// The quantized node as loaded (14 words).
struct QNodeData {
  float4 h;   // origin xyz, quantum exponents
  int4 ch;
  uint4 pa;   // lo x, hi x, lo y, hi y
  uint2 pb;   // lo z, hi z
};
__device__ __forceinline__ QNodeData qnode_load(const GpuQNode* __restrict__ base, int nodeIdx) {
  const char* b0 = (const char*)base + ((unsigned)nodeIdx << 6);
  QNodeData d;
  d.h = *(const float4*)b0;
  d.ch = *(const int4*)(b0 + 16);
  d.pa = *(const uint4*)(b0 + 32);
  d.pb = *(const uint2*)(b0 + 48);
  return d;
}
template <bool ANY>
__device__ __forceinline__ void box4_qdata(const QNodeData& d, const RayPre& r, int planeOff, float tmax, float t[4],
                                           int c[4]);
template <bool ANY>
__device__ __forceinline__ void box4_quant(const RayPre& r, int planeOff, float tmax, float t[4], int c[4],
                                           const GpuQNode* __restrict__ base, int nodeIdx) {
  box4_qdata<ANY>(qnode_load(base, nodeIdx), r, planeOff, tmax, t, c);
}
template <bool ANY>
__device__ __forceinline__ void box4_qdata(const QNodeData& d, const RayPre& r, int planeOff, float tmax, float t[4],
                                           int c[4]) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  const float4 h = d.h;
  const int4 ch = d.ch;
  const uint4 pa = d.pa;
  const uint2 pb = d.pb;
  const uint32_t ex = __float_as_uint(h.w);
  const float sx = __uint_as_float((ex & 0xffu) << 23) * r.inv.x;
  const float sy = __uint_as_float(((ex >> 8) & 0xffu) << 23) * r.inv.y;
  const float sz = __uint_as_float(((ex >> 16) & 0xffu) << 23) * r.inv.z;
  const float ax = __builtin_fmaf(h.x, r.inv.x, -r.oi.x);
  const float ay = __builtin_fmaf(h.y, r.inv.y, -r.oi.y);
  const float az = __builtin_fmaf(h.z, r.inv.z, -r.oi.z);
  const bool hx = (planeOff & 16) != 0, hy = (planeOff & (16 << 8)) != 0, hz = (planeOff & (16 << 16)) != 0;
  const uint32_t nwx = hx ? pa.y : pa.x, fwx = hx ? pa.x : pa.y;
  const uint32_t nwy = hy ? pa.w : pa.z, fwy = hy ? pa.z : pa.w;
  const uint32_t nwz = hz ? pb.y : pb.x, fwz = hz ? pb.x : pb.y;
#define YRT_QB(w, k) ((float)(((w) >> (8 * (k))) & 0xffu))
#define YRT_QSLAB(W, S, A, k0, k1) __builtin_elementwise_fma((f2{YRT_QB(W, k0), YRT_QB(W, k1)}), (f2{S, S}), (f2{A, A}))
  const f2 nx01 = YRT_QSLAB(nwx, sx, ax, 0, 1), nx23 = YRT_QSLAB(nwx, sx, ax, 2, 3);
  const f2 fx01 = YRT_QSLAB(fwx, sx, ax, 0, 1), fx23 = YRT_QSLAB(fwx, sx, ax, 2, 3);
  const f2 ny01 = YRT_QSLAB(nwy, sy, ay, 0, 1), ny23 = YRT_QSLAB(nwy, sy, ay, 2, 3);
  const f2 fy01 = YRT_QSLAB(fwy, sy, ay, 0, 1), fy23 = YRT_QSLAB(fwy, sy, ay, 2, 3);
  const f2 nz01 = YRT_QSLAB(nwz, sz, az, 0, 1), nz23 = YRT_QSLAB(nwz, sz, az, 2, 3);
  const f2 fz01 = YRT_QSLAB(fwz, sz, az, 0, 1), fz23 = YRT_QSLAB(fwz, sz, az, 2, 3);
#undef YRT_QSLAB
#undef YRT_QB
  const float MISS = __int_as_float(ANY ? 0xff800000 : 0x7f800000);
#define YRT_CHILD(k, NX, FX, NY, FY, NZ, FZ, CH)                                            \
  do {                                                                                      \
    float nn, ff, a_, b_;                                                                   \
    asm("v_max_f32 %0, %1, %2" : "=v"(a_) : "v"(NZ), "v"(r.tnear));                         \
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(nn) : "v"(NX), "v"(NY), "v"(a_));                \
    asm("v_min_f32 %0, %1, %2" : "=v"(b_) : "v"(FZ), "v"(tmax));                            \
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(ff) : "v"(FX), "v"(FY), "v"(b_));                \
    t[k] = ((int)(nn <= __builtin_fmaf(ff, YRT_BOX_ROBUST, r.margin)) & (int)((CH) != -1)) ? nn : MISS; \
    c[k] = (CH);                                                                            \
  } while (0)
  YRT_CHILD(0, nx01.x, fx01.x, ny01.x, fy01.x, nz01.x, fz01.x, ch.x);
  YRT_CHILD(1, nx01.y, fx01.y, ny01.y, fy01.y, nz01.y, fz01.y, ch.y);
  YRT_CHILD(2, nx23.x, fx23.x, ny23.x, fy23.x, nz23.x, fz23.x, ch.z);
  YRT_CHILD(3, nx23.y, fx23.y, ny23.y, fy23.y, nz23.y, fz23.y, ch.w);
#undef YRT_CHILD
}

// Sorts the four (t, child) pairs by t ascending (5-comparator network, stable for equal t).
// (A 3-comparator nearest-first order saves 10 VALU per node step but visits 1.4 % more nodes:
// -0.6 % on C3, profiles/r02/trace_variants_r02.txt.)
__device__ __forceinline__ void sort4(float t[4], int c[4]) {
#define YRT_CSWAP(a, b)                          \
  do {                                           \
    const bool sw = t[b] < t[a];                 \
    const float ta = sw ? t[b] : t[a];           \
    const float tb = sw ? t[a] : t[b];           \
    const int ca = sw ? c[b] : c[a];             \
    const int cb = sw ? c[a] : c[b];             \
    t[a] = ta; t[b] = tb; c[a] = ca; c[b] = cb;  \
  } while (0)
  YRT_CSWAP(0, 1);
  YRT_CSWAP(2, 3);
  YRT_CSWAP(0, 2);
  YRT_CSWAP(1, 3);
  YRT_CSWAP(1, 2);
#undef YRT_CSWAP
}

// Any-hit (shadow) rays: the farthest hit child first, the others in slot order — three
// descending comparators (0,1), (2,3), (0,2) move the largest entry distance to slot 0
// (misses are -INF). A shadow ray leaves a surface toward the light: what occludes it lies
// far along the ray, the children near its origin rarely do. On the C3 shadow-ray streams
// (tools/visit_order_exp.py): 7.96 node visits and 1.50 triangle tests per ray against 10.25
// and 1.94 in slot order, 12.5 / 2.46 nearest-first.
__device__ __forceinline__ void sort3_far(float t[4], int c[4]) {
#define YRT_CSWAP_D(a, b)                        \
  do {                                           \
    const bool sw = t[b] > t[a];                 \
    const float ta = sw ? t[b] : t[a];           \
    const float tb = sw ? t[a] : t[b];           \
    const int ca = sw ? c[b] : c[a];             \
    const int cb = sw ? c[a] : c[b];             \
    t[a] = ta; t[b] = tb; c[a] = ca; c[b] = cb;  \
  } while (0)
  YRT_CSWAP_D(0, 1);
  YRT_CSWAP_D(2, 3);
  YRT_CSWAP_D(0, 2);
#undef YRT_CSWAP_D
}

// The triangle test's cross and dot products as separate multiplies and adds (two roundings per
// term pair, -ffp-contract=off), the oracle's tri_cross / tri_dot (oracle/yrt_oracle.c). An
// explicit-FMA form issues 27 instead of 43 VALU per test but ran the closest-hit trace 2 %
// slower on C3 and the C4 cubemap 2 % slower (same-box bisect, profiles/r04/bisect_r04.txt).
__device__ __forceinline__ V3 tri_cross(const V3& a, const V3& b) {
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ float tri_dot(const V3& a, const V3& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

// One triangle without the distance range: true when the ray's line crosses the triangle
// (barycentric and back-face tests); t, U, V, absDen as tri_test_t.
__device__ __forceinline__ bool tri_test_g(const GpuTri& tr, const RayPre& r, float& t, float& U_, float& V_,
                                           float& absDen_) {
  V3 v0 = v3(tr.v0[0], tr.v0[1], tr.v0[2]);
  V3 e1 = v3(tr.e1[0], tr.e1[1], tr.e1[2]);
  V3 e2 = v3(tr.e2[0], tr.e2[1], tr.e2[2]);
  V3 Ng = tri_cross(e1, e2);
  V3 C = v0 - r.org;
  V3 R = tri_cross(r.dir, C);
  float den = tri_dot(Ng, r.dir);
  float absDen = fabsf(den);
  float sgn = den < 0.0f ? -1.0f : 1.0f;
  float U = tri_dot(R, e2) * sgn;
  float V = tri_dot(R, e1) * sgn;
  bool ok = (den != 0.0f) & (U >= 0.0f) & (V >= 0.0f) & (U + V <= absDen);
  int flags = __float_as_int(tr.e1[3]);
  ok &= !((flags & 1) && !(den > 0.0f));
  float T = tri_dot(Ng, C) * sgn;
  t = T / absDen;
  U_ = U;
  V_ = V;
  absDen_ = absDen;
  return ok;
}

// One triangle; returns true and t when the ray hits within (tnear, tfar). U, V, absDen are
// returned undivided: u = U/absDen, v = V/absDen are only needed for an accepted hit.
__device__ __forceinline__ bool tri_test_t(const GpuTri& tr, const RayPre& r, float tfar, float& t, float& U_,
                                           float& V_, float& absDen_) {
  V3 v0 = v3(tr.v0[0], tr.v0[1], tr.v0[2]);
  V3 e1 = v3(tr.e1[0], tr.e1[1], tr.e1[2]);
  V3 e2 = v3(tr.e2[0], tr.e2[1], tr.e2[2]);
  V3 Ng = tri_cross(e1, e2);
  V3 C = v0 - r.org;
  V3 R = tri_cross(r.dir, C);
  float den = tri_dot(Ng, r.dir);
  float absDen = fabsf(den);
  float sgn = den < 0.0f ? -1.0f : 1.0f;
  float U = tri_dot(R, e2) * sgn;
  float V = tri_dot(R, e1) * sgn;
  bool ok = (den != 0.0f) & (U >= 0.0f) & (V >= 0.0f) & (U + V <= absDen);
  int flags = __float_as_int(tr.e1[3]);
  ok &= !((flags & 1) && !(den > 0.0f));
  float T = tri_dot(Ng, C) * sgn;
  t = T / absDen;
  ok &= (t > r.tnear) & (t < tfar);
  U_ = U;
  V_ = V;
  absDen_ = absDen;
  return ok;
}

// Plain depth-first traversal (rtPick, DebugRenderer): nearest child first, the other hit
// children pushed farthest-first; same closest-hit rule as the wavefront kernel.
template <bool ANY>
__device__ __forceinline__ Hit traverse(const GpuNode* __restrict__ nodes, const GpuTri* __restrict__ tris,
                                        const RayPre& r, int* __restrict__ stack /* LDS, unused */) {
  (void)stack;
  Hit best;
  best.t = r.tfar;
  best.u = best.v = 0.0f;
  best.tri = -1;
  // NaN tfar (tMaxShadowRay = inf): every comparison is false, no hit.
  if (!(r.tfar >= r.tnear)) return best;
  int pst[YRT_STACK_DEPTH];
  int sp = 0;
  int cur = 0;  // (index << 5) | count
  while (true) {
    if ((cur & 31) == 0) {
      float t[4];
      int c[4];
      box4(nodes + (cur >> 5), r, best.t, t, c);
      sort4(t, c);
      const float INF = __int_as_float(0x7f800000);
      if (t[3] < INF) pst[sp++] = c[3];
      if (t[2] < INF) pst[sp++] = c[2];
      if (t[1] < INF) pst[sp++] = c[1];
      if (t[0] < INF) {
        cur = c[0];
        continue;
      }
    } else {
      const int idx = cur >> 5, cnt = cur & 31;
      for (int i = 0; i < cnt; ++i) {
        const GpuTri tr = tris[idx + i];
        float t, U, V, absDen;
        bool ok = tri_test_t(tr, r, ANY ? r.tfar : best.t + 0.0f, t, U, V, absDen);
        int gid = __float_as_int(tr.v0[3]);
        if (ANY) {
          if (ok) {
            best.t = t; best.u = U / absDen; best.v = V / absDen; best.tri = gid;
            return best;
          }
        } else {
          // strict (t < best) or tie with smaller id; tri_test used tfar = best.t so ties
          // (t == best.t) were rejected: re-test them against the original tfar.
          if (!ok && best.tri >= 0 && t == best.t && gid < best.tri) {
            float t2, U2, V2, a2;
            ok = tri_test_t(tr, r, r.tfar, t2, U2, V2, a2);
          }
          if (ok) {
            best.t = t; best.u = U / absDen; best.v = V / absDen; best.tri = gid;
          }
        }
      }
    }
    if (sp == 0) break;
    cur = pst[--sp];
  }
  return best;
}

}  // namespace yrt
