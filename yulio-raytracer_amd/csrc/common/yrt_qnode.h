// yrt_qnode.h — half-size (64-byte) BVH4 nodes: the four child boxes quantized to 8 bits per
// plane against a per-node origin and a power-of-two quantum per axis, rounded outward by one
// extra quantum.
//
// Why: the any-hit (shadow) traversal is latency-bound (VALU busy 0.41 of a 0.83 ceiling,
// waves waiting on memory 54 % of their cycles, profiles/pmc_c3.json): its node loads are
// seven 16-byte loads from a 128-byte record, and C3's 2.1 MB of nodes do not fit one XCD's
// 4 MB L2 beside the triangles. A GpuQNode is one 64-byte line: four loads, half the bytes.
//
// Layout: origin xyz + the biased exponents of the three quanta (16 B), the child references
// exactly as GpuNode::child (16 B, same node indices: node i of the quantized array is node i
// of the float one), six words of plane bytes (lo x, hi x, lo y, hi y, lo z, hi z; byte k =
// child k), 8 B of padding. An empty slot has lo = 255, hi = 0 and child -1 (the kernel tests
// the reference).
//
// Dequantized plane = origin + q * 2^e, exactly (real arithmetic). The quantizer (double
// precision, identical on the host builder and in the GPU refit kernel) chooses per axis
//   2^e >= extent / 250 and >= 2 ulp of the node's coordinates,
//   origin = the largest float <= lo_min - 2 * 2^e,
//   q_lo = floor((lo - origin) / 2^e) - 1,  q_hi = ceil((hi - origin) / 2^e) + 1   (in [0, 254]),
// so every dequantized box contains its child's box widened by one quantum on each side.
//
// Why one quantum: the kernel computes a slab distance as fma(q, 2^e * inv, a) with
// a = fma(origin, inv, -org * inv) (2^e * inv is exact), one convert (v_cvt_f32_ubyte) and one
// FMA per plane. Against the float node's fma(plane, inv, -org * inv) the only new error is
// a's rounding, |a| u <= (|t| + 255 * 2^e |inv|) u: its |t| part is of the size the robust
// exit factor (1 + 2^-16) already covers, its quantum part is 2^-16 of the quantum the
// widening adds. So the test stays conservative — no box holding a triangle the triangle test
// accepts is culled — and the closest hit (smallest (t, id)) and occlusion are the same as
// with the float nodes, bit for bit.
#pragma once

#include <stdint.h>

#include "yrt_gpu_types.h"

#if defined(__HIPCC__)
#define YRT_QHD __host__ __device__ __forceinline__
#else
#define YRT_QHD static inline
#endif

namespace yrt {

struct GpuQNode {
  float origin[3];
  uint32_t exps;      // biased exponent of the x, y, z quantum in bits 0-7, 8-15, 16-23
  int32_t child[4];   // GpuNode::child
  uint32_t q[6];      // lo x, hi x, lo y, hi y, lo z, hi z: byte k = child k's plane
  uint32_t pad[2];
};
static_assert(sizeof(GpuQNode) == 64, "quantized node is 64 B");

YRT_QHD uint64_t yrt_q_dbits(double d) {
  uint64_t u;
  __builtin_memcpy(&u, &d, 8);
  return u;
}
YRT_QHD double yrt_q_dval(uint64_t u) {
  double d;
  __builtin_memcpy(&d, &u, 8);
  return d;
}
YRT_QHD uint32_t yrt_q_fbits(float f) {
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  return u;
}
YRT_QHD float yrt_q_fval(uint32_t u) {
  float f;
  __builtin_memcpy(&f, &u, 4);
  return f;
}
// 2^e for e in [-126, 127], exactly
YRT_QHD double yrt_q_pow2(int e) { return yrt_q_dval((uint64_t)(e + 1023) << 52); }
// floor(log2(x)) of a positive finite double
YRT_QHD int yrt_q_ilogb(double x) { return (int)((yrt_q_dbits(x) >> 52) & 0x7ff) - 1023; }
// the largest float <= d (d finite, within the float range)
YRT_QHD float yrt_q_float_down(double d) {
  float f = (float)d;
  if ((double)f > d) {
    const uint32_t u = yrt_q_fbits(f);
    f = f > 0.0f ? yrt_q_fval(u - 1u) : f == 0.0f ? -1.40129846e-45f : yrt_q_fval(u + 1u);
  }
  return f;
}

// One axis: the child planes lo[k], hi[k] of the valid children (mask bit k) -> origin, biased
// exponent, plane bytes (lo word, hi word)
YRT_QHD void yrt_quantize_axis(const float lo[4], const float hi[4], unsigned valid, float& origin, uint32_t& ebias,
                               uint32_t& qlo, uint32_t& qhi) {
  double L = 0.0, H = 0.0;
  bool any = false;
  for (int k = 0; k < 4; ++k)
    if (valid & (1u << k)) {
      L = any ? (lo[k] < L ? lo[k] : L) : lo[k];
      H = any ? (hi[k] > H ? hi[k] : H) : hi[k];
      any = true;
    }
  qlo = 0xffffffffu;  // empty slots: lo 255, hi 0
  qhi = 0u;
  if (!any) {
    origin = 0.0f;
    ebias = 127;
    return;
  }
  const double E = H - L;
  // 2^e >= E / 250
  int e = -126;
  if (E > 0.0) {
    const double r = E / 250.0;
    e = yrt_q_ilogb(r);
    if (yrt_q_pow2(e) < r) ++e;
  }
  // 2^e >= 2 ulp(float) of the node's largest coordinate: origin stays within a quantum below lo
  const double m = (L < 0 ? -L : L) > (H < 0 ? -H : H) ? (L < 0 ? -L : L) : (H < 0 ? -H : H);
  if (m > 0.0) {
    const int eu = yrt_q_ilogb(m) - 22;
    if (e < eu) e = eu;
  }
  if (e < -126) e = -126;
  if (e > 127) e = 127;
  const double s = yrt_q_pow2(e);
  origin = yrt_q_float_down(L - 2.0 * s);
  ebias = (uint32_t)(e + 127);
  const double o = origin;
  for (int k = 0; k < 4; ++k) {
    if (!(valid & (1u << k))) continue;
    int a = (int)__builtin_floor(((double)lo[k] - o) / s) - 1;
    int b = (int)__builtin_ceil(((double)hi[k] - o) / s) + 1;
    a = a < 0 ? 0 : a;      // never: lo - origin >= 2 quanta
    b = b > 255 ? 255 : b;  // never: (hi - origin) / 2^e <= 250 + 3
    qlo = (qlo & ~(0xffu << (8 * k))) | ((uint32_t)a << (8 * k));
    qhi = (qhi & ~(0xffu << (8 * k))) | ((uint32_t)b << (8 * k));
  }
}

YRT_QHD void yrt_quantize_node(const GpuNode& n, GpuQNode& o) {
  unsigned valid = 0;
  for (int k = 0; k < 4; ++k) {
    o.child[k] = n.child[k];
    if (n.child[k] != -1) valid |= 1u << k;
  }
  uint32_t ex, ey, ez;
  yrt_quantize_axis(n.lox, n.hix, valid, o.origin[0], ex, o.q[0], o.q[1]);
  yrt_quantize_axis(n.loy, n.hiy, valid, o.origin[1], ey, o.q[2], o.q[3]);
  yrt_quantize_axis(n.loz, n.hiz, valid, o.origin[2], ez, o.q[4], o.q[5]);
  o.exps = ex | (ey << 8) | (ez << 16);
  o.pad[0] = o.pad[1] = 0;
}

}  // namespace yrt
