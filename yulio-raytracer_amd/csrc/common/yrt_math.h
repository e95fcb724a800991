// yrt_math.h — scalar vector/affine math shared by the device plugin's host code and
// its HIP kernels. Operation order follows the reference math library so that the
// GPU path and the host setup code round identically:
//   normalize(a) = a * rsqrt(dot(a,a))          common/math/vec3.h:159
//   frame(N)                                    common/math/linearspace3.h:118-124
//   LinearSpace3 * v = v.x*vx + v.y*vy + v.z*vz  common/math/linearspace3.h:134
//   AffineSpace3 products / lookAtPoint / rotate common/math/affinespace.h:60-78,
//                                                common/math/linearspace3.h:95-101
// rcp/rsqrt are the reference's own: the Intel SSE estimate (rcpps/rsqrtps, emulated exactly
// with integer arithmetic, yrt_sse_rcp.h) plus the Newton step of common/math/math.h:38-59, on
// host and gfx950 alike. -DYRT_IEEE_RCP restores round 1-5's substitution (correctly rounded
// 1/x and 1/sqrt(x)) for A/B measurements.
#pragma once

#include <math.h>
#include <stdint.h>

#include "yrt_libm.h"
#include "yrt_sse_rcp.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define YRT_HD __host__ __device__ __forceinline__
#else
#define YRT_HD static inline
#endif

namespace yrt {

struct V3 {
  float x, y, z;
};

YRT_HD V3 v3(float x, float y, float z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
YRT_HD V3 v3s(float s) { return v3(s, s, s); }
YRT_HD V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
YRT_HD V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
YRT_HD V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }
YRT_HD V3 operator*(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
YRT_HD V3 operator*(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
YRT_HD V3 operator*(float s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }
YRT_HD V3 operator/(V3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
YRT_HD bool operator==(V3 a, V3 b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
YRT_HD bool operator!=(V3 a, V3 b) { return !(a == b); }
// dot, cross and LinearSpace3 * v in the reference build's operation sequences (x64 MSVC, SSE4.1
// forced by common/sys/platform.h:100-103, no AVX2, so no fused multiply-add anywhere):
//   dot   = _mm_dp_ps(a, b, 0x7F) (common/math/vector3f_sse.h:206-209): the three products,
//           then (x + y) + z. dp_ps adds the masked fourth lane's +0 to z's product, which
//           changes nothing but the sign of an exactly zero sum (dp_ps never returns -0; this
//           returns -0 when both partial sums are -0); it is left out (one VALU per dot);
//   cross = a0*b0 - a1*b1 on shuffled operands (vector3f_sse.h:226-233, the non-AVX2 branch);
//   L * v = v.x*vx + v.y*vy + v.z*vz, left to right (common/math/linearspace3.h:134).
// Host setup, kernels and the oracle (oracle/yrt_oracle.c) use these same sequences. Round 4's
// fused forms (3 / 6 / 9 instead of 5 / 9 / 15 operations, C3 +1.6 %) moved hits between
// coplanar triangles: against this order they changed 35 % of the channels of a C5 face (the
// Frederick stand-in's overlapping decals and walls flip with the last bit of a ray origin),
// 1.8 % on C3 (profiles/r05/arith_sensitivity_r05.txt).
YRT_HD float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
YRT_HD V3 cross(V3 a, V3 b) {
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
#if defined(__HIPCC__)
// Correctly rounded 1/x without the general division sequence (v_div_scale x2, v_rcp, 5 FMAs,
// v_div_fmas, v_div_fixup): the hardware reciprocal estimate refined by one FMA Newton step
// (e = 1 - x*y, y += y*e) is RN(1/x) for every |x| in [2^-124, 2^124) — verified on gfx950
// for all 2^32 inputs against 1.0f/x (yrtDebugCheckMath, tests/test_gpu_parity.py); zero,
// subnormal, huge, infinite and NaN inputs take the IEEE division. Same bits as the host's
// 1/x, so the oracle stays bit-exact.
__host__ __device__ __forceinline__ float rcp_rn(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  float y = __builtin_amdgcn_rcpf(x);
  const float e = __builtin_fmaf(-x, y, 1.0f);
  y = __builtin_fmaf(e, y, y);
  const unsigned ex = (__float_as_uint(x) >> 23) & 0xffu;
  if (__builtin_expect(ex - 3u > 247u, 0)) y = 1.0f / x;
  return y;
#else
  return 1.0f / x;
#endif
}
#endif
#if defined(YRT_IEEE_RCP)
#if defined(__HIPCC__)
YRT_HD float rcpf_(float x) { return rcp_rn(x); }
YRT_HD float rsqrtf_(float x) { return rcp_rn(sqrtf(x)); }
#else
YRT_HD float rcpf_(float x) { return 1.0f / x; }
YRT_HD float rsqrtf_(float x) { return 1.0f / sqrtf(x); }
#endif
#else
YRT_HD float rcpf_(float x) { return yrt_ref_rcp(x); }    // common/math/math.h:38-42
YRT_HD float rsqrtf_(float x) { return yrt_ref_rsqrt(x); }  // common/math/math.h:53-58
#endif
// rcp of a Color / Vector3f: the same sequence per lane (color_sse.h:142-145, vector3f_sse.h:135-138)
YRT_HD V3 rcpv(V3 a) { return v3(rcpf_(a.x), rcpf_(a.y), rcpf_(a.z)); }
YRT_HD V3 normalize(V3 a) { return a * rsqrtf_(dot(a, a)); }
YRT_HD float length(V3 a) { return sqrtf(dot(a, a)); }
YRT_HD float reduce_max(V3 a) { return fmaxf(fmaxf(a.x, a.y), a.z); }
YRT_HD V3 absv(V3 a) { return v3(fabsf(a.x), fabsf(a.y), fabsf(a.z)); }
YRT_HD float clampf(float x, float lo = 0.0f, float hi = 1.0f) {
  // reference clamp = max(lower, min(x, upper)) (common/math/math.h:122)
  return fmaxf(lo, fminf(x, hi));
}
YRT_HD float signf_(float x) { return x < 0 ? -1.0f : 1.0f; }
YRT_HD float sqrf(float x) { return x * x; }
YRT_HD float cos2sin(float x) { return sqrtf(fmaxf(0.0f, 1.0f - x * x)); }
YRT_HD float smoothstepf(float e0, float e1, float x) {
  x = clampf((x - e0) / (e1 - e0), 0.0f, 1.0f);
  return x * x * (3 - 2 * x);
}
YRT_HD float deg2rad(float x) { return x * 1.74532925199432957692e-2f; }
YRT_HD float rad2deg(float x) { return x * 5.72957795130823208768e1f; }

constexpr float kPi = 3.14159265358979323846f;
constexpr float kTwoPi = 6.28318530717958647692f;
constexpr float kOneOverPi = 0.31830988618379069122f;
constexpr float kOneOverTwoPi = 0.15915494309189534561f;
constexpr float kUlp = 1.19209290e-07f;  // FLT_EPSILON (common/sys/constants.h:112-116)

// Column-major 3x3 (vx, vy, vz are the columns), as common/math/linearspace3.h.
struct L3 {
  V3 vx, vy, vz;
};
YRT_HD L3 l3(V3 vx, V3 vy, V3 vz) { L3 r; r.vx = vx; r.vy = vy; r.vz = vz; return r; }
YRT_HD L3 l3_rows(float m00, float m01, float m02, float m10, float m11, float m12,
                  float m20, float m21, float m22) {
  return l3(v3(m00, m10, m20), v3(m01, m11, m21), v3(m02, m12, m22));
}
YRT_HD L3 l3_identity() { return l3(v3(1, 0, 0), v3(0, 1, 0), v3(0, 0, 1)); }
YRT_HD V3 mul(L3 a, V3 b) { return b.x * a.vx + b.y * a.vy + b.z * a.vz; }
YRT_HD L3 mul(L3 a, L3 b) { return l3(mul(a, b.vx), mul(a, b.vy), mul(a, b.vz)); }
YRT_HD L3 l3_rotate(V3 u_, float r) {
  V3 u = normalize(u_);
  float s = yrt_sinf(r), c = yrt_cosf(r);  // shared with the per-ray stereo camera (yrt_libm.h)
  return l3_rows(u.x * u.x + (1 - u.x * u.x) * c, u.x * u.y * (1 - c) - u.z * s, u.x * u.z * (1 - c) + u.y * s,
                 u.x * u.y * (1 - c) + u.z * s, u.y * u.y + (1 - u.y * u.y) * c, u.y * u.z * (1 - c) - u.x * s,
                 u.x * u.z * (1 - c) - u.y * s, u.y * u.z * (1 - c) + u.x * s, u.z * u.z + (1 - u.z * u.z) * c);
}
YRT_HD float det(L3 a) { return dot(a.vx, cross(a.vy, a.vz)); }
YRT_HD L3 transposed(L3 a) {
  return l3(v3(a.vx.x, a.vy.x, a.vz.x), v3(a.vx.y, a.vy.y, a.vz.y), v3(a.vx.z, a.vy.z, a.vz.z));
}
YRT_HD L3 adjoint(L3 a) { return transposed(l3(cross(a.vy, a.vz), cross(a.vz, a.vx), cross(a.vx, a.vy))); }
YRT_HD L3 inverse(L3 a) {
  // rcp(det()) * adjoint()   (common/math/linearspace3.h:66)
  L3 adj = adjoint(a);
  float r = rcpf_(det(a));
  return l3(r * adj.vx, r * adj.vy, r * adj.vz);
}

// frame(N): common/math/linearspace3.h:118-124
YRT_HD L3 frame(V3 N) {
  V3 dx0 = cross(v3(1.0f, 0.0f, 0.0f), N);
  V3 dx1 = cross(v3(0.0f, 1.0f, 0.0f), N);
  V3 dx = normalize(dot(dx0, dx0) > dot(dx1, dx1) ? dx0 : dx1);
  V3 dy = normalize(cross(N, dx));
  return l3(dx, dy, N);
}

struct A3 {
  L3 l;
  V3 p;
};
YRT_HD A3 a3(L3 l, V3 p) { A3 r; r.l = l; r.p = p; return r; }
YRT_HD A3 a3_identity() { return a3(l3_identity(), v3s(0.0f)); }
YRT_HD A3 mul(A3 a, A3 b) { return a3(mul(a.l, b.l), mul(a.l, b.p) + a.p); }
YRT_HD V3 xfmPoint(A3 m, V3 p) { return mul(m.l, p) + m.p; }
YRT_HD V3 xfmVector(A3 m, V3 v) { return mul(m.l, v); }
YRT_HD V3 xfmNormal(A3 m, V3 n) { return mul(transposed(inverse(m.l)), n); }
YRT_HD A3 a3_translate(V3 p) { return a3(l3_identity(), p); }
YRT_HD A3 a3_scale(V3 s) { return a3(l3(v3(s.x, 0, 0), v3(0, s.y, 0), v3(0, 0, s.z)), v3s(0.0f)); }
YRT_HD A3 a3_rotate(V3 u, float r) { return a3(l3_rotate(u, r), v3s(0.0f)); }
YRT_HD A3 a3_rotate_about(V3 p, V3 u, float r) {
  return mul(mul(a3_translate(p), a3_rotate(u, r)), a3_translate(-p));
}
YRT_HD A3 a3_inverse(A3 a) {
  L3 il = inverse(a.l);
  return a3(il, -mul(il, a.p));
}
YRT_HD bool a3_is_identity(A3 a) {
  A3 i = a3_identity();
  return a.l.vx == i.l.vx && a.l.vy == i.l.vy && a.l.vz == i.l.vz && a.p == i.p;
}
// lookAtPoint: common/math/affinespace.h:72-77
YRT_HD A3 lookAtPoint(V3 eye, V3 point, V3 up) {
  V3 Z = normalize(point - eye);
  V3 U = normalize(cross(up, Z));
  V3 V = normalize(cross(Z, U));
  return a3(l3(U, V, Z), eye);
}

}  // namespace yrt
