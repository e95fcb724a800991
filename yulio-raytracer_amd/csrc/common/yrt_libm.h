/* yrt_libm.h — the single-precision elementary functions of the per-ray path (shading, BRDF
 * and light sampling, stereo camera rays, resolve), written out once so the GPU kernels and the
 * CPU oracle evaluate them with the same operations.
 *
 * Why: the reference calls the C runtime's sinf/cosf/powf/acosf/... (MSVC CRT, unpinned); the
 * GPU's device library (OCML) and glibc differ from each other in the last bits, and in a
 * closed interior (config C5: ~10 rays per sample, depth 10) one ulp in a bounce direction
 * changes which triangle the next ray hits often enough to move whole pixels. Using these
 * functions on both sides (a documented substitution, like rcp/rsqrt -> IEEE)
 * makes the device's arithmetic reproducible by the oracle bit for bit. Both sides are built
 * with -ffp-contract=off (no implicit fused multiply-add), IEEE round-to-nearest, correctly
 * rounded division and square root; the polynomials and reductions here use explicit fused
 * multiply-adds (YRT_LM_FMA: v_fma_f32 on the GPU, the FMA3 instruction or C99 fmaf in the
 * oracle — one correctly rounded operation on both sides), so the same source gives the same
 * bits with half the operations of separate multiplies and adds.
 *
 * Algorithms: Cody-Waite range reduction + minimax polynomials of the Cephes single-precision
 * library (sinf/cosf, expf, logf, asinf, atanf; S. L. Moshier, public domain), accurate to
 * ~1-2 ulp over the arguments the renderer uses; powf = expf(y * logf(x)) for x > 0 (the
 * renderer's exponents are BRDF exponents and medium depths, |y log x| small).
 *
 * C and HIP compatible (the oracle is C11).
 */
#ifndef YRT_LIBM_H
#define YRT_LIBM_H

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define YRT_LIBM_FN __host__ __device__ static inline
#else
#define YRT_LIBM_FN static inline
#endif

YRT_LIBM_FN uint32_t yrt_lm_bits(float f) {
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  return u;
}
YRT_LIBM_FN float yrt_lm_float(uint32_t u) {
  float f;
  __builtin_memcpy(&f, &u, 4);
  return f;
}
YRT_LIBM_FN float yrt_lm_floor(float x) { return __builtin_floorf(x); }
#define YRT_LM_FMA(a, b, c) __builtin_fmaf((a), (b), (c))
YRT_LIBM_FN float yrt_lm_sqrt(float x) { return __builtin_sqrtf(x); }

/* 2^n for integer n in [-252, 254] as a product of two exact powers of two */
YRT_LIBM_FN float yrt_lm_ldexp(float x, int n) {
  int a = n / 2, b = n - n / 2;
  if (a < -126) a = -126;
  if (b < -126) b = -126;
  if (a > 127) a = 127;
  if (b > 127) b = 127;
  return x * yrt_lm_float((uint32_t)(a + 127) << 23) * yrt_lm_float((uint32_t)(b + 127) << 23);
}

/* ---- sin / cos: x = q * pi/2 + r, |r| <= pi/4 (three-part Cody-Waite pi/2) */
YRT_LIBM_FN float yrt_lm_sin_poly(float r) {
  const float z = r * r;
  const float p = YRT_LM_FMA(YRT_LM_FMA(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
  return YRT_LM_FMA(p * z, r, r);
}
YRT_LIBM_FN float yrt_lm_cos_poly(float r) {
  const float z = r * r;
  const float p = YRT_LM_FMA(YRT_LM_FMA(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f);
  return YRT_LM_FMA(p, z * z, YRT_LM_FMA(-0.5f, z, 1.0f));
}
YRT_LIBM_FN float yrt_lm_reduce(float x, int* quadrant) {
  const float q = yrt_lm_floor(YRT_LM_FMA(x, 0.636619772367581343f, 0.5f));
  *quadrant = (int)q & 3;
  return YRT_LM_FMA(-q, 7.54978995489188216e-8f, YRT_LM_FMA(-q, 4.837512969970703125e-4f, YRT_LM_FMA(-q, 1.5703125f, x)));
}
YRT_LIBM_FN float yrt_sinf(float x) {
  int k;
  const float r = yrt_lm_reduce(x, &k);
  const float v = (k & 1) ? yrt_lm_cos_poly(r) : yrt_lm_sin_poly(r);
  return (k & 2) ? -v : v;
}
YRT_LIBM_FN float yrt_cosf(float x) {
  int k;
  const float r = yrt_lm_reduce(x, &k);
  const float v = (k & 1) ? yrt_lm_sin_poly(r) : yrt_lm_cos_poly(r);
  return ((k + 1) & 2) ? -v : v;
}

/* ---- exp: x = n ln2 + r, |r| <= ln2/2 */
YRT_LIBM_FN float yrt_expf(float x) {
  if (x != x) return x;
  if (x > 88.72283905206835f) return yrt_lm_float(0x7f800000u);
  if (x < -103.97208f) return 0.0f;
  const float n = yrt_lm_floor(YRT_LM_FMA(1.44269504088896341f, x, 0.5f));
  const float r = YRT_LM_FMA(n, 2.12194440e-4f, YRT_LM_FMA(-n, 0.693359375f, x));
  const float z = r * r;
  float q = YRT_LM_FMA(1.9875691500e-4f, r, 1.3981999507e-3f);
  q = YRT_LM_FMA(q, r, 8.3334519073e-3f);
  q = YRT_LM_FMA(q, r, 4.1665795894e-2f);
  q = YRT_LM_FMA(q, r, 1.6666665459e-1f);
  q = YRT_LM_FMA(q, r, 5.0000001201e-1f);
  const float p = YRT_LM_FMA(q, z, r) + 1.0f;
  return yrt_lm_ldexp(p, (int)n);
}

/* ---- log: x = m 2^e, m in [sqrt(1/2), sqrt(2)) */
YRT_LIBM_FN float yrt_logf(float x) {
  if (x != x || x < 0.0f) return yrt_lm_float(0x7fc00000u);
  if (x == 0.0f) return -yrt_lm_float(0x7f800000u);
  if (x == yrt_lm_float(0x7f800000u)) return x;
  int e = 0;
  if (x < 1.17549435e-38f) {  /* subnormal: scale into the normal range */
    x *= 16777216.0f;
    e = -24;
  }
  const uint32_t u = yrt_lm_bits(x);
  e += (int)((u >> 23) & 0xff) - 126;
  float m = yrt_lm_float((u & 0x007fffffu) | 0x3f000000u); /* [0.5, 1) */
  if (m < 0.707106781186547524f) {
    e -= 1;
    m = m + m - 1.0f;
  } else {
    m = m - 1.0f;
  }
  const float z = m * m;
  float q = YRT_LM_FMA(7.0376836292e-2f, m, -1.1514610310e-1f);
  q = YRT_LM_FMA(q, m, 1.1676998740e-1f);
  q = YRT_LM_FMA(q, m, -1.2420140846e-1f);
  q = YRT_LM_FMA(q, m, 1.4249322787e-1f);
  q = YRT_LM_FMA(q, m, -1.6668057665e-1f);
  q = YRT_LM_FMA(q, m, 2.0000714765e-1f);
  q = YRT_LM_FMA(q, m, -2.4999993993e-1f);
  q = YRT_LM_FMA(q, m, 3.3333331174e-1f);
  const float fe = (float)e;
  float y = YRT_LM_FMA(-2.12194440e-4f, fe, q * m * z);
  y = YRT_LM_FMA(-0.5f, z, y);
  return YRT_LM_FMA(0.693359375f, fe, m + y);
}

/* ---- pow for the renderer's domain (x >= 0): BRDF exponents, medium depths, gamma */
YRT_LIBM_FN float yrt_powf(float x, float y) {
  if (y == 0.0f || x == 1.0f) return 1.0f;
  if (x != x || y != y) return x + y;
  if (x == 0.0f) return y > 0.0f ? 0.0f : yrt_lm_float(0x7f800000u);
  if (x < 0.0f) return yrt_lm_float(0x7fc00000u);
  return yrt_expf(y * yrt_logf(x));
}

/* ---- asin / acos */
YRT_LIBM_FN float yrt_lm_asin_poly(float z) {
  float q = YRT_LM_FMA(4.2163199048e-2f, z, 2.4181311049e-2f);
  q = YRT_LM_FMA(q, z, 4.5470025998e-2f);
  q = YRT_LM_FMA(q, z, 7.4953002686e-2f);
  return YRT_LM_FMA(q, z, 1.6666752422e-1f);
}
YRT_LIBM_FN float yrt_lm_asin_core(float a /* |x| */) {
  float z, v;
  int big = a > 0.5f;
  if (big) {
    z = 0.5f * (1.0f - a);
    v = yrt_lm_sqrt(z);
  } else {
    z = a * a;
    v = a;
  }
  float r = YRT_LM_FMA(yrt_lm_asin_poly(z) * z, v, v);
  if (big) r = 1.5707963267948966192f - (r + r);
  return r;
}
YRT_LIBM_FN float yrt_asinf(float x) {
  if (!(x >= -1.0f && x <= 1.0f)) return yrt_lm_float(0x7fc00000u);
  const float r = yrt_lm_asin_core(x < 0.0f ? -x : x);
  return x < 0.0f ? -r : r;
}
/* acos: x < -1/2: pi - 2 asin(sqrt((1+x)/2)); x > 1/2: 2 asin(sqrt((1-x)/2)); else
   pi/2 - asin(x). Every range's asin argument is <= 1/2 (the core's polynomial branch), so the
   three ranges select one argument and share one sqrt and one polynomial: a wave whose lanes
   span the ranges evaluates the core once instead of once per range. */
YRT_LIBM_FN float yrt_acosf(float x) {
  if (!(x >= -1.0f && x <= 1.0f)) return yrt_lm_float(0x7fc00000u);
  const int lo = x < -0.5f, hi = x > 0.5f;
  const float w = yrt_lm_sqrt(0.5f * (hi ? 1.0f - x : 1.0f + x));
  const float a = (lo || hi) ? w : (x < 0.0f ? -x : x);
  const float z = a * a;
  const float r = YRT_LM_FMA(yrt_lm_asin_poly(z) * z, a, a);
  if (lo) return 3.14159265358979323846f - 2.0f * r;
  if (hi) return 2.0f * r;
  return 1.5707963267948966192f - (x < 0.0f ? -r : r);
}

/* ---- atan / atan2 */
YRT_LIBM_FN float yrt_atanf(float x) {
  if (x != x) return x;
  const float a = x < 0.0f ? -x : x;
  float y, t;
  if (a > 2.414213562373095f) {
    y = 1.5707963267948966192f;
    t = -1.0f / a;
  } else if (a > 0.4142135623730950f) {
    y = 0.7853981633974483096f;
    t = (a - 1.0f) / (a + 1.0f);
  } else {
    y = 0.0f;
    t = a;
  }
  const float z = t * t;
  float q = YRT_LM_FMA(8.05374449538e-2f, z, -1.38776856032e-1f);
  q = YRT_LM_FMA(q, z, 1.99777106478e-1f);
  q = YRT_LM_FMA(q, z, -3.33329491539e-1f);
  y += YRT_LM_FMA(q * z, t, t);
  return x < 0.0f ? -y : y;
}
YRT_LIBM_FN float yrt_atan2f(float y, float x) {
  const float PI = 3.14159265358979323846f, PIO2 = 1.5707963267948966192f;
  if (x != x || y != y) return x + y;
  if (x == 0.0f) {
    if (y > 0.0f) return PIO2;
    if (y < 0.0f) return -PIO2;
    return (yrt_lm_bits(x) >> 31) ? ((yrt_lm_bits(y) >> 31) ? -PI : PI) : y;
  }
  const float r = yrt_atanf(y / x);
  if (x > 0.0f) return r;
  return (yrt_lm_bits(y) >> 31) ? r - PI : r + PI;
}

#endif /* YRT_LIBM_H */
