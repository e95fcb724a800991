/* yrt_sse_rcp.h — the reference's approximate reciprocals, bit for bit.
 *
 * The reference computes every rcp()/rsqrt() of its render path with the SSE estimate
 * instructions plus one Newton step (common/math/math.h:38-59; vector3f_sse.h:135-144 and
 * color_sse.h:142-149 per lane; color_sse.h:161-162 turns Color / float into a * rcp(b)):
 *
 *   rcp(x)   = (r + r) - (r * r) * x                     r = rcpps(x)
 *   rsqrt(x) = 1.5f * r + ((x * -0.5f) * r) * (r * r)    r = rsqrtps(x)
 *
 * (the reference build is x64 MSVC with SSE4.1 and no FMA, so each operation rounds).
 *
 * rcpps / rsqrtps are table lookups whose contents Intel does not document and AMD implements
 * differently. On Intel they are (measured on every input of this container's Xeon,
 * tests/golden/make_sse_tables.py -> tests/golden/sse_rcp_tables.json):
 *   rcpps(x)   = sign * 2^-(E+1) * (1 + m/4096),  m = RN(4096 * (2/mid - 1)),
 *                mid = 1 + (i + 1/2)/2048, i = the top 11 bits of x's mantissa;
 *   rsqrtps(x) = 2^-(k+1) * (1 + m/4096),          m = RN(4096 * (2/sqrt(mid) - 1)),
 *                E = 2k + p, mid = (1 + (j + 1/2)/1024) * 2^p, j = the top 10 mantissa bits
 * — the 12-bit round-to-nearest reciprocal (square root) of the midpoint of the input's
 * 11-bit (10-bit + exponent parity) interval, with no ties (|m - exact| <= 0.49994). Zero
 * and subnormal inputs give +-inf, results below 2^-126 flush to zero, rsqrtps of a negative
 * number is the default NaN.
 *
 * Both are computed here exactly, so the GPU (v_rcp_f32 based) and the host (IEEE division)
 * produce the same bits and neither depends on the CPU vendor:
 *   rcp:   q = RN(2^25 / D), D = 4097 + 2i odd; the estimate q0 is within one of q and
 *          2*(2^25 - q0*D) in (-D, D] decides (no ties: D is odd);
 *   rsqrt: q = RN(8192 / sqrt(A / 2048)), A = (2049 + 2j) << p; the estimate q0 is within one
 *          of q, and q is right iff (2q - 1)^2 A < 2^39 < (2q + 1)^2 A (never equal: A's odd
 *          part is > 1), i.e. iff the high 32 bits of the 64-bit products are < 128 and >= 128:
 *          one 32-bit multiply-high per side.
 * Exhaustive checks: against the host's rcpps/rsqrtps over all 2^32 inputs
 * (tests/test_ref_pin.py, Intel hosts), the GPU against the committed tables over all 2^32
 * inputs (yrtDebugCheckMathTable, tests/test_gpu_parity.py).
 *
 * C and HIP compatible (the oracle is C11).
 */
#ifndef YRT_SSE_RCP_H
#define YRT_SSE_RCP_H

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define YRT_SSE_FN __host__ __device__ static inline
#else
#define YRT_SSE_FN static inline
#endif

YRT_SSE_FN uint32_t yrt_sse_bits(float f) {
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  return u;
}
YRT_SSE_FN float yrt_sse_float(uint32_t u) {
  float f;
  __builtin_memcpy(&f, &u, 4);
  return f;
}

/* an estimate of 1/x for x in [4097, 8191]: any value within a few ulp will do */
YRT_SSE_FN float yrt_sse_rcp_est(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_rcpf(x);
#else
  return 1.0f / x;
#endif
}
/* an estimate of 1/sqrt(x) for x in [1, 4) */
YRT_SSE_FN float yrt_sse_rsq_est(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_rsqf(x);
#else
  return 1.0f / __builtin_sqrtf(x);
#endif
}
/* the high 32 bits of a 32 x 32-bit product (one v_mul_hi_u32 on gfx950) */
YRT_SSE_FN uint32_t yrt_sse_mulhi(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }

/* Intel rcpps (one lane) */
YRT_SSE_FN float yrt_rcpps(float x) {
  const uint32_t u = yrt_sse_bits(x), s = u & 0x80000000u, e = (u >> 23) & 0xffu;
  const int D = 4097 + 2 * (int)((u >> 12) & 0x7ffu);
  int q = (int)(33554432.0f * yrt_sse_rcp_est((float)D) + 0.5f);
  const int r2 = 2 * (33554432 - q * D); /* exact: q*D < 2^27 */
  q += (r2 > D) - (r2 < -D);
  uint32_t out = s | ((253u - e) << 23) | ((uint32_t)(q - 4096) << 11);
  if (e >= 253u) out = s;                                             /* below 2^-126: +-0 */
  if (e == 255u) out = (u & 0x7fffffu) ? (u | 0x400000u) : s;         /* NaN stays (quiet), inf -> 0 */
  if (e == 0u) out = s | 0x7f800000u;                                 /* +-0, subnormal -> +-inf */
  return yrt_sse_float(out);
}

/* the rsqrtps mantissa m = q - 4096 of table entry (p << 10) | j */
YRT_SSE_FN uint32_t yrt_rsqrtps_m(uint32_t p, uint32_t j) {
  const uint32_t A = (2049u + 2u * j) << p;
  int q = (int)(8192.0f * yrt_sse_rsq_est((float)A * (1.0f / 2048.0f)) + 0.5f);
  const uint32_t lo = (uint32_t)(2 * q - 1), hi = (uint32_t)(2 * q + 1); /* < 2^15: squares fit */
  q += (yrt_sse_mulhi(hi * hi, A) < 128u) - (yrt_sse_mulhi(lo * lo, A) >= 128u);
  return (uint32_t)(q - 4096);
}

#if defined(__HIPCC__) && defined(__cplusplus)
/* On the GPU the 2048 mantissas are a 4 KB table in the code object, built at compile time
 * with the same integer test (a binary search for the q with (2q-1)^2 A < 2^39 < (2q+1)^2 A):
 * the arithmetic form's temporaries cost the camera-ray code 20 VGPRs (k_raygen 59 -> 79) and
 * the fused depth-0 trace kernel 60 B of scratch. Equal to yrt_rsqrtps_m for every entry
 * (the exhaustive GPU check against the Intel tables covers all of them). */
struct YrtRsqTab {
  unsigned short m[2048];
};
constexpr YrtRsqTab yrt_make_rsq_tab() {
  YrtRsqTab t{};
  for (unsigned i = 0; i < 2048; ++i) {
    const unsigned long long A = (2049ull + 2ull * (i & 1023u)) << (i >> 10);
    unsigned lo = 4096, hi = 8192; /* largest q with (2q - 1)^2 A < 2^39 */
    while (lo < hi) {
      const unsigned mid = (lo + hi + 1) / 2;
      if ((2ull * mid - 1) * (2ull * mid - 1) * A < (1ull << 39)) lo = mid; else hi = mid - 1;
    }
    t.m[i] = (unsigned short)(lo - 4096);
  }
  return t;
}
__device__ static constexpr YrtRsqTab yrt_rsq_tab = yrt_make_rsq_tab();
#endif

/* Intel rsqrtps (one lane) */
YRT_SSE_FN float yrt_rsqrtps(float x) {
  const uint32_t u = yrt_sse_bits(x), e = (u >> 23) & 0xffu;
  const int E = (int)e - 127, p = E & 1, k = (E - p) / 2;
#if defined(__HIP_DEVICE_COMPILE__) && !defined(YRT_RSQ_ARITH)
  const uint32_t m = yrt_rsq_tab.m[((uint32_t)p << 10) | ((u >> 13) & 0x3ffu)];
#else
  const uint32_t m = yrt_rsqrtps_m((uint32_t)p, (u >> 13) & 0x3ffu);
#endif
  uint32_t out = ((uint32_t)(126 - k) << 23) | (m << 11);
  if (u & 0x80000000u) out = 0xffc00000u;                             /* negative: default NaN */
  if (e == 255u) out = (u & 0x7fffffu) ? (u | 0x400000u) : ((u & 0x80000000u) ? 0xffc00000u : 0u);
  if (e == 0u) out = (u & 0x80000000u) | 0x7f800000u;                 /* +-0, subnormal -> +-inf */
  return yrt_sse_float(out);
}

/* common/math/math.h:38-42 */
YRT_SSE_FN float yrt_ref_rcp(float x) {
  const float r = yrt_rcpps(x);
  return (r + r) - (r * r) * x;
}
/* common/math/math.h:53-58 */
YRT_SSE_FN float yrt_ref_rsqrt(float x) {
  const float r = yrt_rsqrtps(x);
  return 1.5f * r + ((x * -0.5f) * r) * (r * r);
}

#endif
