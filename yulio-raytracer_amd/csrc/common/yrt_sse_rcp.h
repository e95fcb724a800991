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
 *   rcp:   RN(1/mid) in float (correctly rounded on both sides), rounded to 12 bits, with
 *          the one entry where that double rounding differs corrected (see yrt_rcpps); an exact
 *          integer form (q = RN(2^25 / D), D = 4097 + 2i, one multiply to check the remainder)
 *          measured ~8 VALU more per call;
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

/* RN(1/x) for x in [1, 2): the hardware estimate plus one FMA Newton step is correctly rounded
 * there on gfx950 (rcp_rn in yrt_math.h, checked on all 2^32 inputs by yrtDebugCheckMath) */
YRT_SSE_FN float yrt_sse_rcp_rn(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  const float y = __builtin_amdgcn_rcpf(x);
  return __builtin_fmaf(__builtin_fmaf(-x, y, 1.0f), y, y);
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

/* Intel rcpps (one lane): RN(1/mid) rounded to 12 mantissa bits. mid = the input's top 11
 * mantissa bits + a half unit, exponent 0; 1/mid lies in (0.5, 1), so the 12-bit rounding is an
 * add of half a unit and a mask on its bits. That double rounding (24 then 12 bits) matches the
 * direct one on 2047 of the 2048 entries; entry 1984 rounds up across the tie-free midpoint and is
 * corrected (tests/test_sse_rcp.py, ref_check_sse_exhaustive, yrtDebugCheckMathTable). */
YRT_SSE_FN float yrt_rcpps(float x) {
  const uint32_t u = yrt_sse_bits(x), s = u & 0x80000000u, e = (u >> 23) & 0xffu;
  const uint32_t mid = (u & 0x7ff000u) | 0x3f800800u;
  uint32_t y = yrt_sse_bits(yrt_sse_rcp_rn(yrt_sse_float(mid)));  /* exponent 126 */
  y = (y + 0x400u) & 0x7ff800u;
  y -= (mid == 0x3ffc0800u) ? 0x800u : 0u;                       /* entry 1984 */
  uint32_t out = s | ((253u - e) << 23) | y;
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


/* Intel rsqrtps (one lane) */
YRT_SSE_FN float yrt_rsqrtps(float x) {
  const uint32_t u = yrt_sse_bits(x), e = (u >> 23) & 0xffu;
  const int E = (int)e - 127, p = E & 1, k = (E - p) / 2;
  /* (a 4 KB table of the 2048 mantissas in the code object measured 0.6 % slower on C3 and C4:
   * a dependent load where this is ~12 VALU, profiles/r06/ab_r06a.txt) */
  const uint32_t m = yrt_rsqrtps_m((uint32_t)p, (u >> 13) & 0x3ffu);
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
