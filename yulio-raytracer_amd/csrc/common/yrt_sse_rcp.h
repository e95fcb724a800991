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
 *   rsqrt: RN(1 / RN(sqrt(mid))) in float, both correctly rounded on both sides, rounded to
 *          12 bits: equal to the direct rounding on every entry (the closest call is 9e-5 of
 *          a unit from a tie).
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
/* Intel rcpps (one lane): RN(1/mid) rounded to 12 mantissa bits. mid = the input's top 11
 * mantissa bits + a half unit, exponent 0; 1/mid lies in (0.5, 1), so the 12-bit rounding is an
 * add of half a unit and a mask on its bits. That double rounding (24 then 12 bits) matches the
 * direct one on 2047 of the 2048 entries; entry 1984 rounds up across the tie-free midpoint and is
 * corrected (tests/test_sse_rcp.py, ref_check_sse_exhaustive, yrtDebugCheckMathTable). */
/* The inputs outside the normal range (exponent 0, or >= 253 for rcpps; negative, zero,
 * subnormal, inf or NaN for rsqrtps) are rare on the render path: on the GPU their selects run
 * only when some lane of the wave has one (a ballot and a uniform branch, one VALU instead of
 * about ten per call). */
#ifndef YRT_SSE_BRANCH
#define YRT_SSE_BRANCH 0  /* bit 0: rcpps, bit 1: rsqrtps (A/B switch; both cost shade scratch) */
#endif
#if defined(__HIP_DEVICE_COMPILE__)
#define YRT_SSE_ANY(bit, c) (!(YRT_SSE_BRANCH & (bit)) || __builtin_amdgcn_ballot_w64(c) != 0)
#else
#define YRT_SSE_ANY(bit, c) 1
#endif
YRT_SSE_FN float yrt_rcpps(float x) {
  const uint32_t u = yrt_sse_bits(x), s = u & 0x80000000u, e = (u >> 23) & 0xffu;
  const uint32_t mid = (u & 0x7ff000u) | 0x3f800800u;
  uint32_t y = yrt_sse_bits(yrt_sse_rcp_rn(yrt_sse_float(mid)));  /* exponent 126 */
  y = (y + 0x400u) & 0x7ff800u;
  y -= (mid == 0x3ffc0800u) ? 0x800u : 0u;                       /* entry 1984 */
  uint32_t out = s | ((253u - e) << 23) | y;                          /* e in [1, 252] */
  if (YRT_SSE_ANY(1, e - 1u > 251u)) {
    if (e >= 253u) out = s;                                           /* below 2^-126: +-0 */
    if (e == 255u) out = (u & 0x7fffffu) ? (u | 0x400000u) : s;       /* NaN stays (quiet), inf -> 0 */
    if (e == 0u) out = s | 0x7f800000u;                               /* +-0, subnormal -> +-inf */
  }
  return yrt_sse_float(out);
}

/* RN(sqrt(x)) for x in [1, 4): the hardware square root (within an ulp) corrected by the signs
 * of the two neighbours' FMA residuals (LLVM's correctly rounded f32 sqrt, without its
 * subnormal scaling, which this range does not need) */
YRT_SSE_FN float yrt_sse_sqrt_rn(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sdn = yrt_sse_float(yrt_sse_bits(s) - 1u), sup = yrt_sse_float(yrt_sse_bits(s) + 1u);
  float r = __builtin_fmaf(-sdn, s, x) <= 0.0f ? sdn : s;
  r = __builtin_fmaf(-sup, s, x) > 0.0f ? sup : r;
  return r;
#else
  return __builtin_sqrtf(x);
#endif
}
/* Intel rsqrtps (one lane): RN(1 / RN(sqrt(mid))) rounded to 12 mantissa bits, mid = the input's
 * top 10 mantissa bits + a half unit, times 2^p (exponent parity); that double rounding matches
 * the direct one on all 2048 entries (tests/test_sse_rcp.py, exhaustive checks). An exact integer
 * form (a v_rsq estimate checked by (2q -+ 1)^2 A against 2^39) needs two 64-bit multiply-adds,
 * quarter-rate instructions. */
YRT_SSE_FN float yrt_rsqrtps(float x) {
  const uint32_t u = yrt_sse_bits(x), e = (u >> 23) & 0xffu;
  const int E = (int)e - 127, p = E & 1, k = (E - p) / 2;
  const uint32_t mid = ((uint32_t)(127 + p) << 23) | (u & 0x7fe000u) | 0x1000u;
  const uint32_t y = (yrt_sse_bits(yrt_sse_rcp_rn(yrt_sse_sqrt_rn(yrt_sse_float(mid)))) + 0x400u) & 0x7ff800u;
  uint32_t out = ((uint32_t)(126 - k) << 23) | y;                     /* positive, e in [1, 254] */
  if (YRT_SSE_ANY(2, u - 0x00800000u >= 0x7f000000u)) {
    if (u & 0x80000000u) out = 0xffc00000u;                           /* negative: default NaN */
    if (e == 255u) out = (u & 0x7fffffu) ? (u | 0x400000u) : ((u & 0x80000000u) ? 0xffc00000u : 0u);
    if (e == 0u) out = (u & 0x80000000u) | 0x7f800000u;               /* +-0, subnormal -> +-inf */
  }
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
