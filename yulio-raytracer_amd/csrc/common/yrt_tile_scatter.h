// yrt_tile_scatter.h — which image tile a sharded job's logical tile covers.
//
// A job's 16x16 tiles are dealt round-robin: logical tile t (frame-major) goes to shard t mod N
// (SURVEY §8(e)). Read as image tiles directly, shard r of N = 8 gets every 8th tile column of
// a 2048- or 1536-pixel frame, and on the C3 stand-in, whose atrium repeats along x, one such
// column set costs 16 % more than the mean (tools/cube_shard_time.py: shard 2 at 56.3 ms against
// 48.5, three repetitions within 0.4 ms; profiles/r06/scaling_prediction_c3_r06m.txt). So when
// a job is sharded (tile stride > 1), logical tile t of a frame covers image tile
// yrt_tile_scatter(t, T) instead: a fixed pseudo-random bijection of [0, T), which gives every
// shard a uniform sample of the image. Every pixel's samples and seeds depend on its image
// position only, so the frame is bit-identical for every deal; the renderer (batch_tile) and
// the gather (slab_pixel) apply the same map. Unsharded jobs keep the identity (row-major
// batches, the texture locality the single-GPU tuning was measured with).
//
// The map: a bijection h on [0, 2^B), 2^B >= T (two rounds of an odd multiply mod 2^B and a
// right xorshift by ceil(B/2), each invertible), restricted to [0, T) by cycle walking (apply h
// until the value is below T: a bijection of [0, T), fewer than two steps on average since
// T > 2^(B-1)).
#pragma once

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define YRT_TS_FN __host__ __device__ static inline
#else
#define YRT_TS_FN static inline
#endif

YRT_TS_FN uint32_t yrt_tile_mix(uint32_t x, uint32_t m, int h) {
  x = (x * 0x9E3779B1u) & m;
  x ^= x >> h;
  x = (x * 0x85EBCA6Bu) & m;
  x ^= x >> h;
  return x;
}

YRT_TS_FN int yrt_tile_scatter(int t, int T) {
  if (T <= 2) return t;
  const int B = 32 - __builtin_clz((unsigned)(T - 1));  // 2^B >= T, B in [2, 31]
  const uint32_t m = (1u << B) - 1u;
  const int h = (B + 1) >> 1;
  uint32_t x = (uint32_t)t;
  do {
    x = yrt_tile_mix(x, m, h);
  } while (x >= (uint32_t)T);
  return (int)x;
}
