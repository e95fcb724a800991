// ref_kat.cpp — TEST INFRASTRUCTURE ONLY (oracle/_ref). Compiled by `make -C oracle ref`
// against the reference's own, unmodified headers and sources where they lie under
// /root/reference (never copied into this repo):
//   common/math/random.h       embree::Random          (Park-Miller + Bays-Durham shuffle)
//   common/math/permutation.h  embree::Permutation     (Permutation(n, rng), :42-48)
//   common/sys/stl/vector.h    embree::vector_t::shuffle (:129-133)
//   common/sys/platform.cpp    alignedMalloc/alignedFree used by vector_t
// Everything else the reference's sampler needs (devices/device_singleray/default.h, the
// filter's Distribution2D) pulls in common/simd, which does not compile with g++
// (common/simd/sseb.h:108), so it cannot be built here.
//
// The loops below are this build's own driver code around those reference types: they are
// the call patterns of integratorrenderer.cpp:134,149 (per-tile set draw) and of
// SamplerFactory::init (samplers/sampler.cpp:93-139, RNG order pixel/time/lens then 1D then
// 2D dims) with the multi-jittered / jittered constructions of samplers/patterns.h:28-68
// written out against embree::Random / Permutation / vector_t. tests/test_ref_pin.py
// compares them with the C restatement (oracle/yrt_oracle.c) bit for bit.
#include "math/random.h"
#include "math/permutation.h"
#include "sys/ref.h"
#include "sys/stl/vector.h"

#include <stdint.h>
#include <string.h>

#include <vector>

using embree::Permutation;
using embree::Random;

namespace {

void jittered_ref(float* out, unsigned n, Random& rng) {
  const float scale = 1.0f / n;
  Permutation p((int)n, rng);
  for (unsigned i = 0; i < n; i++) out[p[i]] = (float(i) + rng.getFloat()) * scale;
}

void multi_jittered_ref(float* out2, unsigned N, Random& rng) {
  unsigned b = (unsigned)sqrtf(float(N));
  if (b * b < N) b++;
  std::vector<float> gx(b * b), gy(b * b);
  embree::vector_t<unsigned> numbers(b);
  for (unsigned i = 0; i < b; i++) numbers[i] = i;
  for (unsigned i = 0; i < b; i++) {
    numbers.shuffle(rng);
    for (unsigned j = 0; j < b; j++) gx[i * b + j] = float(i) / float(b) + (numbers[j] + rng.getFloat()) / float(b * b);
  }
  for (unsigned i = 0; i < b; i++) {
    numbers.shuffle(rng);
    for (unsigned j = 0; j < b; j++) gy[j * b + i] = float(i) / float(b) + (numbers[j] + rng.getFloat()) / float(b * b);
  }
  Permutation p((int)N, rng);
  for (unsigned n = 0; n < N; n++) {
    const unsigned np = (unsigned)p[n];
    out2[2 * n] = gx[(np / b) * b + np % b];
    out2[2 * n + 1] = gy[(np / b) * b + np % b];
  }
}

}  // namespace

extern "C" {

void ref_random_ints(int seed, int n, int32_t* out) {
  Random r(seed);
  r.setSeed(seed);
  for (int i = 0; i < n; ++i) out[i] = r.getInt();
}

void ref_random_floats(int seed, int n, float* out) {
  Random r(seed);
  r.setSeed(seed);
  for (int i = 0; i < n; ++i) out[i] = r.getFloat();
}

// Permutation(size, Random(seed)) repeated `count` times from the same generator
void ref_permutations(int size, int seed, int count, int32_t* out) {
  Random r(seed);
  r.setSeed(seed);
  for (int c = 0; c < count; ++c) {
    Permutation p(size, r);
    for (int i = 0; i < size; ++i) out[(size_t)c * size + i] = p[i];
  }
}

// vector_t<uint32>::shuffle of 0..n-1, `count` times in place from one generator
void ref_shuffles(int n, int seed, int count, uint32_t* out) {
  Random r(seed);
  r.setSeed(seed);
  embree::vector_t<unsigned> v(n);
  for (int i = 0; i < n; ++i) v[i] = (unsigned)i;
  for (int c = 0; c < count; ++c) {
    v.shuffle(r);
    for (int i = 0; i < n; ++i) out[(size_t)c * n + i] = v[i];
  }
}

// RenderJob::renderTile set draw: Random(tile_x*91711 + tile_y*81551 + 3433*firstActiveLine)
// per 16x16 tile (tile_x, tile_y: the tile's first pixel), one getInt(sets) per in-bounds pixel in scan order (firstActiveLine = 0)
void ref_pixel_sets(int width, int height, int sets, uint8_t* out) {
  const int tx = (width + 15) / 16, ty = (height + 15) / 16;
  for (int t = 0; t < tx * ty; ++t) {
    const int x0 = (t % tx) * 16, y0 = (t / tx) * 16;  // tile_x / tile_y are pixel coordinates
    Random rng(x0 * 91711 + y0 * 81551);
    for (int y = y0; y < y0 + 16; ++y)
      for (int x = x0; x < x0 + 16; ++x) {
        if (x >= width || y >= height) continue;
        out[(size_t)y * width + x] = (uint8_t)rng.getInt(sets);
      }
  }
}

// SamplerFactory::init without a pixel filter (filter "none"): table[dim][set*spp + s] with
// dims pixel.x, pixel.y, lens.x, lens.y, time, 1D[num1D], 2D[num2D] (x, y); spp a power of 2
int ref_sample_table_nofilter(int spp, int sets, int iteration, int num1D, int num2D, float* out) {
  const int chunk = spp > 64 ? spp : 64;
  const int currentChunk = (iteration * spp) / chunk;
  const int offset = (iteration * spp) % chunk;
  Random r;  // default seed, then setSeed (sampler.cpp:96-97)
  r.setSeed(currentChunk * 5897);
  const int rec = sets * spp;
  std::vector<float> pix(2 * chunk), tim(chunk), lens(2 * chunk), s1(chunk), s2(2 * chunk);
  auto T = [&](int d, int rc) -> float& { return out[(size_t)d * rec + rc]; };
  for (int set = 0; set < sets; set++) {
    multi_jittered_ref(pix.data(), chunk, r);
    jittered_ref(tim.data(), chunk, r);
    multi_jittered_ref(lens.data(), chunk, r);
    for (int s = 0; s < spp; s++) {
      const int rc = set * spp + s;
      T(0, rc) = pix[2 * (offset + s)];
      T(1, rc) = pix[2 * (offset + s) + 1];
      T(2, rc) = lens[2 * (offset + s)];
      T(3, rc) = lens[2 * (offset + s) + 1];
      T(4, rc) = tim[offset + s];
    }
    for (int d = 0; d < num1D; d++) {
      jittered_ref(s1.data(), chunk, r);
      for (int s = 0; s < spp; s++) T(5 + d, set * spp + s) = s1[offset + s];
    }
    for (int d = 0; d < num2D; d++) {
      multi_jittered_ref(s2.data(), chunk, r);
      for (int s = 0; s < spp; s++) {
        T(5 + num1D + 2 * d, set * spp + s) = s2[2 * (offset + s)];
        T(5 + num1D + 2 * d + 1, set * spp + s) = s2[2 * (offset + s) + 1];
      }
    }
  }
  return rec;
}

}  // extern "C"
