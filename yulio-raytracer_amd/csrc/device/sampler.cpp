// sampler.cpp — host precompute of the sample table: Distribution1D/2D, the pixel filter
// importance table and SamplerFactory::init.
//
//   Distribution1D::init/sample   samplers/distribution1d.cpp:42-74
//   Distribution2D::init/sample   samplers/distribution2d.cpp:34-68
//   Filter::init/sample           filters/filter.cpp:22-43, BSplineFilter filters/bsplinefilter.h:30-42
//   jittered / multiJittered      samplers/patterns.h:28-68 (Permutation common/math/permutation.h:42-48,
//                                 vector_t::shuffle common/sys/stl/vector.h:129-133)
//   SamplerFactory::init          samplers/sampler.cpp:85-158
//   Random                        common/math/random.h:28-78
#include "sampler.h"

#include <math.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <stdexcept>

#include "../common/yrt_math.h"
#include "distribution.h"

namespace yrt {

// ---------------------------------------------------------------- Random
void HostRandom::setSeed(int s) {
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
int HostRandom::getInt() {
  const int a = 16807, m = 2147483647, q = 127773, r = 2836;
  int k = seed / q;
  seed = a * (seed - k * q) - r * k;
  if (seed < 0) seed += m;
  int j = state / (1 + (2147483647 - 1) / 32);
  state = table[j];
  table[j] = seed;
  return state;
}
float HostRandom::getFloat() { return std::min(getInt() / 2147483647.0f, 1.0f - kUlp); }

// ---------------------------------------------------------------- distributions
static void dist1d_init(const float* f, int size, float* cdf, float* pdf) {
  cdf[0] = 0.0f;
  for (int i = 1; i < size + 1; i++) cdf[i] = cdf[i - 1] + f[i - 1];
  const float rcpSum = cdf[size] == 0.0f ? 0.0f : rcpf_(cdf[size]);
  for (int i = 1; i < size + 1; i++) {
    pdf[i - 1] = f[i - 1] * rcpSum * float(size);
    cdf[i] *= rcpSum;
  }
  cdf[size] = 1.0f;
}
static void dist1d_sample(const float* cdf, const float* pdf, int size, float u, float& x, float& p) {
  const float* ptr = std::upper_bound(cdf, cdf + size, u);
  const int index = std::max(0, std::min(int(ptr - cdf - 1), size - 1));
  const float fraction = (u - cdf[index]) * rcpf_(cdf[index + 1] - cdf[index]);
  x = float(index) + fraction;
  p = pdf[index];
}

void dist2d_init(const float* f, int w, int h, std::vector<float>& ycdf, std::vector<float>& ypdf,
                 std::vector<float>& xcdf, std::vector<float>& xpdf) {
  ycdf.assign(h + 1, 0.f);
  ypdf.assign(h, 0.f);
  xcdf.assign((size_t)h * (w + 1), 0.f);
  xpdf.assign((size_t)h * w, 0.f);
  std::vector<float> fy(h);
  for (int y = 0; y < h; y++) {
    fy[y] = 0.0f;
    for (int x = 0; x < w; x++) fy[y] += f[(size_t)y * w + x];
    dist1d_init(f + (size_t)y * w, w, &xcdf[(size_t)y * (w + 1)], &xpdf[(size_t)y * w]);
  }
  dist1d_init(fy.data(), h, ycdf.data(), ypdf.data());
}

void dist2d_sample(const std::vector<float>& ycdf, const std::vector<float>& ypdf, const std::vector<float>& xcdf,
                   const std::vector<float>& xpdf, int w, int h, float ux, float uy, float& sx, float& sy,
                   float& pdf) {
  float py, px;
  dist1d_sample(ycdf.data(), ypdf.data(), h, uy, sy, py);
  const int y = std::max(0, std::min(int(sy), h - 1));
  dist1d_sample(&xcdf[(size_t)y * (w + 1)], &xpdf[(size_t)y * w], w, ux, sx, px);
  pdf = px * py;
}

// ---------------------------------------------------------------- filters
struct FilterTable {
  float width = 0, height = 0;
  int tableSize = 256;
  std::vector<float> ycdf, ypdf, xcdf, xpdf;
};

static float bspline_eval(float dx, float dy) {
  const float d = sqrtf(dx * dx + dy * dy);
  if (d > 2.0f) return 0.0f;
  if (d < 1.0f) {
    const float t = 1.0f - d;
    return ((((-3.0f * t) + 3.0f) * t + 3.0f) * t + 1.0f) / 6.0f;
  }
  const float t = 2.0f - d;
  return t * t * t / 6.0f;
}
static float box_eval(float dx, float dy) {
  const float halfWidth = 0.5f;
  return (fabsf(dx) <= halfWidth && fabsf(dy) <= halfWidth) ? 1.0f : 0.0f;
}

static const FilterTable& filter_table(const std::string& name) {
  static std::mutex mu;
  static std::map<std::string, FilterTable> cache;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(name);
  if (it != cache.end()) return it->second;
  FilterTable t;
  const bool bs = name == "bspline";
  t.width = t.height = bs ? 4.0f : 2.0f * 0.5f;
  const int n = t.tableSize;
  const float invTableSize = 1.0f / n;
  // Array2D absoluteValues(x, y) handed to Distribution2D as f[x][y] (filters/filter.cpp:24-34)
  std::vector<float> f((size_t)n * n);
  for (int x = 0; x < n; ++x)
    for (int y = 0; y < n; ++y) {
      const float px = (x + 0.5f) * invTableSize * t.width - t.width * 0.5f;
      const float py = (y + 0.5f) * invTableSize * t.height - t.height * 0.5f;
      f[(size_t)x * n + y] = fabsf(bs ? bspline_eval(px, py) : box_eval(px, py));
    }
  dist2d_init(f.data(), n, n, t.ycdf, t.ypdf, t.xcdf, t.xpdf);
  return cache.emplace(name, std::move(t)).first->second;
}

static void filter_sample(const FilterTable& t, float u, float v, float& ox, float& oy) {
  float sx, sy, pdf;
  dist2d_sample(t.ycdf, t.ypdf, t.xcdf, t.xpdf, t.tableSize, t.tableSize, u, v, sx, sy, pdf);
  ox = sx / float(t.tableSize) * t.width - t.width * 0.5f;
  oy = sy / float(t.tableSize) * t.height - t.height * 0.5f;
}

// ---------------------------------------------------------------- patterns
static void permutation(std::vector<int>& perm, int n, HostRandom& rng) {
  perm.resize(n);
  for (int i = 0; i < n; i++) perm[i] = i;
  for (int i = 0; i < n; i++) std::swap(perm[i], perm[rng.getInt(n)]);
}

static void jittered(float* samples, uint32_t n, HostRandom& rng) {
  const float scale = 1.0f / n;
  std::vector<int> perm;
  permutation(perm, (int)n, rng);
  for (uint32_t i = 0; i < n; i++) samples[perm[i]] = (float(i) + rng.getFloat()) * scale;
}

static void multiJittered(float* samples /* 2*N */, uint32_t N, HostRandom& rng) {
  uint32_t b = (uint32_t)sqrtf(float(N));
  if (b * b < N) b++;
  std::vector<float> grid((size_t)b * b * 2);
  std::vector<uint32_t> numbers(b);
  for (uint32_t i = 0; i < b; i++) numbers[i] = i;
  auto shuffle = [&]() {
    for (size_t i = 0; i < b; i++) std::swap(numbers[i], numbers[rng.getInt((int)b)]);
  };
  for (uint32_t i = 0; i < b; i++) {
    shuffle();
    for (uint32_t j = 0; j < b; j++)
      grid[((size_t)i * b + j) * 2 + 0] = float(i) / float(b) + (numbers[j] + rng.getFloat()) / float(b * b);
  }
  for (uint32_t i = 0; i < b; i++) {
    shuffle();
    for (uint32_t j = 0; j < b; j++)
      grid[((size_t)j * b + i) * 2 + 1] = float(i) / float(b) + (numbers[j] + rng.getFloat()) / float(b * b);
  }
  std::vector<int> perm;
  permutation(perm, (int)N, rng);
  for (uint32_t n = 0; n < N; n++) {
    const uint32_t np = perm[n];
    samples[2 * n + 0] = grid[((size_t)(np / b) * b + np % b) * 2 + 0];
    samples[2 * n + 1] = grid[((size_t)(np / b) * b + np % b) * 2 + 1];
  }
}

static uint32_t round_up_pow2(uint32_t x) {
  uint32_t r = 1;
  while (r < x) r <<= 1;
  return r;
}

// SamplerFactory::init restated. Layout: SoA [dim][set*spp + s].
void build_sample_table(const SampleRequest& req, SampleTable& out) {
  const int sets = req.sets;
  const int spp = (int)round_up_pow2((uint32_t)std::max(1, req.spp));  // sampler.cpp:91 rounds UP
  const int n1 = req.num1D, n2 = req.num2D, nl = (int)req.lights.size();
  const int chunkSize = std::max(spp, 64);
  const int currentChunk = int(req.iteration * spp) / chunkSize;
  const int offset = (req.iteration * spp) % chunkSize;
  HostRandom rng;
  rng.setSeed(currentChunk * 5897);
  const FilterTable* ft = req.filter == "none" ? nullptr : &filter_table(req.filter);

  out.spp = spp;
  out.sets = sets;
  out.numRecords = sets * spp;
  out.numDims = 5 + n1 + 2 * n2;
  out.numLightSlots = nl;
  out.dims.assign((size_t)out.numDims * out.numRecords, 0.f);
  out.light.assign((size_t)out.numRecords * std::max(nl, 1) * 8, 0.f);

  std::vector<float> pixel(2 * chunkSize), time(chunkSize), lens(2 * chunkSize), s1(chunkSize), s2(2 * chunkSize);
  auto D = [&](int dim, int rec) -> float& { return out.dims[(size_t)dim * out.numRecords + rec]; };
  for (int set = 0; set < sets; set++) {
    multiJittered(pixel.data(), chunkSize, rng);
    jittered(time.data(), chunkSize, rng);
    multiJittered(lens.data(), chunkSize, rng);
    for (int s = 0; s < spp; s++) {
      const int rec = set * spp + s;
      float px = pixel[2 * (offset + s)], py = pixel[2 * (offset + s) + 1];
      if (ft) {
        float fx, fy;
        filter_sample(*ft, px, py, fx, fy);
        px = fx + 0.5f;
        py = fy + 0.5f;
      }
      D(0, rec) = px;
      D(1, rec) = py;
      D(2, rec) = lens[2 * (offset + s)];
      D(3, rec) = lens[2 * (offset + s) + 1];
      D(4, rec) = time[offset + s];
    }
    for (int d = 0; d < n1; d++) {
      jittered(s1.data(), chunkSize, rng);
      for (int s = 0; s < spp; s++) D(5 + d, set * spp + s) = s1[offset + s];
    }
    for (int d = 0; d < n2; d++) {
      multiJittered(s2.data(), chunkSize, rng);
      for (int s = 0; s < spp; s++) {
        D(5 + n1 + 2 * d, set * spp + s) = s2[2 * (offset + s)];
        D(5 + n1 + 2 * d + 1, set * spp + s) = s2[2 * (offset + s) + 1];
      }
    }
    for (int d = 0; d < nl; d++) {
      const LightSampleSource& L = req.lights[d];
      for (int s = 0; s < spp; s++) {
        const int rec = set * spp + s;
        const float ux = D(5 + n1 + 2 * L.baseSample, rec), uy = D(5 + n1 + 2 * L.baseSample + 1, rec);
        float* o = &out.light[((size_t)rec * nl + d) * 8];
        L.sample(ux, uy, o);
      }
    }
  }
}

}  // namespace yrt
