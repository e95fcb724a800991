// sampler.h — host precompute of sample sets (samplers/sampler.cpp:85-158).
#pragma once

#include <functional>
#include <string>
#include <vector>

namespace yrt {

struct HostRandom {
  int seed = 1, state = 0, table[32] = {0};
  explicit HostRandom(int s = 27) { setSeed(s); }
  void setSeed(int s);
  int getInt();
  int getInt(int limit) { return getInt() % limit; }
  float getFloat();
};

// Light that precomputes its samples (HDRILight::precompute() == true): sample(u,v,out[8])
// writes wi.xyz, pdf, L.rgb, tMax.
struct LightSampleSource {
  int baseSample = 0;
  std::function<void(float, float, float*)> sample;
};

struct SampleRequest {
  int spp = 1, sets = 64, iteration = 0;
  int num1D = 0, num2D = 0;
  std::string filter = "bspline";
  std::vector<LightSampleSource> lights;
};

struct SampleTable {
  int spp = 1, sets = 64, numRecords = 0, numDims = 0, numLightSlots = 0;
  std::vector<float> dims;   // [numDims][numRecords]
  std::vector<float> light;  // [numRecords][numLightSlots][8]
};

void build_sample_table(const SampleRequest& req, SampleTable& out);

}  // namespace yrt
