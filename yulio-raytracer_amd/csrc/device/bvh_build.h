// bvh_build.h — host 4-wide BVH builder (see bvh_build.cpp).
#pragma once

#include <stdint.h>

#include <vector>

#include "../common/yrt_gpu_types.h"

namespace yrt {

struct BvhResult {
  std::vector<GpuNode> nodes;
  std::vector<GpuTri> tris;   // leaf order
  std::vector<int> order;     // leaf slot -> global triangle id
  int maxDepth = 0;           // worst-case traversal stack entries (scene info 'bvhDepth')
};

// v: 9 floats (v0,v1,v2) per global triangle id; flags: per-triangle GpuTri flags (bit0 cull)
// v1 (optional): the triangles' vertices at the end of the frame time (moving geometry); the
// boxes then bound both (trianglemesh_full.cpp:152-166), the leaf records hold the t = 0 triangle
void build_bvh(const std::vector<float>& v, const std::vector<uint32_t>& flags, int stackDepth, BvhResult& out,
               const std::vector<float>* v1 = nullptr);


}  // namespace yrt
