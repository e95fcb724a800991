// bvh_build.cpp — host binned-SAH BVH2 builder for the GPU traversal kernels.
//
// Replaces Embree's rtcCommit SAH build (api/scene_flat.h:72-97).
// Output is the flat 64-B node / 48-B triangle layout of common/yrt_gpu_types.h.
// Guarantees the traversal kernel's invariants: root is an inner node, leaves hold 1..31
// triangles, and no inner node is deeper than YRT_STACK_DEPTH-1 (forced object-median
// splits below a depth chosen from log2(N)), so the per-lane LDS stack never overflows.
#include "bvh_build.h"

#include <math.h>
#include <string.h>

#include <algorithm>
#include <stdexcept>

namespace yrt {

namespace {

struct Box {
  float lo[3], hi[3];
  void reset() {
    for (int k = 0; k < 3; ++k) { lo[k] = INFINITY; hi[k] = -INFINITY; }
  }
  void grow(const Box& b) {
    for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], b.lo[k]); hi[k] = std::max(hi[k], b.hi[k]); }
  }
  void growP(const float* p) {
    for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], p[k]); hi[k] = std::max(hi[k], p[k]); }
  }
  float area() const {
    const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    if (!(dx >= 0 && dy >= 0 && dz >= 0)) return 0.f;
    return 2.f * (dx * dy + dy * dz + dz * dx);
  }
};

struct Prim {
  Box b;
  float c[3];
  int id;
};

struct Builder {
  std::vector<Prim> prims;
  std::vector<GpuNode> nodes;
  int maxLeaf = 8;
  int medianDepth = 24;
  int maxDepthSeen = 0;

  Box bounds(int b, int e) const {
    Box bb;
    bb.reset();
    for (int i = b; i < e; ++i) bb.grow(prims[i].b);
    return bb;
  }

  // returns split position m (b < m < e)
  int split(int b, int e, int depth, bool& makeLeaf) {
    const int n = e - b;
    makeLeaf = false;
    Box cb;
    cb.reset();
    for (int i = b; i < e; ++i) cb.growP(prims[i].c);
    int axis = 0;
    float ext = cb.hi[0] - cb.lo[0];
    for (int k = 1; k < 3; ++k)
      if (cb.hi[k] - cb.lo[k] > ext) { ext = cb.hi[k] - cb.lo[k]; axis = k; }
    if (!(ext > 0.f)) {  // all centroids equal
      if (n <= maxLeaf) { makeLeaf = true; return e; }
      return b + n / 2;
    }
    if (depth >= medianDepth) {
      const int m = b + n / 2;
      std::nth_element(prims.begin() + b, prims.begin() + m, prims.begin() + e,
                       [axis](const Prim& x, const Prim& y) { return x.c[axis] < y.c[axis]; });
      return m;
    }
    const int NB = 32;
    float bestCost = INFINITY;
    int bestAxis = -1, bestBin = -1;
    for (int ax = 0; ax < 3; ++ax) {
      const float lo = cb.lo[ax], hi = cb.hi[ax];
      if (!(hi > lo)) continue;
      const float scale = NB / (hi - lo);
      Box bb[NB];
      int cnt[NB] = {0};
      for (int k = 0; k < NB; ++k) bb[k].reset();
      for (int i = b; i < e; ++i) {
        int bin = std::min(NB - 1, (int)((prims[i].c[ax] - lo) * scale));
        cnt[bin]++;
        bb[bin].grow(prims[i].b);
      }
      float rightArea[NB];
      int rightCnt[NB];
      Box acc;
      acc.reset();
      int ac = 0;
      for (int k = NB - 1; k > 0; --k) {
        acc.grow(bb[k]);
        ac += cnt[k];
        rightArea[k] = acc.area();
        rightCnt[k] = ac;
      }
      acc.reset();
      ac = 0;
      for (int k = 0; k < NB - 1; ++k) {
        acc.grow(bb[k]);
        ac += cnt[k];
        if (ac == 0 || rightCnt[k + 1] == 0) continue;
        const float cost = acc.area() * ac + rightArea[k + 1] * rightCnt[k + 1];
        if (cost < bestCost) { bestCost = cost; bestAxis = ax; bestBin = k; }
      }
    }
    const float parentArea = bounds(b, e).area();
    const float leafCost = (float)n;
    const float splitCost = 1.0f + (parentArea > 0.f ? bestCost / parentArea : (float)n);
    if (n <= maxLeaf && leafCost <= splitCost) { makeLeaf = true; return e; }
    if (bestAxis < 0) return b + n / 2;
    const float lo = cb.lo[bestAxis], hi = cb.hi[bestAxis];
    const float scale = NB / (hi - lo);
    auto mid = std::partition(prims.begin() + b, prims.begin() + e, [&](const Prim& p) {
      return std::min(NB - 1, (int)((p.c[bestAxis] - lo) * scale)) <= bestBin;
    });
    int m = (int)(mid - prims.begin());
    if (m <= b || m >= e) m = b + n / 2;
    return m;
  }

  // Builds the subtree for [b,e); returns packed (index, count) of the child reference.
  void child(int b, int e, int depth, int& idx, int& cnt, Box& bb) {
    bb = bounds(b, e);
    const int n = e - b;
    if (n <= 2 && n < 32) { idx = b; cnt = n; return; }
    bool leaf = false;
    const int m = split(b, e, depth, leaf);
    if (leaf && n <= 31) { idx = b; cnt = n; return; }
    idx = inner(b, m, e, depth);
    cnt = 0;
  }

  int inner(int b, int m, int e, int depth) {
    if (depth > maxDepthSeen) maxDepthSeen = depth;
    const int ni = (int)nodes.size();
    nodes.emplace_back();
    int i0, c0, i1, c1;
    Box b0, b1;
    child(b, m, depth + 1, i0, c0, b0);
    child(m, e, depth + 1, i1, c1, b1);
    GpuNode& n = nodes[ni];
    n.b0[0] = b0.lo[0]; n.b0[1] = b0.hi[0]; n.b0[2] = b0.lo[1]; n.b0[3] = b0.hi[1];
    n.b1[0] = b1.lo[0]; n.b1[1] = b1.hi[0]; n.b1[2] = b1.lo[1]; n.b1[3] = b1.hi[1];
    n.b2[0] = b0.lo[2]; n.b2[1] = b0.hi[2]; n.b2[2] = b1.lo[2]; n.b2[3] = b1.hi[2];
    n.c[0] = i0; n.c[1] = i1; n.c[2] = c0; n.c[3] = c1;
    return ni;
  }
};

}  // namespace

void build_bvh(const std::vector<float>& v /* 9 floats per triangle */, const std::vector<uint32_t>& flags,
               int stackDepth, BvhResult& out) {
  const int N = (int)(v.size() / 9);
  out.nodes.clear();
  out.tris.clear();
  out.order.clear();
  if (N == 0) return;
  Builder B;
  B.prims.resize(N);
  for (int i = 0; i < N; ++i) {
    Prim& p = B.prims[i];
    p.b.reset();
    for (int k = 0; k < 3; ++k) p.b.growP(&v[(size_t)i * 9 + 3 * k]);
    for (int k = 0; k < 3; ++k) p.c[k] = 0.5f * (p.b.lo[k] + p.b.hi[k]);
    p.id = i;
  }
  const int levels = (int)ceil(log2(std::max(1.0, N / 16.0)));
  B.medianDepth = std::max(0, std::min(28, (stackDepth - 2) - levels));
  if (N == 1) {
    GpuNode n;
    Box b = B.prims[0].b;
    n.b0[0] = n.b1[0] = b.lo[0]; n.b0[1] = n.b1[1] = b.hi[0];
    n.b0[2] = n.b1[2] = b.lo[1]; n.b0[3] = n.b1[3] = b.hi[1];
    n.b2[0] = n.b2[2] = b.lo[2]; n.b2[1] = n.b2[3] = b.hi[2];
    n.c[0] = n.c[1] = 0; n.c[2] = n.c[3] = 1;
    B.nodes.push_back(n);
  } else {
    bool leaf = false;
    int m = B.split(0, N, 0, leaf);
    if (leaf || m <= 0 || m >= N) m = N / 2;
    B.inner(0, m, N, 0);
  }
  out.maxDepth = B.maxDepthSeen;
  if (out.maxDepth > stackDepth - 1)
    throw std::runtime_error("BVH deeper than the traversal stack; raise YRT_STACK_DEPTH");
  out.nodes = std::move(B.nodes);
  out.order.resize(N);
  out.tris.resize(N);
  for (int i = 0; i < N; ++i) {
    const int id = B.prims[i].id;
    out.order[i] = id;
    const float* t = &v[(size_t)id * 9];
    GpuTri& g = out.tris[i];
    // e1 = v0 - v1, e2 = v2 - v0 (rtcore convention)
    g.v0[0] = t[0]; g.v0[1] = t[1]; g.v0[2] = t[2];
    g.e1[0] = t[0] - t[3]; g.e1[1] = t[1] - t[4]; g.e1[2] = t[2] - t[5];
    g.e2[0] = t[6] - t[0]; g.e2[1] = t[7] - t[1]; g.e2[2] = t[8] - t[2];
    int gid = id;
    uint32_t fl = flags[id];
    memcpy(&g.v0[3], &gid, 4);
    memcpy(&g.e1[3], &fl, 4);
    g.e2[3] = 0.f;
  }
}

}  // namespace yrt
