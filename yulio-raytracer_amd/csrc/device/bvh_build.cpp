// bvh_build.cpp — host BVH builder for the GPU traversal kernels.
//
// Replaces Embree's rtcCommit SAH build (api/scene_flat.h:72-97).
// A binned-SAH BVH2 is built first and then collapsed into the 4-wide 128-B node /
// 48-B triangle layout of common/yrt_gpu_types.h: each 4-wide node takes a BVH2 node's
// two children and repeatedly opens its largest-area inner child until it has four.
// Guarantees the traversal kernel's invariants: root is an inner node, leaves hold 1..31
// triangles, and the worst-case traversal stack (3 pushes per 4-wide level) stays below
// YRT_STACK_DEPTH (forced object-median splits below a depth chosen from log2(N)).
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

struct Node2 {
  Box b[2];
  int idx[2], cnt[2];  // cnt 0: inner BVH2 node idx; > 0: leaf range [idx, idx+cnt)
};

struct Builder {
  std::vector<Prim> prims;
  std::vector<Node2> nodes;
#ifndef YRT_MAX_LEAF
#define YRT_MAX_LEAF 8
#endif
  int maxLeaf = YRT_MAX_LEAF;
#ifndef YRT_SAH_TRAV
#define YRT_SAH_TRAV 1.0f  // SAH cost of a traversal step relative to one triangle test
#endif
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
    const float splitCost = YRT_SAH_TRAV + (parentArea > 0.f ? bestCost / parentArea : (float)n);
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
    Node2& n = nodes[ni];
    n.b[0] = b0;
    n.b[1] = b1;
    n.idx[0] = i0; n.idx[1] = i1;
    n.cnt[0] = c0; n.cnt[1] = c1;
    return ni;
  }
};

struct Ref {
  Box b;
  int idx, cnt;
};

struct Collapser {
  const std::vector<Node2>& in;
  std::vector<GpuNode> out;
  int maxStack = 0;  // worst-case traversal stack: sum over a root path of (children - 1)
  explicit Collapser(const std::vector<Node2>& n) : in(n) {}

  // Emits the 4-wide node for BVH2 inner node `n2`; returns its index.
  int collapse(int n2, int stackAbove) {
    Ref ch[4];
    int k = 2;
    for (int j = 0; j < 2; ++j) ch[j] = Ref{in[n2].b[j], in[n2].idx[j], in[n2].cnt[j]};
    while (k < 4) {
      int best = -1;
      float bestArea = -1.f;
      for (int j = 0; j < k; ++j)
        if (ch[j].cnt == 0 && ch[j].b.area() > bestArea) { bestArea = ch[j].b.area(); best = j; }
      if (best < 0) break;
      const Node2& o = in[ch[best].idx];
      ch[best] = Ref{o.b[0], o.idx[0], o.cnt[0]};
      ch[k++] = Ref{o.b[1], o.idx[1], o.cnt[1]};
    }
    const int ni = (int)out.size();
    out.emplace_back();
    const int stackHere = stackAbove + (k - 1);
    if (stackHere > maxStack) maxStack = stackHere;
    int refs[4] = {-1, -1, -1, -1};
    for (int j = 0; j < k; ++j) {
      if (ch[j].cnt == 0) refs[j] = collapse(ch[j].idx, stackHere) << 5;
      else refs[j] = (ch[j].idx << 5) | ch[j].cnt;
    }
    GpuNode& g = out[ni];
    memset(&g, 0, sizeof(g));
    for (int j = 0; j < 4; ++j) {
      const bool v = j < k;
      g.lox[j] = v ? ch[j].b.lo[0] : 0.f; g.hix[j] = v ? ch[j].b.hi[0] : 0.f;
      g.loy[j] = v ? ch[j].b.lo[1] : 0.f; g.hiy[j] = v ? ch[j].b.hi[1] : 0.f;
      g.loz[j] = v ? ch[j].b.lo[2] : 0.f; g.hiz[j] = v ? ch[j].b.hi[2] : 0.f;
      g.child[j] = refs[j];
    }
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
  // A BVH2 path of depth D collapses to about D/2 four-wide levels of <= 3 pushes each.
  const int levels = (int)ceil(log2(std::max(1.0, N / 16.0)));
  B.medianDepth = std::max(0, std::min(28, (2 * stackDepth) / 3 - 2 - levels));
  if (N == 1) {
    Node2 n;
    n.b[0] = n.b[1] = B.prims[0].b;
    n.idx[0] = 0; n.cnt[0] = 1;
    n.idx[1] = 0; n.cnt[1] = 1;
    B.nodes.push_back(n);
  } else {
    bool leaf = false;
    int m = B.split(0, N, 0, leaf);
    if (leaf || m <= 0 || m >= N) m = N / 2;
    B.inner(0, m, N, 0);
  }
  Collapser C(B.nodes);
  C.collapse(0, 0);
  out.maxDepth = C.maxStack;
  if (C.maxStack > stackDepth - 1)
    throw std::runtime_error("BVH traversal stack bound exceeds YRT_STACK_DEPTH");
  out.nodes = std::move(C.out);
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
