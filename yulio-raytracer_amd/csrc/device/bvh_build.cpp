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

#include <float.h>
#include <math.h>
#include <stdlib.h>
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

// Spatial-split builder (SBVH, Stich et al. 2009): at each node the binned object split
// (SAH over reference centroids) competes with a binned spatial split, which cuts the node
// box with an axis plane and lets a triangle straddling the plane be referenced from both
// sides with its box clipped to each side. Architectural scenes (long walls, floors, arches)
// have many large triangles whose boxes overlap everything under them; splitting them cuts
// the node visits per ray. The traversal is unaffected: a leaf stores the full triangle, the
// closest hit is the smallest (t, id) over all references, and duplicates only re-test it.
// Spatial splits are tried only where the object split's children overlap by more than
// YRT_SBVH_ALPHA of the root area, and stop once the references exceed (1 + YRT_SBVH_BUDGET) N.
#ifndef YRT_SBVH_ALPHA
#define YRT_SBVH_ALPHA 1e-5f
#endif
#ifndef YRT_SBVH_BUDGET
#define YRT_SBVH_BUDGET 0.5f
#endif
struct SRef {
  Box b;
  int id;
  float c(int k) const { return 0.5f * (b.lo[k] + b.hi[k]); }
};

// Box of triangle t (9 floats) inside the slab lo <= x[axis] <= hi, padded outward by a
// few ulps on the two other axes (edge/plane intersections round), exact on `axis`.
Box clip_tri(const float* t, int axis, float lo, float hi) {
  Box r;
  r.reset();
  for (int e = 0; e < 3; ++e) {
    const float* p = t + 3 * e;
    const float* q = t + 3 * ((e + 1) % 3);
    const float pa = p[axis], qa = q[axis];
    if (pa >= lo && pa <= hi) r.growP(p);
    const float planes[2] = {lo, hi};
    for (float pl : planes) {
      if ((pa < pl && qa > pl) || (pa > pl && qa < pl)) {
        const double tt = ((double)pl - pa) / ((double)qa - pa);
        float x[3];
        for (int k = 0; k < 3; ++k) x[k] = (float)(p[k] + tt * ((double)q[k] - p[k]));
        x[axis] = pl;
        r.growP(x);
      }
    }
  }
  for (int k = 0; k < 3; ++k) {
    if (k == axis || !(r.hi[k] >= r.lo[k])) continue;
    const float pad = 4.0f * FLT_EPSILON * std::max(fabsf(r.lo[k]), fabsf(r.hi[k]));
    r.lo[k] -= pad;
    r.hi[k] += pad;
  }
  return r;
}

Box intersect(const Box& a, const Box& b) {
  Box r;
  for (int k = 0; k < 3; ++k) {
    r.lo[k] = std::max(a.lo[k], b.lo[k]);
    r.hi[k] = std::min(a.hi[k], b.hi[k]);
  }
  return r;
}

struct SplitBuilder {
  const std::vector<float>& v;
  std::vector<Node2> nodes;
  std::vector<int> leafIds;  // leaf ranges index this (global triangle ids, duplicates allowed)
  int maxLeaf = YRT_MAX_LEAF;
  int medianDepth = 24;
  float minOverlap = 0.f;
  size_t refBudget = 0, numRefs = 0;
  explicit SplitBuilder(const std::vector<float>& verts) : v(verts) {}

  static Box bounds(const std::vector<SRef>& r) {
    Box bb;
    bb.reset();
    for (const SRef& x : r) bb.grow(x.b);
    return bb;
  }

  void leaf(std::vector<SRef>& refs, int& idx, int& cnt) {
    idx = (int)leafIds.size();
    cnt = (int)refs.size();
    for (const SRef& x : refs) leafIds.push_back(x.id);
  }

  // Builds the subtree of `refs` (consumed); returns the child reference and its box.
  void child(std::vector<SRef>& refs, int depth, int& idx, int& cnt, Box& bb) {
    bb = bounds(refs);
    const int n = (int)refs.size();
    if (n <= 2) { leaf(refs, idx, cnt); return; }
    std::vector<SRef> L, R;
    const bool mkLeaf = split(refs, bb, depth, L, R);
    if (mkLeaf && n <= 31) { leaf(refs, idx, cnt); return; }
    if (mkLeaf) median(refs, bb, L, R);
    std::vector<SRef>().swap(refs);
    idx = inner(L, R, depth);
    cnt = 0;
  }

  int inner(std::vector<SRef>& L, std::vector<SRef>& R, int depth) {
    const int ni = (int)nodes.size();
    nodes.emplace_back();
    int i0, c0, i1, c1;
    Box b0, b1;
    child(L, depth + 1, i0, c0, b0);
    child(R, depth + 1, i1, c1, b1);
    Node2& nd = nodes[ni];
    nd.b[0] = b0;
    nd.b[1] = b1;
    nd.idx[0] = i0; nd.idx[1] = i1;
    nd.cnt[0] = c0; nd.cnt[1] = c1;
    return ni;
  }

  void median(std::vector<SRef>& refs, const Box& bb, std::vector<SRef>& L, std::vector<SRef>& R) {
    int axis = 0;
    for (int k = 1; k < 3; ++k)
      if (bb.hi[k] - bb.lo[k] > bb.hi[axis] - bb.lo[axis]) axis = k;
    const size_t m = refs.size() / 2;
    std::nth_element(refs.begin(), refs.begin() + m, refs.end(),
                     [axis](const SRef& x, const SRef& y) { return x.c(axis) < y.c(axis); });
    L.assign(refs.begin(), refs.begin() + m);
    R.assign(refs.begin() + m, refs.end());
  }

  // Chooses leaf / object split / spatial split; fills L, R unless a leaf is chosen.
  bool split(std::vector<SRef>& refs, const Box& nodeBox, int depth, std::vector<SRef>& L, std::vector<SRef>& R) {
    const int n = (int)refs.size();
    Box cb;
    cb.reset();
    for (const SRef& x : refs) {
      const float c[3] = {x.c(0), x.c(1), x.c(2)};
      cb.growP(c);
    }
    if (depth >= medianDepth) {
      median(refs, cb, L, R);
      return false;
    }
    const int NB = 32;
    // object split
    float objCost = INFINITY;
    int objAxis = -1, objBin = -1;
    Box objL, objR;
    for (int ax = 0; ax < 3; ++ax) {
      const float lo = cb.lo[ax], hi = cb.hi[ax];
      if (!(hi > lo)) continue;
      const float scale = NB / (hi - lo);
      Box bb[NB];
      int cnt[NB] = {0};
      for (int k = 0; k < NB; ++k) bb[k].reset();
      for (const SRef& x : refs) {
        const int bin = std::min(NB - 1, (int)((x.c(ax) - lo) * scale));
        cnt[bin]++;
        bb[bin].grow(x.b);
      }
      Box rightBox[NB];
      int rightCnt[NB];
      Box acc;
      acc.reset();
      int ac = 0;
      for (int k = NB - 1; k > 0; --k) {
        acc.grow(bb[k]);
        ac += cnt[k];
        rightBox[k] = acc;
        rightCnt[k] = ac;
      }
      acc.reset();
      ac = 0;
      for (int k = 0; k < NB - 1; ++k) {
        acc.grow(bb[k]);
        ac += cnt[k];
        if (ac == 0 || rightCnt[k + 1] == 0) continue;
        const float cost = acc.area() * ac + rightBox[k + 1].area() * rightCnt[k + 1];
        if (cost < objCost) {
          objCost = cost; objAxis = ax; objBin = k; objL = acc; objR = rightBox[k + 1];
        }
      }
    }
    // spatial split, where the object split's children overlap
    float spCost = INFINITY;
    int spAxis = -1, spBin = -1;
    const float overlap = objAxis >= 0 ? intersect(objL, objR).area() : INFINITY;
    if (numRefs < refBudget && overlap > minOverlap) {
      for (int ax = 0; ax < 3; ++ax) {
        const float lo = nodeBox.lo[ax], hi = nodeBox.hi[ax];
        if (!(hi > lo)) continue;
        const float w = (hi - lo) / NB;
        Box bb[NB];
        int enter[NB] = {0}, exit[NB] = {0};
        for (int k = 0; k < NB; ++k) bb[k].reset();
        for (const SRef& x : refs) {
          const int b0 = std::max(0, std::min(NB - 1, (int)((x.b.lo[ax] - lo) / w)));
          const int b1 = std::max(b0, std::min(NB - 1, (int)((x.b.hi[ax] - lo) / w)));
          enter[b0]++;
          exit[b1]++;
          if (b0 == b1) {
            bb[b0].grow(x.b);
            continue;
          }
          const float* t = &v[(size_t)x.id * 9];
          for (int k = b0; k <= b1; ++k) {
            const float s0 = k == b0 ? x.b.lo[ax] : lo + k * w;
            const float s1 = k == b1 ? x.b.hi[ax] : lo + (k + 1) * w;
            const Box cbx = intersect(clip_tri(t, ax, s0, s1), x.b);
            if (cbx.hi[0] >= cbx.lo[0] && cbx.hi[1] >= cbx.lo[1] && cbx.hi[2] >= cbx.lo[2]) bb[k].grow(cbx);
          }
        }
        Box rightBox[NB];
        int rightCnt[NB];
        Box acc;
        acc.reset();
        int ac = 0;
        for (int k = NB - 1; k > 0; --k) {
          acc.grow(bb[k]);
          ac += exit[k];
          rightBox[k] = acc;
          rightCnt[k] = ac;
        }
        acc.reset();
        ac = 0;
        for (int k = 0; k < NB - 1; ++k) {
          acc.grow(bb[k]);
          ac += enter[k];
          if (ac == 0 || rightCnt[k + 1] == 0) continue;
          const float cost = acc.area() * ac + rightBox[k + 1].area() * rightCnt[k + 1];
          if (cost < spCost) { spCost = cost; spAxis = ax; spBin = k; }
        }
      }
    }
    const float parentArea = nodeBox.area();
    const float best = std::min(objCost, spCost);
    const float splitCost = YRT_SAH_TRAV + (parentArea > 0.f ? best / parentArea : (float)n);
    if (n <= maxLeaf && (float)n <= splitCost) return true;
    if (objAxis < 0 && spAxis < 0) return true;  // caller falls back to a median split
    if (spAxis >= 0 && spCost < objCost) {
      const float lo = nodeBox.lo[spAxis], w = (nodeBox.hi[spAxis] - lo) / NB;
      const float plane = lo + (spBin + 1) * w;
      for (const SRef& x : refs) {
        if (x.b.hi[spAxis] <= plane) { L.push_back(x); continue; }
        if (x.b.lo[spAxis] >= plane) { R.push_back(x); continue; }
        const float* t = &v[(size_t)x.id * 9];
        const Box bl = intersect(clip_tri(t, spAxis, x.b.lo[spAxis], plane), x.b);
        const Box br = intersect(clip_tri(t, spAxis, plane, x.b.hi[spAxis]), x.b);
        const bool okL = bl.hi[0] >= bl.lo[0] && bl.hi[1] >= bl.lo[1] && bl.hi[2] >= bl.lo[2];
        const bool okR = br.hi[0] >= br.lo[0] && br.hi[1] >= br.lo[1] && br.hi[2] >= br.lo[2];
        if (okL) L.push_back(SRef{bl, x.id});
        if (okR) R.push_back(SRef{br, x.id});
        if (!okL && !okR) (x.c(spAxis) < plane ? L : R).push_back(x);  // degenerate clip: keep whole
        if (okL && okR) numRefs++;
      }
      if (!L.empty() && !R.empty()) return false;
      // degenerate (everything on one side): fall back to the object split
      refs.clear();
      for (auto* side : {&L, &R})
        for (const SRef& x : *side) refs.push_back(x);
      L.clear();
      R.clear();
      if (objAxis < 0) return true;
    }
    const float lo = cb.lo[objAxis], scale = NB / (cb.hi[objAxis] - lo);
    for (const SRef& x : refs)
      (std::min(NB - 1, (int)((x.c(objAxis) - lo) * scale)) <= objBin ? L : R).push_back(x);
    if (L.empty() || R.empty()) {
      L.clear();
      R.clear();
      return true;
    }
    return false;
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
    // empty slots get an inverted infinite box (lo = +inf, hi = -inf): with sign-ordered slab
    // planes its entry distance is +inf and its exit -inf for every ray, so the kernel culls
    // it without testing the child reference (which stays -1 for the other traversals)
    for (int j = 0; j < 4; ++j) {
      const bool v = j < k;
      const float L = INFINITY, H = -INFINITY;
      g.lox[j] = v ? ch[j].b.lo[0] : L; g.hix[j] = v ? ch[j].b.hi[0] : H;
      g.loy[j] = v ? ch[j].b.lo[1] : L; g.hiy[j] = v ? ch[j].b.hi[1] : H;
      g.loz[j] = v ? ch[j].b.lo[2] : L; g.hiz[j] = v ? ch[j].b.hi[2] : H;
      g.child[j] = refs[j];
    }
    return ni;
  }
};

}  // namespace

void build_bvh(const std::vector<float>& v /* 9 floats per triangle */, const std::vector<uint32_t>& flags,
               int stackDepth, BvhResult& out, const std::vector<float>* v1) {
  const int N = (int)(v.size() / 9);
  out.nodes.clear();
  out.tris.clear();
  out.order.clear();
  if (N == 0) return;
  // A BVH2 path of depth D collapses to about D/2 four-wide levels of <= 3 pushes each.
  const int levels = (int)ceil(log2(std::max(1.0, N / 16.0)));
  const int medianDepth = std::max(0, std::min(28, (2 * stackDepth) / 3 - 2 - levels));
  std::vector<Node2> nodes2;
  std::vector<int> leafIds;  // leaf slot -> global triangle id
  // spatial splits are opt-in (YRT_SBVH=1): on the measured scenes (C2-C4 stand-ins) they cut
  // node visits by < 1 % for 2-5x the build time
  const char* env = getenv("YRT_SBVH");
  const bool spatial = env && atoi(env) != 0 && !v1;  // spatial splits clip static triangles only
  if (N == 1) {
    Node2 n;
    n.b[0].reset();
    for (int k = 0; k < 3; ++k) n.b[0].growP(&v[3 * k]);
    if (v1)
      for (int k = 0; k < 3; ++k) n.b[0].growP(&(*v1)[3 * k]);
    n.b[1] = n.b[0];
    n.idx[0] = 0; n.cnt[0] = 1;
    n.idx[1] = 0; n.cnt[1] = 1;
    nodes2.push_back(n);
    leafIds.push_back(0);
  } else if (spatial) {
    SplitBuilder B(v);
    B.medianDepth = medianDepth;
    std::vector<SRef> refs(N);
    for (int i = 0; i < N; ++i) {
      refs[i].b.reset();
      for (int k = 0; k < 3; ++k) refs[i].b.growP(&v[(size_t)i * 9 + 3 * k]);
      refs[i].id = i;
    }
    const Box root = SplitBuilder::bounds(refs);
    B.minOverlap = YRT_SBVH_ALPHA * root.area();
    B.numRefs = (size_t)N;
    B.refBudget = (size_t)(N * (1.0 + YRT_SBVH_BUDGET));
    std::vector<SRef> L, R;
    bool leaf = B.split(refs, root, 0, L, R);
    if (leaf) B.median(refs, root, L, R);
    std::vector<SRef>().swap(refs);
    B.inner(L, R, 0);
    nodes2 = std::move(B.nodes);
    leafIds = std::move(B.leafIds);
  } else {
    Builder B;
    B.medianDepth = medianDepth;
    B.prims.resize(N);
    for (int i = 0; i < N; ++i) {
      Prim& p = B.prims[i];
      p.b.reset();
      for (int k = 0; k < 3; ++k) p.b.growP(&v[(size_t)i * 9 + 3 * k]);
      if (v1)
        for (int k = 0; k < 3; ++k) p.b.growP(&(*v1)[(size_t)i * 9 + 3 * k]);
      for (int k = 0; k < 3; ++k) p.c[k] = 0.5f * (p.b.lo[k] + p.b.hi[k]);
      p.id = i;
    }
    bool leaf = false;
    int m = B.split(0, N, 0, leaf);
    if (leaf || m <= 0 || m >= N) m = N / 2;
    B.inner(0, m, N, 0);
    nodes2 = std::move(B.nodes);
    leafIds.resize(N);
    for (int i = 0; i < N; ++i) leafIds[i] = B.prims[i].id;
  }
  Collapser C(nodes2);
  C.collapse(0, 0);
  out.maxDepth = C.maxStack;
  if (C.maxStack > stackDepth - 1)
    throw std::runtime_error("BVH traversal stack bound exceeds YRT_STACK_DEPTH");
  // child references pack (index << 5) | count into an int and the traversal addresses a node
  // as (index << 7) bytes in 32 bits (kernels/yrt_traverse.h box4_ordered): bound both
  if (C.out.size() >= (size_t(1) << 25))
    throw std::runtime_error("BVH exceeds 2^25 nodes (32-bit node byte offsets)");
  if (leafIds.size() >= (size_t(1) << 26))
    throw std::runtime_error("BVH exceeds 2^26 leaf triangle references (child reference packing)");
  out.nodes = std::move(C.out);
  const size_t S = leafIds.size();
  out.order = leafIds;
  out.tris.resize(S);
  for (size_t i = 0; i < S; ++i) {
    const int id = leafIds[i];
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
