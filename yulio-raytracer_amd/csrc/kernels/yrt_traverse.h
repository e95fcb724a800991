// yrt_traverse.h — BVH2 traversal + Embree-convention triangle test, device side.
//
// Replaces Embree 2.15 rtcIntersect / rtcOccluded (call sites
// integrators/pathtraceintegrator.cpp:72,160, renderers/debugrenderer.cpp:109).
//
// Hit convention (restated from the in-tree copy lights/trianglelight.h:55-65 and the
// rtcore triangle layout; Embree itself is binary-only so this is "parity unpinned"
// against Embree and pinned against oracle/):
//   e1 = v0-v1, e2 = v2-v0, Ng = cross(e1,e2), C = v0-O, R = cross(D,C)
//   den = dot(Ng,D), U = dot(R,e2)*sgn(den), V = dot(R,e1)*sgn(den), T = dot(Ng,C)*sgn(den)
//   valid: den != 0, U >= 0, V >= 0, U+V <= |den|, tnear < t=T/|den| < tfar
//   back-face filter (cullBackFaces meshes, shapes/trianglemesh_full.cpp:86-106): reject den <= 0
//   closest hit: smallest (t, global triangle id) — order independent, so any BVH gives
//   the same answer (used to pin the GPU against the oracle's own BVH).
// Stack: per-lane short stack in LDS, [depth][lane] so a wave's pushes hit 64 distinct
// banks. Only YRT_LDS_STACK entries live in LDS (16 x 256 B per wave keeps LDS from capping
// occupancy below the VGPR limit); deeper entries, rare, spill to a per-lane scratch array.
// The builder bounds the tree depth to YRT_STACK_DEPTH-1 (device/bvh_build.cpp).
#pragma once

#include "../common/yrt_gpu_types.h"
#include "../common/yrt_math.h"

#ifndef YRT_STACK_DEPTH
#define YRT_STACK_DEPTH 64   // bound on BVH depth + 1 (device/bvh_build.cpp enforces it)
#endif
#ifndef YRT_LDS_STACK
#define YRT_LDS_STACK 16     // top entries kept in LDS; deeper ones spill (power of two)
#endif
static_assert((YRT_LDS_STACK & (YRT_LDS_STACK - 1)) == 0, "YRT_LDS_STACK must be a power of two");
#define YRT_TRACE_BLOCK 128

namespace yrt {

struct Hit {
  float t, u, v;
  int tri;  // global triangle id, -1 = miss
};

// Conservative slab factor 1 + 2*gamma(3) (robust box test; Embree flags ROBUST,
// api/scene_flat.h:75-80).
#define YRT_BOX_ROBUST 1.00000036f

__device__ __forceinline__ float safe_inv(float d) {
  return 1.0f / (fabsf(d) > 1e-20f ? d : copysignf(1e-20f, d));
}

struct RayPre {
  V3 org, dir, inv;
  float tnear, tfar;
};

__device__ __forceinline__ void box2(const GpuNode& n, const RayPre& r, float tmax, bool& h0, bool& h1,
                                     float& t0, float& t1) {
  // child 0
  float lx0 = (n.b0[0] - r.org.x) * r.inv.x, hx0 = (n.b0[1] - r.org.x) * r.inv.x;
  float ly0 = (n.b0[2] - r.org.y) * r.inv.y, hy0 = (n.b0[3] - r.org.y) * r.inv.y;
  float lz0 = (n.b2[0] - r.org.z) * r.inv.z, hz0 = (n.b2[1] - r.org.z) * r.inv.z;
  float lx1 = (n.b1[0] - r.org.x) * r.inv.x, hx1 = (n.b1[1] - r.org.x) * r.inv.x;
  float ly1 = (n.b1[2] - r.org.y) * r.inv.y, hy1 = (n.b1[3] - r.org.y) * r.inv.y;
  float lz1 = (n.b2[2] - r.org.z) * r.inv.z, hz1 = (n.b2[3] - r.org.z) * r.inv.z;
  float n0 = fmaxf(fmaxf(fminf(lx0, hx0), fminf(ly0, hy0)), fmaxf(fminf(lz0, hz0), r.tnear));
  float f0 = fminf(fminf(fmaxf(lx0, hx0), fmaxf(ly0, hy0)), fminf(fmaxf(lz0, hz0), tmax));
  float n1 = fmaxf(fmaxf(fminf(lx1, hx1), fminf(ly1, hy1)), fmaxf(fminf(lz1, hz1), r.tnear));
  float f1 = fminf(fminf(fmaxf(lx1, hx1), fmaxf(ly1, hy1)), fminf(fmaxf(lz1, hz1), tmax));
  h0 = n0 <= f0 * YRT_BOX_ROBUST;
  h1 = n1 <= f1 * YRT_BOX_ROBUST;
  t0 = n0;
  t1 = n1;
}

// One triangle; returns true and t when the ray hits within (tnear, tfar). U, V, absDen are
// returned undivided: u = U/absDen, v = V/absDen are only needed for an accepted hit.
__device__ __forceinline__ bool tri_test_t(const GpuTri& tr, const RayPre& r, float tfar, float& t, float& U_,
                                           float& V_, float& absDen_) {
  V3 v0 = v3(tr.v0[0], tr.v0[1], tr.v0[2]);
  V3 e1 = v3(tr.e1[0], tr.e1[1], tr.e1[2]);
  V3 e2 = v3(tr.e2[0], tr.e2[1], tr.e2[2]);
  V3 Ng = cross(e1, e2);
  V3 C = v0 - r.org;
  V3 R = cross(r.dir, C);
  float den = dot(Ng, r.dir);
  float absDen = fabsf(den);
  float sgn = den < 0.0f ? -1.0f : 1.0f;
  float U = dot(R, e2) * sgn;
  float V = dot(R, e1) * sgn;
  bool ok = (den != 0.0f) & (U >= 0.0f) & (V >= 0.0f) & (U + V <= absDen);
  int flags = __float_as_int(tr.e1[3]);
  ok &= !((flags & 1) && !(den > 0.0f));
  float T = dot(Ng, C) * sgn;
  t = T / absDen;
  ok &= (t > r.tnear) & (t < tfar);
  U_ = U;
  V_ = V;
  absDen_ = absDen;
  return ok;
}

template <bool ANY>
__device__ __forceinline__ Hit traverse(const GpuNode* __restrict__ nodes, const GpuTri* __restrict__ tris,
                                        const RayPre& r, int* __restrict__ stack /* LDS, this lane's column */) {
  Hit best;
  best.t = r.tfar;
  best.u = best.v = 0.0f;
  best.tri = -1;
  // NaN tfar (tMaxShadowRay = inf): every comparison is false, no hit.
  if (!(r.tfar >= r.tnear)) return best;
  int sp = 0;
  int spill[YRT_STACK_DEPTH > YRT_LDS_STACK ? YRT_STACK_DEPTH - YRT_LDS_STACK : 1];
  // stack entry: (index << 5) | count — count 0 => inner node, 1..31 => leaf range
  int curIdx = 0, curCnt = 0;
  while (true) {
    if (curCnt == 0) {
      const GpuNode n = nodes[curIdx];
      bool h0, h1;
      float t0, t1;
      box2(n, r, best.t, h0, h1, t0, t1);
      if (h0 && h1) {
        bool swap = t1 < t0;
        int nearI = swap ? n.c[1] : n.c[0], nearC = swap ? n.c[3] : n.c[2];
        int farI = swap ? n.c[0] : n.c[1], farC = swap ? n.c[2] : n.c[3];
        const int e = (farI << 5) | farC;
        if (sp < YRT_LDS_STACK) stack[sp * YRT_TRACE_BLOCK] = e;
        else spill[sp - YRT_LDS_STACK] = e;
        sp += 1;
        curIdx = nearI;
        curCnt = nearC;
        continue;
      } else if (h0 || h1) {
        curIdx = h0 ? n.c[0] : n.c[1];
        curCnt = h0 ? n.c[2] : n.c[3];
        continue;
      }
    } else {
      for (int i = 0; i < curCnt; ++i) {
        const GpuTri tr = tris[curIdx + i];
        float t, U, V, absDen;
        bool ok = tri_test_t(tr, r, ANY ? r.tfar : best.t + 0.0f, t, U, V, absDen);
        int gid = __float_as_int(tr.v0[3]);
        if (ANY) {
          if (ok) {
            best.t = t; best.u = U / absDen; best.v = V / absDen; best.tri = gid;
            return best;
          }
        } else {
          // strict (t < best) or tie with smaller id; tri_test used tfar = best.t so ties
          // (t == best.t) were rejected: re-test them against the original tfar.
          if (!ok && best.tri >= 0 && t == best.t && gid < best.tri) {
            float t2, U2, V2, a2;
            ok = tri_test_t(tr, r, r.tfar, t2, U2, V2, a2);
          }
          if (ok) {
            best.t = t; best.u = U / absDen; best.v = V / absDen; best.tri = gid;
          }
        }
      }
    }
    if (sp == 0) break;
    sp -= 1;
    const int e = sp < YRT_LDS_STACK ? stack[sp * YRT_TRACE_BLOCK] : spill[sp - YRT_LDS_STACK];
    curIdx = e >> 5;
    curCnt = e & 31;
  }
  return best;
}

}  // namespace yrt
