/* occluder_cache_exp.c — CPU experiment: any-hit traversal on the device BVH4 (farthest hit
 * child first, as k_trace<true>) of a captured shadow stream in queue order, recording per
 * query the node and triangle visits and the leaf slot of the occluder it finds. The driver
 * (tools/occluder_cache_exp.py) then prices testing a cached candidate triangle first (the
 * boolean result does not depend on which occluder is found).
 * Build: gcc -O2 -shared -fPIC -o /tmp/oce.so tools/occluder_cache_exp.c -lm */
#include <math.h>
#include <stdint.h>
#include <string.h>

typedef struct { float lox[4], hix[4], loy[4], hiy[4], loz[4], hiz[4]; int32_t child[4], pad[4]; } DNode;
typedef struct { float v0[4], e1[4], e2[4]; } DTri;

static float safe_inv(float d) { return 1.0f / (fabsf(d) > 1e-20f ? d : copysignf(1e-20f, d)); }

static int tri_test(const DTri* t, const float o[3], const float d[3], float tnear, float tfar) {
  const float v0[3] = {t->v0[0], t->v0[1], t->v0[2]}, e1[3] = {t->e1[0], t->e1[1], t->e1[2]},
              e2[3] = {t->e2[0], t->e2[1], t->e2[2]};
  const float Ng[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
  const float C[3] = {v0[0] - o[0], v0[1] - o[1], v0[2] - o[2]};
  const float R[3] = {d[1] * C[2] - d[2] * C[1], d[2] * C[0] - d[0] * C[2], d[0] * C[1] - d[1] * C[0]};
  const float den = Ng[0] * d[0] + Ng[1] * d[1] + Ng[2] * d[2];
  const float ad = fabsf(den), sg = den < 0 ? -1.f : 1.f;
  const float U = (R[0] * e2[0] + R[1] * e2[1] + R[2] * e2[2]) * sg;
  const float V = (R[0] * e1[0] + R[1] * e1[1] + R[2] * e1[2]) * sg;
  int ok = den != 0 && U >= 0 && V >= 0 && U + V <= ad;
  uint32_t fl;
  memcpy(&fl, &t->e1[3], 4);
  if ((fl & 1) && !(den > 0)) ok = 0;
  const float T = (Ng[0] * C[0] + Ng[1] * C[1] + Ng[2] * C[2]) * sg;
  const float tt = T / ad;
  return ok && tt > tnear && tt < tfar;
}

/* per query: visits[2*i] nodes, visits[2*i+1] triangles, occ[i] occluder leaf slot or -1 */
void any_hit(const void* nodes_, const void* tris_, const float* org4, const float* dir4, int n, int* visits,
             int* occ) {
  const DNode* nodes = (const DNode*)nodes_;
  const DTri* tris = (const DTri*)tris_;
  for (int i = 0; i < n; ++i) {
    const float o[3] = {org4[4 * i], org4[4 * i + 1], org4[4 * i + 2]};
    const float d[3] = {dir4[4 * i], dir4[4 * i + 1], dir4[4 * i + 2]};
    const float tnear = org4[4 * i + 3], tfar = dir4[4 * i + 3];
    int nv = 0, tv = 0, found = -1;
    occ[i] = -1;
    if (!(tfar >= tnear)) { visits[2 * i] = visits[2 * i + 1] = 0; continue; }
    const float iv[3] = {safe_inv(d[0]), safe_inv(d[1]), safe_inv(d[2])};
    const float oi[3] = {o[0] * iv[0], o[1] * iv[1], o[2] * iv[2]};
    const float margin = fmaxf(fmaxf(fabsf(oi[0]), fabsf(oi[1])), fabsf(oi[2])) * 2.384185791015625e-07f;
    int stack[256], sp = 0, cur = 0;
    for (;;) {
      if ((cur & 31) == 0) {
        const DNode* nd = &nodes[cur >> 5];
        nv++;
        float t[4];
        int c[4];
        for (int k = 0; k < 4; ++k) {
          const float lo[3] = {nd->lox[k], nd->loy[k], nd->loz[k]}, hi[3] = {nd->hix[k], nd->hiy[k], nd->hiz[k]};
          float l[3], h[3];
          for (int a = 0; a < 3; ++a) { l[a] = fmaf(lo[a], iv[a], -oi[a]); h[a] = fmaf(hi[a], iv[a], -oi[a]); }
          const float a0 = fmaxf(fmaxf(fminf(l[0], h[0]), fminf(l[1], h[1])), fmaxf(fminf(l[2], h[2]), tnear));
          const float b0 = fminf(fminf(fmaxf(l[0], h[0]), fmaxf(l[1], h[1])), fminf(fmaxf(l[2], h[2]), tfar));
          const int hit = a0 <= fmaf(b0, 1.0000152587890625f, margin) && nd->child[k] != -1;
          t[k] = hit ? a0 : -INFINITY;
          c[k] = nd->child[k];
        }
        static const int net[3][2] = {{0, 1}, {2, 3}, {0, 2}};  /* farthest first */
        for (int m = 0; m < 3; ++m) {
          const int a = net[m][0], b = net[m][1];
          if (t[b] > t[a]) { float tt = t[a]; t[a] = t[b]; t[b] = tt; int cc = c[a]; c[a] = c[b]; c[b] = cc; }
        }
        for (int k = 3; k >= 1; --k) if (t[k] > -INFINITY) stack[sp++] = c[k];
        if (t[0] > -INFINITY) { cur = c[0]; continue; }
      } else {
        const int base = cur >> 5, cnt = cur & 31;
        for (int k = 0; k < cnt; ++k) {
          tv++;
          if (tri_test(&tris[base + k], o, d, tnear, tfar)) { found = base + k; break; }
        }
        if (found >= 0) break;
      }
      if (sp == 0) break;
      cur = stack[--sp];
    }
    visits[2 * i] = nv;
    visits[2 * i + 1] = tv;
    occ[i] = found;
  }
}

/* 1 if leaf slot `slot` occludes query i */
void test_slots(const void* tris_, const float* org4, const float* dir4, int n, const int* slot, int* out) {
  const DTri* tris = (const DTri*)tris_;
  for (int i = 0; i < n; ++i) {
    out[i] = 0;
    if (slot[i] < 0) continue;
    const float o[3] = {org4[4 * i], org4[4 * i + 1], org4[4 * i + 2]};
    const float d[3] = {dir4[4 * i], dir4[4 * i + 1], dir4[4 * i + 2]};
    out[i] = tri_test(&tris[slot[i]], o, d, org4[4 * i + 3], dir4[4 * i + 3]);
  }
}
