/* bvh8_visits_exp.c — CPU experiment: node / triangle visits per any-hit (shadow) query on the
 * device's 4-wide BVH (farthest hit child first, the others in slot order: k_trace<true>'s
 * sort3_far) against the 8-wide BVH collapsed from it by the product's rule
 * (bvh_build.cpp collapse_bvh8: open the largest-area inner child while <= 8 children) with
 * the farthest hit child first (far8). The occlusion answer is order independent.
 * Build: gcc -O2 -shared -fPIC -o /tmp/b8v.so tools/bvh8_visits_exp.c -lm
 * Driven by tools/bvh8_visits_exp.py on gpurun_out/shadow_c3.npz (tools/dump_shadow_stream.py). */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { float lox[4], hix[4], loy[4], hiy[4], loz[4], hiz[4]; int32_t child[4], pad[4]; } N4;
typedef struct { float lo[3][8], hi[3][8]; int32_t child[8]; int n; } N8;
typedef struct { float v0[4], e1[4], e2[4]; } Tri;

static float safe_inv(float d) { return 1.0f / (fabsf(d) > 1e-20f ? d : copysignf(1e-20f, d)); }

static int tri_hit(const Tri* t, const float o[3], const float d[3], float tnear, float tfar) {
  const float* v0 = t->v0; const float* e1 = t->e1; const float* e2 = t->e2;
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

/* entry distance of a box (-INF when missed), the kernel's robust slab test */
static float box_t(const float lo[3], const float hi[3], const float o[3], const float inv[3], float tnear, float tfar) {
  float nn = tnear, ff = tfar;
  for (int a = 0; a < 3; ++a) {
    const float t0 = (lo[a] - o[a]) * inv[a], t1 = (hi[a] - o[a]) * inv[a];
    nn = fmaxf(nn, fminf(t0, t1));
    ff = fminf(ff, fmaxf(t0, t1));
  }
  return nn <= ff * 1.0000152587890625f ? nn : -INFINITY;
}

/* ---- collapse 4 -> 8 (bvh_build.cpp Collapser8) */
static const N4* g4;
static N8* g8;
static int n8, cap8;
static float area4(int n, int s) {
  const N4* g = &g4[n];
  const float dx = g->hix[s] - g->lox[s], dy = g->hiy[s] - g->loy[s], dz = g->hiz[s] - g->loz[s];
  return dx * dy + dy * dz + dz * dx;
}
static int valid4(int n) {
  int m = 0;
  for (int j = 0; j < 4; ++j) m += g4[n].child[j] != -1;
  return m;
}
static int collapse(int n4) {
  int cn[8], cs[8], k = 0;
  for (int j = 0; j < 4; ++j)
    if (g4[n4].child[j] != -1) { cn[k] = n4; cs[k] = j; ++k; }
  for (;;) {
    int best = -1;
    float ba = -1.f;
    for (int i = 0; i < k; ++i) {
      const int r = g4[cn[i]].child[cs[i]];
      if ((r & 31) != 0) continue;
      if (k - 1 + valid4(r >> 5) > 8) continue;
      if (area4(cn[i], cs[i]) > ba) { ba = area4(cn[i], cs[i]); best = i; }
    }
    if (best < 0) break;
    const int c = g4[cn[best]].child[cs[best]] >> 5;
    int first = 1;
    for (int j = 0; j < 4; ++j) {
      if (g4[c].child[j] == -1) continue;
      if (first) { cn[best] = c; cs[best] = j; first = 0; }
      else { cn[k] = c; cs[k] = j; ++k; }
    }
  }
  if (n8 == cap8) { cap8 = cap8 ? 2 * cap8 : 1024; g8 = realloc(g8, (size_t)cap8 * sizeof(N8)); }
  const int ni = n8++;
  int refs[8];
  for (int i = 0; i < k; ++i) {
    const int r = g4[cn[i]].child[cs[i]];
    refs[i] = (r & 31) == 0 ? collapse(r >> 5) << 5 : r;
  }
  N8* g = &g8[ni];
  g->n = k;
  for (int i = 0; i < 8; ++i) {
    const int v = i < k;
    const N4* s = v ? &g4[cn[i]] : 0;
    const int q = v ? cs[i] : 0;
    g->lo[0][i] = v ? s->lox[q] : INFINITY; g->hi[0][i] = v ? s->hix[q] : -INFINITY;
    g->lo[1][i] = v ? s->loy[q] : INFINITY; g->hi[1][i] = v ? s->hiy[q] : -INFINITY;
    g->lo[2][i] = v ? s->loz[q] : INFINITY; g->hi[2][i] = v ? s->hiz[q] : -INFINITY;
    g->child[i] = v ? refs[i] : -1;
  }
  return ni;
}

/* out[0] = 4-wide node visits, out[1] tri tests, out[2] 8-wide node visits, out[3] tri tests,
 * out[4] occlusion disagreements (must be 0), out[5] 8-wide nodes, out[6] mean 8-wide children */
int bvh8_visits(const N4* nodes, int numNodes, const Tri* tris, const float* org4, const float* dir4, int n,
                double* out) {
  (void)numNodes;
  g4 = nodes; n8 = 0;
  collapse(0);
  double cn = 0;
  for (int i = 0; i < n8; ++i) cn += g8[i].n;
  memset(out, 0, 7 * sizeof(double));
  out[5] = n8; out[6] = cn / n8;
  int st[256];
  for (int r = 0; r < n; ++r) {
    const float* O = org4 + 4 * r; const float* D = dir4 + 4 * r;
    const float o[3] = {O[0], O[1], O[2]}, d[3] = {D[0], D[1], D[2]};
    const float inv[3] = {safe_inv(d[0]), safe_inv(d[1]), safe_inv(d[2])};
    const float tn = O[3], tf = D[3];
    int occ[2] = {0, 0};
    if (!(tf >= tn)) continue;
    for (int w = 0; w < 2; ++w) {
      int sp = 0, cur = 0;
      for (;;) {
        if ((cur & 31) == 0) {
          out[w * 2] += 1;
          float t[8]; int c[8]; int k = w ? 8 : 4;
          for (int j = 0; j < k; ++j) {
            float lo[3], hi[3];
            if (w) { for (int a = 0; a < 3; ++a) { lo[a] = g8[cur >> 5].lo[a][j]; hi[a] = g8[cur >> 5].hi[a][j]; } c[j] = g8[cur >> 5].child[j]; }
            else {
              const N4* g = &g4[cur >> 5];
              lo[0] = g->lox[j]; lo[1] = g->loy[j]; lo[2] = g->loz[j]; hi[0] = g->hix[j]; hi[1] = g->hiy[j]; hi[2] = g->hiz[j];
              c[j] = g->child[j];
            }
            t[j] = c[j] == -1 ? -INFINITY : box_t(lo, hi, o, inv, tn, tf);
          }
          /* farthest to slot 0 by the kernel's comparator networks */
#define SW(a, b) do { if (t[b] > t[a]) { float x = t[a]; t[a] = t[b]; t[b] = x; int y = c[a]; c[a] = c[b]; c[b] = y; } } while (0)
          if (w) { SW(0, 1); SW(2, 3); SW(4, 5); SW(6, 7); SW(0, 2); SW(4, 6); SW(0, 4); }
          else if (getenv("B8V_FULLSORT")) { SW(0, 1); SW(2, 3); SW(0, 2); SW(1, 3); SW(1, 2); }
          else { SW(0, 1); SW(2, 3); SW(0, 2); }
#undef SW
          for (int j = k - 1; j >= 1; --j)
            if (t[j] > -INFINITY) st[sp++] = c[j];
          if (t[0] > -INFINITY) { cur = c[0]; continue; }
        } else {
          const int idx = cur >> 5, cnt = cur & 31;
          int hit = 0;
          for (int i = 0; i < cnt && !hit; ++i) {
            out[w * 2 + 1] += 1;
            hit = tri_hit(&tris[idx + i], o, d, tn, tf);
          }
          if (hit) { occ[w] = 1; break; }
        }
        if (sp == 0) break;
        cur = st[--sp];
      }
    }
    if (occ[0] != occ[1]) out[4] += 1;
  }
  for (int k = 0; k < 4; ++k) out[k] /= n;
  return 0;
}
