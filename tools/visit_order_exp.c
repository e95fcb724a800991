/* visit_order_exp.c — CPU experiment: node/triangle visits per query on the device BVH4 for
 * several child orders (the hit result is order independent; only the work changes).
 *   0 distance  : sort hit children by entry distance (k_trace<false> today)
 *   1 octant    : per node and ray octant, children ordered by their box centres projected
 *                 on the octant diagonal (precomputed, no per-step sort)
 *   2 slot      : builder slot order (k_trace<true> today)
 * Build: gcc -O2 -shared -fPIC -o /tmp/voe.so tools/visit_order_exp.c -lm
 * Driven by tools/visit_order_exp.py on gpurun_out/rays_c3.npz (tools/dump_rays.py). */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { float lox[4], hix[4], loy[4], hiy[4], loz[4], hiz[4]; int32_t child[4], pad[4]; } DNode;
typedef struct { float v0[4], e1[4], e2[4]; } DTri;

static float safe_inv(float d) { return 1.0f / (fabsf(d) > 1e-20f ? d : copysignf(1e-20f, d)); }

static int tri_test(const DTri* t, const float o[3], const float d[3], float tnear, float tfar, float* tout) {
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
  *tout = tt;
  return ok && tt > tnear && tt < tfar;
}

/* order[node*8 + octant] = 4 slots packed 2 bits each, first = visited first */
static uint8_t* octant_orders(const DNode* nodes, size_t nn) {
  uint8_t* ord = (uint8_t*)malloc(nn * 8);
  for (size_t i = 0; i < nn; ++i)
    for (int o = 0; o < 8; ++o) {
      const float dx = (o & 1) ? -1.f : 1.f, dy = (o & 2) ? -1.f : 1.f, dz = (o & 4) ? -1.f : 1.f;
      float key[4];
      int s[4] = {0, 1, 2, 3};
      for (int k = 0; k < 4; ++k) {
        const DNode* n = &nodes[i];
        key[k] = n->child[k] == -1 ? INFINITY
                                   : dx * (n->lox[k] + n->hix[k]) + dy * (n->loy[k] + n->hiy[k]) + dz * (n->loz[k] + n->hiz[k]);
      }
      for (int a = 0; a < 4; ++a)
        for (int b = a + 1; b < 4; ++b)
          if (key[s[b]] < key[s[a]]) { int t = s[a]; s[a] = s[b]; s[b] = t; }
      ord[i * 8 + o] = (uint8_t)(s[0] | s[1] << 2 | s[2] << 4 | s[3] << 6);
    }
  return ord;
}

/* One canonical child order per node (children by box centre along one axis, stored that way)
 * and its reversal when the ray's direction on that axis is negative: 13 = the axis of the
 * largest spread of the child centres, 14 = the axis of the node's largest extent. Per node:
 * order bits 0-7, axis bits 8-9. */
static uint16_t* axis_orders(const DNode* nodes, size_t nn, int variant) {
  uint16_t* ord = (uint16_t*)malloc(nn * 2);
  for (size_t i = 0; i < nn; ++i) {
    const DNode* n = &nodes[i];
    float cmin[3] = {INFINITY, INFINITY, INFINITY}, cmax[3] = {-INFINITY, -INFINITY, -INFINITY};
    float bmin[3] = {INFINITY, INFINITY, INFINITY}, bmax[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int k = 0; k < 4; ++k) {
      if (n->child[k] == -1) continue;
      const float lo[3] = {n->lox[k], n->loy[k], n->loz[k]}, hi[3] = {n->hix[k], n->hiy[k], n->hiz[k]};
      for (int a = 0; a < 3; ++a) {
        const float c = lo[a] + hi[a];
        cmin[a] = fminf(cmin[a], c); cmax[a] = fmaxf(cmax[a], c);
        bmin[a] = fminf(bmin[a], lo[a]); bmax[a] = fmaxf(bmax[a], hi[a]);
      }
    }
    int ax = 0;
    for (int a = 1; a < 3; ++a) {
      const float ea = variant == 13 ? cmax[a] - cmin[a] : bmax[a] - bmin[a];
      const float e0 = variant == 13 ? cmax[ax] - cmin[ax] : bmax[ax] - bmin[ax];
      if (ea > e0) ax = a;
    }
    float key[4];
    int s[4] = {0, 1, 2, 3};
    for (int k = 0; k < 4; ++k) {
      const float lo[3] = {n->lox[k], n->loy[k], n->loz[k]}, hi[3] = {n->hix[k], n->hiy[k], n->hiz[k]};
      key[k] = n->child[k] == -1 ? INFINITY : lo[ax] + hi[ax];
    }
    for (int a = 0; a < 4; ++a)
      for (int b = a + 1; b < 4; ++b)
        if (key[s[b]] < key[s[a]]) { int t = s[a]; s[a] = s[b]; s[b] = t; }
    ord[i] = (uint16_t)(s[0] | s[1] << 2 | s[2] << 4 | s[3] << 6 | ax << 8);
  }
  return ord;
}

int visit_counts(const void* nodes_, size_t nn, const void* tris_, const float* org4, const float* dir4, int n,
                 int anyHit, int mode, double* out3) {
  const DNode* nodes = (const DNode*)nodes_;
  const DTri* tris = (const DTri*)tris_;
  uint8_t* ord = (mode == 1 || mode == 6 || mode == 9) ? octant_orders(nodes, nn) : NULL;
  uint16_t* aord = (mode == 13 || mode == 14) ? axis_orders(nodes, nn, mode) : NULL;
  double nv = 0, tv = 0, pushes = 0;
  for (int i = 0; i < n; ++i) {
    const float o[3] = {org4[4 * i], org4[4 * i + 1], org4[4 * i + 2]};
    const float d[3] = {dir4[4 * i], dir4[4 * i + 1], dir4[4 * i + 2]};
    const float tnear = org4[4 * i + 3];
    float best = dir4[4 * i + 3];
    if (!(best >= tnear)) continue;
    if (mode == 10 && i < n) {  /* lower bound: start with the final closest-hit distance */
      double tmp[3];
      static float hitT;
      (void)tmp;
      hitT = best;
      /* brute force over the leaves is too slow; run distance mode first */
      int stack2[256], sp2 = 0, cur2 = 0;
      const float iv2[3] = {safe_inv(d[0]), safe_inv(d[1]), safe_inv(d[2])};
      for (;;) {
        if ((cur2 & 31) == 0) {
          const DNode* nd = &nodes[cur2 >> 5];
          for (int k = 0; k < 4; ++k) if (nd->child[k] != -1) {
            float tn = tnear, tf = hitT;
            const float lo[3] = {nd->lox[k], nd->loy[k], nd->loz[k]}, hi[3] = {nd->hix[k], nd->hiy[k], nd->hiz[k]};
            for (int a = 0; a < 3; ++a) {
              float l = (lo[a] - o[a]) * iv2[a], h = (hi[a] - o[a]) * iv2[a];
              if (l > h) { float q = l; l = h; h = q; }
              tn = fmaxf(tn, l); tf = fminf(tf, h * 1.0001f);
            }
            if (tn <= tf) stack2[sp2++] = nd->child[k];
          }
        } else {
          for (int k = 0; k < (cur2 & 31); ++k) {
            float tt;
            if (tri_test(&tris[(cur2 >> 5) + k], o, d, tnear, hitT, &tt)) hitT = tt;
          }
        }
        if (sp2 == 0) break;
        cur2 = stack2[--sp2];
      }
      best = hitT * 1.00001f + 1e-6f;
    }
    const float iv[3] = {safe_inv(d[0]), safe_inv(d[1]), safe_inv(d[2])};
    const int oct = (d[0] < 0) | (d[1] < 0) << 1 | (d[2] < 0) << 2;
    const float oi[3] = {o[0] * iv[0], o[1] * iv[1], o[2] * iv[2]};
    const float margin = fmaxf(fmaxf(fabsf(oi[0]), fabsf(oi[1])), fabsf(oi[2])) * 2.384185791015625e-07f;
    int stack[256], sp = 0, cur = 0, done = 0;
    while (!done) {
      if ((cur & 31) == 0) {
        const int ni = cur >> 5;
        const DNode* nd = &nodes[ni];
        nv += 1;
        float t[4];
        int c[4];
        for (int k = 0; k < 4; ++k) {
          const float lo[3] = {nd->lox[k], nd->loy[k], nd->loz[k]}, hi[3] = {nd->hix[k], nd->hiy[k], nd->hiz[k]};
          float l[3], h[3];
          for (int a = 0; a < 3; ++a) { l[a] = fmaf(lo[a], iv[a], -oi[a]); h[a] = fmaf(hi[a], iv[a], -oi[a]); }
          const float a0 = fmaxf(fmaxf(fminf(l[0], h[0]), fminf(l[1], h[1])), fmaxf(fminf(l[2], h[2]), tnear));
          const float b0 = fminf(fminf(fmaxf(l[0], h[0]), fmaxf(l[1], h[1])), fminf(fmaxf(l[2], h[2]), best));
          const int hit = a0 <= fmaf(b0, 1.0000152587890625f, margin) && nd->child[k] != -1;
          t[k] = hit ? a0 : INFINITY;
          c[k] = nd->child[k];
        }
        if (mode == 7 || mode == 9) {
          /* 7: the farthest hit child first, the others in slot order;
             9: the child whose box centre is farthest along the octant diagonal first (precomputed) */
          int f = -1;
          if (mode == 7) {
            float bt = -1.f;
            for (int k = 0; k < 4; ++k)
              if (t[k] < INFINITY && t[k] > bt) { bt = t[k]; f = k; }
          } else {
            f = ord[(size_t)ni * 8 + (oct ^ 7)] & 3;
          }
          if (f > 0) {
            const float tf = t[f];
            const int cf = c[f];
            for (int k = f; k > 0; --k) { t[k] = t[k - 1]; c[k] = c[k - 1]; }
            t[0] = tf; c[0] = cf;
          }
        } else if (mode == 8) {  /* descending comparators (0,1),(2,3),(0,2): max first */
          static const int net[3][2] = {{0, 1}, {2, 3}, {0, 2}};
          for (int m = 0; m < 3; ++m) {
            const int a = net[m][0], b = net[m][1];
            const float ka = t[a] < INFINITY ? t[a] : -1.f, kb = t[b] < INFINITY ? t[b] : -1.f;
            if (kb > ka) {
              float tt = t[a]; t[a] = t[b]; t[b] = tt;
              int cc = c[a]; c[a] = c[b]; c[b] = cc;
            }
          }
        } else if (mode == 5) {  /* farthest entry first */
          for (int a = 1; a < 4; ++a)
            for (int b = a; b > 0; --b) {
              const float ka = t[b] < INFINITY ? t[b] : -1.f, kb = t[b - 1] < INFINITY ? t[b - 1] : -1.f;
              if (!(ka > kb)) break;
              float tt = t[b]; t[b] = t[b - 1]; t[b - 1] = tt;
              int cc = c[b]; c[b] = c[b - 1]; c[b - 1] = cc;
            }
        } else if (mode == 6) {  /* octant order reversed (farthest box centre first) */
          const uint8_t p = ord[(size_t)ni * 8 + (oct ^ 7)];
          float t2[4];
          int c2[4];
          for (int k = 0; k < 4; ++k) { const int s = (p >> (2 * k)) & 3; t2[k] = t[s]; c2[k] = c[s]; }
          memcpy(t, t2, sizeof t);
          memcpy(c, c2, sizeof c);
        } else if (mode == 0 || mode == 11 || mode == 12) {
          /* 0: full sort (5 comparators); 11: nearest first only ((0,1),(2,3),(0,2));
             12: nearest first and farthest last (+ (1,3)) */
          static const int net[5][2] = {{0, 1}, {2, 3}, {0, 2}, {1, 3}, {1, 2}};
          const int ncmp = mode == 0 ? 5 : mode == 11 ? 3 : 4;
          for (int m = 0; m < ncmp; ++m) {
            const int a = net[m][0], b = net[m][1];
            if (t[b] < t[a]) {
              float tt = t[a]; t[a] = t[b]; t[b] = tt;
              int cc = c[a]; c[a] = c[b]; c[b] = cc;
            }
          }
        } else if (mode == 3 || mode == 4) {
          /* static per-node order: child boxes by surface area (3 descending, 4 ascending) */
          int s4[4] = {0, 1, 2, 3};
          float ar[4];
          for (int k = 0; k < 4; ++k) {
            const float dx = nd->hix[k] - nd->lox[k], dy = nd->hiy[k] - nd->loy[k], dz = nd->hiz[k] - nd->loz[k];
            ar[k] = nd->child[k] == -1 ? -1.f : dx * dy + dy * dz + dz * dx;
            if (mode == 4 && nd->child[k] != -1) ar[k] = -ar[k] + 0.f;
            if (mode == 4 && nd->child[k] == -1) ar[k] = -INFINITY;
          }
          for (int a = 0; a < 4; ++a)
            for (int b = a + 1; b < 4; ++b)
              if (ar[s4[b]] > ar[s4[a]]) { int tq = s4[a]; s4[a] = s4[b]; s4[b] = tq; }
          float t2[4];
          int c2[4];
          for (int k = 0; k < 4; ++k) { t2[k] = t[s4[k]]; c2[k] = c[s4[k]]; }
          memcpy(t, t2, sizeof t);
          memcpy(c, c2, sizeof c);
        } else if (mode == 13 || mode == 14) {
          const uint16_t p = aord[ni];
          const int ax = p >> 8;
          const int rev = d[ax] < 0.f;
          float t2[4];
          int c2[4];
          for (int k = 0; k < 4; ++k) {
            const int s = (p >> (2 * (rev ? 3 - k : k))) & 3;
            t2[k] = t[s]; c2[k] = c[s];
          }
          memcpy(t, t2, sizeof t);
          memcpy(c, c2, sizeof c);
        } else if (mode == 1) {
          const uint8_t p = ord[(size_t)ni * 8 + oct];
          float t2[4];
          int c2[4];
          for (int k = 0; k < 4; ++k) { const int s = (p >> (2 * k)) & 3; t2[k] = t[s]; c2[k] = c[s]; }
          memcpy(t, t2, sizeof t);
          memcpy(c, c2, sizeof c);
        }
        int first = -1;
        for (int k = 0; k < 4; ++k)
          if (t[k] < INFINITY) { first = k; break; }
        for (int k = 3; k > first && first >= 0; --k)
          if (t[k] < INFINITY) { stack[sp++] = c[k]; pushes += 1; }
        if (first >= 0) {
          cur = c[first];
          continue;
        }
      } else {
        const int ci = cur >> 5, cc = cur & 31;
        for (int k = 0; k < cc; ++k) {
          tv += 1;
          float tt;
          if (tri_test(&tris[ci + k], o, d, tnear, anyHit ? dir4[4 * i + 3] : best, &tt)) {
            if (anyHit) { done = 1; break; }
            best = tt;
          }
        }
        if (done) break;
      }
      if (sp == 0) break;
      cur = stack[--sp];
    }
  }
  free(ord);
  free(aord);
  out3[0] = nv / n;
  out3[1] = tv / n;
  out3[2] = pushes / n;
  return 0;
}

/* ---- BVH8 collapsed from the BVH4 (greedy: open the largest-area inner child while the
 * node has room), distance-sorted closest hit / slot-order any hit; counts node visits. */
typedef struct { float lo[8][3], hi[8][3]; int32_t child[8]; } N8;
static float area3(const float* lo, const float* hi) {
  const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
  return dx * dy + dy * dz + dz * dx;
}
static int build8(const DNode* nodes, int ni, N8* out, int* count) {
  const int me = (*count)++;
  N8 n;
  int m = 0;
  const DNode* d = &nodes[ni];
  for (int k = 0; k < 4; ++k)
    if (d->child[k] != -1) {
      n.lo[m][0] = d->lox[k]; n.lo[m][1] = d->loy[k]; n.lo[m][2] = d->loz[k];
      n.hi[m][0] = d->hix[k]; n.hi[m][1] = d->hiy[k]; n.hi[m][2] = d->hiz[k];
      n.child[m++] = d->child[k];
    }
  for (;;) {
    int best = -1;
    float ba = -1;
    for (int k = 0; k < m; ++k)
      if ((n.child[k] & 31) == 0) {
        const DNode* c = &nodes[n.child[k] >> 5];
        int nc = 0;
        for (int j = 0; j < 4; ++j) nc += c->child[j] != -1;
        if (m - 1 + nc <= 8) {
          const float a = area3(n.lo[k], n.hi[k]);
          if (a > ba) { ba = a; best = k; }
        }
      }
    if (best < 0) break;
    const DNode* c = &nodes[n.child[best] >> 5];
    int slot = best;
    for (int j = 0; j < 4; ++j)
      if (c->child[j] != -1) {
        const int s = slot >= 0 ? slot : m++;
        slot = -1;
        n.lo[s][0] = c->lox[j]; n.lo[s][1] = c->loy[j]; n.lo[s][2] = c->loz[j];
        n.hi[s][0] = c->hix[j]; n.hi[s][1] = c->hiy[j]; n.hi[s][2] = c->hiz[j];
        n.child[s] = c->child[j];
      }
  }
  for (int k = m; k < 8; ++k) n.child[k] = -1;
  for (int k = 0; k < m; ++k)
    if ((n.child[k] & 31) == 0) n.child[k] = build8(nodes, n.child[k] >> 5, out, count) << 5;
  out[me] = n;
  return me;
}

int visit_counts8(const void* nodes_, size_t nn, const void* tris_, const float* org4, const float* dir4, int n,
                  int anyHit, double* out3) {
  const DNode* nodes = (const DNode*)nodes_;
  const DTri* tris = (const DTri*)tris_;
  N8* n8 = (N8*)malloc(sizeof(N8) * nn);
  int cnt = 0;
  build8(nodes, 0, n8, &cnt);
  double nv = 0, tv = 0, pushes = 0;
  for (int i = 0; i < n; ++i) {
    const float o[3] = {org4[4 * i], org4[4 * i + 1], org4[4 * i + 2]};
    const float d[3] = {dir4[4 * i], dir4[4 * i + 1], dir4[4 * i + 2]};
    const float tnear = org4[4 * i + 3];
    float best = dir4[4 * i + 3];
    if (!(best >= tnear)) continue;
    const float iv[3] = {safe_inv(d[0]), safe_inv(d[1]), safe_inv(d[2])};
    const float oi[3] = {o[0] * iv[0], o[1] * iv[1], o[2] * iv[2]};
    const float margin = fmaxf(fmaxf(fabsf(oi[0]), fabsf(oi[1])), fabsf(oi[2])) * 2.384185791015625e-07f;
    int stack[512], sp = 0, cur = 0, done = 0;
    while (!done) {
      if ((cur & 31) == 0) {
        const N8* nd = &n8[cur >> 5];
        nv += 1;
        float t[8];
        int c[8];
        for (int k = 0; k < 8; ++k) {
          float l[3], h[3];
          for (int a = 0; a < 3; ++a) { l[a] = fmaf(nd->lo[k][a], iv[a], -oi[a]); h[a] = fmaf(nd->hi[k][a], iv[a], -oi[a]); }
          const float a0 = fmaxf(fmaxf(fminf(l[0], h[0]), fminf(l[1], h[1])), fmaxf(fminf(l[2], h[2]), tnear));
          const float b0 = fminf(fminf(fmaxf(l[0], h[0]), fmaxf(l[1], h[1])), fminf(fmaxf(l[2], h[2]), best));
          const int hit = nd->child[k] != -1 && a0 <= fmaf(b0, 1.0000152587890625f, margin);
          t[k] = hit ? a0 : INFINITY;
          c[k] = nd->child[k];
        }
        if (!anyHit)
          for (int a = 1; a < 8; ++a)
            for (int b = a; b > 0 && t[b] < t[b - 1]; --b) {
              float tt = t[b]; t[b] = t[b - 1]; t[b - 1] = tt;
              int cc = c[b]; c[b] = c[b - 1]; c[b - 1] = cc;
            }
        int first = -1;
        for (int k = 0; k < 8; ++k)
          if (t[k] < INFINITY) { first = k; break; }
        for (int k = 7; k > first && first >= 0; --k)
          if (t[k] < INFINITY) { stack[sp++] = c[k]; pushes += 1; }
        if (first >= 0) { cur = c[first]; continue; }
      } else {
        const int ci = cur >> 5, cc = cur & 31;
        for (int k = 0; k < cc; ++k) {
          tv += 1;
          float tt;
          if (tri_test(&tris[ci + k], o, d, tnear, anyHit ? dir4[4 * i + 3] : best, &tt)) {
            if (anyHit) { done = 1; break; }
            best = tt;
          }
        }
        if (done) break;
      }
      if (sp == 0) break;
      cur = stack[--sp];
    }
  }
  free(n8);
  out3[0] = nv / n;
  out3[1] = tv / n;
  out3[2] = pushes / n;
  return cnt;
}
