/* anyhit_stack_exp.c — CPU experiment: stack depth of the any-hit traversal on the device BVH4
 * (farthest hit child first, the others pushed in slot order, as k_trace<true>) over a captured
 * shadow stream: per query the deepest stack and the number of pushes beyond a ring of R
 * entries (R = 8, 16, 32), i.e. what an LDS ring of R entries would evict to global memory.
 * Build: gcc -O2 -shared -fPIC -o /tmp/ase.so tools/anyhit_stack_exp.c -lm */
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

/* out[q] = max stack depth of query q; ev[3*q + k] = evictions with a ring of 8 << k entries */
void stack_depths(const void* nodes_, const void* tris_, const float* org4, const float* dir4, int n, int* out,
                  int* ev) {
  const DNode* nodes = (const DNode*)nodes_;
  const DTri* tris = (const DTri*)tris_;
  for (int i = 0; i < n; ++i) {
    const float o[3] = {org4[4 * i], org4[4 * i + 1], org4[4 * i + 2]};
    const float d[3] = {dir4[4 * i], dir4[4 * i + 1], dir4[4 * i + 2]};
    const float tnear = org4[4 * i + 3], tfar = dir4[4 * i + 3];
    out[i] = 0;
    ev[3 * i] = ev[3 * i + 1] = ev[3 * i + 2] = 0;
    if (!(tfar >= tnear)) continue;
    const float iv[3] = {safe_inv(d[0]), safe_inv(d[1]), safe_inv(d[2])};
    int stack[256], sp = 0, cur = 0, maxsp = 0, found = 0;
    for (;;) {
      if ((cur & 31) == 0) {
        const DNode* nd = nodes + (cur >> 5);
        float t[4];
        int c[4];
        for (int k = 0; k < 4; ++k) {
          float l[3], h[3];
          const float lo[3] = {nd->lox[k], nd->loy[k], nd->loz[k]}, hi[3] = {nd->hix[k], nd->hiy[k], nd->hiz[k]};
          for (int a = 0; a < 3; ++a) { l[a] = (lo[a] - o[a]) * iv[a]; h[a] = (hi[a] - o[a]) * iv[a]; }
          const float nn = fmaxf(fmaxf(fminf(l[0], h[0]), fminf(l[1], h[1])), fmaxf(fminf(l[2], h[2]), tnear));
          const float ff = fminf(fminf(fmaxf(l[0], h[0]), fmaxf(l[1], h[1])), fminf(fmaxf(l[2], h[2]), tfar));
          t[k] = (nn <= ff * 1.0000152587890625f && nd->child[k] != -1) ? nn : -INFINITY;
          c[k] = nd->child[k];
        }
#define SW(a, b) do { if (t[b] > t[a]) { float tt = t[a]; t[a] = t[b]; t[b] = tt; int cc = c[a]; c[a] = c[b]; c[b] = cc; } } while (0)
        SW(0, 1); SW(2, 3); SW(0, 2);
#undef SW
        for (int k = 3; k >= 1; --k)
          if (t[k] > -INFINITY) {
            for (int r = 0; r < 3; ++r)
              if (sp >= (8 << r)) ev[3 * i + r]++;
            stack[sp++] = c[k];
          }
        if (sp > maxsp) maxsp = sp;
        if (t[0] > -INFINITY) { cur = c[0]; continue; }
      } else {
        const int idx = cur >> 5, cnt = cur & 31;
        for (int k = 0; k < cnt && !found; ++k) found = tri_test(tris + idx + k, o, d, tnear, tfar);
        if (found) break;
      }
      if (sp == 0) break;
      cur = stack[--sp];
    }
    out[i] = maxsp;
  }
}

/* The closest-hit traversal of k_trace<false>: the hit children sorted by entry distance,
 * nearest next, the others pushed farthest first; tfar shrinks to the closest hit so far.
 * out / ev as stack_depths. */
void closest_stack_depths(const void* nodes_, const void* tris_, const float* org4, const float* dir4, int n,
                          int* out, int* ev) {
  const DNode* nodes = (const DNode*)nodes_;
  const DTri* tris = (const DTri*)tris_;
  for (int i = 0; i < n; ++i) {
    const float o[3] = {org4[4 * i], org4[4 * i + 1], org4[4 * i + 2]};
    const float d[3] = {dir4[4 * i], dir4[4 * i + 1], dir4[4 * i + 2]};
    const float tnear = org4[4 * i + 3];
    float tfar = dir4[4 * i + 3];
    out[i] = 0;
    ev[3 * i] = ev[3 * i + 1] = ev[3 * i + 2] = 0;
    if (!(tfar >= tnear)) continue;
    const float iv[3] = {safe_inv(d[0]), safe_inv(d[1]), safe_inv(d[2])};
    int stack[256], sp = 0, cur = 0, maxsp = 0;
    for (;;) {
      if ((cur & 31) == 0) {
        const DNode* nd = nodes + (cur >> 5);
        float t[4];
        int c[4];
        for (int k = 0; k < 4; ++k) {
          float l[3], h[3];
          const float lo[3] = {nd->lox[k], nd->loy[k], nd->loz[k]}, hi[3] = {nd->hix[k], nd->hiy[k], nd->hiz[k]};
          for (int a = 0; a < 3; ++a) { l[a] = (lo[a] - o[a]) * iv[a]; h[a] = (hi[a] - o[a]) * iv[a]; }
          const float nn = fmaxf(fmaxf(fminf(l[0], h[0]), fminf(l[1], h[1])), fmaxf(fminf(l[2], h[2]), tnear));
          const float ff = fminf(fminf(fmaxf(l[0], h[0]), fmaxf(l[1], h[1])), fminf(fmaxf(l[2], h[2]), tfar));
          t[k] = (nn <= ff * 1.0000152587890625f && nd->child[k] != -1) ? nn : INFINITY;
          c[k] = nd->child[k];
        }
#define SW(a, b) do { if (t[b] < t[a]) { float tt = t[a]; t[a] = t[b]; t[b] = tt; int cc = c[a]; c[a] = c[b]; c[b] = cc; } } while (0)
        SW(0, 1); SW(2, 3); SW(0, 2); SW(1, 3); SW(1, 2);
#undef SW
        for (int k = 3; k >= 1; --k)
          if (t[k] < INFINITY) {
            for (int r = 0; r < 3; ++r)
              if (sp >= (8 << r)) ev[3 * i + r]++;
            stack[sp++] = c[k];
          }
        if (sp > maxsp) maxsp = sp;
        if (t[0] < INFINITY) { cur = c[0]; continue; }
      } else {
        const int idx = cur >> 5, cnt = cur & 31;
        for (int k = 0; k < cnt; ++k) {
          const DTri* tr = tris + idx + k;
          /* shrink tfar to an accepted hit (the same acceptance as tri_test, distance recomputed) */
          if (tri_test(tr, o, d, tnear, tfar)) {
            float lo = tnear, hi = tfar;
            for (int it = 0; it < 40; ++it) {  /* bisect the accepted distance: enough for the stack statistics */
              const float mid = 0.5f * (lo + hi);
              if (tri_test(tr, o, d, tnear, mid)) hi = mid; else lo = mid;
            }
            tfar = hi;
          }
        }
      }
      if (sp == 0) break;
      cur = stack[--sp];
    }
    out[i] = maxsp;
  }
}
