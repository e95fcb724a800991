/* anyhit_order_exp.c — CPU experiment: child visiting orders for the any-hit traversal of the
 * device BVH4 over captured shadow streams. Per query: node steps and triangle tests until the
 * first occluder (or the end). Orders (mode):
 *   0  farthest entry distance first, the others pushed in slot order (k_trace<true> today)
 *   1  nearest entry distance first (the closest-hit order)
 *   2  slot order (no sort)
 *   3  a static per-node order given in `perm` (4 child indices per node): no per-ray sort
 *   4  every hit child by entry distance, farthest first
 *   5  every hit child by exit distance, farthest first
 * The occlusion result is the same in every order (a boolean).
 * Build: gcc -O2 -shared -fPIC -o /tmp/aho.so tools/anyhit_order_exp.c -lm */
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

/* steps[2q] node steps, steps[2q+1] triangle tests, occ[q] occluder slot or -1 */
void anyhit_order(const void* nodes_, const void* tris_, const float* org4, const float* dir4, int n, int mode,
                  const int* perm, int* steps, int* occ) {
  const DNode* nodes = (const DNode*)nodes_;
  const DTri* tris = (const DTri*)tris_;
  for (int i = 0; i < n; ++i) {
    const float o[3] = {org4[4 * i], org4[4 * i + 1], org4[4 * i + 2]};
    const float d[3] = {dir4[4 * i], dir4[4 * i + 1], dir4[4 * i + 2]};
    const float tnear = org4[4 * i + 3], tfar = dir4[4 * i + 3];
    steps[2 * i] = steps[2 * i + 1] = 0;
    occ[i] = -1;
    if (!(tfar >= tnear)) continue;
    const float iv[3] = {safe_inv(d[0]), safe_inv(d[1]), safe_inv(d[2])};
    int stack[256], sp = 0, cur = 0;
    for (;;) {
      if ((cur & 31) == 0) {
        const int ni = cur >> 5;
        const DNode* nd = nodes + ni;
        steps[2 * i]++;
        float t[4];
        int c[4], hit[4];
        for (int k = 0; k < 4; ++k) {
          float l[3], h[3];
          const float lo[3] = {nd->lox[k], nd->loy[k], nd->loz[k]}, hi[3] = {nd->hix[k], nd->hiy[k], nd->hiz[k]};
          for (int a = 0; a < 3; ++a) { l[a] = (lo[a] - o[a]) * iv[a]; h[a] = (hi[a] - o[a]) * iv[a]; }
          const float nn = fmaxf(fmaxf(fminf(l[0], h[0]), fminf(l[1], h[1])), fmaxf(fminf(l[2], h[2]), tnear));
          const float ff = fminf(fminf(fmaxf(l[0], h[0]), fmaxf(l[1], h[1])), fminf(fmaxf(l[2], h[2]), tfar));
          hit[k] = nn <= ff * 1.0000152587890625f && nd->child[k] != -1;
          t[k] = mode == 5 ? ff : nn;
          c[k] = nd->child[k];
        }
        int ord[4] = {0, 1, 2, 3};
        if (mode == 3) {
          for (int k = 0; k < 4; ++k) ord[k] = perm[4 * ni + k];
        } else if (mode == 0 || mode == 1 || mode == 4 || mode == 5) {
          /* insertion sort of the hit children by entry distance (far or near first), misses last */
          for (int a = 1; a < 4; ++a)
            for (int b = a; b > 0; --b) {
              const int x = ord[b], y = ord[b - 1];
              const int better = hit[x] && (!hit[y] || (mode != 1 ? t[x] > t[y] : t[x] < t[y]));
              if (!better) break;
              ord[b] = y;
              ord[b - 1] = x;
            }
          if (mode == 0) {
            /* the device keeps the others in slot order: re-sort ord[1..3] by slot */
            for (int a = 2; a < 4; ++a)
              for (int b = a; b > 1 && ord[b] < ord[b - 1]; --b) { const int x = ord[b]; ord[b] = ord[b - 1]; ord[b - 1] = x; }
          }
        }
        int first = -1;
        for (int k = 3; k >= 0; --k) {
          const int ch = ord[k];
          if (!hit[ch]) continue;
          if (first >= 0) stack[sp++] = c[first];
          first = ch;
        }
        if (first >= 0) { cur = c[first]; continue; }
      } else {
        const int idx = cur >> 5, cnt = cur & 31;
        for (int k = 0; k < cnt && occ[i] < 0; ++k) {
          steps[2 * i + 1]++;
          if (tri_test(tris + idx + k, o, d, tnear, tfar)) occ[i] = idx + k;
        }
        if (occ[i] >= 0) break;
      }
      if (sp == 0) break;
      cur = stack[--sp];
    }
  }
}
