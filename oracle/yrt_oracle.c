/* yrt_oracle.c — CPU restatement of the reference device_singleray path (test infrastructure
 * only; see yrt_oracle.h). Every function cites the reference file:line it restates. */
#define _GNU_SOURCE
#include "yrt_oracle.h"

/* the per-ray path's elementary functions, evaluated exactly as the device does */
#include "../yulio-raytracer_amd/csrc/common/yrt_libm.h"
/* the reference's rcp/rsqrt: Intel rcpps/rsqrtps emulated exactly + math.h's Newton step */
#include "../yulio-raytracer_amd/csrc/common/yrt_sse_rcp.h"
#include "../yulio-raytracer_amd/csrc/common/yrt_tile_scatter.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>
#include <time.h>
#include <unistd.h>

static __thread char g_err[512];
const char* oracle_last_error(void) { return g_err; }
static int fail(const char* msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg);
  return -1;
}

/* ====================================================================== vector math
 * common/math/vec3.h, linearspace3.h, affinespace.h; rcp and rsqrt as common/math/math.h:38-59
 * (the SSE estimate + one Newton step, yrt_sse_rcp.h); -DYRT_ORACLE_IEEE_RCP builds the round 1-5
 * substitution (1/x, 1/sqrt(x)) for the sensitivity measurement (tools/rcp_sensitivity.py). */
typedef struct { float x, y, z; } V3;
static inline V3 v3(float x, float y, float z) { V3 r = {x, y, z}; return r; }
static inline V3 vs(float s) { return v3(s, s, s); }
static inline V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V3 neg(V3 a) { return v3(-a.x, -a.y, -a.z); }
static inline V3 mulv(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline V3 muls(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
/* dot, cross and lmul in the reference build's operation sequences (x64 MSVC, SSE4.1 forced by
 * common/sys/platform.h:100-103, no AVX2: no fused multiply-add), as the product's yrt_math.h:
 *   dot   = _mm_dp_ps(a, b, 0x7F), common/math/vector3f_sse.h:206-209: the products, then
 *           (x + y) + z (dp_ps's +0 fourth lane, which only turns a -0 sum into +0, left out);
 *   cross = a0*b0 - a1*b1, vector3f_sse.h:226-233 (the non-AVX2 branch);
 *   lmul  = v.x*vx + v.y*vy + v.z*vz left to right, common/math/linearspace3.h:134. */
static inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline V3 cross(V3 a, V3 b) { return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
#if defined(YRT_ORACLE_IEEE_RCP)
static inline float rcp(float x) { return 1.0f / x; }
static inline float rsqrt_(float x) { return 1.0f / sqrtf(x); }
#else
static inline float rcp(float x) { return yrt_ref_rcp(x); }      /* math.h:38-42 */
static inline float rsqrt_(float x) { return yrt_ref_rsqrt(x); } /* math.h:53-58 */
#endif
static inline V3 normalize(V3 a) { return muls(a, rsqrt_(dot(a, a))); }
static inline float length(V3 a) { return sqrtf(dot(a, a)); }
static inline float fmax3(V3 a) { return fmaxf(fmaxf(a.x, a.y), a.z); }
static inline V3 absv(V3 a) { return v3(fabsf(a.x), fabsf(a.y), fabsf(a.z)); }
static inline float clampf_(float x, float lo, float hi) { return fmaxf(lo, fminf(x, hi)); }
static inline float clamp01(float x) { return clampf_(x, 0.0f, 1.0f); }
static inline int v3zero(V3 a) { return a.x == 0.0f && a.y == 0.0f && a.z == 0.0f; }
static inline int veq(V3 a, V3 b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
static inline float signf_(float x) { return x < 0 ? -1.0f : 1.0f; }
static inline float smoothstep_(float e0, float e1, float x) {
  x = clampf_((x - e0) / (e1 - e0), 0.0f, 1.0f);
  return x * x * (3 - 2 * x);
}
#define PI_F 3.14159265358979323846f
#define TWO_PI_F 6.28318530717958647692f
#define ONE_OVER_PI_F 0.31830988618379069122f
#define ONE_OVER_TWO_PI_F 0.15915494309189534561f
#define ULP_F 1.19209290e-07f
static inline float deg2rad(float x) { return x * 1.74532925199432957692e-2f; }
static inline float rad2deg(float x) { return x * 5.72957795130823208768e1f; }

typedef struct { V3 vx, vy, vz; } L3;
typedef struct { L3 l; V3 p; } A3;
static inline L3 l3(V3 a, V3 b, V3 c) { L3 r = {a, b, c}; return r; }
static inline L3 l3_rows(float m00, float m01, float m02, float m10, float m11, float m12, float m20, float m21,
                         float m22) {
  return l3(v3(m00, m10, m20), v3(m01, m11, m21), v3(m02, m12, m22));
}
static inline L3 l3_one(void) { return l3(v3(1, 0, 0), v3(0, 1, 0), v3(0, 0, 1)); }
static inline V3 lmul(L3 a, V3 b) { return add(add(muls(a.vx, b.x), muls(a.vy, b.y)), muls(a.vz, b.z)); }
static inline L3 llmul(L3 a, L3 b) { return l3(lmul(a, b.vx), lmul(a, b.vy), lmul(a, b.vz)); }
static inline L3 ltrans(L3 a) { return l3_rows(a.vx.x, a.vx.y, a.vx.z, a.vy.x, a.vy.y, a.vy.z, a.vz.x, a.vz.y, a.vz.z); }
static inline L3 linv(L3 a) {
  /* rcp(det())*adjoint(), adjoint = (cross(vy,vz), cross(vz,vx), cross(vx,vy)).transposed() */
  L3 adj = ltrans(l3(cross(a.vy, a.vz), cross(a.vz, a.vx), cross(a.vx, a.vy)));
  float r = rcp(dot(a.vx, cross(a.vy, a.vz)));
  return l3(muls(adj.vx, r), muls(adj.vy, r), muls(adj.vz, r));
}
static inline L3 lrotate(V3 u_, float r) {
  V3 u = normalize(u_);
  float s = yrt_sinf(r), c = yrt_cosf(r);
  return l3_rows(u.x * u.x + (1 - u.x * u.x) * c, u.x * u.y * (1 - c) - u.z * s, u.x * u.z * (1 - c) + u.y * s,
                 u.x * u.y * (1 - c) + u.z * s, u.y * u.y + (1 - u.y * u.y) * c, u.y * u.z * (1 - c) - u.x * s,
                 u.x * u.z * (1 - c) - u.y * s, u.y * u.z * (1 - c) + u.x * s, u.z * u.z + (1 - u.z * u.z) * c);
}
static inline L3 frame_(V3 N) { /* linearspace3.h:118-124 */
  V3 dx0 = cross(v3(1.0f, 0.0f, 0.0f), N);
  V3 dx1 = cross(v3(0.0f, 1.0f, 0.0f), N);
  V3 dx = normalize(dot(dx0, dx0) > dot(dx1, dx1) ? dx0 : dx1);
  V3 dy = normalize(cross(N, dx));
  return l3(dx, dy, N);
}
static inline A3 a3(L3 l, V3 p) { A3 r = {l, p}; return r; }
static inline A3 a3_one(void) { return a3(l3_one(), vs(0.0f)); }
static inline A3 aamul(A3 a, A3 b) { return a3(llmul(a.l, b.l), add(lmul(a.l, b.p), a.p)); }
static inline V3 xfmPoint(A3 m, V3 p) { return add(lmul(m.l, p), m.p); }
static inline V3 xfmVector(A3 m, V3 v) { return lmul(m.l, v); }
static inline V3 xfmNormal(A3 m, V3 n) { return lmul(ltrans(linv(m.l)), n); }
static inline A3 a3_translate(V3 p) { return a3(l3_one(), p); }
static inline A3 a3_rotate_about(V3 p, V3 u, float r) {
  return aamul(aamul(a3_translate(p), a3(lrotate(u, r), vs(0.0f))), a3_translate(neg(p)));
}
static inline A3 a3_inv(A3 a) {
  L3 il = linv(a.l);
  return a3(il, neg(lmul(il, a.p)));
}
static inline int a3_is_one(A3 a) {
  A3 o = a3_one();
  return veq(a.l.vx, o.l.vx) && veq(a.l.vy, o.l.vy) && veq(a.l.vz, o.l.vz) && veq(a.p, o.p);
}
static inline A3 a3_from12(const float* f) {
  return a3(l3(v3(f[0], f[1], f[2]), v3(f[3], f[4], f[5]), v3(f[6], f[7], f[8])), v3(f[9], f[10], f[11]));
}

/* ====================================================================== frame blob */
typedef struct {
  char name[96];
  uint32_t type;
  int32_t i[4];
  float f[12];
  char* str;
  int obj;
  char dtype[16];
  uint32_t count, esize;
  const uint8_t* data;
} Parm;
typedef struct {
  uint32_t kind;
  char type[64];
  int nparms;
  Parm* parms;
  int imgW, imgH, imgFmt;
  const uint8_t* img;
} Obj;
typedef struct {
  int present, shape, light, material;
  float xfm[12];
  int faceCamera, illumMask, shadowMask;
} Slot;
typedef struct {
  Obj* objs;
  int nobj;
  Slot* slots;
  int nslots;
  int renderer, camera;
  uint32_t seed;
} Blob;

enum { K_CAMERA = 0, K_DATA, K_IMAGE, K_TEXTURE, K_MATERIAL, K_SHAPE, K_LIGHT };
enum { VT_BOOL1 = 1, VT_INT4 = 8, VT_FLOAT1 = 9, VT_FLOAT2 = 10, VT_FLOAT3 = 11, VT_FLOAT4 = 12, VT_STRING = 13,
       VT_IMAGE = 14, VT_TEXTURE = 15, VT_TRANSFORM = 16, VT_DATA = 18 };

typedef struct { const uint8_t* p; const uint8_t* e; int bad; } Rd;
static uint32_t rd_u32(Rd* r) {
  uint32_t v = 0;
  if (r->p + 4 > r->e) { r->bad = 1; return 0; }
  memcpy(&v, r->p, 4);
  r->p += 4;
  return v;
}
static float rd_f32(Rd* r) { uint32_t u = rd_u32(r); float f; memcpy(&f, &u, 4); return f; }
static void rd_str(Rd* r, char* dst, size_t cap, char** heap) {
  uint32_t n = rd_u32(r);
  if (r->p + n > r->e) { r->bad = 1; return; }
  if (heap) {
    *heap = (char*)malloc(n + 1);
    memcpy(*heap, r->p, n);
    (*heap)[n] = 0;
  }
  if (dst) {
    size_t m = n < cap - 1 ? n : cap - 1;
    memcpy(dst, r->p, m);
    dst[m] = 0;
  }
  r->p += n;
}

static void blob_free(Blob* b) {
  if (!b) return;
  for (int i = 0; i < b->nobj; ++i) {
    for (int k = 0; k < b->objs[i].nparms; ++k) free(b->objs[i].parms[k].str);
    free(b->objs[i].parms);
  }
  free(b->objs);
  free(b->slots);
}

static int blob_parse(const void* data, size_t bytes, Blob* b) {
  memset(b, 0, sizeof(*b));
  Rd r = {(const uint8_t*)data, (const uint8_t*)data + bytes, 0};
  if (bytes < 8 || memcmp(data, "YRTF", 4)) return fail("not a frame blob");
  r.p += 4;
  if (rd_u32(&r) != 1) return fail("unsupported blob version");
  b->nobj = (int)rd_u32(&r);
  b->objs = (Obj*)calloc(b->nobj ? b->nobj : 1, sizeof(Obj));
  for (int i = 0; i < b->nobj && !r.bad; ++i) {
    Obj* o = &b->objs[i];
    o->kind = rd_u32(&r);
    rd_str(&r, o->type, sizeof(o->type), NULL);
    o->nparms = (int)rd_u32(&r);
    o->parms = (Parm*)calloc(o->nparms ? o->nparms : 1, sizeof(Parm));
    for (int k = 0; k < o->nparms && !r.bad; ++k) {
      Parm* p = &o->parms[k];
      rd_str(&r, p->name, sizeof(p->name), NULL);
      p->type = rd_u32(&r);
      p->obj = -1;
      if (p->type >= 1 && p->type <= 8) {
        for (int j = 0; j < 4; ++j) p->i[j] = (int32_t)rd_u32(&r);
      } else if (p->type >= 9 && p->type <= 12) {
        for (int j = 0; j < 4; ++j) p->f[j] = rd_f32(&r);
      } else if (p->type == VT_STRING) {
        rd_str(&r, NULL, 0, &p->str);
      } else if (p->type == VT_IMAGE || p->type == VT_TEXTURE) {
        p->obj = (int32_t)rd_u32(&r);
      } else if (p->type == VT_TRANSFORM) {
        for (int j = 0; j < 12; ++j) p->f[j] = rd_f32(&r);
      } else if (p->type == VT_DATA) {
        rd_str(&r, p->dtype, sizeof(p->dtype), NULL);
        p->count = rd_u32(&r);
        p->esize = rd_u32(&r);
        p->data = r.p;
        r.p += (size_t)p->count * p->esize;
        if (r.p > r.e) r.bad = 1;
      } else {
        r.bad = 1;
      }
    }
    if (o->kind == K_IMAGE) {
      o->imgW = (int)rd_u32(&r);
      o->imgH = (int)rd_u32(&r);
      o->imgFmt = (int)rd_u32(&r);
      uint32_t n = rd_u32(&r);
      o->img = r.p;
      r.p += n;
      if (r.p > r.e) r.bad = 1;
    }
  }
  b->nslots = (int)rd_u32(&r);
  b->slots = (Slot*)calloc(b->nslots ? b->nslots : 1, sizeof(Slot));
  for (int i = 0; i < b->nslots && !r.bad; ++i) {
    Slot* s = &b->slots[i];
    s->present = (int)rd_u32(&r);
    if (!s->present) continue;
    s->shape = (int32_t)rd_u32(&r);
    s->light = (int32_t)rd_u32(&r);
    s->material = (int32_t)rd_u32(&r);
    for (int j = 0; j < 12; ++j) s->xfm[j] = rd_f32(&r);
    s->faceCamera = (int)rd_u32(&r);
    s->illumMask = (int32_t)rd_u32(&r);
    s->shadowMask = (int32_t)rd_u32(&r);
  }
  b->renderer = (int32_t)rd_u32(&r);
  b->camera = (int32_t)rd_u32(&r);
  b->seed = rd_u32(&r);
  if (r.bad) { blob_free(b); return fail("truncated frame blob"); }
  return 0;
}

/* Parms getters with defaults (api/parms.h) */
static const Parm* pfind(const Obj* o, const char* n) {
  for (int i = 0; i < o->nparms; ++i)
    if (!strcmp(o->parms[i].name, n)) return &o->parms[i];
  return NULL;
}
static int p_int(const Obj* o, const char* n, int d) {
  const Parm* p = pfind(o, n);
  if (!p) return d;
  if (p->type >= 1 && p->type <= 8) return p->i[0];
  if (p->type == VT_FLOAT1) return (int)p->f[0];
  return d;
}
static float p_float(const Obj* o, const char* n, float d) {
  const Parm* p = pfind(o, n);
  if (!p) return d;
  if (p->type == VT_FLOAT1) return p->f[0];
  if (p->type >= 1 && p->type <= 8) return (float)p->i[0];
  return d;
}
static V3 p_v3(const Obj* o, const char* n, V3 d) {
  const Parm* p = pfind(o, n);
  return (p && p->type == VT_FLOAT3) ? v3(p->f[0], p->f[1], p->f[2]) : d;
}
static void p_v2(const Obj* o, const char* n, float* out, float dx, float dy) {
  const Parm* p = pfind(o, n);
  if (p && p->type == VT_FLOAT2) { out[0] = p->f[0]; out[1] = p->f[1]; }
  else { out[0] = dx; out[1] = dy; }
}
static const char* p_str(const Obj* o, const char* n, const char* d) {
  const Parm* p = pfind(o, n);
  return (p && p->type == VT_STRING) ? p->str : d;
}
static A3 p_xfm(const Obj* o, const char* n, A3 d) {
  const Parm* p = pfind(o, n);
  return (p && p->type == VT_TRANSFORM) ? a3_from12(p->f) : d;
}
static int p_obj(const Obj* o, const char* n) {
  const Parm* p = pfind(o, n);
  return (p && (p->type == VT_IMAGE || p->type == VT_TEXTURE)) ? p->obj : -1;
}

/* ====================================================================== scene objects */
enum { MT_NONE = 0, MT_MATTE, MT_MATTE_TEX, MT_METALLIC, MT_OBJ, MT_UBER, MT_THIN, MT_PLASTIC, MT_DIELECTRIC,
       MT_MIRROR, MT_METAL, MT_BRUSHED, MT_VELVET };
/* materials/medium.h: transmission + refraction index, compared by value */
typedef struct { V3 T; float eta; } Medium;
static inline int med_eq(Medium a, Medium b) { return veq(a.T, b.T) && a.eta == b.eta; }
typedef struct {
  int type;
  V3 reflectance;                               /* Matte */
  int Kd;                                       /* texture object index, -1 */
  float s0[2], ds[2];
  V3 shadeColor, glitterColor; float glitterSpread;  /* MetallicPaint */
  float eta;
  float d; V3 KdC, Ks; float Ns;                /* Obj */
  int map_d, map_Kd, map_Ks, map_Ns, map_Bump;
  V3 diffuse; float roughness, reflectivity, rcpRoughness;  /* Uber */
  V3 transmission; float thickness, transparency;           /* ThinDielectric */
  V3 pigment;                                               /* Plastic (eta, roughness shared) */
  Medium outside, inside;                                   /* Dielectric */
  V3 metalEta, metalK; float roughnessX, roughnessY;        /* Metal / BrushedMetal (reflectance) */
  float backScattering, fallOff; V3 horizon;                /* Velvet (reflectance) */
} Material;

enum { GK_FULL = 0, GK_NORMALS = 1, GK_TRIANGLE = 2 };
typedef struct {
  int kind;
  int nv, nt;
  V3* pos;
  V3* nor;   /* NULL if none */
  float* uv; /* NULL if none */
  int* tri;
  int cull;
  V3 Ng;
  V3* mot;             /* per-vertex motion (TriangleMeshFull "motions", Sphere dPdt), NULL if none */
  V3 *tanX, *tanY;     /* per-vertex tangents ("tangent_x", "tangent_y"), NULL if none */
} Mesh;

enum { LT_AMBIENT = 0, LT_TRIANGLE = 1, LT_HDRI = 2, LT_POINT = 3, LT_SPOT = 4, LT_DIRECTIONAL = 5, LT_DISTANT = 6 };
typedef struct {
  int type;
  V3 L, v0, v1, v2, e1, e2, Ng;
  A3 l2w, w2l;
  int img; /* blob image object, -1 = default 5x5 Image3f(one) */
  int w, h;
  float *ycdf, *ypdf, *xcdf, *xpdf;
  int illumMask, shadowMask;
  int precomp; /* slot or -1 */
  V3 P, D;     /* point/spot position; spot _D, directional/distant _wo */
  float cosMin, cosMax, halfAngle, cosHalf;
} Light;

typedef struct {
  Mesh* mesh; /* world */
  int material, light, illumMask, shadowMask, triBase;
} Geom;

typedef struct {
  float lo[3], hi[3];
  int left, right; /* inner: child indices; leaf: left = -1 - first, right = count */
} BNode;

typedef struct {
  const Blob* blob;
  Material* mats; int nmats;
  Mesh** meshes; int nmeshes;
  Geom* geoms; int ngeoms;
  Light* lights; int nlights;
  int* env; int nenv;
  int ntris;
  int* triGeom;
  float* tv;      /* 9 floats per tri: v0 v1 v2 */
  uint32_t* tflags;
  V3 *te0, *te1, *te2;  /* v0, e1=v0-v1, e2=v2-v0 */
  V3 *tm;               /* 3 motion vectors per tri (NULL: no moving geometry in the scene) */
  BNode* nodes; int nnodes;
  int* order;
} World;

/* ---------------------------------------------------------------- images / textures */
static void img_get(const Blob* B, int img, int x, int y, float c[4]) {
  if (img < 0) { c[0] = c[1] = c[2] = c[3] = 1.0f; return; }
  const Obj* o = &B->objs[img];
  if (o->imgFmt == 1) {
    const float* f = (const float*)o->img + ((size_t)y * o->imgW + x) * 4;
    c[0] = f[0]; c[1] = f[1]; c[2] = f[2]; c[3] = f[3];
    return;
  }
  const float one_over_255 = 1.f / 255.f; /* common/sys/constants.h:28 */
  const uint8_t* p = o->img + ((size_t)y * o->imgW + x) * 4;
  c[0] = p[0] * one_over_255; c[1] = p[1] * one_over_255; c[2] = p[2] * one_over_255;
  c[3] = o->imgFmt == 2 ? 1.0f : p[3] * one_over_255;
}

/* Bilinear::get (textures/Bilinear.h:8-25), NearestNeighbor::get (nearestneighbor.h:25-32) */
static void tex_get(const Blob* B, int texObj, float px, float py, float out[4]) {
  const Obj* t = &B->objs[texObj];
  const int img = p_obj(t, "image");
  const int invert = p_int(t, "invert", 0);
  const Obj* im = &B->objs[img];
  const int W = im->imgW, H = im->imgH;
  const float s1 = px - floorf(px), t1 = py - floorf(py);
  float c[4];
  if (!strcasecmp(t->type, "bilinear")) {
    const float u = s1 * W - .5f, v = t1 * H - .5f;
    int x = (int)floorf(u), y = (int)floorf(v);
    x = x < 0 ? 0 : (x > W - 2 ? W - 2 : x);
    y = y < 0 ? 0 : (y > H - 2 ? H - 2 : y);
    const float ur = u - x, vr = v - y, uo = 1.f - ur, vo = 1.f - vr;
    float a[4], b[4], cc[4], d[4];
    img_get(B, img, x, y, a); img_get(B, img, x + 1, y, b);
    img_get(B, img, x, y + 1, cc); img_get(B, img, x + 1, y + 1, d);
    for (int k = 0; k < 4; ++k) c[k] = (a[k] * uo + b[k] * ur) * vo + (cc[k] * uo + d[k] * ur) * vr;
  } else {
    const int si = (int)(s1 * (float)W), ti = (int)(t1 * (float)H);
    const int ix = si < 0 ? 0 : (si > W - 1 ? W - 1 : si);
    const int iy = ti < 0 ? 0 : (ti > H - 1 ? H - 1 : ti);
    img_get(B, img, ix, iy, c);
  }
  for (int k = 0; k < 4; ++k) out[k] = invert ? 1.f - c[k] : c[k];
}

/* ---------------------------------------------------------------- distributions
 * Distribution1D (samplers/distribution1d.cpp:42-74), Distribution2D (distribution2d.cpp:34-68) */
static void d1_init(const float* f, int n, float* cdf, float* pdf) {
  cdf[0] = 0.0f;
  for (int i = 1; i < n + 1; i++) cdf[i] = cdf[i - 1] + f[i - 1];
  float rs = cdf[n] == 0.0f ? 0.0f : rcp(cdf[n]);
  for (int i = 1; i < n + 1; i++) {
    pdf[i - 1] = f[i - 1] * rs * (float)n;
    cdf[i] *= rs;
  }
  cdf[n] = 1.0f;
}
static void d1_sample(const float* cdf, const float* pdf, int n, float u, float* x, float* p) {
  /* std::upper_bound(CDF, CDF+size, u): first element > u */
  int lo = 0, hi = n;
  while (lo < hi) {
    int mid = (lo + hi) / 2;
    if (!(u < cdf[mid])) lo = mid + 1; else hi = mid;
  }
  int idx = lo - 1;
  idx = idx < 0 ? 0 : (idx > n - 1 ? n - 1 : idx);
  float frac = (u - cdf[idx]) * rcp(cdf[idx + 1] - cdf[idx]);
  *x = (float)idx + frac;
  *p = pdf[idx];
}
typedef struct { int w, h; float *ycdf, *ypdf, *xcdf, *xpdf; } Dist2;
static void d2_init(Dist2* d, const float* f /* [h][w] */, int w, int h) {
  d->w = w; d->h = h;
  d->ycdf = (float*)malloc(sizeof(float) * (h + 1));
  d->ypdf = (float*)malloc(sizeof(float) * h);
  d->xcdf = (float*)malloc(sizeof(float) * (size_t)h * (w + 1));
  d->xpdf = (float*)malloc(sizeof(float) * (size_t)h * w);
  float* fy = (float*)malloc(sizeof(float) * h);
  for (int y = 0; y < h; y++) {
    fy[y] = 0.0f;
    for (int x = 0; x < w; x++) fy[y] += f[(size_t)y * w + x];
    d1_init(f + (size_t)y * w, w, d->xcdf + (size_t)y * (w + 1), d->xpdf + (size_t)y * w);
  }
  d1_init(fy, h, d->ycdf, d->ypdf);
  free(fy);
}
static void d2_sample(const Dist2* d, float ux, float uy, float* sx, float* sy, float* pdf) {
  float px, py;
  d1_sample(d->ycdf, d->ypdf, d->h, uy, sy, &py);
  int y = (int)*sy;
  y = y < 0 ? 0 : (y > d->h - 1 ? d->h - 1 : y);
  d1_sample(d->xcdf + (size_t)y * (d->w + 1), d->xpdf + (size_t)y * d->w, d->w, ux, sx, &px);
  *pdf = px * py;
}
static void d2_free(Dist2* d) { free(d->ycdf); free(d->ypdf); free(d->xcdf); free(d->xpdf); }

/* ---------------------------------------------------------------- object construction */
static void mat_build(const Blob* B, int oi, Material* m) {
  memset(m, 0, sizeof(*m));
  m->Kd = m->map_d = m->map_Kd = m->map_Ks = m->map_Ns = m->map_Bump = -1;
  if (oi < 0) { m->type = MT_NONE; return; }
  const Obj* o = &B->objs[oi];
  const char* t = o->type;
  if (!strcasecmp(t, "Matte")) { /* materials/matte.h:16-18 */
    m->type = MT_MATTE;
    m->reflectance = p_v3(o, "reflectance", vs(1.0f));
  } else if (!strcasecmp(t, "MatteTextured")) { /* matte_textured.h:17-22 */
    m->type = MT_MATTE_TEX;
    m->Kd = p_obj(o, "Kd");
    p_v2(o, "s0", m->s0, 0.f, 0.f);
    p_v2(o, "ds", m->ds, 1.f, 1.f);
  } else if (!strcasecmp(t, "MetallicPaint")) { /* metallicpaint.h:23-34 */
    m->type = MT_METALLIC;
    m->shadeColor = p_v3(o, "shadeColor", vs(1.0f));
    m->glitterColor = p_v3(o, "glitterColor", vs(0.0f));
    m->glitterSpread = p_float(o, "glitterSpread", 1.0f);
    m->eta = p_float(o, "eta", 1.4f);
  } else if (!strcasecmp(t, "Obj")) { /* obj.h:17-33 */
    m->type = MT_OBJ;
    m->map_d = p_obj(o, "map_d"); m->d = p_float(o, "d", 1.0f);
    m->map_Kd = p_obj(o, "map_Kd"); m->KdC = p_v3(o, "Kd", vs(1.0f));
    m->map_Ks = p_obj(o, "map_Ks"); m->Ks = p_v3(o, "Ks", vs(0.0f));
    m->map_Ns = p_obj(o, "map_Ns"); m->Ns = p_float(o, "Ns", 10.0f);
    m->map_Bump = p_obj(o, "map_Bump");
  } else if (!strcasecmp(t, "Uber")) { /* Uber.h:5-15 */
    m->type = MT_UBER;
    m->Kd = p_obj(o, "Kd");
    m->diffuse = p_v3(o, "diffuse", vs(0.0f));
    p_v2(o, "s0", m->s0, 0.f, 0.f);
    p_v2(o, "ds", m->ds, 1.f, 1.f);
    m->eta = p_float(o, "eta", 1.4f);
    m->roughness = p_float(o, "roughness", .9f);
    m->reflectivity = p_float(o, "reflectivity", .0f);
    m->rcpRoughness = rcp(m->roughness);
  } else if (!strcasecmp(t, "ThinDielectric") || !strcasecmp(t, "ThinGlass")) { /* thindielectric.h:18-26 */
    m->type = MT_THIN;
    m->Kd = p_obj(o, "Kd");
    p_v2(o, "s0", m->s0, 0.f, 0.f);
    p_v2(o, "ds", m->ds, 1.f, 1.f);
    m->transmission = p_v3(o, "transmission", vs(1.0f));
    m->eta = p_float(o, "eta", 1.4f);
    m->thickness = p_float(o, "thickness", .1f);
    m->transparency = p_float(o, "transparency", 1.f);
  } else if (!strcasecmp(t, "Plastic")) { /* plastic.h:21-26 */
    m->type = MT_PLASTIC;
    m->pigment = p_v3(o, "pigmentColor", vs(1.0f));
    m->eta = p_float(o, "eta", 1.4f);
    m->roughness = p_float(o, "roughness", 0.01f);
    m->rcpRoughness = rcp(m->roughness);
  } else if (!strcasecmp(t, "Dielectric") || !strcasecmp(t, "Glass")) { /* dielectric.h:13-27 */
    m->type = MT_DIELECTRIC;
    m->outside.eta = p_float(o, "etaOutside", 1.0f);
    m->inside.eta = p_float(o, "etaInside", 1.4f);
    m->outside.T = p_v3(o, "transmissionOutside", vs(1.0f));
    m->inside.T = p_v3(o, "transmission", vs(1.0f));
  } else if (!strcasecmp(t, "Mirror")) { /* mirror.h:15-17 */
    m->type = MT_MIRROR;
    m->reflectance = p_v3(o, "reflectance", vs(1.0f));
  } else if (!strcasecmp(t, "Metal")) { /* metal.h:18-24 */
    m->type = MT_METAL;
    m->reflectance = p_v3(o, "reflectance", vs(1.0f));
    m->metalEta = p_v3(o, "eta", vs(1.4f));
    m->metalK = p_v3(o, "k", vs(0.0f));
    m->roughness = p_float(o, "roughness", 0.01f);
    m->rcpRoughness = rcp(m->roughness);
  } else if (!strcasecmp(t, "BrushedMetal")) { /* brushedmetal.h:19-27 */
    m->type = MT_BRUSHED;
    m->reflectance = p_v3(o, "reflectance", vs(1.0f));
    m->metalEta = p_v3(o, "eta", vs(1.4f));
    m->metalK = p_v3(o, "k", vs(0.0f));
    m->roughnessX = p_float(o, "roughnessX", 0.01f);
    m->roughnessY = p_float(o, "roughnessY", 0.01f);
  } else if (!strcasecmp(t, "Velvet")) { /* velvet.h:16-21 */
    m->type = MT_VELVET;
    m->reflectance = p_v3(o, "reflectance", vs(1.0f));
    m->backScattering = p_float(o, "backScattering", 0.0f);
    m->horizon = p_v3(o, "horizonScatteringColor", vs(1.0f));
    m->fallOff = p_float(o, "horizonScatteringFallOff", 0.0f);
  } else {
    m->type = MT_NONE;
  }
}

static Mesh* mesh_new(void) { return (Mesh*)calloc(1, sizeof(Mesh)); }
static void mesh_free(Mesh* m) {
  if (!m) return;
  free(m->pos); free(m->nor); free(m->uv); free(m->tri); free(m->mot); free(m->tanX); free(m->tanY); free(m);
}

static Mesh* shape_build(const Blob* B, int oi) {
  const Obj* o = &B->objs[oi];
  Mesh* m = mesh_new();
  if (!strcasecmp(o->type, "trianglemesh")) { /* shapes/trianglemesh.h:14-26 */
    const Parm *pos = pfind(o, "positions"), *nor = pfind(o, "normals"), *tc = pfind(o, "texcoords"),
               *tc0 = pfind(o, "texcoords0"), *idx = pfind(o, "indices"), *mot = pfind(o, "motions"),
               *tx = pfind(o, "tangent_x"), *ty = pfind(o, "tangent_y");
    const int withNormals = pos && !mot && nor && !tx && !ty && !tc && !tc0;
    m->kind = withNormals ? GK_NORMALS : GK_FULL;
    if (pos) {
      m->nv = (int)pos->count;
      m->pos = (V3*)malloc(sizeof(V3) * (m->nv ? m->nv : 1));
      for (int i = 0; i < m->nv; ++i) memcpy(&m->pos[i], pos->data + (size_t)i * pos->esize, 12);
    }
    if (nor) {
      m->nor = (V3*)malloc(sizeof(V3) * (nor->count ? nor->count : 1));
      for (uint32_t i = 0; i < nor->count; ++i) memcpy(&m->nor[i], nor->data + (size_t)i * nor->esize, 12);
      if (withNormals) m->nv = (int)nor->count; /* vertices.resize(normals) */
    }
    /* per-vertex vec3 arrays read at vertex count (a shorter array is an out-of-bounds read in
     * the reference; the device rejects it, so a blob never carries one) */
#define RD3(P, DST)                                                                   \
    if (P) {                                                                          \
      DST = (V3*)calloc((size_t)(m->nv > (int)(P)->count ? m->nv : (int)(P)->count) + 1, sizeof(V3)); \
      for (uint32_t i = 0; i < (P)->count; ++i) memcpy(&DST[i], (P)->data + (size_t)i * (P)->esize, 12); \
    }
    RD3(mot, m->mot)
    RD3(tx, m->tanX)
    RD3(ty, m->tanY)
#undef RD3
    const Parm* t = tc0 ? tc0 : tc;
    if (t) {
      m->uv = (float*)malloc(sizeof(float) * 2 * (t->count ? t->count : 1));
      for (uint32_t i = 0; i < t->count; ++i) memcpy(&m->uv[2 * i], t->data + (size_t)i * t->esize, 8);
    }
    if (idx) {
      m->nt = (int)idx->count;
      m->tri = (int*)malloc(sizeof(int) * 3 * (m->nt ? m->nt : 1));
      for (int i = 0; i < m->nt; ++i) memcpy(&m->tri[3 * i], idx->data + (size_t)i * idx->esize, 12);
    }
    m->cull = p_int(o, "cullBackFaces", 0) != 0;
  } else if (!strcasecmp(o->type, "sphere")) { /* shapes/sphere.h:19-66 */
    m->kind = GK_FULL;
    const V3 P = p_v3(o, "P", vs(0.f));
    const float r = p_float(o, "r", 0.f);
    const int numTheta = p_int(o, "numTheta", 0), numPhi = p_int(o, "numPhi", 0);
    const V3 dPdt = p_v3(o, "dPdt", vs(0.f));
    m->nv = (numTheta + 1) * numPhi;
    if (!v3zero(dPdt)) { /* sphere.h:67: one motion vector per vertex */
      m->mot = (V3*)malloc(sizeof(V3) * (m->nv ? m->nv : 1));
      for (int i = 0; i < m->nv; ++i) m->mot[i] = dPdt;
    }
    m->pos = (V3*)malloc(sizeof(V3) * (m->nv ? m->nv : 1));
    m->nor = (V3*)malloc(sizeof(V3) * (m->nv ? m->nv : 1));
    m->uv = (float*)malloc(sizeof(float) * 2 * (m->nv ? m->nv : 1));
    m->tri = (int*)malloc(sizeof(int) * 6 * (size_t)(numTheta + 1) * (numPhi + 1));
    int v = 0, t = 0;
    for (int theta = 0; theta <= numTheta; theta++) {
      const float rcpNumTheta = rcp((float)numTheta);
      for (int phi = 0; phi < numPhi; phi++) {
        const float rcpNumPhi = rcp((float)numPhi);
#define SPH(th, ph) v3(sinf(th) * cosf(ph), cosf(th), sinf(th) * sinf(ph))
        const float th0 = (float)theta * PI_F * rcpNumTheta, ph0 = (float)phi * 2.0f * PI_F * rcpNumPhi;
        V3 p = SPH(th0, ph0);
        const float th1 = ((float)theta + 0.001f) * PI_F * rcpNumTheta;
        const float ph1 = ((float)phi + 0.001f) * 2.0f * PI_F * rcpNumPhi;
        V3 dpdu = sub(SPH(th1, ph0), p);
        V3 dpdv = sub(SPH(th0, ph1), p);
#undef SPH
        p = add(muls(p, r), P);
        m->pos[v] = p;
        m->nor[v] = normalize(cross(dpdv, dpdu));
        m->uv[2 * v] = (float)phi * rcpNumPhi;
        m->uv[2 * v + 1] = (float)theta * rcpNumTheta;
        v++;
      }
      if (theta == 0) continue;
      for (int phi = 1; phi <= numPhi; phi++) {
        const int p00 = (theta - 1) * numPhi + phi - 1, p01 = (theta - 1) * numPhi + phi % numPhi;
        const int p10 = theta * numPhi + phi - 1, p11 = theta * numPhi + phi % numPhi;
        if (theta > 1) { m->tri[3 * t] = p10; m->tri[3 * t + 1] = p00; m->tri[3 * t + 2] = p01; t++; }
        if (theta < numTheta) { m->tri[3 * t] = p11; m->tri[3 * t + 1] = p10; m->tri[3 * t + 2] = p01; t++; }
      }
    }
    m->nt = t;
  } else if (!strcasecmp(o->type, "disk")) { /* shapes/disk.h:33-65; apex normal (0,0,1), texcoord (0,0):
                                                 the reference reads them out of bounds (undefined) */
    m->kind = GK_FULL;
    const V3 P = p_v3(o, "P", vs(0.f));
    const float h = p_float(o, "h", 0.f), r = p_float(o, "r", 0.f);
    const int n = p_int(o, "numTriangles", 0);
    if (n < 1) { mesh_free(m); return NULL; }
    m->nv = n + 1;
    m->nt = n;
    m->pos = (V3*)malloc(sizeof(V3) * (size_t)(n + 1));
    m->nor = (V3*)malloc(sizeof(V3) * (size_t)(n + 1));
    m->uv = (float*)calloc(2 * (size_t)(n + 1), sizeof(float));
    m->tri = (int*)malloc(sizeof(int) * 3 * (size_t)n);
    const float rcpN = rcp((float)n);
    for (int phi = 0; phi < n; phi++) {
      const V3 d = v3(sinf((float)phi * 2.0f * PI_F * rcpN), cosf((float)phi * 2.0f * PI_F * rcpN), 0.0f);
      m->pos[phi] = add(P, muls(d, r));
      m->nor[phi] = v3(0.f, 0.f, 1.f);
    }
    m->pos[n] = add(P, v3(0.f, 0.f, h));
    m->nor[n] = v3(0.f, 0.f, 1.f);
    for (int phi = 0; phi < n; phi++) {
      const int p0 = n, p1 = phi % n, p2 = (phi + 1) % n;
      int* t = &m->tri[3 * phi];
      if (phi % 3 == 0) { t[0] = p0; t[1] = p2; t[2] = p1; }
      else if (phi % 3 == 1) { t[0] = p1; t[1] = p0; t[2] = p2; }
      else { t[0] = p2; t[1] = p1; t[2] = p0; }
    }
  } else if (!strcasecmp(o->type, "triangle")) {
    m->kind = GK_TRIANGLE;
    m->nv = 3;
    m->nt = 1;
    m->pos = (V3*)malloc(sizeof(V3) * 3);
    m->pos[0] = p_v3(o, "v0", vs(0.f));
    m->pos[1] = p_v3(o, "v1", vs(0.f));
    m->pos[2] = p_v3(o, "v2", vs(0.f));
    m->tri = (int*)malloc(sizeof(int) * 3);
    m->tri[0] = 0; m->tri[1] = 1; m->tri[2] = 2;
  } else {
    mesh_free(m);
    return NULL;
  }
  return m;
}

static Mesh* triangle_mesh(V3 a, V3 b, V3 c) {
  Mesh* m = mesh_new();
  m->kind = GK_TRIANGLE;
  m->nv = 3; m->nt = 1;
  m->pos = (V3*)malloc(sizeof(V3) * 3);
  m->pos[0] = a; m->pos[1] = b; m->pos[2] = c;
  m->tri = (int*)malloc(sizeof(int) * 3);
  m->tri[0] = 0; m->tri[1] = 1; m->tri[2] = 2;
  return m;
}

/* Shape::transform (trianglemesh_full.cpp:53-75, trianglemesh_normals.cpp:28-42, triangle.h:32-34) */
static Mesh* mesh_transform(const Mesh* s, A3 x) {
  Mesh* m = mesh_new();
  *m = *s;
  m->pos = (V3*)malloc(sizeof(V3) * (s->nv ? s->nv : 1));
  memcpy(m->pos, s->pos, sizeof(V3) * s->nv);
  m->nor = NULL;
  if (s->nor) {
    m->nor = (V3*)malloc(sizeof(V3) * (s->nv ? s->nv : 1));
    memcpy(m->nor, s->nor, sizeof(V3) * s->nv);
  }
  m->uv = NULL;
  if (s->uv) {
    m->uv = (float*)malloc(sizeof(float) * 2 * (s->nv ? s->nv : 1));
    memcpy(m->uv, s->uv, sizeof(float) * 2 * s->nv);
  }
  m->tri = (int*)malloc(sizeof(int) * 3 * (s->nt ? s->nt : 1));
  memcpy(m->tri, s->tri, sizeof(int) * 3 * s->nt);
  V3** vecs[3] = {&m->mot, &m->tanX, &m->tanY};
  const V3* src[3] = {s->mot, s->tanX, s->tanY};
  for (int k = 0; k < 3; ++k) {
    *vecs[k] = NULL;
    if (src[k]) {
      *vecs[k] = (V3*)malloc(sizeof(V3) * (s->nv ? s->nv : 1));
      memcpy(*vecs[k], src[k], sizeof(V3) * s->nv);
    }
  }
  if (s->kind == GK_TRIANGLE) {
    for (int i = 0; i < 3; ++i) m->pos[i] = xfmPoint(x, s->pos[i]);
    m->Ng = normalize(cross(sub(m->pos[2], m->pos[0]), sub(m->pos[1], m->pos[0])));
    return m;
  }
  if (a3_is_one(x)) return m;
  for (int i = 0; i < m->nv; ++i) m->pos[i] = xfmPoint(x, s->pos[i]);
  if (m->nor)
    for (int i = 0; i < m->nv; ++i) m->nor[i] = xfmNormal(x, s->nor[i]);
  /* trianglemesh_full.cpp:79-85: motions and tangents are vectors */
  for (int k = 0; k < 3; ++k)
    if (*vecs[k])
      for (int i = 0; i < m->nv; ++i) (*vecs[k])[i] = xfmVector(x, src[k][i]);
  return m;
}

/* Light ctors + transform (lights/ambientlight.h:24-42, trianglelight.h:16-49, hdrilight.cpp:8-41) */
static int light_build(const Blob* B, int oi, A3 xfm, int illum, int shadow, Light* L, Mesh** shapeOut) {
  const Obj* o = &B->objs[oi];
  memset(L, 0, sizeof(*L));
  L->illumMask = illum;
  L->shadowMask = shadow;
  L->precomp = -1;
  L->img = -1;
  *shapeOut = NULL;
  if (!strcasecmp(o->type, "ambientlight")) {
    L->type = LT_AMBIENT;
    L->L = p_v3(o, "L", vs(0.f));
  } else if (!strcasecmp(o->type, "trianglelight")) {
    L->type = LT_TRIANGLE;
    V3 a = p_v3(o, "v0", vs(0.f)), b = p_v3(o, "v1", vs(0.f)), c = p_v3(o, "v2", vs(0.f));
    L->L = p_v3(o, "L", vs(0.f));
    L->v0 = xfmPoint(xfm, a);
    L->v1 = xfmPoint(xfm, b);
    L->v2 = xfmPoint(xfm, c);
    L->e1 = sub(L->v0, L->v1);
    L->e2 = sub(L->v2, L->v0);
    L->Ng = cross(L->e1, L->e2);
    Mesh* s = triangle_mesh(a, b, c);
    *shapeOut = mesh_transform(s, xfm);
    mesh_free(s);
  } else if (!strcasecmp(o->type, "hdrilight")) {
    L->type = LT_HDRI;
    A3 l2w = p_xfm(o, "local2world", a3_one());
    L->L = p_v3(o, "L", vs(1.f));
    L->img = p_obj(o, "image");
    L->w = L->img >= 0 ? B->objs[L->img].imgW : 5;
    L->h = L->img >= 0 ? B->objs[L->img].imgH : 5;
    float* imp = (float*)malloc(sizeof(float) * L->w * L->h);
    for (int y = 0; y < L->h; y++)
      for (int x = 0; x < L->w; x++) {
        float c[4];
        img_get(B, L->img, x, y, c);
        imp[(size_t)y * L->w + x] = sinf(PI_F * (y + 0.5f) * rcp((float)L->h)) * (c[0] + c[1] + c[2]);
      }
    Dist2 d;
    d2_init(&d, imp, L->w, L->h);
    free(imp);
    L->ycdf = d.ycdf; L->ypdf = d.ypdf; L->xcdf = d.xcdf; L->xpdf = d.xpdf;
    L->l2w = aamul(xfm, l2w);
    L->w2l = a3_inv(L->l2w);
  } else if (!strcasecmp(o->type, "pointlight")) { /* pointlight.h:24-34 */
    L->type = LT_POINT;
    L->P = xfmPoint(xfm, p_v3(o, "P", vs(0.f)));
    L->L = p_v3(o, "I", vs(0.f));
  } else if (!strcasecmp(o->type, "spotlight")) { /* spotlight.h:24-39 */
    L->type = LT_SPOT;
    L->P = xfmPoint(xfm, p_v3(o, "P", vs(0.f)));
    L->D = xfmVector(xfm, neg(normalize(p_v3(o, "D", vs(0.f)))));
    L->L = p_v3(o, "I", vs(0.f));
    L->cosMin = cosf(0.5f * deg2rad(p_float(o, "angleMin", 0.f)));
    L->cosMax = cosf(0.5f * deg2rad(p_float(o, "angleMax", 0.f)));
  } else if (!strcasecmp(o->type, "directionallight")) { /* directionallight.h:13-29 */
    L->type = LT_DIRECTIONAL;
    L->D = normalize(xfmVector(xfm, neg(normalize(p_v3(o, "D", vs(0.f))))));
    L->L = p_v3(o, "E", vs(0.f));
  } else if (!strcasecmp(o->type, "distantlight")) { /* distantlight.h:16-36 */
    L->type = LT_DISTANT;
    L->D = normalize(xfmVector(xfm, neg(normalize(p_v3(o, "D", vs(0.f))))));
    L->L = p_v3(o, "L", vs(0.f));
    L->halfAngle = deg2rad(p_float(o, "halfAngle", 0.f));
    L->cosHalf = cosf(L->halfAngle);
  } else {
    return -1;
  }
  return 0;
}

/* ---------------------------------------------------------------- oracle BVH (median split) */
/* bounds of triangle i over the frame time [0,1]: its vertices at t = 0 and t = 1 (p + m),
 * as the reference's extract() bounds motion meshes (trianglemesh_full.cpp:152-166) */
static void tri_box(const World* W, int i, float lo[3], float hi[3]) {
  const float* t = &W->tv[(size_t)i * 9];
  for (int k = 0; k < 3; ++k) { lo[k] = INFINITY; hi[k] = -INFINITY; }
  for (int v = 0; v < 3; ++v) {
    const float p[3] = {t[3 * v], t[3 * v + 1], t[3 * v + 2]};
    for (int k = 0; k < 3; ++k) { lo[k] = fminf(lo[k], p[k]); hi[k] = fmaxf(hi[k], p[k]); }
    if (W->tm) {
      const V3 m = W->tm[(size_t)i * 3 + v];
      const float q[3] = {p[0] + m.x, p[1] + m.y, p[2] + m.z};
      for (int k = 0; k < 3; ++k) { lo[k] = fminf(lo[k], q[k]); hi[k] = fmaxf(hi[k], q[k]); }
    }
  }
}
typedef struct { World* W; int* idx; float* cen; } BuildCtx;
static int cmp_axis;
static const float* cmp_cen;
static int cmp_fn(const void* a, const void* b) {
  float ca = cmp_cen[*(const int*)a * 3 + cmp_axis], cb = cmp_cen[*(const int*)b * 3 + cmp_axis];
  if (ca < cb) return -1;
  if (ca > cb) return 1;
  return (*(const int*)a) - (*(const int*)b);
}
static int bvh_rec(World* W, int* idx, const float* cen, int b, int e) {
  const int ni = W->nnodes++;
  BNode* n = &W->nodes[ni];
  for (int k = 0; k < 3; ++k) { n->lo[k] = INFINITY; n->hi[k] = -INFINITY; }
  for (int i = b; i < e; ++i) {
    float lo[3], hi[3];
    tri_box(W, idx[i], lo, hi);
    for (int k = 0; k < 3; ++k) {
      n->lo[k] = fminf(n->lo[k], lo[k]);
      n->hi[k] = fmaxf(n->hi[k], hi[k]);
    }
  }
  if (e - b <= 4) {
    n->left = -1 - b;
    n->right = e - b;
    return ni;
  }
  float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int i = b; i < e; ++i)
    for (int k = 0; k < 3; ++k) {
      clo[k] = fminf(clo[k], cen[idx[i] * 3 + k]);
      chi[k] = fmaxf(chi[k], cen[idx[i] * 3 + k]);
    }
  int ax = 0;
  for (int k = 1; k < 3; ++k)
    if (chi[k] - clo[k] > chi[ax] - clo[ax]) ax = k;
  cmp_axis = ax;
  cmp_cen = cen;
  qsort(idx + b, e - b, sizeof(int), cmp_fn);
  const int m = (b + e) / 2;
  const int l = bvh_rec(W, idx, cen, b, m);
  const int r = bvh_rec(W, idx, cen, m, e);
  W->nodes[ni].left = l;
  W->nodes[ni].right = r;
  return ni;
}
static void bvh_build_oracle(World* W) {
  W->nodes = (BNode*)calloc((size_t)2 * (W->ntris + 1), sizeof(BNode));
  W->nnodes = 0;
  W->order = (int*)malloc(sizeof(int) * (W->ntris ? W->ntris : 1));
  float* cen = (float*)malloc(sizeof(float) * 3 * (W->ntris ? W->ntris : 1));
  for (int i = 0; i < W->ntris; ++i) {
    W->order[i] = i;
    float lo[3], hi[3];
    tri_box(W, i, lo, hi);
    for (int k = 0; k < 3; ++k) cen[i * 3 + k] = 0.5f * (lo[k] + hi[k]);
  }
  if (W->ntris) bvh_rec(W, W->order, cen, 0, W->ntris);
  free(cen);
}

/* ---------------------------------------------------------------- ray / hit
 * Embree-convention Moeller-Trumbore (lights/trianglelight.h:55-65) with the cull filter
 * (trianglemesh_full.cpp:86-106); closest = smallest (t, gid). */
typedef struct { V3 org, dir; float tnear, tfar, time; } Ray;
typedef struct { float t, u, v; int tri; } Hit;

/* the triangle test's cross and dot products as separate multiplies and adds (two roundings per
 * term pair), in the order of the device's tri_cross / tri_dot (kernels/yrt_traverse.h) */
static inline V3 tri_cross(V3 a, V3 b) {
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline float tri_dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

static inline int tri_test(V3 v0, V3 e1, V3 e2, uint32_t flags, const Ray* r, float tfar, float* t, float* u,
                           float* v) {
  const V3 Ng = tri_cross(e1, e2);
  const V3 C = sub(v0, r->org);
  const V3 R = tri_cross(r->dir, C);
  const float den = tri_dot(Ng, r->dir);
  const float absDen = fabsf(den);
  const float sgn = den < 0.0f ? -1.0f : 1.0f;
  const float U = tri_dot(R, e2) * sgn;
  const float V = tri_dot(R, e1) * sgn;
  int ok = (den != 0.0f) && (U >= 0.0f) && (V >= 0.0f) && (U + V <= absDen);
  if ((flags & 1u) && !(den > 0.0f)) ok = 0;
  const float T = tri_dot(Ng, C) * sgn;
  *t = T / absDen;
  ok = ok && (*t > r->tnear) && (*t < tfar);
  *u = U / absDen;
  *v = V / absDen;
  return ok;
}

static inline int box_hit(const float* lo, const float* hi, const Ray* r, V3 inv, float tmax) {
  float l[3], h[3];
  const float o[3] = {r->org.x, r->org.y, r->org.z}, iv[3] = {inv.x, inv.y, inv.z};
  for (int k = 0; k < 3; ++k) {
    l[k] = (lo[k] - o[k]) * iv[k];
    h[k] = (hi[k] - o[k]) * iv[k];
  }
  const float n = fmaxf(fmaxf(fminf(l[0], h[0]), fminf(l[1], h[1])), fmaxf(fminf(l[2], h[2]), r->tnear));
  const float f = fminf(fminf(fmaxf(l[0], h[0]), fmaxf(l[1], h[1])), fminf(fmaxf(l[2], h[2]), tmax));
  return n <= f * 1.0000152587890625f; /* 1 + 2^-16, as the device (yrt_traverse.h YRT_BOX_ROBUST) */
}
static inline float safe_inv(float d) { return 1.0f / (fabsf(d) > 1e-20f ? d : copysignf(1e-20f, d)); }

static Hit trace(const World* W, const Ray* r, int any) {
  Hit best = {r->tfar, 0.f, 0.f, -1};
  if (!(r->tfar >= r->tnear) || W->ntris == 0) return best;
  const V3 inv = v3(safe_inv(r->dir.x), safe_inv(r->dir.y), safe_inv(r->dir.z));
  int stack[128], sp = 0;
  stack[sp++] = 0;
  while (sp) {
    const BNode* n = &W->nodes[stack[--sp]];
    if (!box_hit(n->lo, n->hi, r, inv, best.t)) continue;
    if (n->left < 0) {
      const int first = -1 - n->left;
      for (int i = first; i < first + n->right; ++i) {
        const int g = W->order[i];
        float t, u, v;
        V3 v0 = W->te0[g], e1 = W->te1[g], e2 = W->te2[g];
        if (W->tm) { /* the triangle at the ray's time: p += time * motion (trianglemesh_full.cpp:104-109) */
          const float* tv = &W->tv[(size_t)g * 9];
          const V3* m = &W->tm[(size_t)g * 3];
          const V3 p0 = add(v3(tv[0], tv[1], tv[2]), muls(m[0], r->time));
          const V3 p1 = add(v3(tv[3], tv[4], tv[5]), muls(m[1], r->time));
          const V3 p2 = add(v3(tv[6], tv[7], tv[8]), muls(m[2], r->time));
          v0 = p0; e1 = sub(p0, p1); e2 = sub(p2, p0);
        }
        int ok = tri_test(v0, e1, e2, W->tflags[g], r, any ? r->tfar : best.t, &t, &u, &v);
        if (any) {
          if (ok) { best.t = t; best.u = u; best.v = v; best.tri = g; return best; }
        } else {
          if (!ok && best.tri >= 0 && t == best.t && g < best.tri) {
            float t2, u2, v2;
            ok = tri_test(v0, e1, e2, W->tflags[g], r, r->tfar, &t2, &u2, &v2);
          }
          if (ok) { best.t = t; best.u = u; best.v = v; best.tri = g; }
        }
      }
    } else {
      stack[sp++] = n->right;
      stack[sp++] = n->left;
    }
  }
  return best;
}

/* ---------------------------------------------------------------- world build
 * BackendSceneFlat::Handle::setPrimitive/create (api/scene_flat.h:48-97) and ctor (:105-121) */
static void world_free(World* W) {
  for (int i = 0; i < W->nmeshes; ++i) mesh_free(W->meshes[i]);
  free(W->meshes);
  for (int i = 0; i < W->nlights; ++i) {
    free(W->lights[i].ycdf); free(W->lights[i].ypdf); free(W->lights[i].xcdf); free(W->lights[i].xpdf);
  }
  free(W->mats); free(W->geoms); free(W->lights); free(W->env); free(W->triGeom); free(W->tv); free(W->tflags);
  free(W->te0); free(W->te1); free(W->te2); free(W->tm); free(W->nodes); free(W->order);
}

static int world_build(const Blob* B, World* W) {
  memset(W, 0, sizeof(*W));
  W->blob = B;
  const int n = B->nslots;
  W->mats = (Material*)calloc(n + 1, sizeof(Material));
  W->meshes = (Mesh**)calloc(2 * n + 1, sizeof(Mesh*));
  W->geoms = (Geom*)calloc(n + 1, sizeof(Geom));
  W->lights = (Light*)calloc(n + 1, sizeof(Light));
  W->env = (int*)calloc(n + 1, sizeof(int));
  int* primLight = (int*)malloc(sizeof(int) * (n + 1));
  Mesh** primShape = (Mesh**)calloc(n + 1, sizeof(Mesh*));
  int npre = 0;
  for (int i = 0; i < n; ++i) {
    primLight[i] = -1;
    const Slot* s = &B->slots[i];
    if (!s->present) continue;
    const A3 x = a3_from12(s->xfm);
    if (s->light >= 0) {
      Light* L = &W->lights[W->nlights];
      Mesh* shape = NULL;
      if (light_build(B, s->light, x, s->illumMask, s->shadowMask, L, &shape)) {
        free(primLight); free(primShape);
        return fail("light type outside the oracle's scope");
      }
      /* EnvironmentLight subclasses (api/scene.h:76) */
      if (L->type == LT_AMBIENT || L->type == LT_HDRI || L->type == LT_DISTANT) W->env[W->nenv++] = W->nlights;
      if (L->type == LT_HDRI) L->precomp = npre++;
      primLight[i] = W->nlights++;
      primShape[i] = shape;
    } else if (s->shape >= 0) {
      Mesh* m = shape_build(B, s->shape);
      if (!m) { free(primLight); free(primShape); return fail("shape type outside the oracle's scope"); }
      primShape[i] = mesh_transform(m, x);
      mesh_free(m);
    }
  }
  int tb = 0;
  for (int i = 0; i < n; ++i) {
    if (!primShape[i]) continue;
    const Slot* s = &B->slots[i];
    Geom* g = &W->geoms[W->ngeoms];
    g->mesh = primShape[i];
    W->meshes[W->nmeshes++] = primShape[i];
    mat_build(B, s->material, &W->mats[W->ngeoms]);
    g->material = W->ngeoms;
    g->light = primLight[i];
    g->illumMask = s->illumMask;
    g->shadowMask = s->shadowMask;
    g->triBase = tb;
    tb += g->mesh->nt;
    W->ngeoms++;
  }
  free(primLight);
  free(primShape);
  W->ntris = tb;
  const int nt = tb ? tb : 1;
  W->triGeom = (int*)malloc(sizeof(int) * nt);
  W->tv = (float*)malloc(sizeof(float) * 9 * nt);
  W->tflags = (uint32_t*)malloc(sizeof(uint32_t) * nt);
  W->te0 = (V3*)malloc(sizeof(V3) * nt);
  W->te1 = (V3*)malloc(sizeof(V3) * nt);
  W->te2 = (V3*)malloc(sizeof(V3) * nt);
  int anyMotion = 0;
  for (int gi = 0; gi < W->ngeoms; ++gi) anyMotion |= W->geoms[gi].mesh->mot != NULL;
  W->tm = anyMotion ? (V3*)calloc((size_t)3 * nt, sizeof(V3)) : NULL;
  for (int gi = 0; gi < W->ngeoms; ++gi) {
    const Mesh* m = W->geoms[gi].mesh;
    for (int t = 0; t < m->nt; ++t) {
      const int id = W->geoms[gi].triBase + t;
      const V3 a = m->pos[m->tri[3 * t]], b = m->pos[m->tri[3 * t + 1]], c = m->pos[m->tri[3 * t + 2]];
      W->triGeom[id] = gi;
      float* tv = &W->tv[(size_t)id * 9];
      tv[0] = a.x; tv[1] = a.y; tv[2] = a.z; tv[3] = b.x; tv[4] = b.y; tv[5] = b.z; tv[6] = c.x; tv[7] = c.y; tv[8] = c.z;
      W->tflags[id] = m->cull ? 1u : 0u;
      W->te0[id] = a;
      W->te1[id] = sub(a, b);
      W->te2[id] = sub(c, a);
      if (W->tm && m->mot)
        for (int k = 0; k < 3; ++k) W->tm[(size_t)id * 3 + k] = m->mot[m->tri[3 * t + k]];
    }
  }
  bvh_build_oracle(W);
  return 0;
}

/* ====================================================================== sampling */
/* Random (common/math/random.h:24-78) */
typedef struct { int seed, state, table[32]; } Rnd;
static void rnd_seed(Rnd* r, int s) {
  const int a = 16807, m = 2147483647, q = 127773, rr = 2836;
  r->seed = s == 0 ? 1 : (s < 0 ? -s : s);
  for (int j = 32 + 7; j >= 0; j--) {
    int k = r->seed / q;
    r->seed = a * (r->seed - k * q) - rr * k;
    if (r->seed < 0) r->seed += m;
    if (j < 32) r->table[j] = r->seed;
  }
  r->state = r->table[0];
}
static int rnd_int(Rnd* r) {
  const int a = 16807, m = 2147483647, q = 127773, rr = 2836;
  int k = r->seed / q;
  r->seed = a * (r->seed - k * q) - rr * k;
  if (r->seed < 0) r->seed += m;
  int j = r->state / (1 + (2147483647 - 1) / 32);
  r->state = r->table[j];
  r->table[j] = r->seed;
  return r->state;
}
static float rnd_float(Rnd* r) { return fminf(rnd_int(r) / 2147483647.0f, 1.0f - ULP_F); }

void oracle_random_ints(int seed, int n, int32_t* out) {
  Rnd r;
  rnd_seed(&r, seed);
  for (int i = 0; i < n; ++i) out[i] = rnd_int(&r);
}

/* Permutation (common/math/permutation.h:42-48) */
static void perm_make(int* p, int n, Rnd* r) {
  for (int i = 0; i < n; i++) p[i] = i;
  for (int i = 0; i < n; i++) {
    int j = rnd_int(r) % n;
    int t = p[i]; p[i] = p[j]; p[j] = t;
  }
}
/* KAT exports of the integer layer (pinned against oracle/_ref, tests/test_ref_pin.py) */
void oracle_permutations(int size, int seed, int count, int32_t* out) {
  Rnd r;
  rnd_seed(&r, seed);
  int* p = (int*)malloc(sizeof(int) * size);
  for (int c = 0; c < count; ++c) {
    perm_make(p, size, &r);
    for (int i = 0; i < size; ++i) out[(size_t)c * size + i] = p[i];
  }
  free(p);
}
/* vector_t::shuffle (common/sys/stl/vector.h:129-133) of 0..n-1, count times in place */
void oracle_shuffles(int n, int seed, int count, uint32_t* out) {
  Rnd r;
  rnd_seed(&r, seed);
  uint32_t* v = (uint32_t*)malloc(sizeof(uint32_t) * n);
  for (int i = 0; i < n; ++i) v[i] = (uint32_t)i;
  for (int c = 0; c < count; ++c) {
    for (int k = 0; k < n; k++) { int j = rnd_int(&r) % n; uint32_t t = v[k]; v[k] = v[j]; v[j] = t; }
    for (int i = 0; i < n; ++i) out[(size_t)c * n + i] = v[i];
  }
  free(v);
}
/* the shared elementary functions (yrt_libm.h), for their accuracy tests */
void oracle_libm(int fn, int n, const float* x, const float* y, float* out) {
  for (int i = 0; i < n; ++i) {
    switch (fn) {
      case 0: out[i] = yrt_sinf(x[i]); break;
      case 1: out[i] = yrt_cosf(x[i]); break;
      case 2: out[i] = yrt_expf(x[i]); break;
      case 3: out[i] = yrt_logf(x[i]); break;
      case 4: out[i] = yrt_powf(x[i], y[i]); break;
      case 5: out[i] = yrt_asinf(x[i]); break;
      case 6: out[i] = yrt_acosf(x[i]); break;
      case 7: out[i] = yrt_atanf(x[i]); break;
      default: out[i] = yrt_atan2f(x[i], y[i]); break;
    }
  }
}
/* The vector helpers, element-wise, for the pin against the reference's own common/math
 * (tests/test_ref_pin.py, oracle/ref_math.cpp ref_vec: same fn numbers and layouts):
 * 0 dot, 1 cross, 2 normalize, 3 length, 4 L * v (9 floats, columns), 5 frame, 6 inverse,
 * 7 Color / float (color_sse.h:162: a * rcp(b)), 8 rcp, 9 rsqrt, 10 rcpps, 11 rsqrtps (x = a) */
void oracle_vecmath(int fn, int n, const float* a, const float* b, float* out) {
#define V3P(p) v3((p)[0], (p)[1], (p)[2])
#define PUT3(o, v) ((o)[0] = (v).x, (o)[1] = (v).y, (o)[2] = (v).z)
  for (int i = 0; i < n; ++i) {
    const float* A = a + (fn == 4 || fn == 6 ? 9 : fn >= 8 ? 1 : 3) * i;
    switch (fn) {
      case 0: out[i] = dot(V3P(A), V3P(b + 3 * i)); break;
      case 1: { const V3 r = cross(V3P(A), V3P(b + 3 * i)); PUT3(out + 3 * i, r); break; }
      case 2: { const V3 r = normalize(V3P(A)); PUT3(out + 3 * i, r); break; }
      case 3: out[i] = length(V3P(A)); break;
      case 4: { const V3 r = lmul(l3(V3P(A), V3P(A + 3), V3P(A + 6)), V3P(b + 3 * i)); PUT3(out + 3 * i, r); break; }
      case 5: {
        const L3 f = frame_(V3P(A));
        PUT3(out + 9 * i, f.vx); PUT3(out + 9 * i + 3, f.vy); PUT3(out + 9 * i + 6, f.vz);
        break;
      }
      case 6: {
        const L3 f = linv(l3(V3P(A), V3P(A + 3), V3P(A + 6)));
        PUT3(out + 9 * i, f.vx); PUT3(out + 9 * i + 3, f.vy); PUT3(out + 9 * i + 6, f.vz);
        break;
      }
      case 7: { const V3 r = muls(V3P(A), rcp(b[i])); PUT3(out + 3 * i, r); break; }
      case 8: out[i] = rcp(A[0]); break;
      case 9: out[i] = rsqrt_(A[0]); break;
      case 10: out[i] = yrt_rcpps(A[0]); break;
      default: out[i] = yrt_rsqrtps(A[0]); break;
    }
  }
#undef V3P
#undef PUT3
}

/* AmbientLight's bounding sphere (lights/ambientlight.h:44,71, restated for the pin only: the
 * integrator overwrites the shadow ray's tMax with tMaxShadowRay, pathtraceintegrator.cpp:151,
 * so no render reads it): getBSphere (common/math/bbox.h:75-78), BSphere::rayIntersect
 * (common/math/bsphere.h:93-100), solveQuadratic (common/math/math.h:174-208).
 * out[4i] = hit, near, far, radius */
void oracle_bsphere(int n, const float* lo, const float* hi, const float* org, const float* dir, float* out) {
  for (int i = 0; i < n; ++i) {
    const V3 L = v3(lo[3 * i], lo[3 * i + 1], lo[3 * i + 2]), H = v3(hi[3 * i], hi[3 * i + 1], hi[3 * i + 2]);
    const V3 c = muls(add(L, H), 0.5f);
    const float radius = length(sub(c, H));
    const V3 o = sub(v3(org[3 * i], org[3 * i + 1], org[3 * i + 2]), c);
    const V3 d = v3(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]);
    const float qa = dot(d, d), qb = 2 * dot(o, d), qc = dot(o, o) - radius * radius;
    int hit = 0;
    float x0 = 0.f, x1 = 0.f;
    if (qa == 0) {
      if (qb != 0) { x0 = x1 = -qc / qb; hit = 1; }
    } else {
      const float disc = qb * qb - 4.0f * qa * qc;
      if (!(disc < 0)) {
        const float sd = sqrtf(disc);
        const float tmp = qb < 0 ? -0.5f * (qb - sd) : -0.5f * (qb + sd);
        x0 = tmp / qa;
        x1 = qc / tmp;
        if (x0 > x1) { const float t = x0; x0 = x1; x1 = t; }
        hit = 1;
      }
    }
    out[4 * i] = (float)hit;
    out[4 * i + 1] = hit ? x0 : 0.f;
    out[4 * i + 2] = hit ? x1 : 0.f;
    out[4 * i + 3] = radius;
  }
}
void oracle_random_floats(int seed, int n, float* out) {
  Rnd r;
  rnd_seed(&r, seed);
  for (int i = 0; i < n; ++i) out[i] = rnd_float(&r);
}
/* jittered (samplers/patterns.h:28-35) */
static void jittered_(float* s, int n, Rnd* r) {
  const float scale = 1.0f / (float)(uint32_t)n;
  int* p = (int*)malloc(sizeof(int) * n);
  perm_make(p, n, r);
  for (int i = 0; i < n; i++) s[p[i]] = ((float)i + rnd_float(r)) * scale;
  free(p);
}
/* multiJittered (samplers/patterns.h:39-68) */
static void multijittered_(float* s /* 2n */, int N, Rnd* r) {
  uint32_t b = (uint32_t)sqrtf((float)N);
  if (b * b < (uint32_t)N) b++;
  float* g = (float*)malloc(sizeof(float) * 2 * b * b);
  uint32_t* num = (uint32_t*)malloc(sizeof(uint32_t) * b);
  for (uint32_t i = 0; i < b; i++) num[i] = i;
  for (uint32_t i = 0; i < b; i++) {
    for (uint32_t k = 0; k < b; k++) { uint32_t j = (uint32_t)(rnd_int(r) % (int)b); uint32_t t = num[k]; num[k] = num[j]; num[j] = t; }
    for (uint32_t j = 0; j < b; j++) g[(i * b + j) * 2] = (float)i / (float)b + ((float)num[j] + rnd_float(r)) / (float)(b * b);
  }
  for (uint32_t i = 0; i < b; i++) {
    for (uint32_t k = 0; k < b; k++) { uint32_t j = (uint32_t)(rnd_int(r) % (int)b); uint32_t t = num[k]; num[k] = num[j]; num[j] = t; }
    for (uint32_t j = 0; j < b; j++) g[(j * b + i) * 2 + 1] = (float)i / (float)b + ((float)num[j] + rnd_float(r)) / (float)(b * b);
  }
  int* p = (int*)malloc(sizeof(int) * N);
  perm_make(p, N, r);
  for (int n = 0; n < N; n++) {
    uint32_t np = (uint32_t)p[n];
    s[2 * n] = g[((np / b) * b + np % b) * 2];
    s[2 * n + 1] = g[((np / b) * b + np % b) * 2 + 1];
  }
  free(p); free(num); free(g);
}

/* Filter::init/sample (filters/filter.cpp:22-43) with BSplineFilter/BoxFilter */
typedef struct { float width, height; int n; Dist2 d; } Filt;
static float bspline_(float x, float y) {
  const float d = sqrtf(x * x + y * y);
  if (d > 2.0f) return 0.0f;
  if (d < 1.0f) { const float t = 1.0f - d; return ((((-3.0f * t) + 3.0f) * t + 3.0f) * t + 1.0f) / 6.0f; }
  const float t = 2.0f - d;
  return t * t * t / 6.0f;
}
static void filter_init(Filt* f, const char* name) {
  const int bs = !strcmp(name, "bspline");
  f->width = f->height = bs ? 4.0f : 1.0f;
  f->n = 256;
  const float inv = 1.0f / f->n;
  float* a = (float*)malloc(sizeof(float) * f->n * f->n);
  for (int x = 0; x < f->n; ++x)
    for (int y = 0; y < f->n; ++y) {
      const float px = (x + 0.5f) * inv * f->width - f->width * 0.5f;
      const float py = (y + 0.5f) * inv * f->height - f->height * 0.5f;
      float v = bs ? bspline_(px, py) : ((fabsf(px) <= 0.5f && fabsf(py) <= 0.5f) ? 1.0f : 0.0f);
      a[x * f->n + y] = fabsf(v); /* Array2D data[x][y] read as f[row=x][col=y] */
    }
  d2_init(&f->d, a, f->n, f->n);
  free(a);
}
static void filter_sample(const Filt* f, float u, float v, float* ox, float* oy) {
  float sx, sy, pdf;
  d2_sample(&f->d, u, v, &sx, &sy, &pdf);
  *ox = sx / (float)f->n * f->width - f->width * 0.5f;
  *oy = sy / (float)f->n * f->height - f->height * 0.5f;
}

/* SamplerFactory::init (samplers/sampler.cpp:85-158): table[dim][set*spp+s] */
typedef struct {
  int spp, sets, rec, dims, n1, n2, nl;
  float* t;
  float* light; /* [rec][nl][8] */
} Table;
static int roundup_pow2(int v) { int r = 1; while (r < v) r <<= 1; return r; }
static void table_build(Table* T, int spp_, int sets, int iteration, int n1, int n2, const char* filter,
                        const World* W) {
  const int spp = roundup_pow2(spp_ < 1 ? 1 : spp_);
  const int chunk = spp > 64 ? spp : 64;
  const int currentChunk = (iteration * spp) / chunk;
  const int offset = (iteration * spp) % chunk;
  Rnd r;
  rnd_seed(&r, currentChunk * 5897);
  Filt F;
  int useF = strcmp(filter, "none") != 0;
  if (useF) filter_init(&F, filter);
  T->spp = spp; T->sets = sets; T->rec = sets * spp; T->n1 = n1; T->n2 = n2;
  T->nl = 0;
  if (W)
    for (int i = 0; i < W->nlights; ++i) T->nl += W->lights[i].precomp >= 0;
  T->dims = 5 + n1 + 2 * n2;
  T->t = (float*)calloc((size_t)T->dims * T->rec, sizeof(float));
  T->light = (float*)calloc((size_t)T->rec * (T->nl ? T->nl : 1) * 8, sizeof(float));
  float *pix = malloc(sizeof(float) * 2 * chunk), *tim = malloc(sizeof(float) * chunk),
        *lens = malloc(sizeof(float) * 2 * chunk), *s1 = malloc(sizeof(float) * chunk),
        *s2 = malloc(sizeof(float) * 2 * chunk);
#define TT(d, rc) T->t[(size_t)(d) * T->rec + (rc)]
  for (int set = 0; set < sets; set++) {
    multijittered_(pix, chunk, &r);
    jittered_(tim, chunk, &r);
    multijittered_(lens, chunk, &r);
    for (int s = 0; s < spp; s++) {
      const int rc = set * spp + s;
      float px = pix[2 * (offset + s)], py = pix[2 * (offset + s) + 1];
      if (useF) {
        float fx, fy;
        filter_sample(&F, px, py, &fx, &fy);
        px = fx + 0.5f;
        py = fy + 0.5f;
      }
      TT(0, rc) = px; TT(1, rc) = py;
      TT(2, rc) = lens[2 * (offset + s)]; TT(3, rc) = lens[2 * (offset + s) + 1];
      TT(4, rc) = tim[offset + s];
    }
    for (int d = 0; d < n1; d++) {
      jittered_(s1, chunk, &r);
      for (int s = 0; s < spp; s++) TT(5 + d, set * spp + s) = s1[offset + s];
    }
    for (int d = 0; d < n2; d++) {
      multijittered_(s2, chunk, &r);
      for (int s = 0; s < spp; s++) {
        TT(5 + n1 + 2 * d, set * spp + s) = s2[2 * (offset + s)];
        TT(5 + n1 + 2 * d + 1, set * spp + s) = s2[2 * (offset + s) + 1];
      }
    }
    /* precomputed light samples: HDRILight::sample (lights/hdrilight.cpp:77-87) */
    if (W)
      for (int li = 0; li < W->nlights; ++li) {
        const Light* L = &W->lights[li];
        if (L->precomp < 0) continue;
        Dist2 dd = {L->w, L->h, L->ycdf, L->ypdf, L->xcdf, L->xpdf};
        for (int s = 0; s < spp; s++) {
          const int rc = set * spp + s;
          const float ux = TT(5 + n1 + 0, rc), uy = TT(5 + n1 + 1, rc); /* lightSampleID = 0 */
          float sx, sy, pdf;
          d2_sample(&dd, ux, uy, &sx, &sy, &pdf);
          const float theta = PI_F * sy * rcp((float)L->h);
          const float phi = TWO_PI_F * (1.0f - sx * rcp((float)L->w));
          const V3 _wi = v3(-sinf(theta) * cosf(phi), cosf(theta), -sinf(theta) * sinf(phi));
          const V3 wi = xfmVector(L->l2w, _wi);
          float c[4];
          int ix = (int)sx, iy = (int)sy;
          ix = ix < 0 ? 0 : (ix > L->w - 1 ? L->w - 1 : ix);
          iy = iy < 0 ? 0 : (iy > L->h - 1 ? L->h - 1 : iy);
          img_get(W->blob, L->img, ix, iy, c);
          float* o = &T->light[((size_t)rc * T->nl + L->precomp) * 8];
          o[0] = wi.x; o[1] = wi.y; o[2] = wi.z;
          o[3] = pdf * rcp(TWO_PI_F * PI_F * sinf(theta));
          o[4] = L->L.x * c[0]; o[5] = L->L.y * c[1]; o[6] = L->L.z * c[2];
          o[7] = INFINITY;
        }
      }
  }
#undef TT
  free(pix); free(tim); free(lens); free(s1); free(s2);
  if (useF) d2_free(&F.d);
}

int oracle_sample_table(int spp, int sets, int iteration, int num1D, int num2D, const char* filter, float* out,
                        size_t outFloats) {
  Table T;
  table_build(&T, spp, sets, iteration, num1D, num2D, filter ? filter : "bspline", NULL);
  const size_t n = (size_t)T.dims * T.rec;
  if (out && outFloats >= n) memcpy(out, T.t, n * sizeof(float));
  free(T.t);
  free(T.light);
  return T.rec;
}

void oracle_pixel_sets(int width, int height, int sets, uint8_t* out) {
  const int ntx = (width + 15) / 16, nty = (height + 15) / 16;
  for (int tile = 0; tile < ntx * nty; ++tile) {
    const int tx = (tile % ntx) * 16, ty = (tile / ntx) * 16;
    Rnd r;
    rnd_seed(&r, tx * 91711 + ty * 81551 + 3433 * 0); /* integratorrenderer.cpp:134 */
    for (int dy = 0; dy < 16; dy++) {
      const int y = ty + dy;
      if (y >= height) continue;
      for (int dx = 0; dx < 16; dx++) {
        const int x = tx + dx;
        if (x >= width) continue;
        out[(size_t)y * width + x] = (uint8_t)(rnd_int(&r) % sets); /* :149 */
      }
    }
  }
}

/* ====================================================================== camera */
typedef struct {
  int stereo, face, toeIn, dof;
  A3 p2w[6];
  V3 origin, up, xyz;
  float eyeSep, rcpZpd, falloff, lensRadius, focal;
} Camera;

static int camera_build(const Blob* B, Camera* C) {
  memset(C, 0, sizeof(*C));
  if (B->camera < 0) return fail("no camera");
  const Obj* o = &B->objs[B->camera];
  const A3 l2w = p_xfm(o, "local2world", a3_one());
  if (!strcasecmp(o->type, "pinhole")) { /* cameras/pinholecamera.h:15-21 */
    const float angle = p_float(o, "angle", 64.0f), ar = p_float(o, "aspectRatio", 1.0f);
    const V3 W = xfmVector(l2w, v3(-0.5f * ar, -0.5f, 0.5f * rcp(tanf(deg2rad(0.5f * angle)))));
    C->p2w[0] = a3(l3(muls(l2w.l.vx, ar), l2w.l.vy, W), l2w.p);
    return 0;
  }
  if (!strcasecmp(o->type, "depthoffield")) { /* cameras/depthoffieldcamera.h:13-19 */
    const float angle = p_float(o, "angle", 64.0f), ar = p_float(o, "aspectRatio", 1.0f);
    const V3 W = xfmVector(l2w, v3(-0.5f * ar, -0.5f, 0.5f * rcp(tanf(deg2rad(0.5f * angle)))));
    C->p2w[0] = a3(l3(muls(l2w.l.vx, ar), l2w.l.vy, W), l2w.p);
    C->p2w[1] = l2w;
    C->dof = 1;
    C->lensRadius = p_float(o, "lensRadius", 0.0f);
    C->focal = p_float(o, "focalDistance", 0.0f) /
               length(add(add(muls(C->p2w[0].l.vx, 0.5f), muls(C->p2w[0].l.vy, 0.5f)), C->p2w[0].l.vz));
    return 0;
  }
  if (strcasecmp(o->type, "stereo")) return fail("camera type outside the oracle's scope");
  /* cameras/StereoCubeCamera.h:16-51 */
  C->stereo = 1;
  C->face = p_int(o, "cubeFaceIndex", 0);
  const V3 origin = p_v3(o, "origin", l2w.p);
  const V3 lookAt = p_v3(o, "lookAt", v3(0.f, 0.f, -1.f));
  const V3 up = p_v3(o, "up", v3(0.f, 1.f, 0.f));
  const V3 right = cross(normalize(up), normalize(sub(lookAt, origin)));
  const float sceneScale = p_float(o, "sceneScale", 1.f);
  const float EYE = 6.35f * 0.393701f, ZP = EYE * 30.f;
  C->eyeSep = p_float(o, "eyeSeparation", EYE) * sceneScale;
  const float zpd = p_float(o, "zeroParallaxDistance", ZP) * sceneScale;
  if (zpd != 0.f) { C->rcpZpd = 1.f / zpd; C->toeIn = p_int(o, "toeIn", 0) != 0; }
  else { C->rcpZpd = 0.f; C->toeIn = 0; }
  C->falloff = clampf_(p_float(o, "stereFalloffAngle", 30.f), 0.f, 90.f);
  const float ar = 1.f, angle = 90.f;
  const V3 W = xfmVector(l2w, v3(-.5f * ar, -.5f, .5f * rcp(tanf(deg2rad(.5f * angle)))));
  C->p2w[0] = a3(l3(muls(l2w.l.vx, ar), l2w.l.vy, W), l2w.p);
  C->xyz = normalize(add(add(muls(C->p2w[0].l.vx, .5f), muls(C->p2w[0].l.vy, .5f)), C->p2w[0].l.vz));
  C->p2w[1] = aamul(a3_rotate_about(origin, up, deg2rad(90.f)), C->p2w[0]);
  C->p2w[2] = aamul(a3_rotate_about(origin, up, deg2rad(180.f)), C->p2w[0]);
  C->p2w[3] = aamul(a3_rotate_about(origin, up, deg2rad(-90.f)), C->p2w[0]);
  C->p2w[4] = aamul(a3_rotate_about(origin, right, deg2rad(-90.f)), C->p2w[0]);
  C->p2w[4] = aamul(a3_rotate_about(origin, up, deg2rad(180.f)), C->p2w[4]);
  C->p2w[5] = aamul(a3_rotate_about(origin, right, deg2rad(90.f)), C->p2w[0]);
  C->p2w[5] = aamul(a3_rotate_about(origin, up, deg2rad(180.f)), C->p2w[5]);
  C->origin = origin;
  C->up = up;
  return 0;
}

static void camera_ray(const Camera* C, float fx, float fy, float lx, float ly, V3* org, V3* dir) {
  if (C->dof) { /* depthoffieldcamera.h:20-26, uniformSampleDisk (shapesampler.h:187-191) */
    const A3 m = C->p2w[0];
    const float r = sqrtf(lx), th = TWO_PI_F * ly;
    const V3 begin = xfmPoint(C->p2w[1], v3(C->lensRadius * r * yrt_cosf(th), C->lensRadius * r * yrt_sinf(th), 0.0f));
    const V3 end = add(m.p, muls(add(add(muls(m.l.vx, fx), muls(m.l.vy, 1.0f - fy)), m.l.vz), C->focal));
    *org = begin;
    *dir = normalize(sub(end, begin));
    return;
  }
  if (!C->stereo) { /* pinholecamera.h:23-25 */
    const A3 m = C->p2w[0];
    *org = m.p;
    *dir = normalize(add(add(muls(m.l.vx, fx), muls(m.l.vy, 1.0f - fy)), m.l.vz));
    return;
  }
  /* StereoCubeCamera::ray (StereoCubeCamera.h:68-161) */
  const A3 P0 = C->p2w[0];
  const int ef = C->face % 6;
  const float yPixel = 1.0f - fy;
  A3 p2w = C->p2w[ef];
  float theta = 0.f, absVA = 0.f;
  if (ef <= 3) {
    const V3 xDir = normalize(add(add(muls(P0.l.vx, fx), muls(P0.l.vy, .5f)), P0.l.vz));
    theta = yrt_acosf(clampf_(dot(xDir, C->xyz), -1.f, 1.f)) * signf_(fx - .5f);
    const V3 yDir = normalize(add(add(muls(P0.l.vx, .5f), muls(P0.l.vy, yPixel)), P0.l.vz));
    const float yAngle = rad2deg(yrt_acosf(clampf_(dot(yDir, C->xyz), -1.f, 1.f))) * signf_(yPixel - .5f);
    absVA = fabsf(yAngle);
  } else {
    const V3 xyDirNorm = normalize(v3(fx - .5f, yPixel - .5f, 0.f));
    const V3 xyUp = v3(0.f, ef == 4 ? -1.f : 1.f, 0.f);
    theta = yrt_acosf(clampf_(dot(xyDirNorm, xyUp), -1.f, 1.f)) * signf_(fx - .5f);
    const V3 xyzDir = normalize(add(add(muls(P0.l.vx, fx), muls(P0.l.vy, yPixel)), P0.l.vz));
    const float xyzAngle = rad2deg(yrt_acosf(clampf_(dot(xyzDir, C->xyz), -1.f, 1.f)));
    absVA = 90.f - fabsf(xyzAngle);
  }
  float eyeOffset = C->eyeSep * (C->face < 6 ? -.5f : .5f);
  if (absVA > C->falloff) {
    const float coef = 1.f - smoothstep_(0.f, 1.f, smoothstep_(C->falloff, 90.f, absVA));
    eyeOffset *= coef;
  }
  p2w = aamul(p2w, a3_translate(v3(eyeOffset, 0.f, 0.f)));
  const A3 rot = a3_rotate_about(C->origin, C->up, theta);
  const V3 rayOrigin = aamul(rot, p2w).p;
  if (C->toeIn) {
    const float toe = -yrt_atanf(eyeOffset * C->rcpZpd);
    p2w = aamul(a3_rotate_about(rayOrigin, C->up, toe), p2w);
  }
  *org = rayOrigin;
  *dir = normalize(add(add(muls(p2w.l.vx, fx), muls(p2w.l.vy, yPixel)), p2w.l.vz));
}

/* ====================================================================== shading */
typedef struct {
  V3 P, Ng, Ns, Tx, Ty;
  float s, t, error;
  int material, light, illumMask, shadowMask;
} DG;

/* BackendSceneFlat::postIntersect -> Shape::postIntersect (trianglemesh_full.cpp:192-260,
 * trianglemesh_normals.cpp:125-147, triangle.h:69-78) */
static void post_intersect(const World* W, const Ray* r, const Hit* h, DG* dg) {
  const int gi = W->triGeom[h->tri];
  const Geom* g = &W->geoms[gi];
  const Mesh* m = g->mesh;
  const int prim = h->tri - g->triBase;
  const float u = h->u, v = h->v, w = 1.0f - u - v, t = h->t;
  dg->material = g->material;
  dg->light = g->light;
  dg->illumMask = g->illumMask;
  dg->shadowMask = g->shadowMask;
  dg->P = add(r->org, muls(r->dir, t));
  dg->Tx = dg->Ty = vs(0.f);
  if (m->kind == GK_TRIANGLE) {
    dg->Ng = m->Ng;
    dg->Ns = m->Ng;
    dg->s = u; dg->t = v;
  } else {
    const int i0 = m->tri[3 * prim], i1 = m->tri[3 * prim + 1], i2 = m->tri[3 * prim + 2];
    V3 p0 = m->pos[i0], p1 = m->pos[i1], p2 = m->pos[i2];
    if (m->mot) { /* trianglemesh_full.cpp:211-215 */
      p0 = add(p0, muls(m->mot[i0], r->time));
      p1 = add(p1, muls(m->mot[i1], r->time));
      p2 = add(p2, muls(m->mot[i2], r->time));
    }
    const V3 dPdu = sub(p1, p0), dPdv = sub(p2, p0);
    dg->Ng = normalize(cross(sub(p0, p1), sub(p2, p0)));
    if (m->kind == GK_NORMALS) {
      dg->s = u; dg->t = v;
      V3 Ns = add(add(muls(m->nor[i0], w), muls(m->nor[i1], u)), muls(m->nor[i2], v));
      const float len2 = dot(Ns, Ns);
      Ns = len2 > 0 ? muls(Ns, rsqrt_(len2)) : dg->Ng;
      if (dot(Ns, dg->Ng) < 0) Ns = neg(Ns);
      dg->Ns = Ns;
      dg->Tx = dPdu; dg->Ty = dPdv;
    } else {
      float dsdu, dtdu, dsdv, dtdv;
      if (m->uv) {
        const float *a = &m->uv[2 * i0], *b = &m->uv[2 * i1], *c = &m->uv[2 * i2];
        dg->s = a[0] * w + b[0] * u + c[0] * v;
        dg->t = a[1] * w + b[1] * u + c[1] * v;
        dsdu = b[0] - a[0]; dtdu = b[1] - a[1];
        dsdv = c[0] - a[0]; dtdv = c[1] - a[1];
      } else {
        dg->s = u; dg->t = v;
        dsdu = 1; dtdu = 0; dsdv = 0; dtdv = 1;
      }
      if (m->nor) {
        V3 Ns = add(add(muls(m->nor[i0], w), muls(m->nor[i1], u)), muls(m->nor[i2], v));
        const float len2 = dot(Ns, Ns);
        Ns = len2 > 0 ? muls(Ns, rsqrt_(len2)) : dg->Ng;
        if (dot(Ns, dg->Ng) < 0) Ns = neg(Ns);
        dg->Ns = Ns;
      } else {
        dg->Ns = dg->Ng;
      }
      /* trianglemesh_full.cpp:244-263: interpolated tangents when given, else from dP/dst */
      if (m->tanX) {
        dg->Tx = add(add(muls(m->tanX[i0], w), muls(m->tanX[i1], u)), muls(m->tanX[i2], v));
      } else {
        const V3 dPds = normalize(sub(muls(dPdu, dtdv), muls(dPdv, dtdu)));
        dg->Tx = normalize(sub(dPds, muls(dg->Ns, dot(dPds, dg->Ns))));
      }
      if (m->tanY) {
        dg->Ty = add(add(muls(m->tanY[i0], w), muls(m->tanY[i1], u)), muls(m->tanY[i2], v));
      } else {
        const V3 dPdt = normalize(sub(muls(dPdv, dsdu), muls(dPdu, dsdv)));
        dg->Ty = normalize(sub(dPdt, muls(dg->Ns, dot(dPdt, dg->Ns))));
      }
    }
  }
  dg->error = fmaxf(fabsf(t), fmax3(absv(dg->P)));
}

/* ---- BRDF components (brdfs/ headers); type bits brdfs/brdf.h:10-30 */
#define BT_DIFFUSE 0x000F000Fu
enum { B_LAMBERT, B_DIEL_REFL, B_CONST_TRANS, B_THIN_TRANS, B_LAYER, B_MICRO, B_TRANS, B_SPEC, B_REFL, B_COND,
       B_MICRO_COND, B_MICRO_ANISO, B_MINNAERT, B_VELVETY, B_DIEL_TRANS, B_LAYER_GLITTER };
typedef struct { int kind; uint32_t type; V3 R; float a, b, c; V3 eta, k; } Brdf;
typedef struct { int n; Brdf c[8]; } BSet;
static void bs_add(BSet* s, int kind, uint32_t type, V3 R, float a, float b, float c) {
  if (s->n >= 8) return;
  Brdf* k = &s->c[s->n++];
  k->kind = kind; k->type = type; k->R = R; k->a = a; k->b = b; k->c = c;
  k->eta = k->k = vs(0.f);
}

/* optics.h:64-104 */
static float fres3(float cosi, float cost, float eta) {
  float Rper = (eta * cosi - cost) * rcp(eta * cosi + cost);
  float Rpar = (cosi - eta * cost) * rcp(cosi + eta * cost);
  return 0.5f * (Rpar * Rpar + Rper * Rper);
}
static float fres2(float cosi, float eta, float* outCosT) {
  float k = 1.0f - eta * eta * (1.0f - cosi * cosi);
  if (k < 0.0f) return 1.0f;
  float cost = sqrtf(k);
  if (outCosT) *outCosT = cost;
  return fres3(cosi, cost, eta);
}
static float refract5(V3 V, V3 N, float eta, float cosi, float* cost, V3* out) {
  float k = 1.0f - eta * eta * (1.0f - cosi * cosi);
  if (k < 0.0f) { *cost = 0.0f; *out = vs(0.f); return 0.0f; }
  *cost = sqrtf(k);
  *out = sub(muls(sub(muls(N, cosi), V), eta), muls(N, *cost));
  return eta * eta;
}
static V3 reflect3(V3 V, V3 N, float cosi) { return sub(muls(N, 2.0f * cosi), V); }
static V3 reflect2(V3 V, V3 N) { return reflect3(V, N, dot(V, N)); }

/* cosineSampleHemisphere (samplers/shapesampler.h:80-95) */
static V3 cos_hemi(float u, float v, V3 N, float* pdf) {
  const float phi = TWO_PI_F * u;
  const float cosT = sqrtf(v), sinT = sqrtf(1.0f - v);
  *pdf = cosT * ONE_OVER_PI_F;
  return lmul(frame_(N), v3(yrt_cosf(phi) * sinT, yrt_sinf(phi) * sinT, cosT));
}

static V3 lambert_eval(V3 R, const DG* dg, V3 wi) { return muls(muls(R, ONE_OVER_PI_F), clamp01(dot(wi, dg->Ns))); }

/* fresnelConductor (brdfs/optics.h:123-131), per channel */
static float fres_cond1(float cosi, float eta, float k) {
  const float tmp = eta * eta + k * k;
  const float e2c = 2.0f * eta * cosi;
  const float Rpar = (tmp * cosi * cosi - e2c + 1.0f) * rcp(tmp * cosi * cosi + e2c + 1.0f);
  const float Rper = (tmp - e2c + cosi * cosi) * rcp(tmp + e2c + cosi * cosi);
  return 0.5f * (Rpar + Rper);
}
static V3 fres_cond(float cosi, V3 eta, V3 k) {
  return v3(fres_cond1(cosi, eta.x, k.x), fres_cond1(cosi, eta.y, k.y), fres_cond1(cosi, eta.z, k.z));
}
/* AnisotropicPowerCosineDistribution::eval (microfacet/anisotropic_power_cosine_distribution.h:40-48) */
static float aniso_D(float nx, float ny, const DG* dg, V3 wh) {
  const float norm2 = sqrtf((nx + 2) * (ny + 2)) * ONE_OVER_TWO_PI_F;
  const float cP = dot(wh, dg->Tx), sP = dot(wh, dg->Ty), cT = dot(wh, dg->Ns);
  const float R = cP * cP + sP * sP;
  if (R == 0.0f) return norm2;
  const float n = (nx * (cP * cP) + ny * (sP * sP)) * rcp(R);
  return norm2 * yrt_powf(fabsf(cT), n);
}
/* Microfacet<Fresnel,Distribution>::eval (brdfs/microfacet.h:28-41): dielectric or conductor
 * Fresnel, power-cosine or anisotropic power-cosine distribution */
static V3 micro_eval(const Brdf* c, V3 wo, const DG* dg, V3 wi) {
  if (dot(wi, dg->Ng) <= 0) return vs(0.f);
  const float cO = dot(wo, dg->Ns), cI = dot(wi, dg->Ns);
  if (cI <= 0.0f || cO <= 0.0f) return vs(0.f);
  const V3 wh = normalize(add(wi, wo));
  const float cH = dot(wh, dg->Ns);
  const float cT = dot(wi, wh);
  const V3 F = c->kind == B_MICRO ? vs(fres2(cT, c->a * rcp(c->b), NULL)) : fres_cond(cT, c->eta, c->k);
  float D;
  if (c->kind == B_MICRO_ANISO) {
    D = aniso_D(c->a, c->b, dg, wh);
  } else {
    const float n = c->kind == B_MICRO ? c->c : c->a;
    D = ((n + 2) * ONE_OVER_TWO_PI_F) * yrt_powf(fabsf(dot(wh, dg->Ns)), n);
  }
  const float G = fminf(fminf(1.0f, 2.0f * cH * cO * rcp(cT)), 2.0f * cH * cI * rcp(cT));
  return muls(mulv(muls(muls(c->R, D), G), F), rcp(4.0f * cO));
}
/* Minnaert::eval (brdfs/minnaert.h:20-24), Velvety::eval (brdfs/velvety.h:20-26). Color / float is
 * a * rcp(b) in the reference (common/math/color_sse.h:162), not a division. */
static V3 col_divs(V3 a, float s) { return muls(a, rcp(s)); }
/* Vector3f / float: _mm_div_ps (vector3f_sse.h:155), an IEEE division */
static V3 divs(V3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
static V3 minnaert_eval(const Brdf* c, V3 wo, const DG* dg, V3 wi) {
  const float cI = clamp01(dot(wi, dg->Ns));
  const float bs = yrt_powf(clamp01(dot(wo, wi)), c->a);
  return col_divs(muls(muls(c->R, bs), cI), PI_F);
}
static V3 velvety_eval(const Brdf* c, V3 wo, const DG* dg, V3 wi) {
  const float cO = clamp01(dot(wo, dg->Ns)), cI = clamp01(dot(wi, dg->Ns));
  const float sO = sqrtf(1.0f - cO * cO);
  const float hs = yrt_powf(sO, c->a);
  return col_divs(muls(muls(c->R, hs), cI), PI_F);
}
/* DielectricLayer<Lambertian>::eval (brdfs/dielectriclayer.h:27-38) */
static V3 layer_eval(const Brdf* c, V3 wo, const DG* dg, V3 wi) {
  float cO = dot(wo, dg->Ns), cI = dot(wi, dg->Ns);
  if (cI <= 0.0f || cO <= 0.0f) return vs(0.f);
  float cO1, cI1;
  V3 wo1, wi1;
  refract5(wo, dg->Ns, c->a, cO, &cO1, &wo1);
  refract5(wi, dg->Ns, c->a, cI, &cI1, &wi1);
  float Fi = 1.0f - fres3(cI, cI1, c->a);
  V3 Fg = lambert_eval(c->R, dg, neg(wi1));
  float Fo = 1.0f - fres3(cO, cO1, c->a);
  return muls(mulv(mulv(mulv(vs(Fo), vs(1.f)), Fg), vs(1.f)), Fi);
}
/* MetallicPaint glitter (materials/metallicpaint.h:63-70): DielectricLayer<Microfacet<
 * FresnelConductor(0.62, 4.8), PowerCosineDistribution(rcp(glitterSpread), Ns)>>(one, 1, eta,
 * glitterColor); c->a = etait, c->b = etati, c->c = n. The ground is a B_MICRO_COND record. */
static Brdf glitter_ground(const Brdf* c) {
  Brdf g;
  memset(&g, 0, sizeof(g));
  g.kind = B_MICRO_COND; g.type = 0x10u; g.R = c->R; g.a = c->c;
  g.eta = vs(0.62f); g.k = vs(4.8f);
  return g;
}
static V3 glitter_layer_eval(const Brdf* c, V3 wo, const DG* dg, V3 wi) { /* dielectriclayer.h:27-38 */
  float cO = dot(wo, dg->Ns), cI = dot(wi, dg->Ns);
  if (cI <= 0.0f || cO <= 0.0f) return vs(0.f);
  float cO1, cI1;
  V3 wo1, wi1;
  refract5(wo, dg->Ns, c->a, cO, &cO1, &wo1);
  refract5(wi, dg->Ns, c->a, cI, &cI1, &wi1);
  float Fi = 1.0f - fres3(cI, cI1, c->a);
  const Brdf g = glitter_ground(c);
  V3 Fg = micro_eval(&g, neg(wo1), dg, neg(wi1));
  float Fo = 1.0f - fres3(cO, cO1, c->a);
  return muls(mulv(mulv(mulv(vs(Fo), vs(1.f)), Fg), vs(1.f)), Fi);
}
static V3 brdf_sample(const Brdf* c, V3 wo, const DG* dg, float sx, float sy, V3* wi, float* pdf);

/* Specular::eval (brdfs/specular.h:20-24) */
static V3 spec_eval(const Brdf* c, V3 wo, const DG* dg, V3 wi) {
  V3 r = reflect2(wo, dg->Ns);
  if (dot(r, wi) < 0) return vs(0.f);
  return muls(muls(muls(muls(c->R, c->a + 2), 1.0f / (2.0f * PI_F)), yrt_powf(dot(r, wi), c->a)), clamp01(dot(wi, dg->Ns)));
}
static V3 brdf_eval(const Brdf* c, V3 wo, const DG* dg, V3 wi) {
  switch (c->kind) {
    case B_LAMBERT: return lambert_eval(c->R, dg, wi);
    case B_LAYER: return layer_eval(c, wo, dg, wi);
    case B_MICRO: case B_MICRO_COND: case B_MICRO_ANISO: return micro_eval(c, wo, dg, wi);
    case B_SPEC: return spec_eval(c, wo, dg, wi);
    case B_REFL: return c->R;
    case B_MINNAERT: return minnaert_eval(c, wo, dg, wi);
    case B_VELVETY: return velvety_eval(c, wo, dg, wi);
    case B_LAYER_GLITTER: return glitter_layer_eval(c, wo, dg, wi);
    default: return vs(0.f);
  }
}
static V3 brdf_sample(const Brdf* c, V3 wo, const DG* dg, float sx, float sy, V3* wi, float* pdf) {
  *pdf = 0.f;
  *wi = vs(0.f);
  switch (c->kind) {
    case B_LAMBERT: /* lambertian.h:24-26 */
      *wi = cos_hemi(sx, sy, dg->Ns, pdf);
      return lambert_eval(c->R, dg, *wi);
    case B_DIEL_REFL: { /* dielectric.h:25-31 */
      const float cO = clamp01(dot(wo, dg->Ns));
      *wi = reflect3(wo, dg->Ns, cO);
      *pdf = 1.0f;
      return muls(vs(fres2(cO, c->a, NULL)), c->b);
    }
    case B_CONST_TRANS: { /* dielectric.h:169-173 */
      *wi = neg(wo);
      *pdf = 1.0f;
      const float ct = clamp01(dot(wo, dg->Ns));
      return ct <= 0.0f ? vs(0.f) : c->R;
    }
    case B_THIN_TRANS: { /* dielectric.h:113-123 */
      *wi = neg(wo);
      *pdf = 1.0f;
      const float ct = clamp01(dot(wo, dg->Ns));
      if (ct <= 0.0f) return vs(0.f);
      const float alpha = c->b * rcp(ct);
      float cT;
      const V3 la = muls(c->R, alpha);
      return muls(v3(yrt_expf(la.x), yrt_expf(la.y), yrt_expf(la.z)), 1.f - fres2(ct, c->a, &cT));
    }
    case B_LAYER: { /* dielectriclayer.h:40-62 */
      float cO = dot(wo, dg->Ns);
      if (cO <= 0.0f) return vs(0.f);
      float cO1;
      V3 wo1;
      refract5(wo, dg->Ns, c->a, cO, &cO1, &wo1);
      float p1;
      V3 wi1 = cos_hemi(sx, sy, dg->Ns, &p1);
      V3 Fg = lambert_eval(c->R, dg, wi1);
      float cI1 = dot(wi1, dg->Ns);
      if (cI1 <= 0.0f) return vs(0.f);
      float cI;
      V3 wi0;
      float p0 = refract5(neg(wi1), neg(dg->Ns), c->b, cI1, &cI, &wi0);
      if (p0 == 0.0f) return vs(0.f);
      *wi = wi0;
      *pdf = p1;
      float Fi = 1.0f - fres3(cI, cI1, c->a);
      float Fo = 1.0f - fres3(cO, cO1, c->a);
      return muls(mulv(mulv(mulv(vs(Fo), vs(1.f)), Fg), vs(1.f)), Fi);
    }
    case B_MICRO: { /* microfacet.h:43-50 + power_cosine_distribution.h:27-35 */
      if (dot(wo, dg->Ns) <= 0.0f) return vs(0.f);
      const float n = c->c;
      const float norm1 = (n + 1) * ONE_OVER_TWO_PI_F;
      const float phi = TWO_PI_F * sx;
      const float cP = yrt_cosf(phi), sP = yrt_sinf(phi);
      const float cT = yrt_powf(sy, rcp(n + 1));
      const float sT = sqrtf(fmaxf(0.0f, 1.0f - cT * cT));
      const V3 wh = lmul(frame_(dg->Ns), v3(cP * sT, sP * sT, cT));
      const float whpdf = norm1 * yrt_powf(cT, n);
      *wi = reflect2(wo, wh);
      *pdf = whpdf * rcp(4.0f * fabsf(dot(wo, wh)));
      if (dot(*wi, dg->Ns) <= 0.0f) return vs(0.f);
      return micro_eval(c, wo, dg, *wi);
    }
    case B_TRANS: /* transmission.h:22-24 */
      *wi = neg(wo);
      *pdf = 1.0f;
      return c->R;
    case B_MICRO_COND: { /* microfacet.h:43-50 + power_cosine_distribution.h:27-35 */
      if (dot(wo, dg->Ns) <= 0.0f) return vs(0.f);
      const float n = c->a;
      const float norm1 = (n + 1) * ONE_OVER_TWO_PI_F;
      const float phi = TWO_PI_F * sx;
      const float cP = yrt_cosf(phi), sP = yrt_sinf(phi);
      const float cT = yrt_powf(sy, rcp(n + 1));
      const float sT = sqrtf(fmaxf(0.0f, 1.0f - cT * cT));
      const V3 wh = lmul(frame_(dg->Ns), v3(cP * sT, sP * sT, cT));
      const float whpdf = norm1 * yrt_powf(cT, n);
      *wi = reflect2(wo, wh);
      *pdf = whpdf * rcp(4.0f * fabsf(dot(wo, wh)));
      if (dot(*wi, dg->Ns) <= 0.0f) return vs(0.f);
      return micro_eval(c, wo, dg, *wi);
    }
    case B_MICRO_ANISO: { /* anisotropic_power_cosine_distribution.h:57-73 */
      if (dot(wo, dg->Ns) <= 0.0f) return vs(0.f);
      const float nx = c->a, ny = c->b;
      const float norm1 = sqrtf((nx + 1) * (ny + 1)) * ONE_OVER_TWO_PI_F;
      const float phi = TWO_PI_F * sx;
      const float sP0 = sqrtf(nx + 1) * yrt_sinf(phi);
      const float cP0 = sqrtf(ny + 1) * yrt_cosf(phi);
      const float nrm = rsqrt_(sP0 * sP0 + cP0 * cP0);
      const float sP = sP0 * nrm, cP = cP0 * nrm;
      const float n = nx * (cP * cP) + ny * (sP * sP);
      const float cT = yrt_powf(sy, rcp(n + 1));
      const float sT = sqrtf(fmaxf(0.0f, 1.0f - cT * cT));
      const float whpdf = norm1 * yrt_powf(cT, n);
      const V3 h = v3(cP * sT, sP * sT, cT);
      const V3 wh = add(add(muls(dg->Tx, h.x), muls(dg->Ty, h.y)), muls(dg->Ns, h.z));
      *wi = reflect2(wo, wh);
      *pdf = whpdf * rcp(4.0f * fabsf(dot(wo, wh)));
      if (dot(*wi, dg->Ns) <= 0.0f) return vs(0.f);
      return micro_eval(c, wo, dg, *wi);
    }
    case B_REFL: /* reflection.h:19-22 */
      *wi = reflect2(wo, dg->Ns);
      *pdf = 1.0f;
      return c->R;
    case B_COND: /* conductor.h:21-24 */
      *wi = reflect2(wo, dg->Ns);
      *pdf = 1.0f;
      return mulv(c->R, fres_cond(dot(wo, dg->Ns), c->eta, c->k));
    case B_MINNAERT:
      *wi = cos_hemi(sx, sy, dg->Ns, pdf);
      return minnaert_eval(c, wo, dg, *wi);
    case B_VELVETY:
      *wi = cos_hemi(sx, sy, dg->Ns, pdf);
      return velvety_eval(c, wo, dg, *wi);
    case B_DIEL_TRANS: { /* dielectric.h:82-89 */
      const float cO = clamp01(dot(wo, dg->Ns));
      float cI;
      *pdf = refract5(wo, dg->Ns, c->a, cO, &cI, wi);
      return vs(1.0f - fres3(cO, cI, c->a));
    }
    case B_LAYER_GLITTER: { /* dielectriclayer.h:40-62 over the glitter microfacet's sample */
      float cO = dot(wo, dg->Ns);
      if (cO <= 0.0f) return vs(0.f);
      float cO1;
      V3 wo1;
      refract5(wo, dg->Ns, c->a, cO, &cO1, &wo1);
      const Brdf g = glitter_ground(c);
      V3 wi1 = vs(0.f);
      float p1 = 0.f;
      V3 Fg = brdf_sample(&g, neg(wo1), dg, sx, sy, &wi1, &p1);
      float cI1 = dot(wi1, dg->Ns);
      if (cI1 <= 0.0f) return vs(0.f);
      float cI;
      V3 wi0;
      float p0 = refract5(neg(wi1), neg(dg->Ns), c->b, cI1, &cI, &wi0);
      if (p0 == 0.0f) return vs(0.f);
      *wi = wi0;
      *pdf = p1;
      float Fi = 1.0f - fres3(cI, cI1, c->a);
      float Fo = 1.0f - fres3(cO, cO1, c->a);
      return muls(mulv(mulv(mulv(vs(Fo), vs(1.f)), Fg), vs(1.f)), Fi);
    }
    case B_SPEC: { /* specular.h:26-28, shapesampler.h:104-121 */
      const float e = c->a;
      const float phi = TWO_PI_F * sx;
      const float cT = yrt_powf(sy, rcp(e + 1));
      const float sT = sqrtf(fmaxf(0.0f, 1.0f - cT * cT));
      *pdf = (e + 1.0f) * yrt_powf(cT, e) * ONE_OVER_TWO_PI_F;
      *wi = lmul(frame_(reflect2(wo, dg->Ns)), v3(yrt_cosf(phi) * sT, yrt_sinf(phi) * sT, cT));
      return spec_eval(c, wo, dg, *wi);
    }
  }
  return vs(0.f);
}
/* CompositedBRDF::eval / sample (brdfs/compositedbrdf.h:59-166) */
static V3 bs_eval(const BSet* s, V3 wo, const DG* dg, V3 wi, uint32_t type) {
  V3 c = vs(0.f);
  for (int i = 0; i < s->n; i++)
    if (s->c[i].type & type) c = add(c, brdf_eval(&s->c[i], wo, dg, wi));
  return c;
}
static V3 bs_sample(const BSet* s, V3 wo, const DG* dg, float sx, float sy, float ss, V3* wi_o, float* pdf_o,
                    uint32_t* type_o) {
  float f[8], sum = 0.0f;
  V3 col[8], dir[8];
  float pd[8];
  uint32_t ty[8];
  int num = 0;
  for (int i = 0; i < s->n; i++) {
    V3 wi;
    float pdf;
    V3 c = brdf_sample(&s->c[i], wo, dg, sx, sy, &wi, &pdf);
    if (v3zero(c) || pdf <= 0.0f) continue;
    f[num] = (c.x + c.y + c.z) * rcp(pdf);
    sum += f[num];
    col[num] = c; dir[num] = wi; pd[num] = pdf; ty[num] = s->c[i].type;
    num++;
  }
  if (num == 0) { *wi_o = vs(0.f); *pdf_o = 0.f; *type_o = 0; return vs(0.f); }
  for (int i = 0; i < num; i++) f[i] /= sum;
  float d[8];
  d[0] = f[0];
  for (int i = 1; i < num - 1; i++) d[i] = d[i - 1] + f[i];
  d[num - 1] = 1.0f;
  int i = 0;
  while (i < num - 1 && ss > d[i]) i++;
  *wi_o = dir[i];
  *pdf_o = pd[i] * f[i];
  *type_o = ty[i];
  return col[i];
}

/* Material::shade (materials/ headers) */
static void shade(const World* W, const Material* m, Medium cur, DG* dg, BSet* s) {
  const Blob* B = W->blob;
  s->n = 0;
  float c[4];
  switch (m->type) {
    case MT_PLASTIC: /* DielectricLayer<Lambertian>(one, 1, eta, pigment) + DielectricReflection(1, eta) | Microfacet */
      bs_add(s, B_LAYER, 0x1u, m->pigment, 1.0f * rcp(m->eta), m->eta * rcp(1.0f), 0);
      if (m->roughness == 0.0f) bs_add(s, B_DIEL_REFL, 0x100u, vs(0.f), 1.0f * rcp(m->eta), 1.0f, 0);
      else bs_add(s, B_MICRO, 0x10u, vs(1.0f), 1.0f, m->eta, m->rcpRoughness);
      break;
    case MT_DIELECTRIC: { /* dielectric.h:42-52 */
      const int oi = med_eq(cur, m->outside);
      const float e = oi ? m->outside.eta * rcp(m->inside.eta) : m->inside.eta * rcp(m->outside.eta);
      bs_add(s, B_DIEL_REFL, 0x100u, vs(0.f), e, 1.0f, 0);
      bs_add(s, B_DIEL_TRANS, 0x01000000u, vs(0.f), e, 0, 0);
      break;
    }
    case MT_MIRROR: bs_add(s, B_REFL, 0x100u, m->reflectance, 0, 0, 0); break;
    case MT_METAL:
      if (m->roughness == 0.0f) bs_add(s, B_COND, 0x100u, m->reflectance, 0, 0, 0);
      else bs_add(s, B_MICRO_COND, 0x10u, m->reflectance, m->rcpRoughness, 0, 0);
      s->c[s->n - 1].eta = m->metalEta;
      s->c[s->n - 1].k = m->metalK;
      break;
    case MT_BRUSHED:
      if (m->roughnessX == 0.0f || m->roughnessY == 0.0f) bs_add(s, B_COND, 0x100u, m->reflectance, 0, 0, 0);
      else bs_add(s, B_MICRO_ANISO, 0x10u, m->reflectance, rcp(m->roughnessX), rcp(m->roughnessY), 0);
      s->c[s->n - 1].eta = m->metalEta;
      s->c[s->n - 1].k = m->metalK;
      break;
    case MT_VELVET:
      bs_add(s, B_MINNAERT, 0x1u, m->reflectance, m->backScattering, 0, 0);
      bs_add(s, B_VELVETY, 0x1u, m->horizon, m->fallOff, 0, 0);
      break;
    case MT_MATTE: bs_add(s, B_LAMBERT, 0x1u, m->reflectance, 0, 0, 0); break;
    case MT_MATTE_TEX:
      if (m->Kd >= 0) {
        tex_get(B, m->Kd, m->ds[0] * dg->s + m->s0[0], m->ds[1] * dg->t + m->s0[1], c);
        bs_add(s, B_LAMBERT, 0x1u, v3(c[0], c[1], c[2]), 0, 0, 0);
      }
      break;
    case MT_METALLIC: /* DielectricReflection(1, eta) + DielectricLayer<Lambertian>(one, 1, eta, shadeColor) */
      bs_add(s, B_DIEL_REFL, 0x100u, vs(0.f), 1.0f * rcp(m->eta), 1.0f, 0);
      bs_add(s, B_LAYER, 0x1u, m->shadeColor, 1.0f * rcp(m->eta), m->eta * rcp(1.0f), 0);
      if (m->glitterSpread != 0 && !v3zero(m->glitterColor)) /* metallicpaint.h:63-70 */
        bs_add(s, B_LAYER_GLITTER, 0x10u, m->glitterColor, 1.0f * rcp(m->eta), m->eta * rcp(1.0f),
               rcp(m->glitterSpread));
      break;
    case MT_OBJ: {
      if (m->map_Bump >= 0) {
        tex_get(B, m->map_Bump, dg->s, dg->t, c);
        const V3 b = v3(2.0f * c[0] - 1.0f, 2.0f * c[1] - 1.0f, 2.0f * c[2] - 1.0f);
        dg->Ns = normalize(add(add(muls(dg->Tx, b.x), muls(dg->Ty, b.y)), muls(dg->Ns, b.z)));
      }
      float d = m->d;
      if (m->map_d >= 0) { tex_get(B, m->map_d, dg->s, dg->t, c); d *= c[0]; }
      if (d < 1.0f) bs_add(s, B_TRANS, 0x01000000u, vs(1.0f - d), 0, 0, 0);
      V3 Kd = muls(m->KdC, d);
      if (m->map_Kd >= 0) { tex_get(B, m->map_Kd, dg->s, dg->t, c); Kd = mulv(Kd, v3(c[0], c[1], c[2])); }
      if (!v3zero(Kd)) bs_add(s, B_LAMBERT, 0x1u, Kd, 0, 0, 0);
      float Ns = m->Ns;
      if (m->map_Ns >= 0) { tex_get(B, m->map_Ns, dg->s, dg->t, c); Ns *= c[0]; }
      V3 Ks = muls(m->Ks, d);
      if (m->map_Ks >= 0) { tex_get(B, m->map_Ks, dg->s, dg->t, c); Ks = mulv(Ks, v3(c[0], c[1], c[2])); }
      if (!v3zero(Ks)) bs_add(s, B_SPEC, 0x10u, Ks, Ns, 0, 0);
      break;
    }
    case MT_UBER: {
      float dc[4] = {m->diffuse.x, m->diffuse.y, m->diffuse.z, 1.f};
      float alpha = 1.f, opacity = 0.f;
      if (m->Kd >= 0) {
        tex_get(B, m->Kd, m->ds[0] * dg->s + m->s0[0], m->ds[1] * dg->t + m->s0[1], dc);
        alpha = dc[3];
        opacity = 1.f - alpha;
      }
      bs_add(s, B_LAMBERT, 0x1u, v3(dc[0] * alpha, dc[1] * alpha, dc[2] * alpha), 0, 0, 0);
      if (alpha < 1.f) bs_add(s, B_CONST_TRANS, 0x01000000u, vs(opacity), 0, 0, 0);
      if (m->reflectivity > 0.f) bs_add(s, B_DIEL_REFL, 0x100u, vs(0.f), 1.f * rcp(m->eta), alpha * m->reflectivity, 0);
      else if (m->roughness == 0.f) bs_add(s, B_DIEL_REFL, 0x100u, vs(0.f), 1.f * rcp(m->eta), alpha, 0);
      else bs_add(s, B_MICRO, 0x10u, vs(alpha), 1.f, m->eta, m->rcpRoughness);
      break;
    }
    case MT_THIN: {
      bs_add(s, B_DIEL_REFL, 0x100u, vs(0.f), 1.0f * rcp(m->eta), 1.0f, 0);
      float dc[4] = {m->transmission.x, m->transmission.y, m->transmission.z, 1.f};
      if (m->Kd >= 0) tex_get(B, m->Kd, m->ds[0] * dg->s + m->s0[0], m->ds[1] * dg->t + m->s0[1], dc);
      const V3 T = v3(dc[0] * m->transparency, dc[1] * m->transparency, dc[2] * m->transparency);
      bs_add(s, B_THIN_TRANS, 0x01000000u, v3(yrt_logf(T.x), yrt_logf(T.y), yrt_logf(T.z)), 1.f * rcp(m->eta), m->thickness, 0);
      break;
    }
    default: break;
  }
}

/* HDRILight::Le (lights/hdrilight.cpp:43-71) */
static V3 hdri_Le(const World* W, const Light* L, V3 wo) {
  const V3 wi = xfmVector(L->w2l, neg(wo));
  const float theta = yrt_acosf(clampf_(wi.y, -1.0f, 1.0f));
  float phi = yrt_atan2f(-wi.z, -wi.x);
  if (phi < 0) phi += 2.0f * PI_F;
  const float u = 1.0f - (phi * ONE_OVER_TWO_PI_F), v = theta * ONE_OVER_PI_F;
  int x = (int)(u * L->w);
  x = x < 0 ? 0 : (x > L->w - 1 ? L->w - 1 : x);
  int xn = x + 1;
  if (xn == L->w) xn = 0;
  const float alpha = u * L->w - x;
  int y = (int)(v * L->h);
  y = y < 0 ? 0 : (y > L->h - 1 ? L->h - 1 : y);
  int yn = y + 1;
  if (yn == L->h) yn = L->h - 1;
  const float beta = v * L->h - y;
  float c0[4], c1[4], c2[4], c3[4];
  img_get(W->blob, L->img, x, y, c0);
  img_get(W->blob, L->img, xn, y, c1);
  img_get(W->blob, L->img, xn, yn, c2);
  img_get(W->blob, L->img, x, yn, c3);
  float r[3];
  const float Lc[3] = {L->L.x, L->L.y, L->L.z};
  for (int k = 0; k < 3; ++k) {
    const float t0 = beta * c3[k] + (1 - beta) * c0[k];
    const float t1 = beta * c2[k] + (1 - beta) * c1[k];
    r[k] = Lc[k] * (alpha * t1 + (1 - alpha) * t0);
  }
  return v3(r[0], r[1], r[2]);
}

/* counter hash replacing rand() (identical to the GPU's) */
static inline uint32_t mix32(uint32_t h) {
  h ^= h >> 16; h *= 0x7feb352dU; h ^= h >> 15; h *= 0x846ca68bU; h ^= h >> 16;
  return h;
}
static inline float hash_u01(uint32_t seed, uint32_t pixel, uint32_t sample, uint32_t depthLight) {
  uint32_t h = mix32(seed ^ 0x9e3779b9U);
  h = mix32(h ^ pixel);
  h = mix32(h ^ (sample * 0x85ebca6bU));
  h = mix32(h ^ (depthLight * 0xc2b2ae35U));
  return (float)(h >> 8) * (1.0f / 16777216.0f);
}

typedef struct {
  int maxDepth, rrDepth, spp, sets;
  float minContribution, epsilon, tMaxShadowRay, tMaxShadowJitter;
  V3 up;
  char filter[16];
  int debug;
  int backplate; /* image object or -1 (pathtraceintegrator.cpp:32) */
} RCfg;

/* PathTraceIntegrator::Li (integrators/pathtraceintegrator.cpp:50-217) */
/* path debugging (oracle_debug_path): 32 floats per depth of one (pixel, sample), the layout of the
 * device's YRT_PATH_DEBUG capture in k_shade */
static float* g_pathDbg = NULL;
static void path_dbg(int depth, int tri, const Hit* h, V3 thr, const DG* dg, V3 Lem, V3 wi, float pdf, V3 c, V3 nthr,
                     const Ray* ray, int useDirect) {
  if (!g_pathDbg || depth >= 32) return;
  const V3 z = vs(0.f);
  const V3 P = dg ? dg->P : z, Ns = dg ? dg->Ns : z;
  const float r[32] = {1.f, (float)tri, h->t, h->u, h->v, thr.x, thr.y, thr.z, P.x, P.y, P.z, Ns.x, Ns.y, Ns.z,
                       Lem.x, Lem.y, Lem.z, wi.x, wi.y, wi.z, pdf, c.x, c.y, c.z, nthr.x, nthr.y, nthr.z,
                       ray->dir.x, ray->dir.y, ray->dir.z, ray->org.x, (float)useDirect};
  memcpy(g_pathDbg + depth * 32, r, sizeof(r));
}

static V3 Li(const World* W, const RCfg* R, const Table* T, int rec, Ray ray, uint32_t pixelId, int s, uint32_t seed,
             float pixelX, float pixelY /* state.pixel (integratorrenderer.cpp:162) */, double* nClosest,
             double* nShadow) {
#define S1(d) T->t[(size_t)(5 + (d)) * T->rec + rec]
#define S2X(d) T->t[(size_t)(5 + T->n1 + 2 * (d)) * T->rec + rec]
#define S2Y(d) T->t[(size_t)(5 + T->n1 + 2 * (d) + 1) * T->rec + rec]
  V3 L = vs(0.f), thr = vs(1.f);
  int depth = 0, ignoreVL = 0, unbent = 1;
  Medium medium = {vs(1.0f), 1.0f}; /* Medium::Vacuum() */
  const float eta = 1.f; /* Sample copy drops eta */
  while (depth < R->maxDepth) {
    if (fmax3(thr) < R->minContribution) break;
    Hit h = trace(W, &ray, 0);
    *nClosest += 1;
    const V3 wo = neg(ray.dir);
    if (h.tri < 0) {
      if (R->backplate >= 0 && unbent) { /* pathtraceintegrator.cpp:80-84 */
        const Obj* bp = &W->blob->objs[R->backplate];
        int bx = (int)(pixelX * (float)bp->imgW), by = (int)(pixelY * (float)bp->imgH);
        bx = bx < 0 ? 0 : bx > bp->imgW - 1 ? bp->imgW - 1 : bx;
        by = by < 0 ? 0 : by > bp->imgH - 1 ? bp->imgH - 1 : by;
        float c[4];
        img_get(W->blob, R->backplate, bx, by, c);
        L = add(L, mulv(thr, v3(c[0], c[1], c[2])));
      } else if (!ignoreVL)
        for (int i = 0; i < W->nenv; i++) {
          const Light* E = &W->lights[W->env[i]];
          V3 Le;
          if (E->type == LT_AMBIENT) Le = E->L;
          else if (E->type == LT_DISTANT) Le = dot(neg(wo), E->D) >= E->cosHalf ? E->L : vs(0.f); /* distantlight.h:38-41 */
          else Le = hdri_Le(W, E, wo);
          L = add(L, mulv(thr, Le));
        }
      if (g_pathDbg) { Hit hz = {0.f, 0.f, 0.f, -1}; path_dbg(depth, -1, &hz, thr, NULL, L, vs(0.f), 0.f, vs(0.f), vs(0.f), &ray, 0); }
      break;
    }
    DG dg;
    post_intersect(W, &ray, &h, &dg);
    int backfacing = 0;
    if (dot(dg.Ng, ray.dir) > 0.f) { backfacing = 1; dg.Ng = neg(dg.Ng); dg.Ns = neg(dg.Ns); }
    BSet bs;
    bs.n = 0;
    shade(W, &W->mats[dg.material], medium, &dg, &bs);
    if (!ignoreVL && dg.light >= 0 && !backfacing) L = add(L, mulv(thr, W->lights[dg.light].L));
    int useDirect = 0;
    for (int i = 0; i < bs.n; i++) useDirect |= (bs.c[i].type & BT_DIFFUSE) != 0;
    const V3 Lem = L;
#define PATH_DBG(wi_, pdf_, c_, nthr_) \
  if (g_pathDbg) path_dbg(depth, h.tri, &h, thr, &dg, Lem, wi_, pdf_, c_, nthr_, &ray, useDirect)
    if (useDirect) {
      for (int li = 0; li < W->nlights; li++) {
        const Light* Lt = &W->lights[li];
        if ((Lt->illumMask & dg.illumMask) == 0) continue;
        V3 wi = vs(0.f), Ls = vs(0.f);
        float pdf = 0.f;
        if (Lt->precomp >= 0) {
          const float* ls = &T->light[((size_t)rec * T->nl + Lt->precomp) * 8];
          wi = v3(ls[0], ls[1], ls[2]);
          pdf = ls[3];
          Ls = v3(ls[4], ls[5], ls[6]);
        } else if (Lt->type == LT_AMBIENT) { /* ambientlight.h:52-65 */
          wi = cos_hemi(S2X(0), S2Y(0), dg.Ns, &pdf);
          Ls = Lt->L;
        } else if (Lt->type == LT_TRIANGLE) { /* trianglelight.h:77-85 */
          const float sx = S2X(0), sy = S2Y(0);
          const float su = sqrtf(sx);
          const V3 d = sub(add(add(Lt->v2, muls(sub(Lt->v0, Lt->v2), 1.0f - su)), muls(sub(Lt->v1, Lt->v2), sy * su)), dg.P);
          const float tMax = length(d);
          const float dDotNg = dot(d, Lt->Ng);
          if (dDotNg >= 0) continue; /* returns zero radiance */
          wi = muls(d, rcp(tMax));
          pdf = 2.0f * tMax * tMax * tMax * rcp(fabsf(dDotNg));
          Ls = Lt->L;
        } else if (Lt->type == LT_POINT) { /* pointlight.h:36-42 */
          const V3 d = sub(Lt->P, dg.P);
          const float dist = length(d);
          wi = divs(d, dist);
          pdf = dist * dist;
          Ls = Lt->L;
        } else if (Lt->type == LT_SPOT) { /* spotlight.h:41-52 */
          const V3 d = sub(Lt->P, dg.P);
          const float dist = length(d);
          wi = muls(d, rcp(dist));
          pdf = dist * dist;
          const float ca = dot(wi, Lt->D);
          if (Lt->cosMin != Lt->cosMax) Ls = muls(Lt->L, clamp01((ca - Lt->cosMax) * rcp(Lt->cosMin - Lt->cosMax)));
          else Ls = ca > Lt->cosMin ? Lt->L : vs(0.f);
        } else if (Lt->type == LT_DIRECTIONAL) { /* directionallight.h:31-33 */
          wi = Lt->D;
          pdf = 1.0f;
          Ls = Lt->L;
        } else if (Lt->type == LT_DISTANT) { /* distantlight.h:46-50, shapesampler.h:149-165 */
          const float ang = Lt->halfAngle;
          const float phi = TWO_PI_F * S2X(0);
          const float cT = 1.0f - S2Y(0) * (1.0f - yrt_cosf(ang));
          const float sT = sqrtf(fmaxf(0.0f, 1.0f - cT * cT));
          pdf = rcp(4.0f * PI_F * (yrt_sinf(0.5f * ang) * yrt_sinf(0.5f * ang)));
          wi = lmul(frame_(Lt->D), v3(yrt_cosf(phi) * sT, yrt_sinf(phi) * sT, cT));
          Ls = Lt->L;
        }
        if (v3zero(Ls) || pdf == 0.f) continue;
        const V3 brdf = bs_eval(&bs, wo, &dg, wi, BT_DIFFUSE);
        if (v3zero(brdf)) continue;
        const float r01 = hash_u01(seed, pixelId, (uint32_t)s, (uint32_t)(depth * 64 + li));
        const float jl = 2.f * R->tMaxShadowRay * R->tMaxShadowJitter * r01 - R->tMaxShadowRay * R->tMaxShadowJitter;
        float tMax = R->tMaxShadowRay + jl;
        const float dp = dot(wi, R->up);
        if (dp <= 0.f) tMax += R->tMaxShadowRay * 100.f * smoothstep_(0.f, 1.f, fabsf(dp));
        Ray sr = {dg.P, wi, dg.error * R->epsilon, tMax - dg.error * R->epsilon, ray.time}; /* lastRay.time (:158) */
        Hit sh = trace(W, &sr, 1);
        *nShadow += 1;
        if (sh.tri >= 0) continue;
        L = add(L, muls(mulv(mulv(thr, Ls), brdf), rcp(pdf)));
      }
    }
    if (depth >= R->maxDepth - 1) { PATH_DBG(vs(0.f), 0.f, vs(0.f), vs(0.f)); break; }
    if (R->rrDepth > 0 && depth >= R->rrDepth - 1) {
      const float q = fminf(fmax3(thr) * eta * eta, .95f);
      if (S1(depth) >= q) { PATH_DBG(vs(0.f), 0.f, vs(0.f), vs(0.f)); break; }
    }
    V3 wi;
    float pdf;
    uint32_t type;
    V3 c = bs_sample(&bs, wo, &dg, S2X(1 + depth), S2Y(1 + depth), S1(depth), &wi, &pdf, &type);
    if (v3zero(c) || pdf <= 0.f) { PATH_DBG(wi, pdf, c, vs(0.f)); break; }
    const V3 cDbg = c;
    /* simple volumetric effect and medium tracking (pathtraceintegrator.cpp:197-207) */
    if (!veq(medium.T, vs(1.0f)))
      c = mulv(c, v3(yrt_powf(medium.T.x, h.t), yrt_powf(medium.T.y, h.t), yrt_powf(medium.T.z, h.t)));
    if (type & 0xFFFF0000u) {
      const Material* mt = &W->mats[dg.material];
      if (mt->type == MT_DIELECTRIC) medium = med_eq(medium, mt->inside) ? mt->outside : mt->inside;
    }
    PATH_DBG(wi, pdf, cDbg, muls(mulv(thr, c), rcp(pdf)));
#undef PATH_DBG
    thr = muls(mulv(thr, c), rcp(pdf));
    ignoreVL = (type & BT_DIFFUSE) != 0;
    unbent = unbent && veq(wi, ray.dir); /* LightPath::extended (pathtraceintegrator.h:45) */
    ray.org = dg.P;
    ray.dir = wi;
    ray.tnear = dg.error * R->epsilon;
    ray.tfar = INFINITY;
    depth++;
  }
  return L;
#undef S1
#undef S2X
#undef S2Y
}

static int rcfg_build(const Blob* B, RCfg* R) {
  memset(R, 0, sizeof(*R));
  R->backplate = -1;
  if (B->renderer < 0) return fail("no renderer");
  const Obj* o = &B->objs[B->renderer];
  if (!strcasecmp(o->type, "debug")) { /* debugrenderer.cpp:21-25 */
    R->debug = 1;
    R->maxDepth = p_int(o, "maxDepth", 1);
    R->spp = p_int(o, "sampler.spp", 1);
    R->sets = 64;
    strcpy(R->filter, "none");
    return 0;
  }
  /* integratorrenderer.cpp:31-61, pathtraceintegrator.cpp:21-33, sampler.cpp:23-31 */
  R->maxDepth = p_int(o, "maxDepth", 10);
  R->rrDepth = p_int(o, "rrDepth", 5);
  R->minContribution = p_float(o, "minContribution", .02f);
  R->epsilon = p_float(o, "epsilon", 32.f) * ULP_F;
  R->tMaxShadowRay = p_float(o, "tMaxShadowRay", INFINITY);
  R->tMaxShadowJitter = p_float(o, "tMaxShadowJitter", .15f);
  R->up = p_v3(o, "up", v3(0.f, 1.f, 0.f));
  R->spp = p_int(o, "sampler.spp", 1);
  if (R->spp < 1) R->spp = 1;
  R->sets = p_int(o, "sampler.sets", 64);
  if (R->sets < 1) R->sets = 1;
  snprintf(R->filter, sizeof(R->filter), "%s", p_str(o, "filter", "bspline"));
  R->backplate = p_obj(o, "backplate");
  return 0;
}

/* ====================================================================== render driver */
typedef struct {
  const World* W;
  const RCfg* R;
  const Table* T;
  const Camera* C;
  const uint8_t* sets;
  int width, height, x0, y0, x1, y1, ntx, nty;
  int shardIndex, shardCount; /* only logical tiles with lt % shardCount == shardIndex */
  float gamma;
  uint32_t seed;
  float* out;
  volatile int next;
  double nClosest, nShadow;
  pthread_mutex_t mu;
} Job;

/* RenderJob::renderTile (integratorrenderer.cpp:118-185) */
static void* worker(void* arg) {
  Job* J = (Job*)arg;
  double nc = 0, ns = 0;
  const float rcpW = rcp((float)J->width), rcpH = rcp((float)J->height);
  for (;;) {
    const int lt = __sync_fetch_and_add(&J->next, 1);
    if (lt >= J->ntx * J->nty) break;
    if (lt % J->shardCount != J->shardIndex) continue;
    /* the product's deal (not the reference's): logical tile lt of a sharded frame covers image
     * tile yrt_tile_scatter(lt, T), common/yrt_tile_scatter.h */
    const int tile = J->shardCount > 1 ? yrt_tile_scatter(lt, J->ntx * J->nty) : lt;
    const int tx = (tile % J->ntx) * 16, ty = (tile / J->ntx) * 16;
    for (int dy = 0; dy < 16; dy++) {
      const int y = ty + dy;
      if (y >= J->height || y < J->y0 || y >= J->y1) continue;
      for (int dx = 0; dx < 16; dx++) {
        const int x = tx + dx;
        if (x >= J->width || x < J->x0 || x >= J->x1) continue;
        const int set = J->sets[(size_t)y * J->width + x];
        V3 L = vs(0.f);
        const int spp = J->T->spp;
        for (int s = 0; s < spp; s++) {
          const int rec = set * spp + s;
          const float fx = ((float)x + J->T->t[rec]) * rcpW;
          const float fy = ((float)y + J->T->t[(size_t)J->T->rec + rec]) * rcpH;
          Ray ray;
          camera_ray(J->C, fx, fy, J->T->t[(size_t)2 * J->T->rec + rec], J->T->t[(size_t)3 * J->T->rec + rec], &ray.org,
                     &ray.dir); /* sample.getLens() */
          ray.tnear = 0.f;
          ray.tfar = INFINITY;
          ray.time = J->T->t[(size_t)4 * J->T->rec + rec]; /* primary.time = sample.getTime() (:159) */
          L = add(L, Li(J->W, J->R, J->T, rec, ray, (uint32_t)(y * J->width + x), s, J->seed, fx, fy, &nc, &ns));
        }
        /* AccuBuffer::update + DefaultToneMapper::eval */
        V3 L0 = muls(L, rcp((float)spp));
        if (J->gamma != 1.0f) {
          const float rg = rcp(J->gamma);
          L0 = v3(yrt_powf(L0.x, rg), yrt_powf(L0.y, rg), yrt_powf(L0.z, rg));
        }
        float* o = &J->out[((size_t)y * J->width + x) * 3];
        o[0] = L0.x; o[1] = L0.y; o[2] = L0.z;
      }
    }
  }
  pthread_mutex_lock(&J->mu);
  J->nClosest += nc;
  J->nShadow += ns;
  pthread_mutex_unlock(&J->mu);
  return NULL;
}

/* DebugRenderer::RenderJob::renderTile (debugrenderer.cpp:66-140) */
/* The frame blob's camera rays for pixel coordinates px[2i] = fx, px[2i+1] = fy (lens sample 0):
 * org[3i], dir[3i]. For the pin of the camera path against the reference's own operations. */
int oracle_camera_rays(const void* blob, size_t bytes, int n, const float* px, float* org, float* dir) {
  Blob B;
  if (blob_parse(blob, bytes, &B)) return -1;
  Camera C;
  if (camera_build(&B, &C)) { blob_free(&B); return -1; }
  for (int i = 0; i < n; ++i) {
    V3 o, d;
    camera_ray(&C, px[2 * i], px[2 * i + 1], 0.f, 0.f, &o, &d);
    org[3 * i] = o.x; org[3 * i + 1] = o.y; org[3 * i + 2] = o.z;
    dir[3 * i] = d.x; dir[3 * i + 1] = d.y; dir[3 * i + 2] = d.z;
  }
  blob_free(&B);
  return 0;
}

static void debug_render(const World* W, const RCfg* R, const Camera* C, int width, int height, float* out) {
  const int ntx = (width + 15) / 16, nty = (height + 15) / 16;
  const float rcpW = rcp((float)width), rcpH = rcp((float)height);
  for (int tile = 0; tile < ntx * nty; ++tile) {
    Rnd rnd;
    rnd_seed(&rnd, tile * 1024);
    const int x0 = (tile % ntx) * 16, y0 = (tile / ntx) * 16;
    for (int dy = 0; dy < 16; dy++) {
      const int iy = y0 + dy;
      const float fy = iy * rcpH;
      if (iy >= height) continue;
      for (int dx = 0; dx < 16; dx++) {
        const int ix = x0 + dx;
        const float fx = ix * rcpW;
        if (ix >= width) continue;
        for (int i = 0; i < R->spp; i++) {
          Ray ray;
          camera_ray(C, fx, fy, 0.f, 0.f, &ray.org, &ray.dir);
          ray.tnear = 0.f;
          ray.tfar = INFINITY;
          ray.time = 0.f; /* the debug renderer's rays keep Ray's default time (ray.h:33) */
          int id0 = -1, id1 = -1;
          for (int depth = 0; depth < R->maxDepth; depth++) {
            Hit h = trace(W, &ray, 0);
            if (h.tri < 0) { id0 = id1 = -1; break; }
            id0 = W->triGeom[h.tri];
            id1 = h.tri - W->geoms[id0].triBase;
            if (depth + 1 < R->maxDepth) {
              V3 Nf = normalize(cross(W->te1[h.tri], W->te2[h.tri]));
              if (dot(neg(ray.dir), Nf) < 0) Nf = neg(Nf);
              const float u1 = rnd_float(&rnd), u2 = rnd_float(&rnd);
              float pdf;
              const V3 norg = add(ray.org, muls(ray.dir, 0.999f * h.t));
              ray.dir = cos_hemi(u1, u2, Nf, &pdf);
              ray.org = norg;
              ray.tnear = 4.0f * ULP_F;
              ray.tfar = INFINITY;
            }
          }
          float* o = &out[((size_t)iy * width + ix) * 3];
          if (id0 < 0) { o[0] = o[1] = o[2] = 1.0f; }
          else {
            o[0] = ((3434553u * (unsigned)(id0 + id1 + 3243)) % 255) / 255.0f;
            o[1] = ((7342453u * (unsigned)(id0 + id1 + 8237)) % 255) / 255.0f;
            o[2] = ((9234454u * (unsigned)(id0 + id1 + 2343)) % 255) / 255.0f;
          }
        }
      }
    }
  }
}

int oracle_render(const void* blob, size_t bytes, int width, int height, float gamma, int x0, int y0, int x1, int y1,
                  int threads, float* out, OracleStats* stats) {
  return oracle_render_shard(blob, bytes, width, height, gamma, x0, y0, x1, y1, 0, 1, threads, out, stats);
}

int oracle_render_shard(const void* blob, size_t bytes, int width, int height, float gamma, int x0, int y0, int x1,
                        int y1, int shardIndex, int shardCount, int threads, float* out, OracleStats* stats) {
  if (shardCount < 1 || shardIndex < 0 || shardIndex >= shardCount) return -1;
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  Blob B;
  if (blob_parse(blob, bytes, &B)) return -1;
  World W;
  if (world_build(&B, &W)) { blob_free(&B); return -1; }
  RCfg R;
  Camera C;
  if (rcfg_build(&B, &R) || camera_build(&B, &C)) { world_free(&W); blob_free(&B); return -1; }
  if (R.debug) {
    debug_render(&W, &R, &C, width, height, out);
    if (stats) memset(stats, 0, sizeof(*stats));
    world_free(&W);
    blob_free(&B);
    return 0;
  }
  Table T;
  table_build(&T, R.spp, R.sets, 0, R.maxDepth, 1 + R.maxDepth, R.filter, &W);
  uint8_t* sets = (uint8_t*)malloc((size_t)width * height);
  oracle_pixel_sets(width, height, T.sets, sets);
  Job J;
  memset(&J, 0, sizeof(J));
  J.W = &W; J.R = &R; J.T = &T; J.C = &C; J.sets = sets;
  J.width = width; J.height = height;
  J.x0 = x0 < 0 ? 0 : x0; J.y0 = y0 < 0 ? 0 : y0;
  J.x1 = x1 <= 0 || x1 > width ? width : x1; J.y1 = y1 <= 0 || y1 > height ? height : y1;
  J.ntx = (width + 15) / 16; J.nty = (height + 15) / 16;
  J.shardIndex = shardIndex; J.shardCount = shardCount;
  J.gamma = gamma;
  J.seed = B.seed;
  J.out = out;
  pthread_mutex_init(&J.mu, NULL);
  if (threads <= 0) threads = (int)sysconf(_SC_NPROCESSORS_ONLN);
  if (threads < 1) threads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
  for (int i = 0; i < threads; ++i) pthread_create(&th[i], NULL, worker, &J);
  for (int i = 0; i < threads; ++i) pthread_join(th[i], NULL);
  free(th);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  if (stats) {
    memset(stats, 0, sizeof(*stats));
    stats->raysClosest = J.nClosest;
    stats->raysShadow = J.nShadow;
    stats->samples = (double)(J.x1 - J.x0) * (J.y1 - J.y0) * T.spp;
    stats->seconds = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
  }
  pthread_mutex_destroy(&J.mu);
  free(sets);
  free(T.t);
  free(T.light);
  world_free(&W);
  blob_free(&B);
  return 0;
}

/* Debug: the per-sample radiance Li of one pixel (the terms the pixel's sum adds in s order),
 * out3[3*s..3*s+2] for s < spp; returns spp (or -1). */
static int debug_pixel_impl(const void* blob, size_t bytes, int width, int height, int x, int y, float* out3,
                            int maxSpp, int only);
int oracle_debug_pixel(const void* blob, size_t bytes, int width, int height, int x, int y, float* out3, int maxSpp) {
  return debug_pixel_impl(blob, bytes, width, height, x, y, out3, maxSpp, -1);
}
int oracle_debug_path(const void* blob, size_t bytes, int width, int height, int x, int y, int sample, float* out) {
  float L[3 * 4096];
  if (sample < 0 || sample >= 4096) return -1;
  memset(out, 0, sizeof(float) * 32 * 32);
  g_pathDbg = out;
  const int r = debug_pixel_impl(blob, bytes, width, height, x, y, L, sample + 1, sample);
  g_pathDbg = NULL;
  return r;
}
static int debug_pixel_impl(const void* blob, size_t bytes, int width, int height, int x, int y, float* out3,
                            int maxSpp, int only) {
  Blob B;
  if (blob_parse(blob, bytes, &B)) return -1;
  World W;
  if (world_build(&B, &W)) { blob_free(&B); return -1; }
  RCfg R;
  Camera C;
  if (rcfg_build(&B, &R) || camera_build(&B, &C) || R.debug) { world_free(&W); blob_free(&B); return -1; }
  Table T;
  table_build(&T, R.spp, R.sets, 0, R.maxDepth, 1 + R.maxDepth, R.filter, &W);
  uint8_t* sets = (uint8_t*)malloc((size_t)width * height);
  oracle_pixel_sets(width, height, T.sets, sets);
  const float rcpW = rcp((float)width), rcpH = rcp((float)height);
  const int set = sets[(size_t)y * width + x];
  double nc = 0, ns = 0;
  const int spp = T.spp;
  for (int s = 0; s < spp && s < maxSpp; s++) {
    if (only >= 0 && s != only) continue;
    const int rec = set * spp + s;
    const float fx = ((float)x + T.t[rec]) * rcpW;
    const float fy = ((float)y + T.t[(size_t)T.rec + rec]) * rcpH;
    Ray ray;
    camera_ray(&C, fx, fy, T.t[(size_t)2 * T.rec + rec], T.t[(size_t)3 * T.rec + rec], &ray.org, &ray.dir);
    ray.tnear = 0.f;
    ray.tfar = INFINITY;
    ray.time = T.t[(size_t)4 * T.rec + rec];
    const V3 L = Li(&W, &R, &T, rec, ray, (uint32_t)(y * width + x), s, B.seed, fx, fy, &nc, &ns);
    out3[3 * s] = L.x; out3[3 * s + 1] = L.y; out3[3 * s + 2] = L.z;
  }
  free(sets);
  free(T.t);
  free(T.light);
  world_free(&W);
  blob_free(&B);
  return spp;
}

int oracle_trace(const void* blob, size_t bytes, const float* org4, const float* dir4, int n, int anyHit, float* hit4) {
  Blob B;
  if (blob_parse(blob, bytes, &B)) return -1;
  World W;
  if (world_build(&B, &W)) { blob_free(&B); return -1; }
  for (int i = 0; i < n; ++i) {
    Ray r = {v3(org4[4 * i], org4[4 * i + 1], org4[4 * i + 2]), v3(dir4[4 * i], dir4[4 * i + 1], dir4[4 * i + 2]),
             org4[4 * i + 3], dir4[4 * i + 3]};
    Hit h = trace(&W, &r, anyHit);
    if (anyHit) {
      hit4[4 * i] = hit4[4 * i + 1] = hit4[4 * i + 2] = 0.f;
      int o = h.tri >= 0;
      memcpy(&hit4[4 * i + 3], &o, 4);
    } else {
      hit4[4 * i] = h.t; hit4[4 * i + 1] = h.u; hit4[4 * i + 2] = h.v;
      memcpy(&hit4[4 * i + 3], &h.tri, 4);
    }
  }
  world_free(&W);
  blob_free(&B);
  return 0;
}

int oracle_scene_triangles(const void* blob, size_t bytes, float* out, int maxTris) {
  Blob B;
  if (blob_parse(blob, bytes, &B)) return -1;
  World W;
  if (world_build(&B, &W)) { blob_free(&B); return -1; }
  const int n = W.ntris;
  if (out) memcpy(out, W.tv, sizeof(float) * 9 * (size_t)(n < maxTris ? n : maxTris));
  world_free(&W);
  blob_free(&B);
  return n;
}

/* Device BVH node/tri layout (yulio-raytracer_amd/csrc/common/yrt_gpu_types.h: 4-wide 128-B
 * nodes, 48-B triangles), traversed depth-first in the device kernel's child order (nearest
 * hit child first, the others pushed farthest-first) to count visits for the roofline's
 * algorithmic bytes. The wavefront kernel additionally parks one leaf while it
 * keeps descending (speculative traversal), which can add a few node visits per ray, so
 * these counts are a lower bound on the kernel's node fetches. */
typedef struct { float lox[4], hix[4], loy[4], hiy[4], loz[4], hiz[4]; int32_t child[4], pad[4]; } DNode;
typedef struct { float v0[4], e1[4], e2[4]; } DTri;
/* The 64-B quantized node of the same index (yulio-raytracer_amd/csrc/common/yrt_qnode.h): origin,
 * biased quantum exponents, children, plane bytes (lo x, hi x, lo y, hi y, lo z, hi z; byte k =
 * child k). The kernel's box4_quant: per axis a = fma(origin, inv, -org*inv) and
 * s = 2^e * inv, per plane fma(q, s, a). */
typedef struct { float origin[3]; uint32_t exps; int32_t child[4]; uint32_t q[6], pad[2]; } QNode;
static int count_visits_impl(const void* nodes_, const void* qnodes_, const void* tris_, const float* org4,
                             const float* dir4, int n, int anyHit, double* nodeVisits, double* triVisits, float* hit4,
                             size_t triStride);
int oracle_count_visits(const void* nodes_, size_t numNodes, const void* tris_, size_t numTris, const float* org4,
                        const float* dir4, int n, int anyHit, double* nodeVisits, double* triVisits, float* hit4,
                        size_t triStride /* bytes per leaf record: 48, or 64 with a stored normal */) {
  (void)numNodes; (void)numTris;
  return count_visits_impl(nodes_, NULL, tris_, org4, dir4, n, anyHit, nodeVisits, triVisits, hit4, triStride);
}
/* the same traversal on the quantized nodes (the any-hit kernel's) */
int oracle_count_visits_q(const void* qnodes_, size_t numNodes, const void* tris_, size_t numTris, const float* org4,
                          const float* dir4, int n, int anyHit, double* nodeVisits, double* triVisits, float* hit4,
                          size_t triStride) {
  (void)numNodes; (void)numTris;
  return count_visits_impl(NULL, qnodes_, tris_, org4, dir4, n, anyHit, nodeVisits, triVisits, hit4, triStride);
}
static int count_visits_impl(const void* nodes_, const void* qnodes_, const void* tris_, const float* org4,
                             const float* dir4, int n, int anyHit, double* nodeVisits, double* triVisits, float* hit4,
                             size_t triStride) {
  const DNode* nodes = (const DNode*)nodes_;
  const QNode* qnodes = (const QNode*)qnodes_;
  const char* trisBytes = (const char*)tris_;
  double nv = 0, tv = 0;
  const float INF = (float)INFINITY;
  for (int i = 0; i < n; ++i) {
    Ray r = {v3(org4[4 * i], org4[4 * i + 1], org4[4 * i + 2]), v3(dir4[4 * i], dir4[4 * i + 1], dir4[4 * i + 2]),
             org4[4 * i + 3], dir4[4 * i + 3]};
    Hit best = {r.tfar, 0, 0, -1};
    if (r.tfar >= r.tnear) {
      const V3 inv = v3(safe_inv(r.dir.x), safe_inv(r.dir.y), safe_inv(r.dir.z));
      const float o[3] = {r.org.x, r.org.y, r.org.z}, iv[3] = {inv.x, inv.y, inv.z};
      /* the kernel's fused slab test (yrt_traverse.h box4_ordered): fma(plane, inv, -org*inv),
       * far distances widened by 2^-22 * max|org*inv| on top of the robust factor */
      const float oi[3] = {o[0] * iv[0], o[1] * iv[1], o[2] * iv[2]};
      const float margin = fmaxf(fmaxf(fabsf(oi[0]), fabsf(oi[1])), fabsf(oi[2])) * 2.384185791015625e-07f;
      int stack[128], sp = 0, cur = 0, done = 0;
      while (!done) {
        if ((cur & 31) == 0) {
          nv += 1;
          float t[4];
          int c[4];
          for (int k = 0; k < 4; ++k) {
            float l[3], h[3];
            int child;
            if (qnodes) {
              const QNode* qn = &qnodes[cur >> 5];
              for (int a = 0; a < 3; ++a) {
                uint32_t eb = ((qn->exps >> (8 * a)) & 0xffu) << 23;
                float scale;
                memcpy(&scale, &eb, 4);
                const float s = scale * iv[a], ax = fmaf(qn->origin[a], iv[a], -oi[a]);
                l[a] = fmaf((float)((qn->q[2 * a] >> (8 * k)) & 0xffu), s, ax);
                h[a] = fmaf((float)((qn->q[2 * a + 1] >> (8 * k)) & 0xffu), s, ax);
              }
              child = qn->child[k];
            } else {
              const DNode* nd = &nodes[cur >> 5];
              const float lo[3] = {nd->lox[k], nd->loy[k], nd->loz[k]}, hi[3] = {nd->hix[k], nd->hiy[k], nd->hiz[k]};
              for (int a = 0; a < 3; ++a) { l[a] = fmaf(lo[a], iv[a], -oi[a]); h[a] = fmaf(hi[a], iv[a], -oi[a]); }
              child = nd->child[k];
            }
            const float nn = fmaxf(fmaxf(fminf(l[0], h[0]), fminf(l[1], h[1])), fmaxf(fminf(l[2], h[2]), r.tnear));
            const float ff = fminf(fminf(fmaxf(l[0], h[0]), fmaxf(l[1], h[1])), fminf(fmaxf(l[2], h[2]), best.t));
            const int hit = nn <= fmaf(ff, 1.0000152587890625f, margin) && child != -1;
            t[k] = hit ? nn : INF;
            c[k] = child;
          }
          /* 5-comparator sort network, as the kernel's sort4; any-hit rays take the farthest
           * hit child first, the others in slot order (the kernel's sort3_far: descending
           * comparators (0,1), (2,3), (0,2) with misses at -INF) */
          static const int net[5][2] = {{0, 1}, {2, 3}, {0, 2}, {1, 3}, {1, 2}};
          if (anyHit) {
            for (int k = 0; k < 4; ++k)
              if (!(t[k] < INF)) t[k] = -INF;
            for (int m = 0; m < 3; ++m) {
              const int a = net[m][0], b = net[m][1];
              if (t[b] > t[a]) {
                const float tt = t[a]; t[a] = t[b]; t[b] = tt;
                const int cc = c[a]; c[a] = c[b]; c[b] = cc;
              }
            }
            for (int k = 0; k < 4; ++k)
              if (t[k] == -INF) t[k] = INF;
          } else {
            for (int m = 0; m < 5; ++m) {
              const int a = net[m][0], b = net[m][1];
              if (t[b] < t[a]) {
                const float tt = t[a]; t[a] = t[b]; t[b] = tt;
                const int cc = c[a]; c[a] = c[b]; c[b] = cc;
              }
            }
          }
          if (t[3] < INF) stack[sp++] = c[3];
          if (t[2] < INF) stack[sp++] = c[2];
          if (t[1] < INF) stack[sp++] = c[1];
          if (t[0] < INF) {
            cur = c[0];
            continue;
          }
        } else {
          const int ci = cur >> 5, cc = cur & 31;
          for (int k = 0; k < cc; ++k) {
            const DTri* t = (const DTri*)(trisBytes + (size_t)(ci + k) * triStride);
            tv += 1;
            uint32_t fl;
            int gid;
            memcpy(&fl, &t->e1[3], 4);
            memcpy(&gid, &t->v0[3], 4);
            float tt, u, v;
            int ok = tri_test(v3(t->v0[0], t->v0[1], t->v0[2]), v3(t->e1[0], t->e1[1], t->e1[2]),
                              v3(t->e2[0], t->e2[1], t->e2[2]), fl, &r, anyHit ? r.tfar : best.t, &tt, &u, &v);
            if (anyHit) {
              if (ok) { best.t = tt; best.u = u; best.v = v; best.tri = gid; done = 1; break; }
            } else {
              if (!ok && best.tri >= 0 && tt == best.t && gid < best.tri) {
                float t2, u2, v2;
                ok = tri_test(v3(t->v0[0], t->v0[1], t->v0[2]), v3(t->e1[0], t->e1[1], t->e1[2]),
                              v3(t->e2[0], t->e2[1], t->e2[2]), fl, &r, r.tfar, &t2, &u2, &v2);
              }
              if (ok) { best.t = tt; best.u = u; best.v = v; best.tri = gid; }
            }
          }
          if (done) break;
        }
        if (sp == 0) break;
        cur = stack[--sp];
      }
    }
    if (hit4) {
      hit4[4 * i] = best.t; hit4[4 * i + 1] = best.u; hit4[4 * i + 2] = best.v;
      memcpy(&hit4[4 * i + 3], &best.tri, 4);
    }
  }
  *nodeVisits = nv;
  *triVisits = tv;
  return 0;
}
