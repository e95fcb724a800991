// yrt_shade.h — device-side postIntersect, materials, BRDFs and lights.
//
// Each function restates the reference's CPU code, keeping the order of the float
// operations (left-to-right Color*float products etc.) so the GPU and the oracle agree:
//   postIntersect   shapes/trianglemesh_full.cpp:192-260, trianglemesh_normals.cpp:125-147,
//                   shapes/triangle.h:69-78
//   materials       materials/{matte,matte_textured,metallicpaint,obj,Uber,thindielectric,plastic,
//                   dielectric,mirror,metal,brushedmetal,velvet}.h
//   BRDFs           brdfs/{lambertian,dielectric,dielectriclayer,microfacet,specular,
//                   transmission,optics,reflection,conductor,minnaert,velvety}.h,
//                   brdfs/microfacet/{power_cosine_distribution,anisotropic_power_cosine_distribution,fresnel}.h
//   composition     brdfs/compositedbrdf.h:58-166
//   lights          lights/{ambientlight,trianglelight}.h, lights/hdrilight.cpp
//   textures        textures/{Bilinear,nearestneighbor}.h, texel decode
//                   common/math/color_scalar.h:47 (byte * one_over_255)
// Omitted reference features (no BASELINE config reaches them): motion blur, metallic-paint
// glitter, the Beckmann distributions (no material instantiates them); DESIGN.md §7 lists them.
// The backplate image is read in k_shade (pathtrace.hip) for camera-ray misses.
#pragma once

#include "../common/yrt_gpu_types.h"
#include "../common/yrt_math.h"

namespace yrt {

// BRDF type bits (brdfs/brdf.h:10-30)
enum : uint32_t {
  BT_DIFFUSE = 0x000F000Fu,
  BT_DIFFUSE_REFLECTION = 0x00000001u,
  BT_GLOSSY_REFLECTION = 0x00000010u,
  BT_SPECULAR_REFLECTION = 0x00000100u,
  BT_SPECULAR_TRANSMISSION = 0x01000000u,
  BT_TRANSMISSION = 0xFFFF0000u,
};

enum CompKind : int {
  C_LAMBERT = 0,          // Lambertian(R)
  C_DIEL_REFL = 1,        // DielectricReflection(eta_, alpha)          a=eta_, b=alpha
  C_CONST_DIEL_TRANS = 2, // ConstDielectricTransmission(color)         R=color
  C_THIN_DIEL_TRANS = 3,  // ThinDielectricTransmission(eta_, logT, th) R=logT, a=eta_, b=thickness
  C_DIEL_LAYER_LAMB = 4,  // DielectricLayer<Lambertian>(T=1, etait, etati, R)  a=etait, b=etati
  C_MICROFACET = 5,       // Microfacet<FresnelDielectric(etai,etat),PowerCosine(n,Ns)> R, a=etai, b=etat, c=n
  C_TRANSMISSION = 6,     // Transmission(T)
  C_SPECULAR = 7,         // Specular(R, exp)                            a=exp
  C_REFLECTION = 8,       // Reflection(R)
  C_CONDUCTOR = 9,        // Conductor(R, eta, k)                        c=material id (eta, k)
  C_MICRO_COND = 10,      // Microfacet<FresnelConductor,PowerCosine>    R, a=n, c=material id
  C_MICRO_ANISO = 11,     // Microfacet<FresnelConductor,AnisotropicPowerCosine(Tx,nx,Ty,ny,Ns)>
                          //                                             R, a=nx, b=ny, c=material id
  C_MINNAERT = 12,        // Minnaert(R, b)                              a=b
  C_VELVETY = 13,         // Velvety(R, f)                               a=f
  C_DIEL_TRANS = 14,      // DielectricTransmission(etai, etat)          a=eta_
  C_DIEL_LAYER_GLITTER = 15,  // DielectricLayer<Microfacet<FresnelConductor(Al),PowerCosine(n,Ns)>>
                              // (T=1, etait, etati, glitterColor)           R, a=etait, b=etati, c=n
};

// Material-set specialization: the shade kernel is instantiated for a bitmask of material
// types (bit MAT_x); only the BRDF components those materials can create are compiled in,
// which cuts register pressure for scenes with few material types.
__host__ __device__ constexpr unsigned mat_bit(int m) { return 1u << m; }
__host__ __device__ constexpr unsigned comp_bit(int c) { return 1u << c; }
__host__ __device__ constexpr unsigned comps_of(unsigned mats) {
  return ((mats & (mat_bit(1) | mat_bit(2))) ? comp_bit(0) : 0u) |                                  // Matte(Textured)
         ((mats & mat_bit(3)) ? (comp_bit(1) | comp_bit(4)) : 0u) |                                 // MetallicPaint
         ((mats & mat_bit(4)) ? (comp_bit(6) | comp_bit(0) | comp_bit(7)) : 0u) |                   // Obj
         ((mats & mat_bit(5)) ? (comp_bit(0) | comp_bit(2) | comp_bit(1) | comp_bit(5)) : 0u) |     // Uber
         ((mats & mat_bit(6)) ? (comp_bit(1) | comp_bit(3)) : 0u) |                                 // ThinDielectric
         ((mats & mat_bit(7)) ? (comp_bit(4) | comp_bit(1) | comp_bit(5)) : 0u) |                   // Plastic
         ((mats & mat_bit(8)) ? (comp_bit(1) | comp_bit(14)) : 0u) |                                // Dielectric
         ((mats & mat_bit(9)) ? comp_bit(8) : 0u) |                                                 // Mirror
         ((mats & mat_bit(10)) ? (comp_bit(9) | comp_bit(10)) : 0u) |                               // Metal
         ((mats & mat_bit(11)) ? (comp_bit(9) | comp_bit(11)) : 0u) |                               // BrushedMetal
         ((mats & mat_bit(12)) ? (comp_bit(12) | comp_bit(13)) : 0u) |                              // Velvet
         ((mats & mat_bit(13)) ? (comp_bit(1) | comp_bit(4) | comp_bit(15)) : 0u);                  // MetallicPaint+glitter
}
#define YRT_ALL_MATS 0x3FFEu
// Light types ride in bits 16.. of the same instantiation mask (bit 16 + LIGHT_x).
__host__ __device__ constexpr unsigned light_bit(int t) { return 1u << (16 + t); }
#define YRT_BASIC_LIGHTS (light_bit(0) | light_bit(1) | light_bit(2))  // ambient, triangle, HDRI
#define YRT_ALL_LIGHTS 0x7F0000u

struct Comp {
  int kind;  // its BRDF type bits are a function of the kind (comp_type)
  V3 R;
  float a, b, c;
};

// BRDF type of a component kind (brdfs/*.h constructors): diffuse {Lambertian,
// DielectricLayer<Lambertian>, Minnaert, Velvety}, specular reflection {DielectricReflection,
// Reflection, Conductor}, specular transmission {ConstDielectricTransmission,
// ThinDielectricTransmission, Transmission, DielectricTransmission}, glossy reflection
// {Microfacet (all three), Specular}
__device__ __forceinline__ uint32_t comp_type(int kind) {
  constexpr unsigned kDiff = (1u << C_LAMBERT) | (1u << C_DIEL_LAYER_LAMB) | (1u << C_MINNAERT) | (1u << C_VELVETY);
  constexpr unsigned kSpecR = (1u << C_DIEL_REFL) | (1u << C_REFLECTION) | (1u << C_CONDUCTOR);
  constexpr unsigned kSpecT =
      (1u << C_CONST_DIEL_TRANS) | (1u << C_THIN_DIEL_TRANS) | (1u << C_TRANSMISSION) | (1u << C_DIEL_TRANS);
  const unsigned b = 1u << kind;
  return (b & kDiff) ? BT_DIFFUSE_REFLECTION
                     : (b & kSpecR) ? BT_SPECULAR_REFLECTION
                                    : (b & kSpecT) ? BT_SPECULAR_TRANSMISSION : BT_GLOSSY_REFLECTION;
}

#define YRT_MAX_COMPS 3

struct BRDFSet {
  int n;
  Comp c[YRT_MAX_COMPS];
};

struct DG {
  V3 P, Ng, Ns, Tx, Ty;
  V3 Fx, Fy;    // frame(Ns) = (Fx, Fy, Ns), built once per vertex after Material::shade (dg_frame)
  float s, t;   // st
  float error;
  int material, light, illumMask, shadowMask;
};

// ---------------------------------------------------------------- optics
__device__ __forceinline__ float fresnel3(float cosi, float cost, float eta) {
  float Rper = (eta * cosi - cost) * rcpf_(eta * cosi + cost);
  float Rpar = (cosi - eta * cost) * rcpf_(cosi + eta * cost);
  return 0.5f * (Rpar * Rpar + Rper * Rper);
}
__device__ __forceinline__ float fresnel2(float cosi, float eta, float* outCosT) {
  float k = 1.0f - eta * eta * (1.0f - cosi * cosi);
  if (k < 0.0f) return 1.0f;
  float cost = sqrtf(k);
  if (outCosT) *outCosT = cost;
  return fresnel3(cosi, cost, eta);
}
// refract(V,N,eta,cosi,cost) (brdfs/optics.h:64-70); returns pdf
__device__ __forceinline__ float refract5(V3 V, V3 N, float eta, float cosi, float& cost, V3& out) {
  float k = 1.0f - eta * eta * (1.0f - cosi * cosi);
  if (k < 0.0f) {
    cost = 0.0f;
    out = v3s(0.0f);
    return 0.0f;
  }
  cost = sqrtf(k);
  out = eta * (cosi * N - V) - cost * N;
  return sqrf(eta);
}
__device__ __forceinline__ V3 reflect3(V3 V, V3 N, float cosi) { return 2.0f * cosi * N - V; }
__device__ __forceinline__ V3 reflect2(V3 V, V3 N) { return reflect3(V, N, dot(V, N)); }

// cosineSampleHemisphere(u,v,N) (samplers/shapesampler.h:80-95)
__device__ __forceinline__ V3 cosine_hemi(float u, float v, V3 N, float& pdf) {
  const float phi = kTwoPi * u;
  const float cosTheta = sqrtf(v), sinTheta = sqrtf(1.0f - v);
  V3 l = v3(yrt_cosf(phi) * sinTheta, yrt_sinf(phi) * sinTheta, cosTheta);
  pdf = cosTheta * kOneOverPi;
  return mul(frame(N), l);
}

// frame(Ns) of the shading point, shared by every cosine-weighted / microfacet sample of the
// vertex (BRDF sampling and the dome light): built once instead of once per sample (each
// build is two normalizations); same operations, so the same bits as frame(dg.Ns).
__device__ __forceinline__ void dg_frame(DG& dg) {
  const L3 F = frame(dg.Ns);
  dg.Fx = F.vx;
  dg.Fy = F.vy;
}
__device__ __forceinline__ L3 dg_F(const DG& dg) { return l3(dg.Fx, dg.Fy, dg.Ns); }
// cosineSampleHemisphere(u, v, dg.Ns) with the vertex's prebuilt frame
__device__ __forceinline__ V3 cosine_hemi_dg(float u, float v, const DG& dg, float& pdf) {
  const float phi = kTwoPi * u;
  const float cosTheta = sqrtf(v), sinTheta = sqrtf(1.0f - v);
  V3 l = v3(yrt_cosf(phi) * sinTheta, yrt_sinf(phi) * sinTheta, cosTheta);
  pdf = cosTheta * kOneOverPi;
  return mul(dg_F(dg), l);
}

// ---------------------------------------------------------------- textures
__device__ __forceinline__ void texel(const GpuImage& im, const uint8_t* __restrict__ pool, int x, int y,
                                      float c[4]) {
  const float one_over_255 = 1.0f / 255.0f;
  if (im.format == IMG_RGBAF32) {
    const float4 f = *(const float4*)(pool + im.offset + ((int64_t)y * im.width + x) * 16);
    c[0] = f.x; c[1] = f.y; c[2] = f.z; c[3] = f.w;
    return;
  }
  const uint8_t* p = pool + im.offset + ((int64_t)y * im.width + x) * 4;
  uchar4 b = *(const uchar4*)p;
  c[0] = b.x * one_over_255;
  c[1] = b.y * one_over_255;
  c[2] = b.z * one_over_255;
  c[3] = im.format == IMG_RGB8 ? 1.0f : b.w * one_over_255;
}

// Texture::get (textures/Bilinear.h:8-25, textures/nearestneighbor.h:25-32) -> RGBA
__device__ __forceinline__ void texel_u8(uint32_t w, bool rgb, float c[4]) {
  const float one_over_255 = 1.0f / 255.0f;
  c[0] = (w & 0xffu) * one_over_255;
  c[1] = ((w >> 8) & 0xffu) * one_over_255;
  c[2] = ((w >> 16) & 0xffu) * one_over_255;
  c[3] = rgb ? 1.0f : (w >> 24) * one_over_255;
}
__device__ __forceinline__ void tex_get_rec(const GpuTexture& tx, const uint8_t* __restrict__ pool,
                                            const uint8_t* __restrict__ quads, float px, float py, float out[4]) {
  // the texture record carries its image's descriptor: one dependent load fewer (-2 % shade)
  GpuImage im;
  im.width = tx.width;
  im.height = tx.height;
  im.format = tx.format;
  im.offset = tx.offset;
  const float s1 = px - floorf(px), t1 = py - floorf(py);
  float c[4];
  if (tx.filter == TEX_BILINEAR) {
    const float u = s1 * im.width - .5f;
    const float v = t1 * im.height - .5f;
    const int x = max(0, min((int)floorf(u), im.width - 2));
    const int y = max(0, min((int)floorf(v), im.height - 2));
    const float u_ratio = u - x;
    const float v_ratio = v - y;
    const float u_opposite = 1.f - u_ratio;
    const float v_opposite = 1.f - v_ratio;
    float c00[4], c10[4], c01[4], c11[4];
    if (im.format != IMG_RGBAF32) {
      // the 2x2 footprint of an 8-bit texel in one 16-byte record (device/scene_gpu.cpp): one load
      // on the dependent material -> texture -> texel chain instead of four, in one cache line
      // instead of two (k_shade -6.6 % on C3, profiles/r02/trace_variants_r02.txt)
      const uint4 qd = *(const uint4*)(quads + 4 * (im.offset + ((int64_t)y * im.width + x) * 4));
      const bool rgb = im.format == IMG_RGB8;
      texel_u8(qd.x, rgb, c00);
      texel_u8(qd.y, rgb, c10);
      texel_u8(qd.z, rgb, c01);
      texel_u8(qd.w, rgb, c11);
    } else {
      texel(im, pool, x, y, c00);
      texel(im, pool, x + 1, y, c10);
      texel(im, pool, x, y + 1, c01);
      texel(im, pool, x + 1, y + 1, c11);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      c[k] = (c00[k] * u_opposite + c10[k] * u_ratio) * v_opposite + (c01[k] * u_opposite + c11[k] * u_ratio) * v_ratio;
  } else {
    const int si = (int)(s1 * float(im.width)), ti = (int)(t1 * float(im.height));
    const int ix = max(0, min(si, im.width - 1));
    const int iy = max(0, min(ti, im.height - 1));
    texel(im, pool, ix, iy, c);
  }
  if (tx.invert) {
#pragma unroll
    for (int k = 0; k < 4; ++k) c[k] = 1.f - c[k];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) out[k] = c[k];
}
__device__ __forceinline__ void tex_get(const GpuTexture* __restrict__ textures, const GpuImage* __restrict__ images,
                                        const uint8_t* __restrict__ pool, const uint8_t* __restrict__ quads, int texId,
                                        float px, float py, float out[4]) {
  (void)images;
  const GpuTexture tx = textures[texId];
  tex_get_rec(tx, pool, quads, px, py, out);
}

// ---------------------------------------------------------------- BRDF components
// Component-set guards (CM = the kernel instantiation's component bitmask)
#define YRT_IF(K) if constexpr ((CM & comp_bit(K)) != 0u)
#define YRT_IF_NOT(K) if constexpr ((CM & comp_bit(K)) == 0u)

__device__ __forceinline__ V3 lambert_eval(V3 R, const DG& dg, V3 wi) {
  return R * kOneOverPi * clampf(dot(wi, dg.Ns));
}

// fresnelConductor (brdfs/optics.h:123-131), per channel in the reference's operation order
__device__ __forceinline__ V3 fresnel_conductor(float cosi, V3 eta, V3 k) {
  const V3 tmp = eta * eta + k * k;
  const V3 e2c = 2.0f * eta * cosi;
  const V3 Rpar = (tmp * cosi * cosi - e2c + v3s(1.0f)) * rcpv(tmp * cosi * cosi + e2c + v3s(1.0f));
  const V3 Rper = (tmp - e2c + v3s(cosi * cosi)) * rcpv(tmp + e2c + v3s(cosi * cosi));
  return 0.5f * (Rpar + Rper);
}
__device__ __forceinline__ V3 mat_eta(const GpuMaterial* __restrict__ mats, float id) {
  const GpuMaterial& m = mats[__float_as_int(id)];
  return v3(m.p[3], m.p[4], m.p[5]);
}
__device__ __forceinline__ V3 mat_k(const GpuMaterial* __restrict__ mats, float id) {
  const GpuMaterial& m = mats[__float_as_int(id)];
  return v3(m.p[6], m.p[7], m.p[8]);
}

// AnisotropicPowerCosineDistribution::eval (brdfs/microfacet/anisotropic_power_cosine_distribution.h:40-48)
__device__ __forceinline__ float aniso_D(float nx, float ny, const DG& dg, V3 wh) {
  const float norm2 = sqrtf((nx + 2) * (ny + 2)) * kOneOverTwoPi;
  const float cosPhiH = dot(wh, dg.Tx);
  const float sinPhiH = dot(wh, dg.Ty);
  const float cosThetaH = dot(wh, dg.Ns);
  const float R = sqrf(cosPhiH) + sqrf(sinPhiH);
  if (R == 0.0f) return norm2;
  const float n = (nx * sqrf(cosPhiH) + ny * sqrf(sinPhiH)) * rcpf_(R);
  return norm2 * yrt_powf(fabsf(cosThetaH), n);
}

// Microfacet<Fresnel, Distribution>::eval (brdfs/microfacet.h:28-41) for the dielectric /
// conductor Fresnel terms and the power-cosine / anisotropic power-cosine distributions.
// CM (the kernel's component set) compiles out the conductor / anisotropic branches no
// material of the scene can create (k_shade -5 % on C3, same-box A/B, profiles/r01).
template <unsigned CM>
__device__ __forceinline__ V3 microfacet_eval(const Comp& c, const GpuMaterial* __restrict__ mats, V3 wo, const DG& dg,
                                             V3 wi) {
  if (dot(wi, dg.Ng) <= 0) return v3s(0.0f);
  const float cosThetaO = dot(wo, dg.Ns);
  const float cosThetaI = dot(wi, dg.Ns);
  if (cosThetaI <= 0.0f || cosThetaO <= 0.0f) return v3s(0.0f);
  const V3 wh = normalize(wi + wo);
  const float cosThetaH = dot(wh, dg.Ns);
  const float cosTheta = dot(wi, wh);
  constexpr bool kCond = (CM & (comp_bit(C_MICRO_COND) | comp_bit(C_MICRO_ANISO))) != 0;
  constexpr bool kAniso = (CM & comp_bit(C_MICRO_ANISO)) != 0;
  const bool diel = !kCond || c.kind == C_MICROFACET;
  V3 F;
  if (diel) F = v3s(fresnel2(cosTheta, c.a * rcpf_(c.b), nullptr));
  else F = fresnel_conductor(cosTheta, mat_eta(mats, c.c), mat_k(mats, c.c));
  float D;
  if (kAniso && c.kind == C_MICRO_ANISO) {
    D = aniso_D(c.a, c.b, dg, wh);
  } else {
    const float n = diel ? c.c : c.a;
    const float norm2 = (n + 2) * kOneOverTwoPi;
    D = norm2 * yrt_powf(fabsf(dot(wh, dg.Ns)), n);
  }
  const float G = fminf(fminf(1.0f, 2.0f * cosThetaH * cosThetaO * rcpf_(cosTheta)),
                        2.0f * cosThetaH * cosThetaI * rcpf_(cosTheta));
  return c.R * D * G * F * rcpf_(4.0f * cosThetaO);
}

// The glitter flakes of MetallicPaint (materials/metallicpaint.h:63-70): Microfacet<
// FresnelConductor(eta 0.62, k 4.8: aluminium), PowerCosineDistribution(n, Ns)> with
// reflectivity glitterColor — microfacet.h:28-41 with the constant conductor Fresnel term.
__device__ __forceinline__ V3 glitter_ground_eval(V3 R, float n, V3 wo, const DG& dg, V3 wi) {
  if (dot(wi, dg.Ng) <= 0) return v3s(0.0f);
  const float cosThetaO = dot(wo, dg.Ns);
  const float cosThetaI = dot(wi, dg.Ns);
  if (cosThetaI <= 0.0f || cosThetaO <= 0.0f) return v3s(0.0f);
  const V3 wh = normalize(wi + wo);
  const float cosThetaH = dot(wh, dg.Ns);
  const float cosTheta = dot(wi, wh);
  const V3 F = fresnel_conductor(cosTheta, v3s(0.62f), v3s(4.8f));
  const float D = (n + 2) * kOneOverTwoPi * yrt_powf(fabsf(dot(wh, dg.Ns)), n);
  const float G = fminf(fminf(1.0f, 2.0f * cosThetaH * cosThetaO * rcpf_(cosTheta)),
                        2.0f * cosThetaH * cosThetaI * rcpf_(cosTheta));
  return R * D * G * F * rcpf_(4.0f * cosThetaO);
}
// DielectricLayer<MicrofacetGlitter>::eval (brdfs/dielectriclayer.h:27-38), T = one
__device__ __forceinline__ V3 glitter_layer_eval(const Comp& c, V3 wo, const DG& dg, V3 wi) {
  float cosThetaO = dot(wo, dg.Ns);
  float cosThetaI = dot(wi, dg.Ns);
  if (cosThetaI <= 0.0f || cosThetaO <= 0.0f) return v3s(0.0f);
  float cosThetaO1, cosThetaI1;
  V3 wo1, wi1;
  refract5(wo, dg.Ns, c.a, cosThetaO, cosThetaO1, wo1);
  refract5(wi, dg.Ns, c.a, cosThetaI, cosThetaI1, wi1);
  float Fi = 1.0f - fresnel3(cosThetaI, cosThetaI1, c.a);
  V3 Fg = glitter_ground_eval(c.R, c.c, -wo1, dg, -wi1);
  float Fo = 1.0f - fresnel3(cosThetaO, cosThetaO1, c.a);
  return Fo * v3s(1.0f) * Fg * v3s(1.0f) * Fi;
}

// Minnaert::eval (brdfs/minnaert.h:20-24), Velvety::eval (brdfs/velvety.h:20-26). Color / float
// is a * rcp(b) in the reference (common/math/color_sse.h:162), not a division.
__device__ __forceinline__ V3 minnaert_eval(const Comp& c, V3 wo, const DG& dg, V3 wi) {
  const float cosThetaI = clampf(dot(wi, dg.Ns));
  const float backScatter = yrt_powf(clampf(dot(wo, wi)), c.a);
  return c.R * backScatter * cosThetaI * rcpf_(kPi);
}
__device__ __forceinline__ V3 velvety_eval(const Comp& c, V3 wo, const DG& dg, V3 wi) {
  const float cosThetaO = clampf(dot(wo, dg.Ns));
  const float cosThetaI = clampf(dot(wi, dg.Ns));
  const float sinThetaO = sqrtf(1.0f - cosThetaO * cosThetaO);
  const float horizonScatter = yrt_powf(sinThetaO, c.a);
  return c.R * horizonScatter * cosThetaI * rcpf_(kPi);
}

// DielectricLayer<Lambertian>::eval (brdfs/dielectriclayer.h:27-38), T = one
__device__ __forceinline__ V3 layer_eval(const Comp& c, V3 wo, const DG& dg, V3 wi) {
  float cosThetaO = dot(wo, dg.Ns);
  float cosThetaI = dot(wi, dg.Ns);
  if (cosThetaI <= 0.0f || cosThetaO <= 0.0f) return v3s(0.0f);
  float cosThetaO1, cosThetaI1;
  V3 wo1, wi1;
  refract5(wo, dg.Ns, c.a, cosThetaO, cosThetaO1, wo1);
  refract5(wi, dg.Ns, c.a, cosThetaI, cosThetaI1, wi1);
  float Fi = 1.0f - fresnel3(cosThetaI, cosThetaI1, c.a);
  V3 Fg = lambert_eval(c.R, dg, -wi1);
  float Fo = 1.0f - fresnel3(cosThetaO, cosThetaO1, c.a);
  return Fo * v3s(1.0f) * Fg * v3s(1.0f) * Fi;
}

__device__ __forceinline__ V3 specular_eval(const Comp& c, V3 wo, const DG& dg, V3 wi) {
  V3 r = reflect2(wo, dg.Ns);
  if (dot(r, wi) < 0) return v3s(0.0f);
  return c.R * (c.a + 2) * (1.0f / (2.0f * kPi)) * yrt_powf(dot(r, wi), c.a) * clampf(dot(wi, dg.Ns));
}

template <unsigned CM>
__device__ __forceinline__ V3 comp_eval(const Comp c, const GpuMaterial* __restrict__ mats, V3 wo, const DG& dg,
                                        V3 wi) {
  // YRT_IF(K): the case is compiled only when the component set CM can hold kind K (a runtime
  // bit test does not let the compiler drop switch cases; these constexpr guards do)
  switch (c.kind) {
    case C_LAMBERT: YRT_IF(C_LAMBERT) return lambert_eval(c.R, dg, wi); break;
    case C_DIEL_LAYER_LAMB: YRT_IF(C_DIEL_LAYER_LAMB) return layer_eval(c, wo, dg, wi); break;
    case C_MICROFACET: YRT_IF(C_MICROFACET) return microfacet_eval<CM>(c, mats, wo, dg, wi); break;
    case C_MICRO_COND: YRT_IF(C_MICRO_COND) return microfacet_eval<CM>(c, mats, wo, dg, wi); break;
    case C_MICRO_ANISO: YRT_IF(C_MICRO_ANISO) return microfacet_eval<CM>(c, mats, wo, dg, wi); break;
    case C_SPECULAR: YRT_IF(C_SPECULAR) return specular_eval(c, wo, dg, wi); break;
    case C_REFLECTION: YRT_IF(C_REFLECTION) return c.R; break;  // Reflection::eval (reflection.h:16-18)
    case C_MINNAERT: YRT_IF(C_MINNAERT) return minnaert_eval(c, wo, dg, wi); break;
    case C_VELVETY: YRT_IF(C_VELVETY) return velvety_eval(c, wo, dg, wi); break;
    case C_DIEL_LAYER_GLITTER: YRT_IF(C_DIEL_LAYER_GLITTER) return glitter_layer_eval(c, wo, dg, wi); break;
    default: break;
  }
  return v3s(0.0f);
}

// BRDF::sample of one component; returns color, sets wi/pdf.
template <unsigned CM>
__device__ __forceinline__ V3 comp_sample(const Comp c, const GpuMaterial* __restrict__ mats, V3 wo, const DG& dg,
                                          float sx, float sy, V3& wi, float& pdf) {
  switch (c.kind) {
    case C_LAMBERT: {
      YRT_IF_NOT(C_LAMBERT) break;
      wi = cosine_hemi_dg(sx, sy, dg, pdf);
      return lambert_eval(c.R, dg, wi);
    }
    case C_DIEL_REFL: {
      YRT_IF_NOT(C_DIEL_REFL) break;
      const float cosThetaO = clampf(dot(wo, dg.Ns));
      wi = reflect3(wo, dg.Ns, cosThetaO);
      pdf = 1.0f;
      return c.b * v3s(fresnel2(cosThetaO, c.a, nullptr));
    }
    case C_CONST_DIEL_TRANS: {
      YRT_IF_NOT(C_CONST_DIEL_TRANS) break;
      wi = -wo;
      pdf = 1.0f;
      const float cosTheta = clampf(dot(wo, dg.Ns));
      return cosTheta <= 0.0f ? v3s(0.0f) : c.R;
    }
    case C_THIN_DIEL_TRANS: {
      YRT_IF_NOT(C_THIN_DIEL_TRANS) break;
      wi = -wo;
      pdf = 1.0f;
      const float cosTheta = clampf(dot(wo, dg.Ns));
      if (cosTheta <= 0.0f) return v3s(0.0f);
      const float alpha = c.b * rcpf_(cosTheta);
      float cosThetaT;
      V3 la = c.R * alpha;
      return v3(yrt_expf(la.x), yrt_expf(la.y), yrt_expf(la.z)) * (1.f - fresnel2(cosTheta, c.a, &cosThetaT));
    }
    case C_DIEL_LAYER_LAMB: {
      YRT_IF_NOT(C_DIEL_LAYER_LAMB) break;
      pdf = 0.0f;
      float cosThetaO = dot(wo, dg.Ns);
      if (cosThetaO <= 0.0f) return v3s(0.0f);
      float cosThetaO1;
      V3 wo1;
      refract5(wo, dg.Ns, c.a, cosThetaO, cosThetaO1, wo1);
      float pdf1;
      V3 wi1 = cosine_hemi_dg(sx, sy, dg, pdf1);
      V3 Fg = lambert_eval(c.R, dg, wi1);
      float cosThetaI1 = dot(wi1, dg.Ns);
      if (cosThetaI1 <= 0.0f) return v3s(0.0f);
      float cosThetaI;
      V3 wi0;
      float pdf0 = refract5(-wi1, -dg.Ns, c.b, cosThetaI1, cosThetaI, wi0);
      if (pdf0 == 0.0f) return v3s(0.0f);
      wi = wi0;
      pdf = pdf1;
      float Fi = 1.0f - fresnel3(cosThetaI, cosThetaI1, c.a);
      float Fo = 1.0f - fresnel3(cosThetaO, cosThetaO1, c.a);
      return Fo * v3s(1.0f) * Fg * v3s(1.0f) * Fi;
    }
    case C_MICROFACET: {
      YRT_IF_NOT(C_MICROFACET) break;
      pdf = 0.0f;
      if (dot(wo, dg.Ns) <= 0.0f) return v3s(0.0f);
      const float n = c.c;
      const float norm1 = (n + 1) * kOneOverTwoPi;
      const float phi = kTwoPi * sx;
      const float cosPhi = yrt_cosf(phi);
      const float sinPhi = yrt_sinf(phi);
      const float cosTheta = yrt_powf(sy, rcpf_(n + 1));
      const float sinTheta = cos2sin(cosTheta);
      V3 wh = mul(dg_F(dg), v3(cosPhi * sinTheta, sinPhi * sinTheta, cosTheta));
      float whpdf = norm1 * yrt_powf(cosTheta, n);
      wi = reflect2(wo, wh);
      pdf = whpdf * rcpf_(4.0f * fabsf(dot(wo, wh)));
      if (dot(wi, dg.Ns) <= 0.0f) return v3s(0.0f);
      return microfacet_eval<CM>(c, mats, wo, dg, wi);
    }
    case C_MICRO_COND: {
      YRT_IF_NOT(C_MICRO_COND) break;
      // Microfacet::sample (microfacet.h:43-50) with PowerCosineDistribution::sample
      pdf = 0.0f;
      if (dot(wo, dg.Ns) <= 0.0f) return v3s(0.0f);
      const float n = c.a;
      const float norm1 = (n + 1) * kOneOverTwoPi;
      const float phi = kTwoPi * sx;
      const float cosPhi = yrt_cosf(phi);
      const float sinPhi = yrt_sinf(phi);
      const float cosTheta = yrt_powf(sy, rcpf_(n + 1));
      const float sinTheta = cos2sin(cosTheta);
      V3 wh = mul(dg_F(dg), v3(cosPhi * sinTheta, sinPhi * sinTheta, cosTheta));
      float whpdf = norm1 * yrt_powf(cosTheta, n);
      wi = reflect2(wo, wh);
      pdf = whpdf * rcpf_(4.0f * fabsf(dot(wo, wh)));
      if (dot(wi, dg.Ns) <= 0.0f) return v3s(0.0f);
      return microfacet_eval<CM>(c, mats, wo, dg, wi);
    }
    case C_MICRO_ANISO: {
      YRT_IF_NOT(C_MICRO_ANISO) break;
      // AnisotropicPowerCosineDistribution::sample (:57-73)
      pdf = 0.0f;
      if (dot(wo, dg.Ns) <= 0.0f) return v3s(0.0f);
      const float nx = c.a, ny = c.b;
      const float norm1 = sqrtf((nx + 1) * (ny + 1)) * kOneOverTwoPi;
      const float phi = kTwoPi * sx;
      const float sinPhi0 = sqrtf(nx + 1) * yrt_sinf(phi);
      const float cosPhi0 = sqrtf(ny + 1) * yrt_cosf(phi);
      const float nrm = rsqrtf_(sqrf(sinPhi0) + sqrf(cosPhi0));
      const float sinPhi = sinPhi0 * nrm;
      const float cosPhi = cosPhi0 * nrm;
      const float n = nx * sqrf(cosPhi) + ny * sqrf(sinPhi);
      const float cosTheta = yrt_powf(sy, rcpf_(n + 1));
      const float sinTheta = cos2sin(cosTheta);
      const float whpdf = norm1 * yrt_powf(cosTheta, n);
      const V3 h = v3(cosPhi * sinTheta, sinPhi * sinTheta, cosTheta);
      const V3 wh = h.x * dg.Tx + h.y * dg.Ty + h.z * dg.Ns;
      wi = reflect2(wo, wh);
      pdf = whpdf * rcpf_(4.0f * fabsf(dot(wo, wh)));
      if (dot(wi, dg.Ns) <= 0.0f) return v3s(0.0f);
      return microfacet_eval<CM>(c, mats, wo, dg, wi);
    }
    case C_REFLECTION: {  // reflection.h:19-22
      YRT_IF_NOT(C_REFLECTION) break;
      wi = reflect2(wo, dg.Ns);
      pdf = 1.0f;
      return c.R;
    }
    case C_CONDUCTOR: {  // conductor.h:21-24
      YRT_IF_NOT(C_CONDUCTOR) break;
      wi = reflect2(wo, dg.Ns);
      pdf = 1.0f;
      return c.R * fresnel_conductor(dot(wo, dg.Ns), mat_eta(mats, c.c), mat_k(mats, c.c));
    }
    case C_MINNAERT: {
      YRT_IF_NOT(C_MINNAERT) break;
      wi = cosine_hemi_dg(sx, sy, dg, pdf);
      return minnaert_eval(c, wo, dg, wi);
    }
    case C_VELVETY: {
      YRT_IF_NOT(C_VELVETY) break;
      wi = cosine_hemi_dg(sx, sy, dg, pdf);
      return velvety_eval(c, wo, dg, wi);
    }
    case C_DIEL_TRANS: {  // dielectric.h:82-89 (the sample's eta is dropped)
      YRT_IF_NOT(C_DIEL_TRANS) break;
      const float cosThetaO = clampf(dot(wo, dg.Ns));
      float cosThetaI;
      pdf = refract5(wo, dg.Ns, c.a, cosThetaO, cosThetaI, wi);
      return v3s(1.0f - fresnel3(cosThetaO, cosThetaI, c.a));
    }
    case C_TRANSMISSION: {
      YRT_IF_NOT(C_TRANSMISSION) break;
      wi = -wo;
      pdf = 1.0f;
      return c.R;
    }
    case C_DIEL_LAYER_GLITTER: {
      YRT_IF_NOT(C_DIEL_LAYER_GLITTER) break;
      // DielectricLayer::sample (dielectriclayer.h:40-62) over Microfacet::sample
      // (microfacet.h:43-50) with PowerCosineDistribution::sample (power_cosine_distribution.h:27-35)
      pdf = 0.0f;
      float cosThetaO = dot(wo, dg.Ns);
      if (cosThetaO <= 0.0f) return v3s(0.0f);
      float cosThetaO1;
      V3 wo1;
      refract5(wo, dg.Ns, c.a, cosThetaO, cosThetaO1, wo1);
      const V3 gwo = -wo1;
      V3 wi1 = v3s(0.0f);
      float pdf1 = 0.0f;
      V3 Fg = v3s(0.0f);
      if (dot(gwo, dg.Ns) > 0.0f) {
        const float n = c.c;
        const float norm1 = (n + 1) * kOneOverTwoPi;
        const float phi = kTwoPi * sx;
        const float cosPhi = yrt_cosf(phi);
        const float sinPhi = yrt_sinf(phi);
        const float cosTheta = yrt_powf(sy, rcpf_(n + 1));
        const float sinTheta = cos2sin(cosTheta);
        const V3 wh = mul(dg_F(dg), v3(cosPhi * sinTheta, sinPhi * sinTheta, cosTheta));
        const float whpdf = norm1 * yrt_powf(cosTheta, n);
        wi1 = reflect2(gwo, wh);
        pdf1 = whpdf * rcpf_(4.0f * fabsf(dot(gwo, wh)));
        if (dot(wi1, dg.Ns) > 0.0f) Fg = glitter_ground_eval(c.R, n, gwo, dg, wi1);
      }
      float cosThetaI1 = dot(wi1, dg.Ns);
      if (cosThetaI1 <= 0.0f) return v3s(0.0f);
      float cosThetaI;
      V3 wi0;
      float pdf0 = refract5(-wi1, -dg.Ns, c.b, cosThetaI1, cosThetaI, wi0);
      if (pdf0 == 0.0f) return v3s(0.0f);
      wi = wi0;
      pdf = pdf1;
      float Fi = 1.0f - fresnel3(cosThetaI, cosThetaI1, c.a);
      float Fo = 1.0f - fresnel3(cosThetaO, cosThetaO1, c.a);
      return Fo * v3s(1.0f) * Fg * v3s(1.0f) * Fi;
    }
    case C_SPECULAR: {
      YRT_IF_NOT(C_SPECULAR) break;
      // powerCosineSampleHemisphere(s.x, s.y, reflect(wo, Ns), exp) (shapesampler.h:104-121)
      const float e = c.a;
      const float phi = kTwoPi * sx;
      const float cosTheta = yrt_powf(sy, rcpf_(e + 1));
      const float sinTheta = cos2sin(cosTheta);
      V3 l = v3(yrt_cosf(phi) * sinTheta, yrt_sinf(phi) * sinTheta, cosTheta);
      pdf = (e + 1.0f) * yrt_powf(cosTheta, e) * kOneOverTwoPi;
      wi = mul(frame(reflect2(wo, dg.Ns)), l);
      return specular_eval(c, wo, dg, wi);
    }
  }
  pdf = 0.0f;
  wi = v3s(0.0f);
  return v3s(0.0f);
}

// CompositedBRDF::eval restricted to `type` (compositedbrdf.h:59-65)
template <unsigned CM>
__device__ __forceinline__ V3 set_eval(const BRDFSet& bs, const GpuMaterial* __restrict__ mats, V3 wo, const DG& dg,
                                       V3 wi, uint32_t type) {
  V3 c = v3s(0.0f);
#pragma unroll
  for (int i = 0; i < YRT_MAX_COMPS; ++i)
    if (i < bs.n && (comp_type(bs.c[i].kind) & type)) {
      const Comp ci = bs.c[i];
      c = c + comp_eval<CM>(ci, mats, wo, dg, wi);
    }
  return c;
}

// CompositedBRDF::sample (compositedbrdf.h:104-166). Same arithmetic as the reference
// (f_i = sum(c_i)/pdf_i over the components that sampled something, normalized by their
// running sum, CDF with the last entry forced to 1). The per-component candidates (color,
// direction, pdf) are parked in LDS instead of registers: st points at this lane's slot 0 of a
// [21][64] float array (slot k at st[k * 64], conflict-free) and only the chosen candidate is
// read back (117 instead of 124 VGPRs: k_shade -3.8 %, C3 +0.9 %, profiles/r02/shade_prune_r02.txt).
template <unsigned CM>
__device__ __forceinline__ V3 set_sample(const BRDFSet& bs, const GpuMaterial* __restrict__ mats, V3 wo,
                                            const DG& dg, float sx, float sy, float ss, V3& wi_o, float& pdf_o,
                                            uint32_t& type_o, float* __restrict__ st) {
  float f[YRT_MAX_COMPS];
  bool ok[YRT_MAX_COMPS];
  float sum = 0.0f;
  int num = 0;
#pragma unroll
  for (int i = 0; i < YRT_MAX_COMPS; ++i) {
    ok[i] = false;
    f[i] = 0.0f;
    if (i < bs.n) {
      V3 wi;
      float pdf = 0.0f;
      const Comp ci = bs.c[i];
      const V3 c = comp_sample<CM>(ci, mats, wo, dg, sx, sy, wi, pdf);
      if (!((c.x == 0.0f && c.y == 0.0f && c.z == 0.0f) || pdf <= 0.0f)) {
        ok[i] = true;
        f[i] = (c.x + c.y + c.z) * rcpf_(pdf);
        sum += f[i];
        float* q = st + i * 7 * 64;
        q[0] = c.x; q[64] = c.y; q[128] = c.z;
        q[192] = wi.x; q[256] = wi.y; q[320] = wi.z;
        q[384] = pdf;
        num++;
      }
    }
  }
  if (num == 0) {
    wi_o = v3s(0.0f);
    pdf_o = 0.0f;
    type_o = 0;
    return v3s(0.0f);
  }
  float d = 0.0f;
  int k = 0;
  int chosen = -1;
#pragma unroll
  for (int i = 0; i < YRT_MAX_COMPS; ++i) {
    if (ok[i]) {
      const float fi = f[i] / sum;
      f[i] = fi;
      d = (k == 0) ? fi : d + fi;
      const float dk = (k == num - 1) ? 1.0f : d;
      if (chosen < 0 && (k == num - 1 || !(ss > dk))) chosen = i;
      k++;
    }
  }
  // chosen is a valid component (the last valid one is taken when no earlier one is)
  float fc = f[0];
  int kind = bs.c[0].kind;
#pragma unroll
  for (int i = 1; i < YRT_MAX_COMPS; ++i)
    if (chosen == i) {
      fc = f[i];
      kind = bs.c[i].kind;
    }
  const float* q = st + chosen * 7 * 64;
  wi_o = v3(q[192], q[256], q[320]);
  pdf_o = q[384] * fc;
  type_o = comp_type(kind);
  return v3(q[0], q[64], q[128]);
}

}  // namespace yrt
