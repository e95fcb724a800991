// objects.cpp — rtCommit for every device object type: builds the instance from the Parms
// bag with the reference constructors' defaults.
#include "objects.h"

#include <string.h>
#include <strings.h>

#include <stdexcept>

#include "distribution.h"

namespace yrt {

const char* kind_name(Kind k) {
  switch (k) {
    case Kind::CAMERA: return "camera";
    case Kind::DATA: return "data";
    case Kind::IMAGE: return "image";
    case Kind::TEXTURE: return "texture";
    case Kind::MATERIAL: return "material";
    case Kind::SHAPE: return "shape";
    case Kind::LIGHT: return "light";
    case Kind::PRIMITIVE: return "primitive";
    case Kind::SCENE: return "scene";
    case Kind::TONEMAPPER: return "tonemapper";
    case Kind::RENDERER: return "renderer";
    case Kind::FRAMEBUFFER: return "framebuffer";
  }
  return "?";
}

static bool ieq(const std::string& a, const char* b) { return strcasecmp(a.c_str(), b) == 0; }

void ImageObj::get(int x, int y, float c[4]) const {
  if (format == IMG_RGBAF32) {
    const float* p = (const float*)data.data() + ((size_t)y * width + x) * 4;
    c[0] = p[0]; c[1] = p[1]; c[2] = p[2]; c[3] = p[3];
  } else {
    const float one_over_255 = 1.0f / 255.0f;
    const uint8_t* p = data.data() + ((size_t)y * width + x) * 4;
    c[0] = p[0] * one_over_255; c[1] = p[1] * one_over_255; c[2] = p[2] * one_over_255;
    c[3] = format == IMG_RGB8 ? 1.0f : p[3] * one_over_255;
  }
}

// ---------------------------------------------------------------- textures
// SingleRayDevice::rtNewTexture (api/singleray_device.cpp:254-259), textures/Bilinear.h:2-6
void TextureObj::commit() {
  auto t = std::make_shared<TextureInst>();
  t->filter = ieq(type, "bilinear") ? TEX_BILINEAR : TEX_NEAREST;
  t->image = std::dynamic_pointer_cast<ImageObj>(parms.getObject("image"));
  t->invert = parms.getBool("invert", false);
  if (!t->image) throw std::runtime_error("texture without image");
  inst = t;
}

static std::shared_ptr<const TextureInst> tex_param(const Parms& p, const char* name) {
  auto o = std::dynamic_pointer_cast<TextureObj>(p.getObject(name));
  if (!o) return nullptr;
  if (!o->inst) o->commit();
  return o->inst;
}

// ---------------------------------------------------------------- materials
void MaterialObj::commit() {
  auto m = std::make_shared<MaterialInst>();
  memset(&m->gm, 0, sizeof(m->gm));
  for (int i = 0; i < 5; ++i) m->gm.tex[i] = -1;
  float* p = m->gm.p;
  if (ieq(type, "Matte")) {
    // materials/matte.h:16-18
    m->gm.type = MAT_MATTE;
    V3 r = parms.getV3("reflectance", v3s(1.f));
    p[0] = r.x; p[1] = r.y; p[2] = r.z;
  } else if (ieq(type, "MatteTextured")) {
    // materials/matte_textured.h:17-22
    m->gm.type = MAT_MATTE_TEXTURED;
    m->tex[0] = tex_param(parms, "Kd");
    parms.getV2("s0", p + 0, 0.f, 0.f);
    parms.getV2("ds", p + 2, 1.f, 1.f);
  } else if (ieq(type, "MetallicPaint")) {
    // materials/metallicpaint.h:23-34
    m->gm.type = MAT_METALLIC_PAINT;
    V3 shade = parms.getV3("shadeColor", v3s(1.f));
    V3 glitter = parms.getV3("glitterColor", v3s(0.f));
    float glitterSpread = parms.getFloat("glitterSpread", 1.0f);
    float eta = parms.getFloat("eta", 1.4f);
    p[0] = shade.x; p[1] = shade.y; p[2] = shade.z;
    p[3] = eta;
    p[4] = 1.0f * rcpf_(eta);   // DielectricReflection(1, eta): eta_ = etai*rcp(etat)
    p[5] = 1.0f * rcpf_(eta);   // DielectricLayer etait
    p[6] = eta * rcpf_(1.0f);   // DielectricLayer etati
    // glitter flakes (metallicpaint.h:63-70): a third component, DielectricLayer<Microfacet<
    // FresnelConductor(aluminium), PowerCosine(rcp(glitterSpread), Ns)>>(one, 1, eta, glitterColor)
    if (glitterSpread != 0 && glitter != v3s(0.f)) {
      m->gm.type = MAT_METALLIC_GLITTER;
      p[7] = glitter.x; p[8] = glitter.y; p[9] = glitter.z;
      p[10] = rcpf_(glitterSpread);
    }
  } else if (ieq(type, "Obj")) {
    // materials/obj.h:17-33
    m->gm.type = MAT_OBJ;
    m->tex[0] = tex_param(parms, "map_d");
    p[0] = parms.getFloat("d", 1.0f);
    m->tex[1] = tex_param(parms, "map_Kd");
    V3 Kd = parms.getV3("Kd", v3s(1.f));
    m->tex[2] = tex_param(parms, "map_Ks");
    V3 Ks = parms.getV3("Ks", v3s(0.f));
    m->tex[3] = tex_param(parms, "map_Ns");
    p[7] = parms.getFloat("Ns", 10.0f);
    m->tex[4] = tex_param(parms, "map_Bump");
    p[1] = Kd.x; p[2] = Kd.y; p[3] = Kd.z;
    p[4] = Ks.x; p[5] = Ks.y; p[6] = Ks.z;
  } else if (ieq(type, "Uber")) {
    // materials/Uber.h:5-15
    m->gm.type = MAT_UBER;
    m->tex[0] = tex_param(parms, "Kd");
    V3 diffuse = parms.getV3("diffuse", v3s(0.f));
    parms.getV2("s0", p + 3, 0.f, 0.f);
    parms.getV2("ds", p + 5, 1.f, 1.f);
    float eta = parms.getFloat("eta", 1.4f);
    float roughness = parms.getFloat("roughness", .9f);
    float reflectivity = parms.getFloat("reflectivity", .0f);
    p[0] = diffuse.x; p[1] = diffuse.y; p[2] = diffuse.z;
    p[7] = eta;
    p[8] = roughness;
    p[9] = reflectivity;
    p[10] = rcpf_(roughness);
    p[11] = 1.f * rcpf_(eta);
  } else if (ieq(type, "ThinDielectric") || ieq(type, "ThinGlass")) {
    // materials/thindielectric.h:18-26
    m->gm.type = MAT_THIN_DIELECTRIC;
    m->tex[0] = tex_param(parms, "Kd");
    parms.getV2("s0", p + 3, 0.f, 0.f);
    parms.getV2("ds", p + 5, 1.f, 1.f);
    V3 tr = parms.getV3("transmission", v3s(1.f));
    float eta = parms.getFloat("eta", 1.4f);
    p[0] = tr.x; p[1] = tr.y; p[2] = tr.z;
    p[7] = eta;
    p[8] = parms.getFloat("thickness", .1f);
    p[9] = parms.getFloat("transparency", 1.f);
    p[10] = 1.0f * rcpf_(eta);
  } else if (ieq(type, "Plastic")) {
    // materials/plastic.h:21-26
    m->gm.type = MAT_PLASTIC;
    V3 pc = parms.getV3("pigmentColor", v3s(1.f));
    float eta = parms.getFloat("eta", 1.4f);
    float roughness = parms.getFloat("roughness", 0.01f);
    p[0] = pc.x; p[1] = pc.y; p[2] = pc.z;
    p[3] = eta;
    p[4] = roughness;
    p[5] = rcpf_(roughness);
    p[6] = 1.0f * rcpf_(eta);   // DielectricLayer(one, 1, eta): etait
    p[7] = eta * rcpf_(1.0f);   // etati
    p[8] = 1.0f * rcpf_(eta);   // DielectricReflection(1, eta): eta_
  } else if (ieq(type, "Dielectric") || ieq(type, "Glass")) {
    // materials/dielectric.h:13-27: media interface; components picked per current medium
    m->gm.type = MAT_DIELECTRIC;
    const float etaOut = parms.getFloat("etaOutside", 1.0f), etaIn = parms.getFloat("etaInside", 1.4f);
    const V3 tOut = parms.getV3("transmissionOutside", v3s(1.f)), tIn = parms.getV3("transmission", v3s(1.f));
    p[0] = tOut.x; p[1] = tOut.y; p[2] = tOut.z; p[3] = etaOut;
    p[4] = tIn.x; p[5] = tIn.y; p[6] = tIn.z; p[7] = etaIn;
    p[8] = etaOut * rcpf_(etaIn);  // *_oi: DielectricReflection/Transmission(etaOutside, etaInside)
    p[9] = etaIn * rcpf_(etaOut);  // *_io
  } else if (ieq(type, "Mirror")) {
    // materials/mirror.h:15-17
    m->gm.type = MAT_MIRROR;
    V3 r = parms.getV3("reflectance", v3s(1.f));
    p[0] = r.x; p[1] = r.y; p[2] = r.z;
  } else if (ieq(type, "Metal")) {
    // materials/metal.h:18-24
    m->gm.type = MAT_METAL;
    V3 r = parms.getV3("reflectance", v3s(1.f)), eta = parms.getV3("eta", v3s(1.4f)), k = parms.getV3("k", v3s(0.f));
    float roughness = parms.getFloat("roughness", 0.01f);
    p[0] = r.x; p[1] = r.y; p[2] = r.z;
    p[3] = eta.x; p[4] = eta.y; p[5] = eta.z;
    p[6] = k.x; p[7] = k.y; p[8] = k.z;
    p[9] = roughness;
    p[10] = rcpf_(roughness);
  } else if (ieq(type, "BrushedMetal")) {
    // materials/brushedmetal.h:19-27
    m->gm.type = MAT_BRUSHED_METAL;
    V3 r = parms.getV3("reflectance", v3s(1.f)), eta = parms.getV3("eta", v3s(1.4f)), k = parms.getV3("k", v3s(0.f));
    float rx = parms.getFloat("roughnessX", 0.01f), ry = parms.getFloat("roughnessY", 0.01f);
    p[0] = r.x; p[1] = r.y; p[2] = r.z;
    p[3] = eta.x; p[4] = eta.y; p[5] = eta.z;
    p[6] = k.x; p[7] = k.y; p[8] = k.z;
    p[9] = rx; p[10] = ry;
    p[11] = rcpf_(rx); p[12] = rcpf_(ry);
  } else if (ieq(type, "Velvet")) {
    // materials/velvet.h:16-21
    m->gm.type = MAT_VELVET;
    V3 r = parms.getV3("reflectance", v3s(1.f)), h = parms.getV3("horizonScatteringColor", v3s(1.f));
    p[0] = r.x; p[1] = r.y; p[2] = r.z;
    p[3] = parms.getFloat("backScattering", 0.f);
    p[4] = h.x; p[5] = h.y; p[6] = h.z;
    p[7] = parms.getFloat("horizonScatteringFallOff", 0.f);
  } else {
    throw std::runtime_error("unknown material type: " + type);
  }
  inst = m;
}

// ---------------------------------------------------------------- shapes
static void read_array3(const Variant* v, std::vector<V3>& out) {
  auto d = std::dynamic_pointer_cast<DataObj>(v->obj);
  if (!d) throw std::runtime_error("array without data");
  out.resize(v->size);
  for (size_t i = 0; i < v->size; ++i) {
    const float* f = (const float*)(d->bytes.data() + v->ofs + i * v->stride);
    out[i] = v3(f[0], f[1], f[2]);
  }
}

std::shared_ptr<const MeshInst> MeshInst::transform(const A3& xfm) const {
  if (kind == GEOM_TRIANGLE) {
    // Triangle::transform always builds a new triangle (shapes/triangle.h:32-34)
    auto t = std::make_shared<MeshInst>(*this);
    for (auto& p : t->pos) p = xfmPoint(xfm, p);
    t->Ng = normalize(cross(t->pos[2] - t->pos[0], t->pos[1] - t->pos[0]));
    return t;
  }
  // TriangleMeshFull/WithNormals::transform: identity short-circuit, xfmPoint/xfmNormal
  if (a3_is_identity(xfm)) return std::make_shared<MeshInst>(*this);
  auto t = std::make_shared<MeshInst>(*this);
  for (auto& p : t->pos) p = xfmPoint(xfm, p);
  for (auto& n : t->nor) n = xfmNormal(xfm, n);
  // motions and tangents are vectors (trianglemesh_full.cpp:79-85)
  for (auto& m : t->mot) m = xfmVector(xfm, m);
  for (auto& v : t->tanX) v = xfmVector(xfm, v);
  for (auto& v : t->tanY) v = xfmVector(xfm, v);
  return t;
}

void ShapeObj::commit() {
  auto m = std::make_shared<MeshInst>();
  if (ieq(type, "trianglemesh")) {
    // TriangleMesh::create (shapes/trianglemesh.h:14-26)
    const Variant* pos = parms.find("positions");
    const Variant* mot = parms.find("motions");
    const Variant* nor = parms.find("normals");
    const Variant* tx = parms.find("tangent_x");
    const Variant* ty = parms.find("tangent_y");
    const Variant* tc = parms.find("texcoords");
    const Variant* tc0 = parms.find("texcoords0");
    const Variant* idx = parms.find("indices");
    // TriangleMesh::create (shapes/trianglemesh.h:29-41): WithNormals only without motions,
    // tangents and texcoords
    const bool withNormals = pos && !mot && nor && !tx && !ty && !tc && !tc0;
    m->kind = withNormals ? GEOM_MESH_NORMALS : GEOM_MESH_FULL;
    if (pos) read_array3(pos, m->pos);
    if (nor) read_array3(nor, m->nor);
    if (mot) read_array3(mot, m->mot);
    if (tx) read_array3(tx, m->tanX);
    if (ty) read_array3(ty, m->tanY);
    const Variant* t = tc0 ? tc0 : tc;
    if (t) {
      auto d = std::dynamic_pointer_cast<DataObj>(t->obj);
      m->uv.resize(t->size * 2);
      for (size_t i = 0; i < t->size; ++i) {
        const float* f = (const float*)(d->bytes.data() + t->ofs + i * t->stride);
        m->uv[2 * i] = f[0];
        m->uv[2 * i + 1] = f[1];
      }
    }
    if (idx) {
      auto d = std::dynamic_pointer_cast<DataObj>(idx->obj);
      m->tri.resize(idx->size * 3);
      for (size_t i = 0; i < idx->size; ++i) {
        const int* f = (const int*)(d->bytes.data() + idx->ofs + i * idx->stride);
        m->tri[3 * i] = f[0];
        m->tri[3 * i + 1] = f[1];
        m->tri[3 * i + 2] = f[2];
      }
    }
    if (withNormals && m->nor.size() != m->pos.size()) m->pos.resize(m->nor.size());
    m->cull = parms.getBool("cullBackFaces", false);
    if (m->kind == GEOM_MESH_FULL) {
      if (!m->nor.empty() && m->nor.size() < m->pos.size()) throw std::runtime_error("normal count < vertex count");
      if (!m->uv.empty() && m->uv.size() / 2 < m->pos.size()) throw std::runtime_error("texcoord count < vertex count");
      if (!m->mot.empty() && m->mot.size() < m->pos.size()) throw std::runtime_error("motion count < vertex count");
      if (!m->tanX.empty() && m->tanX.size() < m->pos.size()) throw std::runtime_error("tangent_x count < vertex count");
      if (!m->tanY.empty() && m->tanY.size() < m->pos.size()) throw std::runtime_error("tangent_y count < vertex count");
      m->mot.resize(m->mot.empty() ? 0 : m->pos.size());
      m->tanX.resize(m->tanX.empty() ? 0 : m->pos.size());
      m->tanY.resize(m->tanY.empty() ? 0 : m->pos.size());
    }
    for (int v : m->tri)
      if (v < 0 || (size_t)v >= m->pos.size()) throw std::runtime_error("triangle index out of range");
  } else if (ieq(type, "sphere")) {
    // shapes/sphere.h:19-66
    m->kind = GEOM_MESH_FULL;
    const V3 P = parms.getV3("P");
    const V3 dPdt = parms.getV3("dPdt");
    const float r = parms.getFloat("r");
    const size_t numTheta = (size_t)parms.getInt("numTheta");
    const size_t numPhi = (size_t)parms.getInt("numPhi");

    auto eval = [](float theta, float phi) {
      return v3(sinf(theta) * cosf(phi), cosf(theta), sinf(theta) * sinf(phi));
    };
    for (size_t theta = 0; theta <= numTheta; theta++) {
      const float rcpNumTheta = rcpf_(float(numTheta));
      for (size_t phi = 0; phi < numPhi; phi++) {
        const float rcpNumPhi = rcpf_(float(numPhi));
        V3 p = eval(float(theta) * kPi * rcpNumTheta, float(phi) * 2.0f * kPi * rcpNumPhi);
        V3 dpdu = eval((float(theta) + 0.001f) * kPi * rcpNumTheta, float(phi) * 2.0f * kPi * rcpNumPhi) - p;
        V3 dpdv = eval(float(theta) * kPi * rcpNumTheta, (float(phi) + 0.001f) * 2.0f * kPi * rcpNumPhi) - p;
        p = r * p + P;
        m->pos.push_back(p);
        if (dPdt != v3s(0.f)) m->mot.push_back(dPdt);  // sphere.h:67
        m->nor.push_back(normalize(cross(dpdv, dpdu)));
        m->uv.push_back(float(phi) * rcpNumPhi);
        m->uv.push_back(float(theta) * rcpNumTheta);
      }
      if (theta == 0) continue;
      for (size_t phi = 1; phi <= numPhi; phi++) {
        const int p00 = (int)((theta - 1) * numPhi + phi - 1);
        const int p01 = (int)((theta - 1) * numPhi + phi % numPhi);
        const int p10 = (int)(theta * numPhi + phi - 1);
        const int p11 = (int)(theta * numPhi + phi % numPhi);
        if (theta > 1) { m->tri.push_back(p10); m->tri.push_back(p00); m->tri.push_back(p01); }
        if (theta < numTheta) { m->tri.push_back(p11); m->tri.push_back(p10); m->tri.push_back(p01); }
      }
    }
  } else if (ieq(type, "disk")) {
    // shapes/disk.h:33-65: a fan of numTriangles triangles around an apex at P + (0,0,h), with
    // alternating winding. The reference pushes numTriangles normals and texcoords for
    // numTriangles + 1 positions, so the apex's shading normal is an out-of-bounds read of its
    // vector (undefined); here the apex gets the normal (0,0,1) and texcoord (0,0) every other
    // vertex has (the same substitution in oracle/yrt_oracle.c).
    m->kind = GEOM_MESH_FULL;
    const V3 P = parms.getV3("P");
    const float h = parms.getFloat("h");
    const float r = parms.getFloat("r");
    const int n = parms.getInt("numTriangles");
    if (n < 1) throw std::runtime_error("disk: numTriangles must be >= 1");
    const float rcpNumTriangles = rcpf_(float(n));
    for (int phi = 0; phi < n; phi++) {
      const V3 d = v3(sinf(float(phi) * 2.0f * kPi * rcpNumTriangles), cosf(float(phi) * 2.0f * kPi * rcpNumTriangles), 0.0f);
      m->pos.push_back(P + r * d);
      m->nor.push_back(v3(0.0f, 0.0f, 1.0f));
      m->uv.push_back(0.0f);
      m->uv.push_back(0.0f);
    }
    m->pos.push_back(P + v3(0.0f, 0.0f, h));
    m->nor.push_back(v3(0.0f, 0.0f, 1.0f));
    m->uv.push_back(0.0f);
    m->uv.push_back(0.0f);
    for (int phi = 0; phi < n; phi++) {
      const int p0 = n, p1 = phi % n, p2 = (phi + 1) % n;
      const int w[3][3] = {{p0, p2, p1}, {p1, p0, p2}, {p2, p1, p0}};
      for (int k = 0; k < 3; ++k) m->tri.push_back(w[phi % 3][k]);
    }
  } else if (ieq(type, "triangle")) {
    // shapes/triangle.h:19-24 (Ng is computed by transform())
    m->kind = GEOM_TRIANGLE;
    m->pos = {parms.getV3("v0"), parms.getV3("v1"), parms.getV3("v2")};
    m->tri = {0, 1, 2};
  } else {
    throw std::runtime_error("shape type '" + type + "' is outside the MI355X device's scope");
  }
  inst = m;
}

// ---------------------------------------------------------------- lights
static std::shared_ptr<MeshInst> triangle_shape(V3 a, V3 b, V3 c) {
  auto m = std::make_shared<MeshInst>();
  m->kind = GEOM_TRIANGLE;
  m->pos = {a, b, c};
  m->tri = {0, 1, 2};
  return m;
}

std::shared_ptr<const LightInst> LightInst::transform(const A3& xfm, int illum, int shadow) const {
  auto l = std::make_shared<LightInst>(*this);
  l->illumMask = illum;
  l->shadowMask = shadow;
  if (type == LIGHT_TRIANGLE) {
    // TriangleLight::transform (lights/trianglelight.h:43-49) + ctor :16-26
    l->v0 = xfmPoint(xfm, v0);
    l->v1 = xfmPoint(xfm, v1);
    l->v2 = xfmPoint(xfm, v2);
    l->e1 = l->v0 - l->v1;
    l->e2 = l->v2 - l->v0;
    l->Ng = cross(l->e1, l->e2);
    // l->shape stays the untransformed triangle: the scene applies shape->transform(xfm)
    // itself (api/scene_flat.h:52-56)
  } else if (type == LIGHT_HDRI) {
    // HDRILight::transform: xfm*local2world, world2local = rcp(local2world)
    l->l2w = mul(xfm, l2w);
    l->w2l = a3_inverse(l->l2w);
  } else if (type == LIGHT_POINT) {
    l->v0 = xfmPoint(xfm, v0);  // pointlight.h:30-34
  } else if (type == LIGHT_SPOT) {
    l->v0 = xfmPoint(xfm, v0);  // spotlight.h:33-39 (direction not renormalized)
    l->e1 = xfmVector(xfm, e1);
  } else if (type == LIGHT_DIRECTIONAL || type == LIGHT_DISTANT) {
    l->e1 = normalize(xfmVector(xfm, e1));  // the private ctors normalize _wo
  }
  return l;
}

void LightObj::commit() {
  auto l = std::make_shared<LightInst>();
  if (ieq(type, "ambientlight")) {
    l->type = LIGHT_AMBIENT;
    l->L = parms.getV3("L");
  } else if (ieq(type, "trianglelight")) {
    // lights/trianglelight.h:31-41
    l->type = LIGHT_TRIANGLE;
    l->v0 = parms.getV3("v0");
    l->v1 = parms.getV3("v1");
    l->v2 = parms.getV3("v2");
    l->e1 = l->v0 - l->v1;
    l->e2 = l->v2 - l->v0;
    l->Ng = cross(l->e1, l->e2);
    l->L = parms.getV3("L");
    l->shape = triangle_shape(l->v0, l->v1, l->v2);
  } else if (ieq(type, "hdrilight")) {
    // lights/hdrilight.cpp:24-41
    l->type = LIGHT_HDRI;
    l->l2w = parms.getTransform("local2world", a3_identity());
    l->w2l = a3_inverse(l->l2w);
    l->L = parms.getV3("L", v3s(1.f));
    l->image = std::dynamic_pointer_cast<ImageObj>(parms.getObject("image"));
    if (!l->image) {
      auto im = std::make_shared<ImageObj>();  // new Image3f(5, 5, one)
      im->width = im->height = 5;
      im->format = IMG_RGBAF32;
      im->data.resize(5 * 5 * 16);
      float* f = (float*)im->data.data();
      for (int i = 0; i < 25 * 4; ++i) f[i] = 1.0f;
      l->image = im;
    }
    const int w = l->image->width, h = l->image->height;
    std::vector<float> importance((size_t)w * h);
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) {
        float c[4];
        l->image->get(x, y, c);
        importance[(size_t)y * w + x] = sinf(kPi * (y + 0.5f) * rcpf_(float(h))) * (c[0] + c[1] + c[2]);
      }
    dist2d_init(importance.data(), w, h, l->ycdf, l->ypdf, l->xcdf, l->xpdf);
  } else if (ieq(type, "pointlight")) {
    // lights/pointlight.h:24-27
    l->type = LIGHT_POINT;
    l->v0 = parms.getV3("P", v3s(0.f));
    l->L = parms.getV3("I", v3s(0.f));
  } else if (ieq(type, "spotlight")) {
    // lights/spotlight.h:24-31
    l->type = LIGHT_SPOT;
    l->v0 = parms.getV3("P", v3s(0.f));
    l->e1 = -normalize(parms.getV3("D", v3s(0.f)));
    l->L = parms.getV3("I", v3s(0.f));
    l->cosAngleMin = cosf(0.5f * deg2rad(parms.getFloat("angleMin", 0.f)));
    l->cosAngleMax = cosf(0.5f * deg2rad(parms.getFloat("angleMax", 0.f)));
  } else if (ieq(type, "directionallight")) {
    // lights/directionallight.h:22-25
    l->type = LIGHT_DIRECTIONAL;
    l->e1 = -normalize(parms.getV3("D", v3s(0.f)));
    l->L = parms.getV3("E", v3s(0.f));
  } else if (ieq(type, "distantlight")) {
    // lights/distantlight.h:25-30
    l->type = LIGHT_DISTANT;
    l->e1 = -normalize(parms.getV3("D", v3s(0.f)));
    l->L = parms.getV3("L", v3s(0.f));
    l->halfAngle = deg2rad(parms.getFloat("halfAngle", 0.f));
    l->cosHalfAngle = cosf(l->halfAngle);
  } else {
    throw std::runtime_error("unknown light type: " + type);
  }
  inst = l;
}

// ---------------------------------------------------------------- primitives
void PrimitiveObj::commit() {
  illumMask = parms.getInt("illumMask", illumMask);
  shadowMask = parms.getInt("shadowMask", shadowMask);
}

// ---------------------------------------------------------------- cameras
void CameraObj::commit() {
  memset(&cam, 0, sizeof(cam));
  auto store = [](float* dst, const A3& a) {
    const float v[12] = {a.l.vx.x, a.l.vx.y, a.l.vx.z, a.l.vy.x, a.l.vy.y, a.l.vy.z,
                         a.l.vz.x, a.l.vz.y, a.l.vz.z, a.p.x,    a.p.y,    a.p.z};
    memcpy(dst, v, sizeof(v));
  };
  if (ieq(type, "pinhole")) {
    // cameras/pinholecamera.h:15-21
    cam.type = CAM_PINHOLE;
    const A3 l2w = parms.getTransform("local2world");
    const float angle = parms.getFloat("angle", 64.0f);
    const float aspectRatio = parms.getFloat("aspectRatio", 1.0f);
    const V3 W = xfmVector(l2w, v3(-0.5f * aspectRatio, -0.5f, 0.5f * rcpf_(tanf(deg2rad(0.5f * angle)))));
    store(cam.p2w[0], a3(l3(aspectRatio * l2w.l.vx, l2w.l.vy, W), l2w.p));
  } else if (ieq(type, "depthoffield")) {
    // cameras/depthoffieldcamera.h:13-19 over the pinhole setup
    cam.type = CAM_DOF;
    const A3 l2w = parms.getTransform("local2world");
    const float angle = parms.getFloat("angle", 64.0f);
    const float aspectRatio = parms.getFloat("aspectRatio", 1.0f);
    const V3 W = xfmVector(l2w, v3(-0.5f * aspectRatio, -0.5f, 0.5f * rcpf_(tanf(deg2rad(0.5f * angle)))));
    const A3 p2w = a3(l3(aspectRatio * l2w.l.vx, l2w.l.vy, W), l2w.p);
    store(cam.p2w[0], p2w);
    store(cam.p2w[1], l2w);
    cam.xyzStraight[0] = parms.getFloat("lensRadius", 0.0f);
    cam.xyzStraight[1] = parms.getFloat("focalDistance", 0.0f) / length(0.5f * p2w.l.vx + 0.5f * p2w.l.vy + p2w.l.vz);
  } else if (ieq(type, "stereo")) {
    // cameras/StereoCubeCamera.h:16-51
    cam.type = CAM_STEREO;
    const A3 l2w = parms.getTransform("local2world");
    const float angle = 90.f, aspectRatio = 1.f;
    cam.cubeFaceIndex = parms.getInt("cubeFaceIndex", 0);
    const V3 origin = parms.getV3("origin", l2w.p);
    const V3 lookAt = parms.getV3("lookAt", v3(0.f, 0.f, -1.f));
    const V3 up = parms.getV3("up", v3(0.f, 1.f, 0.f));
    const V3 right = cross(normalize(up), normalize(lookAt - origin));
    const float sceneScale = parms.getFloat("sceneScale", 1.f);
    const float EYE_SEPARATION = 6.35f * 0.393701f;
    const float ZERO_PARALLAX = EYE_SEPARATION * 30.f;
    cam.eyeSeparation = parms.getFloat("eyeSeparation", EYE_SEPARATION) * sceneScale;
    const float zpd = parms.getFloat("zeroParallaxDistance", ZERO_PARALLAX) * sceneScale;
    if (zpd != 0.f) {
      cam.rcpZeroParallaxDistance = 1.f / zpd;
      cam.toeIn = parms.getBool("toeIn", false);
    } else {
      cam.rcpZeroParallaxDistance = 0.f;
      cam.toeIn = 0;
    }
    cam.falloffAngle = clampf(parms.getFloat("stereFalloffAngle", 30.f), 0.f, 90.f);
    const V3 W = xfmVector(l2w, v3(-.5f * aspectRatio, -.5f, .5f * rcpf_(tanf(deg2rad(.5f * angle)))));
    A3 p2w[6];
    p2w[0] = a3(l3(aspectRatio * l2w.l.vx, l2w.l.vy, W), l2w.p);
    const V3 xyz = normalize(.5f * p2w[0].l.vx + .5f * p2w[0].l.vy + p2w[0].l.vz);
    p2w[1] = mul(a3_rotate_about(origin, up, deg2rad(90.f)), p2w[0]);
    p2w[2] = mul(a3_rotate_about(origin, up, deg2rad(180.f)), p2w[0]);
    p2w[3] = mul(a3_rotate_about(origin, up, deg2rad(-90.f)), p2w[0]);
    p2w[4] = mul(a3_rotate_about(origin, right, deg2rad(-90.f)), p2w[0]);
    p2w[4] = mul(a3_rotate_about(origin, up, deg2rad(180.f)), p2w[4]);
    p2w[5] = mul(a3_rotate_about(origin, right, deg2rad(90.f)), p2w[0]);
    p2w[5] = mul(a3_rotate_about(origin, up, deg2rad(180.f)), p2w[5]);
    for (int i = 0; i < 6; ++i) store(cam.p2w[i], p2w[i]);
    cam.origin[0] = origin.x; cam.origin[1] = origin.y; cam.origin[2] = origin.z;
    cam.up[0] = up.x; cam.up[1] = up.y; cam.up[2] = up.z;
    cam.xyzStraight[0] = xyz.x; cam.xyzStraight[1] = xyz.y; cam.xyzStraight[2] = xyz.z;
    // the pixel-independent terms of StereoCubeCamera::ray (StereoCubeCamera.h:142-159), with
    // the same operations the per-ray code would run (GpuCamera::lin ... rotP)
    for (int i = 0; i < 6; ++i) {
      const L3 lin = mul(p2w[i].l, l3_identity());  // (p2w * translate(eyeOffset,0,0)).l
      const float v[9] = {lin.vx.x, lin.vx.y, lin.vx.z, lin.vy.x, lin.vy.y, lin.vy.z, lin.vz.x, lin.vz.y, lin.vz.z};
      memcpy(cam.lin[i], v, sizeof(v));
      const V3 z = 0.f * p2w[i].l.vy + 0.f * p2w[i].l.vz;  // the translation's zero products
      cam.zero[i][0] = z.x; cam.zero[i][1] = z.y; cam.zero[i][2] = z.z;
    }
    const V3 u = normalize(up);  // l3_rotate (common/math/linearspace3.h rotate)
    const float rot[12] = {u.x,     u.y,           u.z,     u.x * u.x, 1 - u.x * u.x, u.y * u.y,
                           1 - u.y * u.y, u.z * u.z, 1 - u.z * u.z, u.x * u.y, u.x * u.z, u.y * u.z};
    memcpy(cam.rot, rot, sizeof(rot));
    const V3 rotP = mul(l3_identity(), v3s(0.0f)) + origin;  // (translate(origin) * rotate).p
    cam.negO[0] = -origin.x; cam.negO[1] = -origin.y; cam.negO[2] = -origin.z;
    cam.rotP[0] = rotP.x; cam.rotP[1] = rotP.y; cam.rotP[2] = rotP.z;
  } else {
    throw std::runtime_error("camera type '" + type + "' is outside the MI355X device's scope");
  }
}

void ToneMapperObj::commit() {
  // tonemappers/defaulttonemapper.h:15-20
  gamma = parms.getFloat("gamma", 1.0f);
  vignetting = parms.getBool("vignetting", false);
  if (vignetting) throw std::runtime_error("vignetting is not supported by the MI355X device");
}

void RendererObj::commit() {
  if (ieq(type, "debug")) {
    // renderers/debugrenderer.cpp:21-25
    debug = true;
    maxDepth = parms.getInt("maxDepth", 1);
    spp = parms.getInt("sampler.spp", 1);
  } else {
    // IntegratorRenderer + PathTraceIntegrator + SamplerFactory ctors
    // (renderers/integratorrenderer.cpp:31-61, integrators/pathtraceintegrator.cpp:21-33,
    //  samplers/sampler.cpp:23-31)
    debug = false;
    const std::string integ = parms.getString("integrator", "pathtracer");
    if (integ != "pathtracer") throw std::runtime_error("unknown integrator type: " + integ);
    maxDepth = parms.getInt("maxDepth", 10);
    rrDepth = parms.getInt("rrDepth", 5);
    minContribution = parms.getFloat("minContribution", .02f);
    epsilon = parms.getFloat("epsilon", 32.f) * kUlp;
    tMaxShadowRay = parms.getFloat("tMaxShadowRay", INFINITY);
    tMaxShadowJitter = parms.getFloat("tMaxShadowJitter", .15f);
    up = parms.getV3("up", v3(0.f, 1.f, 0.f));
    spp = parms.getInt("sampler.spp", 1);
    if (spp < 1) spp = 1;
    sets = parms.getInt("sampler.sets", 64);
    if (sets < 1) sets = 1;
    if (sets > 256) throw std::runtime_error("sampler.sets > 256 is not supported");
    filter = parms.getString("filter", "bspline");
    if (filter != "none" && filter != "box" && filter != "bspline")
      throw std::runtime_error("unknown filter type: " + filter);
    backplate = std::dynamic_pointer_cast<ImageObj>(parms.getObject("backplate"));
    if (parms.getObject("backplate") && !backplate) throw std::runtime_error("backplate is not an image");
    stopFlag = (std::atomic<bool>*)parms.getPointer("stopFlag");
    statusCallback = parms.getPointer("statusCallback");
    statusUser = parms.getPointer("statusUser");
  }
}

}  // namespace yrt
