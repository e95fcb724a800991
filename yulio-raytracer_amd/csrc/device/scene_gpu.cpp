// scene_gpu.cpp — flatten a committed scene into HBM buffers + BVH.
//
// Follows BackendSceneFlat::Handle::create (api/scene_flat.h:72-97) and the
// BackendSceneFlat ctor (:105-121): geomID = index among primitives that have a shape, in
// slot order; allLights in slot order; envLights = ambient/HDRI lights. Geometry is the
// world-space result of Shape::transform, exactly what extract() handed to Embree.
#include "scene_gpu.h"

#include <string.h>

#include <chrono>
#include <map>

#include "bvh_build.h"
#include "distribution.h"

namespace yrt {

// SceneView pointers of the scene's own device buffers (counts already set in S.view)
static void bind_view(GpuScene& S) {
  SceneView& v = S.view;
  v.nodes = S.nodes.as<GpuNode>();
  v.qnodes = S.qnodes.as<GpuQNode>();
  v.tris = S.tris.as<GpuTri>();
  v.triGeom = S.triGeom.as<int>();
  v.indices = S.indices.as<int4>();
  v.positions = S.positions.as<float4>();
  v.normals = S.normals.as<float4>();
  v.texcoords = S.texcoords.as<float2>();
  v.geoms = S.geoms.as<GpuGeom>();
  v.geomRecs = S.geomRecs.as<GpuGeomRec>();
  v.triShade = S.triShade.as<GpuTriShade>();
  v.materials = S.materials.as<GpuMaterial>();
  v.textures = S.textures.as<GpuTexture>();
  v.images = S.images.as<GpuImage>();
  v.texels = S.texels.as<uint8_t>();
  v.texQuads = S.texQuads.as<uint8_t>();
  v.lights = S.lights.as<GpuLight>();
  v.envLights = S.envLights.as<int>();
  v.media = S.media.as<float4>();
  v.motions = S.motions.as<float4>();
  v.tangents = S.tangents.as<float4>();
  v.triMotion = S.triMotion.as<GpuTriMotion>();
  v.hdriDist = nullptr;
}

std::shared_ptr<GpuScene> build_gpu_scene(const std::vector<std::shared_ptr<ScenePrim>>& prims, int stackDepth,
                                          bool upload) {
  auto t0 = std::chrono::steady_clock::now();
  auto S = std::make_shared<GpuScene>();
  if (upload) HIP_CHECK(hipGetDevice(&S->device));

  std::vector<float4> positions, normals, motions, tangents;  // tangents: (x, y) per vertex
  std::vector<float2> texcoords;
  bool anyMotion = false, anyTangent = false;
  for (const auto& p : prims)
    if (p && p->shape) {
      anyMotion |= !p->shape->mot.empty();
      anyTangent |= !p->shape->tanX.empty() || !p->shape->tanY.empty();
    }
  std::vector<float> triVerts1;  // moving scenes: the triangles at the end of the frame time
  std::vector<int4> indices;
  std::vector<int> triGeom;
  std::vector<float> triVerts;
  std::vector<uint32_t> triFlags;
  std::vector<GpuGeom> geoms;
  std::vector<GpuMaterial> materials;
  std::vector<GpuTexture> textures;
  std::vector<GpuImage> images;
  // 8-bit images first, float images (HDRI maps) after them: the bilinear footprint records
  // (texQuads, 4x the bytes) cover only the 8-bit part of the pool
  std::vector<uint8_t> texels, texelsF;
  std::vector<GpuLight> lights;
  std::vector<int> envLights;
  int numEnvZero = 0;
  int numEnvDir = 0;
  std::map<const MaterialInst*, int> matIds;
  std::map<const TextureInst*, int> texIds;
  std::map<const ImageObj*, int> imgIds;

  auto imageId = [&](const std::shared_ptr<ImageObj>& im) -> int {
    auto it = imgIds.find(im.get());
    if (it != imgIds.end()) return it->second;
    GpuImage g;
    memset(&g, 0, sizeof(g));
    g.width = im->width;
    g.height = im->height;
    g.format = im->format;
    std::vector<uint8_t>& pool = im->format == IMG_RGBAF32 ? texelsF : texels;
    size_t off = (pool.size() + 15) & ~size_t(15);
    pool.resize(off);
    g.offset = (int64_t)off;  // float images: relative to the float part until it is placed
    pool.insert(pool.end(), im->data.begin(), im->data.end());
    images.push_back(g);
    return imgIds[im.get()] = (int)images.size() - 1;
  };
  auto textureId = [&](const std::shared_ptr<const TextureInst>& t) -> int {
    if (!t) return -1;
    auto it = texIds.find(t.get());
    if (it != texIds.end()) return it->second;
    GpuTexture g;
    memset(&g, 0, sizeof(g));
    g.image = imageId(t->image);
    g.width = images[g.image].width;
    g.height = images[g.image].height;
    g.format = images[g.image].format;
    g.offset = images[g.image].offset;
    g.filter = t->filter;
    g.invert = t->invert ? 1 : 0;
    textures.push_back(g);
    return texIds[t.get()] = (int)textures.size() - 1;
  };
  // medium table (materials/medium.h): [0] = vacuum; Medium::operator== compares by value, so
  // media are deduplicated by value and compared by index on the GPU
  std::vector<float4> media = {make_float4(1.f, 1.f, 1.f, 1.f)};
  auto mediumId = [&](float tr, float tg, float tb, float eta) -> int {
    for (size_t i = 0; i < media.size(); ++i)
      if (media[i].x == tr && media[i].y == tg && media[i].z == tb && media[i].w == eta) return (int)i;
    media.push_back(make_float4(tr, tg, tb, eta));
    return (int)media.size() - 1;
  };
  auto materialId = [&](const std::shared_ptr<const MaterialInst>& m) -> int {
    if (!m) return -1;
    auto it = matIds.find(m.get());
    if (it != matIds.end()) return it->second;
    GpuMaterial g = m->gm;
    for (int k = 0; k < 5; ++k) g.tex[k] = textureId(m->tex[k]);
    if (g.type == MAT_DIELECTRIC) {
      g.media[0] = mediumId(g.p[0], g.p[1], g.p[2], g.p[3]);  // outside
      g.media[1] = mediumId(g.p[4], g.p[5], g.p[6], g.p[7]);  // inside
    }
    materials.push_back(g);
    return matIds[m.get()] = (int)materials.size() - 1;
  };

  // lights first (allLights in slot order) so geometries can reference their area light
  std::vector<int> primLight(prims.size(), -1);
  int numPrecomp = 0;
  for (size_t i = 0; i < prims.size(); ++i) {
    const auto& p = prims[i];
    if (!p || !p->light) continue;
    const LightInst& L = *p->light;
    GpuLight g;
    memset(&g, 0, sizeof(g));
    g.type = L.type;
    g.illumMask = L.illumMask;
    g.shadowMask = L.shadowMask;
    g.precomputed = -1;
    g.L[0] = L.L.x; g.L[1] = L.L.y; g.L[2] = L.L.z;
    auto st3 = [](float* d, V3 v) { d[0] = v.x; d[1] = v.y; d[2] = v.z; };
    st3(g.v0, L.v0); st3(g.v1, L.v1); st3(g.v2, L.v2);
    st3(g.e1, L.e1); st3(g.e2, L.e2); st3(g.Ng, L.Ng);
    auto stA = [](float* d, const A3& a) {
      const float v[12] = {a.l.vx.x, a.l.vx.y, a.l.vx.z, a.l.vy.x, a.l.vy.y, a.l.vy.z,
                           a.l.vz.x, a.l.vz.y, a.l.vz.z, a.p.x,    a.p.y,    a.p.z};
      memcpy(d, v, sizeof(v));
    };
    stA(g.l2w, L.l2w);
    stA(g.w2l, L.w2l);
    g.bsphere[0] = L.type == LIGHT_SPOT ? L.cosAngleMin : L.halfAngle;
    g.bsphere[1] = L.type == LIGHT_SPOT ? L.cosAngleMax : L.cosHalfAngle;
    // EnvironmentLight subclasses (api/scene.h:76): ambient, HDRI, distant
    if (L.type == LIGHT_AMBIENT || L.type == LIGHT_HDRI || L.type == LIGHT_DISTANT) {
      g.isEnv = 1;
      // an environment light whose Le is exactly 0 for every direction (L = 0 0 0 over finite
      // texels, e.g. C4's HDRILight) only adds throughput * 0 to a missed path: k_shade leaves
      // it out and keeps the NaN such an add makes of a non-finite throughput (numEnvZero)
      bool zero = L.L.x == 0.f && L.L.y == 0.f && L.L.z == 0.f;
      if (zero && L.type == LIGHT_HDRI && L.image && L.image->format == IMG_RGBAF32) {
        const float* f = (const float*)L.image->data.data();
        for (size_t k = 0; k < L.image->data.size() / 4 && zero; ++k) zero = std::isfinite(f[k]);
      }
      if (zero) {
        ++numEnvZero;
      } else {
        envLights.push_back((int)lights.size());
        if (L.type != LIGHT_AMBIENT) ++numEnvDir;
      }
    }
    if (L.type == LIGHT_HDRI) {
      g.image = imageId(L.image);
      g.hdriW = L.image->width;
      g.hdriH = L.image->height;
    }
    if (L.precompute()) {
      g.precomputed = numPrecomp++;
      // HDRILight::sample (lights/hdrilight.cpp:77-87), evaluated once per sample record
      auto lp = p->light;
      LightSampleSource src;
      src.baseSample = 0;  // lightSampleID: first request2D() (pathtraceintegrator.cpp:39)
      src.sample = [lp](float ux, float uy, float* o) {
        const int w = lp->image->width, h = lp->image->height;
        float sx, sy, pdf;
        dist2d_sample(lp->ycdf, lp->ypdf, lp->xcdf, lp->xpdf, w, h, ux, uy, sx, sy, pdf);
        const float theta = kPi * sy * rcpf_(float(h));
        const float phi = kTwoPi * (1.0f - sx * rcpf_(float(w)));
        const V3 _wi = v3(-sinf(theta) * cosf(phi), cosf(theta), -sinf(theta) * sinf(phi));
        const V3 wi = xfmVector(lp->l2w, _wi);
        const float wpdf = pdf * rcpf_(kTwoPi * kPi * sinf(theta));
        float c[4];
        lp->image->get(std::max(0, std::min((int)sx, w - 1)), std::max(0, std::min((int)sy, h - 1)), c);
        o[0] = wi.x; o[1] = wi.y; o[2] = wi.z; o[3] = wpdf;
        o[4] = lp->L.x * c[0]; o[5] = lp->L.y * c[1]; o[6] = lp->L.z * c[2];
        o[7] = INFINITY;
      };
      S->precomputed.push_back(src);
    }
    primLight[i] = (int)lights.size();
    lights.push_back(g);
    S->allLights.push_back(p->light);
  }

  // geometries in slot order (geomID = compacted index)
  int gidBase = 0;
  for (size_t i = 0; i < prims.size(); ++i) {
    const auto& p = prims[i];
    if (!p || !p->shape) continue;
    const MeshInst& m = *p->shape;
    GpuGeom g;
    memset(&g, 0, sizeof(g));
    g.kind = m.kind;
    g.material = materialId(p->material);
    g.light = primLight[i];
    g.illumMask = p->illumMask;
    g.shadowMask = p->shadowMask;
    g.vtxBase = (int)positions.size();
    g.triBase = gidBase;
    g.flags = (m.nor.empty() ? 0 : GF_NORMALS) | (m.uv.empty() ? 0 : GF_TEXCOORDS) | (m.cull ? GF_CULL : 0) |
              (m.mot.empty() ? 0 : GF_MOTION) | (m.tanX.empty() ? 0 : GF_TANGENT_X) |
              (m.tanY.empty() ? 0 : GF_TANGENT_Y);
    g.Ng[0] = m.Ng.x; g.Ng[1] = m.Ng.y; g.Ng[2] = m.Ng.z;
    const int geomId = (int)geoms.size();
    for (size_t k = 0; k < m.pos.size(); ++k) {
      positions.push_back(make_float4(m.pos[k].x, m.pos[k].y, m.pos[k].z, 0.f));
      if (!m.nor.empty()) normals.push_back(make_float4(m.nor[k].x, m.nor[k].y, m.nor[k].z, 0.f));
      else normals.push_back(make_float4(0.f, 0.f, 0.f, 0.f));
      if (!m.uv.empty()) texcoords.push_back(make_float2(m.uv[2 * k], m.uv[2 * k + 1]));
      else texcoords.push_back(make_float2(0.f, 0.f));
      if (anyMotion)
        motions.push_back(m.mot.empty() ? make_float4(0.f, 0.f, 0.f, 0.f)
                                        : make_float4(m.mot[k].x, m.mot[k].y, m.mot[k].z, 0.f));
      if (anyTangent) {
        tangents.push_back(m.tanX.empty() ? make_float4(0.f, 0.f, 0.f, 0.f)
                                          : make_float4(m.tanX[k].x, m.tanX[k].y, m.tanX[k].z, 0.f));
        tangents.push_back(m.tanY.empty() ? make_float4(0.f, 0.f, 0.f, 0.f)
                                          : make_float4(m.tanY[k].x, m.tanY[k].y, m.tanY[k].z, 0.f));
      }
    }
    const int nt = (int)(m.tri.size() / 3);
    for (int t = 0; t < nt; ++t) {
      const int a = m.tri[3 * t], b = m.tri[3 * t + 1], c = m.tri[3 * t + 2];
      indices.push_back(make_int4(g.vtxBase + a, g.vtxBase + b, g.vtxBase + c, geomId));
      triGeom.push_back(geomId);
      const V3 va = m.pos[a], vb = m.pos[b], vc = m.pos[c];
      const float tv[9] = {va.x, va.y, va.z, vb.x, vb.y, vb.z, vc.x, vc.y, vc.z};
      triVerts.insert(triVerts.end(), tv, tv + 9);
      if (anyMotion) {  // p + m: the vertices at time 1 (trianglemesh_full.cpp:152-166)
        const V3 z = v3s(0.f);
        const V3 ma = m.mot.empty() ? z : m.mot[a], mb = m.mot.empty() ? z : m.mot[b], mc = m.mot.empty() ? z : m.mot[c];
        const V3 qa = va + ma, qb = vb + mb, qc = vc + mc;
        const float tv1[9] = {qa.x, qa.y, qa.z, qb.x, qb.y, qb.z, qc.x, qc.y, qc.z};
        triVerts1.insert(triVerts1.end(), tv1, tv1 + 9);
      }
      triFlags.push_back(m.cull ? 1u : 0u);
    }
    gidBase += nt;
    geoms.push_back(g);
  }
  if (gidBase >= (1 << 26)) throw std::runtime_error("scene exceeds 2^26 triangles (stack entry packing)");

  BvhResult bvh;
  build_bvh(triVerts, triFlags, stackDepth, bvh, anyMotion ? &triVerts1 : nullptr);
  // each leaf record carries its triangle's geometry id (GpuTri::e2[3]) for the closest-hit
  // kernels' hitGeom output
  for (size_t i = 0; i < bvh.tris.size(); ++i) memcpy(&bvh.tris[i].e2[3], &triGeom[bvh.order[i]], 4);
  // the any-hit kernels' 64-B nodes (common/yrt_qnode.h), node for node
  std::vector<GpuQNode> qnodes(bvh.nodes.size());
  for (size_t i = 0; i < bvh.nodes.size(); ++i) yrt_quantize_node(bvh.nodes[i], qnodes[i]);
  S->hasMotion = anyMotion;
  S->bvhDepth = bvh.maxDepth;
  S->numTris = gidBase;
  S->numGeoms = (int)geoms.size();
  for (int k = 0; k < 3; ++k) { S->bboxLo[k] = INFINITY; S->bboxHi[k] = -INFINITY; }
  for (size_t i = 0; i < triVerts.size(); i += 3)
    for (int k = 0; k < 3; ++k) {
      S->bboxLo[k] = std::min(S->bboxLo[k], triVerts[i + k]);
      S->bboxHi[k] = std::max(S->bboxHi[k], triVerts[i + k]);
    }

  if (!upload) {
    S->hNodes = std::move(bvh.nodes);
    S->hQNodes = std::move(qnodes);
    S->hTris = std::move(bvh.tris);
    S->hGeoms = geoms;
    S->hTriGeom = triGeom;
    S->view.numLights = (int)lights.size();
    S->buildSeconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return S;
  }
  {
    // place the float images after the 8-bit ones; image and texture records get final offsets
    const size_t base = (texels.size() + 15) & ~size_t(15);
    S->texels8Bytes = base;
    texels.resize(base);
    texels.insert(texels.end(), texelsF.begin(), texelsF.end());
    for (GpuImage& g : images)
      if (g.format == IMG_RGBAF32) g.offset += (int64_t)base;
    for (GpuTexture& t : textures) t.offset = images[t.image].offset;
  }
  for (const GpuMaterial& m : materials) S->materialMask |= 1u << m.type;
  for (const GpuLight& l : lights) S->materialMask |= 1u << (16 + l.type);  // light_bit (kernels/yrt_shade.h)
  S->nodes.upload(bvh.nodes);
  S->qnodes.upload(qnodes);
  S->tris.upload(bvh.tris);
  S->triGeom.upload(triGeom);
  S->indices.upload(indices);
  S->positions.upload(positions);
  if (anyMotion) {
    S->motions.upload(motions);
    // per leaf slot: the moving triangle's other vertices and the vertex motions
    std::vector<GpuTriMotion> tm(bvh.tris.size());
    for (size_t i = 0; i < bvh.tris.size(); ++i) {
      const int gid = bvh.order[i];
      const int4 ix = indices[gid];
      const int vtx[3] = {ix.x, ix.y, ix.z};
      GpuTriMotion& r = tm[i];
      memset(&r, 0, sizeof(r));
      const float4 p1 = positions[vtx[1]], p2 = positions[vtx[2]];
      r.p1[0] = p1.x; r.p1[1] = p1.y; r.p1[2] = p1.z;
      r.p2[0] = p2.x; r.p2[1] = p2.y; r.p2[2] = p2.z;
      float* ms[3] = {r.m0, r.m1, r.m2};
      for (int k = 0; k < 3; ++k) {
        const float4 mv = motions[vtx[k]];
        ms[k][0] = mv.x; ms[k][1] = mv.y; ms[k][2] = mv.z;
      }
    }
    S->triMotion.upload(tm);
  }
  if (anyTangent) S->tangents.upload(tangents);
  S->normals.upload(normals);
  S->texcoords.upload(texcoords);
  S->geoms.upload(geoms);
  {
    std::vector<GpuTriShade> ts(indices.size());
    for (size_t t = 0; t < indices.size(); ++t) {
      const int4 ix = indices[t];
      const int v[3] = {ix.x, ix.y, ix.z};
      GpuTriShade& r = ts[t];
      memset(&r, 0, sizeof(r));
      const float4 p0 = positions[ix.x], p1 = positions[ix.y], p2 = positions[ix.z];
      r.e1[0] = p0.x - p1.x; r.e1[1] = p0.y - p1.y; r.e1[2] = p0.z - p1.z;
      r.e2[0] = p2.x - p0.x; r.e2[1] = p2.y - p0.y; r.e2[2] = p2.z - p0.z;
      r.geom = ix.w;
      for (int k = 0; k < 3; ++k) {
        const float4 n = normals[v[k]];
        r.n[3 * k] = n.x; r.n[3 * k + 1] = n.y; r.n[3 * k + 2] = n.z;
        r.st[2 * k] = texcoords[v[k]].x;
        r.st[2 * k + 1] = texcoords[v[k]].y;
      }
    }
    S->triShade.upload(ts);
  }
  {
    std::vector<GpuGeomRec> recs(geoms.size());
    for (size_t i = 0; i < geoms.size(); ++i) {
      GpuGeomRec& r = recs[i];
      memset(&r, 0, sizeof(r));
      r.g = geoms[i];
      if (r.g.material >= 0) {
        r.m = materials[r.g.material];
        if (r.m.tex[0] >= 0) r.t0 = textures[r.m.tex[0]];
      }
    }
    S->geomRecs.upload(recs);
  }
  S->materials.upload(materials);
  S->textures.upload(textures);
  S->images.upload(images);
  S->texels.upload(texels);
  {
    // bilinear footprints of the 8-bit images (kernels/yrt_shade.h tex_get): record i of an image
    // holds the 4-byte texels i, i+1, i+W, i+W+1 — the bytes the four row-major fetches read —
    // at 4x the texel's byte offset; float images keep the row-major pool only
    std::vector<uint32_t> quads(S->texels8Bytes, 0u);
    auto word = [&](size_t b) -> uint32_t {
      uint32_t w = 0;
      if (b + 4 <= S->texels8Bytes) memcpy(&w, &texels[b], 4);
      return w;
    };
    for (const GpuImage& g : images) {
      if (g.format == IMG_RGBAF32) continue;
      const size_t n = (size_t)g.width * g.height, W = (size_t)g.width;
      for (size_t i = 0; i < n; ++i) {
        const size_t b = (size_t)g.offset + 4 * i, q = b;  // uint32 index of the record = byte offset
        quads[q + 0] = word(b);
        quads[q + 1] = word(b + 4);
        quads[q + 2] = word(b + 4 * W);
        quads[q + 3] = word(b + 4 * W + 4);
      }
    }
    S->texQuads.upload(quads);
  }
  S->lights.upload(lights);
  S->hLights = lights;
  S->hEnvLights = envLights;
  S->envLights.upload(envLights);
  S->media.upload(media);

  S->view.numLights = (int)lights.size();
  S->view.numEnvLights = (int)envLights.size();
  S->view.numEnvZero = numEnvZero;
  S->view.numEnvDir = numEnvDir;
  S->view.numNodes = (int)bvh.nodes.size();
  S->view.numTris = gidBase;
  bind_view(*S);

  // refit support: slot -> geometry, gid -> leaf position, nodes grouped by depth
  S->slotsCommitted = prims;
  S->slotGeom.assign(prims.size(), -1);
  {
    int gcount = 0;
    for (size_t i = 0; i < prims.size(); ++i)
      if (prims[i] && prims[i]->shape) S->slotGeom[i] = gcount++;
    // gid -> leaf slots (CSR: gidBase + 1 offsets, then the slots; spatial splits can put a
    // triangle in several leaves)
    std::vector<int> leafOf(gidBase + 1 + bvh.order.size(), 0);
    for (int g : bvh.order) leafOf[g + 1]++;
    for (int g = 0; g < gidBase; ++g) leafOf[g + 1] += leafOf[g];
    std::vector<int> fill(leafOf.begin(), leafOf.begin() + gidBase);
    for (size_t i = 0; i < bvh.order.size(); ++i) leafOf[gidBase + 1 + fill[bvh.order[i]]++] = (int)i;
    S->triLeaf.upload(leafOf);
    std::vector<std::vector<int>> levels;
    std::vector<std::pair<int, int>> work = {{0, 0}};
    for (size_t w = 0; w < work.size(); ++w) {
      const int ni = work[w].first, d = work[w].second;
      if ((int)levels.size() <= d) levels.resize(d + 1);
      levels[d].push_back(ni);
      for (int k = 0; k < 4; ++k) {
        const int c = bvh.nodes[ni].child[k];
        if (c != -1 && (c & 31) == 0) work.push_back({c >> 5, d + 1});
      }
    }
    std::vector<int> flat;
    S->levelStart.clear();
    for (auto& l : levels) {
      S->levelStart.push_back((int)flat.size());
      flat.insert(flat.end(), l.begin(), l.end());
    }
    S->levelStart.push_back((int)flat.size());
    S->levelNodes.upload(flat);
  }

  S->hNodes = std::move(bvh.nodes);
  S->hQNodes = std::move(qnodes);
  S->hTris = std::move(bvh.tris);
  S->hGeoms = geoms;
  S->hTriGeom = triGeom;
  S->buildSeconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return S;
}

std::shared_ptr<GpuScene> replicate_gpu_scene(const GpuScene& src, int device) {
  HIP_CHECK(hipSetDevice(device));
  auto R = std::make_shared<GpuScene>();
  R->device = device;
  R->serial = src.serial;  // same committed scene: the sample-table caches may key on it
  auto copy = [&](DevBuf& dst, const DevBuf& from) {
    if (!from.p) return;
    dst.alloc(from.bytes);
    HIP_CHECK(hipMemcpyPeer(dst.p, device, from.p, src.device, from.bytes));
  };
  copy(R->nodes, src.nodes);
  copy(R->qnodes, src.qnodes);
  copy(R->tris, src.tris);
  copy(R->triGeom, src.triGeom);
  copy(R->indices, src.indices);
  copy(R->positions, src.positions);
  copy(R->normals, src.normals);
  copy(R->texcoords, src.texcoords);
  copy(R->geoms, src.geoms);
  copy(R->geomRecs, src.geomRecs);
  copy(R->triShade, src.triShade);
  copy(R->materials, src.materials);
  copy(R->textures, src.textures);
  copy(R->images, src.images);
  copy(R->texels, src.texels);
  copy(R->texQuads, src.texQuads);
  copy(R->lights, src.lights);
  copy(R->envLights, src.envLights);
  copy(R->media, src.media);
  copy(R->motions, src.motions);
  copy(R->triMotion, src.triMotion);
  copy(R->tangents, src.tangents);
  R->hasMotion = src.hasMotion;
  R->view = src.view;
  bind_view(*R);
  R->materialMask = src.materialMask;
  R->precomputed = src.precomputed;
  R->hLights = src.hLights;
  R->hEnvLights = src.hEnvLights;
  R->numTris = src.numTris;
  R->numGeoms = src.numGeoms;
  R->bvhDepth = src.bvhDepth;
  R->refits = src.refits;
  R->texels8Bytes = src.texels8Bytes;
  return R;
}

bool refit_gpu_scene(GpuScene& S, const std::vector<std::shared_ptr<ScenePrim>>& prims, hipStream_t stream) {
  // moving geometry: boxes span the frame time and leaf records carry motion (rebuild instead)
  if (!S.nodes.p || prims.size() != S.slotsCommitted.size() || S.hNodes.empty() || S.hasMotion) return false;
  std::vector<size_t> moved;
  for (size_t i = 0; i < prims.size(); ++i) {
    const auto& o = S.slotsCommitted[i];
    const auto& n = prims[i];
    if (o == n) continue;
    if (!o || !n || !o->shape || !n->shape || o->light || n->light) return false;
    if (o->material != n->material || o->illumMask != n->illumMask || o->shadowMask != n->shadowMask) return false;
    const MeshInst& a = *o->shape;
    const MeshInst& b = *n->shape;
    if (a.kind != b.kind || b.kind == GEOM_TRIANGLE || a.cull != b.cull) return false;
    if (a.pos.size() != b.pos.size() || a.nor.size() != b.nor.size() || a.uv != b.uv || a.tri != b.tri) return false;
    // a refit re-uploads positions and normals only: a shape that gains motion (the refit keeps
    // a static scene's boxes and flags), or whose tangents change (a moved mesh's tangents are
    // rotated with it), is rebuilt
    if (!a.mot.empty() || !b.mot.empty()) return false;
    auto same_v3 = [](const std::vector<V3>& x, const std::vector<V3>& y) {
      return x.size() == y.size() && (x.empty() || !memcmp(x.data(), y.data(), x.size() * sizeof(V3)));
    };
    if (!same_v3(a.tanX, b.tanX) || !same_v3(a.tanY, b.tanY)) return false;
    const bool same = !memcmp(a.pos.data(), b.pos.data(), a.pos.size() * sizeof(V3)) &&
                      (a.nor.empty() || !memcmp(a.nor.data(), b.nor.data(), a.nor.size() * sizeof(V3)));
    if (!same) moved.push_back(i);
  }
  S.slotsCommitted = prims;  // unchanged geometry: adopt the new slot objects (export)
  if (moved.empty()) return true;
  const auto t0 = std::chrono::steady_clock::now();
  for (size_t i : moved) {
    const MeshInst& m = *prims[i]->shape;
    const GpuGeom& g = S.hGeoms[S.slotGeom[i]];
    std::vector<float4> pos(m.pos.size()), nor(m.pos.size());
    for (size_t k = 0; k < m.pos.size(); ++k) {
      pos[k] = make_float4(m.pos[k].x, m.pos[k].y, m.pos[k].z, 0.f);
      nor[k] = m.nor.empty() ? make_float4(0.f, 0.f, 0.f, 0.f) : make_float4(m.nor[k].x, m.nor[k].y, m.nor[k].z, 0.f);
    }
    HIP_CHECK(hipMemcpyAsync(S.positions.as<float4>() + g.vtxBase, pos.data(), pos.size() * sizeof(float4),
                             hipMemcpyHostToDevice, stream));
    HIP_CHECK(hipMemcpyAsync(S.normals.as<float4>() + g.vtxBase, nor.data(), nor.size() * sizeof(float4),
                             hipMemcpyHostToDevice, stream));
    launch_refit_tris(S.tris.as<GpuTri>(), S.triShade.as<GpuTriShade>(), S.indices.as<int4>(), S.positions.as<float4>(),
                      S.normals.as<float4>(), S.triLeaf.as<int>(), S.triLeaf.as<int>() + S.numTris + 1, g.triBase,
                      (int)(m.tri.size() / 3), stream);
    // the host copies must outlive the async copies
    HIP_CHECK(hipStreamSynchronize(stream));
  }
  for (int d = (int)S.levelStart.size() - 2; d >= 0; --d)
    launch_refit_nodes(S.nodes.as<GpuNode>(), S.tris.as<GpuTri>(), S.indices.as<int4>(), S.positions.as<float4>(),
                       S.levelNodes.as<int>() + S.levelStart[d], S.levelStart[d + 1] - S.levelStart[d], stream);
  launch_quantize_nodes(S.nodes.as<GpuNode>(), S.qnodes.as<GpuQNode>(), (int)S.hNodes.size(), stream);
  HIP_CHECK(hipStreamSynchronize(stream));
  S.hostBvhStale = true;
  S.refits++;
  S.buildSeconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return true;
}

void sync_host_bvh(GpuScene& S) {
  if (!S.hostBvhStale) return;
  HIP_CHECK(hipMemcpy(S.hNodes.data(), S.nodes.p, S.hNodes.size() * sizeof(GpuNode), hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(S.hQNodes.data(), S.qnodes.p, S.hQNodes.size() * sizeof(GpuQNode), hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(S.hTris.data(), S.tris.p, S.hTris.size() * sizeof(GpuTri), hipMemcpyDeviceToHost));
  S.hostBvhStale = false;
}

}  // namespace yrt
