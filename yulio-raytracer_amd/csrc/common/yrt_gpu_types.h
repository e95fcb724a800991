// yrt_gpu_types.h — HBM layout of a committed scene and of the wavefront path state.
//
// Everything the kernels read is a flat array uploaded once per rtCommit(scene)
// (the reference rebuilt the Embree BVH at every commit, api/scene_flat.h:72-97).
//
//  BVH (4-wide, collapsed from a binned-SAH BVH2 built on the host — device/bvh_build.cpp):
//    GpuNode  128 B  the four children's AABBs as planes [axis lo/hi][child] (so a packed
//                    op tests two children's planes at once) + four child references
//                    (index << 5 | count: count 0 = inner node, 1..31 = leaf triangle
//                    range, -1 = empty slot; an empty slot's box is inverted, lo = +inf, hi = -inf).
//    GpuTri    48 B  Embree-convention Moeller-Trumbore triangle in leaf order:
//                    v0, e1 = v0-v1, e2 = v2-v0 (rtcore triangle convention);
//                    v0.w = global triangle id (int bits), e1.w = flags (cull bit).
//  Shading (indexed by global triangle id = geomTriBase[geomID] + primID):
//    triGeom   int   geomID of every triangle
//    indices   int4  (v0,v1,v2, -) absolute vertex ids
//    positions float4, normals float4, texcoords float2 (world space, per vertex)
//    GpuGeom, GpuMaterial, GpuTexture/GpuImage, GpuLight tables.
#pragma once

#include <stdint.h>

namespace yrt {

enum GeomKind : int32_t { GEOM_MESH_FULL = 0, GEOM_MESH_NORMALS = 1, GEOM_TRIANGLE = 2 };
enum GeomFlags : int32_t { GF_NORMALS = 1, GF_TEXCOORDS = 2, GF_CULL = 4, GF_MOTION = 8, GF_TANGENT_X = 16,
                           GF_TANGENT_Y = 32 };

struct GpuNode {
  float lox[4], hix[4], loy[4], hiy[4], loz[4], hiz[4];  // per child
  int32_t child[4];  // (index << 5) | count ; -1 = empty
  int32_t pad[4];
};
static_assert(sizeof(GpuNode) == 128, "node is one 128-B line");

struct GpuTri {
  float v0[4];  // xyz, w = global triangle id (bits)
  float e1[4];  // xyz, w = flags (bits): bit0 cullBackFaces
  float e2[4];  // xyz, w = geometry id (bits): the closest-hit kernels store it beside the hit
};
static_assert(sizeof(GpuTri) == 48, "tri record size");

// Moving triangles (motion blur, scenes with "motions" / Sphere dPdt): per leaf slot, beside
// its GpuTri (which holds the t = 0 triangle), the other two vertices and the three vertices'
// motion vectors; the triangle at ray time t is p + t * m (trianglemesh_full.cpp:104-109).
struct GpuTriMotion {
  float p1[3], p2[3];
  float m0[3], m1[3], m2[3];
  float pad;
};
static_assert(sizeof(GpuTriMotion) == 64, "moving tri record size");

// Per triangle (global id order): what k_shade's postIntersect reads of a static mesh triangle,
// in one 96-byte record instead of an index record plus nine vertex gathers (positions,
// normals, texcoords): e1 = p0 - p1, e2 = p2 - p0 (the geometric normal's edges; p1 - p0 is
// -e1 bit for bit), the vertex normals and texture coordinates (zero where the mesh has
// none), and the geometry id. Moving meshes and meshes with tangent arrays keep the indexed path.
struct GpuTriShade {
  float e1[3];
  int32_t geom;
  float e2[3];
  float pad0;
  float n[9];   // n0, n1, n2
  float st[6];  // st0, st1, st2
  float pad1;
};
static_assert(sizeof(GpuTriShade) == 96, "shade tri record size");

struct GpuGeom {
  int32_t kind, material, light, flags;
  int32_t vtxBase, triBase, illumMask, shadowMask;
  float Ng[4];  // GEOM_TRIANGLE: normalized cross(v2-v0, v1-v0) (shapes/triangle.h:28)
};

enum MaterialType : int32_t {
  MAT_NONE = 0,
  MAT_MATTE = 1,
  MAT_MATTE_TEXTURED = 2,
  MAT_METALLIC_PAINT = 3,
  MAT_OBJ = 4,
  MAT_UBER = 5,
  MAT_THIN_DIELECTRIC = 6,
  MAT_PLASTIC = 7,
  MAT_DIELECTRIC = 8,
  MAT_MIRROR = 9,
  MAT_METAL = 10,
  MAT_BRUSHED_METAL = 11,
  MAT_VELVET = 12,
  MAT_METALLIC_GLITTER = 13,  // MetallicPaint with glitter (glitterSpread != 0, glitterColor != 0)
};

// Parameter slots per material type (filled by device/materials.cpp from Parms with the
// reference constructors' defaults).
struct GpuMaterial {
  int32_t type;
  int32_t tex[5];   // texture ids (-1 none). Uber/MatteTextured/ThinDielectric: tex[0]=Kd.
                    // Obj: map_d, map_Kd, map_Ks, map_Ns, map_Bump
  int32_t media[2];  // Dielectric: medium table indices (outside, inside); other types unused
  float p[24];
};

enum TexFilter : int32_t { TEX_BILINEAR = 0, TEX_NEAREST = 1 };
// IMG_RGBA8: Image4c (alpha = byte/255); IMG_RGB8: Image3c stored as RGBA8 whose alpha
// reads as exactly 1.0f (common/math/color_scalar.h:45); IMG_RGBAF32: Image3f/4f.
enum ImageFormat : int32_t { IMG_RGBA8 = 0, IMG_RGBAF32 = 1, IMG_RGB8 = 2 };
struct GpuImage {
  int32_t width, height, format, pad;
  int64_t offset;   // byte offset into the texel pool
};
// The image's descriptor is repeated in the texture record so a texel fetch is one dependent
// load after the material (material -> texture -> texels) instead of two.
struct GpuTexture {
  int32_t image, filter, invert, width;
  int32_t height, format;
  int64_t offset;  // byte offset of the image in the texel pool
};
static_assert(sizeof(GpuTexture) == 32, "texture record is 32 B");

// Everything the shade kernel needs about a hit's geometry in one record: the geometry, a copy
// of its material and of the material's first texture descriptor (tex[0]: Kd / map_d). The
// chain hit -> index -> geometry -> material -> texture -> texels becomes hit -> index ->
// record -> texels: two dependent loads fewer per shaded vertex (k_shade is latency-bound).
struct GpuGeomRec {
  GpuGeom g;
  GpuMaterial m;  // zero when the geometry has no material (g.material < 0)
  GpuTexture t0;  // m.tex[0]'s descriptor (zero when none)
};
static_assert(sizeof(GpuGeomRec) % 16 == 0, "16-byte aligned records");

enum LightType : int32_t {
  LIGHT_AMBIENT = 0,
  LIGHT_TRIANGLE = 1,
  LIGHT_HDRI = 2,
  LIGHT_POINT = 3,        // v0 = P, L = I
  LIGHT_SPOT = 4,         // v0 = P, e1 = _D (negative direction), L = I, bsphere = (cosMin, cosMax)
  LIGHT_DIRECTIONAL = 5,  // e1 = _wo, L = E
  LIGHT_DISTANT = 6,      // e1 = _wo, L, bsphere = (halfAngle, cosHalfAngle); also an env light
};
struct GpuLight {
  int32_t type, illumMask, shadowMask, precomputed;  // precomputed: index into light-sample slots or -1
  int32_t isEnv, image, distOffset, pad;             // HDRI: image id, distribution offset (floats)
  float L[4];
  float v0[4], v1[4], v2[4];     // triangle light vertices
  float e1[4], e2[4], Ng[4];     // e1 = v0-v1, e2 = v2-v0, Ng = cross(e1,e2) (lights/trianglelight.h:24)
  float bsphere[4];              // ambient: center.xyz, radius (ambientlight.h:28-32)
  float l2w[12], w2l[12];        // HDRI local2world / world2local (column-major l, then p)
  int32_t hdriW, hdriH, pad2[2];
};

// Division of n in [0, 2^31) by a run-time constant d in [1, 2^31) as multiply-high, add and
// shift (the round-up method of Granlund & Montgomery, PLDI 1994): q = (umulhi(n, mul) + n) >>
// shift, three VALU instead of the ~25 of an integer division. Exact over the whole range
// (tests/test_fastdiv.py checks the construction).
struct FastDiv {
  uint32_t mul, shift;
};
static inline FastDiv fastdiv_make(uint32_t d) {
  uint32_t shift = 0;
  while (shift < 31 && (1u << shift) < d) ++shift;
  const uint64_t magic = ((uint64_t)1 << 32) * (((uint64_t)1 << shift) - d) / d + 1;
  FastDiv f;
  f.mul = (uint32_t)magic;
  f.shift = shift;
  return f;
}

// Renderer parameters (integrators/pathtraceintegrator.cpp:21-33 defaults).
struct GpuRenderParams {
  int32_t maxDepth, rrDepth, spp, sets;
  float minContribution, epsilon, tMaxShadowRay, tMaxShadowJitter;
  float up[4];
  int32_t numLights, numEnvLights, numPrecomp, dim1D;  // dim1D = maxDepth
  int32_t dim2D, lightSampleID, firstScatterSampleID, firstScatterTypeSampleID;
  int32_t width, height, numTilesX, numTilesY;
  float rcpWidth, rcpHeight, gamma, rcpGamma;
  uint32_t frameSeed;
  // frames rendered together (yrtRenderFrames: the 12 faces of a stereo cubemap): tile t of
  // the job is tile t % tilesPerFrame of frame t / tilesPerFrame (numTilesX * numTilesY each)
  int32_t numFrames, tilesPerFrame, pad;
  FastDiv divTilesX, divTilesPerFrame;  // fastdiv_make(numTilesX), fastdiv_make(tilesPerFrame)
  // radiance of a camera ray that misses, for the fused depth 0 (PrimaryRays): the sum over the
  // environment lights of 1 * L, as k_shade's depth-0 miss branch adds it (ambient lights only)
  float missL[4];
};

// Camera (cameras/pinholecamera.h:15-21, cameras/StereoCubeCamera.h:16-65).
// CAM_DOF (cameras/depthoffieldcamera.h): p2w[0] pixel2world, p2w[1] local2world,
// xyzStraight[0] lensRadius, xyzStraight[1] focalDistance (normalized)
enum CameraType : int32_t { CAM_PINHOLE = 0, CAM_STEREO = 1, CAM_DOF = 2 };
struct GpuCamera {
  int32_t type, cubeFaceIndex, toeIn, pad;
  float p2w[6][12];           // pixel2world[face]: vx, vy, vz, p (column-major)
  float origin[4], up[4], xyzStraight[4];
  float eyeSeparation, rcpZeroParallaxDistance, falloffAngle, pad2;
  // CAM_STEREO without toe-in: the terms of StereoCubeCamera::ray that do not depend on the
  // pixel, computed on the host with the device's operations (objects.cpp stereo_precompute):
  //   lin[f]   (pixel2world[f] * translate(eyeOffset, 0, 0)).l = pixel2world[f].l * identity
  //   zero[f]  the translation's zero products of that point, (0 * vy) + (0 * vz), per axis
  //   rot      normalize(up) as in l3_rotate: u.xyz, then u.x*u.x, 1-u.x*u.x, u.y*u.y,
  //            1-u.y*u.y, u.z*u.z, 1-u.z*u.z, u.x*u.y, u.x*u.z, u.y*u.z
  //   negO     -origin;  rotP  (translate(origin) * rotate(up, theta)).p = I*0 + origin
  float lin[6][9];
  float zero[6][3];
  float rot[12];
  float negO[4], rotP[4];
};

// Precomputed sample table (samplers/sampler.cpp:85-158), SoA [dim][set*spp + s].
//   dims: 0,1 pixel.xy | 2,3 lens | 4 time | 5.. 1D (dim1D) | then 2D (dim2D x 2)
//   light samples (HDRI precompute): per slot 8 floats (wi.xyz, pdf, L.rgb, tMax)
struct SampleTableLayout {
  int32_t numRecords;   // sets * spp
  int32_t numDims;      // 5 + dim1D + 2*dim2D
  int32_t numLightSlots;
  int32_t pad;
};

}  // namespace yrt
