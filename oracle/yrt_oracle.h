/* yrt_oracle.h — CPU restatement of the reference device_singleray render path.
 *
 * TEST INFRASTRUCTURE ONLY. This library is the parity checker for the MI355X device
 * plugin: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it. The product (yulio-raytracer_amd/) never links, calls or ships it.
 *
 * It restates, in plain C and independently of the product code, the reference's
 *   integrators/pathtraceintegrator.cpp, renderers/integratorrenderer.cpp,
 *   renderers/debugrenderer.cpp, samplers/{sampler.cpp,patterns.h,distribution1d.cpp,
 *   distribution2d.cpp,shapesampler.h}, filters/{filter.cpp,bsplinefilter.h,boxfilter.h},
 *   cameras/{pinholecamera.h,StereoCubeCamera.h}, shapes/{trianglemesh_full.cpp,
 *   trianglemesh_normals.cpp,triangle.h,sphere.h}, materials/{matte,matte_textured,
 *   metallicpaint,obj,Uber,thindielectric}.h, brdfs/ (all in-scope), lights/{ambientlight.h,trianglelight.h,
 *   hdrilight.cpp}, textures/ (both), api/{scene_flat.h,framebuffer.h},
 *   tonemappers/defaulttonemapper.h, common/math/{random.h,permutation.h,linearspace3.h,
 *   affinespace.h}
 * with these documented substitutions:
 *   - Embree 2.15 rtcIntersect/rtcOccluded (binary-only, absent) -> own median-split BVH and
 *     the Moeller-Trumbore convention of lights/trianglelight.h:55-65 with the back-face
 *     filter of shapes/trianglemesh_full.cpp:86-106; closest hit = smallest (t, triangle id).
 *     Parity against Embree itself is unpinned (no Embree source or binary can run here).
 *   - C rand() in the shadow-ray jitter -> the counter hash hash_u01 (also used on the GPU).
 *   - SSE rcp/rsqrt approximations -> IEEE 1/x and 1/sqrt(x).
 *   - the C runtime's sinf/cosf/powf/expf/logf/acosf/atanf/atan2f on the per-ray path (camera
 *     rays, BRDF/light sampling, shading, resolve) -> the build's own yrt_libm.h
 *     (yulio-raytracer_amd/csrc/common), evaluated with the same operations as the device does;
 *     host-side setup (camera fov, sphere tessellation, HDRI tables) keeps glibc on both sides.
 *
 * Input: the "frame blob" written by yrtExportFrame (yulio-raytracer_amd/csrc/device/export.cpp)
 *   "YRTF" u32 version(1)
 *   u32 nObjects; per object: u32 kind, str type, u32 nParms, parm*, [IMAGE: i32 w,h,fmt, u32 n, bytes]
 *     parm: str name, u32 vtype, payload
 *       BOOL1-4/INT1-4 (1..8): i32[4]; FLOAT1-4 (9..12): f32[4]; STRING (13): str;
 *       IMAGE/TEXTURE (14,15): i32 object index; TRANSFORM (16): f32[12];
 *       DATA (18): str elemType, u32 count, u32 elemBytes, bytes
 *   u32 nSlots; per slot: i32 present [, i32 shapeObj, lightObj, materialObj, f32[12] xfm,
 *     i32 faceCamera, illumMask, shadowMask]
 *   i32 rendererObj, i32 cameraObj, u32 frameSeed
 *   str = u32 length + bytes. Object kinds: 0 camera 1 data 2 image 3 texture 4 material
 *   5 shape 6 light 7 primitive 8 scene 9 tonemapper 10 renderer 11 framebuffer.
 */
#ifndef YRT_ORACLE_H
#define YRT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct OracleStats {
  double raysClosest, raysShadow, samples, seconds;
  double nodeVisits, triVisits;
} OracleStats;

/* Renders the frame described by blob into out_rgb (W*H*3 floats, RGB_FLOAT32 values after
 * tonemapping) for pixels in [x0,x1)x[y0,y1) (pixels outside are left untouched). gamma is
 * the tonemapper gamma. threads: worker threads over 16x16 tiles (0 = all cores).
 * Returns 0 on success, negative on error (message via oracle_last_error()). */
int oracle_render(const void* blob, size_t bytes, int width, int height, float gamma, int x0, int y0, int x1, int y1,
                  int threads, float* out_rgb, OracleStats* stats);

/* oracle_render restricted to the 16x16 tiles with tile % shardCount == shardIndex (the
 * multi-GPU tile split of SURVEY §8(e)); other pixels are left untouched. */
int oracle_render_shard(const void* blob, size_t bytes, int width, int height, float gamma, int x0, int y0, int x1,
                        int y1, int shardIndex, int shardCount, int threads, float* out_rgb, OracleStats* stats);

/* Traces rays against the blob's scene: org4/dir4 as in yrtIntersect; hit4 = (t,u,v,tri)
 * (tri as int bits, -1 miss). anyHit != 0 -> occluded test, hit4.w = 1/0. */
/* Debug: per-sample radiance Li of pixel (x, y), out3[3*s..] for s < min(spp, maxSpp); returns spp. */
int oracle_debug_pixel(const void* blob, size_t bytes, int width, int height, int x, int y, float* out3, int maxSpp);
/* the per-depth record of one sample of one pixel (32 floats per depth, 32 depths), the layout
 * of the device's YRT_PATH_DEBUG capture: for parity debugging only */
int oracle_debug_path(const void* blob, size_t bytes, int width, int height, int x, int y, int sample, float* out);
int oracle_trace(const void* blob, size_t bytes, const float* org4, const float* dir4, int n, int anyHit,
                 float* hit4);

/* Counts node/triangle visits of the GPU's own BVH (exported by yrtExportBVH) for the given
 * closest-hit rays (traversal order of the device kernel, restated). Used for the roofline's
 * algorithmic bytes. */
int oracle_count_visits(const void* nodes, size_t numNodes, const void* tris, size_t numTris, const float* org4,
                        const float* dir4, int n, int anyHit, double* nodeVisits, double* triVisits,
                        float* hit4,
                        size_t triStride);
/* the same traversal on the 64-B quantized nodes (common/yrt_qnode.h) of the same tree */
int oracle_count_visits_q(const void* qnodes, size_t numNodes, const void* tris, size_t numTris, const float* org4,
                          const float* dir4, int n, int anyHit, double* nodeVisits, double* triVisits, float* hit4,
                          size_t triStride);

/* Reference Random (common/math/random.h): n draws of getInt() after setSeed(seed). */
void oracle_random_ints(int seed, int n, int32_t* out);
/* Random::getFloat (random.h:71), Permutation(size, rng) (permutation.h:42-48) `count` times
 * from one generator, vector_t::shuffle (vector.h:129-133) `count` times in place. */
void oracle_random_floats(int seed, int n, float* out);
/* yrt_libm.h functions (fn 0 sin 1 cos 2 exp 3 log 4 pow(x,y) 5 asin 6 acos 7 atan 8 atan2(x,y)) */
void oracle_libm(int fn, int n, const float* x, const float* y, float* out);
/* the vector helpers and the camera path for the pin against the reference's common/math
 * (oracle/ref_math.cpp, tests/test_ref_pin.py) */
void oracle_vecmath(int fn, int n, const float* a, const float* b, float* out);
void oracle_bsphere(int n, const float* lo, const float* hi, const float* org, const float* dir, float* out);
int oracle_camera_rays(const void* blob, size_t bytes, int n, const float* px, float* org, float* dir);
void oracle_permutations(int size, int seed, int count, int32_t* out);
void oracle_shuffles(int n, int seed, int count, uint32_t* out);
/* SamplerFactory::init sample table: dims as in the GPU table ([dim][set*spp+s]);
 * returns the record count (sets*spp, spp rounded up to a power of two). */
int oracle_sample_table(int spp, int sets, int iteration, int num1D, int num2D, const char* filter, float* out,
                        size_t outFloats);
/* Per-pixel sample set index (one Random per 16x16 tile, integratorrenderer.cpp:134,149). */
void oracle_pixel_sets(int width, int height, int sets, uint8_t* out);
/* World-space triangles of the blob's scene (9 floats each, geomID-major order). */
int oracle_scene_triangles(const void* blob, size_t bytes, float* out, int maxTris);
const char* oracle_last_error(void);

#ifdef __cplusplus
}
#endif

#endif
