/* yrt_frontend.h — command-line sessions of the front end (libYulioRT_mi355x.so).
 *
 * The reference renderer executable (devices/renderer/renderer.cpp:1406-1474 embree::main,
 * :974-1403 parseCommandLine, :508-905 outputMode) exposed as a C ABI so a host program (or a
 * test) can parse a reference command line / .ecs file once and then render it repeatedly.
 */
#ifndef YRT_FRONTEND_H
#define YRT_FRONTEND_H

#include <stddef.h>
#include <stdint.h>

#include "yrt_device.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct YRTSession_* YRTSession;

/* Parses argv like `rt.exe` (e.g. {"-c","scenes/cornell_box.ecs","-size","256","256"}).
 * dev may be NULL (the session creates and owns one). Returns NULL on error
 * (message via yrtFrontendLastError()). Scene loading (-i) happens here. */
YRT_API YRTSession yrtSessionCreate(YRTDevice dev, int argc, const char** argv);
YRT_API void yrtSessionDestroy(YRTSession s);
YRT_API const char* yrtFrontendLastError(void);

typedef struct YRTSessionInfo {
  YRTDevice device;
  YRTHandle renderer, tonemapper, framebuffer, scene;
  int width, height, stereo, numFrames;
  int framebufferFormat; /* 0 RGB8, 1 RGBA8, 2 RGB_FLOAT32, 3 RGBA_FLOAT32 */
  float gamma;
} YRTSessionInfo;
/* Commits the scene (createScene) on first call and returns the session's handles. */
YRT_API int yrtSessionInfo(YRTSession s, YRTSessionInfo* out);
/* Camera of the session: face -1 = mono pinhole (createCamera), 0..11 = stereo cube faces
 * (renderer.cpp:747-757). The handle is owned by the session. */
YRT_API YRTHandle yrtSessionCamera(YRTSession s, int face);
/* Stereo cube cameras a Collada scene created: 12 per FPR view, in DAELoader order
 * (devices/device/loaders/ColladaLoader.cpp:402-505). */
YRT_API int yrtSessionNumSceneCameras(YRTSession s);
YRT_API YRTHandle yrtSessionSceneCamera(YRTSession s, int i);
/* One FPR face of scene camera i (renderer.cpp:548-576): faceCamera primitives re-oriented
 * toward the camera origin, scene re-committed, frame rendered; returns the mapped
 * framebuffer (format per yrtSessionInfo). */
YRT_API void* yrtSessionRenderSceneCamera(YRTSession s, int i);
/* Renders one frame (mono: face -1) into the session framebuffer and returns the mapped
 * host pointer (format per yrtSessionInfo). */
YRT_API void* yrtSessionRender(YRTSession s, int face);
/* The 12 stereo cube faces (renderer.cpp:742-878) rendered as one job (yrtRenderFrames) into
 * 12 session-owned framebuffers (yrtSessionCubeFrameBuffer(s, face)). Returns 0 / -1. */
YRT_API int yrtSessionRenderCube(YRTSession s);
/* The 12 faces of FPR view `view` (scene cameras 12*view .. 12*view+11) as one job: the
 * faceCamera primitives re-oriented once toward the view's camera origin, the scene
 * re-committed, then yrtRenderFrames (renderer.cpp:543-576 for the whole view). */
YRT_API int yrtSessionRenderSceneCube(YRTSession s, int view);
YRT_API YRTHandle yrtSessionCubeFrameBuffer(YRTSession s, int face);
/* outputMode(-o file): renders and stores the image (.ppm/.pfm/.png; stereo: 12-face strip;
 * with Collada cameras the FPR branch: <dir>/<name>_<camera>.jpg per view, file ignored). */
YRT_API int yrtSessionOutput(YRTSession s, const char* file);

/* storeImage (common/image/image.cpp:77-104): .jpg (baseline, quality 1..100, the FreeImage
 * path), .png, .ppm, .pfm. format: 0 RGB8, 1 RGBA8, 2 RGB_FLOAT32, 3 RGBA_FLOAT32; rows top
 * first, `stride` bytes apart. */
YRT_API int yrtStoreImage(const char* file, int width, int height, int format, const void* pixels, size_t stride,
                          int quality);
/* rt.exe main: parse + output; returns process-style exit code. */
YRT_API int yrtMain(int argc, const char** argv);

#ifdef __cplusplus
}
#endif

#endif
