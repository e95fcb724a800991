/* YulioRT.h — asynchronous render API of the front-end library (libYulioRT_mi355x.so).
 *
 * Same entry points, enums, struct layout and defaults as the reference DLL interface
 * devices/renderer/YulioRT.h:1-57 (StartRT/WaitRT/StopRT/GetLastErrorRT/GetCurrentStatusRT),
 * rendering on the MI355X device plugin instead of device_singleray + Embree.
 * Semantics (devices/renderer/renderer.cpp:1483-1657):
 *   - one render at a time; StartRT returns after spawning the worker thread;
 *   - WaitRT joins it; StopRT(keepResults) requests a cooperative stop and joins;
 *   - errors are sticky in the status tracker (GetLastErrorRT / GetCurrentStatusRT.lastError).
 * Input: a Collada .dae goes through this build's own Collada loader with the Yulio semantics
 * of devices/device/loaders/ColladaLoader.cpp (FPR cameras YULIO_FPR_VIEW_*, faceCamera meshes
 * YULIO_CAMERA_ALIGNED_*) and the FPR stereo loop (renderer.cpp:543-737); a file the loader
 * rejects or one without FPR cameras reports InvalidColladaFormat. Extension:
 * StartRT also accepts .ecs command files and .xml/.obj scenes, rendered as a stereo cube strip
 * like the reference's non-FPR branch.
 */
#ifndef YULIO_RT_H
#define YULIO_RT_H

#ifdef __cplusplus
extern "C" {
#endif

#define YULIO_DLL_EXPORT __attribute__((visibility("default")))

typedef enum ErrorCodeRT {
  NoError = 0,
  RenderingIsInProgress,
  MissingColladaFile,
  InvalidColladaFormat,
  UnitializedRenderer,
  FailedToPopulateStatus,
  UnknownError = 1000
} ErrorCodeRT;

typedef enum StateRT { Inactive, Initialiazing, Rendering, Stopped, Done } StateRT;

typedef struct StatusRT {
  StateRT state;
  float progress; /* [0,1] */
  ErrorCodeRT lastError;
} StatusRT;

typedef struct ParamsRT {
#ifdef __cplusplus
  const char* renderer = "pathtracer";
  int size = 1536;
  int depth = 10;
  float tMaxShadowRay = 120.f;
  int spp = 256;
  float ambientlight[3] = {.83f, .95f, .98f};
  float eyeSeparation = 2.5f;
  bool toeIn = true;
  float zeroParallax = 75.f;
  int jpegQuality = 90;
  bool debug = false;
  int threadsPriority = 0;
  bool waterMark = false;
  const char* faceCullingMode = "default";
#else
  const char* renderer;
  int size;
  int depth;
  float tMaxShadowRay;
  int spp;
  float ambientlight[3];
  float eyeSeparation;
  _Bool toeIn;
  float zeroParallax;
  int jpegQuality;
  _Bool debug;
  int threadsPriority;
  _Bool waterMark;
  const char* faceCullingMode;
#endif
} ParamsRT;

/* C callers: fills the C++ default member initializers above. */
YULIO_DLL_EXPORT void InitParamsRT(ParamsRT* params);

#ifdef __cplusplus
YULIO_DLL_EXPORT bool StartRT(const char* colladaFile, const ParamsRT* params);
YULIO_DLL_EXPORT bool WaitRT();
YULIO_DLL_EXPORT bool StopRT(bool keepResults);
#else
YULIO_DLL_EXPORT _Bool StartRT(const char* colladaFile, const ParamsRT* params);
YULIO_DLL_EXPORT _Bool WaitRT(void);
YULIO_DLL_EXPORT _Bool StopRT(_Bool keepResults);
#endif
YULIO_DLL_EXPORT ErrorCodeRT GetLastErrorRT(void);
YULIO_DLL_EXPORT void GetCurrentStatusRT(StatusRT* status);

#ifdef __cplusplus
}
#endif

#endif /* YULIO_RT_H */
