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

#define YULIO_DLL_EXPORT __attribute__((visibility("default")))

#ifdef __cplusplus
/* C++: the declarations live in namespace Yulio as in the reference header (YulioRT.h:9-58),
 * so a caller written against it (rt_test_dll/rt_test_dll.cpp:10 `using namespace Yulio;`, or
 * `Yulio::StartRT(...)`) compiles unchanged. The functions keep C linkage: extern "C" inside a
 * namespace binds the plain symbols StartRT, WaitRT, ... that C and ctypes callers use. */
namespace Yulio {

enum ErrorCodeRT {
  NoError = 0,
  RenderingIsInProgress,
  MissingColladaFile,
  InvalidColladaFormat,
  UnitializedRenderer,
  FailedToPopulateStatus,
  UnknownError = 1000
};

enum StateRT { Inactive, Initialiazing, Rendering, Stopped, Done };

struct StatusRT {
  StateRT state;
  float progress; /* [0,1] */
  ErrorCodeRT lastError;
};

struct ParamsRT {
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
};

extern "C" {
YULIO_DLL_EXPORT bool StartRT(const char* colladaFile, const ParamsRT* params);
YULIO_DLL_EXPORT bool WaitRT();
YULIO_DLL_EXPORT bool StopRT(bool keepResults);
YULIO_DLL_EXPORT ErrorCodeRT GetLastErrorRT();
YULIO_DLL_EXPORT void GetCurrentStatusRT(StatusRT* status);
/* Extension for C callers: fills the default member initializers above. */
YULIO_DLL_EXPORT void InitParamsRT(ParamsRT* params);
}

}  // namespace Yulio

/* Global names for callers of this build that predate the namespace (the same entities): opt-in
 * with -DYULIO_RT_GLOBAL_NAMES, since the reference header keeps them inside namespace Yulio only
 * and names such as Done or NoError would clash with other libraries' globals. */
#if defined(YULIO_RT_GLOBAL_NAMES)
using Yulio::ErrorCodeRT;
using Yulio::NoError;
using Yulio::RenderingIsInProgress;
using Yulio::MissingColladaFile;
using Yulio::InvalidColladaFormat;
using Yulio::UnitializedRenderer;
using Yulio::FailedToPopulateStatus;
using Yulio::UnknownError;
using Yulio::StateRT;
using Yulio::Inactive;
using Yulio::Initialiazing;
using Yulio::Rendering;
using Yulio::Stopped;
using Yulio::Done;
using Yulio::StatusRT;
using Yulio::ParamsRT;
using Yulio::StartRT;
using Yulio::WaitRT;
using Yulio::StopRT;
using Yulio::GetLastErrorRT;
using Yulio::GetCurrentStatusRT;
using Yulio::InitParamsRT;
#endif

#else /* C */

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

/* Same layout as the C++ struct; InitParamsRT fills its defaults. */
typedef struct ParamsRT {
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
} ParamsRT;

YULIO_DLL_EXPORT void InitParamsRT(ParamsRT* params);
YULIO_DLL_EXPORT _Bool StartRT(const char* colladaFile, const ParamsRT* params);
YULIO_DLL_EXPORT _Bool WaitRT(void);
YULIO_DLL_EXPORT _Bool StopRT(_Bool keepResults);
YULIO_DLL_EXPORT ErrorCodeRT GetLastErrorRT(void);
YULIO_DLL_EXPORT void GetCurrentStatusRT(StatusRT* status);

#endif /* __cplusplus */

#endif /* YULIO_RT_H */
