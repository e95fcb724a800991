// yulio_rt.cpp — StartRT/WaitRT/StopRT/GetLastErrorRT/GetCurrentStatusRT and command-line
// sessions (include/YulioRT.h, include/yrt_frontend.h).
//
// Reference: devices/renderer/renderer.cpp:99-233 (YulioStatusTracker), :1483-1657 (DLL API),
// :1406-1474 (main).
#include "../../../include/YulioRT.h"

#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>

#include "../../../include/yrt_frontend.h"
#include "frontend.h"

using namespace yrtfe;

static thread_local std::string g_feError;

struct YRTSession_ {
  RtState st;
};

extern "C" {

const char* yrtFrontendLastError(void) { return g_feError.c_str(); }

static YRTSession session_new(YRTDevice dev, const std::vector<std::string>& args, std::atomic<bool>* stop,
                              void* cb, void* user, const std::string& cwd) {
  auto* s = new YRTSession_();
  RtState& st = s->st;
  try {
    st.dev = dev;
    if (!st.dev) {
      // every visible GPU unless YRT_DEVICES names them (the DLL's numThreads = 0 -> all
      // cores default, renderer.cpp:1599-1601), tiles dealt over them
      const char* e = getenv("YRT_DEVICES");
      const std::string parms = std::string("devices=") + (e && *e ? e : "all");
      st.dev = yrtNewDevice(parms.c_str(), 0, 0, "");
      st.ownsDevice = true;
      if (!st.dev) throw std::runtime_error("cannot create the MI355X device (no HIP device?)");
    }
    st.stopFlag = stop;
    st.statusCallback = cb;
    st.statusUser = user;
    st.loader.reset(new Loader(st.dev));
    st.createGlobalObjects();
    st.parseCommandLine(args, cwd);
    return s;
  } catch (const std::exception& e) {
    g_feError = e.what();
    if (st.ownsDevice && st.dev) yrtDeleteDevice(st.dev);
    delete s;
    return nullptr;
  }
}

YRTSession yrtSessionCreate(YRTDevice dev, int argc, const char** argv) {
  return session_new(dev, tokenize_args(argc, argv), nullptr, nullptr, nullptr, "");
}

void yrtSessionDestroy(YRTSession s) {
  if (!s) return;
  if (s->st.ownsDevice && s->st.dev) yrtDeleteDevice(s->st.dev);
  delete s;
}

int yrtSessionInfo(YRTSession s, YRTSessionInfo* out) {
  try {
    RtState& st = s->st;
    out->device = st.dev;
    out->renderer = st.renderer;
    out->tonemapper = st.tonemapper;
    out->framebuffer = st.frameBuffer;
    out->scene = st.createScene();
    out->width = st.width;
    out->height = st.height;
    out->stereo = st.stereo ? 1 : 0;
    out->numFrames = st.numFrames;
    out->framebufferFormat = st.format == "RGB8" ? 0 : st.format == "RGBA8" ? 1 : st.format == "RGB_FLOAT32" ? 2 : 3;
    out->gamma = st.gamma;
    return 0;
  } catch (const std::exception& e) {
    g_feError = e.what();
    return -1;
  }
}

int yrtSessionNumSceneCameras(YRTSession s) { return (int)s->st.stereoCubeCameras.size(); }

YRTHandle yrtSessionSceneCamera(YRTSession s, int i) {
  if (i < 0 || (size_t)i >= s->st.stereoCubeCameras.size()) {
    g_feError = "scene camera index out of range";
    return nullptr;
  }
  return s->st.stereoCubeCameras[i];
}

void* yrtSessionRenderSceneCamera(YRTSession s, int i) {
  try {
    RtState& st = s->st;
    st.renderFprFace((size_t)i);
    return yrtMapFrameBuffer(st.dev, st.frameBuffer, -1);
  } catch (const std::exception& e) {
    g_feError = e.what();
    return nullptr;
  }
}

int yrtSessionRenderCube(YRTSession s) {
  try {
    RtState& st = s->st;
    std::vector<YRTHandle> cams;
    for (int i = 0; i < 12; ++i) cams.push_back(st.createCamera(i));
    st.renderCube(cams);
    return 0;
  } catch (const std::exception& e) {
    g_feError = e.what();
    return -1;
  }
}

int yrtSessionRenderSceneCube(YRTSession s, int view) {
  try {
    if (view < 0) throw std::runtime_error("FPR view index out of range");
    if (!s->st.renderFprView((size_t)view)) throw std::runtime_error("the view's cameras differ in origin");
    return 0;
  } catch (const std::exception& e) {
    g_feError = e.what();
    return -1;
  }
}

YRTHandle yrtSessionCubeFrameBuffer(YRTSession s, int face) {
  if (face < 0 || (size_t)face >= s->st.cubeFrameBuffers.size()) {
    g_feError = "no cube face framebuffer (render a cube first)";
    return nullptr;
  }
  return s->st.cubeFrameBuffers[face];
}

YRTHandle yrtSessionCamera(YRTSession s, int face) {
  try {
    return s->st.createCamera(face);
  } catch (const std::exception& e) {
    g_feError = e.what();
    return nullptr;
  }
}

void* yrtSessionRender(YRTSession s, int face) {
  try {
    RtState& st = s->st;
    YRTHandle sc = st.createScene();
    YRTHandle cam = st.createCamera(face);
    check(st.dev, yrtRenderFrame(st.dev, st.renderer, cam, sc, st.tonemapper, st.frameBuffer, 0), "rtRenderFrame");
    return yrtMapFrameBuffer(st.dev, st.frameBuffer, -1);
  } catch (const std::exception& e) {
    g_feError = e.what();
    return nullptr;
  }
}

int yrtSessionOutput(YRTSession s, const char* file) {
  try {
    s->st.outputMode(file ? file : s->st.outFileName);
    return 0;
  } catch (const std::exception& e) {
    g_feError = e.what();
    return -1;
  }
}

int yrtStoreImage(const char* file, int width, int height, int format, const void* pixels, size_t stride,
                  int quality) {
  try {
    store_image(file, width, height, format, pixels, stride, quality);
    return 0;
  } catch (const std::exception& e) {
    g_feError = e.what();
    return -1;
  }
}

// embree::main (renderer.cpp:1406-1474)
int yrtMain(int argc, const char** argv) {
  YRTSession s = yrtSessionCreate(nullptr, argc, argv);
  if (!s) {
    fprintf(stderr, "Error: %s\n", yrtFrontendLastError());
    return 1;
  }
  int rc = 0;
  if (!s->st.outFileName.empty()) {
    rc = yrtSessionOutput(s, nullptr);
    if (rc) fprintf(stderr, "Error: %s\n", yrtFrontendLastError());
  } else {
    fprintf(stderr, "display mode is not available (no -o output file given)\n");
    rc = 1;
  }
  yrtSessionDestroy(s);
  return rc ? 1 : 0;
}

}  // extern "C"

// ====================================================================== DLL API
// The entry points are declared extern "C" inside namespace Yulio (include/YulioRT.h), so these
// definitions keep C linkage: the exported symbols are the plain names.
namespace Yulio {

static std::mutex g_trackerMu;
static StatusRT g_status = {Inactive, 0.f, NoError};
static std::atomic<bool> g_running{false}, g_stop{false};
static bool g_keepResults = false;
static std::thread g_worker;

static void tracker_error(ErrorCodeRT e) {
  std::lock_guard<std::mutex> g(g_trackerMu);
  g_status.lastError = e;
}
static void tracker_state(StateRT s) {
  std::lock_guard<std::mutex> g(g_trackerMu);
  g_status.state = s;
  if (s == Stopped || s == Done) g_status.progress = 1.f;
}
static int g_faceIndex = 0, g_numFaces = 1;
static void status_cb(int state, float progress, void*) {
  // stage-weighted progress per face (renderer.cpp:184-193, 231-233)
  std::lock_guard<std::mutex> g(g_trackerMu);
  if (state == 1 && g_numFaces > 0)
    g_status.progress = (float(g_faceIndex) + progress) / float(g_numFaces);
}

void InitParamsRT(ParamsRT* p) {
  ParamsRT d;
  *p = d;
}

bool StartRT(const char* colladaFile, const ParamsRT* params) {
  if (g_running) {
    tracker_error(RenderingIsInProgress);
    return false;
  }
  {
    std::lock_guard<std::mutex> g(g_trackerMu);
    g_status = {Inactive, 0.f, NoError};
  }
  if (!colladaFile) {
    tracker_error(MissingColladaFile);
    return false;
  }
  tracker_state(Initialiazing);
  const std::string fn = colladaFile;
  const std::string ext = ext_of(fn);
  if (ext != "dae" && ext != "ecs" && ext != "xml" && ext != "obj") {
    tracker_error(MissingColladaFile);
    return false;
  }
  ParamsRT cur;
  if (params) cur = *params;
  // argv synthesis (renderer.cpp:1557-1585). A .dae is loaded first, with the culling mode
  // of the parameters and g_sceneScale taken from its cameras (workerThreadRT :1494-1505);
  // .ecs/.xml/.obj scenes (an extension of this build) go through the same command line.
  std::vector<std::string> argv;
  if (ext == "ecs") argv = {"-c", fn};
  else if (ext == "dae")
    argv = {"-fprCollada", "-faceCullingMode", cur.faceCullingMode ? cur.faceCullingMode : "default", "-i", fn};
  else argv = {"-i", fn};
  const char* rend = cur.renderer ? cur.renderer : "pathtracer";
  std::vector<std::string> more = {"-stereo", "-renderer", rend, "-spp", std::to_string(cur.spp), "-size",
                                   std::to_string(cur.size), std::to_string(cur.size), "-depth",
                                   std::to_string(cur.depth), "-jpegQuality", std::to_string(cur.jpegQuality),
                                   "-tMaxShadowRay", std::to_string(cur.tMaxShadowRay), "-ambientlight",
                                   std::to_string(cur.ambientlight[0]), std::to_string(cur.ambientlight[1]),
                                   std::to_string(cur.ambientlight[2]), "-eyeSeparation",
                                   std::to_string(cur.eyeSeparation)};
  if (cur.toeIn) more.push_back("-toeIn");
  if (cur.waterMark) more.push_back("-waterMark");
  more.push_back("-faceCullingMode");
  more.push_back(cur.faceCullingMode ? cur.faceCullingMode : "default");
  more.push_back("-zeroParallax");
  more.push_back(std::to_string(cur.zeroParallax));
  if (cur.debug) more.push_back("-debug");
  argv.insert(argv.end(), more.begin(), more.end());
  // output: <dir>/<name>_<camera>.jpg next to the input (renderer.cpp:719-720); scenes
  // without Collada cameras use the camera name "cubemap"
  const std::string base = fn.substr(0, fn.find_last_of('.'));
  const std::string out = base + "_cubemap.jpg";
  g_stop = false;
  g_running = true;
  g_worker = std::thread([argv, out, ext]() {
    YRTSession s = session_new(nullptr, argv, &g_stop, (void*)&status_cb, nullptr, "");
    if (!s) {
      fprintf(stderr, "StartRT: %s\n", yrtFrontendLastError());
      // a Collada file the loader rejects, or one without cameras (:1497-1500)
      tracker_error(ext == "dae" ? InvalidColladaFormat : UnknownError);
      tracker_state(Done);
      return;
    }
    if (ext == "dae" && (s->st.stereoCubeCameras.empty() || s->st.prims.empty())) {
      tracker_error(InvalidColladaFormat);
      yrtSessionDestroy(s);
      tracker_state(Done);
      return;
    }
    tracker_state(Rendering);
    g_faceIndex = 0;
    g_numFaces = s->st.stereo ? 12 : 1;
    s->st.onStage = [](int stage, int numStages) {
      std::lock_guard<std::mutex> g(g_trackerMu);
      g_faceIndex = stage;
      g_numFaces = numStages;
      g_status.progress = float(stage) / float(std::max(1, numStages));
    };
    s->st.fprOutput = true;
    try {
      std::vector<uint8_t> img;
      s->st.outputMode(g_stop ? std::string() : out, &img);
    } catch (const std::exception& e) {
      fprintf(stderr, "StartRT: %s\n", e.what());
      tracker_error(UnknownError);
    }
    const std::vector<std::string> saved = s->st.savedFiles;
    yrtSessionDestroy(s);
    if (g_stop) {
      // StopRT(keepResults = false) removes every image written so far (renderer.cpp:724-731)
      if (!g_keepResults)
        for (const auto& f : saved) remove(f.c_str());
      tracker_state(Stopped);
    } else {
      tracker_state(Done);
    }
  });
  return true;
}

bool WaitRT() {
  if (!g_running) return false;
  if (g_worker.joinable()) g_worker.join();
  g_running = false;
  g_stop = false;
  return true;
}

bool StopRT(bool keepResults) {
  if (!g_running) return false;
  g_keepResults = keepResults;
  g_stop = true;
  if (g_worker.joinable()) g_worker.join();
  g_running = false;
  g_stop = false;
  return true;
}

ErrorCodeRT GetLastErrorRT(void) {
  std::lock_guard<std::mutex> g(g_trackerMu);
  return g_status.lastError;
}

void GetCurrentStatusRT(StatusRT* status) {
  if (!status) return;
  std::lock_guard<std::mutex> g(g_trackerMu);
  *status = g_status;
}

}  // namespace Yulio
