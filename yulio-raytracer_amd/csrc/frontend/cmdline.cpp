// cmdline.cpp — the renderer's command line / .ecs parser and output mode.
//
//   createGlobalObjects        devices/renderer/renderer.cpp:352-369
//   parsePathTracer            :414-442        parseDebugRenderer :393-412
//   parseCommandLine           :974-1403
//   createCamera / createScene :309-345
//   outputMode                 :508-905 (mono and non-FPR stereo branches)
#include <stdio.h>
#include <string.h>
#include <dlfcn.h>
#include <zlib.h>

#include <algorithm>
#include <fstream>
#include <sstream>
#include <stdexcept>

#include "frontend.h"
#include "../common/yrt_sse_rcp.h"

namespace yrtfe {

// AffineSpace3f::lookAtPoint (common/math/affinespace.h:72-77) in the reference's Vector3f
// operations: dot = (x*x + y*y) + z*z (_mm_dp_ps), normalize = a * rsqrt(dot) with the SSE
// rsqrt sequence of common/math/math.h:53-58 (yrt_sse_rcp.h); pinned against the reference's own
// headers by tests/test_ref_pin.py::test_front_end_camera_basis.
yrt_affine look_at(yrt_v3 eye, yrt_v3 point, yrt_v3 up) {
  auto sub = [](yrt_v3 a, yrt_v3 b) { return yrt_v3{a.x - b.x, a.y - b.y, a.z - b.z}; };
  auto cross = [](yrt_v3 a, yrt_v3 b) {
    return yrt_v3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
  };
  auto norm = [](yrt_v3 a) {
    const float r = yrt_ref_rsqrt(a.x * a.x + a.y * a.y + a.z * a.z);
    return yrt_v3{a.x * r, a.y * r, a.z * r};
  };
  const yrt_v3 Z = norm(sub(point, eye));
  const yrt_v3 U = norm(cross(up, Z));
  const yrt_v3 V = norm(cross(Z, U));
  yrt_affine a = {{U.x, U.y, U.z, V.x, V.y, V.z, Z.x, Z.y, Z.z, eye.x, eye.y, eye.z}};
  return a;
}

std::vector<std::string> tokenize_args(int argc, const char** argv) {
  std::vector<std::string> t;
  for (int i = 0; i < argc; ++i) t.push_back(argv[i]);
  return t;
}

// ParseStream over LineCommentFilter(file, "#") (common/lexers)
static std::vector<std::string> tokenize_file(const std::string& file) {
  std::ifstream in(file);
  if (!in) throw std::runtime_error("cannot open file " + file);
  std::vector<std::string> out;
  std::string line;
  while (std::getline(in, line)) {
    const size_t h = line.find('#');
    if (h != std::string::npos) line = line.substr(0, h);
    std::string cur;
    for (char c : line) {
      if (c == ' ' || c == '\t' || c == '\r' || c == '\n') {
        if (!cur.empty()) out.push_back(cur), cur.clear();
      } else if (c == '{' || c == '}' || c == '=') {
        if (!cur.empty()) out.push_back(cur), cur.clear();
        out.push_back(std::string(1, c));
      } else {
        cur += c;
      }
    }
    if (!cur.empty()) out.push_back(cur);
  }
  return out;
}

void RtState::createGlobalObjects() {
  renderer = checkH(dev, yrtNewRenderer(dev, "pathtracer"), "rtNewRenderer");
  if (depth >= 0) check(dev, yrtSetInt1(dev, renderer, "maxDepth", depth), "rtSetInt1");
  check(dev, yrtSetFloat1(dev, renderer, "tMaxShadowRay", tMaxShadowRay), "rtSetFloat1");
  check(dev, yrtSetFloat1(dev, renderer, "tMaxShadowJitter", tMaxShadowJitter), "rtSetFloat1");
  check(dev, yrtSetFloat3(dev, renderer, "up", camUp.x, camUp.y, camUp.z), "rtSetFloat3");
  check(dev, yrtSetInt1(dev, renderer, "sampler.spp", spp), "rtSetInt1");
  check(dev, yrtCommit(dev, renderer), "rtCommit(renderer)");
  tonemapper = checkH(dev, yrtNewToneMapper(dev, "default"), "rtNewToneMapper");
  check(dev, yrtSetFloat1(dev, tonemapper, "gamma", gamma), "rtSetFloat1");
  check(dev, yrtSetBool1(dev, tonemapper, "vignetting", vignetting), "rtSetBool1");
  check(dev, yrtCommit(dev, tonemapper), "rtCommit(tonemapper)");
  frameBuffer = checkH(dev, yrtNewFrameBuffer(dev, format.c_str(), width, height, numBuffers, nullptr), "rtNewFrameBuffer");
}

struct Stream {
  const std::vector<std::string>& t;
  size_t i = 0;
  explicit Stream(const std::vector<std::string>& tk) : t(tk) {}
  std::string peek() const { return i < t.size() ? t[i] : ""; }
  std::string get() { return i < t.size() ? t[i++] : ""; }
  void drop() { i++; }
  float getFloat() {
    const std::string s = get();
    if (s.empty()) throw std::runtime_error("number expected");
    return (float)atof(s.c_str());
  }
  int getInt() {
    const std::string s = get();
    if (s.empty()) throw std::runtime_error("integer expected");
    return atoi(s.c_str());
  }
  yrt_v3 getV3() {
    float x = getFloat(), y = getFloat(), z = getFloat();
    return {x, y, z};
  }
  void force(const char* s) {
    if (get() != s) throw std::runtime_error(std::string("token '") + s + "' expected");
  }
};

void RtState::parseCommandLine(const std::vector<std::string>& tokens, const std::string& path) {
  Stream cin(tokens);
  auto newRendererPathTracer = [&](const char* type) {
    renderer = checkH(dev, yrtNewRenderer(dev, type), "rtNewRenderer");
    if (depth >= 0) check(dev, yrtSetInt1(dev, renderer, "maxDepth", depth), "rtSetInt1");
    if (strcmp(type, "debug") != 0)
      check(dev, yrtSetFloat1(dev, renderer, "tMaxShadowRay", tMaxShadowRay), "rtSetFloat1");
    check(dev, yrtSetInt1(dev, renderer, "sampler.spp", spp), "rtSetInt1");
    if (stopFlag) check(dev, yrtSetStopFlag(dev, renderer, (volatile int*)stopFlag), "stopFlag");
    // parsePathTracer re-applies g_backplate to the new renderer (renderer.cpp:423)
    if (backplate && strcmp(type, "debug") != 0) check(dev, yrtSetImage(dev, renderer, "backplate", backplate), "rtSetImage");
    if (statusCallback)
      check(dev, yrtSetStatusCallback(dev, renderer, (YRTStatusCallback)statusCallback, statusUser), "statusCallback");
  };
  auto addLight = [&](YRTHandle l) {
    check(dev, yrtCommit(dev, l), "rtCommit(light)");
    prims.push_back(checkH(dev, yrtNewLightPrimitive(dev, l, nullptr, nullptr), "rtNewLightPrimitive"));
  };
  while (true) {
    const std::string tag = cin.get();
    if (tag == "") return;
    if (tag == "-c") {
      const std::string file = join_path(path, cin.get());
      parseCommandLine(tokenize_file(file), path_of(file));
    } else if (tag == "--no-logging" || tag == "-profiling") {
    } else if (tag == "-debug") {
      debugging = true;
    } else if (tag == "-i") {
      // rtLoadScene(g_sceneFileName, &g_stereoCubeCameras, g_faceCullingMode) (:1002-1006)
      const std::string file = join_path(path, cin.get());
      sceneFileName = file;
      std::vector<YRTHandle> p;
      if (ext_of(file) == "dae") {
        p = load_dae(*loader, file, faceCullingMode, &stereoCubeCameras);
        loader->images.clear();
        loader->textures.clear();
        // DLL / FPR path: g_sceneScale from the first camera before the options are parsed
        // (renderer.cpp:1453-1456, 1504)
        if (fprCollada && !stereoCubeCameras.empty())
          check(dev, yrtGetFloat1(dev, stereoCubeCameras[0], "sceneScale", &sceneScale), "rtGetFloat1");
      } else {
        p = loader->loadScene(file);
      }
      prims.insert(prims.end(), p.begin(), p.end());
    } else if (tag == "-fprCollada") {
      fprCollada = true;
    } else if (tag == "-trisphere") {
      YRTHandle s = checkH(dev, yrtNewShape(dev, "sphere"), "rtNewShape");
      const yrt_v3 P = cin.getV3();
      check(dev, yrtSetFloat3(dev, s, "P", P.x, P.y, P.z), "rtSetFloat3");
      check(dev, yrtSetFloat1(dev, s, "r", cin.getFloat()), "rtSetFloat1");
      check(dev, yrtSetInt1(dev, s, "numTheta", cin.getInt()), "rtSetInt1");
      check(dev, yrtSetInt1(dev, s, "numPhi", cin.getInt()), "rtSetInt1");
      check(dev, yrtCommit(dev, s), "rtCommit(shape)");
      YRTHandle m = checkH(dev, yrtNewMaterial(dev, "matte"), "rtNewMaterial");
      check(dev, yrtSetFloat3(dev, m, "reflection", 1.0f, 0.0f, 0.0f), "rtSetFloat3");
      check(dev, yrtCommit(dev, m), "rtCommit(material)");
      prims.push_back(checkH(dev, yrtNewShapePrimitive(dev, s, m, nullptr, 0), "rtNewShapePrimitive"));
    } else if (tag == "-ambientlight") {
      YRTHandle l = checkH(dev, yrtNewLight(dev, "ambientlight"), "rtNewLight");
      const yrt_v3 L = cin.getV3();
      check(dev, yrtSetFloat3(dev, l, "L", L.x, L.y, L.z), "rtSetFloat3");
      addLight(l);
    } else if (tag == "-pointlight" || tag == "-masked_pointlight") {
      // renderer.cpp:1035-1059
      YRTHandle l = checkH(dev, yrtNewLight(dev, "pointlight"), "rtNewLight");
      const yrt_v3 P = cin.getV3(), I = cin.getV3();
      check(dev, yrtSetFloat3(dev, l, "P", P.x, P.y, P.z), "rtSetFloat3");
      check(dev, yrtSetFloat3(dev, l, "I", I.x, I.y, I.z), "rtSetFloat3");
      if (tag == "-pointlight") {
        addLight(l);
      } else {
        const int illumMask = cin.getInt(), shadowMask = cin.getInt();
        check(dev, yrtCommit(dev, l), "rtCommit(light)");
        YRTHandle prim = checkH(dev, yrtNewLightPrimitive(dev, l, nullptr, nullptr), "rtNewLightPrimitive");
        check(dev, yrtSetInt1(dev, prim, "illumMask", illumMask), "rtSetInt1");
        check(dev, yrtSetInt1(dev, prim, "shadowMask", shadowMask), "rtSetInt1");
        check(dev, yrtCommit(dev, prim), "rtCommit(primitive)");
        prims.push_back(prim);
      }
    } else if (tag == "-directionallight" || tag == "-dirlight") {
      YRTHandle l = checkH(dev, yrtNewLight(dev, "directionallight"), "rtNewLight");
      const yrt_v3 D = cin.getV3(), E = cin.getV3();
      check(dev, yrtSetFloat3(dev, l, "D", D.x, D.y, D.z), "rtSetFloat3");
      check(dev, yrtSetFloat3(dev, l, "E", E.x, E.y, E.z), "rtSetFloat3");
      addLight(l);
    } else if (tag == "-distantlight") {
      YRTHandle l = checkH(dev, yrtNewLight(dev, "distantlight"), "rtNewLight");
      const yrt_v3 D = cin.getV3(), Lc = cin.getV3();
      check(dev, yrtSetFloat3(dev, l, "D", D.x, D.y, D.z), "rtSetFloat3");
      check(dev, yrtSetFloat3(dev, l, "L", Lc.x, Lc.y, Lc.z), "rtSetFloat3");
      check(dev, yrtSetFloat1(dev, l, "halfAngle", cin.getFloat()), "rtSetFloat1");
      addLight(l);
    } else if (tag == "-spotlight") {
      YRTHandle l = checkH(dev, yrtNewLight(dev, "spotlight"), "rtNewLight");
      const yrt_v3 P = cin.getV3(), D = cin.getV3(), I = cin.getV3();
      const float angleMin = cin.getFloat(), angleMax = cin.getFloat();
      check(dev, yrtSetFloat3(dev, l, "P", P.x, P.y, P.z), "rtSetFloat3");
      check(dev, yrtSetFloat3(dev, l, "D", D.x, D.y, D.z), "rtSetFloat3");
      check(dev, yrtSetFloat3(dev, l, "I", I.x, I.y, I.z), "rtSetFloat3");
      check(dev, yrtSetFloat1(dev, l, "angleMin", angleMin), "rtSetFloat1");
      check(dev, yrtSetFloat1(dev, l, "angleMax", angleMax), "rtSetFloat1");
      addLight(l);
    } else if (tag == "-trianglelight") {
      const yrt_v3 P = cin.getV3(), U = cin.getV3(), V = cin.getV3(), L = cin.getV3();
      YRTHandle l = checkH(dev, yrtNewLight(dev, "trianglelight"), "rtNewLight");
      check(dev, yrtSetFloat3(dev, l, "v0", P.x, P.y, P.z), "rtSetFloat3");
      check(dev, yrtSetFloat3(dev, l, "v1", P.x + U.x, P.y + U.y, P.z + U.z), "rtSetFloat3");
      check(dev, yrtSetFloat3(dev, l, "v2", P.x + V.x, P.y + V.y, P.z + V.z), "rtSetFloat3");
      check(dev, yrtSetFloat3(dev, l, "L", L.x, L.y, L.z), "rtSetFloat3");
      addLight(l);
    } else if (tag == "-quadlight") {
      // renderer.cpp:1118-1140
      const yrt_v3 P = cin.getV3(), U = cin.getV3(), V = cin.getV3(), L = cin.getV3();
      YRTHandle l0 = checkH(dev, yrtNewLight(dev, "trianglelight"), "rtNewLight");
      check(dev, yrtSetFloat3(dev, l0, "v0", P.x + U.x + V.x, P.y + U.y + V.y, P.z + U.z + V.z), "rtSetFloat3");
      check(dev, yrtSetFloat3(dev, l0, "v1", P.x + U.x, P.y + U.y, P.z + U.z), "rtSetFloat3");
      check(dev, yrtSetFloat3(dev, l0, "v2", P.x, P.y, P.z), "rtSetFloat3");
      check(dev, yrtSetFloat3(dev, l0, "L", L.x, L.y, L.z), "rtSetFloat3");
      addLight(l0);
      YRTHandle l1 = checkH(dev, yrtNewLight(dev, "trianglelight"), "rtNewLight");
      check(dev, yrtSetFloat3(dev, l1, "v0", P.x + U.x + V.x, P.y + U.y + V.y, P.z + U.z + V.z), "rtSetFloat3");
      check(dev, yrtSetFloat3(dev, l1, "v1", P.x, P.y, P.z), "rtSetFloat3");
      check(dev, yrtSetFloat3(dev, l1, "v2", P.x + V.x, P.y + V.y, P.z + V.z), "rtSetFloat3");
      check(dev, yrtSetFloat3(dev, l1, "L", L.x, L.y, L.z), "rtSetFloat3");
      addLight(l1);
    } else if (tag == "-hdrilight") {
      YRTHandle l = checkH(dev, yrtNewLight(dev, "hdrilight"), "rtNewLight");
      const yrt_v3 L = cin.getV3();
      check(dev, yrtSetFloat3(dev, l, "L", L.x, L.y, L.z), "rtSetFloat3");
      check(dev, yrtSetImage(dev, l, "image", loader->image(path + cin.get())), "rtSetImage");
      addLight(l);
    } else if (tag == "-vp") camPos = cin.getV3();
    else if (tag == "-vi") camLookAt = cin.getV3();
    else if (tag == "-vd") { yrt_v3 d = cin.getV3(); camLookAt = {camPos.x + d.x, camPos.y + d.y, camPos.z + d.z}; }
    else if (tag == "-vu") camUp = cin.getV3();
    else if (tag == "-angle" || tag == "-fov") camFieldOfView = cin.getFloat();
    else if (tag == "-radius") camRadius = cin.getFloat();
    else if (tag == "-stereo") stereo = true;
    else if (tag == "-toeIn") toeIn = true;
    else if (tag == "-waterMark") waterMark = true;
    else if (tag == "-eyeSeparation") eyeSeparation = cin.getFloat();
    else if (tag == "-zeroParallax") zeroParallaxDistance = cin.getFloat();
    else if (tag == "-size") {
      width = cin.getInt();
      height = cin.getInt();
      frameBuffer = checkH(dev, yrtNewFrameBuffer(dev, format.c_str(), width, height, numBuffers, nullptr), "rtNewFrameBuffer");
    } else if (tag == "-jpegQuality") {
      jpegQuality = std::max(1, std::min(100, cin.getInt()));
    } else if (tag == "-framebuffer" || tag == "-fb") {
      format = cin.get();
      frameBuffer = checkH(dev, yrtNewFrameBuffer(dev, format.c_str(), width, height, numBuffers, nullptr), "rtNewFrameBuffer");
    } else if (tag == "-fullscreen" || tag == "-display") {
      if (tag == "-display") outFileName = "";
    } else if (tag == "-refine") cin.getInt();
    else if (tag == "-scene") sceneType = cin.get();
    else if (tag == "-accel") accel = cin.get();
    else if (tag == "-builder") builder = cin.get();
    else if (tag == "-traverser") traverser = cin.get();
    else if (tag == "-renderer") {
      const std::string r = cin.get();
      if (r == "debug") {
        // parseDebugRenderer (renderer.cpp:393-412)
        newRendererPathTracer("debug");
      } else if (r == "pt" || r == "pathtracer") {
        newRendererPathTracer("pathtracer");
      } else {
        throw std::runtime_error("(when parsing -renderer) : unknown renderer: " + r);
      }
      if (cin.peek() == "{") {
        cin.drop();
        while (cin.peek() != "}" && cin.peek() != "") {
          const std::string t = cin.get();
          cin.force("=");
          if (t == "depth") check(dev, yrtSetInt1(dev, renderer, "maxDepth", cin.getInt()), "rtSetInt1");
          else if (t == "tMaxShadowRay" && r != "debug")
            check(dev, yrtSetFloat1(dev, renderer, "tMaxShadowRay", cin.getFloat() * sceneScale), "rtSetFloat1");
          else if (t == "spp" && r != "debug") check(dev, yrtSetInt1(dev, renderer, "sampler.spp", cin.getInt()), "rtSetInt1");
          else if (t == "minContribution" && r != "debug")
            check(dev, yrtSetFloat1(dev, renderer, "minContribution", cin.getFloat()), "rtSetFloat1");
          else if (t == "backplate" && r != "debug")  // renderer.cpp:435
            check(dev, yrtSetImage(dev, renderer, "backplate", loader->image(path + cin.get())), "rtSetImage");
          else cin.get();  // unknown tag (reference prints a warning)
        }
        cin.drop();
      }
      check(dev, yrtCommit(dev, renderer), "rtCommit(renderer)");
    } else if (tag == "-gamma") {
      gamma = cin.getFloat();
      check(dev, yrtSetFloat1(dev, tonemapper, "gamma", gamma), "rtSetFloat1");
      check(dev, yrtCommit(dev, tonemapper), "rtCommit(tonemapper)");
    } else if (tag == "-vignetting") {
      vignetting = cin.getInt() != 0;
      check(dev, yrtSetBool1(dev, tonemapper, "vignetting", vignetting), "rtSetBool1");
      check(dev, yrtCommit(dev, tonemapper), "rtCommit(tonemapper)");
    } else if (tag == "-depth") {
      depth = cin.getInt();
      check(dev, yrtSetInt1(dev, renderer, "maxDepth", depth), "rtSetInt1");
      check(dev, yrtCommit(dev, renderer), "rtCommit(renderer)");
    } else if (tag == "-tMaxShadowRay") {
      tMaxShadowRay = cin.getFloat() * sceneScale;
      check(dev, yrtSetFloat1(dev, renderer, "tMaxShadowRay", tMaxShadowRay), "rtSetFloat1");
      check(dev, yrtCommit(dev, renderer), "rtCommit(renderer)");
    } else if (tag == "-tMaxShadowJitter") {
      tMaxShadowJitter = cin.getFloat();
      check(dev, yrtSetFloat1(dev, renderer, "tMaxShadowJitter", tMaxShadowJitter), "rtSetFloat1");
      check(dev, yrtCommit(dev, renderer), "rtCommit(renderer)");
    } else if (tag == "-faceCullingMode") {
      faceCullingMode = cin.get();
    } else if (tag == "-spp") {
      spp = cin.getInt();
      check(dev, yrtSetInt1(dev, renderer, "sampler.spp", spp), "rtSetInt1");
      check(dev, yrtCommit(dev, renderer), "rtCommit(renderer)");
    } else if (tag == "-backplate") {
      // renderer.cpp:1259-1263
      backplate = loader->image(path + cin.get());
      check(dev, yrtSetImage(dev, renderer, "backplate", backplate), "rtSetImage");
      check(dev, yrtCommit(dev, renderer), "rtCommit(renderer)");
    } else if (tag == "-frames") {
      numFrames = cin.getInt();
    } else if (tag == "-o") {
      const std::string fn = cin.get();
      outFileName = (!fn.empty() && fn[0] == '/') ? fn : path + fn;
    } else if (tag == "-threads" || tag == "-device" || tag == "-rtcore") {
      cin.get();
    } else if (tag == "-regression") {
      throw std::runtime_error("-regression (interactive GLUT mode) is out of scope");
    } else {
      throw std::runtime_error("unknown command line parameter: " + tag);
    }
  }
}

// createCamera (renderer.cpp:309-332) / stereo faces (renderer.cpp:747-757)
YRTHandle RtState::createCamera(int face) {
  auto it = cameras.find(face);
  if (it != cameras.end()) return it->second;
  const yrt_affine space = look_at(camPos, camLookAt, camUp);
  YRTHandle c;
  if (face < 0) {
    // pinhole, or the depth-of-field camera when -radius != 0 (renderer.cpp:312-331)
    c = checkH(dev, yrtNewCamera(dev, camRadius == 0.0f ? "pinhole" : "depthoffield"), "rtNewCamera");
    check(dev, yrtSetTransform(dev, c, "local2world", space.v), "rtSetTransform");
    check(dev, yrtSetFloat1(dev, c, "angle", camFieldOfView), "rtSetFloat1");
    check(dev, yrtSetFloat1(dev, c, "aspectRatio", float(width) / float(height)), "rtSetFloat1");
    if (camRadius != 0.0f) {
      const float dx = camLookAt.x - camPos.x, dy = camLookAt.y - camPos.y, dz = camLookAt.z - camPos.z;
      check(dev, yrtSetFloat1(dev, c, "lensRadius", camRadius), "rtSetFloat1");
      check(dev, yrtSetFloat1(dev, c, "focalDistance", sqrtf(dx * dx + dy * dy + dz * dz)), "rtSetFloat1");
    }
  } else {
    c = checkH(dev, yrtNewCamera(dev, "stereo"), "rtNewCamera");
    check(dev, yrtSetTransform(dev, c, "local2world", space.v), "rtSetTransform");
    check(dev, yrtSetInt1(dev, c, "cubeFaceIndex", face), "rtSetInt1");
    check(dev, yrtSetFloat3(dev, c, "origin", camPos.x, camPos.y, camPos.z), "rtSetFloat3");
    check(dev, yrtSetFloat3(dev, c, "lookAt", camLookAt.x, camLookAt.y, camLookAt.z), "rtSetFloat3");
    check(dev, yrtSetFloat3(dev, c, "up", camUp.x, camUp.y, camUp.z), "rtSetFloat3");
    check(dev, yrtSetBool1(dev, c, "toeIn", toeIn), "rtSetBool1");
  }
  check(dev, yrtCommit(dev, c), "rtCommit(camera)");
  return cameras[face] = c;
}

// createScene (renderer.cpp:335-345)
YRTHandle RtState::createScene() {
  if (scene) return scene;
  scene = checkH(dev, yrtNewScene(dev, sceneType.c_str()), "rtNewScene");
  check(dev, yrtSetString(dev, scene, "accel", accel.c_str()), "rtSetString");
  check(dev, yrtSetString(dev, scene, "builder", builder.c_str()), "rtSetString");
  check(dev, yrtSetString(dev, scene, "traverser", traverser.c_str()), "rtSetString");
  for (size_t i = 0; i < prims.size(); i++) check(dev, yrtSetPrimitive(dev, scene, i, prims[i]), "rtSetPrimitive");
  check(dev, yrtCommit(dev, scene), "rtCommit(scene)");
  return scene;
}

static int fb_format(const std::string& f) {
  if (f == "RGB8") return 0;
  if (f == "RGBA8") return 1;
  if (f == "RGB_FLOAT32") return 2;
  return 3;
}
static size_t fb_stride(int fmt, int w) {
  switch (fmt) {
    case 0: return (3 * (size_t)w + 3) / 4 * 4;
    case 1: return 4 * (size_t)w;
    case 2: return 12 * (size_t)w;
    default: return 16 * (size_t)w;
  }
}

// ---------------------------------------------------------------- image store
static void write_png(const std::string& file, int w, int h, const std::vector<uint8_t>& rgb) {
  std::vector<uint8_t> raw;
  raw.reserve((size_t)(3 * w + 1) * h);
  for (int y = 0; y < h; ++y) {
    raw.push_back(0);
    raw.insert(raw.end(), rgb.begin() + (size_t)y * w * 3, rgb.begin() + (size_t)(y + 1) * w * 3);
  }
  uLongf zl = compressBound(raw.size());
  std::vector<uint8_t> z(zl);
  compress2(z.data(), &zl, raw.data(), raw.size(), 6);
  z.resize(zl);
  FILE* f = fopen(file.c_str(), "wb");
  if (!f) throw std::runtime_error("cannot write " + file);
  auto be = [](uint32_t v, uint8_t* o) { o[0] = v >> 24; o[1] = v >> 16; o[2] = v >> 8; o[3] = v; };
  auto chunk = [&](const char* t, const std::vector<uint8_t>& d) {
    uint8_t b[4];
    be((uint32_t)d.size(), b);
    fwrite(b, 1, 4, f);
    fwrite(t, 1, 4, f);
    if (!d.empty()) fwrite(d.data(), 1, d.size(), f);
    uLong c = crc32(0, (const Bytef*)t, 4);
    if (!d.empty()) c = crc32(c, d.data(), d.size());
    be((uint32_t)c, b);
    fwrite(b, 1, 4, f);
  };
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  fwrite(sig, 1, 8, f);
  std::vector<uint8_t> ihdr(13, 0);
  be(w, &ihdr[0]);
  be(h, &ihdr[4]);
  ihdr[8] = 8;
  ihdr[9] = 2;
  chunk("IHDR", ihdr);
  chunk("IDAT", z);
  chunk("IEND", {});
  fclose(f);
}

// Image3c/Image4c -> Color4 -> byte round trip of the reference's image classes
// (common/math/color_scalar.h:45-60): byte * one_over_255, then char(clamp(c) * 255): a byte
// can lose 1 LSB.
static inline uint8_t requant(uint8_t b) {
  const float c = b * (1.0f / 255.0f);
  return (uint8_t)(std::max(0.0f, std::min(c, 1.0f)) * 255.0f);
}

// 8-bit RGB, top row first, as the reference's storers read it through Image::get.
static std::vector<uint8_t> to_rgb8(int w, int h, int fmt, const void* px, size_t stride, bool viaColor4) {
  std::vector<uint8_t> rgb((size_t)w * h * 3);
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      const uint8_t* row = (const uint8_t*)px + (size_t)y * stride;
      uint8_t* o = &rgb[((size_t)y * w + x) * 3];
      if (fmt >= 2) {
        const float* p = (const float*)row + x * (fmt == 2 ? 3 : 4);
        for (int k = 0; k < 3; ++k) o[k] = (uint8_t)(std::max(0.0f, std::min(p[k], 1.0f)) * 255.0f);
      } else {
        const uint8_t* p = row + x * (fmt == 0 ? 3 : 4);
        for (int k = 0; k < 3; ++k) o[k] = viaColor4 ? requant(p[k]) : p[k];
      }
    }
  return rgb;
}

void store_image(const std::string& file, int w, int h, int fmt, const void* px, size_t stride, int quality) {
  const std::string ext = ext_of(file);
  if (ext == "pfm") {
    FILE* f = fopen(file.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot write " + file);
    fprintf(f, "PF\n%d %d\n-1\n", w, h);
    for (int y = h - 1; y >= 0; --y)
      for (int x = 0; x < w; ++x) {
        float c[3];
        const uint8_t* row = (const uint8_t*)px + (size_t)y * stride;
        if (fmt >= 2) {
          const float* p = (const float*)row + x * (fmt == 2 ? 3 : 4);
          c[0] = p[0]; c[1] = p[1]; c[2] = p[2];
        } else {
          const uint8_t* p = row + x * (fmt == 0 ? 3 : 4);
          for (int k = 0; k < 3; ++k) c[k] = p[k] / 255.0f;
        }
        fwrite(c, 4, 3, f);
      }
    fclose(f);
    return;
  }
  if (ext == "jpg" || ext == "jpeg") {
    // storeFreeImage (common/image/freeimage.cpp:191-232): 24-bit, (uchar)(clamp(c)*255)
    const std::vector<uint8_t> rgb = to_rgb8(w, h, fmt, px, stride, true);
    const std::vector<uint8_t> jpg = encode_jpeg(rgb.data(), w, h, (size_t)w * 3, quality);
    FILE* f = fopen(file.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot write " + file);
    fwrite(jpg.data(), 1, jpg.size(), f);
    fclose(f);
    return;
  }
  const std::vector<uint8_t> rgb = to_rgb8(w, h, fmt, px, stride, false);
  if (ext == "ppm") {
    FILE* f = fopen(file.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot write " + file);
    fprintf(f, "P6\n%d %d\n255\n", w, h);
    fwrite(rgb.data(), 1, rgb.size(), f);
    fclose(f);
  } else if (ext == "png") {
    write_png(file, w, h, rgb);
  } else {
    throw std::runtime_error("image format ." + ext + " not supported (use .jpg, .png, .ppm or .pfm)");
  }
}

// Yulio watermark (renderer.cpp:51-97): the 100x100 RGBA resource, loaded through
// loadFreeImage(data, size, 1, flipVertical, flipHorizontal) into an Image4c.
static bool load_watermark(std::vector<uint8_t>& rgba, int& w, int& h) {
  Dl_info info;
  if (!dladdr((void*)&load_watermark, &info) || !info.dli_fname) return false;
  std::string dir = path_of(info.dli_fname);
  const std::string file = dir + "../resources/watermarkwhitetrasp_100x100.png";
  int c = 0;
  if (yrtDebugDecodeImage(file.c_str(), &w, &h, &c, nullptr, 0) != 0 || c != 4) return false;
  std::vector<uint8_t> px((size_t)w * h * 4);
  if (yrtDebugDecodeImage(file.c_str(), &w, &h, &c, px.data(), px.size()) != 0) return false;
  // decoded rows are top-first; FreeImage's DIB is bottom-up, so its FlipVertical yields
  // top-first rows; FlipHorizontal mirrors the columns. Bytes go through b/255.0f and the
  // Image4c store char(clamp(c)*255).
  rgba.resize(px.size());
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x)
      for (int k = 0; k < 4; ++k) {
        const float f = (float)px[((size_t)y * w + (w - 1 - x)) * 4 + k] / 255.0f;
        rgba[((size_t)y * w + x) * 4 + k] = (uint8_t)(std::max(0.0f, std::min(f, 1.0f)) * 255.0f);
      }
  return true;
}

// Watermark blend (renderer.cpp:637-655) into an RGB8 / RGBA8 face (Image3c / Image4c).
static void apply_watermark(uint8_t* img, int width, int height, int fmt, size_t stride) {
  static std::vector<uint8_t> wm;
  static int ww = 0, wh = 0;
  static bool loaded = false, ok = false;
  if (!loaded) {
    ok = load_watermark(wm, ww, wh);
    loaded = true;
  }
  if (!ok || fmt >= 2) return;
  const int bpp = fmt == 0 ? 3 : 4;
  const float one_over_255 = 1.0f / 255.0f;
  for (int y = 0; y < wh; ++y)
    for (int x = 0; x < ww; ++x) {
      const uint8_t* w4 = &wm[((size_t)y * ww + x) * 4];
      const float wc[4] = {w4[0] * one_over_255, w4[1] * one_over_255, w4[2] * one_over_255, w4[3] * one_over_255};
      const int xDst = (int)(x + (width - ww) * .5f);
      const int yDst = (int)(y + (height - wh) * .5f);
      if (xDst < 0 || xDst >= width || yDst < 0 || yDst >= height) continue;
      uint8_t* p = img + (size_t)yDst * stride + (size_t)xDst * bpp;
      for (int k = 0; k < 3; ++k) {
        const float ic = p[k] * one_over_255;
        const float b = (1.f - wc[3]) * ic + wc[3] * wc[k];
        p[k] = (uint8_t)(std::max(0.0f, std::min(b, 1.0f)) * 255.0f);
      }
    }
}

std::vector<uint8_t> assemble_strip(const std::vector<std::vector<uint8_t>>& faces, int width, int height, int fmt,
                                    size_t stride);

void RtState::renderFprFace(size_t i) {
  YRTHandle sc = createScene();
  YRTHandle cam = stereoCubeCameras.at(i);
  // update the dynamic geometry (self-aligning instances) for this view (:550-559)
  float camPos[3], up[3] = {camUp.x, camUp.y, camUp.z};
  check(dev, yrtGetFloat3(dev, cam, "origin", &camPos[0], &camPos[1], &camPos[2]), "rtGetFloat3");
  for (size_t j = 0; j < prims.size(); ++j)
    check(dev, yrtUpdatePrimitive(dev, sc, j, prims[j], camPos, up), "rtUpdatePrimitive");
  check(dev, yrtCommit(dev, sc), "rtCommit(scene)");
  if (toeIn) {  // :569-574
    check(dev, yrtSetBool1(dev, cam, "toeIn", 1), "rtSetBool1");
    check(dev, yrtCommit(dev, cam), "rtCommit(camera)");
  }
  check(dev, yrtRenderFrame(dev, renderer, cam, sc, tonemapper, frameBuffer, 0), "rtRenderFrame");
  for (int j = 0; j < numBuffers; ++j) check(dev, yrtSwapBuffers(dev, frameBuffer), "rtSwapBuffers");
}

void RtState::renderCube(const std::vector<YRTHandle>& cams) {
  if (cubeFrameBuffers.size() != cams.size() || cubeWidth != width || cubeHeight != height || cubeFormat != format) {
    for (YRTHandle f : cubeFrameBuffers) yrtDecRef(dev, f);
    cubeFrameBuffers.clear();
    for (size_t k = 0; k < cams.size(); ++k)
      cubeFrameBuffers.push_back(
          checkH(dev, yrtNewFrameBuffer(dev, format.c_str(), width, height, 1, nullptr), "rtNewFrameBuffer"));
    cubeWidth = width;
    cubeHeight = height;
    cubeFormat = format;
  }
  YRTHandle sc = createScene();
  check(dev, yrtRenderFrames(dev, renderer, cams.data(), (int)cams.size(), sc, tonemapper, cubeFrameBuffers.data(), 0),
        "rtRenderFrames");
}

std::vector<uint8_t> RtState::cubeFace(int k) {
  const size_t bytes = fb_stride(fb_format(format), width) * height;
  const uint8_t* p = (const uint8_t*)yrtMapFrameBuffer(dev, cubeFrameBuffers.at(k), -1);
  if (!p) throw std::runtime_error(std::string("rtMapFrameBuffer: ") + yrtGetLastError(dev));
  std::vector<uint8_t> out(p, p + bytes);
  check(dev, yrtUnmapFrameBuffer(dev, cubeFrameBuffers.at(k), -1), "rtUnmapFrameBuffer");
  return out;
}

bool RtState::renderFprView(size_t v) {
  if (12 * v + 12 > stereoCubeCameras.size()) throw std::runtime_error("FPR view index out of range");
  float o0[3], o[3];
  check(dev, yrtGetFloat3(dev, stereoCubeCameras[12 * v], "origin", &o0[0], &o0[1], &o0[2]), "rtGetFloat3");
  for (int k = 1; k < 12; ++k) {
    check(dev, yrtGetFloat3(dev, stereoCubeCameras[12 * v + k], "origin", &o[0], &o[1], &o[2]), "rtGetFloat3");
    if (memcmp(o, o0, sizeof(o)) != 0) return false;
  }
  YRTHandle sc = createScene();
  float up[3] = {camUp.x, camUp.y, camUp.z};
  for (size_t j = 0; j < prims.size(); ++j)
    check(dev, yrtUpdatePrimitive(dev, sc, j, prims[j], o0, up), "rtUpdatePrimitive");
  check(dev, yrtCommit(dev, sc), "rtCommit(scene)");
  std::vector<YRTHandle> cams(stereoCubeCameras.begin() + 12 * v, stereoCubeCameras.begin() + 12 * v + 12);
  if (toeIn)  // :569-574
    for (YRTHandle c : cams) {
      check(dev, yrtSetBool1(dev, c, "toeIn", 1), "rtSetBool1");
      check(dev, yrtCommit(dev, c), "rtCommit(camera)");
    }
  renderCube(cams);
  return true;
}

void RtState::fprOutputMode() {
  const size_t numViews = stereoCubeCameras.size();
  if (onStage) onStage(0, (int)numViews);
  // the cube faces must be square (:528-532)
  if (width != height) {
    width = height = std::max(width, height);
    frameBuffer = checkH(dev, yrtNewFrameBuffer(dev, format.c_str(), width, height, numBuffers, nullptr), "rtNewFrameBuffer");
  }
  const int fmt = fb_format(format);
  const size_t stride = fb_stride(fmt, width);
  static const char* kFaceName[6] = {"front", "right", "back", "left", "top", "bottom"};
  // <path>\<name>_<camera>... (:584-586, 719-720)
  const std::string dir = path_of(sceneFileName);
  std::string base = sceneFileName.substr(dir.size());
  base = base.substr(0, base.find_last_of('.'));
  std::vector<std::vector<uint8_t>> faces;
  // whole views as one job each (renderFprView) unless YRT_FACE_LOOP=1 asks for the
  // reference's face-by-face loop (same images)
  const bool faceLoop = getenv("YRT_FACE_LOOP") != nullptr;
  bool viewDone = false;
  for (size_t i = 0; i < numViews && !(stopFlag && stopFlag->load()); ++i) {
    const size_t cubeFaceIndex = i % 12;
    if (cubeFaceIndex == 0) {
      faces.clear();
      viewDone = false;
      if (!faceLoop && i + 12 <= numViews) {
        if (onStage) onStage((int)(i / 12), (int)(numViews / 12));
        viewDone = renderFprView(i / 12);
        if (stopFlag && stopFlag->load()) break;
      }
    }
    if (!viewDone && onStage) onStage((int)i, (int)numViews);
    char nameBuf[1024];
    int n = yrtGetString(dev, stereoCubeCameras[i], "name", nameBuf, sizeof(nameBuf));
    const std::string cameraName = n >= 0 ? std::string(nameBuf) : std::string();
    if (viewDone) {
      faces.push_back(cubeFace((int)cubeFaceIndex));
    } else {
      renderFprFace(i);
      const uint8_t* p = (const uint8_t*)yrtMapFrameBuffer(dev, frameBuffer, -1);
      faces.emplace_back(p, p + stride * height);
      check(dev, yrtUnmapFrameBuffer(dev, frameBuffer, -1), "rtUnmapFrameBuffer");
    }
    if (waterMark && (cubeFaceIndex % 6) < 4) apply_watermark(faces.back().data(), width, height, fmt, stride);
    const std::string faceFile = dir + base + "_" + cameraName + "_" + kFaceName[cubeFaceIndex % 6] + "_image_" +
                                 (cubeFaceIndex < 6 ? "left" : "right") + ".jpg";
    if (debugging) {
      store_image(faceFile, width, height, fmt, faces.back().data(), stride, jpegQuality);
      savedFiles.push_back(faceFile);
    }
    if (cubeFaceIndex == 11) {
      std::vector<uint8_t> strip = assemble_strip(faces, width, height, fmt, stride);
      const int bpp = fmt == 0 ? 3 : fmt == 1 ? 4 : fmt == 2 ? 12 : 16;
      store_image(dir + base + "_" + cameraName + ".jpg", width * 12, height, fmt, strip.data(),
                  (size_t)bpp * width * 12, jpegQuality);
      // the reference records the last face's file name here, not the strip's (:716), so
      // StopRT(false) never removes a finished strip
      savedFiles.push_back(faceFile);
    }
  }
}

// strip = right eye first, each eye L,R,U,D,B,F (renderer.cpp:663-715, 820-877); bytes go
// through Color4 (finalImage->set(x, y, face->get(x, y)))
std::vector<uint8_t> assemble_strip(const std::vector<std::vector<uint8_t>>& faces, int width, int height, int fmt,
                                    size_t stride) {
  const int bpp = fmt == 0 ? 3 : fmt == 1 ? 4 : fmt == 2 ? 12 : 16;
  const size_t sstride = (size_t)bpp * width * 12;
  std::vector<uint8_t> strip(sstride * height);
  static const int seg2face[6] = {3, 1, 4, 5, 2, 0};
  for (int y = 0; y < height; ++y)
    for (int seg = 0; seg < 12; ++seg) {
      const int eye = seg / 6 == 0 ? 1 : 0;
      const int face = 6 * eye + seg2face[seg % 6];
      uint8_t* dst = &strip[(size_t)y * sstride + (size_t)seg * width * bpp];
      const uint8_t* src = &faces[face][(size_t)y * stride];
      memcpy(dst, src, (size_t)width * bpp);
      if (fmt < 2)
        for (int k = 0; k < width * bpp; ++k)
          if (fmt == 0 || (k & 3) != 3) dst[k] = requant(dst[k]);
    }
  return strip;
}

void RtState::outputMode(const std::string& fileName, std::vector<uint8_t>* outImage) {
  if (!renderer) throw std::runtime_error("no renderer set");
  if (stereo && !stereoCubeCameras.empty()) {
    fprOutputMode();
    return;
  }
  const int fmt = fb_format(format);
  const size_t stride = fb_stride(fmt, width);
  YRTHandle sc = createScene();
  if (stereo) {
    if (onStage) onStage(0, 12);
    // stereo branch (renderer.cpp:742-878; DLL/FPR variant :543-737 adds the watermark):
    // 12 faces, strip = right eye first, each eye L,R,U,D,B,F
    std::vector<std::vector<uint8_t>> faces(12);
    static const char* kFaceName[6] = {"front", "right", "back", "left", "top", "bottom"};
    const std::string base = fileName.empty() ? std::string() : fileName.substr(0, fileName.find_last_of('.'));
    // the 12 faces as one job (the scene does not change between them in this branch);
    // YRT_FACE_LOOP=1: the reference's face-by-face loop (same images)
    const bool faceLoop = getenv("YRT_FACE_LOOP") != nullptr;
    if (!faceLoop) {
      std::vector<YRTHandle> cams;
      for (int i = 0; i < 12; ++i) cams.push_back(createCamera(i));
      if (onStage) onStage(0, 1);
      renderCube(cams);
      if (stopFlag && stopFlag->load()) return;
    }
    for (int i = 0; i < 12; ++i) {
      if (faceLoop) {
        if (onStage) onStage(i, 12);
        YRTHandle cam = createCamera(i);
        check(dev, yrtRenderFrame(dev, renderer, cam, sc, tonemapper, frameBuffer, 0), "rtRenderFrame");
        for (int j = 0; j < numBuffers; ++j) check(dev, yrtSwapBuffers(dev, frameBuffer), "rtSwapBuffers");
        const uint8_t* p = (const uint8_t*)yrtMapFrameBuffer(dev, frameBuffer, -1);
        faces[i].assign(p, p + stride * height);
        check(dev, yrtUnmapFrameBuffer(dev, frameBuffer, -1), "rtUnmapFrameBuffer");
      } else {
        faces[i] = cubeFace(i);
      }
      // only the front, back and side faces carry the watermark (renderer.cpp:636-637)
      if (fprOutput && waterMark && (i % 6) < 4) apply_watermark(faces[i].data(), width, height, fmt, stride);
      if (debugging && !fileName.empty()) {
        // <name>_<face>_image_<eye>.<ext> (renderer.cpp:763-799; FPR inserts the camera name)
        const std::string faceFile = base + "_" + kFaceName[i % 6] + "_image_" + (i < 6 ? "left" : "right") +
                                     (fprOutput ? std::string(".jpg") : "." + ext_of(fileName));
        store_image(faceFile, width, height, fmt, faces[i].data(), stride, jpegQuality);
        savedFiles.push_back(faceFile);
      }
      if (stopFlag && stopFlag->load()) return;
    }
    const int bpp = fmt == 0 ? 3 : fmt == 1 ? 4 : fmt == 2 ? 12 : 16;
    const size_t sstride = (size_t)bpp * width * 12;
    std::vector<uint8_t> strip = assemble_strip(faces, width, height, fmt, stride);
    if (!fileName.empty()) {
      store_image(fileName, width * 12, height, fmt, strip.data(), sstride, jpegQuality);
      savedFiles.push_back(fileName);
    }
    if (outImage) *outImage = strip;
  } else {
    YRTHandle cam = createCamera(-1);
    check(dev, yrtSetInt1(dev, renderer, "showprogress", 1), "rtSetInt1");
    check(dev, yrtCommit(dev, renderer), "rtCommit(renderer)");
    for (int i = 0; i < numFrames; i++)
      check(dev, yrtRenderFrame(dev, renderer, cam, sc, tonemapper, frameBuffer, 0), "rtRenderFrame");
    for (int i = 0; i < numBuffers; i++) check(dev, yrtSwapBuffers(dev, frameBuffer), "rtSwapBuffers");
    const uint8_t* p = (const uint8_t*)yrtMapFrameBuffer(dev, frameBuffer, -1);
    if (!fileName.empty()) {
      store_image(fileName, width, height, fmt, p, stride, jpegQuality);
      savedFiles.push_back(fileName);
    }
    if (outImage) outImage->assign(p, p + stride * height);
    check(dev, yrtUnmapFrameBuffer(dev, frameBuffer, -1), "rtUnmapFrameBuffer");
  }
}

}  // namespace yrtfe
