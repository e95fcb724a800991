// loaders.cpp — scene loaders of the front end, driving the device through its C ABI.
//
//   rtLoadImage / rtLoadTexture caches     devices/device/loaders/loaders.cpp:27-66
//   XML scene loader                       devices/device/loaders/xml_loader.cpp:274-620
//   OBJ + MTL loader                       devices/device/loaders/obj_loader.cpp:28-411
// Collada (.dae): collada.cpp.
#include "frontend.h"

#include <ctype.h>
#include <stdio.h>
#include <string.h>

#include <fstream>
#include <map>
#include <sstream>
#include <stdexcept>

namespace yrtfe {

// ---------------------------------------------------------------- helpers
std::string path_of(const std::string& f) {
  const size_t p = f.find_last_of("\\/");
  return p == std::string::npos ? "" : f.substr(0, p + 1);
}
std::string ext_of(const std::string& f) {
  const size_t d = f.find_last_of('.');
  const size_t s = f.find_last_of("\\/");
  if (d == std::string::npos || (s != std::string::npos && d < s)) return "";
  std::string e = f.substr(d + 1);
  for (auto& c : e) c = (char)tolower(c);
  return e;
}
std::string join_path(const std::string& dir, const std::string& f) {
  if (f.empty() || f[0] == '/' || dir.empty()) return f;
  return dir + f;
}

void check(YRTDevice dev, int rc, const char* what) {
  if (rc != 0) throw std::runtime_error(std::string(what) + ": " + yrtGetLastError(dev));
}
YRTHandle checkH(YRTDevice dev, YRTHandle h, const char* what) {
  if (!h) throw std::runtime_error(std::string(what) + ": " + yrtGetLastError(dev));
  return h;
}

YRTHandle Loader::image(const std::string& file) {
  auto it = images.find(file);
  if (it != images.end()) return it->second;
  return images[file] = checkH(dev, yrtNewImageFromFile(dev, file.c_str()), "rtNewImageFromFile");
}

YRTHandle Loader::texture(const std::string& file, const std::string& filtering, bool invert) {
  auto it = textures.find(file);
  if (it != textures.end()) return it->second;
  YRTHandle t = checkH(dev, yrtNewTexture(dev, filtering.c_str()), "rtNewTexture");
  check(dev, yrtSetImage(dev, t, "image", image(file)), "rtSetImage");
  check(dev, yrtSetBool1(dev, t, "invert", invert), "rtSetBool1");
  check(dev, yrtCommit(dev, t), "rtCommit(texture)");
  return textures[file] = t;
}

// ---------------------------------------------------------------- XML parsing
struct XML {
  std::string name;
  std::map<std::string, std::string> parms;
  std::vector<std::shared_ptr<XML>> children;
  std::vector<std::string> body;
  std::string loc;
  std::string parm(const std::string& n) const {
    auto it = parms.find(n);
    return it == parms.end() ? "" : it->second;
  }
  std::shared_ptr<XML> childOpt(const std::string& n) const {
    for (auto& c : children)
      if (c->name == n) return c;
    return nullptr;
  }
  std::shared_ptr<XML> child(const std::string& n) const {
    auto c = childOpt(n);
    if (!c) throw std::runtime_error(loc + ": child " + n + " not found");
    return c;
  }
};
using XMLp = std::shared_ptr<XML>;

struct XmlReader {
  std::string s;
  size_t i = 0;
  std::string file;
  int line() const { return 1 + (int)std::count(s.begin(), s.begin() + std::min(i, s.size()), '\n'); }
  std::string where() const { return file + ":" + std::to_string(line()); }
  void ws() {
    while (i < s.size() && isspace((unsigned char)s[i])) i++;
  }
  void skipMisc() {
    for (;;) {
      ws();
      if (s.compare(i, 4, "<!--") == 0) {
        size_t e = s.find("-->", i);
        i = e == std::string::npos ? s.size() : e + 3;
      } else if (s.compare(i, 2, "<?") == 0) {
        size_t e = s.find("?>", i);
        i = e == std::string::npos ? s.size() : e + 2;
      } else {
        return;
      }
    }
  }
  void tokens(const std::string& text, std::vector<std::string>& out) {
    size_t k = 0;
    while (k < text.size()) {
      while (k < text.size() && isspace((unsigned char)text[k])) k++;
      if (k >= text.size()) break;
      if (text[k] == '"') {
        size_t e = text.find('"', k + 1);
        if (e == std::string::npos) e = text.size();
        out.push_back(text.substr(k + 1, e - k - 1));
        k = e + 1;
      } else {
        size_t e = k;
        while (e < text.size() && !isspace((unsigned char)text[e])) e++;
        out.push_back(text.substr(k, e - k));
        k = e;
      }
    }
  }
  // Every scan is bounded by the end of the text and every malformed construct throws: a
  // truncated or mangled file (a broken comment opener, an attribute without its quote, an
  // end tag without '>') used to wrap an index past std::string::npos back to the start and
  // loop forever (found by the sanitizer driver's mutation fuzz, tools/run_sanitizers.sh).
  XMLp node(int depth = 0) {
    if (depth > 512) throw std::runtime_error(where() + ": elements nested too deeply");
    skipMisc();
    if (i >= s.size() || s[i] != '<') throw std::runtime_error(where() + ": '<' expected");
    auto x = std::make_shared<XML>();
    x->loc = where();
    i++;
    size_t b = i;
    while (i < s.size() && !isspace((unsigned char)s[i]) && s[i] != '>' && s[i] != '/') i++;
    x->name = s.substr(b, i - b);
    if (x->name.empty()) throw std::runtime_error(x->loc + ": element name expected");
    for (;;) {
      ws();
      if (i >= s.size()) throw std::runtime_error(where() + ": unterminated tag");
      if (s[i] == '/') {
        if (s.compare(i, 2, "/>") != 0) throw std::runtime_error(where() + ": '/>' expected");
        i += 2;
        return x;
      }
      if (s[i] == '>') { i++; break; }
      b = i;
      while (i < s.size() && s[i] != '=' && s[i] != '>' && s[i] != '/' && !isspace((unsigned char)s[i])) i++;
      std::string key = s.substr(b, i - b);
      ws();
      if (key.empty() || i >= s.size() || s[i] != '=') throw std::runtime_error(where() + ": malformed attribute");
      i++;  // '='
      ws();
      if (i >= s.size() || (s[i] != '"' && s[i] != '\'')) throw std::runtime_error(where() + ": quoted value expected");
      const char q = s[i++];
      const size_t e = s.find(q, i);
      if (e == std::string::npos) throw std::runtime_error(where() + ": unterminated attribute value");
      x->parms[key] = s.substr(i, e - i);
      i = e + 1;
    }
    for (;;) {
      // text
      size_t b2 = i;
      while (i < s.size() && s[i] != '<') i++;
      tokens(s.substr(b2, i - b2), x->body);
      if (i >= s.size()) throw std::runtime_error(where() + ": unexpected end of file");
      if (s.compare(i, 4, "<!--") == 0) {
        size_t e = s.find("-->", i);
        i = e == std::string::npos ? s.size() : e + 3;
        continue;
      }
      if (s.compare(i, 2, "</") == 0) {
        const size_t e = s.find('>', i);
        if (e == std::string::npos) throw std::runtime_error(where() + ": unterminated end tag");
        i = e + 1;
        return x;
      }
      x->children.push_back(node(depth + 1));
    }
  }
};

static XMLp parse_xml(const std::string& file) {
  std::ifstream in(file);
  if (!in) throw std::runtime_error("cannot open " + file);
  XmlReader r;
  r.file = file;
  r.s.assign(std::istreambuf_iterator<char>(in), std::istreambuf_iterator<char>());
  return r.node();
}

// ---------------------------------------------------------------- XML scene loader
struct XMLLoader {
  Loader& L;
  YRTDevice dev;
  std::string path;
  FILE* binFile = nullptr;
  std::vector<yrt_affine> transforms;
  std::map<std::string, YRTHandle> materialMap;
  std::map<const XML*, YRTHandle> materialCache;
  std::map<std::string, std::vector<YRTHandle>> sceneMap;
  std::vector<YRTHandle> model;

  XMLLoader(Loader& l, const std::string& file) : L(l), dev(l.dev) {
    path = path_of(file);
    std::string bin = file.substr(0, file.find_last_of('.')) + ".bin";
    binFile = fopen(bin.c_str(), "rb");
    transforms.push_back(yrt_affine::identity());
    XMLp xml = parse_xml(file);
    if (xml->name != "scene") throw std::runtime_error(xml->loc + ": invalid scene tag");
    for (auto& c : xml->children) {
      auto prims = loadScene(c);
      model.insert(model.end(), prims.begin(), prims.end());
    }
  }
  ~XMLLoader() {
    if (binFile) fclose(binFile);
  }

  static float F(const XMLp& x, size_t i) { return (float)atof(x->body.at(i).c_str()); }
  static int I(const XMLp& x, size_t i) { return atoi(x->body.at(i).c_str()); }
  static void need(const XMLp& x, size_t n, const char* what) {
    if (x->body.size() != n) throw std::runtime_error(x->loc + ": wrong " + what + " body");
  }
  float f1(const XMLp& x) {
    need(x, 1, "float");
    return F(x, 0);
  }
  yrt_v3 v3(const XMLp& x) {
    need(x, 3, "float3");
    return {F(x, 0), F(x, 1), F(x, 2)};
  }
  // load<AffineSpace3f> (xml_loader.cpp:138-175)
  yrt_affine affine(const XMLp& x) {
    float a, b, c;
    if (x->parm("translate") != "") {
      sscanf(x->parm("translate").c_str(), "%f %f %f", &a, &b, &c);
      return yrt_affine::translate(a, b, c);
    }
    if (x->parm("scale") != "") {
      sscanf(x->parm("scale").c_str(), "%f %f %f", &a, &b, &c);
      return yrt_affine::scale(a, b, c);
    }
    if (x->parm("rotate_x") != "" || x->parm("rotate_y") != "" || x->parm("rotate_z") != "" ||
        (x->parm("rotate") != "" && x->parm("axis") != "")) {
      float deg = 0, ax = 0, ay = 0, az = 0;
      if (x->parm("rotate_x") != "") { sscanf(x->parm("rotate_x").c_str(), "%f", &deg); ax = 1; }
      else if (x->parm("rotate_y") != "") { sscanf(x->parm("rotate_y").c_str(), "%f", &deg); ay = 1; }
      else if (x->parm("rotate_z") != "") { sscanf(x->parm("rotate_z").c_str(), "%f", &deg); az = 1; }
      else {
        sscanf(x->parm("rotate").c_str(), "%f", &deg);
        sscanf(x->parm("axis").c_str(), "%f %f %f", &ax, &ay, &az);
      }
      return yrt_affine::rotate(ax, ay, az, deg * 1.74532925199432957692e-2f);
    }
    need(x, 12, "AffineSpace");
    yrt_affine m;
    // rows: (m00 m01 m02 p.x) (m10 m11 m12 p.y) (m20 m21 m22 p.z); columns vx,vy,vz
    m.v[0] = F(x, 0); m.v[1] = F(x, 4); m.v[2] = F(x, 8);
    m.v[3] = F(x, 1); m.v[4] = F(x, 5); m.v[5] = F(x, 9);
    m.v[6] = F(x, 2); m.v[7] = F(x, 6); m.v[8] = F(x, 10);
    m.v[9] = F(x, 3); m.v[10] = F(x, 7); m.v[11] = F(x, 11);
    return m;
  }

  YRTHandle array(const XMLp& x, int comps, bool isInt, size_t& size) {
    size = 0;
    if (!x) return nullptr;
    std::vector<uint8_t> bytes;
    if (x->parm("ofs") != "") {
      if (!binFile) throw std::runtime_error("cannot open .bin file for " + x->loc);
      const long ofs = atol(x->parm("ofs").c_str());
      size = (size_t)atol(x->parm("size").c_str());
      bytes.resize(size * comps * 4);
      fseek(binFile, ofs, SEEK_SET);
      if (fread(bytes.data(), comps * 4, size, binFile) != size) throw std::runtime_error("error reading .bin");
    } else {
      if (x->body.size() % comps) throw std::runtime_error(x->loc + ": wrong array body");
      size = x->body.size() / comps;
      bytes.resize(size * comps * 4);
      for (size_t i = 0; i < x->body.size(); ++i) {
        if (isInt) { int v = atoi(x->body[i].c_str()); memcpy(&bytes[i * 4], &v, 4); }
        else { float v = (float)atof(x->body[i].c_str()); memcpy(&bytes[i * 4], &v, 4); }
      }
    }
    if (!size) return nullptr;
    return checkH(dev, yrtNewData(dev, "immutable_managed", bytes.size(), bytes.data()), "rtNewData");
  }

  YRTHandle prim_light(YRTHandle light) {
    return checkH(dev, yrtNewLightPrimitive(dev, light, nullptr, transforms.back().v), "rtNewLightPrimitive");
  }

  // loadMaterialParms (xml_loader.cpp:384-404)
  void materialParms(YRTHandle m, const XMLp& parms) {
    for (auto& e : parms->children) {
      const std::string n = e->parm("name");
      const char* nm = n.c_str();
      if (e->name == "int") { need(e, 1, "int"); check(dev, yrtSetInt1(dev, m, nm, I(e, 0)), "rtSetInt1"); }
      else if (e->name == "int2") { need(e, 2, "int2"); check(dev, yrtSetInt2(dev, m, nm, I(e, 0), I(e, 1)), "rtSetInt2"); }
      else if (e->name == "int3") { need(e, 3, "int3"); check(dev, yrtSetInt3(dev, m, nm, I(e, 0), I(e, 1), I(e, 2)), "rtSetInt3"); }
      else if (e->name == "int4") { need(e, 4, "int4"); check(dev, yrtSetInt4(dev, m, nm, I(e, 0), I(e, 1), I(e, 2), I(e, 3)), "rtSetInt4"); }
      else if (e->name == "float") { need(e, 1, "float"); check(dev, yrtSetFloat1(dev, m, nm, F(e, 0)), "rtSetFloat1"); }
      else if (e->name == "float2") { need(e, 2, "float2"); check(dev, yrtSetFloat2(dev, m, nm, F(e, 0), F(e, 1)), "rtSetFloat2"); }
      else if (e->name == "float3") { need(e, 3, "float3"); check(dev, yrtSetFloat3(dev, m, nm, F(e, 0), F(e, 1), F(e, 2)), "rtSetFloat3"); }
      else if (e->name == "float4") { need(e, 4, "float4"); check(dev, yrtSetFloat4(dev, m, nm, F(e, 0), F(e, 1), F(e, 2), F(e, 3)), "rtSetFloat4"); }
      else if (e->name == "texture") {
        if (e->body.size() < 1) throw std::runtime_error(e->loc + ": wrong string body");
        check(dev, yrtSetTexture(dev, m, nm, L.texture(join_path(path, e->body[0]))), "rtSetTexture");
      } else throw std::runtime_error(e->loc + ": invalid type: " + e->name);
    }
    check(dev, yrtCommit(dev, m), "rtCommit(material)");
  }

  // loadMaterial (xml_loader.cpp:406-430)
  YRTHandle material(const XMLp& x) {
    if (x->parm("file") != "") throw std::runtime_error(x->loc + ": external material files are not supported");
    if (x->parm("id") != "") return materialMap[x->parm("id")];
    XMLp parms = x->child("parameters");
    auto it = materialCache.find(parms.get());
    if (it != materialCache.end()) return it->second;
    XMLp code = x->child("code");
    if (code->body.size() < 1) throw std::runtime_error(code->loc + ": wrong string body");
    YRTHandle m = checkH(dev, yrtNewMaterial(dev, code->body[0].c_str()), "rtNewMaterial");
    materialParms(m, parms);
    return materialCache[parms.get()] = m;
  }

  std::vector<YRTHandle> loadScene(const XMLp& x) {
    std::vector<YRTHandle> prims;
    if (x->name == "assign") {
      if (x->parm("type") == "material") materialMap[x->parm("id")] = material(x->children.at(0));
      else if (x->parm("type") == "scene") sceneMap[x->parm("id")] = loadScene(x->children.at(0));
      else throw std::runtime_error(x->loc + ": unknown type: " + x->parm("type"));
      return prims;
    }
    if (x->name == "xml" || x->name == "obj" || x->name == "extern" || x->name == "ref")
      throw std::runtime_error(x->loc + ": <" + x->name + "> (rtTransformPrimitive) is not supported by this build");
    if (x->name == "AmbientLight") {
      yrt_v3 Lc = v3(x->child("L"));
      YRTHandle l = checkH(dev, yrtNewLight(dev, "ambientlight"), "rtNewLight");
      check(dev, yrtSetFloat3(dev, l, "L", Lc.x, Lc.y, Lc.z), "rtSetFloat3");
      check(dev, yrtCommit(dev, l), "rtCommit(light)");
      prims.push_back(prim_light(l));
    } else if (x->name == "TriangleLight" || x->name == "QuadLight") {
      // loadTriangleLight / loadQuadLight (xml_loader.cpp:310-381)
      const yrt_affine s = affine(x->child("AffineSpace"));
      const yrt_v3 Lc = v3(x->child("L"));
      auto mk = [&](yrt_v3 a, yrt_v3 b, yrt_v3 c) {
        YRTHandle l = checkH(dev, yrtNewLight(dev, "trianglelight"), "rtNewLight");
        check(dev, yrtSetFloat3(dev, l, "L", Lc.x, Lc.y, Lc.z), "rtSetFloat3");
        check(dev, yrtSetFloat3(dev, l, "v0", a.x, a.y, a.z), "rtSetFloat3");
        check(dev, yrtSetFloat3(dev, l, "v1", b.x, b.y, b.z), "rtSetFloat3");
        check(dev, yrtSetFloat3(dev, l, "v2", c.x, c.y, c.z), "rtSetFloat3");
        check(dev, yrtCommit(dev, l), "rtCommit(light)");
        prims.push_back(prim_light(l));
      };
      if (x->name == "TriangleLight") {
        mk(s.point(1, 0, 0), s.point(0, 1, 0), s.point(0, 0, 0));
      } else {
        const yrt_v3 v0 = s.point(0, 0, 0), v1 = s.point(0, 1, 0), v2 = s.point(1, 1, 0), v3_ = s.point(1, 0, 0);
        mk(v1, v3_, v0);
        mk(v2, v3_, v1);
      }
    } else if (x->name == "HDRILight") {
      const yrt_affine s = affine(x->child("AffineSpace"));
      const yrt_v3 Lc = v3(x->child("L"));
      YRTHandle l = checkH(dev, yrtNewLight(dev, "hdrilight"), "rtNewLight");
      check(dev, yrtSetTransform(dev, l, "local2world", s.v), "rtSetTransform");
      check(dev, yrtSetFloat3(dev, l, "L", Lc.x, Lc.y, Lc.z), "rtSetFloat3");
      XMLp im = x->child("image");
      if (im->body.size() < 1) throw std::runtime_error(im->loc + ": wrong string body");
      check(dev, yrtSetImage(dev, l, "image", L.image(join_path(path, im->body[0]))), "rtSetImage");
      check(dev, yrtCommit(dev, l), "rtCommit(light)");
      prims.push_back(prim_light(l));
    } else if (x->name == "PointLight" || x->name == "SpotLight" || x->name == "DirectionalLight" ||
               x->name == "DistantLight") {
      // loadPointLight / loadSpotLight / loadDirectionalLight / loadDistantLight (xml_loader.cpp:274-324)
      const yrt_affine sp = affine(x->child("AffineSpace"));
      YRTHandle l;
      if (x->name == "PointLight") {
        const yrt_v3 I = v3(x->child("I"));
        l = checkH(dev, yrtNewLight(dev, "pointlight"), "rtNewLight");
        check(dev, yrtSetFloat3(dev, l, "P", sp.v[9], sp.v[10], sp.v[11]), "rtSetFloat3");
        check(dev, yrtSetFloat3(dev, l, "I", I.x, I.y, I.z), "rtSetFloat3");
      } else if (x->name == "SpotLight") {
        const yrt_v3 I = v3(x->child("I"));
        l = checkH(dev, yrtNewLight(dev, "spotlight"), "rtNewLight");
        check(dev, yrtSetFloat3(dev, l, "P", sp.v[9], sp.v[10], sp.v[11]), "rtSetFloat3");
        check(dev, yrtSetFloat3(dev, l, "D", sp.v[6], sp.v[7], sp.v[8]), "rtSetFloat3");
        check(dev, yrtSetFloat3(dev, l, "I", I.x, I.y, I.z), "rtSetFloat3");
        check(dev, yrtSetFloat1(dev, l, "angleMin", f1(x->child("angleMin"))), "rtSetFloat1");
        check(dev, yrtSetFloat1(dev, l, "angleMax", f1(x->child("angleMax"))), "rtSetFloat1");
      } else if (x->name == "DirectionalLight") {
        const yrt_v3 E = v3(x->child("E"));
        l = checkH(dev, yrtNewLight(dev, "directionallight"), "rtNewLight");
        check(dev, yrtSetFloat3(dev, l, "D", sp.v[6], sp.v[7], sp.v[8]), "rtSetFloat3");
        check(dev, yrtSetFloat3(dev, l, "E", E.x, E.y, E.z), "rtSetFloat3");
      } else {
        const yrt_v3 Lc = v3(x->child("L"));
        l = checkH(dev, yrtNewLight(dev, "distantlight"), "rtNewLight");
        check(dev, yrtSetFloat3(dev, l, "D", sp.v[6], sp.v[7], sp.v[8]), "rtSetFloat3");
        check(dev, yrtSetFloat3(dev, l, "L", Lc.x, Lc.y, Lc.z), "rtSetFloat3");
        check(dev, yrtSetFloat1(dev, l, "halfAngle", f1(x->child("halfAngle"))), "rtSetFloat1");
      }
      check(dev, yrtCommit(dev, l), "rtCommit(light)");
      prims.push_back(prim_light(l));
    } else if (x->name == "TriangleMesh") {
      // loadTriangleMesh (xml_loader.cpp:432-459)
      YRTHandle mat = material(x->child("material"));
      size_t np, nm, nn, nt, ni;
      YRTHandle pos = array(x->childOpt("positions"), 3, false, np);
      YRTHandle mot = array(x->childOpt("motions"), 3, false, nm);
      YRTHandle nor = array(x->childOpt("normals"), 3, false, nn);
      YRTHandle tex = array(x->childOpt("texcoords"), 2, false, nt);
      YRTHandle tri = array(x->childOpt("triangles"), 3, true, ni);
      XMLp fc = x->childOpt("faceCamera");
      bool faceCamera = false;
      if (fc) { need(fc, 1, "bool"); faceCamera = I(fc, 0) != 0; }
      YRTHandle mesh = checkH(dev, yrtNewShape(dev, "trianglemesh"), "rtNewShape");
      if (np) check(dev, yrtSetArray(dev, mesh, "positions", "float3", pos, np, 12, 0), "rtSetArray");
      if (nm) check(dev, yrtSetArray(dev, mesh, "motions", "float3", mot, nm, 12, 0), "rtSetArray");
      if (nn) check(dev, yrtSetArray(dev, mesh, "normals", "float3", nor, nn, 12, 0), "rtSetArray");
      if (nt) check(dev, yrtSetArray(dev, mesh, "texcoords", "float2", tex, nt, 8, 0), "rtSetArray");
      if (ni) check(dev, yrtSetArray(dev, mesh, "indices", "int3", tri, ni, 12, 0), "rtSetArray");
      check(dev, yrtSetString(dev, mesh, "accel", "default"), "rtSetString");
      check(dev, yrtCommit(dev, mesh), "rtCommit(shape)");
      prims.push_back(checkH(dev, yrtNewShapePrimitive(dev, mesh, mat, transforms.back().v, faceCamera),
                             "rtNewShapePrimitive"));
    } else if (x->name == "Sphere") {
      // loadSphere (xml_loader.cpp:461-478)
      YRTHandle mat = material(x->child("material"));
      const yrt_v3 P = v3(x->child("position"));
      yrt_v3 dPdt = {0, 0, 0};
      if (x->childOpt("motion")) dPdt = v3(x->child("motion"));
      YRTHandle s = checkH(dev, yrtNewShape(dev, "sphere"), "rtNewShape");
      XMLp r = x->child("radius"), th = x->child("numTheta"), ph = x->child("numPhi");
      need(r, 1, "float");
      need(th, 1, "int");
      need(ph, 1, "int");
      check(dev, yrtSetFloat3(dev, s, "P", P.x, P.y, P.z), "rtSetFloat3");
      check(dev, yrtSetFloat3(dev, s, "dPdt", dPdt.x, dPdt.y, dPdt.z), "rtSetFloat3");
      check(dev, yrtSetFloat1(dev, s, "r", F(r, 0)), "rtSetFloat1");
      check(dev, yrtSetInt1(dev, s, "numTheta", I(th, 0)), "rtSetInt1");
      check(dev, yrtSetInt1(dev, s, "numPhi", I(ph, 0)), "rtSetInt1");
      check(dev, yrtCommit(dev, s), "rtCommit(shape)");
      prims.push_back(checkH(dev, yrtNewShapePrimitive(dev, s, mat, transforms.back().v, 0), "rtNewShapePrimitive"));
    } else if (x->name == "Disk") {
      // loadDisk (xml_loader.cpp:491-504)
      YRTHandle mat = material(x->child("material"));
      const yrt_v3 P = v3(x->child("position"));
      YRTHandle s = checkH(dev, yrtNewShape(dev, "disk"), "rtNewShape");
      XMLp r = x->child("radius"), nt = x->child("numTriangles");
      need(r, 1, "float");
      need(nt, 1, "int");
      float h = 0.0f;
      if (XMLp hx = x->childOpt("height")) {
        need(hx, 1, "float");
        h = F(hx, 0);
      }
      check(dev, yrtSetFloat3(dev, s, "P", P.x, P.y, P.z), "rtSetFloat3");
      check(dev, yrtSetFloat1(dev, s, "r", F(r, 0)), "rtSetFloat1");
      check(dev, yrtSetFloat1(dev, s, "h", h), "rtSetFloat1");
      check(dev, yrtSetInt1(dev, s, "numTriangles", I(nt, 0)), "rtSetInt1");
      check(dev, yrtCommit(dev, s), "rtCommit(shape)");
      prims.push_back(checkH(dev, yrtNewShapePrimitive(dev, s, mat, transforms.back().v, 0), "rtNewShapePrimitive"));
    } else if (x->name == "Group") {
      for (auto& c : x->children) {
        auto p = loadScene(c);
        prims.insert(prims.end(), p.begin(), p.end());
      }
    } else if (x->name == "Transform") {
      // loadTransformNode (xml_loader.cpp:495-511)
      transforms.push_back(transforms.back() * affine(x->children.at(0)));
      for (size_t i = 1; i < x->children.size(); ++i) {
        auto p = loadScene(x->children[i]);
        prims.insert(prims.end(), p.begin(), p.end());
      }
      transforms.pop_back();
    } else {
      throw std::runtime_error(x->loc + ": unknown tag: " + x->name);
    }
    return prims;
  }
};

// ---------------------------------------------------------------- OBJ loader
namespace {
struct OVertex {
  int v, vt, vn;
  bool operator<(const OVertex& b) const {
    if (v != b.v) return v < b.v;
    if (vn != b.vn) return vn < b.vn;
    if (vt != b.vt) return vt < b.vt;
    return false;
  }
};

struct OBJLoader {
  Loader& L;
  YRTDevice dev;
  std::string path;
  std::vector<yrt_v3> v, vn;
  std::vector<float> vt;
  std::vector<std::vector<OVertex>> curGroup;
  YRTHandle curMaterial = nullptr;
  std::map<std::string, YRTHandle> material;
  std::vector<YRTHandle> model;

  static const char* skipSep(const char* t) { return t + strspn(t, " \t"); }
  static float getFloat(const char*& t) {
    t += strspn(t, " \t");
    float n = (float)atof(t);
    t += strcspn(t, " \t\r");
    return n;
  }
  int fix_v(int i) { return i > 0 ? i - 1 : (i == 0 ? 0 : (int)v.size() + i); }
  int fix_vt(int i) { return i > 0 ? i - 1 : (i == 0 ? 0 : (int)(vt.size() / 2) + i); }
  int fix_vn(int i) { return i > 0 ? i - 1 : (i == 0 ? 0 : (int)vn.size() + i); }
  // getInt3 (obj_loader.cpp:289-313)
  OVertex getInt3(const char*& t) {
    OVertex r{-1, -1, -1};
    r.v = fix_v(atoi(t));
    t += strcspn(t, "/ \t\r");
    if (t[0] != '/') return r;
    t++;
    if (t[0] == '/') {
      t++;
      r.vn = fix_vn(atoi(t));
      t += strcspn(t, " \t\r");
      return r;
    }
    r.vt = fix_vt(atoi(t));
    t += strcspn(t, "/ \t\r");
    if (t[0] != '/') return r;
    t++;
    r.vn = fix_vn(atoi(t));
    t += strcspn(t, " \t\r");
    return r;
  }

  static bool readLine(std::istream& in, std::string& line) {
    line.clear();
    std::string part;
    while (std::getline(in, part)) {
      if (!part.empty() && part.back() == '\r') part.pop_back();
      if (!part.empty() && part.back() == '\\') {
        part.back() = ' ';
        line += part;
        continue;
      }
      line += part;
      return true;
    }
    return !line.empty();
  }
  static std::string trim(const std::string& s) {
    size_t b = s.find_first_not_of(" \t"), e = s.find_last_not_of(" \t\r");
    return b == std::string::npos ? "" : s.substr(b, e - b + 1);
  }

  OBJLoader(Loader& l, const std::string& file) : L(l), dev(l.dev), path(path_of(file)) {
    std::ifstream in(file);
    if (!in) throw std::runtime_error("cannot open " + file);
    YRTHandle defaultMaterial = checkH(dev, yrtNewMaterial(dev, "matte"), "rtNewMaterial");
    check(dev, yrtSetFloat3(dev, defaultMaterial, "reflectance", 0.5f, 0.5f, 0.5f), "rtSetFloat3");
    check(dev, yrtCommit(dev, defaultMaterial), "rtCommit");
    curMaterial = defaultMaterial;
    std::string raw;
    while (readLine(in, raw)) {
      const std::string line = trim(raw);
      const char* t = line.c_str();
      if (!t[0]) continue;
      auto sep = [](char c) { return c == ' ' || c == '\t'; };
      if (t[0] == 'v' && sep(t[1])) {
        t += 2;
        float x = getFloat(t), y = getFloat(t), z = getFloat(t);
        v.push_back({x, y, z});
      } else if (t[0] == 'v' && t[1] == 'n' && sep(t[2])) {
        t += 3;
        float x = getFloat(t), y = getFloat(t), z = getFloat(t);
        vn.push_back({x, y, z});
      } else if (t[0] == 'v' && t[1] == 't' && sep(t[2])) {
        t += 3;
        float x = getFloat(t), y = getFloat(t);
        vt.push_back(x);
        vt.push_back(y);
      } else if (t[0] == 'f' && sep(t[1])) {
        t = skipSep(t + 1);
        std::vector<OVertex> face;
        while (t[0]) {
          const char* t0 = t;
          face.push_back(getInt3(t));
          t = skipSep(t);
          // a separator getInt3 does not consume (a stray '\r' inside the line) would leave t
          // in place and grow the face without bound (mutation fuzz finding)
          if (t == t0) throw std::runtime_error("OBJ: malformed face line");
        }
        curGroup.push_back(face);
      } else if (!strncmp(t, "usemtl", 6) && sep(t[6])) {
        flushFaceGroup();
        std::string name(skipSep(t + 6));
        auto it = material.find(name);
        curMaterial = it == material.end() ? defaultMaterial : it->second;
      } else if (!strncmp(t, "mtllib", 6) && sep(t[6])) {
        loadMTL(path + std::string(skipSep(t + 6)));
      }
    }
    flushFaceGroup();
  }

  // loadMTL (obj_loader.cpp:219-280)
  void loadMTL(const std::string& file) {
    std::ifstream in(file);
    if (!in) return;  // reference prints "cannot open" and continues
    YRTHandle cur = nullptr;
    std::string raw;
    while (readLine(in, raw)) {
      const std::string line = trim(raw);
      const char* t = line.c_str();
      if (!t[0] || t[0] == '#') continue;
      if (!strncmp(t, "newmtl", 6)) {
        if (cur) check(dev, yrtCommit(dev, cur), "rtCommit(material)");
        std::string name(skipSep(t + 6));
        material[name] = cur = checkH(dev, yrtNewMaterial(dev, "obj"), "rtNewMaterial");
        continue;
      }
      if (!cur) throw std::runtime_error("invalid material file: newmtl expected first");
      auto f3 = [&](const char* name, int skip) {
        const char* p = skipSep(t + skip);
        float x = getFloat(p), y = getFloat(p), z = getFloat(p);
        check(dev, yrtSetFloat3(dev, cur, name, x, y, z), "rtSetFloat3");
      };
      auto f1 = [&](const char* name, int skip) {
        const char* p = skipSep(t + skip);
        check(dev, yrtSetFloat1(dev, cur, name, getFloat(p)), "rtSetFloat1");
      };
      auto tx = [&](const char* name, int skip) {
        check(dev, yrtSetTexture(dev, cur, name, L.texture(path + std::string(skipSep(t + skip)))), "rtSetTexture");
      };
      if (!strncmp(t, "illum", 5)) continue;
      if (!strncmp(t, "d", 1)) { f1("d", 1); continue; }
      if (!strncmp(t, "Ns", 2)) { f1("Ns", 2); continue; }
      if (!strncmp(t, "Ni", 2)) { f1("Ni", 2); continue; }
      if (!strncmp(t, "Ka", 2)) { f3("Ka", 2); continue; }
      if (!strncmp(t, "Kd", 2)) { f3("Kd", 2); continue; }
      if (!strncmp(t, "Ks", 2)) { f3("Ks", 2); continue; }
      if (!strncmp(t, "Tf", 2)) { f3("Tf", 2); continue; }
      if (!strncmp(t, "map_d", 5)) { tx("map_d", 5); continue; }
      if (!strncmp(t, "map_Ns", 6)) { tx("map_Ns", 6); continue; }
      if (!strncmp(t, "map_Ka", 6)) { tx("map_Ka", 6); continue; }
      if (!strncmp(t, "map_Kd", 6)) { tx("map_Kd", 6); continue; }
      if (!strncmp(t, "map_Ks", 6)) { tx("map_Ks", 6); continue; }
      if (!strncmp(t, "map_Refl", 8)) { tx("map_Refl", 8); continue; }
      if (!strncmp(t, "map_Bump", 8)) { tx("map_Bump", 8); continue; }
    }
    if (cur) check(dev, yrtCommit(dev, cur), "rtCommit(material)");
  }

  // flushFaceGroup (obj_loader.cpp:330-380): fan triangulation, vertex dedupe per group
  void flushFaceGroup() {
    if (curGroup.empty()) return;
    std::vector<float> positions, normals, texcoords;
    std::vector<int> triangles;
    std::map<OVertex, int> vertexMap;
    auto getVertex = [&](const OVertex& i) -> int {
      auto it = vertexMap.find(i);
      if (it != vertexMap.end()) return it->second;
      const yrt_v3 p = v.at(i.v);
      positions.insert(positions.end(), {p.x, p.y, p.z});
      if (i.vn >= 0) { const yrt_v3 n = vn.at(i.vn); normals.insert(normals.end(), {n.x, n.y, n.z}); }
      if (i.vt >= 0) { texcoords.push_back(vt.at(2 * i.vt)); texcoords.push_back(vt.at(2 * i.vt + 1)); }
      return vertexMap[i] = (int)(positions.size() / 3) - 1;
    };
    for (auto& face : curGroup) {
      // a face of fewer than three vertices yields no triangle (the reference's fan reads
      // face[1] regardless: a heap overread on "f 1", found by the mutation fuzz)
      if (face.size() < 3) continue;
      OVertex i0 = face[0], i1{-1, -1, -1}, i2 = face[1];
      for (size_t k = 2; k < face.size(); k++) {
        i1 = i2;
        i2 = face[k];
        const int v0 = getVertex(i0), v1 = getVertex(i1), v2 = getVertex(i2);
        triangles.insert(triangles.end(), {v0, v1, v2});
      }
    }
    curGroup.clear();
    // vertices with and without normals (or texture coordinates) in one group would give
    // arrays shorter than the positions, which the mesh would index past their end
    if ((!normals.empty() && normals.size() != positions.size()) ||
        (!texcoords.empty() && texcoords.size() / 2 != positions.size() / 3))
      throw std::runtime_error("OBJ: a face group mixes vertices with and without normals or texture coordinates");
    if (triangles.empty()) return;
    YRTHandle dp = checkH(dev, yrtNewData(dev, "immutable", positions.size() * 4, positions.data()), "rtNewData");
    YRTHandle dt = checkH(dev, yrtNewData(dev, "immutable", triangles.size() * 4, triangles.data()), "rtNewData");
    YRTHandle mesh = checkH(dev, yrtNewShape(dev, "trianglemesh"), "rtNewShape");
    check(dev, yrtSetArray(dev, mesh, "positions", "float3", dp, positions.size() / 3, 12, 0), "rtSetArray");
    check(dev, yrtSetArray(dev, mesh, "indices", "int3", dt, triangles.size() / 3, 12, 0), "rtSetArray");
    if (!normals.empty()) {
      YRTHandle dn = checkH(dev, yrtNewData(dev, "immutable", normals.size() * 4, normals.data()), "rtNewData");
      check(dev, yrtSetArray(dev, mesh, "normals", "float3", dn, normals.size() / 3, 12, 0), "rtSetArray");
    }
    if (!texcoords.empty()) {
      YRTHandle dx = checkH(dev, yrtNewData(dev, "immutable", texcoords.size() * 4, texcoords.data()), "rtNewData");
      check(dev, yrtSetArray(dev, mesh, "texcoords", "float2", dx, texcoords.size() / 2, 8, 0), "rtSetArray");
    }
    check(dev, yrtCommit(dev, mesh), "rtCommit(shape)");
    model.push_back(checkH(dev, yrtNewShapePrimitive(dev, mesh, curMaterial, nullptr, 0), "rtNewShapePrimitive"));
  }
};
}  // namespace

// rtLoadScene (devices/device/loaders/loaders.cpp:68-74)
std::vector<YRTHandle> Loader::loadScene(const std::string& file) {
  const std::string ext = ext_of(file);
  std::vector<YRTHandle> prims;
  if (ext == "obj") {
    OBJLoader l(*this, file);
    prims = l.model;
  } else if (ext == "xml") {
    XMLLoader l(*this, file);
    prims = l.model;
  } else if (ext == "dae") {
    prims = load_dae(*this, file, "default", nullptr);  // cameras: see RtState "-i
  } else {
    throw std::runtime_error("unknown scene file format: " + file);
  }
  // loaders clear the image/texture caches when they finish (xml_loader.cpp:613-619)
  images.clear();
  textures.clear();
  return prims;
}

}  // namespace yrtfe
