// parms.h — property bag of a device object (mirrors device_singleray/api/parms.h and
// api/variant.h: rtSet* buffers typed values under a name, rtCommit constructs the object
// from them with the constructor's defaults, e.g. parms.getFloat("eta", 1.4f)).
#pragma once

#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../common/yrt_math.h"

namespace yrt {

struct Object;

struct Variant {
  enum Type {
    EMPTY, BOOL1, BOOL2, BOOL3, BOOL4, INT1, INT2, INT3, INT4, FLOAT1, FLOAT2, FLOAT3, FLOAT4,
    STRING, IMAGE, TEXTURE, TRANSFORM, POINTER, DATA
  };
  Type type = EMPTY;
  float f[12] = {0};
  int i[4] = {0};
  std::string str;
  std::shared_ptr<Object> obj;  // IMAGE / TEXTURE / DATA handle (kept alive)
  void* ptr = nullptr;
  // DATA arrays (rtSetArray): element type name, count, stride, offset
  std::string dataType;
  size_t size = 0, stride = 0, ofs = 0;
};

class Parms {
 public:
  void set(const std::string& name, const Variant& v) { m_[name] = v; }
  void clear() { m_.clear(); }
  const Variant* find(const std::string& name) const {
    auto it = m_.find(name);
    return it == m_.end() ? nullptr : &it->second;
  }
  bool has(const std::string& name) const { return find(name) != nullptr; }

  int getInt(const std::string& n, int def = 0) const {
    const Variant* v = find(n);
    if (!v) return def;
    if (v->type == Variant::INT1) return v->i[0];
    if (v->type == Variant::BOOL1) return v->i[0];
    if (v->type == Variant::FLOAT1) return (int)v->f[0];
    throw std::runtime_error("wrong type for int parameter " + n);
  }
  bool getBool(const std::string& n, bool def = false) const {
    const Variant* v = find(n);
    if (!v) return def;
    if (v->type == Variant::BOOL1 || v->type == Variant::INT1) return v->i[0] != 0;
    throw std::runtime_error("wrong type for bool parameter " + n);
  }
  float getFloat(const std::string& n, float def = 0.f) const {
    const Variant* v = find(n);
    if (!v) return def;
    if (v->type == Variant::FLOAT1) return v->f[0];
    if (v->type == Variant::INT1) return (float)v->i[0];
    throw std::runtime_error("wrong type for float parameter " + n);
  }
  V3 getV3(const std::string& n, V3 def = v3s(0.f)) const {
    const Variant* v = find(n);
    if (!v) return def;
    if (v->type == Variant::FLOAT3) return v3(v->f[0], v->f[1], v->f[2]);
    throw std::runtime_error("wrong type for float3 parameter " + n);
  }
  void getV2(const std::string& n, float out[2], float dx, float dy) const {
    const Variant* v = find(n);
    if (!v) { out[0] = dx; out[1] = dy; return; }
    if (v->type == Variant::FLOAT2) { out[0] = v->f[0]; out[1] = v->f[1]; return; }
    throw std::runtime_error("wrong type for float2 parameter " + n);
  }
  std::string getString(const std::string& n, const std::string& def = "") const {
    const Variant* v = find(n);
    if (!v) return def;
    if (v->type == Variant::STRING) return v->str;
    throw std::runtime_error("wrong type for string parameter " + n);
  }
  A3 getTransform(const std::string& n, A3 def = a3_identity()) const {
    const Variant* v = find(n);
    if (!v) return def;
    if (v->type != Variant::TRANSFORM) throw std::runtime_error("wrong type for transform parameter " + n);
    // rtSetTransform takes 12 floats: vx, vy, vz, p (copyToArray, device/handle.h)
    const float* f = v->f;
    return a3(l3(v3(f[0], f[1], f[2]), v3(f[3], f[4], f[5]), v3(f[6], f[7], f[8])), v3(f[9], f[10], f[11]));
  }
  std::shared_ptr<Object> getObject(const std::string& n) const {
    const Variant* v = find(n);
    return v ? v->obj : nullptr;
  }
  void* getPointer(const std::string& n) const {
    const Variant* v = find(n);
    return v ? v->ptr : nullptr;
  }
  const std::map<std::string, Variant>& all() const { return m_; }

 private:
  std::map<std::string, Variant> m_;
};

}  // namespace yrt
