// export.cpp — yrtExportFrame: serializes what the device was told through the API
// (objects with their raw rtSet* property bags, the scene's primitive slots, renderer and
// camera) so the CPU oracle can rebuild the frame independently with the reference
// constructors' defaults. Format documented in oracle/yrt_oracle.h ("frame blob").
#include <string.h>

#include <map>
#include <stdexcept>
#include <vector>

#include "../../../include/yrt_device.h"
#include "objects.h"

namespace yrt {

struct BlobWriter {
  std::vector<uint8_t> b;
  std::map<const Object*, int> ids;
  std::vector<const Object*> order;
  void u32(uint32_t v) { b.insert(b.end(), (uint8_t*)&v, (uint8_t*)&v + 4); }
  void i32(int32_t v) { u32((uint32_t)v); }
  void f32(float v) { b.insert(b.end(), (uint8_t*)&v, (uint8_t*)&v + 4); }
  void str(const std::string& s) {
    u32((uint32_t)s.size());
    b.insert(b.end(), s.begin(), s.end());
  }
  void bytes(const void* p, size_t n) { b.insert(b.end(), (const uint8_t*)p, (const uint8_t*)p + n); }

  int collect(const Object* o) {
    if (!o) return -1;
    auto it = ids.find(o);
    if (it != ids.end()) return it->second;
    for (auto& kv : o->parms.all())
      if (kv.second.obj && kv.second.type != Variant::DATA) collect(kv.second.obj.get());
    const int id = (int)order.size();
    ids[o] = id;
    order.push_back(o);
    return id;
  }

  void object(const Object* o) {
    u32((uint32_t)o->kind);
    str(o->type);
    uint32_t n = 0;
    for (auto& kv : o->parms.all())
      if (kv.second.type != Variant::POINTER) n++;
    u32(n);
    for (auto& kv : o->parms.all()) {
      const Variant& v = kv.second;
      if (v.type == Variant::POINTER) continue;
      str(kv.first);
      u32((uint32_t)v.type);
      switch (v.type) {
        case Variant::BOOL1: case Variant::BOOL2: case Variant::BOOL3: case Variant::BOOL4:
        case Variant::INT1: case Variant::INT2: case Variant::INT3: case Variant::INT4:
          for (int k = 0; k < 4; ++k) i32(v.i[k]);
          break;
        case Variant::FLOAT1: case Variant::FLOAT2: case Variant::FLOAT3: case Variant::FLOAT4:
          for (int k = 0; k < 4; ++k) f32(v.f[k]);
          break;
        case Variant::STRING: str(v.str); break;
        case Variant::TRANSFORM:
          for (int k = 0; k < 12; ++k) f32(v.f[k]);
          break;
        case Variant::IMAGE: case Variant::TEXTURE: i32(collect(v.obj.get())); break;
        case Variant::DATA: {
          const DataObj* d = dynamic_cast<const DataObj*>(v.obj.get());
          size_t es = 12;
          if (v.dataType == "float2" || v.dataType == "int2") es = 8;
          else if (v.dataType == "float4" || v.dataType == "int4") es = 16;
          else if (v.dataType == "float1" || v.dataType == "int1") es = 4;
          str(v.dataType);
          u32((uint32_t)v.size);
          u32((uint32_t)es);
          for (size_t i = 0; i < v.size; ++i) bytes(d->bytes.data() + v.ofs + i * v.stride, es);
          break;
        }
        default: break;
      }
    }
    if (o->kind == Kind::IMAGE) {
      const ImageObj* im = dynamic_cast<const ImageObj*>(o);
      i32(im->width);
      i32(im->height);
      i32(im->format);
      u32((uint32_t)im->data.size());
      bytes(im->data.data(), im->data.size());
    }
  }
};

}  // namespace yrt

using namespace yrt;

struct YRTDevice_;
namespace yrt {
// defined in device.cpp
}

extern "C" int64_t yrt_export_frame_impl(const Object* renderer, const Object* camera, const SceneObj* scene,
                                         uint32_t frameSeed, void* buf, size_t bytes) {
  BlobWriter w;
  // collect every object reachable from the scene slots, renderer, camera
  for (auto& sp : scene->slots) {
    if (!sp || !sp->prim) continue;
    const PrimitiveObj* p = sp->prim.get();
    w.collect(p->shapeHandle.get());
    w.collect(p->lightHandle.get());
    w.collect(p->materialHandle.get());
  }
  const int rid = w.collect(renderer);
  const int cid = w.collect(camera);
  BlobWriter out;
  out.bytes("YRTF", 4);
  out.u32(1);
  out.u32((uint32_t)w.order.size());
  for (const Object* o : w.order) {
    w.b.clear();
    w.object(o);
    out.bytes(w.b.data(), w.b.size());
  }
  out.u32((uint32_t)scene->slots.size());
  for (auto& sp : scene->slots) {
    if (!sp || !sp->prim) {
      out.i32(0);
      continue;
    }
    const PrimitiveObj* p = sp->prim.get();
    out.i32(1);
    auto id = [&](const Object* o) { return o ? w.ids.at(o) : -1; };
    out.i32(id(p->shapeHandle.get()));
    out.i32(id(p->lightHandle.get()));
    out.i32(id(p->materialHandle.get()));
    const A3& a = p->transform;
    const float t[12] = {a.l.vx.x, a.l.vx.y, a.l.vx.z, a.l.vy.x, a.l.vy.y, a.l.vy.z,
                         a.l.vz.x, a.l.vz.y, a.l.vz.z, a.p.x,    a.p.y,    a.p.z};
    for (float f : t) out.f32(f);
    out.i32(p->faceCamera ? 1 : 0);
    out.i32(p->illumMask);
    out.i32(p->shadowMask);
  }
  out.i32(rid);
  out.i32(cid);
  out.u32(frameSeed);
  if (buf) {
    if (bytes < out.b.size()) return -(int64_t)out.b.size();
    memcpy(buf, out.b.data(), out.b.size());
  }
  return (int64_t)out.b.size();
}
