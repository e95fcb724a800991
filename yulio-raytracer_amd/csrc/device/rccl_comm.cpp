// rccl_comm.cpp — lazy librccl binding (see rccl_comm.h).
#include "rccl_comm.h"

#include <dlfcn.h>

#include <mutex>
#include <stdexcept>
#include <string>

namespace yrt {

const RcclApi& rccl() {
  static RcclApi api{};
  static std::string err;
  static std::once_flag once;
  std::call_once(once, [] {
    // an RCCL already in the process (e.g. PyTorch's) is reused by soname; else ROCm's
    void* h = nullptr;
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
      h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
      if (h) break;
    }
    if (!h) {
      err = std::string("cannot load librccl: ") + dlerror();
      return;
    }
    auto sym = [&](const char* n) {
      void* p = dlsym(h, n);
      if (!p && err.empty()) err = std::string("librccl lacks ") + n;
      return p;
    };
    api.GetUniqueId = (decltype(api.GetUniqueId))sym("ncclGetUniqueId");
    api.CommInitRank = (decltype(api.CommInitRank))sym("ncclCommInitRank");
    api.CommInitAll = (decltype(api.CommInitAll))sym("ncclCommInitAll");
    api.CommDestroy = (decltype(api.CommDestroy))sym("ncclCommDestroy");
    // abort and async-error polling bound the gather's waits (gather.cpp); optional
    api.CommAbort = (decltype(api.CommAbort))dlsym(h, "ncclCommAbort");
    api.CommGetAsyncError = (decltype(api.CommGetAsyncError))dlsym(h, "ncclCommGetAsyncError");
    api.GroupStart = (decltype(api.GroupStart))sym("ncclGroupStart");
    api.GroupEnd = (decltype(api.GroupEnd))sym("ncclGroupEnd");
    api.Send = (decltype(api.Send))sym("ncclSend");
    api.Recv = (decltype(api.Recv))sym("ncclRecv");
    api.AllReduce = (decltype(api.AllReduce))sym("ncclAllReduce");
    api.GetErrorString = (decltype(api.GetErrorString))sym("ncclGetErrorString");
  });
  if (!err.empty()) throw std::runtime_error(err);
  return api;
}

void rccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess)
    throw std::runtime_error(std::string("RCCL ") + what + ": " + rccl().GetErrorString(r));
}

}  // namespace yrt
