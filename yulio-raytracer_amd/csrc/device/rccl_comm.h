// rccl_comm.h — RCCL (librccl, over xGMI between MI355X GPUs) for the multi-GPU frame gather.
//
// The reference has no GPU collective: its multi-node analogue is device_network's TCP row
// bands (devices/device_network/network_device.cpp:255-300, api/swapchain.h:57-70). Here the
// 16x16 tiles of a frame are dealt round-robin over GPUs and the one exchange
// step is a grouped send/recv of every peer's tile slab to GPU 0 (a gather: each peer uses its
// own xGMI link). librccl is opened on first use (dlopen), so the single-GPU path never loads
// it; a multi-GPU render that needs it fails loudly when it is missing.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <vector>

namespace yrt {

struct RcclApi {
  ncclResult_t (*GetUniqueId)(ncclUniqueId*);
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int);
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*);
  ncclResult_t (*CommDestroy)(ncclComm_t);
  ncclResult_t (*CommAbort)(ncclComm_t);                         // optional (nullptr: CommDestroy)
  ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*);  // optional
  ncclResult_t (*GroupStart)();
  ncclResult_t (*GroupEnd)();
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
  const char* (*GetErrorString)(ncclResult_t);
};

// The loaded API (throws std::runtime_error when librccl cannot be opened).
const RcclApi& rccl();
// Throws with the RCCL error string on failure.
void rccl_check(ncclResult_t r, const char* what);

}  // namespace yrt
