// gather.h — the transport under the multi-GPU frame gather (Device::gather_process).
//
// The frame's 16x16 tiles are dealt round-robin over the ranks; after each
// render every rank (1) joins a status exchange (the min of every rank's "my render
// succeeded" flag, so one failing rank makes every rank fail instead of leaving rank 0 waiting
// for a slab) and (2) rank r > 0 sends its packed tile slab to rank 0, which receives every
// peer's. The reference's analogue is device_network's row bands sent back over TCP
// (devices/device_network/network_device.cpp:255-300, api/swapchain.h:57-70).
//
// Two transports implement the same three operations:
//   - RCCL (yrtSetShardComm): one process per GPU, an ncclComm over xGMI; the status is a
//     4-byte AllReduce(min), the slabs a grouped Send/Recv.
//   - an in-process hub (yrtNewShardHub + yrtSetShardHub): several Device objects of one
//     process (threads; they may share one GPU) meet in host memory and the slabs move by
//     hipMemcpyPeerAsync / device-to-device copy. It runs gather_process's bookkeeping on a
//     one-GPU box, bit-exact against a one-device render (tests/test_gather.py).
// Every wait is bounded (GatherTransport timeout, YRT_GATHER_TIMEOUT_S): a peer that never
// arrives, never sends or sends a wrong size ends the call with an error that names the phase
// and the rank, and the transport is aborted (ncclCommAbort for RCCL), so every later gather
// on it fails at once instead of hanging.
#pragma once

#include <hip/hip_runtime.h>

#include <chrono>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace yrt {

using Clock = std::chrono::steady_clock;

// Seconds a gather phase may wait for its peers before the transport is aborted
// (YRT_GATHER_TIMEOUT_S, default 300: the status exchange also waits for the slowest rank's
// render to end).
double default_gather_timeout();

// Waits for the work enqueued on `st` (hipStreamQuery polling, backing off to 1 ms) until
// `deadline`; false when it expired with the work still pending. `poll` runs between queries
// (RCCL: its async-error check) and may throw.
bool stream_wait_until(hipStream_t st, Clock::time_point deadline, void (*poll)(void*) = nullptr,
                       void* pollArg = nullptr);

class GatherTransport {
 public:
  virtual ~GatherTransport() = default;
  virtual const char* kind() const = 0;  // "rccl" | "hub"
  virtual int rank() const = 0;
  virtual int world() const = 0;
  // The min over every rank of `flag` (1 = this rank's render succeeded). Throws on timeout.
  virtual int exchange_status(int flag, int device, hipStream_t st, double timeoutS) = 0;
  // Rank > 0: `bytes` of the device buffer `slab` (on HIP device `device`, enqueued work on
  // `st` first) to rank 0; complete when it returns.
  virtual void send_root(const void* slab, size_t bytes, int device, hipStream_t st, double timeoutS) = 0;
  // Rank 0: bytes[r] into bufs[r] from every rank r > 0 (bufs[0] unused); complete when it
  // returns.
  virtual void recv_all(const std::vector<void*>& bufs, const std::vector<size_t>& bytes, int device,
                        hipStream_t st, double timeoutS) = 0;
  // True once a timeout or a protocol error aborted the transport.
  virtual bool aborted() const = 0;
};

// RCCL: ncclCommInitRank(world, id, rank) on the current HIP device.
std::unique_ptr<GatherTransport> make_rccl_transport(int rank, int world, const void* id128);

// The in-process hub: `world` ranks of one process.
struct ShardHub;
std::shared_ptr<ShardHub> make_shard_hub(int world);
int shard_hub_world(const ShardHub& hub);
std::unique_ptr<GatherTransport> make_hub_transport(std::shared_ptr<ShardHub> hub, int rank);
// Host-memory forms of the hub's two phases (device = -1: memcpy instead of HIP copies), for
// the CPU tests of its deadlines and size checks.
int hub_host_status(ShardHub& hub, int rank, int flag, double timeoutS);
void hub_host_slab(ShardHub& hub, int rank, const void* slab, size_t bytes, void* recv, size_t recvBytesPerRank,
                   double timeoutS);

}  // namespace yrt
