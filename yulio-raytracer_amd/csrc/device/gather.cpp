// gather.cpp — the gather transports of gather.h: RCCL (one process per GPU) and the
// in-process hub (several Device objects of one process), both with bounded waits.
#include "gather.h"

#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <map>
#include <mutex>
#include <thread>
#include <utility>

#include "rccl_comm.h"

namespace yrt {

double default_gather_timeout() {
  if (const char* e = getenv("YRT_GATHER_TIMEOUT_S")) {
    const double v = atof(e);
    if (v > 0) return v;
  }
  return 300.0;
}

static Clock::time_point deadline_after(double s) {
  return Clock::now() + std::chrono::microseconds((long long)(std::max(0.0, s) * 1e6));
}

static std::string secs(double s) {
  char b[32];
  snprintf(b, sizeof(b), "%.3g s", s);
  return b;
}

bool stream_wait_until(hipStream_t st, Clock::time_point deadline, void (*poll)(void*), void* pollArg) {
  const Clock::time_point t0 = Clock::now();
  int us = 10;
  while (true) {
    const hipError_t e = hipStreamQuery(st);
    if (e == hipSuccess) return true;
    if (e != hipErrorNotReady)
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e) + " while waiting for a gather");
    if (poll) poll(pollArg);
    const Clock::time_point now = Clock::now();
    if (now >= deadline) return false;
    // short sleeps while a gather is normally in flight (a few ms), 1 ms once it is clearly
    // waiting for a slow peer
    us = now - t0 > std::chrono::milliseconds(100) ? 1000 : std::min(us * 2, 100);
    std::this_thread::sleep_for(std::chrono::microseconds(us));
  }
}

// ============================================================== RCCL
namespace {

class RcclTransport final : public GatherTransport {
 public:
  RcclTransport(int rank, int world, const void* id128) : r_(rank), w_(world) {
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId id;
    memcpy(&id, id128, sizeof(id));
    const RcclApi& nc = rccl();
    if (hipMalloc(&dFlag_, sizeof(int)) != hipSuccess || hipHostMalloc((void**)&hFlag_, sizeof(int)) != hipSuccess) {
      release_flags();
      throw std::runtime_error("RCCL gather: cannot allocate the status flag");
    }
    const ncclResult_t res = nc.CommInitRank(&comm_, world, id, rank);
    if (res != ncclSuccess) {
      release_flags();
      rccl_check(res, "ncclCommInitRank");
    }
  }
  ~RcclTransport() override {
    try {
      if (comm_ && !dead_) rccl().CommDestroy(comm_);
    } catch (...) {
    }
    release_flags();
  }
  const char* kind() const override { return "rccl"; }
  int rank() const override { return r_; }
  int world() const override { return w_; }
  bool aborted() const override { return dead_; }

  int exchange_status(int flag, int device, hipStream_t st, double timeoutS) override {
    live("status exchange");
    (void)hipSetDevice(device);
    *hFlag_ = flag;
    // a failing upload still joins the collective, with flag 0 (the peers must not wait)
    if (hipMemcpyAsync(dFlag_, hFlag_, sizeof(int), hipMemcpyHostToDevice, st) != hipSuccess)
      (void)hipMemsetAsync(dFlag_, 0, sizeof(int), st);
    const RcclApi& nc = rccl();
    rccl_check(nc.AllReduce(dFlag_, dFlag_, 1, ncclInt32, ncclMin, comm_, st), "ncclAllReduce");
    if (hipMemcpyAsync(hFlag_, dFlag_, sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess) *hFlag_ = 0;
    wait(st, timeoutS, "status exchange (AllReduce-min over " + std::to_string(w_) + " ranks)");
    return *hFlag_;
  }
  void send_root(const void* slab, size_t bytes, int device, hipStream_t st, double timeoutS) override {
    live("slab send");
    (void)hipSetDevice(device);
    if (bytes) rccl_check(rccl().Send(slab, bytes, ncclUint8, 0, comm_, st), "ncclSend");
    wait(st, timeoutS, "slab send of " + std::to_string(bytes) + " bytes to rank 0");
  }
  void recv_all(const std::vector<void*>& bufs, const std::vector<size_t>& bytes, int device, hipStream_t st,
                double timeoutS) override {
    live("slab receive");
    (void)hipSetDevice(device);
    const RcclApi& nc = rccl();
    rccl_check(nc.GroupStart(), "ncclGroupStart");
    for (int r = 1; r < w_; ++r)
      if (bytes[r]) rccl_check(nc.Recv(bufs[r], bytes[r], ncclUint8, r, comm_, st), "ncclRecv");
    rccl_check(nc.GroupEnd(), "ncclGroupEnd");
    wait(st, timeoutS, "slab receives on rank 0 from ranks 1.." + std::to_string(w_ - 1));
  }

 private:
  void live(const char* what) const {
    if (dead_) throw std::runtime_error(std::string("RCCL gather: ") + what +
                                        " on a communicator aborted by an earlier gather: " + why_);
  }
  static void poll_async(void* self) {
    auto* t = (RcclTransport*)self;
    ncclResult_t a = ncclSuccess;
    const RcclApi& nc = rccl();
    if (nc.CommGetAsyncError && nc.CommGetAsyncError(t->comm_, &a) == ncclSuccess && a != ncclSuccess &&
        a != ncclInProgress)
      throw std::runtime_error(std::string("RCCL asynchronous error: ") + nc.GetErrorString(a));
  }
  void wait(hipStream_t st, double timeoutS, const std::string& phase) {
    std::string err;
    try {
      if (!stream_wait_until(st, deadline_after(timeoutS), &RcclTransport::poll_async, this))
        err = "timed out after " + secs(timeoutS);
    } catch (const std::exception& e) {
      err = e.what();
    }
    if (err.empty()) return;
    why_ = phase + ": " + err + " (rank " + std::to_string(r_) + " of " + std::to_string(w_) + ")";
    abort_comm();
    throw std::runtime_error("RCCL gather " + why_ + "; communicator aborted");
  }
  void abort_comm() {
    if (dead_) return;
    dead_ = true;
    try {
      const RcclApi& nc = rccl();
      if (nc.CommAbort) nc.CommAbort(comm_);
      else nc.CommDestroy(comm_);
    } catch (...) {
    }
  }
  void release_flags() {
    if (dFlag_) (void)hipFree(dFlag_);
    if (hFlag_) (void)hipHostFree(hFlag_);
    dFlag_ = nullptr;
    hFlag_ = nullptr;
  }
  ncclComm_t comm_ = nullptr;
  int r_, w_;
  bool dead_ = false;
  std::string why_;
  void* dFlag_ = nullptr;
  int* hFlag_ = nullptr;
};

}  // namespace

std::unique_ptr<GatherTransport> make_rccl_transport(int rank, int world, const void* id128) {
  return std::unique_ptr<GatherTransport>(new RcclTransport(rank, world, id128));
}

// ============================================================== in-process hub
// Gather number s of the hub is the s-th status exchange of every rank (each rank counts its
// own); its slabs are posted under (s, rank). Rank 0 copies a peer's slab only after every
// peer has posted, and marks them consumed once its copies have completed, which releases the
// senders (their slab buffers stay untouched until then).
struct ShardHub {
  explicit ShardHub(int w) : world(w), seq(w, 0) {}
  const int world;
  std::mutex mu;
  std::condition_variable cv;
  bool aborted = false;
  std::string why;
  std::vector<uint64_t> seq;
  struct Status {
    int arrived = 0, left = 0, minFlag = 1;
    std::vector<char> who;
  };
  std::map<uint64_t, Status> status;
  struct Post {
    const void* p = nullptr;
    size_t bytes = 0;
    int device = -1;
    hipEvent_t ready = nullptr;
    bool consumed = false;
  };
  std::map<std::pair<uint64_t, int>, Post> posts;

  [[noreturn]] void fail_locked(const std::string& msg) {
    if (!aborted) {
      aborted = true;
      why = msg;
    }
    cv.notify_all();
    throw std::runtime_error("gather hub: " + msg + "; hub aborted");
  }
  void live_locked(int rank) const {
    if (aborted)
      throw std::runtime_error("gather hub (rank " + std::to_string(rank) + "): aborted by an earlier gather: " + why);
  }
  static std::string list(const std::vector<int>& v) {
    std::string s;
    for (size_t k = 0; k < v.size(); ++k) s += (k ? "," : "") + std::to_string(v[k]);
    return s;
  }

  int exchange(int rank, int flag, double timeoutS) {
    std::unique_lock<std::mutex> lk(mu);
    live_locked(rank);
    const uint64_t s = ++seq[rank];
    Status& S = status[s];
    if (S.who.empty()) S.who.assign(world, 0);
    S.who[rank] = 1;
    S.arrived++;
    S.minFlag = std::min(S.minFlag, flag);
    cv.notify_all();
    const Clock::time_point dl = deadline_after(timeoutS);
    while (S.arrived < world && !aborted) {
      if (cv.wait_until(lk, dl) == std::cv_status::timeout && S.arrived < world && !aborted) {
        std::vector<int> missing;
        for (int r = 0; r < world; ++r)
          if (!S.who[r]) missing.push_back(r);
        fail_locked("status exchange #" + std::to_string(s) + " timed out after " + secs(timeoutS) + " on rank " +
                    std::to_string(rank) + ": rank(s) " + list(missing) + " never arrived");
      }
    }
    live_locked(rank);
    const int m = S.minFlag;
    if (++S.left == world) status.erase(s);
    return m;
  }

  void send(int rank, const void* slab, size_t bytes, int device, hipStream_t st, double timeoutS) {
    hipEvent_t ev = nullptr;
    if (device >= 0) {
      (void)hipSetDevice(device);
      if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess || hipEventRecord(ev, st) != hipSuccess) {
        if (ev) (void)hipEventDestroy(ev);
        std::unique_lock<std::mutex> lk(mu);
        fail_locked("rank " + std::to_string(rank) + " cannot record its slab's ready event");
      }
    }
    std::unique_lock<std::mutex> lk(mu);
    try {
      live_locked(rank);
      const std::pair<uint64_t, int> key(seq[rank], rank);
      Post& P = posts[key];
      P.p = slab;
      P.bytes = bytes;
      P.device = device;
      P.ready = ev;
      cv.notify_all();
      const Clock::time_point dl = deadline_after(timeoutS);
      while (!P.consumed && !aborted)
        if (cv.wait_until(lk, dl) == std::cv_status::timeout && !P.consumed && !aborted)
          fail_locked("slab of rank " + std::to_string(rank) + " (gather #" + std::to_string(key.first) +
                      ", " + std::to_string(bytes) + " bytes) not received by rank 0 within " + secs(timeoutS));
      posts.erase(key);
      live_locked(rank);
    } catch (...) {
      lk.unlock();
      if (ev) (void)hipEventDestroy(ev);
      throw;
    }
    lk.unlock();
    if (ev) (void)hipEventDestroy(ev);
  }

  void recv(const std::vector<void*>& bufs, const std::vector<size_t>& bytes, int device, hipStream_t st,
            double timeoutS) {
    const Clock::time_point dl = deadline_after(timeoutS);
    std::vector<Post> got(world);
    uint64_t s;
    {
      std::unique_lock<std::mutex> lk(mu);
      live_locked(0);
      s = seq[0];
      auto all_posted = [&] {
        for (int r = 1; r < world; ++r)
          if (!posts.count({s, r})) return false;
        return true;
      };
      while (!all_posted() && !aborted)
        if (cv.wait_until(lk, dl) == std::cv_status::timeout && !all_posted() && !aborted) {
          std::vector<int> missing;
          for (int r = 1; r < world; ++r)
            if (!posts.count({s, r})) missing.push_back(r);
          fail_locked("slab receive on rank 0 (gather #" + std::to_string(s) + ") timed out after " +
                      secs(timeoutS) + ": rank(s) " + list(missing) + " never sent");
        }
      live_locked(0);
      for (int r = 1; r < world; ++r) {
        got[r] = posts[{s, r}];
        if (got[r].bytes != bytes[r])
          fail_locked("rank " + std::to_string(r) + " sent " + std::to_string(got[r].bytes) +
                      " bytes, rank 0 expects " + std::to_string(bytes[r]) + " (gather #" + std::to_string(s) + ")");
      }
    }
    std::string err;
    if (device >= 0) {
      (void)hipSetDevice(device);
      for (int r = 1; r < world && err.empty(); ++r) {
        if (!bytes[r]) continue;
        hipError_t e = got[r].ready ? hipStreamWaitEvent(st, got[r].ready, 0) : hipSuccess;
        if (e == hipSuccess)
          e = got[r].device == device
                  ? hipMemcpyAsync(bufs[r], got[r].p, bytes[r], hipMemcpyDeviceToDevice, st)
                  : hipMemcpyPeerAsync(bufs[r], device, got[r].p, got[r].device, bytes[r], st);
        if (e != hipSuccess) err = std::string("copy of rank ") + std::to_string(r) + "'s slab: " + hipGetErrorString(e);
      }
      if (err.empty()) {
        try {
          if (!stream_wait_until(st, dl)) err = "slab copies did not complete within " + secs(timeoutS);
        } catch (const std::exception& e) {
          err = e.what();
        }
      }
    } else {
      for (int r = 1; r < world; ++r)
        if (bytes[r]) memcpy(bufs[r], got[r].p, bytes[r]);
    }
    std::unique_lock<std::mutex> lk(mu);
    if (!err.empty()) fail_locked("rank 0, gather #" + std::to_string(s) + ": " + err);
    for (int r = 1; r < world; ++r) {
      auto it = posts.find({s, r});
      if (it != posts.end()) it->second.consumed = true;
    }
    cv.notify_all();
  }
};

namespace {

class HubTransport final : public GatherTransport {
 public:
  HubTransport(std::shared_ptr<ShardHub> hub, int rank) : hub_(std::move(hub)), r_(rank) {}
  const char* kind() const override { return "hub"; }
  int rank() const override { return r_; }
  int world() const override { return hub_->world; }
  bool aborted() const override {
    std::lock_guard<std::mutex> lk(hub_->mu);
    return hub_->aborted;
  }
  int exchange_status(int flag, int, hipStream_t, double timeoutS) override {
    return hub_->exchange(r_, flag, timeoutS);
  }
  void send_root(const void* slab, size_t bytes, int device, hipStream_t st, double timeoutS) override {
    hub_->send(r_, slab, bytes, device, st, timeoutS);
  }
  void recv_all(const std::vector<void*>& bufs, const std::vector<size_t>& bytes, int device, hipStream_t st,
                double timeoutS) override {
    hub_->recv(bufs, bytes, device, st, timeoutS);
  }

 private:
  std::shared_ptr<ShardHub> hub_;
  int r_;
};

}  // namespace

std::shared_ptr<ShardHub> make_shard_hub(int world) {
  if (world < 1) throw std::runtime_error("shard hub: world < 1");
  return std::make_shared<ShardHub>(world);
}
int shard_hub_world(const ShardHub& hub) { return hub.world; }

std::unique_ptr<GatherTransport> make_hub_transport(std::shared_ptr<ShardHub> hub, int rank) {
  if (!hub || rank < 0 || rank >= hub->world) throw std::runtime_error("shard hub: invalid rank");
  return std::unique_ptr<GatherTransport>(new HubTransport(std::move(hub), rank));
}

int hub_host_status(ShardHub& hub, int rank, int flag, double timeoutS) {
  if (rank < 0 || rank >= hub.world) throw std::runtime_error("shard hub: invalid rank");
  return hub.exchange(rank, flag, timeoutS);
}

void hub_host_slab(ShardHub& hub, int rank, const void* slab, size_t bytes, void* recv, size_t recvBytesPerRank,
                   double timeoutS) {
  if (rank < 0 || rank >= hub.world) throw std::runtime_error("shard hub: invalid rank");
  if (rank) {
    hub.send(rank, slab, bytes, -1, nullptr, timeoutS);
    return;
  }
  std::vector<void*> bufs(hub.world, nullptr);
  std::vector<size_t> sizes(hub.world, recvBytesPerRank);
  for (int r = 1; r < hub.world; ++r) bufs[r] = (char*)recv + (size_t)(r - 1) * recvBytesPerRank;
  hub.recv(bufs, sizes, -1, nullptr, timeoutS);
}

}  // namespace yrt
