// Communicators: native RCCL (device) and a c10d ProcessGroup adapter (gloo /
// CPU plumbing).  See pdrnn/runtime.h.
//
// The RCCL communicator is the MI355X-native replacement of the reference's
// ProcessGroupMPI (reference: src/motion/trainer/ddp.py:18,
// src/example/example_distributed.py:18-19):
//  * bootstrapped from an ncclUniqueId that the Python side distributes
//    through the torch.distributed TCPStore rendezvous,
//  * asynchronous collectives (all_reduce, broadcast, all_gather, ...) run on
//    ONE dedicated high-priority HIP stream per communicator, fenced against
//    the caller's compute stream with events, so gradient all-reduce overlaps
//    the BPTT kernels still running on the compute stream; all_reduce_inline
//    runs straight on the caller's stream (nothing to overlap),
//  * payloads are torch tensors; their storage is recorded on the comm stream
//    so the caching allocator never recycles memory a collective still reads,
//  * an in-place all_reduce over ONE rank is the identity and issues nothing
//    (PDRNN_FORCE_COLLECTIVE=1 keeps issuing it: tests and forced-sync timing),
//  * a watchdog thread bounds every collective: each one is followed by a
//    completion event; a collective still pending after `timeout_s` (or an
//    asynchronous RCCL error) aborts the communicator (ncclCommAbort makes
//    the spinning RCCL kernels exit, so a host blocked in a device
//    synchronize wakes up), every later call raises, and -- unless
//    PDRNN_COMM_WATCHDOG_EXIT=0 -- the process exits with kWatchdogExit after
//    a grace period.  This is the native counterpart of the reference's
//    bounded waits (RPC timeout 60 s, master.py:56 / worker.py:105;
//    horovodrun --start-timeout 300, fabfile.py:227).
#include <ATen/hip/impl/HIPCachingAllocatorMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <stdexcept>
#include <thread>

#include "pdrnn/api.h"
#include "pdrnn/runtime.h"

namespace pdrnn {
namespace {

namespace py = pybind11;

#define NCCL_CHECK(expr)                                                                   \
  do {                                                                                     \
    ncclResult_t _r = (expr);                                                              \
    TORCH_CHECK(_r == ncclSuccess, "RCCL error: ", ncclGetErrorString(_r), " @ " #expr); \
  } while (0)
#define HIP_CHECK(expr)                                                                    \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    TORCH_CHECK(_e == hipSuccess, "HIP error: ", hipGetErrorString(_e), " @ " #expr);     \
  } while (0)

ncclDataType_t to_nccl(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return ncclFloat32;
    case at::kHalf: return ncclFloat16;
    case at::kBFloat16: return ncclBfloat16;
    case at::kDouble: return ncclFloat64;
    case at::kLong: return ncclInt64;
    case at::kInt: return ncclInt32;
    case at::kByte: return ncclUint8;
    case at::kChar: return ncclInt8;
    case at::kBool: return ncclUint8;
    default: TORCH_CHECK(false, "RCCL: unsupported dtype ", t);
  }
}

ncclRedOp_t to_nccl(RedOp op) {
  switch (op) {
    case RedOp::kSum: return ncclSum;
    case RedOp::kAvg: return ncclAvg;
    case RedOp::kMax: return ncclMax;
    case RedOp::kMin: return ncclMin;
  }
  return ncclSum;
}

bool env_flag(const char* name, bool dflt) {
  const char* e = std::getenv(name);
  if (e == nullptr || e[0] == '\0') return dflt;
  return e[0] == '1' || e[0] == 'y' || e[0] == 'Y' || e[0] == 't' || e[0] == 'T';
}

double env_double(const char* name, double dflt) {
  const char* e = std::getenv(name);
  if (e == nullptr || e[0] == '\0') return dflt;
  char* end = nullptr;
  const double v = std::strtod(e, &end);
  return end != e ? v : dflt;
}

using Clock = std::chrono::steady_clock;

// PDRNN_RCCL_MAX_CTAS (default 8; 0 = RCCL's own choice): workgroups an RCCL
// collective of our communicators may occupy.  The motion all-reduce (56.6 KB)
// is latency-bound and needs few; a 32 MiB char-LM bucket over 7 xGMI peers
// still gets 8 channels.
std::atomic<int> g_cta_reserve{0};

}  // namespace

int rccl_max_ctas() {
  static const int v = [] {
    const char* e = std::getenv("PDRNN_RCCL_MAX_CTAS");
    return e && *e ? std::max(0, std::atoi(e)) : 8;
  }();
  return v;
}
int rccl_cta_reserve() { return g_cta_reserve.load(); }

namespace {

class RcclComm final : public Comm {
 public:
  RcclComm(const std::string& uid, int rank, int world, int device, bool high_priority, double timeout_s)
      : rank_(rank), world_(world), device_(device), timeout_s_(timeout_s > 0 ? timeout_s : 600.0) {
    TORCH_CHECK(uid.size() == sizeof(ncclUniqueId), "bad RCCL unique id size");
    ncclUniqueId id;
    std::memcpy(&id, uid.data(), sizeof(id));
    c10::DeviceGuard guard(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device_));
    int lo = 0, hi = 0;
    HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIP_CHECK(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, high_priority ? hi : lo));
    HIP_CHECK(hipEventCreateWithFlags(&ev_in_, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&ev_out_, hipEventDisableTiming));
    // every peer has just joined the torch.distributed rendezvous that carried
    // the unique id, so a blocking init cannot wait on a dead rank for long
    // Cap the CUs RCCL's kernels may take (config.maxCTAs): a bucket
    // all-reduce runs beside the grid-synced persistent recurrences of the
    // large-H layers, which need all their workgroups co-resident.  The
    // persistent planner leaves that many CUs free in every multi-rank
    // process (rccl_cta_reserve, bindings.cpp large_persist_plan), so an
    // all-reduce already resident can never keep a persistent grid waiting.
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    const int max_ctas = rccl_max_ctas();
    if (max_ctas > 0) cfg.maxCTAs = max_ctas;
    NCCL_CHECK(ncclCommInitRankConfig(&comm_, world_, id, rank_, &cfg));
    // (a forced one-rank collective rehearses the multi-rank overlap on one GPU)
    if ((world_ > 1 || env_flag("PDRNN_FORCE_COLLECTIVE", false)) && max_ctas > 0)
      g_cta_reserve.store(std::max(g_cta_reserve.load(), max_ctas));
    exit_on_abort_ = env_flag("PDRNN_COMM_WATCHDOG_EXIT", true);
    grace_s_ = env_double("PDRNN_COMM_WATCHDOG_GRACE_S", 5.0);
    poll_ms_ = std::max(1.0, env_double("PDRNN_COMM_WATCHDOG_POLL_MS", 100.0));
    watchdog_ = std::thread([this] { watchdog_loop(); });
  }
  ~RcclComm() override { close(); }
  void close() override {
    // api_mu_ only after the watchdog is joined: it may be waiting for it to abort
    if (closed_.exchange(true)) return;
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (watchdog_.joinable()) watchdog_.join();
    // The watchdog is gone: now wait (bounded) for an API call another thread
    // may still be inside (daemon threads survive to atexit) -- closed_ makes
    // every later call raise in live(), so once api_mu_ is ours no enqueue can
    // touch the stream / works_ being torn down below.
    std::unique_lock<std::mutex> api(api_mu_, std::defer_lock);
    for (const auto until = Clock::now() + std::chrono::seconds(10); !api.try_lock();) {
      if (Clock::now() > until) {
        std::fprintf(stderr, "[pdrnn] RCCL communicator (rank %d/%d) teardown: an API call still holds the "
                     "communicator after 10 s; tearing down anyway\n", rank_, world_);
        break;
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    if (comm_ && !aborted_.load()) {
      // Teardown is where a dead peer usually shows up (an exception unwinds,
      // reset_comms(), interpreter exit): a collective still pending would
      // block hipStreamSynchronize / ncclCommDestroy for ever.  Drain with a
      // deadline instead and abort the communicator if it passes.
      const double limit = std::min(timeout_s_, env_double("PDRNN_COMM_TEARDOWN_S", 30.0));
      std::string why;
      if (drain(limit, why)) {
        ncclCommDestroy(comm_);
      } else {
        std::fprintf(stderr, "[pdrnn] RCCL communicator (rank %d/%d) teardown: %s -- aborting instead of destroying\n",
                     rank_, world_, why.c_str());
        std::fflush(stderr);
        ncclCommAbort(comm_);
      }
    }
    comm_ = nullptr;
    for (auto& w : works_) hipEventDestroy(w.ev);
    works_.clear();
    for (auto ev : free_events_) hipEventDestroy(ev);
    free_events_.clear();
    if (ev_in_) hipEventDestroy(ev_in_);
    if (ev_out_) hipEventDestroy(ev_out_);
    if (stream_) hipStreamDestroy(stream_);
    ev_in_ = ev_out_ = nullptr;
    stream_ = nullptr;
  }
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  bool native_avg() const override { return true; }

  void all_reduce(at::Tensor& t, RedOp op) override {
    check(t);
    // an in-place reduction over one rank is the identity: no collective, no
    // comm-stream hop (the autograd DDP path at N = 1) -- unless forced
    if (world_ == 1 && !force_collective()) return;
    {
      std::lock_guard<std::mutex> api(api_mu_);
      live();
      enter();
      NCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), to_nccl(op), comm_, stream_));
      leave({t}, "all_reduce");
    }
    if (serialize_comm()) host_wait(stream_, "all_reduce");
  }
  void broadcast(at::Tensor& t, int root) override {
    check(t);
    {
      std::lock_guard<std::mutex> api(api_mu_);
      live();
      enter();
      NCCL_CHECK(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), root, comm_, stream_));
      leave({t}, "broadcast");
    }
    if (serialize_comm()) host_wait(stream_, "broadcast");
  }
  void all_gather(at::Tensor& out, const at::Tensor& in) override {
    check(out); check(in);
    TORCH_CHECK(out.numel() == in.numel() * world_, "all_gather: out must hold world * in elements");
    {
      std::lock_guard<std::mutex> api(api_mu_);
      live();
      enter();
      NCCL_CHECK(ncclAllGather(in.data_ptr(), out.data_ptr(), in.numel(), to_nccl(in.scalar_type()), comm_, stream_));
      leave({out, in}, "all_gather");
    }
    if (serialize_comm()) host_wait(stream_, "all_gather");
  }
  void reduce_scatter(at::Tensor& out, const at::Tensor& in, RedOp op) override {
    check(out); check(in);
    TORCH_CHECK(in.numel() == out.numel() * world_, "reduce_scatter: in must hold world * out elements");
    {
      std::lock_guard<std::mutex> api(api_mu_);
      live();
      enter();
      NCCL_CHECK(ncclReduceScatter(in.data_ptr(), out.data_ptr(), out.numel(), to_nccl(in.scalar_type()), to_nccl(op),
                                   comm_, stream_));
      leave({out, in}, "reduce_scatter");
    }
    if (serialize_comm()) host_wait(stream_, "reduce_scatter");
  }
  void all_to_all(at::Tensor& out, const at::Tensor& in) override {
    check(out); check(in);
    TORCH_CHECK(in.numel() % world_ == 0 && out.numel() == in.numel(), "all_to_all: equal splits required");
    const int64_t chunk = in.numel() / world_;
    const size_t esz = in.element_size();
    const auto dt = to_nccl(in.scalar_type());
    {
      std::lock_guard<std::mutex> api(api_mu_);
      live();
      enter();
      NCCL_CHECK(ncclGroupStart());
      for (int p = 0; p < world_; ++p) {
        NCCL_CHECK(ncclSend(static_cast<const char*>(in.data_ptr()) + p * chunk * esz, chunk, dt, p, comm_, stream_));
        NCCL_CHECK(ncclRecv(static_cast<char*>(out.data_ptr()) + p * chunk * esz, chunk, dt, p, comm_, stream_));
      }
      NCCL_CHECK(ncclGroupEnd());
      leave({out, in}, "all_to_all");
    }
    if (serialize_comm()) host_wait(stream_, "all_to_all");
  }
  void send(const at::Tensor& t, int peer) override {
    check(t);
    {
      std::lock_guard<std::mutex> api(api_mu_);
      live();
      enter();
      NCCL_CHECK(ncclSend(t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), peer, comm_, stream_));
      leave({t}, "send");
    }
    if (serialize_comm()) host_wait(stream_, "send");
  }
  void recv(at::Tensor& t, int peer) override {
    check(t);
    {
      std::lock_guard<std::mutex> api(api_mu_);
      live();
      enter();
      NCCL_CHECK(ncclRecv(t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), peer, comm_, stream_));
      leave({t}, "recv");
    }
    if (serialize_comm()) host_wait(stream_, "recv");
  }
  void all_reduce_inline(at::Tensor& t, RedOp op) override {
    check(t);
    // keep this communicator's collectives strictly ordered: join any still
    // queued on the comm stream first
    if (pending_) wait();
    c10::DeviceGuard guard(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device_));
    hipStream_t cs = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA((c10::DeviceIndex)device_).stream();
    if (cs == nullptr) {
      // never put RCCL on the legacy NULL stream (it synchronises with every
      // blocking stream): go through the comm stream instead
      all_reduce(t, op);
      wait();
      return;
    }
    {
      std::lock_guard<std::mutex> api(api_mu_);
      live();
      NCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), to_nccl(op), comm_, cs));
      track(cs, "all_reduce_inline");
    }
    if (serialize_comm()) host_wait(cs, "all_reduce_inline");
  }
  void wait() override {
    live();
    c10::DeviceGuard guard(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device_));
    HIP_CHECK(hipEventRecord(ev_out_, stream_));
    HIP_CHECK(hipStreamWaitEvent(c10::hip::getCurrentHIPStreamMasqueradingAsCUDA((c10::DeviceIndex)device_).stream(), ev_out_, 0));
    pending_ = false;
  }
  void barrier() override {
    auto t = at::zeros({1}, at::TensorOptions().device(at::kCUDA, device_).dtype(at::kFloat));
    if (world_ > 1 || force_collective()) {
      {
        std::lock_guard<std::mutex> api(api_mu_);
        live();
        enter();
        NCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), 1, ncclFloat32, ncclSum, comm_, stream_));
        leave({t}, "barrier");
      }
    }
    wait();
    host_wait(stream_, "barrier");
  }
  void debug_stall(double seconds) override {
    // a stand-in for a collective whose peer never arrives: bounded spin on
    // the comm stream, tracked like a collective (watchdog tests)
    std::lock_guard<std::mutex> api(api_mu_);
    live();
    enter();
    HIP_CHECK(pdrnn_debug_spin((uint64_t)(seconds * 1e6), stream_));
    leave({}, "debug_stall");
  }
  bool aborted() const override { return aborted_.load(); }
  double timeout_s() const override { return timeout_s_; }
  int64_t tracked() const override { return tracked_.load(); }
  hipStream_t stream() const { return stream_; }

 private:
  struct Work {
    hipEvent_t ev;
    Clock::time_point t;
    const char* what;
  };

  // read per call (a getenv): tests flip it inside one process
  static bool force_collective() { return env_flag("PDRNN_FORCE_COLLECTIVE", false); }
  void check(const at::Tensor& t) const {
    TORCH_CHECK(t.is_cuda() && t.get_device() == device_, "RCCL tensors must live on device ", device_);
    TORCH_CHECK(t.is_contiguous(), "RCCL tensors must be contiguous");
  }
  // raise once the watchdog has aborted the communicator
  void live() const {
    TORCH_CHECK(!closed_.load(), "RCCL communicator (rank ", rank_, "/", world_, ") was closed");
    if (aborted_.load()) {
      std::lock_guard<std::mutex> lk(mu_);
      TORCH_CHECK(false, "RCCL communicator (rank ", rank_, "/", world_, ") was aborted by the watchdog: ",
                  abort_reason_);
    }
  }
  // Order the comm stream after everything enqueued on the caller's stream.
  void enter() {
    pending_ = true;
    c10::DeviceGuard guard(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device_));
    HIP_CHECK(hipEventRecord(ev_in_, c10::hip::getCurrentHIPStreamMasqueradingAsCUDA((c10::DeviceIndex)device_).stream()));
    HIP_CHECK(hipStreamWaitEvent(stream_, ev_in_, 0));
  }
  void leave(std::initializer_list<at::Tensor> ts, const char* what) {
    auto s = c10::hip::getStreamFromExternalMasqueradingAsCUDA(stream_, (c10::DeviceIndex)device_);
    for (const auto& t : ts)
      if (t.defined() && t.storage().data_ptr().get())
        c10::hip::HIPCachingAllocatorMasqueradingAsCUDA::recordStreamMasqueradingAsCUDA(t.storage().data_ptr(), s);
    track(stream_, what);
  }
  void track_current() override {
    hipStream_t cs = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA((c10::DeviceIndex)device_).stream();
    track(cs, "graph replay");
  }
  // completion event after the collective just enqueued on `st` (skipped while
  // `st` is being captured into a graph: a captured event cannot be queried)
  void track(hipStream_t st, const char* what) {
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone) return;
    hipEvent_t ev = nullptr;
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (!free_events_.empty()) {
        ev = free_events_.back();
        free_events_.pop_back();
      }
    }
    if (ev == nullptr) HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    HIP_CHECK(hipEventRecord(ev, st));
    {
      std::lock_guard<std::mutex> lk(mu_);
      works_.push_back({ev, Clock::now(), what});
    }
    tracked_.fetch_add(1);
  }
  // Destructor helper (watchdog already stopped): poll the comm stream and
  // every still-tracked collective (inline ones run on compute streams) until
  // all completed, an error shows up, or `limit_s` passes.
  bool drain(double limit_s, std::string& why) {
    const auto until = Clock::now() + std::chrono::duration<double>(limit_s);
    for (int spins = 0;; ++spins) {
      bool done = true;
      const hipError_t qs = hipStreamQuery(stream_);
      if (qs == hipErrorNotReady) done = false;
      else if (qs != hipSuccess) { why = std::string("comm stream error: ") + hipGetErrorString(qs); return false; }
      while (done && !works_.empty()) {
        const hipError_t q = hipEventQuery(works_.front().ev);
        if (q == hipErrorNotReady) { done = false; break; }
        if (q != hipSuccess) { why = std::string("error on ") + works_.front().what + ": " + hipGetErrorString(q); return false; }
        free_events_.push_back(works_.front().ev);
        works_.pop_front();
      }
      if (done) return true;
      if (comm_ != nullptr) {
        ncclResult_t ae = ncclSuccess;
        if (ncclCommGetAsyncError(comm_, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
          why = std::string("asynchronous RCCL error: ") + ncclGetErrorString(ae);
          return false;
        }
      }
      if (Clock::now() > until) {
        char buf[160];
        std::snprintf(buf, sizeof(buf), "collectives still pending after %.1f s", limit_s);
        why = buf;
        return false;
      }
      std::this_thread::sleep_for(std::chrono::microseconds(spins < 64 ? 50 : 1000));
    }
  }

  // host-side wait that raises (instead of hanging) once the watchdog aborts
  void host_wait(hipStream_t st, const char* what) {
    hipEvent_t ev;
    HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    HIP_CHECK(hipEventRecord(ev, st));
    // poll without sleeping for the first 2 ms (a barrier normally completes
    // in tens of us: a fixed 200 us sleep after 64 polls made every world-1
    // barrier cost ~0.3 ms, profiles/r6/bench_trace.md), then back off to
    // 200 us sleeps so a long wait does not burn a core
    const auto t0 = std::chrono::steady_clock::now();
    int64_t nap_us = 10;
    for (;;) {
      const hipError_t q = hipEventQuery(ev);
      if (q == hipSuccess) break;
      if (q != hipErrorNotReady) {
        hipEventDestroy(ev);
        TORCH_CHECK(false, "HIP error while waiting for ", what, ": ", hipGetErrorString(q));
      }
      if (aborted_.load()) {
        hipEventDestroy(ev);
        live();
      }
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) {
        std::this_thread::sleep_for(std::chrono::microseconds(nap_us));
        nap_us = std::min<int64_t>(200, nap_us * 2);
      }
    }
    hipEventDestroy(ev);
  }

  void watchdog_loop() {
    hipSetDevice(device_);
    std::unique_lock<std::mutex> lk(mu_);
    while (!stop_) {
      cv_.wait_for(lk, std::chrono::microseconds((int64_t)(poll_ms_ * 1000)));
      if (stop_) break;
      // retire completed work (FIFO: collectives of one communicator complete in order per stream)
      std::string reason;
      while (!works_.empty()) {
        const hipError_t q = hipEventQuery(works_.front().ev);
        if (q == hipSuccess) {
          free_events_.push_back(works_.front().ev);
          works_.pop_front();
          continue;
        }
        if (q != hipErrorNotReady) reason = std::string("HIP error on ") + works_.front().what + ": " + hipGetErrorString(q);
        break;
      }
      if (reason.empty() && !works_.empty()) {
        const double age = std::chrono::duration<double>(Clock::now() - works_.front().t).count();
        if (age > timeout_s_) {
          char buf[256];
          std::snprintf(buf, sizeof(buf), "%s did not complete within %.1f s (%zu collective(s) pending)",
                        works_.front().what, timeout_s_, works_.size());
          reason = buf;
        }
      }
      if (reason.empty() && comm_ != nullptr) {
        ncclResult_t ae = ncclSuccess;
        if (ncclCommGetAsyncError(comm_, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress)
          reason = std::string("asynchronous RCCL error: ") + ncclGetErrorString(ae);
      }
      if (!reason.empty()) {
        abort_reason_ = reason;
        lk.unlock();
        abort_and_maybe_exit();
        return;
      }
    }
  }

  void abort_and_maybe_exit() {
    std::fprintf(stderr, "[pdrnn] RCCL watchdog (rank %d/%d): %s -- aborting the communicator\n", rank_, world_,
                 abort_reason_.c_str());
    std::fflush(stderr);
    aborted_.store(true);
    // never abort while the main thread is inside an RCCL enqueue; a thread
    // stuck inside one for seconds is itself the hang: exit without abort
    bool locked = false;
    for (int i = 0; i < 50 && !locked; ++i) {
      locked = api_mu_.try_lock();
      if (!locked) std::this_thread::sleep_for(std::chrono::milliseconds(100));
    }
    if (locked) {
      ncclCommAbort(comm_);  // in-flight RCCL kernels observe the abort flag and exit
      api_mu_.unlock();
    }
    if (!exit_on_abort_) return;
    // give the main thread a chance to raise out of its next call (clean
    // Python exit with a traceback); otherwise end the process non-zero
    const auto until = Clock::now() + std::chrono::duration<double>(grace_s_);
    while (Clock::now() < until) {
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (stop_) return;
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
    std::fprintf(stderr, "[pdrnn] RCCL watchdog (rank %d/%d): exiting with status %d\n", rank_, world_, kWatchdogExit);
    std::fflush(stderr);
    std::_Exit(kWatchdogExit);
  }

  int rank_, world_, device_;
  double timeout_s_;
  double grace_s_ = 5.0, poll_ms_ = 100.0;
  bool exit_on_abort_ = true;
  ncclComm_t comm_ = nullptr;
  hipStream_t stream_ = nullptr;
  hipEvent_t ev_in_ = nullptr, ev_out_ = nullptr;
  bool pending_ = false;  // collectives on stream_ not yet joined by wait()
  // watchdog state (mu_ guards works_, free_events_, stop_, abort_reason_)
  mutable std::mutex mu_;
  std::mutex api_mu_;  // held around every RCCL enqueue (abort never races one)
  std::condition_variable cv_;
  std::deque<Work> works_;
  std::vector<hipEvent_t> free_events_;
  bool stop_ = false;
  std::string abort_reason_;
  std::atomic<bool> aborted_{false};
  std::atomic<bool> closed_{false};
  std::atomic<int64_t> tracked_{0};
  std::thread watchdog_;
};

// c10d adapter: drives torch.distributed collectives (gloo on CPU, or torch's
// own RCCL process group) through Python.  Used for the CPU plumbing path and
// as a fallback; async work handles are waited in wait().
class ProcessGroupComm final : public Comm {
  void maybe_serialize() {
    if (serialize_comm()) wait();
  }

 public:
  explicit ProcessGroupComm(py::object pg) : pg_(std::move(pg)) {
    py::gil_scoped_acquire gil;
    dist_ = py::module_::import("torch.distributed");
    rank_ = dist_.attr("get_rank")(pg_).cast<int>();
    world_ = dist_.attr("get_world_size")(pg_).cast<int>();
    backend_ = py::str(dist_.attr("get_backend")(pg_)).cast<std::string>();
  }
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  bool native_avg() const override { return backend_ == "nccl"; }

  void all_reduce(at::Tensor& t, RedOp op) override {
    py::gil_scoped_acquire gil;
    works_.push_back(dist_.attr("all_reduce")(t, py::arg("op") = pyop(op), py::arg("group") = pg_,
                                               py::arg("async_op") = true));
    maybe_serialize();
  }
  void broadcast(at::Tensor& t, int root) override {
    py::gil_scoped_acquire gil;
    const int groot = dist_.attr("get_global_rank")(pg_, root).cast<int>();
    works_.push_back(dist_.attr("broadcast")(t, py::arg("src") = groot, py::arg("group") = pg_,
                                              py::arg("async_op") = true));
    maybe_serialize();
  }
  void all_gather(at::Tensor& out, const at::Tensor& in) override {
    py::gil_scoped_acquire gil;
    works_.push_back(dist_.attr("all_gather_into_tensor")(out, in, py::arg("group") = pg_, py::arg("async_op") = true));
    maybe_serialize();
  }
  void reduce_scatter(at::Tensor& out, const at::Tensor& in, RedOp op) override {
    py::gil_scoped_acquire gil;
    if (backend_ == "gloo") {
      // gloo has no reduce_scatter: all_reduce a copy and slice.
      auto tmp = in.clone();
      dist_.attr("all_reduce")(tmp, py::arg("op") = pyop(op), py::arg("group") = pg_);
      out.copy_(tmp.view({world_, -1}).select(0, rank_).view_as(out));
      return;
    }
    works_.push_back(dist_.attr("reduce_scatter_tensor")(out, in, py::arg("op") = pyop(op), py::arg("group") = pg_,
                                                         py::arg("async_op") = true));
    maybe_serialize();
  }
  void all_to_all(at::Tensor& out, const at::Tensor& in) override {
    py::gil_scoped_acquire gil;
    works_.push_back(dist_.attr("all_to_all_single")(out, in, py::arg("group") = pg_, py::arg("async_op") = true));
    maybe_serialize();
  }
  void send(const at::Tensor& t, int peer) override {
    py::gil_scoped_acquire gil;
    const int g = dist_.attr("get_global_rank")(pg_, peer).cast<int>();
    dist_.attr("send")(t, g, py::arg("group") = pg_);
  }
  void recv(at::Tensor& t, int peer) override {
    py::gil_scoped_acquire gil;
    const int g = dist_.attr("get_global_rank")(pg_, peer).cast<int>();
    dist_.attr("recv")(t, g, py::arg("group") = pg_);
  }
  void wait() override {
    py::gil_scoped_acquire gil;
    for (auto& w : works_) w.attr("wait")();
    works_.clear();
  }
  void barrier() override {
    wait();
    py::gil_scoped_acquire gil;
    dist_.attr("barrier")(py::arg("group") = pg_);
  }

 private:
  py::object pyop(RedOp op) {
    auto R = dist_.attr("ReduceOp");
    switch (op) {
      case RedOp::kSum: return R.attr("SUM");
      case RedOp::kAvg: return R.attr("AVG");
      case RedOp::kMax: return R.attr("MAX");
      case RedOp::kMin: return R.attr("MIN");
    }
    return R.attr("SUM");
  }
  py::object pg_, dist_;
  std::vector<py::object> works_;
  int rank_ = 0, world_ = 1;
  std::string backend_;
};

}  // namespace

bool serialize_comm() {
  static const bool on = [] {
    const char* e = std::getenv("PDRNN_SERIALIZE_COMM");
    return e != nullptr && e[0] == '1';
  }();
  return on;
}

std::string rccl_unique_id() {
  ncclUniqueId id;
  NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

std::shared_ptr<Comm> make_rccl_comm(const std::string& uid, int rank, int world, int device, bool high_priority,
                                     double timeout_s) {
  return std::make_shared<RcclComm>(uid, rank, world, device, high_priority, timeout_s);
}

std::shared_ptr<Comm> make_pg_comm(const pybind11::object& process_group) {
  return std::make_shared<ProcessGroupComm>(process_group);
}

}  // namespace pdrnn
